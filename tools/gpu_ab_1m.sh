# cornell_1m A/B in one call: variants of the product library, then of an
# experiment build (FRT_LIB_PATH), each its own process with interleaved rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab1m}; mkdir -p $O
timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 32 --rounds 3 --variants ${V1:-default} > $O/ab_main.jsonl 2> $O/ab_main.log || exit $?
if [ -n "$EXP" ]; then
  FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_$EXP.so timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 32 --rounds 3 --variants ${V2:-default} > $O/ab_$EXP.jsonl 2> $O/ab_$EXP.log || exit $?
fi
if [ -n "$EXP2" ]; then
  FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_$EXP2.so timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 32 --rounds 3 --variants ${V2:-default} > $O/ab_$EXP2.jsonl 2> $O/ab_$EXP2.log || exit $?
fi
