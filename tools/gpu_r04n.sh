# Round 4, fourteenth call: timing build with one mix32 round per path random
# number (invalid against the oracle, timing only: build/exp/libfrt_rngcheap.so
# vs libfrt_rngref.so, the same source) on Cornell and cornell_1m.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04n; mkdir -p $O
E=first_raytracer_amd/build/exp
C="--scene cornell --spp 512 --rounds 3 --bvh gsah --variants default"
M="--scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default"
ab() { local l=$1; shift; FRT_LIB_PATH=$E/$l timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_rng.jsonl 2>> $O/ab.log; }
ab libfrt_rngref.so $C && ab libfrt_rngcheap.so $C && ab libfrt_rngref.so $C && ab libfrt_rngcheap.so $C \
 && ab libfrt_rngref.so $M && ab libfrt_rngcheap.so $M
