# GPU check of the current tree: parity tests, A/B of register caps, then the
# three bench lines (C1 Cornell, C4 1M triangles, C5 PSS-MLT).  Chained,
# every GPU step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-round}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 420 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python tools/perf_ab.py --scene cornell --spp 64 --variants ${AB_CORNELL:-default,waves4,waves6} > $O/ab_cornell.jsonl 2> $O/ab_cornell.log \
 && timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 32 --rounds 3 --variants ${AB_1M:-default,waves4,waves5} > $O/ab_1m.jsonl 2> $O/ab_1m.log \
 && timeout -k 10 400 python bench.py --cpu-seconds ${CPU_S:-4} > $O/bench_cornell.json 2> $O/bench_cornell.log \
 && timeout -k 10 400 python bench.py --scene cornell_1m --cpu-seconds ${CPU_S:-4} > $O/bench_1m.json 2> $O/bench_1m.log \
 && timeout -k 10 400 python bench.py --integrator pssmlt --steps 2 --warmup 1 --cpu-seconds ${CPU_S:-4} > $O/bench_mlt.json 2> $O/bench_mlt.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
