# GPU perf iteration: parity tests, A/B variants, bench.  Chained, each step time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-perf}
mkdir -p gpurun_out/$TAG
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/$TAG/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python tools/perf_ab.py --scene cornell --spp 64 --variants default,waves5,waves6,default/leaf1,waves5/leaf1,no_lds > gpurun_out/$TAG/ab_cornell.jsonl 2> gpurun_out/$TAG/ab_cornell.log \
 && timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 32 --variants default,waves5,waves6,default/leaf1,waves5/leaf2 --rounds 3 > gpurun_out/$TAG/ab_1m.jsonl 2> gpurun_out/$TAG/ab_1m.log \
 && timeout -k 10 400 python bench.py --cpu-pixels 8192 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.log
rc=$?
echo "rc=$rc" > gpurun_out/$TAG/rc.txt
exit $rc
