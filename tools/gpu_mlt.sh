# PSS-MLT GPU tests + C5 bench line, then the default bench.  Chained, time-limited steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-mlt}
mkdir -p gpurun_out/$TAG
timeout -k 10 420 python -m pytest tests -m gpu -x -q -s > gpurun_out/$TAG/pytest_gpu.log 2>&1 \
 && timeout -k 10 400 python bench.py --integrator pssmlt --steps 2 --warmup 1 > gpurun_out/$TAG/bench_mlt.json 2> gpurun_out/$TAG/bench_mlt.log
rc=$?
echo "rc=$rc" > gpurun_out/$TAG/rc.txt
exit $rc
