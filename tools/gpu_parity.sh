# GPU parity + first measurements.  Every GPU step has its own time limit and
# the steps are chained: the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r1}
timeout -k 10 420 python -m pytest tests -m gpu -x -q -s > gpurun_out/${TAG}_pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python bench.py --spp 16 --steps 2 --warmup 1 --cpu-pixels 2048 > gpurun_out/${TAG}_bench_spp16.json 2> gpurun_out/${TAG}_bench_spp16.log \
 && timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log
rc=$?
echo "rc=$rc" > gpurun_out/${TAG}_rc.txt
exit $rc
