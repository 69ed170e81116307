# GPU check of the current tree: parity tests, then the C2 / C3 / C4 bench
# lines.  Every GPU step has its own time limit; steps are chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-check}
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python bench.py --cpu-seconds ${CPU_S:-4} > $O/bench_cornell.json 2> $O/bench_cornell.log \
 && timeout -k 10 300 python bench.py --scene veach --spp 1024 --cpu-seconds ${CPU_S:-4} > $O/bench_veach.json 2> $O/bench_veach.log \
 && timeout -k 10 300 python bench.py --scene cornell_1m --cpu-seconds ${CPU_S:-4} > $O/bench_1m.json 2> $O/bench_1m.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
