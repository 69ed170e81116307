# Round 4, tenth call: the GPU suite + smoke on the build with LDS-path
# trav_min 20, then the default bench command under rocprofv3 kernel-trace
# (the launch averages bench.py's roofline divides by) and its Cornell /
# cornell_1m PMC passes (tools/gpu_roofline.sh PART=a).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && TAG=r04j/roof PART=a bash tools/gpu_roofline.sh
