# Round 3: the full -m gpu suite on the current build, then the lean-state A/B
# (lean only on HBM plans) against the pre-change build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03j}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && TAG=${TAG:-r03j}/ab PMC=0 bash tools/gpu_ab_libs.sh
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
