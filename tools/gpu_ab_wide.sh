# 8-wide vs 4-wide HBM tree (FRT_WIDE at upload), interleaved in one process
# per scene (tools/perf_ab.py variants), after the GPU parity tests that cover
# the wide plans.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abwide}
mkdir -p $O
FRT_WIDE=8 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c4.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_wide8.log 2>&1 \
 && timeout -k 10 600 python tools/perf_ab.py --scene cornell_1m --spp 256 --rounds 3 --bvh gsah \
    --variants default,default/wide=8 > $O/cornell_1m.jsonl 2>> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
