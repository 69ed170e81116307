# Round 3 (re-entry): wave-local item ranges (FRT_GRAB items per queue atomic).
# Parity suite under grab 64, then same-process A/B on AO, Cornell path and
# cornell_1m.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03z}
mkdir -p $O
FRT_GRAB=64 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_integrators.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_grab64.log 2>&1 \
 && timeout -k 10 200 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --integrator ao \
      --variants default,default/grab16,default/grab64,default/grab256,default/spi512,default/spi512/grab64 > $O/ao.jsonl 2>> $O/log.txt \
 && timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 \
      --variants default,default/grab16,default/grab64,default/grab256 > $O/cornell.jsonl 2>> $O/log.txt \
 && timeout -k 10 400 python -u tools/perf_ab.py --scene cornell_1m --spp 256 --rounds 3 --bvh gsah \
      --variants default,default/grab16,default/grab64 > $O/c1m.jsonl 2>> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
