# Round 3 (re-entry): the work granule re-checked under 64-item queue grabs
# (the 40-items-per-lane rule was tuned with one atomic per refill).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03g2}
mkdir -p $O
timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 \
    --variants default,default/spi128,default/spi64,default/spi43,default/spi32 > $O/spi_cornell.jsonl 2>> $O/log.txt \
 && timeout -k 10 500 python -u tools/perf_ab.py --scene cornell_1m --spp 512 --rounds 2 --bvh gsah \
    --variants default,default/spi43,default/spi32,default/spi22 > $O/spi_1m.jsonl 2>> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
