# Round 3 (re-entry): the work granule under 64-item grabs, smaller items.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03g3}
mkdir -p $O
timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 \
    --variants default/spi32,default/spi22,default/spi16,default/spi11,default/spi8 > $O/spi_cornell.jsonl 2>> $O/log.txt \
 && timeout -k 10 200 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --integrator ao \
    --variants default,default/spi32,default/spi16,default/spi8 > $O/spi_ao.jsonl 2>> $O/log.txt \
 && timeout -k 10 500 python -u tools/perf_ab.py --scene cornell_1m --spp 512 --rounds 2 --bvh gsah \
    --variants default/spi22,default/spi16,default/spi11,default/spi8 > $O/spi_1m.jsonl 2>> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
