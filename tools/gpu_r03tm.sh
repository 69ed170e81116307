# Round 3 (re-entry): trav_min / min_desc re-checked under the final work queue
# (64-item grabs, <= 24 samples an item).  Same process, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03tm}
mkdir -p $O
timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 \
    --variants default,default/trav20,default/trav36,default/trav44 > $O/trav_cornell.jsonl 2>> $O/log.txt \
 && timeout -k 10 500 python -u tools/perf_ab.py --scene cornell_1m --spp 256 --rounds 2 --bvh gsah \
    --variants default,default/trav32,default/trav48,default/desc12,default/trav48/desc12 > $O/trav_1m.jsonl 2>> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
