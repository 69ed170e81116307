# Scheduling knobs re-checked on the round-3 build, interleaved in one process
# per scene (tools/perf_ab.py variants): trav_min on Cornell 512 spp,
# trav_min x min_desc on cornell_1m 256 spp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-knobs}
mkdir -p $O
timeout -k 10 400 python tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --bvh gsah \
    --variants default/trav20,default/trav24,default/trav28,default/trav32,default/trav36 > $O/cornell.jsonl 2>> $O/log.txt \
 && timeout -k 10 500 python tools/perf_ab.py --scene cornell_1m --spp 256 --rounds 3 --bvh gsah \
    --variants default/trav32/desc8,default/trav40/desc8,default/trav48/desc8,default/trav40/desc4,default/trav40/desc12,default/trav48/desc12 > $O/cornell_1m.jsonl 2>> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
