# Scheduling knobs re-checked on the round-3 build, interleaved in one process
# per scene (tools/perf_ab.py variants): trav_min on Cornell 512 spp,
# trav_min x min_desc on cornell_1m 256 spp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-knobs}
mkdir -p $O
timeout -k 10 400 python tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --bvh gsah \
    --variants default/trav=20,default/trav=24,default/trav=28,default/trav=32,default/trav=36 > $O/cornell.jsonl 2>> $O/log.txt \
 && timeout -k 10 500 python tools/perf_ab.py --scene cornell_1m --spp 256 --rounds 3 --bvh gsah \
    --variants default/trav=32/desc=8,default/trav=40/desc=8,default/trav=48/desc=8,default/trav=40/desc=4,default/trav=40/desc=12,default/trav=48/desc=12 > $O/cornell_1m.jsonl 2>> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
