# 8-wide HBM tree against the 4-wide default, with its scheduling and leaf
# knobs, interleaved in one process (tools/perf_ab.py variants: option values
# follow the key directly, e.g. wide8, trav48, desc16, leaf2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abwide2}
mkdir -p $O
timeout -k 10 900 python tools/perf_ab.py --scene cornell_1m --spp 256 --rounds 3 --bvh gsah \
    --variants ${VARIANTS:-default,default/wide8,default/wide8/desc4,default/wide8/desc16,default/wide8/trav48,default/wide8/trav32,default/wide8/leaf2,default/wide8/leaf6} > $O/cornell_1m.jsonl 2>> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
