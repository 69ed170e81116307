# Launch-plan A/B on the binned SAH tree: leaf sizes, register caps and
# shading thresholds for the Cornell (LDS) and cornell_1m (HBM) plans.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tune}
mkdir -p $O
timeout -k 10 300 python tools/perf_ab.py --scene cornell --spp 64 --rounds 3 \
    --variants default,default/leaf1,default/leaf3,default/leaf4,waves4,waves6,default/trav4,default/trav24 \
    > $O/cornell.jsonl 2> $O/cornell.log \
 && timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 16 --rounds 3 \
    --variants default,default/leaf2,default/leaf6,default/leaf8,waves5,waves4,default/trav16,default/trav48,bvh2 \
    > $O/1m.jsonl 2> $O/1m.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
