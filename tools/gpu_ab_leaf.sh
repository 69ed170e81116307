# Leaf-size A/B at the bench's 1080p / 512 spp on the bench's default tree
# (GPU binned SAH): cornell_1m (HBM plan) and Cornell (LDS plan), interleaved
# rounds in one process per scene.  FRT_LEAF_SIZE per context.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-ableaf}; mkdir -p $O
timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 512 --rounds 3 --bvh gsah --variants default,default/leaf3,default/leaf5,default/leaf6 > $O/ab_1m.jsonl 2> $O/ab_1m.log || exit $?
timeout -k 10 300 python tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,default/leaf1,default/leaf3 > $O/ab_cornell.jsonl 2> $O/ab_cornell.log || exit $?
