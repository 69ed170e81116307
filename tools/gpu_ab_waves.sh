# Register-cap A/B at the bench's 1080p / 512 spp on the bench default tree
# (GPU binned SAH): cornell_1m (HBM plan, default cap 6) and Cornell (LDS plan,
# default cap 5), interleaved rounds in one process per scene.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-abwaves}; mkdir -p $O
timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 512 --rounds 3 --bvh gsah --variants default,waves5,waves4 > $O/ab_1m.jsonl 2> $O/ab_1m.log || exit $?
timeout -k 10 300 python tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,waves6,waves4 > $O/ab_cornell.jsonl 2> $O/ab_cornell.log || exit $?
