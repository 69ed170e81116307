# Binned-SAH bin count A/B (FRT_SAH_BINS) on the bench scenes: Cornell (LDS)
# and cornell_1m (HBM, BVH4Q).  Chained; each bench has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-sahbins}
mkdir -p $O
run() {  # bins scene
  FRT_SAH_BINS=$1 timeout -k 10 200 python bench.py --scene $2 --steps 2 --warmup 1 --no-cpu-baseline \
      > $O/$2_b$1.json 2> $O/$2_b$1.log
}
run 32 cornell_1m && run 8 cornell_1m && run 16 cornell_1m && run 64 cornell_1m && run 128 cornell_1m \
 && run 32 cornell && run 16 cornell && run 64 cornell && run 128 cornell
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
