# Round 3: ray-query throughput on large batches (32 rays per pixel).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03g}
mkdir -p $O
timeout -k 10 400 python tools/trace_bench.py --scene cornell_1m --rays-per-pixel 32 --rounds 2 > $O/trace_1m.jsonl 2> $O/trace_1m.log \
 && timeout -k 10 300 python tools/trace_bench.py --scene cornell --rays-per-pixel 32 --rounds 2 > $O/trace_cornell.jsonl 2> $O/trace_cornell.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
