# Round 3: ray-query throughput (tools/trace_bench.py) on cornell_1m and
# Cornell for camera / bounce / shadow rays at register caps 6 / 8 / 10.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03e}
mkdir -p $O
timeout -k 10 400 python tools/trace_bench.py --scene cornell_1m > $O/trace_1m.jsonl 2> $O/trace_1m.log \
 && timeout -k 10 300 python tools/trace_bench.py --scene cornell > $O/trace_cornell.jsonl 2> $O/trace_cornell.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
