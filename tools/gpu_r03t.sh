# Round 3 (re-entry): node-order A/B on cornell_1m (FRT_NODE_ORDER 0/1/2, same
# process, interleaved), then the caps table, -m gpu suite, smoke() and the
# default bench line on the rebuilt library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03t}
mkdir -p $O
timeout -k 10 300 python -u tools/perf_ab.py --scene cornell_1m --spp 256 --rounds 4 \
    --variants default,default/order1,default/order2 > $O/order_1m.jsonl 2> $O/order_1m.log \
 && timeout -k 10 240 python -u tools/caps_table.py --tag final > $O/caps.jsonl 2> $O/caps.log \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && timeout -k 10 420 python bench.py > $O/bench_default.json 2> $O/bench_default.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
