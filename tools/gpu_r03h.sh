# Round 3: register caps incl. the reinstated 6-wave specular kernels
# (test_register_caps_agree + the conductor probe), the ray-query kernel with
# per-lane ray prefetch (tests + throughput on large batches).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03h}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_conductors.py tests/test_gpu_trace.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
 && PROBE_FLAGS=1,17,0 PROBE_CAPS=3,4,5,6 timeout -k 10 300 python tools/probe_conductors.py > $O/probe_caps.txt 2>&1 \
 && timeout -k 10 400 python tools/trace_bench.py --scene cornell_1m --rays-per-pixel 32 --rounds 2 > $O/trace_1m.jsonl 2> $O/trace_1m.log \
 && timeout -k 10 300 python tools/trace_bench.py --scene cornell --rays-per-pixel 32 --rounds 2 > $O/trace_cornell.jsonl 2> $O/trace_cornell.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
