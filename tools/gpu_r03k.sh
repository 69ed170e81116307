# Round 3: caps table (tools/caps_table.py) of the in-tree build, then the
# full -m gpu suite (every test, no -x: one line per result in the log).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03k}
mkdir -p $O
timeout -k 10 240 python -u tools/caps_table.py --tag cur > $O/caps.jsonl 2> $O/caps.log \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
