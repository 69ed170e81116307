# GPU parity suite of the current tree, then the bench lines of the default
# run (Cornell C2 + the cornell_1m north-star block).  Every GPU step under
# its own time limit; chained with && so the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-suite}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" > $O/rc.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi   # 1 = test failures: still bench; anything else (fault, timeout) stops
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.log
rc2=$?
echo "bench rc=$rc2" >> $O/rc.txt
exit $(( rc > rc2 ? rc : rc2 ))
