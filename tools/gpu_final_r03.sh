# Round 3, final build: caps table, the full -m gpu suite, smoke(), then the
# default bench line (Cornell + north star), veach and PSS-MLT lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03final}
mkdir -p $O
timeout -k 10 240 python -u tools/caps_table.py --tag final > $O/caps.jsonl 2> $O/caps.log \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && timeout -k 10 420 python bench.py > $O/bench_default.json 2> $O/bench_default.log \
 && timeout -k 10 300 python bench.py --scene veach --spp 1024 --steps 3 > $O/bench_veach.json 2> $O/bench_veach.log \
 && timeout -k 10 300 python bench.py --integrator pssmlt --steps 3 > $O/bench_pssmlt.json 2> $O/bench_pssmlt.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
