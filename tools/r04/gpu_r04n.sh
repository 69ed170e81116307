# Round 4, fourteenth call: the GPU suite + smoke with one mix32 round per
# random number (kernel and oracle changed together); the default and PSS-MLT
# bench lines; cornell_1m min_desc 8 / 12 / 16 at 512 spp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && timeout -k 10 420 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log \
 && timeout -k 10 400 python -u bench.py --integrator pssmlt > $O/bench_pssmlt.json 2> $O/bench_pssmlt.log \
 && timeout -k 10 400 python -u tools/perf_ab.py --scene cornell_1m --spp 512 --rounds 2 --bvh gsah \
      --variants default,default/desc12,default/desc16 > $O/ab_1m_desc.jsonl 2> $O/ab.log
