# GPU BVH builders: their tests, then cornell_1m traversal speed on each tree
# (one perf_ab process per tree) and the bench line with the PLOC build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-bvh}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lbvh.py tests/test_gpu_c4.py -m gpu -q -rA --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for t in ${TREES:-sah gsah ploc}; do
  timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 32 --rounds 3 --bvh $t --variants default > $O/ab_1m_$t.jsonl 2> $O/ab_1m_$t.log || exit $?
  timeout -k 10 300 python tools/perf_ab.py --scene cornell --spp 64 --rounds 3 --bvh $t --variants default > $O/ab_c_$t.jsonl 2> $O/ab_c_$t.log || exit $?
done
timeout -k 10 300 python bench.py --scene cornell_1m --bvh ${BENCH_BVH:-gsah} --steps 3 --warmup 1 --north-star off --cpu-seconds 3 > $O/bench_1m_${BENCH_BVH:-gsah}.json 2> $O/bench_1m_${BENCH_BVH:-gsah}.log
