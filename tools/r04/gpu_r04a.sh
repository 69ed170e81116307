# Round 4, first call: the GPU suite + smoke on the cleaned-up build, the
# ray-pool A/B, the diagnostic build's per-phase lane counts on Cornell at
# 512 spp, the shard-balance measurement (tools/shard_balance.py) on C2 and
# cornell_1m, then the default and veach bench lines.  Every GPU step under
# its own limit, chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,default/pool1,default/pool2,default/pool1/trav12,default/pool1/trav40 > $O/ab_pool.jsonl 2> $O/ab_pool.log \
 && FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_diag.so timeout -k 10 200 python -u tools/diag_phases.py --scene cornell --spp 512 > $O/diag_cornell.json 2> $O/diag_cornell.log \
 && timeout -k 10 300 python -u tools/shard_balance.py --scene cornell > $O/shard_cornell.json 2> $O/shard_cornell.log \
 && timeout -k 10 400 python -u tools/shard_balance.py --scene cornell_1m --reps 1 > $O/shard_1m.json 2> $O/shard_1m.log \
 && timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log \
 && timeout -k 10 400 python -u bench.py --scene veach --spp 1024 > $O/bench_veach.json 2> $O/bench_veach.log \
 && true
# register-cap reproducer (the round-3 state cut, 0a75e3c) under WWM / spill
# allocator options: build/exp/libfrt_{fail,wwmb,wwmf,ssize}.so
[ -f first_raytracer_amd/build/exp/libfrt_fail.so ] && TAG=r04a_caps LIBS="fail wwmb wwmf ssize" bash tools/gpu_caps_exp.sh
