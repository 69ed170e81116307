# Round 4, second call: GPU suite; veach (C3) with the single-pass fp32
# filter vs the plain fp64 list (experiment build nolf); ray-pool hand-out
# thresholds; shard balance with the whole-frame granule (films identical for
# every shard count); the veach bench line.  Each GPU step time-limited, chained.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 300 python -u tools/perf_ab.py --scene veach --spp 256 --rounds 3 --variants default > $O/ab_veach_filter.jsonl 2> $O/ab_veach.log \
 && FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_nolf.so timeout -k 10 300 python -u tools/perf_ab.py --scene veach --spp 256 --rounds 3 --variants default > $O/ab_veach_nolf.jsonl 2>> $O/ab_veach.log \
 && timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,default/pool1/pmin8,default/pool1/pmin16,default/pool1/pmin32,default/pool2/pmin16 > $O/ab_pool.jsonl 2> $O/ab_pool.log \
 && timeout -k 10 300 python -u tools/shard_balance.py --scene cornell > $O/shard_cornell.json 2> $O/shard_cornell.log \
 && timeout -k 10 400 python -u bench.py --scene veach --spp 1024 > $O/bench_veach.json 2> $O/bench_veach.log
