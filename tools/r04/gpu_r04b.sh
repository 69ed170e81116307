# Round 4, second call: GPU suite on the current build; the slab tests on
# v_maximum3 / v_minimum3 (this build) against the previous build
# (build/exp/libfrt_r04b0.so) and the build with leaf postponing compiled out
# of the LDS plans (build/exp/libfrt_md.so) on Cornell and cornell_1m; veach (C3) with the
# single-pass fp32 filter vs the plain fp64 list (build/exp/libfrt_nolf.so);
# ray-pool hand-out thresholds; shard balance with the whole-frame granule
# (films identical for every shard count); the veach bench line.  Each GPU
# step time-limited, chained.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
E=first_raytracer_amd/build/exp
ab() {  # tag, lib ('' = in-tree), perf_ab args...
  local t=$1 l=$2; shift 2
  if [ -n "$l" ]; then FRT_LIB_PATH=$E/$l timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log
  else timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log; fi
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && ab smax "" --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default \
 && ab smax libfrt_r04b0.so --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default \
 && ab smax libfrt_md.so --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default \
 && ab smax "" --scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default \
 && ab smax libfrt_r04b0.so --scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default \
 && ab smax libfrt_md.so --scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default \
 && ab smax "" --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default \
 && ab smax libfrt_r04b0.so --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default \
 && ab smax libfrt_md.so --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default \
 && ab veach "" --scene veach --spp 256 --rounds 3 --variants default \
 && ab veach libfrt_nolf.so --scene veach --spp 256 --rounds 3 --variants default \
 && ab pool "" --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,default/pool1/pmin8,default/pool1/pmin16,default/pool1/pmin32,default/pool2/pmin16 \
 && timeout -k 10 300 python -u tools/shard_balance.py --scene cornell > $O/shard_cornell.json 2> $O/shard_cornell.log \
 && timeout -k 10 400 python -u bench.py --scene veach --spp 1024 > $O/bench_veach.json 2> $O/bench_veach.log
