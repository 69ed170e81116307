# Round 4, sixth call: the GPU suite + smoke on the build whose 4-wide traversal
# keeps one leaf loop for both primitive kinds (spills 24 -> 17 VGPRs); same-call
# A/B against the r04e build (build/exp/libfrt_r04e.so) on cornell_1m and
# Cornell; the shard balance of the bench config under smaller work items
# (FRT_SPI_TARGET 12 and 8 samples an item against the default 24); the
# cornell_1m PMC passes on this build; the veach and PSS-MLT roofline passes
# (tools/gpu_roofline.sh PART=b).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04f; mkdir -p $O
E=first_raytracer_amd/build/exp
ab() {  # tag, lib ('' = in-tree), perf_ab args...
  local t=$1 l=$2; shift 2
  if [ -n "$l" ]; then FRT_LIB_PATH=$E/$l timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log
  else timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log; fi
}
C="--scene cornell --spp 512 --rounds 2 --bvh gsah --variants default"
M="--scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
pmc() {  # name, counters, bench args...
  local n=$1 c=$2; shift 2
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d $O/roof/$n -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/roof/$n.json 2> $O/roof/$n.log
}
mkdir -p $O/roof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && ab m "" $M && ab m libfrt_r04e.so $M && ab m "" $M && ab m libfrt_r04e.so $M \
 && ab c "" $C && ab c libfrt_r04e.so $C \
 && timeout -k 10 300 python -u tools/shard_balance.py --scene cornell > $O/shard_cornell_spt24.json 2> $O/shard.log \
 && FRT_SPI_TARGET=12 timeout -k 10 300 python -u tools/shard_balance.py --scene cornell > $O/shard_cornell_spt12.json 2>> $O/shard.log \
 && FRT_SPI_TARGET=8 timeout -k 10 300 python -u tools/shard_balance.py --scene cornell > $O/shard_cornell_spt8.json 2>> $O/shard.log \
 && pmc sq_1m "$SQ" --scene cornell_1m && pmc fetch_1m FETCH_SIZE --scene cornell_1m \
 && pmc write_1m WRITE_SIZE --scene cornell_1m && pmc tcc_1m "TCC_HIT TCC_MISS" --scene cornell_1m \
 && TAG=r04f/roofb PART=b bash tools/gpu_roofline.sh
