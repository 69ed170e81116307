# Round 4, seventh call: work-item size vs the N-way split (whole-frame chunks,
# so films stay identical for every shard count): the bench configs at N = 1
# with 8 samples an item (29 chunks under the 192-items-per-lane cap) and with
# the cap raised to 384 (build/exp/libfrt_cap384.so: 57 chunks), and the shard
# balance of both; PSS-MLT register caps 4 / 6 (libfrt_mltw4 / mltw6) and
# trav_min; the AO and normals PMC passes on the round-4 build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O/roof
E=first_raytracer_amd/build/exp
ab() {  # tag, lib ('' = in-tree), perf_ab args...
  local t=$1 l=$2; shift 2
  if [ -n "$l" ]; then FRT_LIB_PATH=$E/$l timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log
  else timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log; fi
}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
pmc() {  # name, counters, bench args...
  local n=$1 c=$2; shift 2
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d $O/roof/$n -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/roof/$n.json 2> $O/roof/$n.log
}
P="--scene cornell --spp 512 --rounds 2 --bvh gsah --integrator pssmlt"
ab c "" --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default,default/spt8 \
 && ab c libfrt_cap384.so --scene cornell --spp 512 --rounds 3 --bvh gsah --variants default/spt8 \
 && ab m "" --scene cornell_1m --spp 512 --rounds 1 --bvh gsah --variants default,default/spt8 \
 && ab m libfrt_cap384.so --scene cornell_1m --spp 512 --rounds 1 --bvh gsah --variants default/spt8 \
 && FRT_LIB_PATH=$E/libfrt_cap384.so FRT_SPI_TARGET=8 timeout -k 10 300 python -u tools/shard_balance.py --scene cornell > $O/shard_cornell_cap384_spt8.json 2> $O/shard.log \
 && FRT_LIB_PATH=$E/libfrt_cap384.so FRT_SPI_TARGET=8 timeout -k 10 300 python -u tools/shard_balance.py --scene cornell_1m --reps 1 > $O/shard_1m_cap384_spt8.json 2>> $O/shard.log \
 && FRT_SPI_TARGET=8 timeout -k 10 300 python -u tools/shard_balance.py --scene cornell_1m --reps 1 > $O/shard_1m_spt8.json 2>> $O/shard.log \
 && ab mlt "" $P --variants default,default/trav6,default/trav20,default/trav28 \
 && ab mlt libfrt_mltw4.so $P --variants default && ab mlt libfrt_mltw6.so $P --variants default \
 && ab mlt "" $P --variants default \
 && pmc sq_ao "$SQ" --integrator ao && pmc fetch_ao FETCH_SIZE --integrator ao && pmc write_ao WRITE_SIZE --integrator ao \
 && pmc sq_normals "$SQ" --integrator normals && pmc fetch_normals FETCH_SIZE --integrator normals \
 && pmc write_normals WRITE_SIZE --integrator normals
