# Round 4, seventeenth call (final build): kernel-trace and PMC passes of veach
# and PSS-MLT (tools/gpu_roofline.sh PART=b) and of AO and normals.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04q; mkdir -p $O/roof
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
pmc() {  # name, counters, bench args...
  local n=$1 c=$2; shift 2
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d $O/roof/$n -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/roof/$n.json 2> $O/roof/$n.log
}
TAG=r04q/roofb PART=b bash tools/gpu_roofline.sh \
 && pmc sq_ao "$SQ" --integrator ao && pmc fetch_ao FETCH_SIZE --integrator ao && pmc write_ao WRITE_SIZE --integrator ao \
 && pmc sq_normals "$SQ" --integrator normals && pmc fetch_normals FETCH_SIZE --integrator normals \
 && pmc write_normals WRITE_SIZE --integrator normals
rc=$?
# veach's fp64 list kernel (modified_phong set: 248 VGPRs, 2 waves/SIMD) under a
# 3-wave cap (168 VGPRs, 70 spilled): build/exp/libfrt_f64w3.so vs libfrt_f64w1.so
E=first_raytracer_amd/build/exp
V="--scene veach --spp 256 --rounds 3 --variants default"
[ $rc = 0 ] && FRT_LIB_PATH=$E/libfrt_f64w1.so timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64w.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_f64w3.so timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64w.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_f64w1.so timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64w.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_f64w3.so timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64w.jsonl 2>> $O/ab.log
rc=$?
# rehearsal of the N-rank bench path (tools/gpu_multirank.sh: 2 ranks on the one
# GPU, gloo collectives) on the final build
[ $rc = 0 ] && TAG=r04q/mr bash tools/gpu_multirank.sh
