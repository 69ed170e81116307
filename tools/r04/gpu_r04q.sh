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
