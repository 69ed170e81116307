# Round 3 (re-entry): PMC passes for the AO and normals bench lines, so every
# line carries a counter-based roofline (tools/roofline_pmc.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03ao}
mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
trace() {  # name, seconds, bench args...
  local n=$1 s=$2; shift 2
  timeout -k 10 $s rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n -o run -- \
      python3 bench.py "$@" > $O/trace_$n.json 2> $O/trace_$n.log
}
pmc() {  # name, counters, bench args...
  local n=$1 c=$2; shift 2
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d $O/$n -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
}
pmc sq_ao "$SQ" --integrator ao && pmc fetch_ao FETCH_SIZE --integrator ao && pmc write_ao WRITE_SIZE --integrator ao \
 && pmc sq_normals "$SQ" --integrator normals && pmc fetch_normals FETCH_SIZE --integrator normals \
 && pmc write_normals WRITE_SIZE --integrator normals \
 && trace ao 300 --integrator ao --steps 3 --warmup 1 --no-cpu-baseline --north-star off \
 && trace normals 300 --integrator normals --steps 3 --warmup 1 --no-cpu-baseline --north-star off
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
