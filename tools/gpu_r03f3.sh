# Round 3 (re-entry), final build (queue grabs + samples-per-item target):
# roofline passes of the default command (Cornell, cornell_1m) and its
# kernel-trace summary, then the AO / normals lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03f3}
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
b() { name=$1; shift; timeout -k 10 300 python bench.py --steps 2 --warmup 1 --north-star off --cpu-seconds 3 "$@" > $O/line_$name.json 2> $O/line_$name.log; }
trace default 420 --steps 5 --warmup 1 \
 && pmc sq_cornell "$SQ" && pmc fetch_cornell FETCH_SIZE && pmc write_cornell WRITE_SIZE \
 && pmc sq_1m "$SQ" --scene cornell_1m && pmc fetch_1m FETCH_SIZE --scene cornell_1m \
 && pmc write_1m WRITE_SIZE --scene cornell_1m && pmc tcc_1m "TCC_HIT TCC_MISS" --scene cornell_1m \
 && b ao --integrator ao && b normals --integrator normals && b veach --scene veach --spp 1024
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
