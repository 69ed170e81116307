# Round-3 roofline evidence for bench.py, on the final build:
#  * kernel-trace + stats of the default bench command (Cornell + the
#    cornell_1m north-star block), of veach (fp64 list world) and of PSS-MLT
#    on Cornell -- the launch averages bench.py's roofline divides by;
#  * per config the PMC passes tools/roofline_pmc.py reads, one counter group
#    per run (MI355X_MICROARCH.md PMC slots): SQ issue counters, FETCH_SIZE,
#    WRITE_SIZE; cornell_1m adds TCC_HIT/TCC_MISS, veach the fp64 VALU
#    counters.
# PART=a: default bench + Cornell / cornell_1m passes; PART=b: veach and
# PSS-MLT.  Chained with &&: the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03roof}
mkdir -p $O
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
F64="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64"
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
if [ "${PART:-a}" = a ]; then
  trace default 420 --steps ${STEPS:-5} --warmup 1 \
   && pmc sq_cornell "$SQ" && pmc fetch_cornell FETCH_SIZE && pmc write_cornell WRITE_SIZE \
   && pmc sq_1m "$SQ" --scene cornell_1m && pmc fetch_1m FETCH_SIZE --scene cornell_1m \
   && pmc write_1m WRITE_SIZE --scene cornell_1m && pmc tcc_1m "TCC_HIT TCC_MISS" --scene cornell_1m
else
  trace veach 300 --scene veach --spp 1024 --steps 3 --warmup 1 --no-cpu-baseline --north-star off \
   && trace pssmlt 300 --integrator pssmlt --steps 3 --warmup 1 --no-cpu-baseline --north-star off \
   && pmc sq_veach "$SQ" --scene veach --spp 1024 && pmc fetch_veach FETCH_SIZE --scene veach --spp 1024 \
   && pmc write_veach WRITE_SIZE --scene veach --spp 1024 && pmc f64_veach "$F64" --scene veach --spp 1024 \
   && pmc sq_pssmlt "$SQ" --integrator pssmlt && pmc fetch_pssmlt FETCH_SIZE --integrator pssmlt \
   && pmc write_pssmlt WRITE_SIZE --integrator pssmlt
fi
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
