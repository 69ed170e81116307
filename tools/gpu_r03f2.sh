# Round 3 (re-entry), final build (64 items per queue grab): -m gpu suite,
# smoke(), roofline passes of the default command (Cornell, cornell_1m) and of
# veach, then the AO / normals lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03f2}
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
b() { name=$1; shift; timeout -k 10 300 python bench.py --steps 2 --warmup 1 --north-star off --cpu-seconds 3 "$@" > $O/line_$name.json 2> $O/line_$name.log; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && trace default 420 --steps 5 --warmup 1 \
 && pmc sq_cornell "$SQ" && pmc fetch_cornell FETCH_SIZE && pmc write_cornell WRITE_SIZE \
 && pmc sq_1m "$SQ" --scene cornell_1m && pmc fetch_1m FETCH_SIZE --scene cornell_1m \
 && pmc write_1m WRITE_SIZE --scene cornell_1m && pmc tcc_1m "TCC_HIT TCC_MISS" --scene cornell_1m \
 && trace veach 300 --scene veach --spp 1024 --steps 3 --warmup 1 --no-cpu-baseline --north-star off \
 && pmc sq_veach "$SQ" --scene veach --spp 1024 && pmc fetch_veach FETCH_SIZE --scene veach --spp 1024 \
 && pmc write_veach WRITE_SIZE --scene veach --spp 1024 && pmc f64_veach "$F64" --scene veach --spp 1024 \
 && b ao --integrator ao && b normals --integrator normals && b ao_1m --scene cornell_1m --integrator ao --spp 256
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
