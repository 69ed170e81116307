# Round 3 (re-entry), final: PSS-MLT roofline passes on the current build (its
# chain kernel changed: flat row materialisation), kernel-trace summaries of the
# default and PSS-MLT bench commands, then the -m gpu suite and smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03x}
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
trace pssmlt 300 --integrator pssmlt --steps 3 --warmup 1 --no-cpu-baseline --north-star off \
 && pmc sq_pssmlt "$SQ" --integrator pssmlt && pmc fetch_pssmlt FETCH_SIZE --integrator pssmlt \
 && pmc write_pssmlt WRITE_SIZE --integrator pssmlt \
 && trace default 420 --steps 5 --warmup 1 \
 && timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
