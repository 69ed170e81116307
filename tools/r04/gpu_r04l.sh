# Round 4, twelfth call: the GPU suite + smoke with PSS-MLT's one-round
# primary-sample hash (the oracle in lockstep), the PSS-MLT bench line, and its
# kernel-trace and PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O/roof
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
pmc() {  # name, counters, bench args...
  local n=$1 c=$2; shift 2
  timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d $O/roof/$n -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/roof/$n.json 2> $O/roof/$n.log
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && timeout -k 10 400 python -u bench.py --integrator pssmlt > $O/bench_pssmlt.json 2> $O/bench_pssmlt.log \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/roof/trace_pssmlt -o run -- \
      python3 bench.py --integrator pssmlt --steps 3 --warmup 1 --no-cpu-baseline --north-star off > $O/roof/trace_pssmlt.json 2> $O/roof/trace_pssmlt.log \
 && pmc sq_pssmlt "$SQ" --integrator pssmlt && pmc fetch_pssmlt FETCH_SIZE --integrator pssmlt \
 && pmc write_pssmlt WRITE_SIZE --integrator pssmlt
