# Round 4, twenty-first call: LDS counters of the LDS-resident kernels (Cornell
# path, PSS-MLT): bank-conflict and unaligned-stall cycles against all LDS-array
# cycles, to see whether the node loop's LDS reads replay; then the same for the
# octant plan with an odd copy stride (build/exp/libfrt_octodd.so,
# FRT_EXP_OCT_ODD) and a same-call A/B of the two.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04u; mkdir -p $O
E=first_raytracer_amd/build/exp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQ_LDS[A-Z_]*\|SQ_WAIT_INST_LDS\|SQ_INSTS_LDS" $O/counters.txt | sort -u > $O/lds_counters.txt || true
LDS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
pmc() {  # name, bench args...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc $LDS --output-format csv -d $O/$n -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --north-star off "$@" > $O/$n.json 2> $O/$n.log
}
V="--scene cornell --spp 512 --rounds 3 --variants default"
pmc lds_cornell --spp 128 && pmc lds_pssmlt --integrator pssmlt \
 && FRT_LIB_PATH=$E/libfrt_octodd.so pmc lds_cornell_octodd --spp 128 \
 && timeout -k 10 200 python -u tools/perf_ab.py $V >> $O/ab_oct.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_octodd.so timeout -k 10 200 python -u tools/perf_ab.py $V >> $O/ab_oct.jsonl 2>> $O/ab.log \
 && timeout -k 10 200 python -u tools/perf_ab.py $V >> $O/ab_oct.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_octodd.so timeout -k 10 200 python -u tools/perf_ab.py $V >> $O/ab_oct.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_octodd.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity_octodd.txt 2>&1
