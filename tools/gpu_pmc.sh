# PMC characterisation of the path / MLT kernels: SQ instruction mix and cycles,
# LDS and L2 behaviour.  Counter-only passes (no trace domains), one rocprofv3
# process per pass, each time-limited; chained.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run() {  # name, counters, perf_ab args
  timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o run -- python3 tools/perf_ab.py $3 > $OUT/$1.log 2>&1
}
run c_sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "--scene cornell --spp 16 --rounds 1 --variants default" \
 && run c_sq2 "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" "--scene cornell --spp 16 --rounds 1 --variants default" \
 && run m_sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "--scene cornell_1m --spp 8 --rounds 1 --variants default" \
 && run m_sq2 "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM TCC_HIT_sum TCC_MISS_sum" "--scene cornell_1m --spp 8 --rounds 1 --variants default"
rc=$?
echo "rc=$rc" > $OUT/rc.txt
exit $rc
