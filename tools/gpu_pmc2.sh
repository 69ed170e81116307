# PMC characterisation, round 1 part 2: divergence (thread vs wave VALU
# cycles), VMEM latency (level / instructions), L2 hits, per kernel variant.
# Counter-only passes, one rocprofv3 process per pass, each time-limited.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-pmc2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
A="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS"
B="SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS"
C="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_REQ_sum"
run() {  # name, counters, perf_ab args
  timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o run -- python3 tools/perf_ab.py $3 > $OUT/$1.log 2>&1
}
M4="--scene cornell_1m --spp 8 --rounds 1 --variants default"
M2="--scene cornell_1m --spp 8 --rounds 1 --variants bvh2"
CO="--scene cornell --spp 16 --rounds 1 --variants default"
run m4_a "$A" "$M4" && run m4_b "$B" "$M4" && run m4_c "$C" "$M4" \
 && run m2_a "$A" "$M2" && run m2_b "$B" "$M2" && run m2_c "$C" "$M2" \
 && run co_a "$A" "$CO" && run co_b "$B" "$CO"
rc=$?
echo "rc=$rc" > $OUT/rc.txt
exit $rc
