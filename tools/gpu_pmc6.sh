# cornell_1m: instruction mix, issue vs wait for the 4-wide and binary BVH
# plans (one perf_ab process per counter pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmc6}
mkdir -p $O
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
B="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"
run() { timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- python3 tools/perf_ab.py $3 > $O/$1.log 2>&1; }
run d_a "$A" "--scene cornell_1m --spp 8 --rounds 1 --variants default" \
 && run d_b "$B" "--scene cornell_1m --spp 8 --rounds 1 --variants default" \
 && run b_a "$A" "--scene cornell_1m --spp 8 --rounds 1 --variants bvh2" \
 && run b_b "$B" "--scene cornell_1m --spp 8 --rounds 1 --variants bvh2"
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
