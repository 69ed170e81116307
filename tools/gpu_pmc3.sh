# Is the cornell_1m traffic scratch?  FETCH/WRITE per dispatch for kernel
# variants with and without scratch (register caps, 4-wide overflow stack).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmc3}
mkdir -p $O
V="default,bvh2,waves4,bvh2+waves4"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 tools/perf_ab.py --scene cornell_1m --spp 16 --rounds 1 --variants $V > $O/fetch.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 tools/perf_ab.py --scene cornell_1m --spp 16 --rounds 1 --variants $V > $O/write.log 2>&1 \
 && timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $O/ea -o run -- python3 tools/perf_ab.py --scene cornell_1m --spp 16 --rounds 1 --variants $V > $O/ea.log 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
