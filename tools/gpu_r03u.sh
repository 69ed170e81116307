# Round 3 (re-entry): does the LDS plan gain from a 6th wave per SIMD?  The
# octant copies hold Cornell's blocks to 5 per CU by LDS (30 KiB each);
# without them 6 blocks fit.  Same process, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03u}
mkdir -p $O
timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 4 \
    --variants default,waves6,no_oct,no_oct+waves6,waves4 > $O/lds_waves.jsonl 2> $O/lds_waves.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
