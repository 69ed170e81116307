# Round 3 (re-entry): the HBM plan's register cap re-checked on the current
# build at the north-star config (cornell_1m 1080p 512 spp): 6 waves (14
# spilled VGPRs, ~2.7 MB of scratch per XCD against a 4 MB L2) vs 5 waves.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03w}
mkdir -p $O
timeout -k 10 400 python -u tools/perf_ab.py --scene cornell_1m --spp 512 --rounds 3 --bvh gsah \
    --variants default,waves5,spec > $O/waves_1m_512.jsonl 2> $O/waves_1m_512.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
