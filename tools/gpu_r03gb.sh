# Round 3 (re-entry): queue grab size around the default 64, final build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03gb}
mkdir -p $O
timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 \
    --variants default,default/grab32,default/grab128 > $O/grab_cornell.jsonl 2>> $O/log.txt \
 && timeout -k 10 200 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --integrator ao \
    --variants default,default/grab32,default/grab128 > $O/grab_ao.jsonl 2>> $O/log.txt \
 && timeout -k 10 400 python -u tools/perf_ab.py --scene cornell_1m --spp 256 --rounds 2 --bvh gsah \
    --variants default,default/grab32,default/grab128 > $O/grab_1m.jsonl 2>> $O/log.txt
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
