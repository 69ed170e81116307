# Guided granule A/B (FRT_GRANULE=guided: chunk-major items, chunk lengths
# falling linearly) against the default equal-chunk granule, one process per
# scene, interleaved rounds (tools/perf_ab.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-guided}
mkdir -p $O
V="default,default/granguided,default/granguided/gk8,default/granguided/gk16,default/granguided/gk32"
timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 5 --variants $V > $O/cornell.jsonl 2> $O/cornell.log \
 && timeout -k 10 400 python -u tools/perf_ab.py --scene cornell_1m --spp 512 --rounds 3 --variants $V > $O/cornell_1m.jsonl 2> $O/cornell_1m.log \
 && timeout -k 10 300 python -u tools/perf_ab.py --scene veach --spp 1024 --rounds 3 --variants $V > $O/veach.jsonl 2> $O/veach.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
