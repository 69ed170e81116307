# Work-queue bands A/B (FRT_QUEUE_BANDS 1 vs 8), alternated, one process per
# run (tools/perf_ab.py), after the band-invariance GPU test.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abbands}
mkdir -p $O
rc=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "bands or trav_min" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || rc=$?
run() {  # bands, scene, spp
  FRT_QUEUE_BANDS=$1 timeout -k 10 300 python tools/perf_ab.py --scene $2 --spp $3 --rounds ${ROUNDS:-2} --variants default --bvh gsah >> $O/b$1_$2.jsonl 2>> $O/log.txt
}
if [ $rc = 0 ]; then
  for rep in 1 2; do
    for sc in ${SCENES:-cornell_1m:256 cornell:512}; do
      scene=${sc%%:*}; spp=${sc##*:}
      run 1 $scene $spp && run 8 $scene $spp || { rc=$?; break 2; }
    done
  done
fi
echo "rc=$rc" > $O/rc.txt
exit $rc
