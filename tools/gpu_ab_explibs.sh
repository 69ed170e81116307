# Same-call A/B of experiment builds (first_raytracer_amd/build/exp/libfrt_$NAME.so)
# against the in-tree build, alternated, one process per run (tools/perf_ab.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abexp}
mkdir -p $O
rc=0
run() {  # tag, lib or "", scene, spp
  if [ -n "$2" ]; then export FRT_LIB_PATH=$2; else unset FRT_LIB_PATH; fi
  timeout -k 10 300 python tools/perf_ab.py --scene $3 --spp $4 --rounds ${ROUNDS:-2} --variants ${VARIANTS:-default} --bvh gsah >> $O/$1_$3.jsonl 2>> $O/log.txt
}
for rep in 1 2; do
  for sc in ${SCENES:-cornell_1m:256}; do
    scene=${sc%%:*}; spp=${sc##*:}
    run cur "" $scene $spp || { rc=$?; break 2; }
    for n in $LIBS; do
      run $n first_raytracer_amd/build/exp/libfrt_$n.so $scene $spp || { rc=$?; break 3; }
    done
  done
done
echo "rc=$rc" > $O/rc.txt
exit $rc
