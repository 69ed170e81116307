# Same-call A/B of source revisions: each revision's package (binding +
# libfrt.so, built out of tree under first_raytracer_amd/build/<rev>/) against
# the in-tree build, alternated, one process per run (tools/perf_ab.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abrev}
mkdir -p $O
rc=0
run() {  # tag, package root or "", scene, spp
  if [ -n "$2" ]; then export FRT_PKG_ROOT=$2; else unset FRT_PKG_ROOT; fi
  timeout -k 10 300 python tools/perf_ab.py --scene $3 --spp $4 --rounds ${ROUNDS:-2} --variants default --bvh gsah >> $O/$1_$3.jsonl 2>> $O/log.txt
}
for rep in 1 2; do
  for sc in ${SCENES:-cornell_1m:256 cornell:512}; do
    scene=${sc%%:*}; spp=${sc##*:}
    run cur "" $scene $spp || { rc=$?; break 2; }
    for r in ${REVS:-r2src r3a}; do
      run $r first_raytracer_amd/build/$r $scene $spp || { rc=$?; break 3; }
    done
  done
done
echo "rc=$rc" > $O/rc.txt
exit $rc
