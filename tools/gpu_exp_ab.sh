# Code-variant timing: perf_ab with the default libfrt.so and each experiment
# build (first_raytracer_amd/build/exp/libfrt_<name>.so, Makefile `exp`),
# alternated twice, one process per run.  EXPS="branchy cheaprng".
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-expab}
mkdir -p $O
run() {  # tag, lib or "", scene, spp
  if [ -n "$2" ]; then export FRT_LIB_PATH=$2; else unset FRT_LIB_PATH; fi
  timeout -k 10 200 python tools/perf_ab.py --scene $3 --spp $4 --rounds 3 --variants default >> $O/$1_$3.jsonl 2>> $O/log.txt
}
rc=0
for rep in 1 2; do
  for scene in cornell cornell_1m; do
    spp=64; [ $scene = cornell_1m ] && spp=16
    run base "" $scene $spp || { rc=$?; break 2; }
    for e in ${EXPS:-branchy}; do
      run $e first_raytracer_amd/build/exp/libfrt_$e.so $scene $spp || { rc=$?; break 3; }
    done
  done
done
echo "rc=$rc" > $O/rc.txt
exit $rc
