# PSS-MLT code-variant timing: bench.py --integrator pssmlt with the default
# libfrt.so and each experiment build, alternated twice.  EXPS="mltw5 mltw6".
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-expmlt}
mkdir -p $O
run() {
  if [ -n "$2" ]; then export FRT_LIB_PATH=$2; else unset FRT_LIB_PATH; fi
  timeout -k 10 200 python bench.py --integrator pssmlt --steps 2 --warmup 1 --no-cpu-baseline >> $O/$1.jsonl 2>> $O/log.txt
}
rc=0
for rep in 1 2; do
  run base "" || { rc=$?; break; }
  for e in ${EXPS:-mltw5}; do
    run $e first_raytracer_amd/build/exp/libfrt_$e.so || { rc=$?; break 2; }
  done
done
echo "rc=$rc" > $O/rc.txt
exit $rc
