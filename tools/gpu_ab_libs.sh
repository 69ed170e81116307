# Same-call A/B of two library builds at the bench's 1080p config: the
# default libfrt.so ("new") against first_raytracer_amd/build/exp/libfrt_$BASE.so
# ("base"), alternated, one process per run (tools/perf_ab.py), on Cornell at
# 512 spp and cornell_1m at $SPP_1M spp; then WRITE_SIZE / FETCH_SIZE passes of
# the new build on both scenes (bench.py, 1 frame).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ablibs}
mkdir -p $O
BASE=${BASE:-base}
run() {  # tag, lib or "", scene, spp
  if [ -n "$2" ]; then export FRT_LIB_PATH=$2; else unset FRT_LIB_PATH; fi
  timeout -k 10 300 python tools/perf_ab.py --scene $3 --spp $4 --rounds ${ROUNDS:-2} --variants default --bvh gsah >> $O/$1_$3.jsonl 2>> $O/log.txt
}
pmc() {  # name, counters, scene, spp
  unset FRT_LIB_PATH
  timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- \
      python3 bench.py --scene $3 --spp $4 --steps 1 --warmup 0 --no-cpu-baseline --north-star off > $O/$1.json 2> $O/$1.log
}
rc=0
for rep in 1 2; do
  for scene in cornell cornell_1m; do
    spp=512; [ $scene = cornell_1m ] && spp=${SPP_1M:-256}
    run base first_raytracer_amd/build/exp/libfrt_$BASE.so $scene $spp || { rc=$?; break 2; }
    run new "" $scene $spp || { rc=$?; break 2; }
  done
done
if [ $rc = 0 ] && [ "${PMC:-1}" = 1 ]; then
  pmc write_1m WRITE_SIZE cornell_1m 128 && pmc write_cornell WRITE_SIZE cornell 128 \
    && pmc fetch_1m FETCH_SIZE cornell_1m 128
  rc=$?
fi
echo "rc=$rc" > $O/rc.txt
exit $rc
