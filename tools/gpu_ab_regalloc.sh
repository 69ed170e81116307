# Register allocator A/B: the in-tree build (greedy allocators) against
# builds of the same source with the basic SGPR or VGPR allocator
# (first_raytracer_amd/build/exp/libfrt_cur_{sbasic,vbasic}.so): the caps table
# of each, then alternated timing (tools/perf_ab.py) on Cornell 512 spp,
# cornell_1m 256 spp and veach 256 spp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abra}
mkdir -p $O
rc=0
for n in cur_sbasic cur_vbasic; do
  FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_$n.so timeout -k 10 240 python -u tools/caps_table.py --tag $n >> $O/caps.jsonl 2>> $O/log.txt || { rc=$?; break; }
done
run() {  # tag, lib or "", scene, spp
  if [ -n "$2" ]; then export FRT_LIB_PATH=$2; else unset FRT_LIB_PATH; fi
  timeout -k 10 300 python tools/perf_ab.py --scene $3 --spp $4 --rounds ${ROUNDS:-2} --variants default --bvh gsah >> $O/$1_$3.jsonl 2>> $O/log.txt
}
if [ $rc = 0 ]; then
  for rep in 1 2; do
    for sc in cornell:512 cornell_1m:256 veach:256; do
      scene=${sc%%:*}; spp=${sc##*:}
      run greedy "" $scene $spp || { rc=$?; break 2; }
      run sbasic first_raytracer_amd/build/exp/libfrt_cur_sbasic.so $scene $spp || { rc=$?; break 2; }
      run vbasic first_raytracer_amd/build/exp/libfrt_cur_vbasic.so $scene $spp || { rc=$?; break 2; }
    done
  done
fi
echo "rc=$rc" > $O/rc.txt
exit $rc
