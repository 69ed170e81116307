# Round 3 (re-entry): AO on Cornell 1080p 512 spp went 51.3 -> 72.6 ms per launch
# since round 2.  Suspects: the work granule (samples per item) and the basic
# SGPR allocator of the material unit (AO kernels live there).  Main library
# with granule variants, then the greedy-allocator experiment build, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03y}
mkdir -p $O
rc=0
for rep in 1 2; do
  unset FRT_LIB_PATH
  timeout -k 10 200 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 2 --integrator ao \
      --variants default,default/spi512,default/spi171,default/spi64 >> $O/ao_main.jsonl 2>> $O/log.txt || { rc=$?; break; }
  export FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_greedy.so
  timeout -k 10 200 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 2 --integrator ao \
      --variants default,default/spi171 >> $O/ao_greedy.jsonl 2>> $O/log.txt || { rc=$?; break; }
done
echo "rc=$rc" > $O/rc.txt
exit $rc
