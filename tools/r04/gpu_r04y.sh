# Round 4, twenty-fifth call: wave priority by megakernel phase (s_setprio),
# experiment builds build/exp/libfrt_prio{1,2}.so (FRT_EXP_PRIO: 1 = shading
# phase first, 2 = traversal phase first) against the in-tree library,
# alternated in one call: Cornell 512 spp and cornell_1m 256 spp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04y; mkdir -p $O
E=first_raytracer_amd/build/exp
C="--scene cornell --spp 512 --rounds 3 --variants default"
M="--scene cornell_1m --spp 256 --rounds 2 --variants default"
ab() {  # lib, args...
  local lib=$1; shift
  if [ "$lib" = base ]; then timeout -k 10 300 python -u tools/perf_ab.py "$@" | sed "s/^{/{\"lib\": \"$lib\", /" >> $O/ab.jsonl
  else FRT_LIB_PATH=$E/libfrt_$lib.so timeout -k 10 300 python -u tools/perf_ab.py "$@" | sed "s/^{/{\"lib\": \"$lib\", /" >> $O/ab.jsonl; fi
}
ab base $C && ab prio1 $C && ab prio2 $C && ab base $C && ab prio1 $C && ab prio2 $C \
 && ab base $M && ab prio1 $M && ab prio2 $M
