# Round 4, fourth call: the GPU suite + smoke on the build whose triangle leaves
# skip the sphere test and whose straight-line triangle test is used by the
# 4-wide traversal only; same-call A/B on Cornell (in-tree vs build/exp/
# libfrt_slabnf.so, the r04c build without either) and cornell_1m (in-tree vs
# libfrt_tribf.so, the r04c build); PSS-MLT cost attribution: timing builds
# that skip one part of the chain kernel each (invalid films, timing only):
# libfrt_noload (primary samples not read or mutated), libfrt_nomat (small-step
# accepts not materialised), libfrt_nosplat (no splats), against libfrt_mltbase
# (the same source unchanged).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
E=first_raytracer_amd/build/exp
ab() {  # tag, lib ('' = in-tree), perf_ab args...
  local t=$1 l=$2; shift 2
  if [ -n "$l" ]; then FRT_LIB_PATH=$E/$l timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log
  else timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log; fi
}
C="--scene cornell --spp 512 --rounds 3 --bvh gsah --variants default"
M="--scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default"
P="--scene cornell --spp 512 --rounds 2 --bvh gsah --integrator pssmlt --variants default"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && ab c "" $C && ab c libfrt_slabnf.so $C && ab c "" $C && ab c libfrt_slabnf.so $C \
 && ab m "" $M && ab m libfrt_tribf.so $M \
 && ab mlt "" $P && ab mlt libfrt_mltbase.so $P && ab mlt libfrt_noload.so $P \
 && ab mlt libfrt_nomat.so $P && ab mlt libfrt_nosplat.so $P
