# Round 4, fifteenth call: the GPU suite + smoke on the build whose octant node
# records are regrouped into plane pairs for packed FMAs (6 v_pk_fma_f32 per
# node instead of 12 v_fma_f32) and whose HBM plans postpone leaves at 12;
# same-call A/B against the r04n build (build/exp/libfrt_rng1.so) on every
# LDS-plan integrator (path, PSS-MLT, AO, normals) and cornell_1m.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04o; mkdir -p $O
E=first_raytracer_amd/build/exp
ab() {  # tag, lib ('' = in-tree), perf_ab args...
  local t=$1 l=$2; shift 2
  if [ -n "$l" ]; then FRT_LIB_PATH=$E/$l timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log
  else timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log; fi
}
C="--scene cornell --spp 512 --rounds 3 --bvh gsah --variants default"
M="--scene cornell_1m --spp 512 --rounds 1 --bvh gsah --variants default"
P="--scene cornell --spp 512 --rounds 2 --bvh gsah --integrator pssmlt --variants default"
A="--scene cornell --spp 512 --rounds 3 --bvh gsah --integrator ao --variants default"
N="--scene cornell --spp 512 --rounds 3 --bvh gsah --integrator normals --variants default"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && ab c "" $C && ab c libfrt_rng1.so $C && ab c "" $C && ab c libfrt_rng1.so $C \
 && ab m "" $M && ab m libfrt_rng1.so $M \
 && ab mlt "" $P && ab mlt libfrt_rng1.so $P \
 && ab ao "" $A && ab ao libfrt_rng1.so $A && ab nrm "" $N && ab nrm libfrt_rng1.so $N
rc=$?
# the 4-wide node test's plane pairs as packed FMAs too (build/exp/libfrt_pk4.so:
# this source + 3 v_pk_fma_f32 per child instead of 6 v_fma_f32; round 3 measured
# a similar build 3 % slower)
[ $rc = 0 ] && ab m4 "" --scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default \
 && ab m4 libfrt_pk4.so --scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default \
 && ab m4 "" --scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default \
 && ab m4 libfrt_pk4.so --scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default
