# Round 4, third call: the GPU suite + smoke on the build with the octant
# plan's 48-B node records (one LDS address per node step), its interval hit
# test (slab_nf: tn <= tf), the branch-free fp32 triangle test, leaf postponing
# compiled out of the LDS plans, and the list filter and the ray pool removed.
# Same-call A/B of the steps on Cornell: in-tree = all, build/exp/
# libfrt_slabnf.so = without the triangle test, libfrt_oct48.so = without
# slab_nf either, libfrt_md.so = the r04b build with leaf postponing compiled
# out (before the 48-B records); cornell_1m in-tree vs md; veach in-tree vs
# the r04b plain-list build (libfrt_nolf.so); the default and veach bench
# lines; shard balance on cornell_1m with the whole-frame work granule.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
E=first_raytracer_amd/build/exp
ab() {  # tag, lib ('' = in-tree), perf_ab args...
  local t=$1 l=$2; shift 2
  if [ -n "$l" ]; then FRT_LIB_PATH=$E/$l timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log
  else timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_$t.jsonl 2>> $O/ab.log; fi
}
C="--scene cornell --spp 512 --rounds 3 --bvh gsah --variants default"
M="--scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && ab c "" $C && ab c libfrt_slabnf.so $C && ab c libfrt_oct48.so $C && ab c libfrt_md.so $C \
 && ab c "" $C && ab c libfrt_slabnf.so $C && ab c libfrt_oct48.so $C && ab c libfrt_md.so $C \
 && ab m "" $M && ab m libfrt_md.so $M \
 && ab veach "" --scene veach --spp 256 --rounds 3 --variants default \
 && ab veach libfrt_nolf.so --scene veach --spp 256 --rounds 3 --variants default \
 && timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log \
 && timeout -k 10 300 python -u bench.py --scene veach --spp 1024 > $O/bench_veach.json 2> $O/bench_veach.log \
 && timeout -k 10 300 python -u tools/shard_balance.py --scene cornell_1m --reps 1 > $O/shard_1m.json 2> $O/shard_1m.log
