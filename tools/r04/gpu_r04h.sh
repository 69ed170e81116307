# Round 4, eighth call: the GPU suite + smoke on the build with 8-sample path
# items (at most 384 items per lane) and the 4-wave PSS-MLT cap; the bench
# lines (default = Cornell + the cornell_1m north star, veach, PSS-MLT, AO,
# normals); Cornell trav_min and leaf-size re-checks on the round-4 node loop.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
b() {  # name, seconds, bench args...
  local n=$1 s=$2; shift 2
  timeout -k 10 $s python -u bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.log
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && b default 420 \
 && b veach 300 --scene veach --spp 1024 \
 && b pssmlt 400 --integrator pssmlt \
 && b ao 200 --integrator ao \
 && b normals 200 --integrator normals \
 && timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --bvh gsah \
      --variants default,default/trav20,default/trav36,default/leaf1,default/leaf3 > $O/ab_knobs.jsonl 2> $O/ab.log
