# Round 4, twenty-third call (final build of this session): the GPU suite +
# smoke + the default bench line + the veach / PSS-MLT lines on the library
# built from HEAD.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04w; mkdir -p $O
b() {  # name, seconds, bench args...
  local n=$1 s=$2; shift 2
  timeout -k 10 $s python -u bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.log
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && b default 420 && b veach 300 --scene veach --spp 1024 && b pssmlt 400 --integrator pssmlt
