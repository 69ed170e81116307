# Round 4, sixteenth call (final build): the GPU suite + smoke; the bench lines
# (default = Cornell + the cornell_1m north star, veach, PSS-MLT, AO, normals);
# the default bench under rocprofv3 kernel-trace with its Cornell / cornell_1m
# PMC passes (tools/gpu_roofline.sh PART=a).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04p; mkdir -p $O
b() {  # name, seconds, bench args...
  local n=$1 s=$2; shift 2
  timeout -k 10 $s python -u bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.log
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && b default 420 && b veach 300 --scene veach --spp 1024 && b pssmlt 400 --integrator pssmlt \
 && b ao 200 --integrator ao && b normals 200 --integrator normals \
 && TAG=r04p/roof PART=a bash tools/gpu_roofline.sh
