# Round 3: (1) the register-cap probe on the experiment build with 6-wave
# specular kernels (FRT_EXP_SPEC_W6); (2) the fp64 / list-prefilter GPU tests;
# (3) the C3 veach line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03b}
mkdir -p $O
PROBE_FLAGS=1,17,0 PROBE_CAPS=4,5,6 FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_w6.so \
  timeout -k 10 300 python tools/probe_conductors.py > $O/probe_w6.txt 2>&1 \
 && timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/pytest_prec.log 2>&1 \
 && timeout -k 10 400 python bench.py --scene veach --spp 1024 > $O/bench_veach.json 2> $O/bench_veach.log \
 && timeout -k 10 400 python bench.py --scene veach --spp 1024 --precision fp32 --cpu-pixels 20000 > $O/bench_veach32.json 2> $O/bench_veach32.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
