# PSS-MLT tests, then the C5 bench line on the product library and on an
# experiment build (FRT_LIB_PATH), alternating, each its own process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-mltab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pssmlt.py tests/test_gpu_conductors.py tests/test_gpu_textures.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for lib in main $EXP; do
    if [ $lib = main ]; then unset FRT_LIB_PATH; else export FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_$lib.so; fi
    timeout -k 10 300 python bench.py --integrator pssmlt --steps 2 --warmup 1 --no-cpu-baseline > $O/mlt_${lib}_$rep.json 2> $O/mlt_${lib}_$rep.log || exit $?
  done
done
