# Material kernels: conductor parity tests on the product library, then a
# same-call A/B of perf_mats.py against experiment builds (FRT_LIB_PATH),
# processes alternating main, exp, main, exp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-matsab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_conductors.py ${TESTS} > $O/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for lib in main $EXPS; do
    if [ $lib = main ]; then unset FRT_LIB_PATH; else export FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_$lib.so; fi
    timeout -k 10 300 python tools/perf_mats.py --spp 64 --rounds 3 > $O/${lib}_$rep.jsonl 2> $O/${lib}_$rep.log || exit $?
  done
done
