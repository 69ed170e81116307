# Same-call A/B of the product library against experiment builds
# (FRT_LIB_PATH) on cornell_1m and Cornell; processes alternate A, B, A, B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-abx}; mkdir -p $O
for rep in 1 2; do
  for lib in main $EXPS; do
    if [ $lib = main ]; then unset FRT_LIB_PATH; else export FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_$lib.so; fi
    timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 32 --rounds 2 --variants ${V1:-default} > $O/1m_${lib}_$rep.jsonl 2> $O/1m_${lib}_$rep.log || exit $?
    timeout -k 10 300 python tools/perf_ab.py --scene cornell --spp 64 --rounds 2 --variants ${V2:-default} > $O/c_${lib}_$rep.jsonl 2> $O/c_${lib}_$rep.log || exit $?
  done
done
