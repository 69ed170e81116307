# Round 4, fifth call: the GPU suite + smoke on the build whose PSS-MLT
# shading fetches a vertex's primary samples in two 16-B loads; same-call A/B
# of PSS-MLT against the r04d build (build/exp/libfrt_r04d.so); then the
# PMC roofline passes of the default bench command (Cornell + cornell_1m;
# tools/gpu_roofline.sh PART=a), whose path kernels are the r04d build's.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
E=first_raytracer_amd/build/exp
P="--scene cornell --spp 512 --rounds 3 --bvh gsah --integrator pssmlt --variants default"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && timeout -k 10 300 python -u tools/perf_ab.py $P >> $O/ab_mlt.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_r04d.so timeout -k 10 300 python -u tools/perf_ab.py $P >> $O/ab_mlt.jsonl 2>> $O/ab.log \
 && timeout -k 10 300 python -u tools/perf_ab.py $P >> $O/ab_mlt.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_r04d.so timeout -k 10 300 python -u tools/perf_ab.py $P >> $O/ab_mlt.jsonl 2>> $O/ab.log \
 && TAG=r04e/roof PART=a bash tools/gpu_roofline.sh
