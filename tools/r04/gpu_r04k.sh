# Round 4, eleventh call: the GPU suite + smoke (the PSS-MLT oracle comparison
# now over four runs), the default bench under rocprofv3 kernel-trace with
# its Cornell / cornell_1m PMC passes (tools/gpu_roofline.sh PART=a); then a
# PSS-MLT timing build with one mix32 round per primary sample (invalid
# against the oracle, timing only: build/exp/libfrt_mltcheap.so vs
# libfrt_mltref.so, the same source) and Cornell under the other trees.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04k; mkdir -p $O
E=first_raytracer_amd/build/exp
P="--scene cornell --spp 512 --rounds 2 --bvh gsah --integrator pssmlt --variants default"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && TAG=r04k/roof PART=a bash tools/gpu_roofline.sh \
 && FRT_LIB_PATH=$E/libfrt_mltref.so timeout -k 10 300 python -u tools/perf_ab.py $P >> $O/ab_mlt.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_mltcheap.so timeout -k 10 300 python -u tools/perf_ab.py $P >> $O/ab_mlt.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_mltref.so timeout -k 10 300 python -u tools/perf_ab.py $P >> $O/ab_mlt.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_mltcheap.so timeout -k 10 300 python -u tools/perf_ab.py $P >> $O/ab_mlt.jsonl 2>> $O/ab.log \
 && for b in gsah sah host ploc; do timeout -k 10 200 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 2 --bvh $b --variants default >> $O/ab_tree.jsonl 2>> $O/ab.log || exit 1; done
