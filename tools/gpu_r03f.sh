# Round 3: (1) the failing round-2 state (5a5829a, 6-wave specular kernels)
# rebuilt with compiler-side variants -- the AMDGPU high-register-pressure
# rescheduling stage disabled, and -O1 -- to tell a source hazard from a
# code-generation one; (2) the ray-query kernel with wave-local ray chunks:
# GPU parity tests and throughput.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03f}
mkdir -p $O
R2=first_raytracer_amd/build/r2
for v in nohirp o1; do
  PYTHONPATH=$R2 FRT_LIB_PATH=$R2/first_raytracer_amd/libfrt_$v.so timeout -k 10 300 python tools/probe_r2_caps.py > $O/probe_r2_$v.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_trace.py -x -v --timeout 200 --timeout-method thread > $O/pytest_trace.log 2>&1 \
 && timeout -k 10 400 python tools/trace_bench.py --scene cornell_1m > $O/trace_1m.jsonl 2> $O/trace_1m.log \
 && timeout -k 10 300 python tools/trace_bench.py --scene cornell > $O/trace_cornell.jsonl 2> $O/trace_cornell.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
