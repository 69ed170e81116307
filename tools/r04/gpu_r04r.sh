# Round 4, eighteenth call (re-built container, HEAD 13ef74b + this script):
# the GPU suite + smoke + default bench on the rebuilt library; the register-cap
# reproducer (the round-3 state cut, 0a75e3c, built from its own tree) at -O3 and
# with every automatic variable zero- / pattern-initialised (an uninitialised
# read would change with those); then the N-rank rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 \
 && timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
 && timeout -k 10 420 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log \
 && TAG=r04r/caps LIBS="fail zinit pinit" bash tools/gpu_caps_exp.sh \
 && TAG=r04r/mr bash tools/gpu_multirank.sh
rc=$?
# veach's fp64 list kernel (kMatsSpec: 249 VGPRs, 2 waves/SIMD) under a 3-wave
# cap (168 VGPRs): build/exp/libfrt_f64w3.so against the in-tree library
E=first_raytracer_amd/build/exp
V="--scene veach --spp 256 --rounds 3 --variants default"
[ $rc = 0 ] && timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64w.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_f64w3.so timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64w.jsonl 2>> $O/ab.log \
 && timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64w.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_f64w3.so timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64w.jsonl 2>> $O/ab.log
