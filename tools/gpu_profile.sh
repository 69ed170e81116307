# rocprofv3 kernel-trace summary + PMC HBM-traffic passes (FETCH_SIZE and
# WRITE_SIZE in separate passes, MI355X_MICROARCH.md "rocprofv3 PMC slots"),
# then the cornell_1m bench.  Chained: the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r01}
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG/trace -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG/trace_bench.json 2> gpurun_out/prof_$TAG/trace_bench.log \
 && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_$TAG/pmc_fetch -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$TAG/pmc_fetch.json 2> gpurun_out/prof_$TAG/pmc_fetch.log \
 && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_$TAG/pmc_write -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_$TAG/pmc_write.json 2> gpurun_out/prof_$TAG/pmc_write.log \
 && timeout -k 10 400 python3 bench.py --scene cornell_1m > gpurun_out/prof_$TAG/bench_1m.json 2> gpurun_out/prof_$TAG/bench_1m.log
rc=$?
echo "rc=$rc" > gpurun_out/prof_$TAG/rc.txt
exit $rc
