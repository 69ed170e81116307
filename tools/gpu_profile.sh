# rocprofv3 kernel-trace summaries of the bench command (Cornell, cornell_1m),
# then PMC HBM-traffic passes (FETCH_SIZE and WRITE_SIZE in separate passes,
# MI355X_MICROARCH.md "rocprofv3 PMC slots").  Chained: the first failure ends
# the script.  Summaries: python tools/pmc_traffic.py (on the CPU side).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r01}
O=gpurun_out/prof_$TAG
mkdir -p $O
trace() {  # name, bench args
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$1 -o run -- \
      python3 bench.py $2 > $O/trace_$1.json 2> $O/trace_$1.log
}
pmc() {  # name, counter, bench args
  timeout -k 10 300 rocprofv3 --pmc $2 --output-format csv -d $O/pmc_$1 -o run -- \
      python3 bench.py $3 > $O/pmc_$1.json 2> $O/pmc_$1.log
}
trace cornell "--steps 3 --warmup 1 --no-cpu-baseline" \
 && trace 1m "--scene cornell_1m --steps 2 --warmup 1 --no-cpu-baseline" \
 && pmc fetch_cornell FETCH_SIZE "--steps 1 --warmup 0 --no-cpu-baseline" \
 && pmc write_cornell WRITE_SIZE "--steps 1 --warmup 0 --no-cpu-baseline" \
 && pmc fetch_1m FETCH_SIZE "--scene cornell_1m --steps 1 --warmup 0 --no-cpu-baseline" \
 && pmc write_1m WRITE_SIZE "--scene cornell_1m --steps 1 --warmup 0 --no-cpu-baseline"
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
