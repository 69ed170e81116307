# Roofline evidence for bench.py: the default bench command (Cornell + the
# cornell_1m north-star block) under rocprofv3 --kernel-trace --stats, then
# per config the PMC passes bench.py's roofline reads (one counter group per
# run: SQ issue counters, FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md PMC
# slots).  Chained: the first failure ends the script.  Afterwards, on the CPU
# side: tools/roofline_pmc.py KEY --sq .. --fetch .. --write .. --bench ..
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-roof}
mkdir -p $O
( nproc; cat /sys/fs/cgroup/cpu.max; python3 -c 'import os; print(len(os.sched_getaffinity(0)), os.cpu_count())' ) > $O/host_cpus.txt 2>&1
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY"
pmc() {  # name, counters, scene
  timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- \
      python3 bench.py --scene $3 --steps 1 --warmup 0 --no-cpu-baseline --north-star off > $O/$1.json 2> $O/$1.log
}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
      python3 bench.py --steps ${STEPS:-5} --warmup 1 > $O/trace.json 2> $O/trace.log \
 && pmc sq_cornell "$SQ" cornell && pmc fetch_cornell FETCH_SIZE cornell && pmc write_cornell WRITE_SIZE cornell \
 && pmc sq_1m "$SQ" cornell_1m && pmc fetch_1m FETCH_SIZE cornell_1m && pmc write_1m WRITE_SIZE cornell_1m
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
