# Round 3: (1) the register-cap hazard on the round-2 state that showed it
# (5a5829a, 6-wave specular kernels enabled; tools/probe_r2_caps.py);
# (2) cache PMC of the cornell_1m path megakernel (L2 and L1 hit rates, wait
# cycles) for the roofline's "bound", one counter group per pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03d}
mkdir -p $O
pmc() {  # name, counters
  timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- \
      python3 bench.py --scene cornell_1m --spp 128 --steps 1 --warmup 0 --no-cpu-baseline --north-star off > $O/$1.json 2> $O/$1.log
}
PYTHONPATH=first_raytracer_amd/build/r2 timeout -k 10 300 python tools/probe_r2_caps.py > $O/probe_r2.txt 2>&1 \
 && pmc tcc_1m "TCC_HIT_sum TCC_MISS_sum" \
 && pmc tcp_1m "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
 && pmc sq_1m "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD" \
 && pmc fetch_1m FETCH_SIZE && pmc write_1m WRITE_SIZE
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
