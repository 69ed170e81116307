set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/mltpmc; mkdir -p $O
pmc() { timeout -k 10 240 rocprofv3 --pmc $2 --output-format csv -d $O/$1 -o run -- python3 bench.py --integrator pssmlt --steps 1 --warmup 0 --no-cpu-baseline > $O/$1.json 2> $O/$1.log; }
pmc sq "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY" && pmc fetch FETCH_SIZE && pmc write WRITE_SIZE
