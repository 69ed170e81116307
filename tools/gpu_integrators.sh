# GPU check of the ao / normals integrators: parity tests, bench lines
# (Cornell 1080p, cornell_1m) and a rocprofv3 kernel summary of the AO bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-integ}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -m pytest tests/test_gpu_integrators.py tests/test_gpu_cli.py -m gpu -x -q > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python bench.py --integrator ao --spp 512 --cpu-seconds ${CPU_S:-4} > $O/bench_ao.json 2> $O/bench_ao.log \
 && timeout -k 10 300 python bench.py --integrator normals --spp 512 --cpu-seconds ${CPU_S:-4} > $O/bench_normals.json 2> $O/bench_normals.log \
 && timeout -k 10 400 python bench.py --integrator ao --scene cornell_1m --spp 256 --cpu-seconds ${CPU_S:-4} > $O/bench_ao_1m.json 2> $O/bench_ao_1m.log \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ao -o ao -- python3 bench.py --integrator ao --spp 512 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_ao_prof.json 2> $O/bench_ao_prof.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
