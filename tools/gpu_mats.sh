# Material kernels (MATS) vs the lambertian kernel: perf_mats.py with the
# default plan and with FRT_MATS_WAVES register caps, each its own process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-mats}; mkdir -p $O
timeout -k 10 300 python tools/perf_mats.py --spp 64 --rounds 3 > $O/default.jsonl 2> $O/default.log || exit $?
for w in ${CAPS:-3 4}; do
  FRT_MATS_WAVES=$w timeout -k 10 300 python tools/perf_mats.py --spp 64 --rounds 3 > $O/w$w.jsonl 2> $O/w$w.log || exit $?
done
