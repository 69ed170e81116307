# Parity subset, then a cornell_1m / Cornell A/B, in one call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-chk}; mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_c4.py} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 32 --rounds 3 --variants ${V1:-default} > $O/ab_1m.jsonl 2> $O/ab_1m.log || exit $?
timeout -k 10 300 python tools/perf_ab.py --scene cornell --spp 64 --rounds 3 --variants ${V2:-default} > $O/ab_cornell.jsonl 2> $O/ab_cornell.log
