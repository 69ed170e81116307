# Round-3 GPU check: the -m gpu suite, then the bench lines named by LINES
# (default: the driver's default line with the north star, and C3 veach at its
# own config).  Every GPU step under its own time limit, chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=gpurun_out/$TAG
mkdir -p $O
run_tests() {
    [ "${TESTS:-1}" = "0" ] && return 0
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1
}
run_lines() {
    for l in ${LINES:-default veach}; do
        case $l in
        default) timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.log || return 1 ;;
        veach) timeout -k 10 400 python bench.py --scene veach --spp 1024 > $O/bench_veach.json 2> $O/bench_veach.log || return 1 ;;
        veach32) timeout -k 10 400 python bench.py --scene veach --spp 1024 --precision fp32 > $O/bench_veach32.json 2> $O/bench_veach32.log || return 1 ;;
        mlt) timeout -k 10 400 python bench.py --integrator pssmlt --steps 2 --warmup 1 > $O/bench_mlt.json 2> $O/bench_mlt.log || return 1 ;;
        esac
    done
}
run_tests && run_lines
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
