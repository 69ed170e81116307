# PC sampling (rocprofv3 beta, host-trap method) of the path megakernel on a
# short Cornell run, to see where its cycles go.  One time-limited step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pcs}
mkdir -p $O
rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 50 --output-format csv -d $O/pcs -o run -- \
    python3 tools/perf_ab.py --scene cornell --spp 16 --rounds 1 --variants default > $O/pcs.log 2>&1
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
