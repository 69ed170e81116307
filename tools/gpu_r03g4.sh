# Round 3 (re-entry): the samples-per-item target (FRT_SPI_TARGET; 0 = the
# 40-items-per-lane rule alone): GPU suite, smoke, same-process A/B on Cornell,
# veach (fp64 list world), normals, then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03g4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 \
      --variants default,default/spt0 > $O/spt_cornell.jsonl 2>> $O/log.txt \
 && timeout -k 10 400 python -u tools/perf_ab.py --scene veach --spp 1024 --rounds 2 \
      --variants default,default/spt0 > $O/spt_veach.jsonl 2>> $O/log.txt \
 && timeout -k 10 200 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --integrator normals \
      --variants default,default/spt0 > $O/spt_normals.jsonl 2>> $O/log.txt \
 && timeout -k 10 420 python bench.py > $O/bench_default.json 2> $O/bench_default.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
