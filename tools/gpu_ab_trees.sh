# Same-box A/B of two source trees: ab/old (a previous commit, built in
# place) against the current tree, alternated, one process per run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abtrees}
mkdir -p $O
rc=0
for rep in 1 2; do
  for scene in ${SCENES:-cornell cornell_1m}; do
    spp=64; [ $scene = cornell_1m ] && spp=16
    for t in old new; do
      root=.; [ $t = old ] && root=ab/old
      timeout -k 10 200 python $root/tools/perf_ab.py --scene $scene --spp $spp --rounds 3 --variants default \
        >> $O/${t}_$scene.jsonl 2>> $O/log.txt || { rc=$?; break 3; }
    done
  done
done
echo "rc=$rc" > $O/rc.txt
exit $rc
