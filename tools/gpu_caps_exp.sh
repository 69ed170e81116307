# Register-cap hazard: the caps table (tools/caps_table.py) for the in-tree
# library and for experiment builds that differ only in compiler options
# (first_raytracer_amd/build/exp/libfrt_$NAME.so).  Each library runs in its
# own process under its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-capsx}
mkdir -p $O
rc=0
for n in cur ${LIBS:-base wz sgv nohirp o1}; do
  if [ $n = cur ]; then unset FRT_LIB_PATH; else export FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_$n.so; fi
  timeout -k 10 240 python -u tools/caps_table.py --tag $n >> $O/caps.jsonl 2>> $O/log.txt || { rc=$?; break; }
done
echo "rc=$rc" > $O/rc.txt
# DBG=<lib name>: then the per-vertex capture of that build (tools/caps_dbg.py)
if [ $rc = 0 ] && [ -n "$DBG" ]; then
  FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_$DBG.so timeout -k 10 240 python -u tools/caps_dbg.py \
      --flags ${DBG_FLAGS:-17} --good 0 --bad ${DBG_BAD:-4} > $O/dbg.txt 2>> $O/log.txt
  rc=$?
  echo "rc=$rc" > $O/rc.txt
fi
exit $rc
