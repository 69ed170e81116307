# Round 4, thirteenth call: scheduling knobs re-checked on the round-4 kernels.
# cornell_1m 512 spp: (trav_min, min_desc) and the 4-wide leaf size with the
# straight-line triangle test; AO on Cornell: trav_min.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 400 python -u tools/perf_ab.py --scene cornell_1m --spp 512 --rounds 1 --bvh gsah \
      --variants default,default/trav32,default/trav48,default/desc4,default/desc12 > $O/ab_1m_knobs.jsonl 2> $O/ab.log \
 && timeout -k 10 400 python -u tools/perf_ab.py --scene cornell_1m --spp 512 --rounds 1 --bvh gsah \
      --variants default,default/leaf3,default/leaf5 > $O/ab_1m_leaf.jsonl 2>> $O/ab.log \
 && timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --bvh gsah --integrator ao \
      --variants default,default/trav6,default/trav20,default/trav28 > $O/ab_ao_trav.jsonl 2>> $O/ab.log
rc0=$?
# C3 timing build: fp64 reciprocal / division as v_rcp_f64 + two Newton steps
# instead of the IEEE sequence (not correctly rounded; timing only):
# build/exp/libfrt_f64fast.so vs libfrt_f64ref.so (the same source)
E=first_raytracer_amd/build/exp
V="--scene veach --spp 256 --rounds 3 --variants default"
[ $rc0 = 0 ] && FRT_LIB_PATH=$E/libfrt_f64ref.so timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64div.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_f64fast.so timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64div.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_f64ref.so timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64div.jsonl 2>> $O/ab.log \
 && FRT_LIB_PATH=$E/libfrt_f64fast.so timeout -k 10 300 python -u tools/perf_ab.py $V >> $O/ab_f64div.jsonl 2>> $O/ab.log
rc=$?
# timing build with one mix32 round per path random number (invalid against the
# oracle, timing only: build/exp/libfrt_rngcheap.so vs libfrt_rngref.so)
C="--scene cornell --spp 512 --rounds 3 --bvh gsah --variants default"
M="--scene cornell_1m --spp 256 --rounds 2 --bvh gsah --variants default"
ab() { local l=$1; shift; FRT_LIB_PATH=$E/$l timeout -k 10 300 python -u tools/perf_ab.py "$@" >> $O/ab_rng.jsonl 2>> $O/ab.log; }
[ $rc = 0 ] && ab libfrt_rngref.so $C && ab libfrt_rngcheap.so $C && ab libfrt_rngref.so $C && ab libfrt_rngcheap.so $C \
 && ab libfrt_rngref.so $M && ab libfrt_rngcheap.so $M
