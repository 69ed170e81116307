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
