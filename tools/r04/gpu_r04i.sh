# Round 4, ninth call: Cornell trav_min on the round-4 node loop; C3 probe
# (veach as the reference's list world vs the same primitives under a BVH, both
# fp64: tools/veach_bvh_probe.py); PSS-MLT's mean against the path tracer at
# 512 and 2048 mutations per pixel (chain length 4,050 vs 16,200: start-up
# bias of the reference's algorithm at 1080p), with the 10^7-path reference b.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 300 python -u tools/perf_ab.py --scene cornell --spp 512 --rounds 3 --bvh gsah \
      --variants default,default/trav16,default/trav20,default/trav24 > $O/ab_trav.jsonl 2> $O/ab.log \
 && timeout -k 10 300 python -u tools/veach_bvh_probe.py --spp 256 --rounds 2 > $O/veach_bvh.jsonl 2> $O/veach_bvh.log \
 && timeout -k 10 400 python -u bench.py --integrator pssmlt > $O/bench_pssmlt.json 2> $O/bench_pssmlt.log \
 && timeout -k 10 400 python -u bench.py --integrator pssmlt --spp 2048 --steps 1 --warmup 0 > $O/bench_pssmlt_2048.json 2> $O/bench_pssmlt_2048.log
