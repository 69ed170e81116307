# A/B of leaf postponing (FRT_MIN_DESC) on Cornell and cornell_1m, one
# process per scene with interleaved rounds; then the phase diagnostics at
# the chosen setting.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-desc}; mkdir -p $O
V=${VARIANTS:-default/desc0,default/desc8,default/desc16,default/desc24,default/desc32,default/desc40}
timeout -k 10 300 python tools/perf_ab.py --scene cornell --spp 64 --rounds 3 --variants $V > $O/ab_cornell.jsonl 2> $O/ab_cornell.log \
 && timeout -k 10 300 python tools/perf_ab.py --scene cornell_1m --spp 32 --rounds 3 --variants $V > $O/ab_1m.jsonl 2> $O/ab_1m.log \
 && FRT_MIN_DESC=${DIAG_DESC:-16} FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_diag.so timeout -k 10 200 python tools/diag_phases.py --scene cornell --spp 32 > $O/diag_cornell.json 2> $O/diag_cornell.log \
 && FRT_MIN_DESC=${DIAG_DESC:-16} FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_diag.so timeout -k 10 200 python tools/diag_phases.py --scene cornell_1m --spp 32 > $O/diag_1m.json 2> $O/diag_1m.log
