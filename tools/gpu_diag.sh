set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/diag1; mkdir -p $O
export FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_diag.so
timeout -k 10 200 python tools/diag_phases.py --scene cornell --spp 32 > $O/cornell.json 2> $O/cornell.log \
 && timeout -k 10 200 python tools/diag_phases.py --scene cornell_1m --spp 32 > $O/1m.json 2> $O/1m.log
