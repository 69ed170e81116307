# Round 4, twentieth call: the register-cap reproducer's films (tools/caps_films.py)
# on the failing plan (HBM binary, flags 17) for caps 0/4/5/6 and max_depth
# 1..33, to find the first bounce at which the capped films go wrong.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r04t; mkdir -p $O
FRT_LIB_PATH=first_raytracer_amd/build/exp/libfrt_fail.so timeout -k 10 300 python -u tools/caps_films.py \
    --out $O/films_fail.npz > $O/films_fail.txt 2> $O/log.txt
