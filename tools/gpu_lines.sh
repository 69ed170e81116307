# The other bench lines (README / DESIGN tables): veach C3, PSS-MLT C5, AO,
# normals, and the reference / GPU-built trees.  Each its own process and time
# limit, chained.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-lines}; mkdir -p $O
b() { name=$1; shift; timeout -k 10 300 python bench.py --steps 2 --warmup 1 --north-star off --cpu-seconds 3 "$@" > $O/$name.json 2> $O/$name.log; }
b veach --scene veach --spp 1024 \
 && b pssmlt --integrator pssmlt \
 && b ao --integrator ao \
 && b normals --integrator normals \
 && b cornell_ref --bvh host \
 && b c1m_ref --scene cornell_1m --bvh host \
 && b c1m_gpu --scene cornell_1m --bvh gpu \
 && b ao_1m --scene cornell_1m --integrator ao --spp 256
