# Register-cap hazard (DESIGN.md §5 "Register-cap hazard"): the failing kernel
# as LLVM IR, and the llc commands that turn it into the greedy-allocated
# machine code (wrong radiance on the GPU) and the basic-SGPR-allocated one
# (right).  CPU only; no GPU minutes.
#
# path_megakernel_hbm_bvh2_cap4.ll.gz: path_megakernel<16, 0 (binary BVH),
# LDS false, 4 waves, -, 7 (every material set), 0 (path), float> of the
# round-3 state cut (commit 0a75e3c), i.e. the HBM binary plan at the 4-wave
# register cap -- one of the failing (plan, cap) pairs.  Made by
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=on -I../include -Icsrc \
#         --cuda-device-only -emit-llvm -S -o repro.ll csrc/frt_render.hip      (in a worktree of 0a75e3c)
#   opt -S -passes='internalize,globaldce' -internalize-public-api-list=<kernel> repro.ll -o k4.ll
# (REGEN=1 below redoes both).  llc on it reproduces the allocation state of the
# kernel that ran on the GPU: 49 VGPRs and 115 SGPRs spilled, 88 B of scratch,
# the figures of the failing build; with
# -sgpr-regalloc=basic: 59 / 131 / 80 B, the build that renders right.
# The 44-45 wrong pixels of its first shading step are in depth1_film_diff.json.
set -e
D=$(cd "$(dirname "$0")" && pwd)
LLVM=/opt/rocm/lib/llvm/bin
W=${W:-/tmp/frt_caps_ir}; mkdir -p $W
K=_ZN12_GLOBAL__N_115path_megakernelILi16ELi0ELb0ELi4ELb0ELi7ELi0EfEEvN3frt8DevSceneENS_7DevWorkE
if [ -n "$REGEN" ]; then
  WT=${WT:-/tmp/frt_caps_repro}
  ROOT=$(cd "$D/../.." && pwd)
  [ -d "$WT" ] || git -C "$ROOT" worktree add "$WT" 0a75e3c
  (cd "$WT/first_raytracer_amd" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=on \
     -I../include -Icsrc --cuda-device-only -emit-llvm -S -o $W/repro.ll csrc/frt_render.hip)
  $LLVM/opt -S -passes='internalize,globaldce' -internalize-public-api-list=$K $W/repro.ll -o $W/k4.ll
else
  gunzip -c $D/path_megakernel_hbm_bvh2_cap4.ll.gz > $W/k4.ll
fi
$LLVM/llc -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -O3 $W/k4.ll -o $W/k4_greedy.s
$LLVM/llc -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -O3 -sgpr-regalloc=basic $W/k4.ll -o $W/k4_basic_sgpr.s
$LLVM/llc -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -O3 -vgpr-regalloc=basic $W/k4.ll -o $W/k4_basic_vgpr.s
for f in k4_greedy k4_basic_sgpr k4_basic_vgpr; do
  printf '%-14s ' $f
  grep -E "ScratchSize:|\.sgpr_spill_count|\.vgpr_spill_count" $W/$f.s | tr -s ' \n' ' '; echo
done
# For an allocator trace of the greedy run (what a compiler engineer would read first):
#   $LLVM/llc ... -debug-only=regalloc   (needs an assertions-enabled llc; ROCm's is not)
#   $LLVM/llc ... -print-after=greedy -filter-print-funcs=$K 2> greedy.mir
