# Register-cap reproducer builds (DESIGN.md "Register-cap hazard"), on the CPU
# container: the round-3 state cut (0a75e3c) from its own tree in a git
# worktree, as build/exp/libfrt_<name>.so of this repository, for
# tools/gpu_caps_exp.sh (LIBS="fail ...").  Variants:
#   fail   : the reproducer as committed (-O3, greedy allocator everywhere)
#   pinit  : -ftrivial-auto-var-init=pattern (right on every pair)
#   snop7  : -mllvm -amdgpu-snop-padding=7 (same machine code plus nops; still wrong)
#   nocnt  : the wave's ray counters back in SGPR pairs (right on every pair)
#   ASM=1  : also the device assembly of the reproducer (build/exp/repro.s)
# Usage: bash tools/caps_repro_build.sh [names...]   (default: fail)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=${WT:-/tmp/frt_caps_repro}
[ -d "$WT" ] || git -C "$ROOT" worktree add "$WT" 0a75e3c
cd "$WT/first_raytracer_amd"
make build/scene.o build/film.o build/frt_lbvh.o
mkdir -p build/exp "$ROOT/first_raytracer_amd/build/exp"
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=on -I../include -Icsrc"
for n in ${@:-fail}; do
  src=csrc/frt_render.hip; extra=""
  case $n in
    fail) ;;
    pinit) extra="-ftrivial-auto-var-init=pattern" ;;
    snop7) extra="-mllvm -amdgpu-snop-padding=7" ;;
    nocnt)
      python3 - "$src" csrc/frt_render_nocnt.hip << 'EOF'
import sys
s = open(sys.argv[1]).read()
s = s.replace("    auto count = [&](int k, bool x) {\n",
              "    unsigned long long nc[4] = {0, 0, 0, 0};\n    auto count = [&](int k, bool x) {\n", 1)
s = s.replace("        if (lane == 0 && v) cnt[k] += v;\n", "        nc[k] += v;\n", 1)
s = s.replace("W.wave_rays[4 * wv + k] = cnt[k];", "W.wave_rays[4 * wv + k] = nc[k];", 1)
open(sys.argv[2], "w").write(s)
EOF
      src=csrc/frt_render_nocnt.hip ;;
    *) echo "unknown variant $n"; exit 2 ;;
  esac
  $HIPCC $FLAGS $extra -c $src -o build/exp/frt_render_$n.o
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o "$ROOT/first_raytracer_amd/build/exp/libfrt_$n.so" \
      build/exp/frt_render_$n.o build/frt_lbvh.o build/scene.o build/film.o -lpthread -lz -lrccl
done
if [ -n "$ASM" ]; then
  $HIPCC $FLAGS --cuda-device-only -S -o "$ROOT/first_raytracer_amd/build/exp/repro.s" csrc/frt_render.hip
fi
