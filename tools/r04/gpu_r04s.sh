# Round 4, nineteenth call: the register-cap reproducer (0a75e3c, built from its
# own tree) with `s_nop` padding before every instruction
# (-mllvm -amdgpu-snop-padding=N, inserted after register allocation: the same
# registers and instruction order, only wait states added).  If the padded build
# is right where the plain one is wrong, the fault is a missing wait state
# (a hazard), not a wrong allocation.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=r04s/caps LIBS="fail snop7 snop2" bash tools/gpu_caps_exp.sh
