# Round 4, twenty-second call: which part of the round-3 state cut the
# register-cap fault needs.  The reproducer (0a75e3c) with one of its three
# changes undone at a time (variants built from its own tree): ray counters back
# in SGPRs (nocnt), no radiance flush inside the traversal loop (noflush), the
# RNG key kept live instead of re-derived at shading (nokey); each variant's
# caps table against its own uncapped film.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=r04v/caps LIBS="fail nocnt noflush nokey" bash tools/gpu_caps_exp.sh
