# Round 4, twenty-fourth call: the register-cap reproducer with its LDS ray
# counters moved back to SGPRs at one group of call sites at a time (traversal
# loop: cloop; after shading: cshade; camera start: cstart), each variant's caps
# table against its own uncapped film.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=r04x/caps LIBS="cloop cshade cstart" bash tools/gpu_caps_exp.sh
