# Round 3: the round-2 source's 6-wave specular kernels (register-cap hazard
# reproduction), then the list-world kernel A/B (tools/ab_veach.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03c}
mkdir -p $O
PYTHONPATH=first_raytracer_amd/build/r2 timeout -k 10 300 python tools/probe_r2_caps.py > $O/probe_r2.txt 2>&1 \
 && timeout -k 10 300 python tools/ab_veach.py --spp 256 --rounds 3 > $O/ab_veach.jsonl 2> $O/ab_veach.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
