# Rehearsal of the N-rank bench path on a one-GPU box: 2 ranks share the GPU,
# collectives over gloo with host staging (RCCL needs one GPU per rank; the
# driver's 8-GPU runs use it).  Compares image means with the 1-rank run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-mr}
mkdir -p $O
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 300 python bench.py --steps 1 --warmup 1 --spp 64 --no-cpu-baseline > $O/n1.json 2> $O/n1.log \
 && timeout -k 10 300 $R --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --spp 64 --backend gloo > $O/n2.json 2> $O/n2.log \
 && timeout -k 10 300 $R --master-port 29512 bench.py --gpus 2 --steps 1 --warmup 1 --spp 16 --scene cornell_1m --backend gloo > $O/n2_1m.json 2> $O/n2_1m.log \
 && timeout -k 10 300 $R --master-port 29513 bench.py --gpus 2 --steps 1 --warmup 1 --integrator pssmlt --spp 16 --backend gloo > $O/n2_mlt.json 2> $O/n2_mlt.log \
 && timeout -k 10 400 $R --master-port 29514 bench.py --gpus 2 --steps 1 --warmup 1 --ns-steps 1 --north-star on --backend gloo > $O/n2_default.json 2> $O/n2_default.log
rc=$?
echo "rc=$rc" > $O/rc.txt
exit $rc
