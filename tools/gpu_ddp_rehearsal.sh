# N > 1 rehearsal on a 1-GPU box: bench.py under torch.distributed.run, 2 ranks sharing the GPU over gloo
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
VPT_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu-baseline > $O/ddp2.json 2> $O/ddp2.err || { echo "DDP REHEARSAL FAILED"; tail -30 $O/ddp2.err; exit 1; }
cut -c1-400 $O/ddp2.json
