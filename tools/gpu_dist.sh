#!/bin/bash
# GPU box: rehearse the multi-rank bench paths on one GPU (2 ranks share the
# device over gloo; the driver's 8-GPU run uses nccl = RCCL, one GPU per rank).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export DF_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/dist_fwd.log 2>&1 && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 2 --mode nll > gpurun_out/dist_nll.log 2>&1 && \
unset DF_DIST_BACKEND && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29513 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu > gpurun_out/dist_1.log 2>&1
export DF_DIST_BACKEND=gloo && \
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29514 bench.py --gpus 2 --steps 5 --warmup 2 --mode train > gpurun_out/dist_train.log 2>&1
