#!/bin/bash
# Four ranks on one GPU: the bench's distributed path (rendezvous, barriers,
# max-over-ranks timing, counter all-reduce over the host group) end to end,
# started by bench.py's own launcher and by torch.distributed.run.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/dist; rm -rf $O; mkdir -p $O
# the stdlib launcher (bench.py --gpus 4 outside any launcher), then the driver's form (torch.distributed.run)
BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 4 --steps 3 --warmup 1 --cpu-seconds 0 --batch 64 --bp-batch 1024 --sc-batch 64 --concat-batch 64 --detail-dir $O/d_launch > $O/launch.json 2> $O/launch.err
BENCH_REHEARSAL=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 4 --steps 3 --warmup 1 --cpu-seconds 0 --batch 64 --bp-batch 1024 --sc-batch 64 --concat-batch 64 --detail-dir $O/d_torchrun > $O/torchrun.json 2> $O/torchrun.err
# (RCCL itself needs one GPU per rank: with two ranks on one GPU ncclCommInitRank
# reports "invalid usage", so the RCCL counter path runs only on multi-GPU nodes)
# BENCH_FORCE_RCCL=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 3 --warmup 1 --no-bp --no-concat --cpu-seconds 0 --batch 64 > $O/rccl.json 2> $O/rccl.err
