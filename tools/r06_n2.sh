#!/bin/bash
# rehearsal of the driver's N > 1 launch on the one-GPU box: torch.distributed.run with 2 ranks sharing GPU 0
# (PG_BENCH_SHARE_GPU=1: gloo collectives instead of RCCL, which refuses two ranks on one GPU), config 2 at 16
# segments per rank, weak scaling; the line's parity_full checks the merged result against the oracle
set -o pipefail
mkdir -p gpurun_out
PG_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --segments 16 --steps 20 --warmup 3 \
  > gpurun_out/r06e_n2_shared_bench.json 2> gpurun_out/r06e_n2_shared_bench.err || { echo "N=2 failed"; tail -40 gpurun_out/r06e_n2_shared_bench.err; exit 1; }
tail -c 600 gpurun_out/r06e_n2_shared_bench.json
