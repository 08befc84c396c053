#!/bin/bash
# the in-flight timed loop at N = 2 ranks sharing the one GPU (gloo), serial vs 4 in flight, and N = 1
set -o pipefail
mkdir -p gpurun_out
for n in 1 4; do
  PG_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --segments 16 --no-cpu --steps 30 --warmup 3 --inflight $n \
    > gpurun_out/ifr_$n.json 2> gpurun_out/ifr_$n.err || { echo "2-rank bench inflight $n failed"; tail -30 gpurun_out/ifr_$n.err; exit 1; }
  tail -1 gpurun_out/ifr_$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=2 inflight', d['inflight'], d['ms_per_step'], d['serial_ms_per_step'], d['parity_full'])"
done
timeout -k 10 300 python -u bench.py --segments 16 --no-cpu --steps 30 --warmup 3 > gpurun_out/ifr_n1.json 2> gpurun_out/ifr_n1.err || { echo "1-rank failed"; tail -30 gpurun_out/ifr_n1.err; exit 1; }
tail -1 gpurun_out/ifr_n1.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=1 inflight', d['inflight'], d['ms_per_step'], d['serial_ms_per_step'])"
