#!/bin/bash
# config 3: the stream's default geometry vs the exact mode's (PG_STREAM_WIDE_RANGE=1), serial queries, plus a parity check
set -o pipefail
mkdir -p gpurun_out
for v in 0 1; do
  PG_STREAM_WIDE_RANGE=$v timeout -k 10 300 python -u bench.py --workload ssb --no-cpu --steps 30 --warmup 5 --inflight ${INFLIGHT:-1} ${EXTRA_ARGS} \
    > gpurun_out/wr_$v.json 2> gpurun_out/wr_$v.err || { echo "bench wr $v failed"; tail -20 gpurun_out/wr_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['step_breakdown_ms'], d.get('parity_full'))" gpurun_out/wr_$v.json
done
