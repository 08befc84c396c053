#!/bin/bash
# per-step GPU timeline (kernel + memory-copy trace) of a few bench steps per workload, for the gaps between the
# hot path's dispatches and the host's part of a step; analysed by tools/timeline.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-tl}
for w in ${WORKLOADS:-adanalytics index}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${TAG}_$w -o run \
    -- python3 bench.py --workload $w --no-cpu --steps 6 --warmup 2 $BENCH_ARGS > gpurun_out/${TAG}_$w.json \
    2> gpurun_out/${TAG}_$w.err || { echo "$w failed"; tail -20 gpurun_out/${TAG}_$w.err; exit 1; }
  echo "$w ok"
done
