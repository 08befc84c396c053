#!/bin/bash
# round 6 closing profiles of the final library (tools/profile_bench.sh per workload: bench line with the CPU baseline,
# rocprofv3 kernel trace, FETCH_SIZE / WRITE_SIZE passes), then config 2 at 16 segments per GPU.
# WORKLOADS selects a subset; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r06d}
for W in ${WORKLOADS:-adanalytics ssb highcard index}; do
  bash tools/profile_bench.sh $TAG $W 10 || exit 1
done
if [ -n "${SEG16:-1}" ]; then
  timeout -k 10 300 python -u bench.py --segments 16 --no-cpu --steps 50 --warmup 10 > gpurun_out/${TAG}_seg16_bench.json 2> gpurun_out/${TAG}_seg16_bench.err || { echo "seg16 failed"; tail -20 gpurun_out/${TAG}_seg16_bench.err; exit 1; }
  timeout -k 10 300 python -u bench.py --segments 16 --no-cpu --steps 50 --warmup 10 --inflight 1 > gpurun_out/${TAG}_seg16_serial_bench.json 2> gpurun_out/${TAG}_seg16_serial_bench.err || { echo "seg16 serial failed"; exit 1; }
  tail -c 400 gpurun_out/${TAG}_seg16_bench.json
fi
echo "r06_e ok"
