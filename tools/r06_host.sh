#!/bin/bash
# config 2: host phase profile (PG_HOST_PROFILE=1) of bench steps, and a kernel timeline of a few steps
set -o pipefail
mkdir -p gpurun_out
PG_HOST_PROFILE=1 timeout -k 10 240 python -u bench.py --workload adanalytics --no-cpu --steps 30 --warmup 5 --no-full-parity > gpurun_out/hp_ad.json 2> gpurun_out/hp_ad.err || { echo "host profile failed"; tail -20 gpurun_out/hp_ad.err; exit 1; }
grep "pg host" gpurun_out/hp_ad.err | tail -8
TAG=tl06 WORKLOADS=adanalytics BENCH_ARGS=--no-full-parity bash tools/timeline.sh && python3 tools/timeline.py gpurun_out/tl06_adanalytics/* 2>/dev/null | tail -30 || python3 tools/timeline.py $(ls -d gpurun_out/tl06_adanalytics/*/ | head -1) | tail -30
