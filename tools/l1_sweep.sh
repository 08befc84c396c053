#!/bin/bash
# Level-1 digit width sweep for config 4 (PG_PART_L1_BITS): parity tests + a kernel-traced highcard bench per width.
set -o pipefail
mkdir -p gpurun_out
for B in ${BITS:-8 7}; do
  PG_PART_L1_BITS=$B timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    --tb=short -k "radix or config4 or speculative or trim" > gpurun_out/l1_tests_$B.log 2>&1 || { echo "tests failed ($B)"; tail -30 gpurun_out/l1_tests_$B.log; exit 1; }
  echo "bits $B: $(tail -1 gpurun_out/l1_tests_$B.log)"
  PG_PART_L1_BITS=$B timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/l1_$B -o run -- python3 -u bench.py --workload highcard \
    --steps 10 --warmup 3 --no-cpu > gpurun_out/l1_$B.json 2> gpurun_out/l1_$B.err || { echo "bench failed ($B)"; tail -20 gpurun_out/l1_$B.err; exit 1; }
  python3 - "$B" <<'PY'
import csv, glob, json, sys
b = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/l1_{b}.json") if l.startswith("{")][-1])
print("  ", d["ms_per_step"], d["step_breakdown_ms"])
for f in glob.glob(f"gpurun_out/l1_{b}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "pg::part" in r["Name"]:
            print("   %-50s %5s %9.1f us" % (r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1000))
PY
  rm -rf gpurun_out/l1_$B
done
