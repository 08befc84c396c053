#!/bin/bash
# Launch-parameter sweep (BENCH_ARGS: extra bench.py arguments, e.g. --workload ssb) of the config-2 bench (env knobs of pg_runtime); one bench per setting, first failure ends it.
set -o pipefail
O=gpurun_out/sweep
mkdir -p $O
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python3 bench.py --no-cpu --steps 20 --warmup 5 $BENCH_ARGS > "$O/${TAG:-}$(echo $cfg | tr ' =' '_-').json" 2>/dev/null \
    || { echo "failed: $cfg"; exit 1; }
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/sweep/*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], round(d["value"] / 1e9, 1), "Grows/s  scan_ms", round(d["roofline"]["kernel_ms"], 4))
PY
