#!/bin/bash
# A/B of two library builds on one box: kernel-trace stats of the bench line per library (LIBS: names of
# pinot_amd/libpinot_gpu_<name>.so, "main" = the main build), alternating; first failure ends it
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
W=${W:-adanalytics}
for r in 1 2; do
  for L in ${LIBS:-main v0}; do
    if [ "$L" = main ]; then LIB=pinot_amd/libpinot_gpu.so; else LIB=pinot_amd/libpinot_gpu_$L.so; fi
    PINOT_GPU_LIB=$PWD/$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_${L}_$r -o run \
      -- python3 bench.py --workload $W --no-cpu --steps 20 --warmup 3 $BENCH_ARGS > gpurun_out/ab_${L}_$r.json \
      2> gpurun_out/ab_${L}_$r.err || { echo "$L failed"; tail -20 gpurun_out/ab_${L}_$r.err; exit 1; }
    S=$(find gpurun_out/ab_${L}_$r -name "*kernel_stats.csv" | head -1)
    python3 - "$S" "$L" gpurun_out/ab_${L}_$r.json <<'PY'
import csv, json, sys
rows = {r["Name"].split("(")[0]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(sys.argv[1]))}
d = json.load(open(sys.argv[3]))
print(sys.argv[2], round(d["ms_per_step"], 4), {k.split("::")[-1][:28]: round(v, 2) for k, v in rows.items() if k.startswith(("pg::", "void pg::"))})
PY
    rm -rf gpurun_out/ab_${L}_$r
  done
done
