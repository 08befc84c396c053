#!/bin/bash
# A/B of the streaming pre-filter on the scan probes (config 2 and config 3 shapes); each step time-limited
set -o pipefail
mkdir -p gpurun_out
for W in adanalytics ssb; do
  for PF in 0 1; do
    PG_PREFILTER=$PF timeout -k 10 240 python -u tools/scan_probe.py --workload $W --segments ${SEGS:-64} --reps 10 > gpurun_out/probe_${W}_$PF.log 2>&1 || { echo "probe $W $PF failed"; tail -20 gpurun_out/probe_${W}_$PF.log; exit 1; }
    echo "== $W PG_PREFILTER=$PF"; grep -v amdgpu.ids gpurun_out/probe_${W}_$PF.log
  done
done
