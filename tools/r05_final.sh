#!/bin/bash
# round-5 closing check: smoke, the whole GPU suite, every workload's bench line (full parity), then config 2 at 16
# segments per GPU with its kernel trace (the strong-scaling slice of the 1 B-row table).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05f_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/r05f_smoke.log; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05f_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/r05f_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r05f_gpu_tests.log
bash tools/r05_bench_all.sh || exit 1
R=$(pwd); O=$R/gpurun_out
timeout -k 10 300 python3 bench.py --segments 16 --no-cpu > $O/r05f_seg16_bench.json 2> $O/r05f_seg16_bench.err || { echo "seg16 bench failed"; tail -5 $O/r05f_seg16_bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05f_seg16_prof -o run -- \
  python3 $R/bench.py --segments 16 --no-cpu --steps 20 --warmup 5 > $O/r05f_seg16_prof_bench.json 2> $O/r05f_seg16_prof.err || { echo "seg16 trace failed"; exit 1; }
cp $(find $O/r05f_seg16_prof -name '*kernel_stats.csv' | head -1) $O/r05f_seg16_kernel_stats.csv
python3 $R/tools/trace_summary.py $O/r05f_seg16_prof "pg::(scan|stream)_kernel" > $O/r05f_seg16_scan_trace.txt
rm -rf $O/r05f_seg16_prof
cd $R && python3 -c "import json; d=json.load(open('gpurun_out/r05f_seg16_bench.json')); print('seg16', round(d['ms_per_step'],4), d['step_breakdown_ms'])"
cat gpurun_out/r05f_seg16_scan_trace.txt
echo "r05 final ok"
