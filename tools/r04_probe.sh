#!/bin/bash
# round-4 probe: index-path GPU tests, the index bench line, host phase profiles of config 4 and of config 2 at 16
# segments (one rank's share at N = 8); each GPU step under its own limit, first failure ends it
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread \
  -k "inverted or index or config5 or sorted or sv_queries" > $O/probe_tests.log 2>&1 || { echo "tests failed"; tail -30 $O/probe_tests.log; exit 1; }
tail -1 $O/probe_tests.log
timeout -k 10 300 python3 bench.py --workload index --no-cpu --steps 20 --warmup 3 > $O/probe_index.json 2> $O/probe_index.err || { echo "index bench failed"; tail -20 $O/probe_index.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/probe_index.json'));print('index', round(d['ms_per_step'],3), d['step_breakdown_ms'], d['roofline']['frac'], d['parity_sample'])"
PG_HOST_PROFILE=1 timeout -k 10 300 python3 bench.py --workload highcard --no-cpu --steps 3 --warmup 1 > $O/probe_hc.json 2> $O/probe_hc.err || { echo "highcard failed"; tail -20 $O/probe_hc.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/probe_hc.json'));print('highcard', round(d['ms_per_step'],3), d['step_breakdown_ms'])"
PG_HOST_PROFILE=1 timeout -k 10 300 python3 bench.py --workload adanalytics --segments 16 --no-cpu --steps 20 --warmup 3 > $O/probe_seg16.json 2> $O/probe_seg16.err || { echo "seg16 failed"; tail -20 $O/probe_seg16.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/probe_seg16.json'));print('seg16', round(d['ms_per_step'],3), d['step_breakdown_ms'])"
