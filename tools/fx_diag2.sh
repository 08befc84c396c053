#!/bin/bash
set -o pipefail
timeout -k 10 200 python -u tools/fx_diag2.py > gpurun_out/fx_diag2.log 2>&1 || exit 1
PG_STAGE_KB=0 timeout -k 10 200 python -u tools/fx_diag2.py >> gpurun_out/fx_diag2.log 2>&1
