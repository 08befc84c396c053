#!/bin/bash
# PMC passes over the scan probe (one counter group per run, separate processes)
R=$(pwd)
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
Q=${1:-count,config2}
run() { timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex scan_kernel --output-format csv -d $R/gpurun_out/pmc_$1 -o run -- python3 $R/tools/scan_probe.py --reps 1 --only $Q > $R/gpurun_out/pmc_$1.log 2>&1; }
run sq "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" && \
run sq2 "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT" && \
run tcc "FETCH_SIZE" && echo pmc-ok
python3 $R/tools/pmc_summary.py scan_kernel $R/gpurun_out/pmc_sq $R/gpurun_out/pmc_sq2 $R/gpurun_out/pmc_tcc > $R/gpurun_out/pmc_summary.txt
rm -rf $R/gpurun_out/pmc_sq $R/gpurun_out/pmc_sq2 $R/gpurun_out/pmc_tcc
