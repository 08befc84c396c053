#!/bin/bash
# TCP (L1) counters of one bench workload's kernels: translation misses and the TCP->TCC read latency (dev tool, one
# counter pass): tools/pmc_tcp.sh <workload>
set -o pipefail
WL=${1:-index}; R=$(pwd); O=$R/gpurun_out; mkdir -p $O
KRE=${KRE:-pg::(scan|stream|part_[a-z0-9]+|index_count)_kernel}
CTR=${CTR:-TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc $CTR --kernel-include-regex "$KRE" --output-format csv -d $O/tcp_$WL -o run -- \
  python3 $R/bench.py --workload $WL --no-cpu --no-full-parity --steps 2 --warmup 1 > $O/tcp_$WL.log 2>&1 || { echo "pmc failed"; tail -5 $O/tcp_$WL.log; exit 1; }
python3 $R/tools/pmc_summary.py "$KRE" $O/tcp_$WL > $O/tcp_$WL.txt
rm -rf $O/tcp_$WL
tail -4 $O/tcp_$WL.txt
