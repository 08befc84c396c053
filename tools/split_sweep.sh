#!/bin/bash
# A/B of the config-4 split kernels' chunk / block size: one libpinot_gpu.so per variant under variants/ (built on
# the CPU with -DPG_SPLIT_CHUNK / -DPG_SPLIT_THREADS), each profiled over bench.py --workload highcard.
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  export PINOT_GPU_LIB=$R/variants/lib_$v.so
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ss_$v -o run -- \
    python3 $R/bench.py --workload highcard --no-cpu --steps 10 --warmup 3 > $O/ss_$v.json 2> $O/ss_$v.err \
    || { echo "variant $v failed"; tail -20 $O/ss_$v.err; exit 1; }
  python3 $R/tools/trace_summary.py $O/ss_$v "pg::(scan|stream|part_[a-z0-9]+)_kernel" > $O/ss_${v}_trace.txt
  rm -rf $O/ss_$v
  echo "== $v $(grep -o '"ms_per_step": [0-9.]*' $O/ss_$v.json)"; cat $O/ss_${v}_trace.txt
done
