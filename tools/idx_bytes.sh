#!/bin/bash
# config 5 byte attribution: FETCH_SIZE of index_count_kernel for the main library and for ablation
# variants that skip one load source each (tools/variant.sh pg_index skip<N> -DPG_IDX_SKIP=<N>: 8 the COUNTMV count
# words, 2 the large array containers' payload, 4 the bitmap containers), plus the L2->fabric request-size mix of the
# main library (TCC_EA0_RDREQ / _32B): how many of its requests are 32-B, i.e. whether FETCH_SIZE's x2 applies here.
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
KRE="pg::index_count_kernel"
for v in base skip8 skip2 skip4; do
  LIB=$R/pinot_amd/libpinot_gpu.so; [ $v != base ] && LIB=$R/pinot_amd/libpinot_gpu_$v.so
  PINOT_GPU_LIB=$LIB timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv \
    -d $O/ib_$v -o run -- python3 $R/bench.py --workload index --no-cpu --no-full-parity --steps 3 --warmup 1 \
    > $O/ib_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/ib_$v.log; exit 1; }
  python3 $R/tools/pmc_summary.py "$KRE" $O/ib_$v | tail -2
done
timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex "$KRE" --output-format csv \
  -d $O/ib_req -o run -- python3 $R/bench.py --workload index --no-cpu --no-full-parity --steps 3 --warmup 1 \
  > $O/ib_req.log 2>&1 || { echo "pmc req failed"; tail -5 $O/ib_req.log; exit 1; }
python3 $R/tools/pmc_summary.py "$KRE" $O/ib_req | tail -2
grep -h '"plan_bytes"' $O/ib_base.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('plan_bytes', d['roofline']['plan_bytes'], 'kernel_ms', d['roofline']['kernel_ms'])"
for v in base skip8 skip2 skip4 req; do rm -rf $O/ib_$v; done
