#!/bin/bash
# Link a variant libpinot_gpu with pg_kernels.hip built under extra -D flags: tools/kernels_variant.sh <name> <flags...>
# -> pinot_amd/libpinot_gpu_<name>.so (select it with PINOT_GPU_LIB).  Needs the main build's objects, up to date.
set -e
N=$1; shift
cd "$(dirname "$0")/../pinot_amd/csrc"
HIPCC=/opt/rocm/bin/hipcc
make -q || { echo "main build out of date: run make first"; exit 1; }
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-value -Wno-unused-result -I../../include"
$HIPCC $FL "$@" -c pg_kernels.hip -o build/pg_kernels_$N.o
OBJS=$(ls build/*.o | grep -v 'pg_kernels' | grep -v 'pg_part_' | tr '\n' ' ')
$HIPCC --offload-arch=gfx950 -shared -o ../libpinot_gpu_$N.so $OBJS build/pg_kernels_$N.o
echo "$*" > ../libpinot_gpu_$N.flags
echo built ../libpinot_gpu_$N.so "($*)"
