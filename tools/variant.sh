#!/bin/bash
# Link a variant libpinot_gpu with one source built under extra -D flags:
#   tools/variant.sh <source stem, e.g. pg_part> <name> <flags...>  -> pinot_amd/libpinot_gpu_<name>.so
# (select it with PINOT_GPU_LIB; delete it after the run -- every gpurun call ships the tree).  Needs the main build's
# objects, up to date: a spec struct whose layout differs between the runtime object and the variant kernel is an
# out-of-bounds read waiting to happen.
set -e
SRC=$1; N=$2; shift 2
cd "$(dirname "$0")/../pinot_amd/csrc"
HIPCC=/opt/rocm/bin/hipcc
make -q || { echo "main build out of date: run make first"; exit 1; }
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-value -Wno-unused-result -I../../include"
$HIPCC $FL "$@" -c $SRC.hip -o build/var_${SRC}_$N.o
OBJS=$(ls build/*.o | grep -v "/$SRC.o" | grep -v '/var_' | tr '\n' ' ')
$HIPCC --offload-arch=gfx950 -shared -o ../libpinot_gpu_$N.so $OBJS build/var_${SRC}_$N.o
rm -f build/var_${SRC}_$N.o
echo "$SRC $*" > ../libpinot_gpu_$N.flags
echo built ../libpinot_gpu_$N.so "($SRC $*)"
