#!/bin/bash
# Link a variant libpinot_gpu with pg_part.hip built under extra -D flags: tools/part_variant.sh <name> <flags...>
# -> pinot_amd/libpinot_gpu_<name>.so (select it with PINOT_GPU_LIB).  Needs the main build's objects.
set -e
N=$1; shift
cd "$(dirname "$0")/../pinot_amd/csrc"
HIPCC=/opt/rocm/bin/hipcc
# the variant links the main build's other objects: they must be built from the current headers (a PartSpec /
# QuerySpec layout that differs between the runtime object and the variant kernel is an out-of-bounds read waiting
# to happen -- one of the two candidate causes of the r03 sw_abl4 fault, the other a knob outside its LDS bounds)
make -q || { echo "main build out of date: run make first"; exit 1; }
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -munsafe-fp-atomics -Wall -Wno-unused-function -Wno-unused-variable -Wno-unused-value -Wno-unused-result -I../../include"
$HIPCC $FL "$@" -c pg_part.hip -o build/pg_part_$N.o
OBJS=$(ls build/*.o | grep -v 'pg_part' | tr '\n' ' ')
$HIPCC --offload-arch=gfx950 -shared -o ../libpinot_gpu_$N.so $OBJS build/pg_part_$N.o
echo "$*" > ../libpinot_gpu_$N.flags  # the -D flags of this variant, read back by part_sweep.sh
echo built ../libpinot_gpu_$N.so "($*)"
