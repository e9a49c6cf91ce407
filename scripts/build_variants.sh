#!/bin/bash
# EXPERIMENT: bound-analysis builds of libmahout_cms.so into _variants/ (one per -D flag set).
set -e
cd "$(dirname "$0")/.."
mkdir -p _variants
SRC=$(python -c "import os; from mahout_amd import build_lib as b; print(' '.join(os.path.join(b.CSRC, s) for s in b.SOURCES))")
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=off -mcode-object-version=5 \
    -I/opt/rocm/include -D$v $SRC -o _variants/lib_$v.so -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &
done
wait
ls -la _variants
