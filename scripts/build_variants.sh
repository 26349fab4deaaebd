#!/bin/bash
# Diagnostic: libnsgpu variants of the p2p engine built with one -D override each (lib/libnsgpu_<name>.so),
# for scripts/variants.py.  Usage: build_variants.sh NAME=-DFLAG=V ...
set -e
cd "$(dirname "$0")/../ns-3-dev-dnemu_amd"
make -s -j8 lib/libnsgpu.so
OTHERS=$(ls build/nsgpu_*.o | grep -v nsgpu_p2p.o)
for spec in "$@"; do
  name=${spec%%=*}
  flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -Wall \
    -Wno-unused-function -I../include $flags -c csrc/nsgpu_p2p.hip -o build/var_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libnsgpu_$name.so build/var_$name.o $OTHERS \
    -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl
  echo "lib/libnsgpu_$name.so"
done
