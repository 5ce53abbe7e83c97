#!/bin/bash
# build profiling variants of libringo (jindo.hip with -DRG_VAR=n) into lib/var<n>/libringo.so
set -e
cd $(dirname $0)/../ringo-snark_amd
for v in "$@"; do
  mkdir -p build/var$v lib/var$v
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -DRG_VAR=$v -c -o build/var$v/jindo.o csrc/jindo.hip &
done
wait
for v in "$@"; do
  objs=$(ls build/*.o | grep -v jindo.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/var$v/libringo.so $objs build/var$v/jindo.o
done
