#!/bin/bash
# Build product-library variants that differ only in the wide-field NTT (ntt_wide.hpp /
# ntt_lwide.hip) into ringo-snark_amd/vlib/libringo_<name>.so, for tools/wide_ab.sh.
# usage: wide_ab_build.sh name:ntt_wide.hpp:ntt_lwide.hip ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/ringo-snark_amd
mkdir -p $C/vlib
for spec in "$@"; do
  IFS=: read -r name hpp hip <<< "$spec"
  T=$(mktemp -d)
  cp $C/csrc/*.hpp $C/csrc/*.hip $T/
  cp "$hpp" $T/ntt_wide.hpp
  cp "$hip" $T/ntt_lwide.hip
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wno-unused-function -Wno-unused-result \
    -I$R/include -I$C/csrc -c $T/ntt_lwide.hip -o $T/ntt_lwide.o
  objs=$(ls $C/build/*.o | grep -v -e ntt_lwide.o -e knobs_env.o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -Wl,-Bsymbolic -o $C/vlib/libringo_$name.so $objs $T/ntt_lwide.o
  rm -rf $T
  echo built $C/vlib/libringo_$name.so
done
