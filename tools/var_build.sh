#!/bin/bash
# Build a product-library variant into ringo-snark_amd/vlib/libringo_<name>.so: the current
# objects, with the given translation units recompiled from replacement sources.
# usage: var_build.sh <name> <tu.hip>=<source path> [<header.hpp>=<path> ...]
#   (headers only replace the copy the recompiled units see)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/ringo-snark_amd
name=$1; shift
mkdir -p $C/vlib
T=$(mktemp -d)
cp $C/csrc/*.hpp $C/csrc/*.hip $T/
tus=()
for spec in "$@"; do
  f=${spec%%=*}; src=${spec#*=}
  cp "$src" $T/$f
  case $f in *.hip) tus+=($f);; esac
done
skip=""
for f in "${tus[@]}"; do
  b=${f%.hip}
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wno-unused-function -Wno-unused-result \
    -I$R/include -I$C/csrc -c $T/$f -o $T/$b.o
  skip="$skip -e /$b.o"
done
# a name starting with exp_ links the experiments build's knobs (RINGO_* switches, rg_set_probe)
case $name in exp_*) drop=knobs.o;; *) drop=knobs_env.o;; esac
objs=$(ls $C/build/*.o | grep -v -e "/$drop" $skip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -Wl,-Bsymbolic -o $C/vlib/libringo_$name.so $objs $(for f in "${tus[@]}"; do echo $T/${f%.hip}.o; done)
rm -rf $T
echo built $C/vlib/libringo_$name.so
