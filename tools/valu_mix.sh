#!/bin/bash
# profiles/valu_mix.json for the current libringo.so: gfx950 assembly of the translation units
# whose kernels bench.py profiles, then tools/valu_mix.py (static VALU mix x measured class costs).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
for f in jindo mac_mfma ntt_l1_lazy ntt_l4_fast; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -std=c++17 -Wno-unused-function -Wno-unused-result \
    -I"$R/include" --cuda-device-only -S -o "$T/$f.s" "$R/ringo-snark_amd/csrc/$f.hip" 2>/dev/null &
done
wait
python3 "$R/tools/valu_mix.py" "$R/profiles/valu_mix.json" "$R/ringo-snark_amd/lib/libringo.so" "$T"/*.s
rm -rf "$T"
