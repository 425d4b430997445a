#!/bin/bash
# Fused-read work-distribution variants (csrc/shim.hip knobs) for
# tools/exp/run_read_ab.py: libread_<name>.so = shim.hip + runtime.hip.
# LDS per workgroup (static): Golay tiles 52 KiB at block 512 / 42 KiB at 256
# (32 KiB tables + 2.25 KiB tile + 256 B scales per wave); byte codecs 20 / 10 KiB.
# *_LDS_PAD adds dynamic LDS so only the named workgroups fit in a CU's 160 KiB.
set -e
cd "$(dirname "$0")"
ROOT=$(cd ../.. && pwd)
CSRC=$ROOT/quantized-kv-cache-ecc-protection_amd/csrc
CC="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -fvisibility=hidden -I$ROOT/include -I$CSRC"
build() {  # name flags...
  local name=$1; shift
  $CC "$@" -o libread_$name.so $CSRC/shim.hip $CSRC/runtime.hip &
}
# dynamic tile schedule: off; per wave (DYN 1, the product) at 65 %;
# per workgroup (DYN 2) at 50 / 75 / 90 % static
build nodyn -DKVECC_SHIM_TILE_DYN=0
build pct65 -DKVECC_SHIM_TILE_DYN_STATIC_PCT=65
for p in 50 75 90; do
  build wg$p -DKVECC_SHIM_TILE_DYN=2 -DKVECC_SHIM_BYTES_DYN=1 -DKVECC_SHIM_TILE_DYN_STATIC_PCT=$p
done
wait
ls -la libread_*.so
