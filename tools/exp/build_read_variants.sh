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
# (both kernels use at most 128 VGPRs: 16 waves per CU at most)
# block 512: Golay 2 WG/CU (16 waves) with pad 8192; bytes 2 WG/CU with pad 40960
for c in 1 2 4 8; do
  build c${c}b512w16 -DKVECC_SHIM_TILE_CHUNK=$c -DKVECC_SHIM_TILE_LDS_PAD=8192 -DKVECC_SHIM_BYTES_LDS_PAD=40960
done
# block 1024: 1 WG/CU (16 waves): Golay pad 12288, bytes pad 45056
for c in 1 2 4; do
  build c${c}b1024w16 -DKVECC_SHIM_TILE_BLOCK=1024 -DKVECC_SHIM_TILE_CHUNK=$c -DKVECC_SHIM_TILE_LDS_PAD=12288 \
    -DKVECC_SHIM_BYTES_LDS_PAD=45056
done
wait
ls -la libread_*.so
