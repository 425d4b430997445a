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
# full grid (CHUNK P: wave w takes tiles [wP, wP + P), workgroups retire and are
# replaced) for the byte-codec kernel at 8 / 4 / 2 / 1 workgroups per CU
# (LDS 20 KiB + pad), and for the Golay kernel (its 32 KiB table per workgroup)
build bc1 -DKVECC_SHIM_BYTES_CHUNK=1
build bc1p4 -DKVECC_SHIM_BYTES_CHUNK=1 -DKVECC_SHIM_BYTES_LDS_PAD=16384
build bc1p2 -DKVECC_SHIM_BYTES_CHUNK=1 -DKVECC_SHIM_BYTES_LDS_PAD=40960
build bc1p1 -DKVECC_SHIM_BYTES_CHUNK=1 -DKVECC_SHIM_BYTES_LDS_PAD=65536
build bc2p2 -DKVECC_SHIM_BYTES_CHUNK=2 -DKVECC_SHIM_BYTES_LDS_PAD=40960
build tc4 -DKVECC_SHIM_TILE_CHUNK=4 -DKVECC_SHIM_BYTES_CHUNK=0
build tc8 -DKVECC_SHIM_TILE_CHUNK=8 -DKVECC_SHIM_BYTES_CHUNK=0
wait
ls -la libread_*.so
