#!/bin/bash
# Packed Golay decode variants (csrc/packed.hip knobs) for
# tools/exp/run_packed_dec_ab.py: libpk_<name>.so = packed.hip + runtime.hip.
set -e
cd "$(dirname "$0")"
ROOT=$(cd ../.. && pwd)
CSRC=$ROOT/quantized-kv-cache-ecc-protection_amd/csrc
CC="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -fvisibility=hidden -I$ROOT/include -I$CSRC"
build() {  # name flags...
  local name=$1; shift
  $CC "$@" -o libpk_$name.so $CSRC/packed.hip $CSRC/runtime.hip &
}
# round-2 staged workgroup-tile kernel at 2 and 32 workgroups per CU
build old2 -DKVECC_PACKED_DEC_V2=0 -DKVECC_PACKED_DEC_PER_CU=2
build old32 -DKVECC_PACKED_DEC_V2=0
# wave-tile kernel: static schedule; 2 / 4 workgroups per CU
build v2nodyn -DKVECC_PACKED_DEC_DYN=0
build v2cu2 -DKVECC_PACKED_DEC_V2_PER_CU=2
build v2cu4 -DKVECC_PACKED_DEC_V2_PER_CU=4
# Hamming(8,4) packed decode: the round-2 grid-stride kernel; 2 / 8 chunks per lane
build h84old -DKVECC_H84_PACKED_V2=0
build h84c2 -DKVECC_H84_PACKED_CHUNKS=2
build h84c8 -DKVECC_H84_PACKED_CHUNKS=8
wait
ls -la libpk_*.so
