#!/bin/bash
# Fused reads (tools/exp/run_read_ab.py on the product library) under rocprofv3
# counters, one pass per counter group, for the cases in $CASES.
# usage: tools/gpu_read_pmc2.sh <tag>
set -u
TAG=${1:-readpmc2}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp ROUNDS=${ROUNDS:-6}
LIB=$ROOT/quantized-kv-cache-ecc-protection_amd/kvecc/libkvecc.so
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"
P3="TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
P4="FETCH_SIZE"
P5="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/p$i" -o p -- \
    python "$ROOT/tools/exp/run_read_ab.py" "$LIB" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
echo done
