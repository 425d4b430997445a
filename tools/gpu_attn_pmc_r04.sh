#!/bin/bash
# PMC of the MHA paged-attention kernels (packed Golay split kernel, H(8,4)
# matrix-core kernel): three counter passes and a kernel trace per codec,
# each under its own limit; summary: tools/pmc_table.py
# usage: tools/gpu_attn_pmc_r04.sh <tag>
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$1
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD"
for CODEC in golay_packed hamming84 golay; do
  i=0
  for P in "$P1" "$P2" "FETCH_SIZE"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex paged_attn --output-format csv \
      -d "$OUT/${CODEC}_p$i" -o p -- python tools/bench_attention.py --codec $CODEC --iters 20 --passes 1 \
      --warmup-s 0.2 > "$OUT/${CODEC}_p$i.log" 2>&1 || { echo "$CODEC pass $i failed"; tail -5 "$OUT/${CODEC}_p$i.log"; exit 1; }
  done
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${CODEC}_prof" -o p -- \
    python tools/bench_attention.py --codec $CODEC --iters 20 --passes 1 --warmup-s 0.2 > "$OUT/${CODEC}_prof.log" 2>&1 || exit 1
  echo "$CODEC done"
done
