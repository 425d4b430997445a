#!/bin/bash
# PMC of the GQA paged-attention kernels at 32 query / 8 cache heads (fp16
# queries: the matrix-core split kernels and the combine kernel), H(8,4) and
# packed Golay: two counter passes, a FETCH pass and a kernel trace per codec,
# each under its own limit; summary: tools/pmc_table.py.
# usage: tools/gpu_attn_gqa_pmc.sh <tag>
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$1
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
for CODEC in hamming84 golay_packed; do
  i=0
  for P in "$P1" "$P2" "FETCH_SIZE"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex paged_attn --output-format csv \
      -d "$OUT/gqa_${CODEC}_p$i" -o p -- python tools/bench_attention.py --codec $CODEC --kv-heads 8 --iters 20 \
      --passes 1 --warmup-s 0.2 > "$OUT/gqa_${CODEC}_p$i.log" 2>&1 || { echo "$CODEC pass $i failed"; tail -5 "$OUT/gqa_${CODEC}_p$i.log"; exit 1; }
  done
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/gqa_${CODEC}_prof" -o p -- \
    python tools/bench_attention.py --codec $CODEC --kv-heads 8 --iters 20 --passes 1 --warmup-s 0.2 \
    > "$OUT/gqa_${CODEC}_prof.log" 2>&1 || exit 1
  echo "$CODEC done"
done
