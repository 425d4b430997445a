#!/bin/bash
# Round 4, GPU call A: the fused Golay read variants (tools/exp/libgread.so:
# timing A/B, a rocprofv3 trace, and SQ counter passes that attribute the LDS
# bank conflicts), then SQ counters of the MHA paged-attention kernels
# (Hamming(8,4) and packed Golay).  Every step has its own time limit; the
# script stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-r04a}
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
}
step ab 300 python -u tools/exp/run_golay_read_exp.py
tail -30 "$OUT/ab.log"
SEL="pers:2 pers_cfree:2 pers_nogather:2 full1_glds:0:0 full1_glds:0:28 full2_glds:0:0 pk_pers:2 pk_full1_glds:0:0"
export ROUNDS=6
step prof 180 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/prof" -o p -- \
  python -u tools/exp/run_golay_read_exp.py $SEL
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  step pmc$i 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d "$OUT/pmc$i" -o p -- \
    python -u tools/exp/run_golay_read_exp.py $SEL
done
unset ROUNDS
PA1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
PA2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD"
for CODEC in hamming84 golay_packed golay; do
  j=0
  for P in "$PA1" "$PA2" "FETCH_SIZE"; do
    j=$((j + 1))
    step attn_${CODEC}_$j 120 rocprofv3 --pmc $P --kernel-trace --kernel-include-regex paged_attn --output-format csv \
      -d "$OUT/attn_${CODEC}_$j" -o p -- python -u tools/bench_attention.py --codec $CODEC --iters 10 --warmup 20
  done
  step attn_${CODEC}_prof 120 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/attn_${CODEC}_prof" -o p -- \
    python -u tools/bench_attention.py --codec $CODEC --iters 100
done
echo done
