#!/bin/bash
# The fused shim reads one variant per rocprofv3 run (int32 / packed Golay,
# plain / interpolating Hamming(8,4)), so each variant gets its own kernel
# average and HBM counters: a kernel trace with --stats, then FETCH_SIZE and
# WRITE_SIZE in passes of their own (MI355X_MICROARCH.md, HBM section).
# Driver: tools/exp/run_read_ab.py on the product library.
# usage: tools/gpu_read_variants.sh <tag>     (summary: tools/pmc_summary.py --variants)
set -u
TAG=${1:-readvar}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp ROUNDS=${ROUNDS:-20}
LIB=$ROOT/quantized-kv-cache-ecc-protection_amd/kvecc/libkvecc.so
for CASE in golay golay_packed hamming84 hamming84+interp; do
  D=$OUT/${CASE/+/_}
  mkdir -p "$D"
  for PASS in prof pmc_fetch pmc_write; do
    case $PASS in
      prof) ARGS="--kernel-trace --stats" ;;
      pmc_fetch) ARGS="--pmc FETCH_SIZE --kernel-trace" ;;
      pmc_write) ARGS="--pmc WRITE_SIZE --kernel-trace" ;;
    esac
    CASES=$CASE timeout -s KILL 120 rocprofv3 $ARGS -T --output-format csv -d "$D/$PASS" -o p -- \
      python "$ROOT/tools/exp/run_read_ab.py" "$LIB" > "$D/$PASS.log" 2>&1 ||
      { echo "$CASE $PASS failed"; tail -5 "$D/$PASS.log"; exit 1; }
  done
  echo "$CASE done"
done
echo done
