#!/bin/bash
# Fused shim reads under rocprofv3 counters: the byte-codec tile kernel
# (tools/exp/run_shim_read_h84.py: H84, H84+interp, H74, raw INT4) and the
# Golay tile kernel (tools/exp/run_shim_read.py), one counter pass per run.
# usage: tools/gpu_read_pmc.sh <tag>
set -u
TAG=${1:-readpmc}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
for prog in run_shim_read_h84 run_shim_read; do
  timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace -T --output-format csv -d "$OUT/$prog/sq" -o sq -- \
    python "$ROOT/tools/exp/$prog.py" > "$OUT/$prog.sq.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d "$OUT/$prog/fetch" -o f -- \
    python "$ROOT/tools/exp/$prog.py" > "$OUT/$prog.fetch.log" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d "$OUT/$prog/write" -o w -- \
    python "$ROOT/tools/exp/$prog.py" > "$OUT/$prog.write.log" 2>&1 || exit $?
done
echo done
