#!/bin/bash
# kbench variants under rocprofv3: kernel trace + the two HBM counter passes.
# usage: tools/gpu_kpmc.sh <tag> <kbench --which list> [rounds]
set -u
TAG=$1; WHICH=$2; R=${3:-5}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/kbench.py --which "$WHICH" --rounds "$R" > "$OUT/kbench.json" 2> "$OUT/kbench.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/trace" -o t -- \
  python "$ROOT/tools/kbench.py" --which "$WHICH" --rounds 3 > "$OUT/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d "$OUT/fetch" -o f -- \
  python "$ROOT/tools/kbench.py" --which "$WHICH" --rounds 2 > "$OUT/fetch.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d "$OUT/write" -o w -- \
  python "$ROOT/tools/kbench.py" --which "$WHICH" --rounds 2 > "$OUT/write.log" 2>&1 || exit $?
echo done
