#!/bin/bash
# One GPU call: the whole -m gpu suite, then the config-5 sweep (36 trials,
# [8,4096,32,128]) timed and under a rocprofv3 kernel trace.
# usage: tools/gpu_suite_sweep.sh <tag>
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-suite}
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/sweep.py > "$OUT/sweep_1gpu.log" 2>&1 || { echo "sweep failed"; tail -5 "$OUT/sweep_1gpu.log"; exit 1; }
tail -1 "$OUT/sweep_1gpu.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/sweep_prof" -o p -- \
  python -u tools/sweep.py > "$OUT/sweep_prof.log" 2>&1 || { echo "sweep prof failed"; exit 1; }
echo done
exit $rc
