#!/bin/bash
# One GPU call: selected GPU tests, then an A/B script.  Each step has its own
# time limit; anything but success / test failure stops the script.
# usage: tools/gpu_ab.sh <tag> "<pytest targets or ->" <ab script> [ab args...]
set -u
TAG=$1; TESTS=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
if [ "$TESTS" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u "$@" > "$OUT/ab.log" 2>&1
  rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.log" | tail -40
  exit $rc
fi
