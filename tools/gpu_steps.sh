#!/bin/bash
# One GPU call running several steps, each under its own time limit; stops at
# the first failure (pytest exit 1 = test failures also stops the run).
# usage: tools/gpu_steps.sh <tag> "<step 1 command>" "<step 2 command>" ...
#   a step "pytest:<targets>" runs python -m pytest <targets> -m gpu
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
i=0
for STEP in "$@"; do
  i=$((i + 1))
  if [[ "$STEP" == pytest:* ]]; then
    timeout -k 10 900 python -u -m pytest ${STEP#pytest:} -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread > "$OUT/step$i.log" 2>&1
  else
    timeout -k 10 600 bash -c "$STEP" > "$OUT/step$i.log" 2>&1
  fi
  rc=$?
  echo "step $i rc=$rc: $STEP"
  tail -25 "$OUT/step$i.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo done
