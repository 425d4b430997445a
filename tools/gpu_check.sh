#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace and
# HBM counter passes.  Each GPU step has its own time limit; a step that ends
# in anything but success/test-failure (fault, abort, timeout) stops the script.
# usage: tools/gpu_check.sh <tag> [steps...]   steps: test smoke bench dist prof pmc
set -u
TAG=${1:-r02}
shift || true
STEPS=${@:-test smoke bench prof pmc}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp

run() {  # name seconds cmd...
  local name=$1 to=$2
  shift 2
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/status.txt"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name ended with rc=$rc" | tee -a "$OUT/status.txt"
    exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    test)  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider \
             --timeout 120 --timeout-method thread ;;
    dist)  run bench_dist 300 python bench.py --dist --steps 20 --no-cpu-baseline --no-packed ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    prof)  run prof_trace 600 rocprofv3 --kernel-trace --stats -T --output-format csv \
             -d "$OUT/prof" -o trace -- python "$ROOT/bench.py" --steps 20 --no-cpu-baseline ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv \
             -d "$OUT/pmc_fetch" -o fetch -- python "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-inject
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv \
             -d "$OUT/pmc_write" -o write -- python "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --no-inject ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "done" | tee -a "$OUT/status.txt"
