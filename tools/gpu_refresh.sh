#!/bin/bash
# Refresh the per-config measurements: every BASELINE config (bench_configs),
# config 4 through the shim (hip fused, golay), and a kernel trace of the shim.
# usage: tools/gpu_refresh.sh <tag>
set -u
TAG=${1:-refresh}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
step() {  # name seconds cmd... ; stops the script on anything but success
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/status.txt"
  [ $rc -eq 0 ] || exit $rc
}
step configs 400 python tools/bench_configs.py
step shim_h84 300 python tools/bench_shim.py
step shim_golay 300 python tools/bench_shim.py --codec golay --interp 0
step shim_trace 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/shim_trace" -o s -- \
  python "$ROOT/tools/bench_shim.py" --bers 1e-3 --steps 5 --warmup 2
echo done
