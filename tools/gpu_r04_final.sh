#!/bin/bash
# Round-4 end-of-round evidence in one GPU call: the GPU suite, smoke, bench.py,
# its rocprofv3 kernel trace and FETCH/WRITE passes (tools/gpu_check.sh), then
# every fused-read variant in a rocprofv3 run of its own
# (tools/gpu_read_variants.sh).  Stops at the first failing step.
# usage: tools/gpu_r04_final.sh <tag>
set -u
TAG=${1:-r04final}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$ROOT"
bash tools/gpu_check.sh "$TAG" test smoke bench prof pmc || exit $?
grep -q "stopping" "gpurun_out/$TAG/status.txt" && exit 1
bash tools/gpu_read_variants.sh "${TAG}_readvar" || exit $?
echo final done
