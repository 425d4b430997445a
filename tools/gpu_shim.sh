set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r01i
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/r01i/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/r01i/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_shim.py --cpu-backend > gpurun_out/r01i/shim_fused.json 2> gpurun_out/r01i/shim_fused.err || exit $?
timeout -k 10 300 python tools/bench_shim.py --composed > gpurun_out/r01i/shim_composed.json 2> gpurun_out/r01i/shim_composed.err || exit $?
timeout -k 10 300 python tools/bench_shim.py --codec golay --interp 0 > gpurun_out/r01i/shim_golay_fused.json 2>&1 || exit $?
cat gpurun_out/r01i/shim_fused.json gpurun_out/r01i/shim_composed.json
