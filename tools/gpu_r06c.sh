set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06c
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_shim_read_batch.py tests/test_geometry_sweep.py tests/test_sched_counters.py tests/test_shim.py tests/test_shim_fp16.py -m gpu > gpurun_out/r06c/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --sections fused > gpurun_out/r06c/bench_fused.json 2> gpurun_out/r06c/bench.err
