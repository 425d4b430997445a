set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06a
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_launch.py tests/test_sched_counters.py tests/test_montecarlo.py -m gpu > gpurun_out/r06a/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r06a/bench.json 2> gpurun_out/r06a/bench.err
