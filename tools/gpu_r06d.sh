set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06d
TORCH_LOGS=recompiles timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_torch_ops.py tests/test_kv_cache.py tests/test_shim.py -m gpu > gpurun_out/r06d/pytest.log 2>&1 && \
timeout -k 10 900 python -u tools/bench_shim.py --bers 0 1e-3 1e-2 --graph --compile inductor > gpurun_out/r06d/shim_compiled.json 2> gpurun_out/r06d/shim_compiled.err && \
timeout -k 10 600 python -u tools/bench_shim.py --no-gpu --bers 0 1e-3 1e-2 --steps 3 > gpurun_out/r06d/shim_cpu_backend.json 2> gpurun_out/r06d/shim_cpu.err
