# Golay spread-table attention: GPU attention/shim tests, then the A/B vs the 16-bit tables
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-spread}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_attention.py tests/test_shim.py tests/test_gpu_large.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python tools/exp/run_attn.py > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
