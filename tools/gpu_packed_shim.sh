# packed Golay shim cache + paged attention: GPU tests, attention timing, kernel trace
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pks
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_attention.py tests/test_shim.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for c in hamming84 golay golay_packed; do
  timeout -k 10 300 python tools/bench_attention.py --codec $c > $OUT/attn_$c.json 2>&1 || exit $?
done
cat $OUT/attn_*.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o attn -- python tools/bench_attention.py --codec golay_packed --iters 20 > $OUT/prof.log 2>&1 || exit $?
find $OUT/prof -name "*stats*"
