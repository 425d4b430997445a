set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r01j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_attention.py tests/test_shim.py -m gpu -x -q -p no:cacheprovider > $OUT/pytest_attn.log 2>&1; rc=$?
tail -5 $OUT/pytest_attn.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_attention.py > $OUT/attn_h84.json 2>&1 || exit $?
timeout -k 10 300 python tools/bench_attention.py --codec golay > $OUT/attn_golay.json 2>&1 || exit $?
timeout -k 10 300 python tools/bench_attention.py --batch 1 --heads 12 --kv-heads 12 --d 64 --ctx 1024 > $OUT/attn_gpt2.json 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o attn -- python tools/bench_attention.py --iters 20 > $OUT/prof.log 2>&1 || exit $?
cat $OUT/attn_h84.json $OUT/attn_golay.json $OUT/attn_gpt2.json
find $OUT/prof -name "*stats*" | head
