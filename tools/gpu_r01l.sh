set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r01l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_attention.py > $OUT/attn_h84.json 2>&1 || exit $?
timeout -k 10 300 python tools/bench_attention.py --codec golay > $OUT/attn_golay.json 2>&1 || exit $?
timeout -k 10 300 python tools/bench_shim.py --bers 0.001 > $OUT/shim_h84.json 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o shim -- python tools/bench_shim.py --bers 0.001 --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || exit $?
tail -1 $OUT/attn_h84.json; tail -1 $OUT/attn_golay.json; tail -1 $OUT/shim_h84.json
