# packed Golay: >4 GiB attention test, shim bench int32 vs packed (eager + graph)
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pk3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -m gpu -x -v -k "past_4g" --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python tools/bench_shim.py --codec golay --interp 0 --bers 0 1e-3 --graph > $OUT/shim_golay_int32.json 2> $OUT/shim_golay_int32.err || exit $?
timeout -k 10 300 python tools/bench_shim.py --codec golay --interp 0 --bers 0 1e-3 --graph --golay-storage packed > $OUT/shim_golay_packed.json 2> $OUT/shim_golay_packed.err || exit $?
cat $OUT/shim_golay_int32.json $OUT/shim_golay_packed.json
