set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r01q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_torchrun1.log 2>&1 || exit $?
tail -1 $OUT/bench_torchrun1.log | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 tools/sweep.py --output $OUT/sweep.jsonl > $OUT/sweep.log 2>&1 || exit $?
tail -2 $OUT/sweep.log
