#!/bin/bash
# GPU session steps for gpurun (each step under its own time limit; a fault,
# abort or timeout stops the script, so nothing else runs on a sick GPU).
#
#   usage: bash tools/gpu_session.sh <tag> <step> [step ...]
#   output: gpurun_out/<tag>/<step>.log and status.txt
#
# Steps
#   test      the whole -m gpu suite              smoke    __graft_entry__.smoke()
#   launch    tests/test_gpu_launch.py            bench    bench.py (every section)
#   shimtest  the fused shim reads' tests, sweeps and fuzz   fused  bench.py --sections fused
#   prof      rocprofv3 kernel trace + stats of bench.py (the roofline's kernel times)
#   pmc       FETCH_SIZE / WRITE_SIZE passes of bench.py (traffic.json)
#   injpmc    VALU counter passes of the injection + the VALU microbenchmark
#   attnpmc   SQ counter pass (VALU, LDS, bank conflicts, waits) of MHA paged attention per codec
#   valu      tools/exp/run_valu_rate2.py (issue cost vs chains / waves)
#   configs   tools/bench_configs.py (every BASELINE config's kernels)
#   shim      tools/bench_shim.py: config 4 eager, HIP graph, inductor; host backend
#   attn      tools/bench_attention.py, MHA and GQA, every codec
#   fuzz40    the geometry sweep + GPU fuzz at 40x (KVECC_SWEEP_SCALE), seed $SEED
#   ipe       tools/exp/run_interp_read_exp.py (interpolating read A/B)
#   gread     tools/exp/run_golay_read_exp.py $GREAD (fused Golay read A/B)
#   attnexp   tools/exp/run_attn_exp.py $ATTN (attention A/B)
set -u
TAG=${1:?tag}
shift
STEPS=${@:-test bench}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
PYT="python -u -m pytest -p no:cacheprovider --timeout 600 --timeout-method thread"

run() {  # name seconds cmd...
  local name=$1 to=$2
  shift 2
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/status.txt"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then
    echo "stopping: $name ended with rc=$rc" | tee -a "$OUT/status.txt"
    exit $rc
  fi
}

pmc() {  # name counters... -- one rocprofv3 --pmc pass over a python program
  local name=$1
  shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  run "$name" 180 timeout -s KILL 170 rocprofv3 --pmc "${ctr[@]}" --kernel-trace --output-format csv \
    -d "$OUT/$name" -o p -- python "$@"
}

for s in $STEPS; do
  case $s in
    test)    run pytest_gpu 1500 $PYT tests -m gpu -x -v ;;
    launch)  run pytest_launch 600 $PYT tests/test_gpu_launch.py -m gpu -x -v ;;
    shimtest) run pytest_shim 900 $PYT tests/test_shim_read_batch.py tests/test_geometry_sweep.py tests/test_gpu_fuzz.py \
               tests/test_shim.py tests/test_shim_fp16.py tests/test_sched_counters.py -m gpu -x -v ;;
    fused)   run bench_fused 600 python bench.py --sections fused ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   run bench 600 python bench.py ;;
    prof)    run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o trace -- \
               python "$ROOT/bench.py" --steps 20 --sections inject,packed,fused,rows,interp,quant,montecarlo ;;
    pmc)     pmc pmc_fetch FETCH_SIZE -- "$ROOT/bench.py" --steps 5 --warmup 1 --sections fused,rows,interp,quant \
               --side-warmup 5
             pmc pmc_write WRITE_SIZE -- "$ROOT/bench.py" --steps 5 --warmup 1 --sections fused,rows,interp,quant \
               --side-warmup 5 ;;
    injpmc)  run inj_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/inj_trace" -o t -- \
               python "$ROOT/tools/inject_pmc.py"
             pmc inj_pmc3 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_BUSY_CYCLES -- \
               "$ROOT/tools/inject_pmc.py"
             QUICK=1 pmc valu_pmc3 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_BUSY_CYCLES -- \
               "$ROOT/tools/exp/run_valu_rate2.py" ;;
    attnpmc) for c in golay golay_packed hamming84; do
               pmc attnpmc_$c SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
                 SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES -- "$ROOT/tools/bench_attention.py" --codec $c \
                 --iters 20 --passes 1 --warmup 20 --warmup-s 0.1
             done ;;
    valu)    run valu_rate2 300 python tools/exp/run_valu_rate2.py "$OUT/valu_rate2.json" ;;
    configs) run configs 900 python tools/bench_configs.py ;;
    shim)    run shim_compiled 900 python tools/bench_shim.py --bers 0 1e-3 1e-2 --graph --compile inductor
             run shim_host 900 python tools/bench_shim.py --no-gpu --bers 0 1e-3 1e-2 --steps 3 ;;
    attn)    run attn_mha 300 python tools/bench_attention.py --codec hamming84
             run attn_mha_golay 300 python tools/bench_attention.py --codec golay
             run attn_mha_pk 300 python tools/bench_attention.py --codec golay_packed
             run attn_gqa 300 python tools/bench_attention.py --codec hamming84 --kv-heads 8
             run attn_gqa_golay 300 python tools/bench_attention.py --codec golay --kv-heads 8
             run attn_gqa_pk 300 python tools/bench_attention.py --codec golay_packed --kv-heads 8 ;;
    fuzz40)  KVECC_SWEEP_SCALE=40 KVECC_SWEEP_SEED=${SEED:-8} run pytest_sweep40 1400 $PYT \
               tests/test_geometry_sweep.py tests/test_shim_read_batch.py tests/test_gpu_fuzz.py -m gpu -v ;;
    ipe)     run ipe 300 python tools/exp/run_interp_read_exp.py ${IPE:-} ;;
    gread)   ROUNDS=${ROUNDS:-60} run gread 900 python tools/exp/run_golay_read_exp.py ${GREAD:-} ;;
    attnexp) run attn_exp 600 python tools/exp/run_attn_exp.py ${ATTN:-} ;;
    *) echo "unknown step $s" | tee -a "$OUT/status.txt"; exit 2 ;;
  esac
done
echo "done" | tee -a "$OUT/status.txt"
