#!/bin/bash
# Round-5 GPU session steps (each with its own time limit; a fault, abort or
# timeout stops the script).  usage: tools/gpu_r05.sh <tag> [steps...]
#   launch  tests/test_gpu_launch.py (bench.py / tools/sweep.py spawn their ranks)
#   test    the whole -m gpu suite          bench  bench.py (all sections)
#   exp     tools/exp/run_r05.py            injpmc rocprofv3 VALU passes of the injection
#   prof    rocprofv3 kernel trace of bench.py       smoke  __graft_entry__.smoke()
set -u
TAG=${1:-r05}
shift || true
STEPS=${@:-launch bench}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp

run() {  # name seconds cmd...
  local name=$1 to=$2
  shift 2
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/status.txt"
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name ended with rc=$rc" | tee -a "$OUT/status.txt"
    exit $rc
  fi
  return 0
}

for s in $STEPS; do
  case $s in
    launch) run pytest_launch 600 python -u -m pytest tests/test_gpu_launch.py -x -v -p no:cacheprovider \
              --timeout 300 --timeout-method thread ;;
    test)   run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider \
              --timeout 300 --timeout-method thread ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    mctest) run pytest_mc 600 python -u -m pytest tests/test_montecarlo.py -m gpu -x -v -p no:cacheprovider \
              --timeout 300 --timeout-method thread ;;
    bench)  run bench 600 python bench.py ;;
    exp)    run exp_r05 600 python tools/exp/run_r05.py all ;;
    valu)   run valu_rate 300 python tools/exp/run_valu_rate.py ;;
    mc)     run mc_time 300 python tools/mc_time.py ;;
    gqapmc) run gqa_pmc 900 bash tools/gpu_attn_gqa_pmc.sh "$TAG" ;;
    gtf)    run gtf 600 python tools/exp/run_golay_tf_exp.py ;;
    qtest)  run pytest_quant 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider -k "quant or fused or dequant" \
              --timeout 300 --timeout-method thread ;;
    attnexp) run attn_exp 600 python tools/exp/run_attn_exp.py hamming84 golay_packed ;;
    shimtest) run pytest_shim_fp16 600 python -u -m pytest tests/test_shim_fp16.py -m gpu -x -v -p no:cacheprovider \
              --timeout 300 --timeout-method thread ;;
    itest)  run pytest_interp 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider -k "interp" \
              --timeout 300 --timeout-method thread ;;
    expi)   run exp_interp 600 python tools/exp/run_r05.py interp ;;
    expr)   run exp_rows 600 python tools/exp/run_r05.py rows ;;
    exppk)  run exp_pk 600 python tools/exp/run_r05.py pk ;;
    exprd)  run exp_rowsdec 600 python tools/exp/run_r05.py rowsdec ;;
    fuzz)   run pytest_fuzz 900 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -v -p no:cacheprovider \
              --timeout 300 --timeout-method thread ;;
    fuzz8)  KVECC_SWEEP_SCALE=8 KVECC_SWEEP_SEED=3 run pytest_fuzz8 1100 python -u -m pytest tests/test_gpu_fuzz.py \
              -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    gread)  run gread_ab 900 python tools/exp/run_golay_read_exp.py pers:2 pers_u16:2 pers_u16:3 pers_u16:4 pers:3 \
              pers_b256_p50:3 pers_b256_p50:4 full1_u16:0:0 full2_u16:0:0 ;;
    gread2) ROUNDS=60 run gread_ab2 900 python tools/exp/run_golay_read_exp.py pers:2 pers_b256:3 pers_b256_p50:3 \
              pers_b256_p40:3 pers_b256_p75:3 pers_b512_p50:2 pk_pers:2 pk_pers_b256:3 pk_pers_b256_p50:3 pk_pers_b256_p40:3 ;;
    gread3) ROUNDS=60 run gread_ab3 900 python tools/exp/run_golay_read_exp.py pers:2 pers_b256_p50:3 pers_b256_p40:3 \
              pers_b256_p30:3 pers_b256_p20:3 pers_b256_p10:3 pers_b256_p40:2 pk_pers:2 pk_pers_b256_p40:3 \
              pk_pers_b256_p30:3 pk_pers_b256_p20:3 ;;
    gread4) ROUNDS=60 run gread_ab4 900 python tools/exp/run_golay_read_exp.py pers:2 pers_b256_p30:3 pk_pers:2 \
              pk_pers_b256_p30:3 ;;
    gread5) ROUNDS=60 run gread_ab5 900 python tools/exp/run_golay_read_exp.py pers_b256_p30:3 pers_b128_p30:4 \
              pers_b128_p30:5 pers_b128_p30:6 pers_b384_p30:2 pers_u16_b256_p30:3 pers_u16_b256_p30:4 \
              pers_u16_b256_p30:5 pers_u16_b512_p30:2 pers_u16_b512_p30:3 pers_splitp_b256_p30:3 pers_splitp_b256_p30:4 \
              pk_pers_b256_p30:3 pk_pers_u16_b256_p30:3 pk_pers_u16_b256_p30:4 ;;
    pkdec)  ROUNDS=60 run pkdec_ab 900 python tools/exp/run_packed_dec_exp.py pk:2 pk_p50:2 pk_p30:2 pk_b256:3 \
              pk_b256_p50:3 pk_b256_p40:3 pk_b256_p30:3 pk_b256_p20:3 pk_b256_p30:4 pk_b256_p50:4 ;;
    fuzz40) KVECC_SWEEP_SCALE=40 KVECC_SWEEP_SEED=4 run pytest_fuzz40 1100 python -u -m pytest tests/test_gpu_fuzz.py \
              -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    sweep40b) KVECC_SWEEP_SCALE=40 KVECC_SWEEP_SEED=5 run pytest_sweep40b 1100 python -u -m pytest \
              tests/test_geometry_sweep.py tests/test_shim_read_batch.py -m gpu -v -p no:cacheprovider \
              --timeout 300 --timeout-method thread ;;
    sweep40c) KVECC_SWEEP_SCALE=40 KVECC_SWEEP_SEED=6 run pytest_sweep40c 1100 python -u -m pytest \
              tests/test_geometry_sweep.py tests/test_shim_read_batch.py tests/test_gpu_fuzz.py -m gpu -v \
              -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    sweep40d) KVECC_SWEEP_SCALE=40 KVECC_SWEEP_SEED=7 run pytest_sweep40d 1100 python -u -m pytest \
              tests/test_geometry_sweep.py tests/test_shim_read_batch.py tests/test_gpu_fuzz.py -m gpu -v \
              -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    sweep40) KVECC_SWEEP_SCALE=40 KVECC_SWEEP_SEED=2 run pytest_sweep40 1100 python -u -m pytest \
              tests/test_geometry_sweep.py tests/test_shim_read_batch.py -m gpu -v -p no:cacheprovider \
              --timeout 300 --timeout-method thread ;;
    sweep8) KVECC_SWEEP_SCALE=8 KVECC_SWEEP_SEED=1 run pytest_sweep8 1000 python -u -m pytest \
              tests/test_geometry_sweep.py tests/test_shim_read_batch.py -m gpu -x -v -p no:cacheprovider \
              --timeout 300 --timeout-method thread ;;
    rtest)  run pytest_rows 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider -k "rows or geometry or shim or golay" \
              --timeout 300 --timeout-method thread ;;
    sched)  run pytest_sched 600 python -u -m pytest tests/test_sched_counters.py -m gpu -x -v -p no:cacheprovider \
              --timeout 300 --timeout-method thread ;;
    configs) run configs 600 python tools/bench_configs.py ;;
    shim)   run shim_eager 300 python tools/bench_shim.py
            run shim_graph 300 python tools/bench_shim.py --graph ;;
    attn)   run attn_mha 300 python tools/bench_attention.py --codec hamming84
            run attn_gqa 300 python tools/bench_attention.py --codec hamming84 --kv-heads 8
            run attn_pk 300 python tools/bench_attention.py --codec golay_packed
            run attn_pk_gqa 300 python tools/bench_attention.py --codec golay_packed --kv-heads 8 ;;
    mcprof) run mc_trace 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT/mc_trace" -o t -- \
              python "$ROOT/tools/mc_time.py" --only fused ;;
    injpmc)
      run inj_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/inj_trace" -o t -- \
        python "$ROOT/tools/inject_pmc.py"
      run inj_pmc1 120 timeout -s KILL 110 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_SALU \
        --kernel-trace --output-format csv -d "$OUT/inj_pmc1" -o p -- python "$ROOT/tools/inject_pmc.py"
      run inj_pmc2 120 timeout -s KILL 110 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        --kernel-trace --output-format csv -d "$OUT/inj_pmc2" -o p -- python "$ROOT/tools/inject_pmc.py" ;;
    prof)   run prof_trace 600 rocprofv3 --kernel-trace --stats --output-format csv \
              -d "$OUT/prof" -o trace -- python "$ROOT/bench.py" --steps 20 --no-cpu-baseline ;;
    pmc)    run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
              -d "$OUT/pmc_fetch" -o fetch -- python "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline \
              --no-inject --side-warmup 5
            run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv \
              -d "$OUT/pmc_write" -o write -- python "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline \
              --no-inject --side-warmup 5 ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "done" | tee -a "$OUT/status.txt"
