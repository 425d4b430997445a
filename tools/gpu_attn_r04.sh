#!/bin/bash
# Paged attention, every codec, MHA 32/32 and GQA 32q/8kv, one JSON line each
# (tools/bench_attention.py) into gpurun_out/$1/attn_bench.jsonl: random cache
# bytes (the decode tables' worst case) and encoded values with bit errors
set -u
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$1
mkdir -p "$OUT"
for data in random encoded; do
  for codec in hamming84 golay golay_packed; do
    for kvh in 32 8; do
      timeout -k 10 120 python -u tools/bench_attention.py --codec $codec --kv-heads $kvh --data $data \
        >> "$OUT/attn_bench.jsonl" || exit $?
    done
  done
done
