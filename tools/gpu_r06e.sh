# VALU evidence for the injection roofline: issue cost vs
# chains / waves in flight, and an independent VALU-busy counter pass
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/r06e
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u $ROOT/tools/exp/run_valu_rate2.py $OUT/valu_rate2.json > $OUT/valu_rate2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/inj_trace -o t -- \
  python $ROOT/tools/inject_pmc.py > $OUT/inj_trace.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_BUSY_CYCLES \
  --kernel-trace --output-format csv -d $OUT/inj_pmc3 -o p -- python $ROOT/tools/inject_pmc.py > $OUT/inj_pmc3.log 2>&1 && \
QUICK=1 timeout -s KILL 120 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_BUSY_CYCLES \
  --kernel-trace --output-format csv -d $OUT/valu_pmc3 -o p -- python $ROOT/tools/exp/run_valu_rate2.py > $OUT/valu_pmc3.log 2>&1
