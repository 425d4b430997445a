set -u
cd $GRAFT_REPO_ROOT
CODEC=${1:-golay}
OUT=gpurun_out/attn_pmc_$CODEC
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex paged_attn_split --output-format csv -d $OUT/sq -o sq -- python tools/bench_attention.py --codec $CODEC --iters 5 > $OUT/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE --kernel-include-regex paged_attn_split --output-format csv -d $OUT/sq2 -o sq2 -- python tools/bench_attention.py --codec $CODEC --iters 5 > $OUT/sq2.log 2>&1 || exit $?
find $OUT -name "*counter_collection.csv"
