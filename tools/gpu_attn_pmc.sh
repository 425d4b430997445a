set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r01k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex paged_attn --output-format csv -d $OUT/sq -o sq -- python tools/bench_attention.py --iters 5 > $OUT/sq.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-include-regex paged_attn --output-format csv -d $OUT/fetch -o fetch -- python tools/bench_attention.py --iters 5 > $OUT/fetch.log 2>&1 || exit $?
find $OUT -name "*counter_collection.csv"
