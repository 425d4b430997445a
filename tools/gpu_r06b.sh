set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06b
timeout -k 10 200 python -u tools/exp/run_interp_read_exp.py > gpurun_out/r06b/ipe_1e-3.log 2>&1 && \
BER=1e-2 timeout -k 10 200 python -u tools/exp/run_interp_read_exp.py product plain ipe8:16 ipe4:8 ipe2:0 ipe1:0 > gpurun_out/r06b/ipe_1e-2.log 2>&1 && \
BER=0 timeout -k 10 200 python -u tools/exp/run_interp_read_exp.py product plain ipe8:16 ipe4:8 ipe2:0 > gpurun_out/r06b/ipe_0.log 2>&1
