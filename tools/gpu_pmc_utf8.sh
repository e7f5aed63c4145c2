# SQ counters of the C5 descriptor kernels (fused unmask + UTF-8, plain unmask)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
LIB=${1:-flashws_amd/lib/libfws_gpu.so}
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
P3="SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $P1 -f csv -d $R/gpurun_out/pmc_u1 -o run -- python3 $R/tools/utf8_exp.py $LIB 0 3 > $R/gpurun_out/pmc_u1.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc $P2 -f csv -d $R/gpurun_out/pmc_u2 -o run -- python3 $R/tools/utf8_exp.py $LIB 0 3 > $R/gpurun_out/pmc_u2.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc $P3 -f csv -d $R/gpurun_out/pmc_u3 -o run -- python3 $R/tools/utf8_exp.py $LIB 0 3 > $R/gpurun_out/pmc_u3.log 2>&1
echo rc=$?
