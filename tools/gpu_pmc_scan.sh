set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH"
timeout -s KILL 90 rocprofv3 --pmc $P1 -f csv -d $R/gpurun_out/pmc_scan1 -o run -- python3 $R/tools/run_decode.py c3 4 > $R/gpurun_out/pmc_scan1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $P2 -f csv -d $R/gpurun_out/pmc_scan2 -o run -- python3 $R/tools/run_decode.py c3 4 > $R/gpurun_out/pmc_scan2.log 2>&1
echo rc=$?
