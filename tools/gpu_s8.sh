set -e
mkdir -p gpurun_out/s8
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -u tools/ab_tx_lib.py > gpurun_out/s8/base.jsonl 2>/dev/null
FWS_LIB_VARIANT=noseam timeout -k 10 120 python -u tools/ab_tx_lib.py > gpurun_out/s8/noseam.jsonl 2>/dev/null
timeout -k 10 120 python -u tools/ab_tx_lib.py > gpurun_out/s8/base2.jsonl 2>/dev/null
FWS_LIB_VARIANT=noseam timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY -f csv -d gpurun_out/s8/noseam_sq -- python3 tools/run_tx.py > /dev/null 2>&1
echo done
