set -e
mkdir -p gpurun_out/s6
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/ab_c4.py 5 50 -1:512:4,-2:512:4,3:512:4,2:512:4 > gpurun_out/s6/ab_c4.jsonl 2>gpurun_out/s6/ab_c4.err
for f in 1 2; do
  FWS_TX_FORM=$f timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -f csv -d gpurun_out/s6/tx$f/fetch -- python3 tools/run_tx.py > /dev/null 2>&1
  FWS_TX_FORM=$f timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -f csv -d gpurun_out/s6/tx$f/rdreq -- python3 tools/run_tx.py > /dev/null 2>&1
  FWS_TX_FORM=$f timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY -f csv -d gpurun_out/s6/tx$f/sq -- python3 tools/run_tx.py > /dev/null 2>&1
done
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -f csv -d gpurun_out/s6/c4/rdreq -- python3 tools/run_c4.py > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY -f csv -d gpurun_out/s6/c4/sq -- python3 tools/run_c4.py > /dev/null 2>&1
echo done
