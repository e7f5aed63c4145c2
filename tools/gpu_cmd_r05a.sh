set -o pipefail
O=gpurun_out/r05; mkdir -p $O
for v in "" swar "" swar; do FWS_LIB_VARIANT=$v timeout -k 10 200 python tools/ab_c5d.py >> $O/ab_c5d.jsonl 2>> $O/ab_c5d.err || exit 1; done
cat $O/ab_c5d.jsonl
cd /tmp && export TMPDIR=/tmp
for v in "" swar; do
FWS_LIB_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -f csv -d $GRAFT_REPO_ROOT/$O/sq_c5d_${v:-product} -o run -- python3 $GRAFT_REPO_ROOT/tools/run_c5_desc.py > $GRAFT_REPO_ROOT/$O/sq_c5d_${v:-product}.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT && python3 tools/sq_summary.py $O/sq_c5d_product --note product | grep -A10 'k_unmask_sorted_utf8' && python3 tools/sq_summary.py $O/sq_c5d_swar --note swar | grep -A10 'k_unmask_sorted_utf8'
