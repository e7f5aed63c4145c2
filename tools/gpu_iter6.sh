# merge/link/emit per-workgroup trace (FWS_SCAN_PROF build), then C2 / C3 / dense kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python -u tools/prof_merge_trace.py > gpurun_out/prof_merge.json 2> gpurun_out/prof_merge.err || exit 1
cd /tmp && export TMPDIR=/tmp
for c in c2 c3 dense; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/kt_$c -o run -- python3 $R/tools/run_decode.py $c 12 > $R/gpurun_out/kt_$c.log 2>&1 || exit 1
done
echo done
