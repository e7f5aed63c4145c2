# kernel-trace (stats) of the stream decode on C2 and C3 (profiles/r02/*_kernel_stats.csv)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in c2 c3 dense; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/kt_$c -o run -- python3 $R/tools/run_decode.py $c 12 > $R/gpurun_out/kt_$c.log 2>&1 || exit 1
done
echo done
