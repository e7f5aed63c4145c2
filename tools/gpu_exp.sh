set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in exp6; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/se_$v -o run -- python3 $R/tools/scan_exp.py flashws_amd/lib/libfws_gpu_$v.so > $R/gpurun_out/se_$v.log 2>&1 || exit 1
done
echo done
