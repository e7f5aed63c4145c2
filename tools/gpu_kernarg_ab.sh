# k_merge / k_link / k_emit durations with kernel arguments in device memory vs the runtime default
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/ka_$v -o run -- python3 $R/tools/run_decode.py c3 12 > $R/gpurun_out/ka_$v.log 2>&1 || exit 1
done
echo done
