# k_scan phase clocks on C2 / C3 / a 256 MiB C5 slice, and the kernel stats of that slice
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u tools/prof_scan.py > gpurun_out/prof_scan.json 2> gpurun_out/prof_scan.err || { tail -5 gpurun_out/prof_scan.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/kt_c5s -o run -- python3 $R/tools/run_decode.py c5_256m 12 > $R/gpurun_out/kt_c5s.log 2>&1 || exit 1
echo done
