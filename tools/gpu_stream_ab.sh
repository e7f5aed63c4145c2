set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python tools/tune_stream.py 40 > gpurun_out/tune_stream.json 2>gpurun_out/tune_stream.err || { tail gpurun_out/tune_stream.err; exit 1; }
cat gpurun_out/tune_stream.json
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_dec_v$v -o run -- python3 $R/tools/run_decode.py c3 12 $v > $R/gpurun_out/prof_dec_v$v.log 2>&1 || { tail -5 $R/gpurun_out/prof_dec_v$v.log; exit 1; }
done
echo done
