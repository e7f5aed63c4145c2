# C5 descriptor fused unmask+UTF-8 through each variant library, then a kernel
# trace of the same runs
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
: > gpurun_out/utf8_exp.jsonl
for tv in "$@"; do   # tag:variant
  t=${tv%%:*}; v=${tv#*:}; [ "$v" = "$tv" ] && v=0
  timeout -k 10 150 python tools/utf8_exp.py flashws_amd/lib/libfws_gpu_$t.so $v >> gpurun_out/utf8_exp.jsonl 2> gpurun_out/utf8_exp.err || { tail -5 gpurun_out/utf8_exp.err; exit 1; }
done
cat gpurun_out/utf8_exp.jsonl
echo done
