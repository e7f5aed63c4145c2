set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/tr
for w in tx c4 c3 dense; do
  case $w in
    tx) cmd="python3 $R/tools/run_tx.py";;
    c4) cmd="python3 $R/tools/run_c4.py";;
    c3) cmd="python3 $R/tools/run_decode.py c3 20";;
    dense) cmd="python3 $R/tools/run_decode.py dense 20";;
  esac
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr/$w -o run -- $cmd > $R/gpurun_out/tr/$w.log 2>&1
done
