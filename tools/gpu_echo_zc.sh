# mux parity tests (both transfer modes), then the loopback echo with the mux
# copying every batch (FWS_MUX_ZC_MAX=0) vs small batches on the pinned
# staging (default), beside the reference engine
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_mux.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/mux_tests.log 2>&1 || { tail -30 gpurun_out/mux_tests.log; exit 1; }
tail -1 gpurun_out/mux_tests.log
: > gpurun_out/echo_zc.jsonl
run() {  # tag engine clients window msgs msg_len
  local tag=$1; shift
  echo -n "{\"mode\": \"$tag\"} " >> gpurun_out/echo_zc.jsonl
  timeout -k 10 120 tools/bin/ws_echo --engine $1 --ref-lib oracle/_ref/libfwsref.so --clients $2 --window $3 --msgs $4 --msg-len $5 >> gpurun_out/echo_zc.jsonl 2>> gpurun_out/echo.err || { echo "echo $*: failed"; tail -5 gpurun_out/echo.err; exit 1; }
}
for cfg in "1 1 10000 4096" "8 1 4000 4096" "8 16 3000 4096" "64 1 1000 4096" "64 16 400 4096" "8 4 300 65536"; do
  set -- $cfg
  FWS_MUX_ZC_MAX=0 run copy gpu-mux $1 $2 $3 $4 || exit 1
  run zc gpu-mux $1 $2 $3 $4 || exit 1
  run ref ref $1 $2 $3 $4 || exit 1
done
echo done
