# mux / session parity tests, then the loopback echo (BASELINE C1 shape) on the
# GPU engines (per-read session, per-round mux) and the reference engine,
# 1 / 8 / 64 clients, and a message-size sweep for the crossover
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_mux.py tests/test_gpu_session.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/mux_tests.log 2>&1 || { tail -30 gpurun_out/mux_tests.log; exit 1; }
tail -1 gpurun_out/mux_tests.log
: > gpurun_out/echo.jsonl
run() {  # engine clients window msgs msg_len
  timeout -k 10 120 tools/bin/ws_echo --engine $1 --ref-lib oracle/_ref/libfwsref.so --clients $2 --window $3 --msgs $4 --msg-len $5 >> gpurun_out/echo.jsonl 2>> gpurun_out/echo.err || { echo "echo $*: failed"; tail -5 gpurun_out/echo.err; exit 1; }
}
for cfg in "1 1 10000" "8 1 4000" "8 16 3000" "64 1 1000" "64 16 400"; do
  set -- $cfg
  for eng in gpu-mux gpu ref; do run $eng $1 $2 $3 4096 || exit 1; done
done
for len in 65536 1048576; do
  for eng in gpu-mux gpu ref; do run $eng 8 4 300 $len || exit 1; done
done
echo done
