# loopback echo (C1 shape and windowed) on the GPU engine and the reference
# engine, plus the session parity tests the echo's receive path runs through
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_session.py tests/test_gpu_pipe.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/echo_session_tests.log 2>&1 || { tail -30 gpurun_out/echo_session_tests.log; exit 1; }
tail -1 gpurun_out/echo_session_tests.log
: > gpurun_out/echo.jsonl
for cfg in "1 1 20000" "8 1 5000" "8 16 5000" "8 64 4000"; do
  set -- $cfg
  for eng in gpu ref; do
    timeout -k 10 120 tools/bin/ws_echo --engine $eng --ref-lib oracle/_ref/libfwsref.so --clients $1 --window $2 --msgs $3 >> gpurun_out/echo.jsonl 2>> gpurun_out/echo.err || { echo "echo $eng $cfg failed"; cat gpurun_out/echo.err; exit 1; }
  done
done
cat gpurun_out/echo.jsonl
