# GPU pass: the drop-in tests, then C1 numbers -- the reference-API echo server
# (oracle/_ref/ws_dropin) with and without the GPU hook under the reference's
# WSClientSocket load, 4 KiB messages, 1 / 8 / 64 connections.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_limits.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dropin_tests.log 2>&1 || { tail -40 gpurun_out/dropin_tests.log; exit 1; }
tail -3 gpurun_out/dropin_tests.log
B=$R/oracle/_ref/ws_dropin
: > gpurun_out/dropin_c1.jsonl
for eng in cpu gpu; do
  for n in 1 8 64; do
    G=""; [ $eng = gpu ] && G="--gpu"
    $B server --conns $n --max-seconds 100 $G > gpurun_out/srv.out 2>gpurun_out/srv.err &
    SP=$!
    for i in $(seq 50); do grep -q listening gpurun_out/srv.out 2>/dev/null && break; sleep 0.1; done
    PORT=$(awk '/listening/{print $2}' gpurun_out/srv.out)
    timeout -k 5 100 $B client --port $PORT --clients $n --msg-len 4096 --msgs 20000 --warmup 500 --max-seconds 90 > gpurun_out/cli.out || { cat gpurun_out/srv.err; exit 1; }
    wait $SP || exit 1
    python3 -c "import json,sys; c=json.loads(open('gpurun_out/cli.out').read().splitlines()[-1]); s=json.loads(open('gpurun_out/srv.out').read().splitlines()[-1]); c['server']=s; c['engine']='$eng'; print(json.dumps(c))" >> gpurun_out/dropin_c1.jsonl
  done
done
cat gpurun_out/dropin_c1.jsonl | cut -c1-300
