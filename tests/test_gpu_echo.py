"""GPU: BASELINE config 1 -- the loopback WebSocket echo with 4 KiB masked
binary frames, the server's receive path on the GPU (tools/ws_echo.cpp,
fws_rx_session_feed per read). The client checks every echoed payload byte
for byte against what it sent (the reference's harness hashes every 16 384th
message, tests/new-ws-echo/test_ws_client.cpp:260-277), so a green run is
end-to-end parity of the unmask over real socket reads."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ECHO = os.path.join(ROOT, "tools", "bin", "ws_echo")


@pytest.mark.parametrize("clients,window,msg_len", [(1, 1, 4096), (4, 8, 4096), (2, 4, 100), (2, 2, 70000)])
def test_echo_loopback_gpu_engine(cuda, clients, window, msg_len):
    assert os.path.exists(ECHO), "build first: make -C flashws_amd/csrc"
    r = subprocess.run([ECHO, "--engine", "gpu", "--clients", str(clients), "--window", str(window),
                        "--msg-len", str(msg_len), "--msgs", "1500", "--warmup", "50"],
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, (r.stdout, r.stderr[-2000:])
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["verified"] is True and rec["server_ret"] == 0
    assert rec["msgs_per_client"] == 1500
