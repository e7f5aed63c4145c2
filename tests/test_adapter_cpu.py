"""CPU: the header-only C++ adapter (include/flashws_amd/gpu_ws.hpp) compiles
and links against the REAL flashws headers and libfws_gpu.so -- the drop-in
check for the reference's IOBuffer / on_read() types. Build container only
(needs /root/reference); the binary is not run (no GPU here)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/include"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference headers only exist in the build container")
def test_adapter_compiles_against_reference(tmp_path):
    out = tmp_path / "adapter_dropin"
    cmd = ["g++", "-std=c++17", "-O1", "-mavx2", "-w", f"-I{REF}", f"-I{ROOT}/include",
           os.path.join(ROOT, "tests", "cpp", "adapter_dropin.cpp"), "-o", str(out),
           f"-L{ROOT}/flashws_amd/lib", "-lfws_gpu", f"-Wl,-rpath,{ROOT}/flashws_amd/lib", "-lssl", "-lcrypto"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    assert out.exists()
