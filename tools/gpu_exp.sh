set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python tools/prof_merge_trace.py > gpurun_out/merge_trace.json 2> gpurun_out/merge_trace.err || { tail -5 gpurun_out/merge_trace.err; exit 1; }
timeout -k 10 200 python - > gpurun_out/emit_cnt.txt 2>&1 <<'PY'
import torch
from flashws_amd import gpu
for name, mk in (("C2", gpu.config_c2), ("C3", gpu.config_c3)):
    w, d, _ = mk()
    c = gpu.Ctx(0, max_frames=len(d) + 16, max_stream_bytes=len(w))
    x = torch.from_numpy(w).cuda()
    gpu.decode_stream(c, x, cap=len(d) + 16)
    torch.cuda.synchronize()
    import ctypes as C
    from flashws_amd import _lib
    out = (C.c_uint32 * 16)()
    _lib.lib().fws_internal_decode_counters(c.h, out, 16)
    print(name, list(out))
PY
echo done
