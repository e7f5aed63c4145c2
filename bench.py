#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric on MI355X:
"GiB/s masked WS payload unmasked, device-resident frame batch; % HBM roofline".

Workload (BASELINE configs[1]): 65 536 client-masked BIN frames
x 4 096 B payload (8-B headers, one random key each, seed 42), packed
contiguously, resident in HBM before timing starts. One step = one
fws_gpu_unmask_batch over one batch (plan kernels + the unmask kernel). Steps
rotate over NBUF >= 4 distinct device copies (>= 1 GiB) so the 256 MiB
Infinity Cache cannot serve a batch from the previous step.

Multi-GPU (torchrun): every rank unmasks its own batch (independent frames,
weak scaling, no collective on the data path); the timed region is bracketed
by barrier + synchronize and the slowest rank's time is reported.

Output: ONE JSON line on rank 0 (contract in the task statement), with
`roofline` for the dominant kernel (k_unmask, timed live with HIP events on
its stream) and `cpu_baseline` (the compiled reference's
WSocket::OnRecvData on this host, rank 0, N=1 only).
"""
import argparse
import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist

from flashws_amd import gpu

ROOT = os.path.dirname(os.path.abspath(__file__))
METRIC = "GiB/s masked WS payload unmasked, device-resident frame batch; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--frames", type=int, default=65536)
    ap.add_argument("--payload", type=int, default=4096)
    ap.add_argument("--nbuf", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--extra", action="store_true", help="also time the fused stream decode")
    return ap.parse_args()


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(world, x):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(wire, seconds):
    """The reference's own OnRecvData (oracle/_ref, compiled from the flashws
    headers in the build container) on this host: 1 thread, the C2 batch fed as
    2 MiB reads (MAX_READABLE_SIZE_ONE_TIME, constants.h:49-53). Falls back to
    the C restatement (oracle/liborc.so, kind "port") if the reference build is
    absent. Bounded to about `seconds` of CPU work."""
    import ctypes as C
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc
    read = 2 << 20
    if orc.ref_available():
        lib = orc.ref()
        pb, rc = C.c_uint64(0), C.c_int(0)
        t1 = lib.ref_time_onrecv(wire.ctypes.data, len(wire), read, 1, C.byref(pb), C.byref(rc))
        iters = max(2, int(seconds / max(t1, 1e-6)) // 2 * 2)    # even: XOR restores the input
        t = lib.ref_time_onrecv(wire.ctypes.data, len(wire), read, iters, C.byref(pb), C.byref(rc))
        kind = "reference"
        payload = pb.value
    else:
        st_bytes = bytearray(512)
        buf = wire.copy()
        t0 = time.perf_counter()
        iters, payload = 0, 0
        while time.perf_counter() - t0 < seconds:
            s = orc.OrcSession()
            for off in range(0, len(buf), read):
                part = buf[off:off + read]
                ret, _, ev, _ = s.feed(part, ev_cap=1 << 12, ctl_cap=16)
                payload += int(ev[ev["kind"] == 0]["size"].sum())
            iters += 1
        t = time.perf_counter() - t0
        kind = "port"
        del st_bytes
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(payload / t / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": kind,
            "sample": f"{iters} passes of the C2 batch ({len(wire)} wire B) through "
                      f"WSocket::OnRecvData as 2 MiB reads, {t:.1f} s, g++ -O3 -mavx2, {model}"}


def pmc_traffic():
    """HBM bytes per k_unmask launch from the committed rocprofv3 PMC summary
    (profiles/pmc_unmask.json, made by tools/pmc_summary.py), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_unmask.json")
    try:
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    world, rank, local = setup_dist(args)
    dev = torch.device("cuda", torch.cuda.current_device())

    wire, descs, _ = gpu.config_c2(seed=42 + rank, n_frames=args.frames, payload=args.payload)
    n = len(descs)
    payload_bytes = int(descs["payload_len"].sum())
    wire_bytes = len(wire)
    # algorithmic bytes per launch: read every wire byte + write every payload byte
    alg_bytes = wire_bytes + payload_bytes

    ctx = gpu.Ctx(local, max_frames=n, max_stream_bytes=wire_bytes)
    host = torch.from_numpy(wire)
    bufs = [host.to(dev) for _ in range(args.nbuf)]
    dd = gpu.descs_to_device(descs, dev)
    stream = torch.cuda.current_stream()

    for i in range(args.warmup):
        gpu.unmask_batch(ctx, bufs[i % args.nbuf], dd, n)
    torch.cuda.synchronize()

    # ---- timed region: K whole steps
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        gpu.unmask_batch(ctx, bufs[i % args.nbuf], dd, n)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    step_s = max_over_ranks(world, (t1 - t0) / args.steps)

    # ---- dominant kernel alone (k_unmask), HIP events on its stream
    gpu.unmask_plan(ctx, bufs[0], dd, n)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev0.record(stream)
    for i in range(args.steps):
        gpu.unmask_run(ctx, bufs[i % args.nbuf], dd, n)
    ev1.record(stream)
    torch.cuda.synchronize()
    kern_s = ev0.elapsed_time(ev1) / 1e3 / args.steps
    # restore input parity (even number of passes per buffer is not required for timing)

    extra = {}
    if args.extra:
        extra = stream_decode_extra(ctx, wire, dev, args)

    value = world * payload_bytes / step_s / GIB
    achieved = alg_bytes / kern_s / 1e9
    traffic = pmc_traffic()
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (fws_gen_batch, mt19937_64 seed 42+rank): client-masked BIN frames",
        "config": {"workload": "C2: device-resident 65536 x 4 KiB masked BIN frames, "
                               "descriptor-mode unmask (fws_gpu_unmask_batch)",
                   "frames_per_gpu": n, "payload_bytes_per_frame": args.payload,
                   "wire_bytes_per_gpu": wire_bytes, "rotating_buffers": args.nbuf,
                   "parallelism": f"batch split x{world} (no collective)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "kernel": "k_unmask<false>", "kernel_us": round(kern_s * 1e6, 2),
                     "alg_bytes_per_launch": alg_bytes},
    }
    out.update(extra)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(wire, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def stream_decode_extra(ctx, wire, dev, args):
    return {}


if __name__ == "__main__":
    main()
