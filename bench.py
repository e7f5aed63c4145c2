#!/usr/bin/env python3
"""bench.py -- BASELINE.json's metric on MI355X:
"GiB/s masked WS payload unmasked, device-resident frame batch; % HBM roofline".

Workload (BASELINE configs[1]): 65 536 client-masked BIN frames
x 4 096 B payload (8-B headers, one random key each, seed 42), packed
contiguously, resident in HBM before timing starts. One step = one
fws_gpu_unmask_sorted over one batch (a packed batch is sorted by
construction; one launch, k_unmask_sorted, which finds each 4 KiB unit's
frames itself). The any-order path fws_gpu_unmask_batch (k_plan +
k_unmask_desc) is timed beside it in extra.C2_unmask_batch_any_order. Steps
rotate over NBUF >= 4 distinct device copies (>= 1 GiB) so the 256 MiB
Infinity Cache cannot serve a batch from the previous step.

Multi-GPU: `bench.py --gpus N` (N > 1) started without torchrun's environment
starts `python -m torch.distributed.run --nproc-per-node N bench.py ...` as a
child process before anything touches a GPU and exits with its code; under
torchrun (the driver's launch) one rank per GPU. Every rank unmasks its own
batch (independent frames, weak scaling, no collective on the data path); the
timed region is bracketed by barrier + synchronize and the slowest rank's time
is reported. At N > 1 the 8-GPU BASELINE config (C5: 4 GiB of 16 KiB TEXT
frames per GPU, unmask + UTF-8 flags) is timed the same way -> extra.

Output: ONE JSON line on rank 0 (contract in the task statement), with
`roofline` for the dominant kernel (k_unmask_sorted, timed live with HIP events on
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
DENSE_FRAMES, DENSE_PAYLOAD = 200000, 64   # SURVEY §6 dense small-frame workload
# untimed calls before an extra config's timed ones: the 4 GiB C5 descriptor pass
# measured 1.76 ms over its first 10 calls after one warm-up call and 1.58 ms over
# the next 10 (tools/c5_warmup_probe.py, profiles/r03/c5_warmup.txt)
EXTRA_WARMUP = 10
ENGINE_JOBS = 16               # batches per fws_decode_engine run (distinct buffers)
SRC_COPIES = 4                 # C4 / TX: rotating sources (>= 1 GiB with the outputs, past the 256 MB MALL)
EXTRA_WARM_S = 0.05            # and at least this long (s) of untimed calls before each extra config
HEAD_WARM_S = 0.25             # the headline's warmup: at least W calls and this long (s) of them
EXTRA_CONFIGS = ("c2s", "c3", "dense", "c4", "tx", "c5s", "c5d", "e2e", "c1", "batch")
C5_STREAM_STEPS = 16           # timed C5 stream calls, each on its own freshly masked 4 GiB buffer
# rocprofv3 kernel stats of each extra config, captured warm (bench.py --only <cfg> under
# rocprofv3 --kernel-trace --stats; tools/gpu_round.sh prof_extras)
PROFILE_DIR = "profiles/r06"


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
    ap.add_argument("--no-batch-extra", action="store_true",
                    help="skip the fws_gpu_unmask_batch (plan + run) comparison line")
    ap.add_argument("--extra", action="store_true",
                    help="also time C2 stream decode, C3, C4, TX, e2e (PCIe) -> 'extra' "
                         "(default at N=1; multi-GPU runs time the headline only)")
    ap.add_argument("--c5", action="store_true", help="with --extra: the 4 GiB C5 UTF-8 config (default at N=1)")
    ap.add_argument("--no-extra", action="store_true", help="headline line only")
    ap.add_argument("--no-c5-split", action="store_true", help="N > 1: skip the C5 batch-split config")
    ap.add_argument("--share-device", action="store_true",
                    help="N > 1 validation on one GPU: every rank on device 0, gloo process group "
                         "(exercises the N-rank path on real HIP; not a scaling measurement)")
    ap.add_argument("--only", default="",
                    help="comma list of extra configs to run (c2s,c3,dense,c4,tx,c5s,c5d,e2e,c1,batch): one "
                         "config per process, e.g. under rocprofv3 (profiles/r05/*_kernel_stats.csv)")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="skip the two-in-flight and engine runs of the stream configs (profiling: a config's "
                         "timed calls are then the last dispatches of its kernels, tools/prof_window.py)")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="CPU only (gloo): exercise the N-rank launch, barrier and max-over-ranks timing on a "
                         "host XOR of each rank's shard; prints a self-test line, not the metric")
    a = ap.parse_args()
    if int(os.environ.get("WORLD_SIZE", "1")) == 1 and not a.no_extra:
        a.extra = a.c5 = True
    if a.no_extra:
        a.extra = a.c5 = False
    a.only = {x.strip() for x in a.only.split(",") if x.strip()}
    bad = a.only - set(EXTRA_CONFIGS)
    if bad:
        ap.error(f"--only: unknown config(s) {sorted(bad)}; known: {EXTRA_CONFIGS}")
    if a.only:
        a.extra = True
        a.c5 = bool(a.only & {"c5s", "c5d"})
    return a


def want(args, name):
    """extra config `name` runs: every config by default, only the listed ones with --only"""
    return not args.only or name in args.only


def launch_ranks(args):
    """`--gpus N` without torchrun's environment: start N ranks through
    torch.distributed.run as a child process (nothing here has touched a GPU;
    torch.cuda.device_count() does not initialise one) and return its exit code."""
    import socket
    import subprocess
    import sys
    have = kfd_gpu_count()
    if not args.launcher_selftest and not args.share_device and have is not None and have < args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus}: only {have} GPU(s) visible")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["FWS_BENCH_KFD_GPUS"] = "none" if have is None else str(have)
    return subprocess.call(cmd, env=env)


def kfd_gpu_count(topology="/sys/class/kfd/kfd/topology/nodes", env=None):
    """GPUs this process could use, counted without initialising HIP (the
    launcher forks torch.distributed.run afterwards; torch.cuda.device_count()
    may fall back to hipGetDeviceCount): KFD topology nodes with a non-zero
    gfx_target_version, narrowed by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES when set. None when the topology is not readable."""
    env = os.environ if env is None else env
    try:
        nodes = sorted(os.listdir(topology), key=lambda x: int(x) if x.isdigit() else 1 << 30)
    except OSError:
        return None
    n = 0
    for d in nodes:
        try:
            with open(os.path.join(topology, d, "properties")) as f:
                for line in f:
                    k, _, v = line.partition(" ")
                    if k == "gfx_target_version" and int(v.strip() or 0) != 0:
                        n += 1
                        break
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def dist_env():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def setup_dist(world, local, share_device=False):
    """One process per GPU. The data path has no exchange step:
    the process group only carries the barriers, the max-over-ranks reduction
    of the step time and the flag check, all outside the timed region and all
    on CPU tensors, so it is a gloo group and no device collective (RCCL) is
    initialised at all. share_device (validation on a one-GPU box): every rank
    on device 0, so the N-rank path (shard seeds, C5 split, max over ranks) runs
    on real HIP; its times are contended and not a scaling claim."""
    torch.cuda.set_device(0 if (share_device or world == 1) else local)
    init_group(world)


def init_group(world):
    """the N > 1 control group: gloo (CPU tensors only; tests/test_dist_cpu.py)"""
    if world > 1:
        dist.init_process_group(backend="gloo")
        return dist.get_backend()
    return None


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(world, x):
    """Slowest rank's value (the timed region ends when every rank is done)."""
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64)          # CPU tensor on the gloo group
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_seed(rank):
    """Each rank decodes its own independent batch: frames shard trivially
    (SURVEY §8e), so there is no collective on the data path."""
    return 42 + rank


def aggregate_gib_s(world, payload_bytes_per_rank, step_s):
    """Whole-job throughput: all ranks' payload / the slowest rank's step."""
    return world * payload_bytes_per_rank / step_s / GIB


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _physical_cores():
    """Distinct (package, core) pairs in /proc/cpuinfo, or the logical count."""
    seen, cur = set(), {}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if ":" in line:
                    k, v = (x.strip() for x in line.split(":", 1))
                    cur[k] = v
                elif cur:
                    seen.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
        if cur:
            seen.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    return len(seen) if len(seen) > 1 else (os.cpu_count() or 1)


def cpu_share():
    """Cores the all-core leg may use: this process's affinity set, capped by
    OMP_NUM_THREADS (the GPU box's per-GPU CPU share) and the physical cores."""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, min(n, _physical_cores()))


def cpu_baseline(wire, descs, seconds):
    """The reference's own OnRecvData (oracle/_ref, compiled from the flashws
    headers in the build container) on this host, on the C2 batch fed as 2 MiB
    reads (MAX_READABLE_SIZE_ONE_TIME, constants.h:49-53), bounded to about
    `seconds` of CPU work per leg: (1) one core, (2) all cores of this process's
    CPU share, one process per core, each decoding its own copy of the batch
    (the reference scales as one event loop per core; its buffer singletons are
    not thread-safe). The all-core figure is `value`. Must run before this process
    touches a GPU (the all-core leg forks). Falls back to the C restatement
    (oracle/liborc.so, kind "port", one core) if the reference build is absent."""
    import ctypes as C
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import orc
    read = 2 << 20
    model = _cpu_model()
    if not orc.ref_available():
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
        return {"value": round(payload / t / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                "sample": f"{iters} passes of the C2 batch through the C restatement of OnRecvData, {t:.1f} s, "
                          f"{model}"}
    lib = orc.ref()
    lib.ref_time_onrecv_procs.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_size_t, C.c_int,
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_int)]
    lib.ref_time_onrecv_procs.restype = C.c_double
    pb, rc = C.c_uint64(0), C.c_int(0)
    t1 = lib.ref_time_onrecv(wire.ctypes.data, len(wire), read, 1, C.byref(pb), C.byref(rc))
    iters = max(2, int(seconds / max(t1, 1e-6)) // 2 * 2)    # even: XOR restores the input
    t = lib.ref_time_onrecv(wire.ctypes.data, len(wire), read, iters, C.byref(pb), C.byref(rc))
    one = {"value": round(pb.value / t / GIB, 3), "cores": 1,
           "sample": f"{iters} passes of the C2 batch ({len(wire)} wire B), {t:.1f} s"}
    # all cores: every process decodes its own copy of the whole C2 batch (one
    # event loop per core, each with its own stream), so each streams 269 MB
    # per pass from DRAM, as a core does on fresh socket data, instead of a
    # cache-resident slice
    procs = cpu_share()
    begin = np.zeros(procs, dtype=np.uint64)
    end = np.full(procs, len(wire), dtype=np.uint64)
    it_all = max(2, int(seconds / max(t1, 1e-6)) // 3)
    pb2, rc2 = C.c_uint64(0), C.c_int(0)
    ta = lib.ref_time_onrecv_procs(wire.ctypes.data, begin.ctypes.data, end.ctypes.data, procs, read, it_all,
                                   C.byref(pb2), C.byref(rc2))
    if ta <= 0 or rc2.value != 0 or rc.value != 0:
        raise RuntimeError(f"reference CPU baseline failed: t={ta} rc={rc.value},{rc2.value}")
    # SURVEY §6's dense workload (200 000 x 64 B BIN frames), one core, beside the GPU's
    # dense_64B_stream_decode extra
    wd, dd, _ = gpu.config_c2(n_frames=DENSE_FRAMES, payload=DENSE_PAYLOAD)
    pbd, rcd = C.c_uint64(0), C.c_int(0)
    td1 = lib.ref_time_onrecv(wd.ctypes.data, len(wd), read, 1, C.byref(pbd), C.byref(rcd))
    it_d = max(2, int(min(seconds, 3.0) / max(td1, 1e-6)) // 2 * 2)
    td = lib.ref_time_onrecv(wd.ctypes.data, len(wd), read, it_d, C.byref(pbd), C.byref(rcd))
    dense = {"value": round(pbd.value / td / GIB, 3), "unit": "GiB/s", "cores": 1,
             "sample": f"{it_d} passes of {DENSE_FRAMES} x {DENSE_PAYLOAD} B BIN frames ({len(wd)} wire B) "
                       f"as 2 MiB reads, {td:.2f} s"}
    if rcd.value != 0:
        raise RuntimeError(f"reference CPU baseline (dense) failed: rc={rcd.value}")
    return {"value": round(pb2.value / ta / GIB, 3), "unit": "GiB/s", "cores": procs, "kind": "reference",
            "sample": f"{procs} processes (one per core, the reference's one-event-loop-per-core model), each "
                      f"running WSocket::OnRecvData over its own copy of the C2 batch ({len(wire)} wire B) as "
                      f"2 MiB reads {it_all} times ({ta:.1f} s, slowest process); g++ -O3 -mavx2; {model}; "
                      f"host has {os.cpu_count()} logical CPUs, {_physical_cores()} physical cores, this "
                      f"process's CPU share {procs}",
            "one_core": one, "dense_64B_one_core": dense}


def source_sha16(rel="flashws_amd/csrc/unmask_kernels.hip"):
    """sha256 (16 hex) of the headline kernel's source file."""
    import hashlib
    try:
        with open(os.path.join(ROOT, rel), "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def pmc_traffic():
    """HBM bytes per k_unmask_sorted launch from the committed rocprofv3 PMC
    summary (profiles/pmc_unmask.json, made by tools/pmc_summary.py) and where
    it came from. The bytes count only if the summary was measured on the
    kernel source this tree builds (its recorded sha of unmask_kernels.hip);
    a stale summary gives traffic None."""
    p = os.path.join(ROOT, "profiles", "pmc_unmask.json")
    try:
        with open(p) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None, {"file": "profiles/pmc_unmask.json", "status": "absent"}
    src = {"file": "profiles/pmc_unmask.json", "commit": rec.get("commit"),
           "kernel_source_sha16": rec.get("kernel_source_sha16"), "measured": rec.get("measured")}
    current = rec.get("kernel") == "k_unmask_sorted" and rec.get("kernel_source_sha16") == source_sha16()
    src["status"] = "current" if current else "stale (kernel source changed since the PMC passes)"
    return (rec.get("hbm_bytes_per_launch") if current else None), src


def launcher_selftest(args, world, rank):
    """CPU (gloo) rehearsal of the N-rank path: the same launch, shard seeds,
    barriers, max-over-ranks and aggregate as the GPU run, with a host XOR of
    each rank's C2 shard standing in for the device step. Prints a self-test
    line (no metric claim)."""
    if world > 1:
        dist.init_process_group(backend="gloo")
    wire, descs, _ = gpu.config_c2(seed=shard_seed(rank), n_frames=args.frames, payload=args.payload)
    payload = int(descs["payload_len"].sum())
    buf = wire.copy()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        np.bitwise_xor(buf, 0x5A, out=buf)
    t1 = time.perf_counter()
    barrier(world)
    own = (t1 - t0) / args.steps
    step = max_over_ranks(world, own)
    dig = torch.tensor([int(np.frombuffer(wire[:4096].tobytes(), dtype=np.uint64).sum() & 0x7FFFFFFFFFFF)],
                       dtype=torch.int64)
    digs = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_gather(digs, dig)
    else:
        digs = [dig]
    line = {"selftest": True, "n_gpus": world, "rank": rank, "steps": args.steps, "step_s": step,
            "own_step_s": own, "value": aggregate_gib_s(world, payload, step), "payload_bytes_per_rank": payload,
            "shard_digests": [int(d.item()) for d in digs],
            "launcher_kfd_gpus": os.environ.get("FWS_BENCH_KFD_GPUS")}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    world, rank, local = dist_env()
    if args.gpus > 1 and world == 1:
        raise SystemExit(launch_ranks(args))
    if args.launcher_selftest:
        return launcher_selftest(args, world, rank)

    wire, descs, _ = gpu.config_c2(seed=shard_seed(rank), n_frames=args.frames, payload=args.payload)
    # the host-core reference baseline runs first: its all-core leg forks, which
    # must happen before this process initialises a GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(wire, descs, args.cpu_seconds)

    setup_dist(world, local, args.share_device)
    local = torch.cuda.current_device()
    dev = torch.device("cuda", local)
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

    # a packed batch is sorted by construction: the one-launch fws_gpu_unmask_sorted.
    # Warmup: at least W untimed steps and at least HEAD_WARM_S seconds of them (the
    # host-side CPU baseline and setup before it leave the GPU idle for tens of
    # seconds; the first ~100 launches after that run 1-5 % slower while the clocks
    # ramp up, profiles/r06/ab_*.jsonl first rounds)
    _warm(lambda i: gpu.unmask_sorted(ctx, bufs[i % args.nbuf], dd, n), args.warmup, HEAD_WARM_S)

    # ---- timed region: K whole steps. The dominant kernel (k_unmask_sorted, the
    # step's only launch) is timed by HIP events on its stream (the current
    # stream, where the ABI call launches it) around the same K launches, inside
    # the wall-clock bracket: the per-launch kernel time cannot exceed the step.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        gpu.unmask_sorted(ctx, bufs[i % args.nbuf], dd, n)
    ev1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    own_s = (t1 - t0) / args.steps
    step_s = max_over_ranks(world, own_s)
    kern_s = min(ev0.elapsed_time(ev1) / 1e3 / args.steps, own_s)

    extra = {}
    if not args.no_batch_extra and world == 1 and want(args, "batch"):
        extra["C2_unmask_batch_any_order"] = batch_extra(ctx, bufs, dd, n, payload_bytes, args, stream)
    if args.extra:
        extra.update(stream_decode_extra(ctx, wire, dev, args)["extra"])
        if want(args, "c1"):
            extra["C1_echo"] = c1_echo_extra(local)
    del bufs
    if world > 1 and not args.no_c5_split:
        extra["C5_batch_split"] = c5_split(args, world, rank, local, dev)
    extra = {"extra": extra} if extra else {}

    value = aggregate_gib_s(world, payload_bytes, step_s)
    achieved = alg_bytes / kern_s / 1e9
    traffic, traffic_src = pmc_traffic()
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
                               "descriptor-mode unmask of the packed (sorted) batch, "
                               "one launch (fws_gpu_unmask_sorted)",
                   "frames_per_gpu": n, "payload_bytes_per_frame": args.payload,
                   "wire_bytes_per_gpu": wire_bytes, "rotating_buffers": args.nbuf,
                   "parallelism": f"batch split x{world} (no collective)"},
        "warmup_policy": f"at least {args.warmup} untimed steps and at least {HEAD_WARM_S} s of them",
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "k_unmask_sorted", "kernel_us": round(kern_s * 1e6, 2),
                     "kernel_timing": "HIP events on the launch stream around the K timed steps",
                     "alg_bytes_per_launch": alg_bytes},
    }
    out.update(extra)
    if cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def c5_split(args, world, rank, local, dev):
    """BASELINE config 5 (the 8-GPU one): every rank unmasks + UTF-8-validates
    its own 4 GiB of 16 KiB TEXT frames (seed 42 + rank), descriptor mode
    (fws_gpu_unmask_sorted_utf8) and as a raw stream (fws_gpu_decode_stream with
    UTF-8 flags); barrier + synchronize around K steps, slowest rank's time,
    aggregate = all ranks' payload / that time. As in c5_extra, every timed call
    decodes its own freshly masked copy (K + 1 copies per rank: K timed, one for
    the untimed warm-up calls); the flags of the last timed call of each mode
    are checked against the generator on every rank."""
    w5, d5, ok5 = gpu.config_c5(seed=shard_seed(rank))
    n5 = len(d5)
    pl5 = int(d5["payload_len"].sum())
    expect = np.asarray(ok5, dtype=np.uint8)[:n5]
    c = gpu.Ctx(local, max_frames=n5 + 64, max_stream_bytes=len(w5))
    master = torch.from_numpy(w5).to(dev)
    del w5
    k = max(2, min(args.steps, 8))
    warm = master.clone()
    bufs = [master.clone() for _ in range(k)]
    dd5 = gpu.descs_to_device(d5, dev)
    ok = torch.empty(n5, dtype=torch.uint8, device=dev)

    def timed(fn):
        _warm(lambda i: fn(warm), warmup=EXTRA_WARMUP)
        torch.cuda.synchronize()
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b in bufs:
            fn(b)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        barrier(world)
        return max_over_ranks(world, (t1 - t0) / k), (t1 - t0) / k

    t_desc, own_desc = timed(lambda b: gpu.unmask_sorted_utf8(c, b, dd5, n5, ok))
    flags_ok = bool(np.array_equal(ok.cpu().numpy(), expect))
    for b in bufs:
        b.copy_(master)
    warm.copy_(master)
    cap = n5 + 64
    frames = torch.empty(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
    res = torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
    okd = torch.zeros(cap, dtype=torch.uint8, device=dev)

    def dec(b):
        rc, _, _, _ = gpu.decode_stream(c, b, cap, frames=frames, result=res, utf8_ok=okd)
        assert rc == 0, rc

    t_str, own_str = timed(dec)
    r = gpu.read_result(res)
    stream_ok = int(r["status"]) == 0 and int(r["n_frames"]) == n5 and bool(
        np.array_equal(okd[:n5].cpu().numpy(), expect))
    all_ok = max_over_ranks(world, 0.0 if (flags_ok and stream_ok) else 1.0) == 0.0
    c.close()
    del master, warm, bufs
    torch.cuda.empty_cache()
    return {"workload": "C5: per GPU 262144 x 16 KiB masked TEXT frames (4 GiB payload), unmask + per-frame "
                        "UTF-8 flags; ranks split the 8 x 4 GiB job, no collective on the data path",
            "descriptor_mode": {"GiB_per_s": round(world * pl5 / t_desc / GIB, 1),
                                "ms_per_step": round(t_desc * 1e3, 4),
                                "path": "fws_gpu_unmask_sorted_utf8"},
            "stream_decode": {"GiB_per_s": round(world * pl5 / t_str / GIB, 1),
                              "ms_per_step": round(t_str * 1e3, 4),
                              "path": "fws_gpu_decode_stream + UTF-8 flags"},
            "payload_bytes_per_gpu": pl5, "steps": k, "n_gpus": world,
            "timed_input": f"{k} freshly masked copies per rank, one per timed call",
            "flags_match_generator_all_ranks": all_ok}


def c1_echo_extra(device=0):
    """BASELINE config 1: loopback echo of 4 KiB masked BIN
    frames through the drop-in server -- the reference's own FLoop +
    WSServerSocket<false> (oracle/_ref/ws_dropin, tools/dropin/ws_dropin.cpp)
    with and without the one-line GpuRxHook -- for 1, 8 and 64 clients (window 1,
    every echoed byte checked; 20,000 / 12,000 / 3,000 messages per client, so a
    case runs ~0.5-1 s: the 64-client case at 500 messages, 0.1 s, measured the
    ramp-up -- first-touch registration of the pool's read buffers, the resident
    grid's first launch -- as much as the steady state, 17 against 21 Gbit/s,
    tools/echo_prof.py), goodput rx+tx and RTT p50/p99; and the
    reference's own unchanged echo client (tests/new-ws-echo/test_ws_client.cpp,
    oracle/_ref/ws_ref_client_1, 40,000 messages, its HashArr check every
    16,384th) against the hooked and the plain server. Host-memory path: every
    read crosses PCIe twice when hooked. `gpu_hook_batched`:
    GpuRxHook::EnableBatched, the reads of all connections of one loop step in
    one GPU round trip; since r06 a step's last chunk is
    dispatched in the next step when the loop has events waiting
    (SetDeferLastChunk, the default). `gpu_hook_batched_flush`: the same with
    SetDeferLastChunk(false) (env FWS_HOOK_DEFER=0), every step's chunks
    dispatched at its end (the r05 hook)."""
    import subprocess
    import tempfile
    dropin = os.path.join(ROOT, "oracle", "_ref", "ws_dropin")
    refcli = os.path.join(ROOT, "oracle", "_ref", "ws_ref_client_1")
    if not os.path.exists(dropin):
        return {"status": "absent: oracle/_ref/ws_dropin not built"}

    def server(mode, conns, port=0):
        args = [dropin, "server", "--port", str(port), "--conns", str(conns), "--max-seconds", "60"]
        if mode != "reference":
            args += ["--gpu-batch" if mode.startswith("gpu_hook_batched") else "--gpu", "--device", str(device)]
        env = dict(os.environ)
        if mode == "gpu_hook_batched_flush":
            env["FWS_HOOK_DEFER"] = "0"          # GpuRxHook::SetDeferLastChunk(false): every step flushed (r05)
        p = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env)
        line = p.stdout.readline()
        if not line.startswith("listening"):
            p.kill()
            raise RuntimeError(f"ws_dropin server did not start: {line!r} {p.stderr.read()[-500:]}")
        return p, int(line.split()[1])

    def finish(p):
        out, err = p.communicate(timeout=60)
        if p.returncode != 0:
            raise RuntimeError(f"ws_dropin server rc={p.returncode}: {err[-500:]}")
        return json.loads(out.strip().splitlines()[-1])

    out = {"workload": "C1: loopback echo, 4 KiB masked BIN frames, window 1, plain ws:// on 127.0.0.1",
           "server": "reference FLoop + WSServerSocket<false> (ws_dropin); hooked = + fws_amd::GpuRxHook::Enable"}
    for clients, msgs in ((1, 20000), (8, 12000), (64, 3000)):
        for mode in ("reference", "gpu_hook", "gpu_hook_batched", "gpu_hook_batched_flush"):
            if clients == 1 and mode.startswith("gpu_hook_batched"):
                continue                     # one read per loop step: the per-read path's round trip
            p, port = server(mode, clients)
            r = subprocess.run([dropin, "client", "--port", str(port), "--clients", str(clients), "--msgs", str(msgs),
                                "--warmup", "200", "--msg-len", "4096", "--max-seconds", "60"],
                               capture_output=True, text=True, timeout=120)
            st = finish(p)
            rec = json.loads(r.stdout.strip().splitlines()[-1]) if r.stdout.strip() else {}
            out[f"{clients}_client{'s' if clients > 1 else ''}_{mode}"] = {
                "goodput_rx_tx_mbps": rec.get("goodput_rx_tx_mbps"), "rtt_us": rec.get("rtt_us"),
                "msgs_per_s": rec.get("msgs_per_s"), "verified": bool(rec.get("verified")) and r.returncode == 0,
                "gpu_reads": st.get("gpu_reads"), "gpu_batches": st.get("gpu_batches"),
                "deferred_chunks": st.get("deferred_chunks")}
    if os.path.exists(refcli):
        for hooked in (False, True):
            p, port = server("gpu_hook" if hooked else "reference", 1, port=58600)   # the reference client's port
            with tempfile.TemporaryDirectory() as td:
                r = subprocess.run([refcli], capture_output=True, text=True, timeout=120, cwd=td)
            st = finish(p)
            lines = r.stdout.splitlines()
            dh = [x.split(":")[1].strip() for x in lines if x.startswith("data hash:")]
            hv = [x.rsplit("hash value:", 1)[1].split(",")[0].strip() for x in lines if "hash value:" in x]
            gp = [float(x.split(":")[1].split()[0]) for x in lines if x.startswith("avg (rx+tx) goodput")]
            lat = [x for x in lines if x.startswith("Latency (us)")]
            p50 = float(lat[0].split("P50:")[1].split(",")[0]) if lat else None
            p99 = float(lat[0].split("P99:")[1].split(",")[0]) if lat else None
            out[f"reference_client_1_{'gpu_hook' if hooked else 'reference'}"] = {
                "goodput_rx_tx_mbps": gp[0] if gp else None, "rtt_us": {"p50": p50, "p99": p99},
                "hash_checks_passed": len(hv) if (dh and hv and all(h == dh[0] for h in hv)) else 0,
                "rc": r.returncode, "msgs": st.get("msgs"), "gpu_reads": st.get("gpu_reads"),
                "client": "tests/new-ws-echo/test_ws_client.cpp unchanged (oracle/refclient/test_def.h: "
                          "127.0.0.1, 4 KiB, 40000 msgs)"}
    # both ends the reference's own code: tests/new-ws-echo/test_ws_server.cpp compiled
    # unchanged, plain (CPU OnRecvData) and with the GPU hook line supplied by our
    # test_def.h (oracle/Makefile refserver), against the unchanged client
    for hooked in (False, True):
        exe = os.path.join(ROOT, "oracle", "_ref", "ws_ref_server_gpu" if hooked else "ws_ref_server")
        if not (os.path.exists(exe) and os.path.exists(refcli)):
            continue
        with tempfile.TemporaryDirectory() as td:
            p = subprocess.Popen([exe], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, cwd=td)
            try:
                if hooked:                   # the hook line flushes once the socket listens
                    for ln in p.stdout:
                        if ln.startswith("gpu hook enabled"):
                            break
                else:
                    time.sleep(1.0)
                r = subprocess.run([refcli], capture_output=True, text=True, timeout=120, cwd=td)
            finally:
                p.terminate()
                sout, _ = p.communicate(timeout=30)
        lines = r.stdout.splitlines()
        dh = [x.split(":")[1].strip() for x in lines if x.startswith("data hash:")]
        hv = [x.rsplit("hash value:", 1)[1].split(",")[0].strip() for x in lines if "hash value:" in x]
        gp = [float(x.split(":")[1].split()[0]) for x in lines if x.startswith("avg (rx+tx) goodput")]
        lat = [x for x in lines if x.startswith("Latency (us)")]
        gr = [int(x.split()[1]) for x in sout.splitlines() if x.startswith("gpu_reads ")]
        out[f"reference_server_and_client_1_{'gpu_hook' if hooked else 'reference'}"] = {
            "goodput_rx_tx_mbps": gp[0] if gp else None,
            "rtt_us": {"p50": float(lat[0].split("P50:")[1].split(",")[0]) if lat else None,
                       "p99": float(lat[0].split("P99:")[1].split(",")[0]) if lat else None},
            "hash_checks_passed": len(hv) if (dh and hv and all(h == dh[0] for h in hv)) else 0,
            "rc": r.returncode, "gpu_reads": gr[0] if gr else None,
            "server": "tests/new-ws-echo/test_ws_server.cpp unchanged" + (" + GpuRxHook::Enable via test_def.h"
                                                                          if hooked else "")}
    return out


def check_c5_stream(rec):
    """Fail the bench when the C5 stream record's correctness fields disagree:
    the per-frame UTF-8 flags of the call on the masked batch must equal the
    generator's (count and frame by frame), and that call must decode every frame."""
    bad = []
    if rec.get("utf8_invalid_frames") != rec.get("utf8_invalid_frames_expected"):
        bad.append(f"utf8_invalid_frames {rec.get('utf8_invalid_frames')} != expected "
                   f"{rec.get('utf8_invalid_frames_expected')}")
    if rec.get("flags_match_generator") is not True:
        bad.append("per-frame UTF-8 flags differ from the generator's")
    if rec.get("checked_call_status") != 0 or rec.get("checked_call_frames") != rec.get("frames"):
        bad.append(f"checked call status {rec.get('checked_call_status')} frames {rec.get('checked_call_frames')}")
    if bad:
        raise RuntimeError("C5 stream decode record failed its checks: " + "; ".join(bad))
    return rec


def _profile(rec, cfg):
    """name the warm rocprofv3 kernel summary of this config in its roofline block"""
    path = f"{PROFILE_DIR}/{cfg}_kernel_stats.csv"
    rec.setdefault("roofline", {})["profile"] = path if os.path.exists(os.path.join(ROOT, path)) else None
    return rec


def _step_roofline(alg_bytes, t, basis):
    """roofline block of a whole extra step (every launch) against HBM peak"""
    a = alg_bytes / t / 1e9
    return {"bound": "hbm", "achieved": round(a, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(a / HBM_PEAK_GBS, 4), "basis": basis, "alg_bytes_per_step": int(alg_bytes)}


def _warm(fn, warmup=1, warm_s=EXTRA_WARM_S):
    """untimed calls in rounds of max(2, warmup) until both `warmup` calls and warm_s
    seconds have passed: a config whose timed region lasts a few ms otherwise runs
    on clocks still ramping up after the host-side setup before it (C4 measured
    0.088 ms over its first 110 calls, 0.085 after; tools/c4_thermal_probe.py)"""
    i = 0
    t0 = time.perf_counter()
    while True:
        for _ in range(max(2, warmup)):
            fn(i)
            i += 1
        torch.cuda.synchronize()
        if i >= warmup and time.perf_counter() - t0 >= warm_s:
            return


def _time(fn, steps, stream, warmup=1, warm_s=EXTRA_WARM_S):
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    _warm(fn, warmup, warm_s)
    ev0.record(stream)
    for i in range(steps):
        fn(i)
    ev1.record(stream)
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / 1e3 / steps


def batch_extra(ctx, bufs, dd, n, payload_bytes, args, stream):
    """fws_gpu_unmask_batch (k_plan + k_unmask_desc: any descriptor order) on
    the same C2 batches: the step, and the unmask kernel alone."""
    steps = max(20, args.steps // 2)
    t = _time(lambda i: gpu.unmask_batch(ctx, bufs[i % args.nbuf], dd, n), steps, stream, warmup=EXTRA_WARMUP)
    gpu.unmask_plan(ctx, bufs[0], dd, n)
    tk = _time(lambda i: gpu.unmask_run(ctx, bufs[i % args.nbuf], dd, n), steps, stream, warmup=EXTRA_WARMUP)
    # the same regions with the descriptor array permuted (planned in chunk space)
    perm = torch.from_numpy(np.random.default_rng(5).permutation(n)).to(dd.device)
    dp = dd.view(n, -1)[perm].reshape(-1).contiguous()
    tp = _time(lambda i: gpu.unmask_batch(ctx, bufs[i % args.nbuf], dp, n), steps, stream, warmup=EXTRA_WARMUP)
    return {"GiB_per_s": round(payload_bytes / t / GIB, 1), "ms_per_step": round(t * 1e3, 4),
            "k_unmask_desc_us": round(tk * 1e6, 2), "permuted_ms_per_step": round(tp * 1e3, 4),
            "path": "fws_gpu_unmask_batch: k_plan + k_unmask_desc (descriptors in any order; permuted_ms_per_step: "
                    "the same batch with its descriptor array shuffled)"}


def stream_decode_extra(ctx, wire_c2, dev, args):
    """The other BASELINE configs and the
    PCIe-inclusive end-to-end rate; reported as `extra`, not as `value`."""
    stream = torch.cuda.current_stream()
    steps = max(4, min(args.steps, 50)) // 2 * 2         # even: in-place XOR restores the input
    out = {}

    def decode_cfg(name, wire, n_frames, nbuf=None, pipelined=True):
        if nbuf is None:
            # rotate >= 1 GiB of distinct batches so the 256 MB Infinity Cache cannot
            # serve a step from the one before: 4 for C2 / C3, 77 of the
            # 14 MB dense batch
            nbuf = max(4, -(-(1 << 30) // len(wire)))
        c = gpu.Ctx(dev.index or 0, max_frames=n_frames + 64, max_stream_bytes=len(wire))
        bufs = [torch.from_numpy(wire).to(dev) for _ in range(nbuf)]
        cap = n_frames + 64
        frames = torch.empty(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
        res = torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
        def step(i):
            rc, _, _, _ = gpu.decode_stream(c, bufs[i % nbuf], cap, frames=frames, result=res)
            assert rc == 0, rc
        t = _time(step, steps, stream, warmup=EXTRA_WARMUP)
        r = gpu.read_result(res)
        assert int(r["status"]) == 0 and int(r["n_frames"]) == n_frames, (name, r)
        payload = int(gpu.read_frames(frames, n_frames)["payload_len"].sum())
        alg = (len(wire) + payload) / t / 1e9
        rec = {"GiB_per_s": round(payload / t / GIB, 1), "ms_per_step": round(t * 1e3, 4), "frames": n_frames,
               "wire_bytes": len(wire), "alg_GB_per_s": round(alg, 1), "rotating_buffers": nbuf,
               "big_super_tiles": gpu.decode_counters(c)["big_super_tiles"],
               # the whole decode step (scan .. stream unmask, every launch) against HBM peak:
               # algorithmic bytes = every wire byte read + every payload byte written
               "roofline": {"bound": "hbm", "achieved": round(alg, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(alg / HBM_PEAK_GBS, 4), "basis": "whole fws_gpu_decode_stream step",
                            "alg_bytes_per_step": len(wire) + payload}}
        if pipelined and nbuf >= 4 and not args.no_pipelined:
            # two batches in flight (two connections' reads): a context, a frame list and a
            # stream each, so one batch's latency-bound resolve overlaps the other's streaming
            c2 = gpu.Ctx(dev.index or 0, max_frames=n_frames + 64, max_stream_bytes=len(wire))
            ctxs = [c, c2]
            fr2 = [frames, torch.empty_like(frames)]
            rs2 = [res, torch.empty_like(res)]
            sts = [gpu.hip_stream(), gpu.hip_stream()]     # non-blocking HIP streams (the library's kind)
            def pstep(i):
                rc, _, _, _ = gpu.decode_stream(ctxs[i % 2], bufs[i % nbuf], cap, frames=fr2[i % 2],
                                                result=rs2[i % 2], stream=sts[i % 2])
                assert rc == 0, rc
            for i in range(4):
                pstep(i)
            torch.cuda.synchronize()
            reps = []
            for r in range(3):
                # median of 3 repetitions, each on a fresh stream pair: whether two streams'
                # kernels overlap depends on the hardware queues they land on, which HIP
                # does not expose (one created pair in 4-7 serialises: tools/queue_pair_probe.py)
                if r:
                    for st in sts:
                        st.close()
                    sts[:] = [gpu.hip_stream(), gpu.hip_stream()]
                    for i in range(2):
                        pstep(i)
                    torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(steps):
                    pstep(i)
                torch.cuda.synchronize()
                reps.append((time.perf_counter() - t0) / steps)
            tp = sorted(reps)[1]
            rec["two_in_flight"] = {"GiB_per_s": round(payload / tp / GIB, 1), "ms_per_batch": round(tp * 1e3, 4),
                                    "ms_per_batch_reps": [round(x * 1e3, 4) for x in reps],
                                    "roofline_frac": round((len(wire) + payload) / tp / 1e9 / HBM_PEAK_GBS, 4),
                                    "path": "2 contexts x 2 non-blocking HIP streams, batches alternate (median of 3 repetitions, a fresh stream pair each)"}
            for st in sts:
                st.close()
            c2.close()
            # the batched-stream engine (fws_decode_engine): ENGINE_JOBS distinct batches in one
            # run, the scan of one pipelined with the resolve + unmask of another
            ebufs = bufs + [torch.from_numpy(wire).to(dev) for _ in range(ENGINE_JOBS - nbuf)]
            efr = [torch.empty_like(frames) for _ in range(ENGINE_JOBS)]
            ers = [torch.zeros_like(res) for _ in range(ENGINE_JOBS)]
            eng = gpu.DecodeEngine(dev.index or 0, max_frames=cap, max_stream_bytes=len(wire))
            jobs = [(ebufs[j], cap, efr[j], ers[j]) for j in range(ENGINE_JOBS)]
            def estep(i):
                rc = eng.run(jobs, stream=stream)
                assert rc == 0, rc
            # the median of 5 timed runs after 3 untimed ones (the first runs of a fresh
            # engine come out ~5 % slower, profiles/r04/engine/sweep_schedules.jsonl)
            for i in range(3):
                estep(i)
            te = sorted(_time(estep, 1, stream, warmup=0) for _ in range(5))[2] / ENGINE_JOBS
            for j in range(ENGINE_JOBS):
                rj = gpu.read_result(ers[j])
                assert int(rj["status"]) == 0 and int(rj["n_frames"]) == n_frames, (name, "engine", j, rj)
            rec["engine"] = {"GiB_per_s": round(payload / te / GIB, 1), "ms_per_batch": round(te * 1e3, 4),
                             "roofline_frac": round((len(wire) + payload) / te / 1e9 / HBM_PEAK_GBS, 4),
                             "jobs_per_run": ENGINE_JOBS,
                             "path": "fws_decode_engine_run: one run of distinct batches, whole decodes alternating "
                                     "over two HIP streams with a workspace each; every job's status and frame "
                                     "count checked"}
            eng.close()
            del ebufs, efr, ers
        del bufs
        c.close()
        return rec

    if want(args, "c2s"):
        out["C2_stream_decode"] = decode_cfg("C2", wire_c2, args.frames)
        _profile(out["C2_stream_decode"], "c2s")
    if want(args, "c3"):
        w3, d3, _ = gpu.config_c3()
        out["C3_mixed_stream_decode"] = decode_cfg("C3", w3, len(d3))
        _profile(out["C3_mixed_stream_decode"], "c3")
        del w3
    # SURVEY §6's dense workload: 200 000 x 64 B frames (~3 700 headers per 256 KiB super
    # tile: the big-ST resolve path); the reference's 1-core rate is cpu_baseline.dense_64B_one_core
    if want(args, "dense"):
        wd, dd, _ = gpu.config_c2(n_frames=DENSE_FRAMES, payload=DENSE_PAYLOAD)
        out["dense_64B_stream_decode"] = decode_cfg("dense", wd, DENSE_FRAMES, pipelined=False)
        _profile(out["dense_64B_stream_decode"], "dense")
        del wd
    if want(args, "c4"):
        out.update(c4_extra(dev, steps, stream))
    if want(args, "tx"):
        out.update(tx_extra(dev, args, steps, stream))
    if args.c5 and (want(args, "c5s") or want(args, "c5d")):
        out.update(c5_extra(dev, args, stream))
    if want(args, "e2e"):
        out.update(e2e_extra(ctx, wire_c2, dev, args, stream))
    return {"extra": out}


def c4_extra(dev, steps, stream):
    """C4: one 256 MiB fragmented message, unmask + reassemble out of place. The
    source rotates over SRC_COPIES copies (1 GiB with the destinations' 1 GiB):
    one source re-read every step is partly served by the 256 MB Infinity Cache
    (r06: 0.084 against 0.100 ms, profiles/r06/ab_mall.jsonl)."""
    out = {}
    w4, d4, _ = gpu.config_c4()
    c = gpu.Ctx(dev.index or 0, max_frames=len(d4) + 8, max_stream_bytes=len(w4))
    srcs = [torch.from_numpy(w4).to(dev) for _ in range(SRC_COPIES)]
    total = int(d4["payload_len"].sum())
    dsts = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(4)]
    dd4 = gpu.descs_to_device(d4, dev)
    t = _time(lambda i: gpu.unmask_gather(c, dsts[i % 4], srcs[i % SRC_COPIES], dd4, len(d4)), steps, stream,
              warmup=EXTRA_WARMUP)
    out["C4_fragmented_reassemble"] = {"GiB_per_s": round(total / t / GIB, 1), "ms_per_step": round(t * 1e3, 4),
                                       "fragments": len(d4), "alg_GB_per_s": round((len(w4) + total) / t / 1e9, 1),
                                       "rotating_sources": SRC_COPIES,
                           "note": "r06: sources rotate past the 256 MB MALL; r05 and earlier re-read one source "
                                   "(91.0 against 103.5 us, profiles/r06/ab_mall.jsonl)",
                                       "note": "r06: sources rotate past the 256 MB MALL; r05 and earlier re-read one "
                                               "source (one source: 84.4 us, four: 99.9 us before r06's plan + "
                                               "k_gather_fast<kFlat> default, profiles/r06/ab_mall.jsonl)",
                                       "roofline": _step_roofline(len(w4) + total, t, "whole fws_gpu_unmask_gather step: wire read + payload written out of place")}
    _profile(out["C4_fragmented_reassemble"], "c4")
    c.close()
    del srcs, dsts, w4
    return out


def tx_extra(dev, args, steps, stream):
    """TX: the C2 shape sent by a client -- 65 536 x 4 KiB payloads (back to
    back in HBM) framed and masked into one wire buffer by fws_gpu_encode_frames"""
    out = {}
    n = args.frames
    pl = args.payload
    rng = np.random.default_rng(7)
    txd = np.zeros(n, dtype=gpu.TX_DESC)
    txd["src_off"] = np.arange(n, dtype=np.uint64) * pl
    txd["len"] = pl
    txd["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    txd["opcode"] = 2
    txd["fin"] = 1
    txd["masked"] = 1
    payload = rng.integers(0, 256, n * pl, dtype=np.uint8)
    # the payloads rotate over SRC_COPIES copies (see c4_extra: 0.091 against 0.103 ms
    # with one source re-read every step, profiles/r06/ab_mall.jsonl)
    tsrcs = [torch.from_numpy(payload).to(dev) for _ in range(SRC_COPIES)]
    tdd = torch.from_numpy(txd.view(np.uint8).copy()).to(dev)
    hdr = 2 + 4 + (0 if pl < 126 else 2 if pl < 65536 else 8)
    tx_total = n * (pl + hdr)
    c = gpu.Ctx(dev.index or 0, max_frames=n, max_stream_bytes=tx_total)
    touts = [torch.empty(tx_total, dtype=torch.uint8, device=dev) for _ in range(4)]
    olen = torch.empty(1, dtype=torch.int64, device=dev)
    t = _time(lambda i: gpu.encode_frames(c, touts[i % 4], tsrcs[i % SRC_COPIES], tdd, n, out_len=olen), steps, stream,
              warmup=EXTRA_WARMUP)
    assert int(olen.item()) == tx_total
    out["C2_tx_encode"] = {"GiB_per_s": round(n * pl / t / GIB, 1), "ms_per_step": round(t * 1e3, 4),
                           "frames": n, "alg_GB_per_s": round((n * pl + tx_total) / t / 1e9, 1),
                           "rotating_sources": SRC_COPIES,
                           "path": "fws_gpu_encode_frames: client frames (header + key + masked payload)",
                           "roofline": _step_roofline(n * pl + tx_total, t, "whole fws_gpu_encode_frames step: payload read + frames written")}
    _profile(out["C2_tx_encode"], "tx")
    c.close()
    del touts, tsrcs
    return out


def c5_extra(dev, args, stream):
    """C5 per-GPU share: 262 144 x 16 KiB TEXT frames (4 GiB), unmask + per-frame UTF-8 flags,
    as a raw stream (fws_gpu_decode_stream) and in descriptor mode (fws_gpu_unmask_sorted_utf8).
    Both decode in place, and an in-place unmask of already unmasked text is a different
    workload (plain text in, masked bytes out, every flag "invalid"), so every timed call
    gets its own freshly masked copy of the batch: C5_STREAM_STEPS device copies (~69 GB of
    the 288 GB HBM), re-masked by device copies between the two modes; the untimed warm-up
    calls run on one more copy. The flags of every timed call are valid; the last call's
    are checked against the generator's."""
    out = {}
    w5, d5, ok5 = gpu.config_c5()
    n5 = len(d5)
    pl5 = int(d5["payload_len"].sum())
    expect = np.asarray(ok5, dtype=np.uint8)[:n5]
    master = torch.from_numpy(w5).to(dev)
    k = C5_STREAM_STEPS
    warm = master.clone()
    bufs = [master.clone() for _ in range(k)]
    c = gpu.Ctx(dev.index or 0, max_frames=n5 + 64, max_stream_bytes=len(w5))

    def timed(fn):
        _warm(lambda i: fn(warm), warmup=EXTRA_WARMUP)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record(stream)
        for b in bufs:
            fn(b)
        ev1.record(stream)
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) / 1e3 / k

    if want(args, "c5s"):
        cap = n5 + 64
        frames = torch.empty(cap * gpu.FRAME_INFO.itemsize, dtype=torch.uint8, device=dev)
        res = torch.empty(gpu.DECODE_RESULT.itemsize, dtype=torch.uint8, device=dev)
        ok = torch.zeros(cap, dtype=torch.uint8, device=dev)

        def dec(b):
            rc, _, _, _ = gpu.decode_stream(c, b, cap, frames=frames, result=res, utf8_ok=ok)
            assert rc == 0, rc
        t = timed(dec)
        r = gpu.read_result(res)
        flags = ok[:n5].cpu().numpy()
        payload = int(gpu.read_frames(frames, n5)["payload_len"].sum())
        rec = {"GiB_per_s": round(payload / t / GIB, 1), "ms_per_step": round(t * 1e3, 4), "frames": n5,
               "wire_bytes": len(w5), "alg_GB_per_s": round((len(w5) + payload) / t / 1e9, 1),
               "rotating_buffers": k, "big_super_tiles": gpu.decode_counters(c)["big_super_tiles"],
               "roofline": _step_roofline(len(w5) + payload, t, "whole fws_gpu_decode_stream step"),
               "utf8_invalid_frames": int((flags == 0).sum()),
               "utf8_invalid_frames_expected": int((expect == 0).sum()),
               "flags_match_generator": bool(np.array_equal(flags, expect)),
               "checked_call_status": int(r["status"]), "checked_call_frames": int(r["n_frames"]),
               "timed_input": f"{k} distinct freshly masked copies of the batch, one per timed call (the "
                              "warm-up calls run on another); status, frame count and flags checked on the "
                              "last timed call"}
        check_c5_stream(rec)
        _profile(rec, "c5s")
        out["C5_utf8_text_decode"] = rec
        for b in bufs:
            b.copy_(master)                                  # masked again for the descriptor mode
        warm.copy_(master)
        del frames, res, ok
    if want(args, "c5d"):
        # the same batch in descriptor mode (a batch split at frame boundaries knows its
        # frames): one pass of unmask + UTF-8 flags, fws_gpu_unmask_sorted_utf8
        dd5 = gpu.descs_to_device(d5, dev)
        ok = torch.empty(n5, dtype=torch.uint8, device=dev)
        t = timed(lambda b: gpu.unmask_sorted_utf8(c, b, dd5, n5, ok))
        flags_ok = bool(np.array_equal(ok.cpu().numpy(), expect))
        if not flags_ok:
            raise RuntimeError("C5 descriptor mode: UTF-8 flags differ from the generator's")
        out["C5_utf8_descriptor"] = {"GiB_per_s": round(pl5 / t / GIB, 1), "ms_per_step": round(t * 1e3, 4),
                                     "frames": n5, "alg_GB_per_s": round((len(w5) + pl5) / t / 1e9, 1),
                                     "flags_match_generator": flags_ok, "rotating_buffers": k,
                                     "timed_input": f"{k} distinct freshly masked copies, one per timed call; "
                                                    "flags of the last call checked",
                                     "path": "fws_gpu_unmask_sorted_utf8: k_unmask_sorted_utf8 + k_utf8_seam_sorted",
                                     "roofline": _step_roofline(len(w5) + pl5, t, "whole fws_gpu_unmask_sorted_utf8 step: wire read + payload written")}
        _profile(out["C5_utf8_descriptor"], "c5d")
    c.close()
    del master, warm, bufs, w5
    torch.cuda.empty_cache()
    return out


def e2e_extra(ctx, wire_c2, dev, args, stream):
    """end-to-end: pinned host -> HBM -> unmask -> host (PCIe-inclusive), C2"""
    out = {}
    n = args.frames
    host_in = torch.from_numpy(wire_c2).pin_memory()
    host_out = torch.empty_like(host_in).pin_memory()
    dbuf = torch.empty(len(wire_c2), dtype=torch.uint8, device=dev)
    _, descs, _ = gpu.config_c2(seed=42, n_frames=n, payload=args.payload)
    dd = gpu.descs_to_device(descs, dev)
    def e2e(i):
        dbuf.copy_(host_in, non_blocking=True)
        gpu.unmask_batch(ctx, dbuf, dd, n)
        host_out.copy_(dbuf, non_blocking=True)
    t = _time(e2e, 10, stream)
    out["C2_end_to_end_pcie"] = {"GiB_per_s": round(int(descs["payload_len"].sum()) / t / GIB, 1),
                                 "ms_per_step": round(t * 1e3, 3),
                                 "path": "pinned H2D + fws_gpu_unmask_batch + D2H, one stream"}
    # zero copy: the same batch unmasked by fws_gpu_unmask_sorted on the pinned host
    # buffer itself -- the kernel's loads and stores cross PCIe in both directions at
    # once, no copy engine and no device staging (tools/zc_probe.py)
    zc = torch.from_numpy(wire_c2.copy()).pin_memory()
    t = _time(lambda i: gpu.unmask_sorted(ctx, zc, dd, n), 10, stream, warmup=2)
    zc_ok = bool(np.array_equal(zc.numpy(), wire_c2))      # 12 in-place passes: masked again
    out["C2_end_to_end_zero_copy"] = {"GiB_per_s": round(int(descs["payload_len"].sum()) / t / GIB, 1),
                                      "ms_per_step": round(t * 1e3, 3), "bytes_restored": zc_ok,
                                      "path": "fws_gpu_unmask_sorted on the pinned host batch (zero copy over PCIe)"}
    del zc
    # end to end, pipelined: C2 wire batches from pinned host memory through fws_rx_pipe
    # (H2D -> parse + unmask -> D2H of bytes, frames, result; depth 3 streams)
    del dbuf
    pipe = gpu.RxPipe(dev.index or 0, max_batch_bytes=len(wire_c2), max_frames=n + 64, depth=3)
    hosts = [torch.from_numpy(wire_c2.copy()).pin_memory() for _ in range(4)]
    for i in range(3):
        pipe.wait(pipe.submit(hosts[i]), copy_frames=False)
    k = 12
    t0 = time.perf_counter()
    tickets = [pipe.submit(hosts[i % 4]) for i in range(k)]   # submit waits when a slot is busy
    for tk in tickets[-3:]:
        pipe.wait(tk, copy_frames=False)
    t = (time.perf_counter() - t0) / k
    _, res, _ = pipe.wait(tickets[-1], copy_frames=False)
    assert int(res["status"]) == 0 and int(res["n_frames"]) == n
    out["C2_stream_end_to_end_pipelined"] = {
        "GiB_per_s": round(int(descs["payload_len"].sum()) / t / GIB, 1), "ms_per_batch": round(t * 1e3, 3),
        "path": "fws_rx_pipe: pinned H2D -> fws_gpu_decode_stream -> D2H (bytes + frames + result), 3 streams; "
                "bound by PCIe: H2D and D2H do not overlap on this box (profiles/r01/pcie_probe.json)",
        "batches": k}
    pipe.close()
    return out


if __name__ == "__main__":
    main()
