"""CPU, world_size 2 over gloo: the multi-GPU path of bench.py (one process
per GPU, independent shards, barrier + max-over-ranks timing, aggregate =
sum of shards / slowest rank) with the oracle standing in for the device
decode. No collective touches frame data; bench.py's control group is gloo at
every N (bench.init_group), so no RCCL initialisation is on the N > 1 path."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import bench
    backend = bench.init_group(world)                # bench.py's own N > 1 control group
    import orc
    from flashws_amd import gpu
    wire, descs, _ = gpu.config_c2(seed=bench.shard_seed(rank), n_frames=512)
    dist.barrier()
    import time
    t0 = time.perf_counter()
    buf = wire.copy()
    ret, frames, _, _ = orc.orc_decode_stream(buf)
    t1 = time.perf_counter()
    dist.barrier()
    step = bench.max_over_ranks(world, t1 - t0)
    payload = int(descs["payload_len"].sum())
    agg = bench.aggregate_gib_s(world, payload, step)
    digest = torch.tensor([int(buf[:4096].sum())], dtype=torch.int64)
    gathered = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gathered, digest)          # test-only check that shards differ
    q.put((rank, ret, len(frames), step, t1 - t0, agg, payload, [int(g) for g in gathered], backend))
    dist.destroy_process_group()


def test_two_rank_batch_split_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    steps = [r[3] for r in res]
    assert steps[0] == steps[1] == max(r[4] for r in res)        # both report the slowest rank
    for rank, ret, nf, step, own, agg, payload, gathered, backend in res:
        assert backend == "gloo"                                   # no device collective is initialised
        assert ret == 0 and nf == 512
        assert np.isclose(agg, world * payload / step / (1 << 30))
    assert res[0][7][0] != res[0][7][1]                           # independent shards


def test_bench_launcher_two_ranks_gloo():
    """bench.py --gpus 2 starts its own ranks (torch.distributed.run as a child
    process) and reports the slowest rank's step and the whole-job aggregate;
    --launcher-selftest swaps the device step for a host XOR over gloo."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--launcher-selftest",
                          "--steps", "3", "--warmup", "1", "--frames", "512", "--no-cpu"],
                         cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout                               # rank 0 prints one line
    rec = lines[0]
    assert rec["selftest"] and rec["n_gpus"] == 2 and rec["rank"] == 0
    assert rec["step_s"] >= rec["own_step_s"]                        # max over ranks
    assert np.isclose(rec["value"], 2 * rec["payload_bytes_per_rank"] / rec["step_s"] / (1 << 30))
    d = rec["shard_digests"]
    assert len(d) == 2 and d[0] != d[1]                              # independent shards (seed 42 + rank)
    # the launcher counted GPUs from the KFD topology (no HIP init) before forking
    assert rec["launcher_kfd_gpus"] is not None


def test_kfd_gpu_count(tmp_path):
    """bench.launch_ranks counts GPUs from /sys/class/kfd topology nodes with a
    gfx target (CPU nodes have gfx_target_version 0), narrowed by the
    *_VISIBLE_DEVICES lists, instead of torch.cuda.device_count()."""
    import bench
    for i, ver in enumerate([0, 90500, 90500, 90500]):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 0\ngfx_target_version {ver}\nsimd_count 1024\n")
    assert bench.kfd_gpu_count(str(tmp_path), env={}) == 3
    assert bench.kfd_gpu_count(str(tmp_path), env={"ROCR_VISIBLE_DEVICES": "0,1"}) == 2
    assert bench.kfd_gpu_count(str(tmp_path), env={"HIP_VISIBLE_DEVICES": ""}) == 0
    assert bench.kfd_gpu_count(str(tmp_path / "absent"), env={}) is None


def test_c5_stream_record_check_fails_loudly():
    """bench.py's C5 stream record: its UTF-8 flags come from the call on the
    masked batch and a mismatch with the generator makes the bench raise
    (a record once showed 262144 invalid frames against 2692)."""
    import bench
    good = {"frames": 262144, "utf8_invalid_frames": 2692, "utf8_invalid_frames_expected": 2692,
            "flags_match_generator": True, "checked_call_status": 0, "checked_call_frames": 262144}
    assert bench.check_c5_stream(dict(good)) == good
    for bad in ({"utf8_invalid_frames": 262144}, {"utf8_invalid_frames_expected": 2693},
                {"flags_match_generator": False}, {"checked_call_status": -1}, {"checked_call_frames": 5}):
        with pytest.raises(RuntimeError):
            bench.check_c5_stream({**good, **bad})
