"""GPU: the persistent receive decode (fws_gpu_ctx_set_rx_persistent, r05).
A context with the service decodes its sessions' and muxes' small reads on a
resident grid instead of a launch per read; the results must be exactly the
launch path's: every tests/golden/ KAT case replayed read by read against the
compiled reference's results (w_socket.h:543-769), in place (registered
memory) and staged (pinned), through a session and through a mux; random
multi-connection traffic and the declined (>256 headers) path against
standalone sessions on a context without the service; the grid's lifecycle
(exit after its linger time, relaunch on the next read, teardown while it is
resident)."""
import time

import numpy as np
import pytest
import torch

from flashws_amd import gpu
from test_gpu_inplace import CASES, _declined_reads, _state
from test_gpu_mux import _random_stream
from test_gpu_session import _out_matches, session_view

pytestmark = pytest.mark.gpu


def _set_push(on):
    from flashws_amd._lib import lib
    return lib().fws_internal_set_rx_push(on)


@pytest.fixture(scope="module", params=[1, 0], ids=["push", "pull"])
def sctx(cuda, request):
    """A context with the service in push mode (the session's small reads
    written into device memory by the CPU, where the device has a large BAR)
    and in pull mode (the grid reads them over PCIe)."""
    old = _set_push(request.param)
    c = gpu.Ctx(0, max_frames=1 << 16, max_stream_bytes=1 << 24)
    c.set_rx_persistent(16)
    c.push_mode = request.param
    yield c
    c.close()
    _set_push(old)


@pytest.fixture(scope="module")
def plain_ctx(cuda):
    c = gpu.Ctx(0, max_frames=1 << 16, max_stream_bytes=1 << 24)
    yield c
    c.close()


@pytest.fixture(scope="module")
def arena(cuda):
    a = gpu.HostArena(32 << 20)
    yield a
    a.close()


@pytest.mark.parametrize("align_off", [0, 5], ids=["in_place", "staged"])
def test_service_session_kat(sctx, arena, align_off):
    before = sctx.rx_service_stats()
    for name in sorted(CASES):
        case = CASES[name]
        s = gpu.RxSession(sctx)
        for i, (rd, exp) in enumerate(zip(case["reads"], case["expected"])):
            ret, buf, ev, ctl = s.feed(bytes.fromhex(rd), arena=arena, align_off=align_off)
            assert ret == exp["ret"], (name, i)
            assert _out_matches(exp["out"], buf), (name, i)
            assert session_view(ev, ctl) == exp["events"], (name, i)
            if ret < 0:
                break
            assert _state(s.state()) == exp["state"], (name, i)
        s.close()
    launches, requests = sctx.rx_service_stats()
    assert requests - before[1] > 100                  # the reads went through the resident grid
    assert launches - before[0] < requests - before[1]  # which was not relaunched per read
    pushes = sctx.rx_service_pushes()
    if sctx.push_mode:
        assert pushes > 100                            # (the MI355X boxes have a large BAR)
    else:
        assert pushes == 0


def test_service_mux_kat(sctx, arena, monkeypatch):
    monkeypatch.setenv("FWS_MUX_ZC_MAX", str(1 << 40))
    names = sorted(CASES)
    mux = gpu.RxMux(sctx, len(names))
    closed = set()
    before = sctx.rx_service_stats()[1]
    for r in range(max(len(CASES[n]["reads"]) for n in names)):
        live = [ci for ci, n in enumerate(names) if r < len(CASES[n]["reads"]) and ci not in closed]
        got = mux.feed([(ci, bytes.fromhex(CASES[names[ci]]["reads"][r])) for ci in live], arena=arena,
                       align_off=lambda i: 7 if i % 3 == 2 else 0)
        for ci, (ret, buf, ev, ctl) in zip(live, got):
            name, exp = names[ci], CASES[names[ci]]["expected"][r]
            assert ret == exp["ret"], (name, r)
            assert _out_matches(exp["out"], buf), (name, r)
            assert session_view(ev, ctl) == exp["events"], (name, r)
            if ret < 0:
                closed.add(ci)
            else:
                assert _state(mux.state(ci)) == exp["state"], (name, r)
    mux.close()
    assert sctx.rx_service_stats()[1] > before


def test_service_mux_random_vs_sessions(sctx, plain_ctx, arena):
    rng = np.random.default_rng(505)
    n = 48
    streams = [_random_stream(rng, int(rng.integers(5, 40))) for _ in range(n)]
    cuts = []
    for st in streams:
        pos, c = 0, []
        while pos < len(st):
            k = int(rng.choice([1, 7, 100, 4096, 5000, 70000]))
            c.append(st[pos:pos + k])
            pos += k
        cuts.append(c)
    mux = gpu.RxMux(sctx, n)
    ref = [gpu.RxSession(plain_ctx) for _ in range(n)]
    dead = set()
    for r in range(max(len(c) for c in cuts)):
        live = [i for i in range(n) if r < len(cuts[i]) and i not in dead]
        got = mux.feed([(i, cuts[i][r]) for i in live], arena=arena)
        for i, (ret, buf, ev, ctl) in zip(live, got):
            eret, ebuf, eev, ectl = ref[i].feed(cuts[i][r])
            assert ret == eret, (i, r)
            assert bytes(buf) == bytes(ebuf), (i, r)
            assert session_view(ev, ctl) == session_view(eev, ectl), (i, r)
            if ret < 0:
                dead.add(i)
    mux.close()
    for s in ref:
        s.close()


def test_service_mux_split_interleaved(sctx, plain_ctx, arena):
    """fws_rx_mux_submit / _complete with other requests of the same context in
    between (the batched hook's pipeline): chunks of at most 12 reads go to the
    resident grid (posted, not waited for), chunks of 20-24 to a launch; while
    a chunk decodes, another connection's session read on the same context
    (which waits for the posted chunk first) and a second mux's whole batch
    run. Every read equals a standalone session on a context without the
    service."""
    rng = np.random.default_rng(707)
    n = 40
    streams = [_random_stream(rng, int(rng.integers(5, 30))) for _ in range(n + 1)]
    cuts = []
    for st in streams:
        pos, c = 0, []
        while pos < len(st):
            k = int(rng.choice([1, 9, 300, 4096, 6000]))
            c.append(st[pos:pos + k])
            pos += k
        cuts.append(c)
    mux, mux2 = gpu.RxMux(sctx, n), gpu.RxMux(sctx, 1)
    side = gpu.RxSession(sctx)                          # connection n: fed between submit and complete
    ref = [gpu.RxSession(plain_ctx) for _ in range(n + 2)]
    side_r, dead = [0], set()
    extra = _random_stream(rng, 40)
    extra_cuts = [extra[i:i + 777] for i in range(0, len(extra), 777)]
    extra_r = [0]

    def between():
        i = side_r[0]
        if i < len(cuts[n]) and n not in dead:
            ret, buf, ev, ctl = side.feed(cuts[n][i], arena=arena, align_off=0)
            eret, ebuf, eev, ectl = ref[n].feed(cuts[n][i])
            assert (ret, bytes(buf), session_view(ev, ctl)) == (eret, bytes(ebuf), session_view(eev, ectl))
            if ret < 0:
                dead.add(n)
            side_r[0] += 1
        j = extra_r[0]
        if j < len(extra_cuts):                        # a whole second mux batch in between
            (ret, buf, ev, ctl), = mux2.feed([(0, extra_cuts[j])], arena=arena)
            eret, ebuf, eev, ectl = ref[n + 1].feed(extra_cuts[j])
            assert (ret, bytes(buf), session_view(ev, ctl)) == (eret, bytes(ebuf), session_view(eev, ectl))
            extra_r[0] += 1

    chunks = 0
    for r in range(max(len(c) for c in cuts[:n])):
        live = [i for i in range(n) if r < len(cuts[i]) and i not in dead]
        while live:
            k = int(rng.choice([3, 12, 20, 24]))
            part, live = live[:k], live[k:]
            got = mux.feed([(i, cuts[i][r]) for i in part], arena=arena, between=between)
            chunks += 1
            for i, (ret, buf, ev, ctl) in zip(part, got):
                eret, ebuf, eev, ectl = ref[i].feed(cuts[i][r])
                assert ret == eret, (i, r)
                assert bytes(buf) == bytes(ebuf), (i, r)
                assert session_view(ev, ctl) == session_view(eev, ectl), (i, r)
                if ret < 0:
                    dead.add(i)
    assert chunks > 20
    mux.close()
    mux2.close()
    side.close()
    for s in ref:
        s.close()


def test_service_declined_small_read(sctx, plain_ctx, arena):
    rng = np.random.default_rng(606)
    reads = _declined_reads(rng, 700)
    s, ref = gpu.RxSession(sctx), gpu.RxSession(plain_ctx)
    for rd in reads:
        ret, buf, ev, ctl = s.feed(rd, arena=arena, align_off=0)
        eret, ebuf, eev, ectl = ref.feed(rd)
        assert ret == eret == 0
        assert bytes(buf) == bytes(ebuf)
        assert session_view(ev, ctl) == session_view(eev, ectl)
    s.close()
    ref.close()


def test_service_relaunch_after_linger(cuda, arena):
    """The grid leaves after its linger time without a read; the next read
    relaunches it and decodes as before."""
    from flashws_amd._lib import lib
    old = lib().fws_internal_set_rx_linger_us(40)
    c = gpu.Ctx(0)
    try:
        c.set_rx_persistent(4)
        rng = np.random.default_rng(7)
        data = _random_stream(rng, 30)
        s, ref_ctx = gpu.RxSession(c), gpu.Ctx(0)
        ref = gpu.RxSession(ref_ctx)
        for k in range(6):
            rd = data[k * 500:(k + 1) * 500] if k < 5 else data[2500:]
            got, exp = s.feed(rd, arena=arena), ref.feed(rd)
            assert got[0] == exp[0] and bytes(got[1]) == bytes(exp[1])
            assert session_view(got[2], got[3]) == session_view(exp[2], exp[3])
            time.sleep(0.005)                                # >> 40 us: the grid has left
        launches, requests = c.rx_service_stats()
        assert requests >= 5 and launches >= 3         # (the last read may exceed the small-read path)
        s.close()
        ref.close()
        ref_ctx.close()
    finally:
        c.close()
        lib().fws_internal_set_rx_linger_us(old)


def test_service_teardown_while_resident(cuda, arena):
    """Closing a context whose grid is resident (default linger) sends the quit
    request and waits for the grid to drain; a new context works after it."""
    for _ in range(3):
        c = gpu.Ctx(0)
        c.set_rx_persistent(8)
        s = gpu.RxSession(c)
        ret, buf, ev, ctl = s.feed(bytes.fromhex(CASES[sorted(CASES)[0]]["reads"][0]), arena=arena)
        s.close()
        t0 = time.perf_counter()
        c.close()                                            # the grid is still lingering
        assert time.perf_counter() - t0 < 1.0


@pytest.mark.parametrize("queue", [1, 0, 2], ids=["high_priority", "pooled", "cu_masked"])
def test_service_grid_beside_other_streams(cuda, arena, queue):
    """The resident grid's hardware queue. The box runs
    GPU_MAX_HW_QUEUES=4; torch's stream plus 7 non-blocking HIP streams are
    more than that, so pooled streams share queues, and a shared queue runs
    its packets in order. With the grid resident (a 300 ms linger), a small
    unmask on every one of those streams must finish in far less than the
    linger, and the grid must still be the one that was launched (no
    relaunch: nothing forced it out). The default service stream is a
    non-blocking stream of the highest priority, whose queue pool no
    normal-priority stream shares; the r05 pooled stream and a CU-masked one
    (never pooled, but blocking: the legacy null stream waits for it) are
    measured too. The test prints, per stream, whether its work waited for
    the grid, and requires that none did for the default."""
    from flashws_amd._lib import lib
    old_q = lib().fws_internal_set_rx_service_queue(queue)
    old_l = lib().fws_internal_set_rx_linger_us(300000)
    c = gpu.Ctx(0)
    streams = [gpu.hip_stream() for _ in range(7)]
    try:
        c.set_rx_persistent(8)
        wire, descs, _ = gpu.config_c2(seed=5, n_frames=256)
        dev = torch.from_numpy(wire).to(cuda)
        dd = gpu.descs_to_device(descs, cuda)
        every = [torch.cuda.current_stream()] + streams

        def one(st):
            t0 = time.perf_counter()
            gpu.unmask_sorted(c, dev, dd, len(descs), stream=st)
            st.synchronize()
            return time.perf_counter() - t0

        for st in every:                                   # warm, no grid yet
            one(st)
        s = gpu.RxSession(c)
        reads = [bytes.fromhex(r) for r in CASES[sorted(CASES)[0]]["reads"]]
        got = s.feed(reads[0], arena=arena)
        launches0, _ = c.rx_service_stats()
        assert launches0 == 1
        times = [one(st) for st in every]
        s2 = gpu.RxSession(c)
        s2.feed(reads[0], arena=arena)                    # the same grid serves it
        launches1, _ = c.rx_service_stats()
        waited = [t > 0.05 for t in times]
        print(f"queue={queue} per-stream ms {[round(t * 1e3, 2) for t in times]} waited {waited} "
              f"launches {launches0}->{launches1}")
        if queue == 1:
            assert not any(waited), times
            assert launches1 == launches0
        assert torch.equal(dev.cpu(), torch.from_numpy(wire))   # 16 unmasks: an even count
        s.close()
        s2.close()
        del got
    finally:
        c.close()
        for st in streams:
            st.close()
        lib().fws_internal_set_rx_linger_us(old_l)
        lib().fws_internal_set_rx_service_queue(old_q)


def test_service_mux_complete_after_persistent_off(cuda, arena):
    """fws_rx_mux_submit posts a chunk to the resident grid; the service is
    switched off (fws_gpu_ctx_set_rx_persistent(ctx, 0), whose teardown drains
    the grid) before fws_rx_mux_complete. The chunk's results still come back,
    equal to a context without the service, and later chunks use launches."""
    rng = np.random.default_rng(808)
    n = 6
    streams = [_random_stream(rng, 12) for _ in range(n)]
    c, plain = gpu.Ctx(0), gpu.Ctx(0)
    try:
        c.set_rx_persistent(16)
        mux = gpu.RxMux(c, n)
        ref = [gpu.RxSession(plain) for _ in range(n)]
        cuts = [[st[i:i + 700] for i in range(0, len(st), 700)] for st in streams]
        toggled = [False]

        def between():
            if not toggled[0]:
                c.set_rx_persistent(0)
                toggled[0] = True

        for r in range(max(len(x) for x in cuts)):
            part = [i for i in range(n) if r < len(cuts[i])]
            got = mux.feed([(i, cuts[i][r]) for i in part], arena=arena, between=between)
            for i, (ret, buf, ev, ctl) in zip(part, got):
                eret, ebuf, eev, ectl = ref[i].feed(cuts[i][r])
                assert (ret, bytes(buf)) == (eret, bytes(ebuf)), (i, r)
                assert session_view(ev, ctl) == session_view(eev, ectl), (i, r)
        assert toggled[0]
        mux.close()
        for s in ref:
            s.close()
    finally:
        c.close()
        plain.close()
