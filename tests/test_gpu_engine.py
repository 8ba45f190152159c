"""Engine-level guarantees of the device surface (include/uvhttp_ws_amd.h, "Streams and graphs"
and UVHTTP_WS_FRAME_ERR_DEVICE):

* a look-back wait that gives up is reported, never turned into wrong descriptors: the call
  delivers nothing, its summary / results say ERR_DEVICE and engine_sync raises;
* a decode captured into a hipGraph and replayed over CHANGING frame bytes stays bit-exact
  (each replay draws a fresh device-side epoch, so tags left by the previous replay — first
  failure, tile maps, look-back records — never match);
* calls on different streams serialise on the engine's one workspace.
Every check compares with the oracle (oracle/ws_oracle.c)."""
import os
import random

import numpy as np
import pytest

import _oracle
from test_gpu_parity import _frame

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _engine(env=None):
    import uvhttp_amd as U
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        return U.GpuEngine(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _batch(rng, n, fail_at=None, sizes=(0, 1, 125, 126, 300, 4000, 70000)):
    frames, offs, pos = [], [], 0
    for i in range(n):
        payload = rng.randbytes(rng.choice(sizes))
        f = _frame(2, 1, payload, rng.randbytes(4), True, 4 if i == fail_at else 0)
        frames.append(f)
        offs.append(pos)
        pos += len(f)
    return b"".join(frames), np.array(offs, np.uint64)


def test_lookback_give_up_is_reported(torch):
    """UVHTTP_WS_MAX_POLLS=0 makes every block with a predecessor give up at once: the call
    must report ERR_DEVICE, unmask nothing and make engine_sync fail — then a normal engine
    decodes the same bytes correctly."""
    import uvhttp_amd as U
    rng = random.Random(11)
    wire, offs = _batch(rng, 4096, sizes=(0, 1, 20, 125, 200))
    w = np.frombuffer(wire, np.uint8)
    eng = _engine({"UVHTTP_WS_MAX_POLLS": "0"})
    d = torch.from_numpy(np.concatenate([w, np.zeros(64, np.uint8)])).to("cuda")
    before = d.clone()
    o = torch.from_numpy(offs.view(np.int64)).to("cuda")
    desc, summ = eng.decode_inplace(d, len(offs), offsets=o, wire_len=w.size)
    torch.cuda.synchronize()
    s = eng.read_summary(summ)
    assert s["status"] == -1 and s["first_status"] == -11 and s["n_delivered"] == 0, s
    assert (eng.read_desc(desc, len(offs))["status"] == 2).all()
    assert torch.equal(d, before)
    with pytest.raises(U.GpuError):
        eng.sync()
    eng.sync()  # reported once
    # a stride batch of small frames: nothing unmasked either
    sw = b"".join(_frame(2, 1, rng.randbytes(40), rng.randbytes(4), True, 0) for _ in range(30000))
    sd = torch.from_numpy(np.frombuffer(sw + bytes(64), np.uint8).copy()).to("cuda")
    sbefore = sd.clone()
    desc, summ = eng.decode_inplace(sd, 30000, stride=len(sw) // 30000, wire_len=len(sw))
    torch.cuda.synchronize()
    s = eng.read_summary(summ)
    assert s["status"] == -1 and s["first_status"] == -11 and s["n_delivered"] == 0, s
    assert torch.equal(sd, sbefore)
    with pytest.raises(U.GpuError):
        eng.sync()
    # the stream decode has no look-back (per-connection walk + one-block scan) unless the wave
    # walk runs fused (UVHTTP_WS_WALK_FUSE=1: k_swalk_fused finds first frames by a look-back
    # over blocks of connections; the speculative decode, which has none and would take these
    # connections first, is off).  Fused, every block after the first gives up, so every
    # stream reports ERR_DEVICE and nothing is unmasked ...
    st = np.zeros(64, U.STREAM_DT)
    per = w.size // 64
    idx = np.minimum(np.searchsorted(offs, np.arange(64) * per), len(offs) - 1)
    cut = [int(offs[i]) for i in idx] + [w.size]
    for k in range(64):
        st[k] = (cut[k], cut[k + 1] - cut[k], 1 << 30, 0, 0, 1 << 24, 1 << 26, 1, 0, 0, 0)
    sdev = torch.from_numpy(st.view(np.uint8).copy()).to("cuda")
    eng.close()
    eng = _engine({"UVHTTP_WS_MAX_POLLS": "0", "UVHTTP_WS_WALK_FUSE": "1", "UVHTTP_WS_STREAM_SPEC": "0"})
    d2 = before.clone()
    _, res = eng.decode_streams(d2, sdev, 64, 8192, wire_len=w.size)
    torch.cuda.synchronize()
    rs = eng.read_stream_results(res, 64)
    assert all(r.status == -1 and r.first_status == -11 and r.n_delivered == 0 for r in rs)
    assert torch.equal(d2, before)
    with pytest.raises(U.GpuError):
        eng.sync()
    eng.close()
    # ... while the walk, its one-block scan and k_stream_desc apart (the default) have no
    # look-back: an engine with the same poll bound decodes the streams normally
    eng = _engine({"UVHTTP_WS_MAX_POLLS": "0"})
    d2 = before.clone()
    _, res = eng.decode_streams(d2, sdev, 64, 8192, wire_len=w.size)
    torch.cuda.synchronize()
    rs = eng.read_stream_results(res, 64)
    assert all(r.status == 0 for r in rs)
    assert sum(r.n_delivered for r in rs) == len(offs)
    eng.sync()
    eng.close()
    good = _engine()
    desc, summ = good.decode_inplace(d, len(offs), offsets=o, wire_len=w.size)
    torch.cuda.synchronize()
    good.sync()
    ref = _oracle.decode_batch(w, len(offs), offsets=offs)
    assert good.read_summary(summ) == ref["summary"]
    assert np.array_equal(d[:w.size].cpu().numpy(), ref["wire"])
    good.close()


def test_graph_capture_replay_changing_batches(torch):
    """Capture one decode_inplace (offset-table layout) and replay it over four different
    batches of the same frame count and wire length: a failing frame early, none, a failure
    late, then different frame sizes.  Each replay must equal the oracle; a stale first-
    failure tag or tile map from the previous replay would break the second and fourth."""
    t = torch
    rng = random.Random(12)
    n = 3000
    batches = [_batch(rng, n, fail_at=40), _batch(rng, n), _batch(rng, n, fail_at=2500),
               _batch(rng, n, sizes=(2, 60, 9000))]
    wl = max(len(b[0]) for b in batches)
    eng = _engine()
    wire = t.zeros(wl + 64, dtype=t.uint8, device="cuda")
    offs = t.zeros(n, dtype=t.int64, device="cuda")
    desc, summ = eng.alloc_outputs(n)
    eng.reserve(n, wl, 0)

    def load(k):
        b, o = batches[k]
        host = np.zeros(wl, np.uint8)
        host[:len(b)] = np.frombuffer(b, np.uint8)
        wire[:wl].copy_(t.from_numpy(host))
        offs.copy_(t.from_numpy(o.view(np.int64)))
        return host

    # warm (uncaptured) call on the capture stream's shapes, then capture
    load(0)
    s = t.cuda.Stream()
    with t.cuda.stream(s):
        eng.decode_inplace(wire, n, offsets=offs, wire_len=wl, desc=desc, summary=summ, stream=s)
    s.synchronize()
    g = t.cuda.CUDAGraph()
    with t.cuda.graph(g, stream=s):
        eng.decode_inplace(wire, n, offsets=offs, wire_len=wl, desc=desc, summary=summ, stream=s)
    for k in [0, 1, 2, 3, 1]:
        host = load(k)
        t.cuda.synchronize()
        g.replay()
        t.cuda.synchronize()
        ref = _oracle.decode_batch(host, n, offsets=batches[k][1], wire_len=wl)
        got = eng.read_summary(summ)
        assert got == ref["summary"], (k, got, ref["summary"])
        assert np.array_equal(wire[:wl].cpu().numpy(), ref["wire"]), k
        assert np.array_equal(eng.read_desc(desc, n)["status"], ref["status"]), k
    # host calls after the replays, then replays again: the workspace holds the replays' tags,
    # whose device epochs are larger than any host call's — the host call's claims (first
    # failure, tile maps) must still win over them (round 5: they did not, and a host call after
    # a replay delivered frames after a failure)
    for k in [2, 0, 3]:
        host = load(k)
        eng.decode_inplace(wire, n, offsets=offs, wire_len=wl, desc=desc, summary=summ, stream=s)
        s.synchronize()
        ref = _oracle.decode_batch(host, n, offsets=batches[k][1], wire_len=wl)
        assert eng.read_summary(summ) == ref["summary"], ("host after replay", k)
        assert np.array_equal(wire[:wl].cpu().numpy(), ref["wire"]), ("host after replay", k)
        assert np.array_equal(eng.read_desc(desc, n)["status"], ref["status"]), ("host after replay", k)
        host = load((k + 1) % 4)
        t.cuda.synchronize()
        g.replay()
        t.cuda.synchronize()
        ref = _oracle.decode_batch(host, n, offsets=batches[(k + 1) % 4][1], wire_len=wl)
        assert eng.read_summary(summ) == ref["summary"], ("replay after host", k)
        assert np.array_equal(wire[:wl].cpu().numpy(), ref["wire"]), ("replay after host", k)
    eng.sync()
    eng.close()


def test_calls_on_two_streams_serialise(torch):
    """Back-to-back calls on two streams with no host sync between them share one workspace;
    the engine orders the second after the first.  Both must equal the oracle."""
    t = torch
    rng = random.Random(13)
    eng = _engine()
    runs = []
    s1, s2 = t.cuda.Stream(), t.cuda.Stream()
    for k in range(4):
        b, o = _batch(rng, 5000, fail_at=[None, 1000, 4000, None][k], sizes=(0, 1, 126, 600))
        w = np.frombuffer(b, np.uint8)
        d = t.from_numpy(np.concatenate([w, np.zeros(64, np.uint8)])).to("cuda")
        od = t.from_numpy(o.view(np.int64)).to("cuda")
        desc, summ = eng.alloc_outputs(len(o))
        runs.append((w, o, d, od, desc, summ))
    t.cuda.synchronize()
    for (w, o, d, od, desc, summ), s in zip(runs, [s1, s2, s1, s2]):
        eng.decode_inplace(d, len(o), offsets=od, wire_len=w.size, desc=desc, summary=summ,
                           stream=s)
    t.cuda.synchronize()
    for w, o, d, od, desc, summ in runs:
        ref = _oracle.decode_batch(w, len(o), offsets=o)
        assert eng.read_summary(summ) == ref["summary"]
        assert np.array_equal(d[:w.size].cpu().numpy(), ref["wire"])
    eng.close()


def test_graph_capture_replay_stride_batches(torch):
    """A stride-layout decode captured and replayed over changing frame bytes of one stride: no
    failure, a state-machine failure early, none again, a failure late."""
    t = torch
    rng = random.Random(14)
    n, plen = 20000, 200

    def batch(fail_at):
        frames = []
        for i in range(n):
            op = 0 if i == fail_at else 2  # CONTINUATION with nothing open
            frames.append(_frame(op, 1, rng.randbytes(plen), rng.randbytes(4), True, 0))
        return b"".join(frames)
    batches = [batch(None), batch(37), batch(None), batch(19000)]
    stride = len(batches[0]) // n
    wl = len(batches[0])
    eng = _engine()
    wire = t.zeros(wl + 64, dtype=t.uint8, device="cuda")
    desc, summ = eng.alloc_outputs(n)
    eng.reserve(n, wl, 0)
    s = t.cuda.Stream()
    wire[:wl].copy_(t.from_numpy(np.frombuffer(batches[0], np.uint8).copy()))
    with t.cuda.stream(s):
        eng.decode_inplace(wire, n, stride=stride, wire_len=wl, desc=desc, summary=summ, stream=s)
    s.synchronize()
    g = t.cuda.CUDAGraph()
    with t.cuda.graph(g, stream=s):
        eng.decode_inplace(wire, n, stride=stride, wire_len=wl, desc=desc, summary=summ, stream=s)
    for k in [0, 1, 2, 3, 1]:
        host = np.frombuffer(batches[k], np.uint8).copy()
        wire[:wl].copy_(t.from_numpy(host))
        t.cuda.synchronize()
        g.replay()
        t.cuda.synchronize()
        ref = _oracle.decode_batch(host, n, stride=stride, wire_len=wl)
        assert eng.read_summary(summ) == ref["summary"], k
        assert np.array_equal(wire[:wl].cpu().numpy(), ref["wire"]), k
        assert np.array_equal(eng.read_desc(desc, n)["status"], ref["status"]), k
    # host calls (fused path, summary-only, compact) after the replays: their failure claims must
    # displace the replays' larger-epoch tags
    for k, mode in ((1, "desc"), (3, "no_desc"), (1, "compact")):
        host = np.frombuffer(batches[k], np.uint8).copy()
        wire[:wl].copy_(t.from_numpy(host))
        ref = _oracle.decode_batch(host, n, stride=stride, wire_len=wl, compact=mode == "compact",
                                   arena_cap=wl + 64)
        if mode == "compact":
            arena = t.zeros(wl + 64, dtype=t.uint8, device="cuda")
            eng.decode_compact(wire, n, arena, stride=stride, wire_len=wl, desc=desc, summary=summ, stream=s)
        else:
            eng.decode_inplace(wire, n, stride=stride, wire_len=wl, desc=desc, summary=summ, stream=s,
                               no_desc=mode == "no_desc")
        s.synchronize()
        assert eng.read_summary(summ) == ref["summary"], ("host after replay", k, mode)
        assert np.array_equal(wire[:wl].cpu().numpy(), ref["wire"]), ("host after replay", k, mode)
        g.replay()
        t.cuda.synchronize()
    eng.sync()
    eng.close()
