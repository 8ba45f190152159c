"""Batched stateful stream decode against the oracle.

Many connections, each with its own limits and history (an open fragmented message and/or a
partial frame already buffered from earlier reads), decoded in ONE device call from raw
bytes (frame boundaries found on the device).  For every connection the product's host
delivery (uvhttp_ws_deliver_stream) must leave exactly what the oracle's
uvhttp_ws_process_data(conn, new_bytes) leaves: return code, callback transcript (messages,
closes, pongs, close echoes), recv-buffer position/size, fragment state.
"""
import ctypes as C
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


@pytest.fixture(scope="module", params=["lane", "wave", "wave-twopass"])
def eng(torch, request):
    """Every frame-discovery walk (a lane per connection; a wave per connection, single pass
    through the offset scratch or the two-walk fallback) must decode alike."""
    import os
    import uvhttp_amd as U
    env = {"UVHTTP_WS_WALK": request.param.split("-")[0],
           "UVHTTP_WS_WALK_SINGLE": "0" if request.param.endswith("twopass") else "1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        e = U.GpuEngine(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    yield e
    e.close()


SINK = {}


@pytest.fixture(scope="module")
def hooks():
    import uvhttp_amd as U

    @U.CONTEXT_RESOLVER
    def resolver(conn):
        return 0x77

    @U.CONTROL_SINK
    def sink(ctx, conn, op, p, n):
        SINK.setdefault(conn, []).append(("pong" if op == 0xA else "close_echo",
                                          C.string_at(p, n) if n else b""))

    U.lib().uvhttp_ws_amd_set_control_hooks(resolver, sink)
    yield
    U.lib().uvhttp_ws_amd_set_control_hooks(U.CONTEXT_RESOLVER(), U.CONTROL_SINK())


def _frames(rng, n, open_msg, bad):
    out = []
    for _ in range(n):
        key = bytes(rng.getrandbits(8) for _ in range(4))
        if rng.random() < 0.15:
            op, fin = rng.choice([8, 9, 10]), 1
            payload = rng.randbytes(rng.choice([0, 1, 2, 7, 125]))
        else:
            payload = rng.randbytes(rng.choice([0, 1, 3, 50, 125, 126, 1000, 5000, 70000]))
            if open_msg:
                op, fin = 0, rng.random() < 0.4
            else:
                op, fin = rng.choice([1, 2]), rng.random() < 0.6
            open_msg = not fin
        rsv, masked = 0, True
        if bad and rng.random() < 0.05:
            kind = rng.choice(["rsv", "unmasked", "cont", "ping_big"])
            rsv = 4 if kind == "rsv" else 0
            masked = kind != "unmasked"
            if kind == "cont":
                op = 0
            if kind == "ping_big":
                op, payload, fin = 9, bytes(200), 1
        out.append(_frame(op, fin, payload, key, masked, rsv))
    return out, open_msg


def _conn_case(rng, U, bad):
    mf = rng.choice([16 * 1024 * 1024, 65536, 4000])
    mm = rng.choice([64 * 1024 * 1024, 9000, 0])
    prod = U.WsConnection(1, mf, mm, user_data=True)
    orc = _oracle.OracleConn(1, mf, mm, record=1, wrapper=True)
    pre, open_msg = _frames(rng, rng.randint(0, 4), False, False)
    prefix = b"".join(pre)
    new, _ = _frames(rng, rng.randint(0, 6), open_msg, bad)
    new = b"".join(new)
    if rng.random() < 0.4:  # a partial frame already buffered from an earlier read
        tail = _frame(2, 1, rng.randbytes(rng.choice([10, 300, 3000])), b"\x01\x02\x03\x04")
        cut = rng.randint(1, len(tail) - 1)
        prefix += tail[:cut]
        new = tail[cut:] + new
    if rng.random() < 0.4 and new:  # and the new read may end mid-frame
        new = new[: rng.randint(0, len(new))]
    r1, r2 = prod.process_data(prefix), orc.process_data(prefix)
    assert r1 == r2
    if r1 != 0:
        return None
    return prod, orc, new


def _run_cases(torch, eng, U, cases, rng, max_frames):
    """One decode_streams call over every (product conn, oracle conn, new bytes) case, then the
    reference semantics: deliver_stream on the product side vs process_data on the oracle."""
    # batch wire: each connection's buffered bytes + new read, 16-B aligned starts, gaps allowed
    chunks, streams, pos = [], [], 0
    for prod, orc, new in cases:
        st = prod.struct
        buffered = C.string_at(st.recv_buffer, st.recv_buffer_pos) if st.recv_buffer_pos else b""
        data = buffered + new
        pos = (pos + 15) & ~15
        pos += rng.choice([0, 0, 16, 48])
        s = U.Stream()
        U.lib().uvhttp_ws_stream_init(prod.ptr, pos, len(data), C.byref(s))
        streams.append(s)
        chunks.append((pos, data))
        pos += len(data)
    wire = np.zeros(pos + 64, np.uint8)
    for p, d in chunks:
        wire[p:p + len(d)] = np.frombuffer(d, np.uint8)
    n = len(streams)
    sbytes = b"".join(bytes(s) for s in streams)
    dev_streams = torch.from_numpy(np.frombuffer(sbytes, np.uint8).copy()).to("cuda")
    dw = torch.from_numpy(wire.copy()).to("cuda")
    desc, res = eng.decode_streams(dw, dev_streams, n, max_frames, wire_len=pos)
    torch.cuda.synchronize()
    results = eng.read_stream_results(res, n)
    host_wire = dw.cpu().numpy()
    host_desc = desc.cpu().numpy()
    hw = (C.c_uint8 * host_wire.size).from_buffer(host_wire)
    hd = (C.c_uint8 * host_desc.size).from_buffer(host_desc)
    for k, (prod, orc, new) in enumerate(cases):
        SINK.pop(C.addressof(prod.ptr.contents), None)
        rc = U.lib().uvhttp_ws_deliver_stream(prod.ptr, hw, hd, C.byref(streams[k]),
                                              C.byref(results[k]))
        orc_rc = orc.process_data(new)
        assert rc == orc_rc, (k, results[k].as_dict())
        pev = [(t, a, p) for t, a, p in prod.events if t in ("message", "close")]
        oev = [(t, a, p if t == "message" else None) for t, a, p in orc.events()
               if t in ("message", "close")]
        assert pev == oev, k
        st = prod.struct
        assert st.recv_buffer_pos == _oracle.load().oracle_conn_recv_pos(orc.c), k
        assert st.recv_buffer_size == orc.recv_size, k
        frag = st.fragmented_size if st.fragmented_message else 0
        assert frag == _oracle.load().oracle_conn_frag_size(orc.c), k
        if rc == 0:
            assert results[k].pending_bytes == frag
        sink = SINK.get(C.addressof(prod.ptr.contents), [])
        exp = [(t, p) for t, a, p in orc.events() if t in ("pong", "close_echo")]
        # the prefix's control frames went through process_data before this test's sink
        # snapshot; compare the tail the stream delivery produced
        assert sink == exp[len(exp) - len(sink):], k


@pytest.mark.parametrize("seed", range(10))
def test_streams_match_process_data(torch, eng, hooks, seed):
    import uvhttp_amd as U
    rng = random.Random(9000 + seed)
    bad = seed % 2 == 1
    cases = [c for c in (_conn_case(rng, U, bad) for _ in range(rng.choice([1, 5, 40, 200]))) if c]
    _run_cases(torch, eng, U, cases, rng, 4096)


def test_streams_capacity_overflow(torch, eng):
    import uvhttp_amd as U
    frames = b"".join(_frame(2, 1, b"x", b"\x00\x00\x00\x01") for _ in range(50))
    s = U.Stream()
    s.begin, s.len, s.recv_buffer_size = 0, len(frames), 65536
    s.max_frame_size, s.max_message_size, s.is_server = 1 << 24, 1 << 26, 1
    dev_streams = torch.from_numpy(np.frombuffer(bytes(s), np.uint8).copy()).to("cuda")
    dw = torch.zeros(len(frames) + 64, dtype=torch.uint8, device="cuda")
    dw[: len(frames)] = torch.from_numpy(np.frombuffer(frames, np.uint8).copy()).to("cuda")
    before = dw.clone()
    desc, res = eng.decode_streams(dw, dev_streams, 1, 10, wire_len=len(frames))
    torch.cuda.synchronize()
    r = eng.read_stream_results(res, 1)[0]
    assert r.status == -1 and r.first_status == -10
    assert torch.equal(dw, before)


@pytest.mark.parametrize("seed", range(2))
def test_streams_many_small_frames(torch, eng, hooks, seed):
    """Connections with hundreds of frames: the wave walk crosses many 4 KiB blocks through
    its prefetch ring, and jumps over blocks on the larger frames."""
    import uvhttp_amd as U
    rng = random.Random(777 + seed)
    cases = []
    for _ in range(9):
        prod = U.WsConnection(1, 16 * 1024 * 1024, 64 * 1024 * 1024, user_data=True)
        orc = _oracle.OracleConn(1, 16 * 1024 * 1024, 64 * 1024 * 1024, record=1, wrapper=True)
        frames = []
        for _ in range(rng.randint(200, 1200)):
            payload = rng.randbytes(rng.choice([0, 1, 125, 126, 200, 260, 700, 4000, 9000]))
            frames.append(_frame(2, 1, payload, rng.randbytes(4), True, 0))
        new = b"".join(frames)
        if rng.random() < 0.5:
            new = new[: rng.randint(1, len(new))]
        cases.append((prod, orc, new))
    _run_cases(torch, eng, U, cases, rng, 16384)
