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


@pytest.fixture(scope="module", params=["lane", "lane-twopass", "wave", "wave-norec", "wave-twopass",
                                        "wave-fuse", "wave-fuse-norec", "wave-spec"])
def eng(torch, request):
    """Every frame-discovery walk (a lane per connection, single pass or two walks; a wave per
    connection, single pass
    through the offset scratch — with the fast path's frame records or re-reading every header
    for the descriptors; in one launch (k_swalk_fused) or with the scan and k_stream_desc
    apart — or the two-walk fallback) must decode alike, and so must the default engine, whose
    speculative decode takes the calls of connections with several equal frames first (the walk
    variants run with it off, so that they see every call)."""
    import os
    import uvhttp_amd as U
    env = {"UVHTTP_WS_WALK": request.param.split("-")[0],
           "UVHTTP_WS_WALK_SINGLE": "0" if request.param.endswith("twopass") else "1",
           "UVHTTP_WS_WALK_REC": "0" if request.param.endswith("norec") else "1",
           "UVHTTP_WS_WALK_FUSE": "1" if "-fuse" in request.param else "0",
           "UVHTTP_WS_STREAM_SPEC": "1" if request.param.endswith("spec") else "0"}
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
    return prod, orc, _cut(rng, new)


def _cut(rng, data, sizes=(0, 1, 2, 3, 7, 100, 1000, 4096, 16384)):
    """Split `data` into the reads a libuv loop would deliver (zero-length reads included)."""
    reads, pos = [], 0
    while pos < len(data):
        n = rng.choice(sizes) if rng.random() < 0.8 else rng.randint(1, 20000)
        reads.append(data[pos:pos + n])
        pos += n
    if not reads or rng.random() < 0.1:
        reads.append(b"")
    return reads


def _run_cases(torch, eng, U, cases, rng, max_frames, use_reads=False, gaps=(0, 0, 16, 48)):
    """One device call over every (product conn, oracle conn, reads) case, then the reference
    semantics: deliver_stream on the product side vs the oracle's process_data called once per
    read until a call fails (on_websocket_read, src/uvhttp_connection.c:1128-1164).  With
    use_reads=False each case's reads are joined into ONE call (n_reads = 0).  The gaps between
    connections (rng.choice(gaps) bytes after 16-byte alignment) hold random bytes no kernel may
    touch."""
    # batch wire: each connection's buffered bytes + new reads, 16-B aligned starts, gaps
    chunks, streams, read_end, pos = [], [], [], 0
    for prod, orc, reads in cases:
        if not use_reads:
            reads[:] = [b"".join(reads)]
        st = prod.struct
        buffered = C.string_at(st.recv_buffer, st.recv_buffer_pos) if st.recv_buffer_pos else b""
        data = buffered + b"".join(reads)
        pos = (pos + 15) & ~15
        pos += rng.choice(gaps)
        s = U.Stream()
        U.lib().uvhttp_ws_stream_init(prod.ptr, pos, len(data), C.byref(s))
        if use_reads:
            s.first_read, s.n_reads = len(read_end), len(reads)
            e = len(buffered)
            for r in reads:
                e += len(r)
                read_end.append(e)
        streams.append(s)
        chunks.append((pos, data))
        pos += len(data)
    wire = np.random.default_rng(rng.getrandbits(32)).integers(0, 256, pos + 64, dtype=np.uint8)
    guard = wire[pos:].copy()  # bytes past wire_len: never written
    for p, d in chunks:
        wire[p:p + len(d)] = np.frombuffer(d, np.uint8)
    outside = np.ones(pos, bool)  # the gaps between connections
    for p, d in chunks:
        outside[p:p + len(d)] = False
    n = len(streams)
    sbytes = b"".join(bytes(s) for s in streams)
    dev_streams = torch.from_numpy(np.frombuffer(sbytes, np.uint8).copy()).to("cuda")
    dw = torch.from_numpy(wire.copy()).to("cuda")
    re_dev = None
    if use_reads:
        re_dev = torch.from_numpy(np.array(read_end or [0], np.uint64).view(np.int64)).to("cuda")
    desc_t = torch.full(((max_frames + 2) * 32,), 0xA5, dtype=torch.uint8, device="cuda")
    res_t = torch.full(((n + 1) * U.STREAM_RESULT_BYTES,), 0x5A, dtype=torch.uint8, device="cuda")
    desc, res = eng.decode_streams(dw, dev_streams, n, max_frames, wire_len=pos, desc=desc_t,
                                   results=res_t, read_end=re_dev, n_reads=len(read_end))
    torch.cuda.synchronize()
    eng.sync()
    results = eng.read_stream_results(res, n)
    host_wire = dw.cpu().numpy()
    host_desc = desc.cpu().numpy()
    # guard bytes: nothing past the wire, the desc array or the results array was written
    assert np.array_equal(host_wire[pos:], guard)
    assert np.array_equal(host_wire[:pos][outside], wire[:pos][outside])
    assert (host_desc[max_frames * 32:] == 0xA5).all()
    assert (res.cpu().numpy()[n * U.STREAM_RESULT_BYTES:] == 0x5A).all()
    hw = (C.c_uint8 * host_wire.size).from_buffer(host_wire)
    hd = (C.c_uint8 * host_desc.size).from_buffer(host_desc)
    L = _oracle.load()
    for k, (prod, orc, reads) in enumerate(cases):
        SINK.pop(C.addressof(prod.ptr.contents), None)
        rc = U.lib().uvhttp_ws_deliver_stream(prod.ptr, hw, hd, C.byref(streams[k]),
                                              C.byref(results[k]))
        orc_rc, calls = orc.process_reads(reads)
        info = (k, results[k].as_dict(), [len(r) for r in reads])
        assert rc == orc_rc, info
        assert results[k].calls == calls, info
        pev = [(t, a, p) for t, a, p in prod.events if t in ("message", "close")]
        oev = [(t, a, p if t == "message" else None) for t, a, p in orc.events()
               if t in ("message", "close")]
        assert pev == oev, info
        st = prod.struct
        assert st.recv_buffer_pos == L.oracle_conn_recv_pos(orc.c), info
        assert C.string_at(st.recv_buffer, st.recv_buffer_pos) == orc.recv_bytes(), info
        assert st.recv_buffer_size == orc.recv_size, info
        frag = st.fragmented_size if st.fragmented_message else 0
        assert frag == L.oracle_conn_frag_size(orc.c), info
        assert bool(st.fragmented_message) == orc.frag_pending, info
        assert st.fragmented_opcode == orc.frag_opcode, info
        assert (st.state == 3) == (orc.state == 3), info  # CLOSED after a CLOSE frame
        if rc == 0:
            assert results[k].pending_bytes == frag
        sink = SINK.get(C.addressof(prod.ptr.contents), [])
        exp = [(t, p) for t, a, p in orc.events() if t in ("pong", "close_echo")]
        # the prefix's control frames went through process_data before this test's sink
        # snapshot; compare the tail the stream delivery produced
        assert sink == exp[len(exp) - len(sink):], k
    return results


@pytest.mark.parametrize("seed", range(10))
def test_streams_match_process_data(torch, eng, hooks, seed):
    import uvhttp_amd as U
    rng = random.Random(9000 + seed)
    bad = seed % 2 == 1
    cases = [c for c in (_conn_case(rng, U, bad) for _ in range(rng.choice([1, 5, 40, 200]))) if c]
    _run_cases(torch, eng, U, cases, rng, 4096)


@pytest.mark.parametrize("seed", range(3))
def test_streams_tile_sized_gaps(torch, eng, hooks, seed):
    """Gaps between connections of up to several 16 KiB map tiles (random bytes that must stay
    as they are) and long undecoded tails: map tiles wholly between connections' frames stay
    unclaimed (k_stream_desc's claim rule), every connection still decodes as process_data."""
    import uvhttp_amd as U
    rng = random.Random(9500 + seed)
    cases = [c for c in (_conn_case(rng, U, seed == 1) for _ in range(rng.choice([20, 60]))) if c]
    _run_cases(torch, eng, U, cases, rng, 4096, gaps=(0, 16, 16384, 20000, 49152, 70000))


def _layout(U, cases, rng, gaps=(0, 16, 48)):
    """the wire and stream table of a one-call decode of `cases` (their reads joined)"""
    chunks, streams, pos = [], [], 0
    for prod, _orc, reads in cases:
        st = prod.struct
        buffered = C.string_at(st.recv_buffer, st.recv_buffer_pos) if st.recv_buffer_pos else b""
        data = buffered + b"".join(reads)
        pos = ((pos + 15) & ~15) + rng.choice(gaps)
        s = U.Stream()
        U.lib().uvhttp_ws_stream_init(prod.ptr, pos, len(data), C.byref(s))
        streams.append(s)
        chunks.append((pos, data))
        pos += len(data)
    wire = np.zeros(pos + 64, np.uint8)
    for p, d in chunks:
        wire[p:p + len(d)] = np.frombuffer(d, np.uint8)
    return wire, b"".join(bytes(s) for s in streams), len(streams), pos


@pytest.mark.parametrize("side", [False, True], ids=["default_stream", "nonblocking_stream"])
def test_streams_back_to_back_growth(torch, hooks, side):
    """A call issued while the previous one still runs, with more connections and a longer wire
    (the engine's stream scratch, slices and frame records grow under it — round 5's closing
    run crashed on this in the batcher): both decode exactly as each does alone on a fresh
    engine (wire, descriptors, results).  nonblocking_stream: the crash's own conditions — the
    calls on a torch side stream (non-blocking: the legacy null stream does not order it), issued
    back to back with no host sync, the scratch grown on that stream (ws_gpu.hip scratch_grow)."""
    import uvhttp_amd as U
    rng = random.Random(4242)
    calls = []
    for nconn in (3, 120, 400):
        cases = [c for c in (_conn_case(rng, U, False) for _ in range(nconn)) if c]
        calls.append(_layout(U, cases, rng))

    def inputs(k):
        wire, sb, n, wl = calls[k]
        dw = torch.from_numpy(wire.copy()).to("cuda")
        ds = torch.from_numpy(np.frombuffer(sb, np.uint8).copy()).to("cuda")
        return dw, ds

    def run(eng, k, dw, ds, stream=None):
        _, _, n, wl = calls[k]
        desc, res = eng.decode_streams(dw, ds, n, 16384, wire_len=wl, stream=stream)
        return dw, desc, res, ds

    eng = U.GpuEngine(0)
    ins = [inputs(k) for k in range(len(calls))]
    torch.cuda.synchronize()
    st = torch.cuda.Stream() if side else torch.cuda.current_stream()
    with torch.cuda.stream(st):
        outs = [run(eng, k, *ins[k], stream=st) for k in range(len(calls))]  # no sync between
    st.synchronize()
    torch.cuda.synchronize()
    eng.sync(st)
    for k, (dw, desc, res, _ds) in enumerate(outs):
        alone = U.GpuEngine(0)
        aw, adesc, ares, _ = run(alone, k, *inputs(k))
        torch.cuda.synchronize()
        alone.sync()
        n = calls[k][2]
        ra, rb = eng.read_stream_results(res, n), alone.read_stream_results(ares, n)
        assert [r.as_dict() for r in ra] == [r.as_dict() for r in rb], k
        assert torch.equal(dw, aw), k
        nf = max((r.first_frame + r.n_frames for r in ra), default=0)
        assert torch.equal(desc[:nf * 32], adesc[:nf * 32]), k
        alone.close()
    eng.close()


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
        cases.append((prod, orc, [new]))
    _run_cases(torch, eng, U, cases, rng, 16384)


def test_streams_runs_without_frames(torch, eng, hooks):
    """Long runs of connections holding no complete frame (a partial frame each, up to 40 KB:
    16 KiB map tiles start inside them) between connections with frames: the payload kernel's
    tile map must still lead to the next connection's frames (the wave path's k_stream_desc
    searches back past the run, 64 connections per step)."""
    import uvhttp_amd as U
    rng = random.Random(4040)
    cases = []
    for run in (70, 1, 200, 0, 65, 3):
        for _ in range(run):
            prod = U.WsConnection(1, 16 * 1024 * 1024, 64 * 1024 * 1024, user_data=True)
            orc = _oracle.OracleConn(1, 16 * 1024 * 1024, 64 * 1024 * 1024, record=1, wrapper=True)
            f = _frame(2, 1, rng.randbytes(rng.choice([300, 9000, 40000])), rng.randbytes(4))
            cases.append((prod, orc, [f[: rng.randint(1, len(f) - 1)]]))
        prod = U.WsConnection(1, 16 * 1024 * 1024, 64 * 1024 * 1024, user_data=True)
        orc = _oracle.OracleConn(1, 16 * 1024 * 1024, 64 * 1024 * 1024, record=1, wrapper=True)
        frames = [_frame(2, 1, rng.randbytes(rng.choice([1, 200, 5000, 20000])), rng.randbytes(4))
                  for _ in range(rng.randint(1, 40))]
        cases.append((prod, orc, [b"".join(frames)]))
    _run_cases(torch, eng, U, cases, rng, 8192)


@pytest.mark.parametrize("seed", range(10))
def test_streams_per_read_calls(torch, eng, hooks, seed):
    """Several process_data calls per connection in one launch: every connection's new bytes
    are cut into libuv-sized reads (zero-length reads too) and decoded with a read table;
    the oracle runs process_data once per read.  Growth, buffered bytes, fragment state and
    the call that failed must all agree."""
    import uvhttp_amd as U
    rng = random.Random(5100 + seed)
    bad = seed % 2 == 1
    cases = [c for c in (_conn_case(rng, U, bad) for _ in range(rng.choice([1, 7, 60, 250]))) if c]
    _run_cases(torch, eng, U, cases, rng, 8192, use_reads=True)


def test_streams_every_cut(torch, eng, hooks):
    """A connection's bytes cut at every point of the headers and around every frame boundary
    (7-, 16- and 64-bit lengths, masked, an empty frame, control frames): one connection per cut
    in one launch, as one call and as 1-byte-then-rest calls.  A read that ends inside an
    extended length (b0 b1 of a 126 / 127 header and nothing more) must only buffer."""
    import uvhttp_amd as U
    rng = random.Random(31)
    frames = [_frame(1, 1, rng.randbytes(126), rng.randbytes(4)),
              _frame(2, 0, b"", rng.randbytes(4)),
              _frame(0, 0, rng.randbytes(70000), rng.randbytes(4), len_form=64),
              _frame(9, 1, rng.randbytes(5), rng.randbytes(4)),
              _frame(0, 1, rng.randbytes(125), rng.randbytes(4)),
              _frame(2, 1, rng.randbytes(300), rng.randbytes(4))]
    data = b"".join(frames)
    cuts, at = set(), 0
    for f in frames:
        cuts.update(range(at, at + 16))
        cuts.update(range(at + len(f) - 3, at + len(f) + 1))
        at += len(f)
    cuts = sorted(c for c in cuts if 0 <= c <= len(data))
    for use_reads in (False, True):
        for mm in (64 * 1024 * 1024, 0):
            cases = []
            for c in cuts:
                prod = U.WsConnection(1, 16 * 1024 * 1024, mm, user_data=True)
                orc = _oracle.OracleConn(1, 16 * 1024 * 1024, mm, record=1, wrapper=True)
                cases.append((prod, orc, [data[:1], data[1:c]] if use_reads else [data[:c]]))
            _run_cases(torch, eng, U, cases, rng, 4096, use_reads=use_reads)


def test_streams_wire_ends_in_header(torch, eng, hooks):
    """The launch's wire ends inside a header (one connection, wire_len = its bytes): the
    walks' bounded block loads must still see every byte before wire_len (a range check at
    dword granularity once read a 2-byte wire 81 FE as zeros — an "unmasked" frame — and
    failed the connection; tests/test_batcher_group.py seed 2 found it)."""
    import uvhttp_amd as U
    rng = random.Random(32)
    heads = [_frame(1, 1, rng.randbytes(126), rng.randbytes(4)),
             _frame(2, 1, rng.randbytes(70000), rng.randbytes(4), len_form=64),
             _frame(2, 1, rng.randbytes(5), rng.randbytes(4))]
    for f in heads:
        for c in list(range(1, 19)) + [len(f) - 1, len(f)]:
            for use_reads in (False, True):
                prod = U.WsConnection(1, 16 * 1024 * 1024, 0, user_data=True)
                orc = _oracle.OracleConn(1, 16 * 1024 * 1024, 0, record=1, wrapper=True)
                reads = [f[:1], f[1:c]] if use_reads else [f[:c]]
                _run_cases(torch, eng, U, [(prod, orc, reads)], random.Random(0), 64,
                           use_reads=use_reads)


def _small_frames(rng, total, plen=256):
    out = []
    while sum(len(f) for f in out) < total:
        out.append(_frame(2, 1, rng.randbytes(plen), rng.randbytes(4), True, 0))
    return b"".join(out)


def test_reads_exceed_cap_only_when_joined(torch, eng, hooks):
    """max_frame_size 4000 with the default 64 KiB buffer: 80 KB of 262-byte frames fed as
    16 KiB reads is fine (every call holds < 64 KiB), the same bytes as one call fail the
    growth cap (:851-857).  Per-read decode must succeed exactly as the per-read oracle."""
    import uvhttp_amd as U
    rng = random.Random(77)
    data = _small_frames(rng, 80000)
    for use_reads in (True, False):
        prod = U.WsConnection(1, 4000, 64 * 1024 * 1024, user_data=True)
        orc = _oracle.OracleConn(1, 4000, 64 * 1024 * 1024, record=1, wrapper=True)
        reads = [data[i:i + 16384] for i in range(0, len(data), 16384)]
        res = _run_cases(torch, eng, U, [(prod, orc, reads)], rng, 4096, use_reads=use_reads)[0]
        if use_reads:
            assert res.status == 0 and res.n_delivered == len(data) // 264
            assert res.calls == len(reads)
        else:
            assert res.status == -1 and res.first_status == -6 and res.n_delivered == 0


def test_reads_growth_fails_midway(torch, eng, hooks):
    """A frame whose payload passes max_frame_size (100 000) but whose wire bytes (100 009)
    do not fit the capped buffer: the call in which the buffered bytes pass the cap fails
    with ERR_BUFFER, after the earlier calls delivered their frames."""
    import uvhttp_amd as U
    rng = random.Random(78)
    head = _small_frames(rng, 3000, 100)
    big = _frame(2, 1, rng.randbytes(99995), rng.randbytes(4), True, 0)
    data = head + big + _small_frames(rng, 40000, 100)  # reads after the failing call never run
    prod = U.WsConnection(1, 100000, 64 * 1024 * 1024, user_data=True)
    orc = _oracle.OracleConn(1, 100000, 64 * 1024 * 1024, record=1, wrapper=True)
    reads = [data[i:i + 16384] for i in range(0, len(data), 16384)]
    res = _run_cases(torch, eng, U, [(prod, orc, reads)], rng, 4096, use_reads=True)[0]
    assert res.status == -1 and res.first_status == -6
    assert 1 < res.calls < len(reads) and res.n_delivered > 0


def test_fragment_error_leaves_reference_bytes(torch, eng, hooks):
    """ERR_FRAGMENT / ERR_MESSAGE: the reference unmasks the failing frame in recv_buffer
    (:944) before the fragment checks reject it (:964-1000), and a rejected start still
    records its opcode.  recv_buffer bytes and fragment state must match byte for byte."""
    import uvhttp_amd as U
    rng = random.Random(79)
    key = b"\x11\x22\x33\x44"
    scenarios = [
        # data frame inside a fragmented message (ERR_FRAGMENT)
        [_frame(1, 0, b"abc", key), _frame(2, 1, b"interrupt!", key), _frame(2, 1, b"x", key)],
        # continuation with nothing open (ERR_FRAGMENT)
        [_frame(0, 1, b"orphan-cont", key), _frame(2, 1, b"tail", key)],
        # fragments over max_message_size (ERR_MESSAGE), start fits, continuation does not
        [_frame(2, 0, bytes(600), key), _frame(0, 1, rng.randbytes(700), key)],
        # a start alone over max_message_size: its opcode is recorded before the check fails
        [_frame(1, 0, rng.randbytes(1200), key), _frame(2, 1, b"after", key)],
    ]
    for use_reads in (False, True):
        cases = []
        for frames in scenarios:
            prod = U.WsConnection(1, 16 * 1024 * 1024, 1000, user_data=True)
            orc = _oracle.OracleConn(1, 16 * 1024 * 1024, 1000, record=1, wrapper=True)
            cases.append((prod, orc, [f for f in frames]))
        res = _run_cases(torch, eng, U, cases, rng, 64, use_reads=use_reads)
        assert [r.first_status for r in res] == [-7, -7, -8, -8]


def test_reads_layout_errors(torch, eng):
    """Malformed descriptors are API errors (ERR_LAYOUT): a decreasing read table, a last
    read that does not end at len, a read table out of range, a stream past the wire (also
    with begin near 2^64, which must not wrap the bounds test).  Nothing is decoded."""
    import uvhttp_amd as U
    frame = _frame(2, 1, b"hello", b"\x01\x02\x03\x04")
    L = len(frame)
    wire = torch.zeros(4 * 64 + 64, dtype=torch.uint8, device="cuda")
    for k in range(4):
        wire[k * 64:k * 64 + L] = torch.tensor(list(frame), dtype=torch.uint8)
    before = wire.clone()
    specs = [(0, L, 0, 2), (64, L, 2, 2), (128, L, 4, 5), (2**64 - 16, L, 0, 0)]
    read_end = [L, 3, 3, L - 1]
    st = np.zeros(4, U.STREAM_DT)
    for k, (b, ln, fr, nr) in enumerate(specs):
        st[k] = (b, ln, 65536, 0, 0, 1 << 24, 1 << 26, 1, fr, nr, 0)
    dev_st = torch.from_numpy(st.view(np.uint8).copy()).to("cuda")
    re_dev = torch.tensor(read_end, dtype=torch.int64, device="cuda")
    desc, res = eng.decode_streams(wire, dev_st, 4, 16, wire_len=4 * 64, read_end=re_dev,
                                   n_reads=len(read_end))
    torch.cuda.synchronize()
    rs = eng.read_stream_results(res, 4)
    assert [(r.status, r.first_status, r.n_delivered) for r in rs] == [(-1, -9, 0)] * 4
    assert torch.equal(wire, before)
