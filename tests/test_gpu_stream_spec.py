"""The speculative stream decode (ws_gpu.hip k_sspec_plan / k_sspec_pass / k_sspec_emit, VERDICT
r05 item 3): single-read connections whose frames all have their first frame's wire length are
decoded by the payload pass itself (headers parsed from the tile it loads), with no per-
connection walk over the headers.  Whatever the bytes, the result must equal the walk path's
(UVHTTP_WS_STREAM_SPEC=0) field for field — every result record, every descriptor, the wire — and
the oracle's (oracle_decode_streams: process_data per connection, src/uvhttp_websocket.c:825-1097).
Batches that break the speculation (a frame of another length, a failing frame, a fragment-
state failure, a complete frame of another size after the last speculated one, tiny frames,
several reads, too many frames) must come out the same through the fall-back: the pass's unmask
undone, then the walk.  Which way a call went is read off the device stamps ("walk" runs only in
the fall-back)."""
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


@pytest.fixture(scope="module")
def engines(torch):
    import os
    import uvhttp_amd as U
    spec = U.GpuEngine(0)
    spec.set_stamps(True)
    os.environ["UVHTTP_WS_STREAM_SPEC"] = "0"
    try:
        walk = U.GpuEngine(0)
    finally:
        del os.environ["UVHTTP_WS_STREAM_SPEC"]
    yield spec, walk
    spec.close()
    walk.close()


def _conn_frames(rng, n, plen, open_msg, p_frag=0.4, p_ctrl=0.0):
    """n frames of one wire length (payload plen, masked): data frames continuing / opening
    messages, control frames of the same size when plen <= 125"""
    out = []
    for _ in range(n):
        key = rng.randbytes(4)
        if p_ctrl and plen <= 125 and rng.random() < p_ctrl:
            out.append(_frame(rng.choice([9, 10]), 1, rng.randbytes(plen), key))
            continue
        if open_msg:
            op, fin = 0, rng.random() > p_frag
        else:
            op, fin = rng.choice([1, 2]), rng.random() > p_frag
        out.append(_frame(op, fin, rng.randbytes(plen), key))
        open_msg = not fin
    return out, open_msg


def _build(conns, gap=0, tail=None):
    """conns: [(frames bytes list, extra tail bytes, pending_bytes, pending_opcode, limits)] ->
    wire, STREAM_DT records"""
    st = np.zeros(len(conns), _oracle.STREAM_DT)
    parts, pos = [], 0
    for i, (frames, extra, pend, pop, mf, mm) in enumerate(conns):
        body = b"".join(frames) + extra
        st[i]["begin"] = pos
        st[i]["len"] = len(body)
        st[i]["recv_buffer_size"] = 65536
        st[i]["pending_bytes"] = pend
        st[i]["pending_opcode"] = pop
        st[i]["max_frame_size"] = mf
        st[i]["max_message_size"] = mm
        st[i]["is_server"] = 1
        g = gap(i) if callable(gap) else gap
        parts.append(body + bytes(g))
        pos += len(body) + g
    wire = np.frombuffer(b"".join(parts) + (tail or b""), np.uint8).copy()
    st.flags.writeable = True
    _build.frames = sum(len(c[0]) for c in conns)
    return wire, st


def _run(torch, engines, wire, st, max_frames=None, spec_expected=None, read_end=None):
    import uvhttp_amd as U
    n_st = st.size
    total_cap = max_frames or max(8 * n_st, _build.frames + n_st, 64)
    outs = []
    for k, e in enumerate(engines):
        d = torch.from_numpy(np.concatenate([wire, np.full(64, 0xA5, np.uint8)])).to("cuda")
        dev_st = torch.from_numpy(st.view(np.uint8).copy()).to("cuda")
        desc_t = torch.full(((total_cap + 1) * 32,), 0xA5, dtype=torch.uint8, device="cuda")
        if k == 0:
            e.read_stamps()
        re_dev = None if read_end is None else torch.from_numpy(read_end.view(np.int64).copy()).to("cuda")
        desc, res = e.decode_streams(d, dev_st, n_st, total_cap, desc=desc_t, wire_len=wire.size,
                                     read_end=re_dev, n_reads=0 if read_end is None else read_end.size)
        torch.cuda.synchronize()
        e.sync()
        kinds = {r[1] for r in e.read_stamps()} if k == 0 else set()
        r = res[: n_st * U.STREAM_RESULT_BYTES].cpu().numpy().view(U.STREAM_RESULT_DT).copy()
        nf = int(r["n_frames"].sum()) if (r["first_status"] != -10).all() else 0
        outs.append(dict(res=r, desc=e.read_desc(desc, max(nf, 1))[:nf].copy(),
                         wire=d[: wire.size].cpu().numpy(), kinds=kinds, nf=nf))
        assert (d[wire.size:].cpu().numpy() == 0xA5).all(), "write past the wire"
        assert (desc_t[(total_cap) * 32:] == 0xA5).all(), "write past the descriptors"
    a, b = outs
    if spec_expected is not None:
        assert ("walk" not in a["kinds"]) == spec_expected, a["kinds"]
    assert np.array_equal(a["res"], b["res"]), (a["res"][a["res"] != b["res"]][:3], b["res"][a["res"] != b["res"]][:3])
    assert np.array_equal(a["desc"], b["desc"]), np.nonzero(a["desc"] != b["desc"])[0][:5]
    assert np.array_equal(a["wire"], b["wire"]), np.nonzero(a["wire"] != b["wire"])[0][:8]
    # and the oracle
    host = wire.copy()
    out, frames, total = _oracle.decode_streams(host, st, read_end, max_frames=total_cap)
    r, o = a["res"], out
    if (r["first_status"] == -10).all():  # capacity: nothing decoded
        assert np.array_equal(a["wire"], wire)
        return a
    assert np.array_equal(r["n_delivered"], o["n_frames"])
    assert np.array_equal(r["status"], o["rc"]) and np.array_equal(r["first_status"], o["reason"])
    assert np.array_equal(r["calls"], o["calls"])
    assert np.array_equal(r["consumed_bytes"], o["consumed"])
    assert np.array_equal(r["recv_buffer_size"], o["recv_size"])
    assert np.array_equal(r["pending_bytes"], o["frag_size"])
    assert np.array_equal(r["buffered_end"], o["consumed"] + o["recv_pos"])
    assert np.array_equal(a["wire"], host)
    return a


@pytest.mark.parametrize("plen", [58, 60, 100, 125, 126, 250, 1000, 4090, 20000])
def test_uniform_connections(torch, engines, plen):
    """connections of equal frames (the speculation holds): various lengths, counts, open
    messages carried in and left open, partial frames left in the buffer, control frames"""
    rng = random.Random(plen)
    conns, open_msg = [], False
    for i in range(rng.randint(1, 40)):
        nfr = rng.choice([1, 2, 9, 63, 64, 65, 200])
        pend = rng.choice([0, 0, 77]) if not open_msg else 0
        om = open_msg or pend > 0
        frames, om2 = _conn_frames(rng, nfr, plen, om, p_ctrl=0.1)
        extra = rng.choice([b"", frames[0][:1], frames[0][:rng.randrange(2, 14)], frames[0][:-1]])
        conns.append((frames, extra, pend, 2 if pend else 0, 16 << 20, 0))
        open_msg = False
    wire, st = _build(conns, gap=lambda i: rng.choice([0, 0, 5, 1000]))
    _run(torch, engines, wire, st, spec_expected=True)


def test_many_connections_per_tile(torch, engines):
    """connections of a few 64-byte frames: up to 32 of them share a 16 KiB tile; more than 32
    send the call to the walk"""
    rng = random.Random(5)
    for per, n_conns, ok in ((10, 200, True), (5, 200, False), (2, 300, False)):
        conns = [(_conn_frames(rng, per, 58, False, p_frag=0.0)[0], b"", 0, 0, 16 << 20, 0)
                 for _ in range(n_conns)]
        wire, st = _build(conns)
        _run(torch, engines, wire, st, spec_expected=ok)


BREAKS = ["other_length", "rsv", "unmasked", "cont_without_start", "start_inside", "complete_other_tail",
          "small_frames", "first_bad", "too_big"]


@pytest.mark.parametrize("kind", BREAKS)
def test_breaks_fall_back_to_the_walk(torch, engines, kind):
    """a connection that breaks the speculation anywhere (first, middle, last connection; a frame
    at a tile boundary) — the pass's unmask is undone and the walk decodes the call"""
    rng = random.Random(kind)
    plen = 250
    for where_conn in (0, 7, 15):
        conns = []
        for i in range(16):
            frames, _ = _conn_frames(rng, 100, plen, False, p_frag=0.3)
            extra = b""
            if i == where_conn:
                at = rng.choice([0, 1, 62, 63, 99])
                if kind == "other_length":
                    frames[at] = _frame(2, 1, rng.randbytes(plen + 9), rng.randbytes(4))
                elif kind == "rsv":
                    frames[at] = _frame(2, 1, rng.randbytes(plen), rng.randbytes(4), rsv=2)
                elif kind == "unmasked":
                    frames[at] = _frame(2, 1, rng.randbytes(plen + 4), None, False)
                elif kind == "cont_without_start":
                    frames = [_frame(2, 1, rng.randbytes(plen), rng.randbytes(4)) for _ in range(100)]
                    frames[at] = _frame(0, 1, rng.randbytes(plen), rng.randbytes(4))
                elif kind == "start_inside":
                    frames = [_frame(2 if j == 0 else 0, 0, rng.randbytes(plen), rng.randbytes(4)) for j in range(100)]
                    frames[max(at, 1)] = _frame(1, 1, rng.randbytes(plen), rng.randbytes(4))
                elif kind == "complete_other_tail":
                    extra = _frame(2, 1, rng.randbytes(10), rng.randbytes(4))
                elif kind == "small_frames":
                    frames, _ = _conn_frames(rng, 100, 20, False, p_frag=0.0)
                elif kind == "first_bad":
                    frames[0] = _frame(2, 1, rng.randbytes(plen), rng.randbytes(4), rsv=4)
                elif kind == "too_big":
                    frames[at] = _frame(2, 1, rng.randbytes(plen), rng.randbytes(4))
            mf = 200 if (kind == "too_big" and i == where_conn) else 16 << 20
            conns.append((frames, extra, 0, 0, mf, 0))
        wire, st = _build(conns)
        _run(torch, engines, wire, st, spec_expected=False)


def test_limits_and_capacity(torch, engines):
    """a message limit that could bind, and a frame capacity below the frames: the walk"""
    rng = random.Random(9)
    conns = [(_conn_frames(rng, 50, 300, False, p_frag=0.0)[0], b"", 0, 0, 16 << 20, 0) for _ in range(8)]
    wire, st = _build(conns)
    _run(torch, engines, wire, st, spec_expected=True)
    st2 = st.copy()
    st2["max_message_size"][3] = 1000  # 50 frames of 300 bytes could exceed it
    _run(torch, engines, wire, st2, spec_expected=False)
    _run(torch, engines, wire, st, max_frames=399, spec_expected=False)  # (400 frames)


def test_repeated_calls_alternate_paths(torch, engines):
    """calls taking either path on one engine: no claim, gate or record of one call leaks into
    the next"""
    rng = random.Random(12)
    good = [(_conn_frames(rng, 80, 500, False)[0], b"", 0, 0, 16 << 20, 0) for _ in range(20)]
    bad = [list(c) for c in good]
    fr = list(bad[10][0])
    fr[40] = _frame(2, 1, rng.randbytes(100), rng.randbytes(4))
    bad[10][0] = fr
    for conns, ok in ((good, True), (bad, False), (good, True), (bad, False)):
        wire, st = _build([tuple(c) for c in conns])
        _run(torch, engines, wire, st, spec_expected=ok)


def _reads(rng, st, cuts, max_reads=None):
    """a read table per connection: cut points at random sizes from `cuts` (the last = len)"""
    re, first = [], 0
    for i in range(st.size):
        ln = int(st[i]["len"])
        ends, pos = [], 0
        while pos < ln:
            pos = min(ln, pos + rng.choice(cuts))
            ends.append(pos)
        if not ends:
            ends = [0]
        if max_reads and len(ends) > max_reads:
            ends = ends[:max_reads - 1] + [ln]
        st[i]["first_read"] = first
        st[i]["n_reads"] = len(ends)
        re += ends
        first += len(ends)
    return np.array(re, dtype=np.uint64)


@pytest.mark.parametrize("cuts", [[1 << 30], [16384], [1000, 7, 16384], [100, 65536]])
def test_read_tables(torch, engines, cuts):
    """connections fed several process_data calls (the batcher's live shape): the calls' growth
    checks (a 4 KiB starting buffer growing by doubling, a max_frame_size the growth can hit) and
    which call delivers a frame — the speculation holds unless a growth check fails"""
    rng = random.Random(str(cuts))
    conns = []
    for i in range(24):
        plen = rng.choice([250, 1000, 3000])
        frames, _ = _conn_frames(rng, rng.choice([8, 40, 100]), plen, False, p_frag=0.3)
        conns.append((frames, frames[0][:rng.randrange(0, 20)], 0, 0, rng.choice([16 << 20, 8192]), 0))
    wire, st = _build(conns)
    st["recv_buffer_size"] = 4096
    re = _reads(rng, st, cuts)
    # a growth check can fail only where max_frame_size (8 KiB) caps the buffer below what a
    # call holds: then the call goes to the walk
    _run(torch, engines, wire, st, read_end=re)
