"""Summary-only in-place decode (uvhttp_ws_gpu_decode_inplace with d_desc = NULL, include/
uvhttp_ws_amd.h).  Fixed-stride batches of frames of >= 140 wire bytes whose messages cannot reach
max_message_size decode in one payload pass (k_unmask_stride<..., SUM>: header parse, local
checks, the fragment state machine from the previous frame, speculative unmask, one summary part
per tile) plus k_sum_tail (summary; re-mask from the first failure on).  Every other batch takes
the descriptor paths with the engine's scratch.  Either way the summary and the wire must equal
the oracle's process_data per frame (src/uvhttp_websocket.c:825-1097) and the descriptor path's.

Cases: strides around the 16 KiB tile geometry (headers on and across tile ends, frames that
start exactly at a tile start, whose fragment check needs the previous tile's last frame),
fragmented messages, every failure kind at the first / middle / last frame (the speculative
unmask must be undone), a control frame as the last frame (CLOSE sets state_closed), mixed
length encodings in one stride (payload sums of unequal frames), client-side unmasked frames,
trailing bytes and a cut last frame, and the fall-backs (stride < 140, a message limit that can
bind, an offset table)."""
import random

import numpy as np
import pytest

import _oracle
from test_gpu_parity import GUARD, _frame, _guard_ok, _to_dev

pytestmark = pytest.mark.gpu
MF = 16 * 1024 * 1024


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
    fast = U.GpuEngine(0)
    os.environ["UVHTTP_WS_SUMMARY_FAST"] = "0"
    try:
        slow = U.GpuEngine(0)  # d_desc = NULL through the descriptor paths (scratch)
    finally:
        del os.environ["UVHTTP_WS_SUMMARY_FAST"]
    yield fast, slow
    fast.close()
    slow.close()


def _hs(p):
    return 2 if p < 126 else 4 if p < 65536 else 10


def _payload_for(stride, form=None, masked=True):
    """payload length that makes a frame of exactly `stride` wire bytes (len_form: 7/16/64)"""
    m = 4 if masked else 0
    for f, h in ((7, 2), (16, 4), (64, 10)):
        if form and f != form:
            continue
        p = stride - h - m
        if p >= 0 and (f != 7 or p < 126) and (f != 16 or p < 65536):
            if form or _hs(p) == h:
                return p, f
    raise ValueError(stride)


def _batch(rng, n, stride, frag=0.3, tweak=None, forms=None):
    frames, open_msg = [], False
    for i in range(n):
        form = rng.choice(forms) if forms else None
        p, f = _payload_for(stride, form)
        op = 0 if open_msg else rng.choice([1, 2])
        fin = rng.random() > frag
        fr = _frame(op, fin, rng.randbytes(p), rng.randbytes(4), len_form=f)
        open_msg = not fin
        if tweak:
            fr, open_msg = tweak(i, fr, open_msg)
        frames.append(fr)
    return np.frombuffer(b"".join(frames), np.uint8).copy()


def _check(torch, engines, wire, n, stride, wl=None, mm=0, is_server=1, mf=MF):
    """both engines, summary-only, vs the oracle; and the descriptor path's summary"""
    wl = wire.size if wl is None else wl
    ref = _oracle.decode_batch(wire, n, stride=stride, wire_len=wl, max_frame_size=mf,
                               max_message_size=mm, is_server=is_server)
    for e in engines:
        d = _to_dev(torch, wire)
        _, summ = e.decode_inplace(d, n, stride=stride, wire_len=wl, max_frame_size=mf,
                                   max_message_size=mm, is_server=is_server, no_desc=True)
        torch.cuda.synchronize()
        s = e.read_summary(summ)
        assert s == ref["summary"], (s, ref["summary"])
        got = d[: wire.size].cpu().numpy()
        assert np.array_equal(got, ref["wire"]), np.nonzero(got != ref["wire"])[0][:8]
        assert _guard_ok(d, wire.size), "write past the wire"
    return ref


@pytest.mark.parametrize("stride", [140, 141, 200, 256, 264, 300, 512, 1000, 1024, 2048, 2560])
def test_strides(torch, engines, stride):
    rng = random.Random(stride)
    n = max(3, min(20000, (3 << 20) // stride))
    wire = _batch(rng, n, stride)
    _check(torch, engines, wire, n, stride)
    # trailing bytes after the last frame; the last frame cut short (INCOMPLETE)
    _check(torch, engines, np.concatenate([wire, np.frombuffer(rng.randbytes(37), np.uint8)]), n, stride)
    _check(torch, engines, wire, n, stride, wl=wire.size - 1 - rng.randrange(min(stride - 1, 60)))
    # unfragmented and fully fragmented
    _check(torch, engines, _batch(rng, n, stride, frag=0.0), n, stride)
    r = _check(torch, engines, _batch(rng, n, stride, frag=1.0), n, stride)
    assert r["summary"]["pending_bytes"] > 0 or r["summary"]["n_delivered"] < n


def test_frames_on_tile_starts(torch, engines):
    """strides dividing the 16 KiB tile: a header sits exactly at every tile start, so the
    fragment check of a tile's first frame reads the previous tile's last frame"""
    rng = random.Random(5)
    for stride in (256, 512, 1024, 2048):
        n = 20000
        for frag in (0.0, 0.5, 1.0):
            _check(torch, engines, _batch(rng, n, stride, frag=frag), n, stride)
        # a CONT right after a FIN at a tile boundary (fails), and a start inside an open
        # message there (fails)
        per = 16384 // stride
        for k, kind in ((7 * per, "cont"), (9 * per, "start")):
            def tw(i, f, o, k=k, kind=kind):
                if i == k - 1:  # the frame before the boundary: FIN for "cont", open for "start"
                    b = bytearray(f)
                    b[0] = (b[0] & 0x7F) | (0x80 if kind == "cont" else 0)
                    return bytes(b), kind != "cont"
                if i == k:
                    b = bytearray(f)
                    b[0] = (b[0] & 0xF0) | (0 if kind == "cont" else 2)
                    return bytes(b), o
                return f, o
            r = _check(torch, engines, _batch(rng, n, stride, frag=0.0, tweak=tw), n, stride)
            assert r["summary"]["n_delivered"] == k and r["summary"]["first_status"] == -7


def _fail_tweak(kind, at, p):
    def tw(i, f, o):
        if i != at:
            return f, o
        b = bytearray(f)
        if kind == "rsv":
            b[0] |= 0x40
        elif kind == "cont_without_start":
            b[0] = (b[0] & 0xF0) | 0
            return bytes(b), o
        elif kind == "bad_opcode":
            b[0] = (b[0] & 0xF0) | 3
        elif kind == "unmasked":
            b[1] &= 0x7F
        elif kind == "layout":  # declares 3 bytes fewer than its slot holds
            if b[1] & 0x7F == 126:
                b[2:4] = (p - 3).to_bytes(2, "big")
            else:
                b[1] = (b[1] & 0x80) | (p - 3)
        elif kind == "msb":
            b = bytearray(_frame(2, 1, b"", bytes(4), len_form=64))
            b[2] = 0x80
            b += bytes(len(f) - len(b))
        return bytes(b), o
    return tw


@pytest.mark.parametrize("kind", ["rsv", "cont_without_start", "bad_opcode", "unmasked", "layout",
                                  "msb", "too_big"])
def test_failures_are_undone(torch, engines, kind):
    rng = random.Random(kind)
    for stride, n in ((264, 30000), (1000, 5000), (2560, 2000)):
        p, _ = _payload_for(stride)
        for at in (0, 1, n // 2, n // 2 + 1, n - 1):
            wire = _batch(rng, n, stride, frag=0.4, tweak=None if kind == "too_big" else
                          _fail_tweak(kind, at, p))
            mf = p - 1 if kind == "too_big" else MF  # every frame is too big: fails at 0
            r = _check(torch, engines, wire, n, stride, mf=mf)
            # (opcode 3 is delivered; a last frame shorter than its slot is too)
            if kind not in ("cont_without_start", "too_big", "bad_opcode") and \
                    not (kind == "layout" and at == n - 1):
                assert r["summary"]["n_delivered"] <= at
            if kind == "too_big":
                break


def test_reserved_opcodes_between_fragments(torch, engines):
    """opcodes 3-7 are delivered by the reference and leave the fragment state alone: runs of
    them inside and between messages, across tile ends, and one right before a frame whose
    check depends on the message they hide (a CONT after them, a start after them)"""
    rng = random.Random(17)
    for stride in (264, 1000):
        n = 20000
        p, f = _payload_for(stride)
        res = set()

        def tw(i, fr, o, runs={}):
            # runs of 1..90 reserved frames at random places; keep the message state
            if i in runs or (rng.random() < 0.01 and i > 0):
                ln = runs.get(i) or rng.randrange(1, 90)
                for k in range(ln):
                    runs[i + k] = ln - k
                return _frame(rng.choice([3, 4, 5, 6, 7]), rng.random() < 0.5, rng.randbytes(p),
                              rng.randbytes(4), len_form=f), o
            return fr, o
        for frag in (0.0, 0.5, 0.9):
            r = _check(torch, engines, _batch(rng, n, stride, frag=frag, tweak=tw), n, stride)
            res.add(r["summary"]["n_delivered"])
        # a wrong frame right after a run: CONT after a run that ended no message, start inside
        for bad in ("cont", "start"):
            k0 = 5000

            def tw2(i, fr, o, bad=bad):
                if i == k0 - 1:
                    b = bytearray(fr)
                    b[0] = (b[0] & 0x7F) | (0x80 if bad == "cont" else 0)
                    return bytes(b), bad != "cont"
                if k0 <= i < k0 + 70:
                    return _frame(3, 1, rng.randbytes(p), rng.randbytes(4), len_form=f), o
                if i == k0 + 70:
                    b = bytearray(fr)
                    b[0] = (b[0] & 0xF0) | (0 if bad == "cont" else 1)
                    return bytes(b), o
                return fr, o
            r = _check(torch, engines, _batch(rng, n, stride, frag=0.0, tweak=tw2), n, stride)
            assert r["summary"]["n_delivered"] == k0 + 70 and r["summary"]["first_status"] == -7


def test_last_frame_control(torch, engines):
    """the last frame may be a control frame (a slot longer than it): CLOSE sets state_closed,
    PING does not; a fragmented message stays open across it"""
    rng = random.Random(11)
    stride, n = 300, 4000
    for op, payload, frag in ((8, b"\x03\xe8bye", 0.0), (9, b"ping", 0.5), (8, b"", 1.0)):
        wire = _batch(rng, n - 1, stride, frag=frag)
        last = np.frombuffer(_frame(op, 1, payload, rng.randbytes(4)), np.uint8)
        w = np.concatenate([wire, last])
        r = _check(torch, engines, w, n, stride)
        assert r["summary"]["n_delivered"] == n
        assert r["summary"]["state_closed"] == (1 if op == 8 else 0)


def test_mixed_length_forms(torch, engines):
    """16- and 64-bit length forms (non-minimal, legal) in one stride: payloads differ by 6 B"""
    rng = random.Random(12)
    for stride in (300, 1000):
        n = 6000
        r = _check(torch, engines, _batch(rng, n, stride, frag=0.3, forms=[16, 64]), n, stride)
        assert r["summary"]["n_delivered"] == n


def test_client_side(torch, engines):
    """is_server = 0: unmasked frames are legal (nothing to XOR) beside masked ones"""
    rng = random.Random(13)
    stride, n = 264, 8000
    frames = []
    for i in range(n):
        if i % 3:
            p, f = _payload_for(stride, masked=False)
            frames.append(_frame(2, 1, rng.randbytes(p), None, False, len_form=f))
        else:
            p, f = _payload_for(stride)
            frames.append(_frame(2, 1, rng.randbytes(p), rng.randbytes(4), len_form=f))
    wire = np.frombuffer(b"".join(frames), np.uint8).copy()
    _check(torch, engines, wire, n, stride, is_server=0)


def test_message_limits(torch, engines):
    """max_message_size that can bind takes the descriptor path (ERR_MESSAGE part-way); one
    that cannot (>= the batch's largest possible message) stays on the one-pass decode"""
    rng = random.Random(14)
    stride, n = 264, 10000
    wire = _batch(rng, n, stride, frag=0.9)
    for mm in (256 * 10, 256 * 1000, 256 * n, 256 * n - 1, 0):
        _check(torch, engines, wire, n, stride, mm=mm)


def test_small_strides_and_offsets(torch, engines):
    """strides below 140 (a control frame could fill a slot) and offset tables: descriptor paths
    with the scratch, same results"""
    import uvhttp_amd as U
    rng = random.Random(15)
    for stride in (64, 100, 131, 139):
        n = 5000
        _check(torch, engines, _batch(rng, n, stride, frag=0.3), n, stride)
    # offset table (frames of any size)
    frames = [_frame(2, 1, rng.randbytes(rng.choice([0, 5, 300, 5000])), rng.randbytes(4)) for _ in range(500)]
    wire = np.frombuffer(b"".join(frames), np.uint8).copy()
    offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
    ref = _oracle.decode_batch(wire, 500, offsets=offs, max_message_size=0)
    e = engines[0]
    d = _to_dev(torch, wire)
    doff = torch.from_numpy(offs.astype(np.int64)).to("cuda")
    _, summ = e.decode_inplace(d, 500, offsets=doff, max_message_size=0, no_desc=True)
    torch.cuda.synchronize()
    assert e.read_summary(summ) == ref["summary"]
    assert np.array_equal(d[: wire.size].cpu().numpy(), ref["wire"])
    assert U.GpuError


def test_repeated_calls_and_graph(torch, engines):
    """back-to-back calls on one engine (tail counter reset, epoch tags) and a captured graph
    replayed over changing bytes: every call's summary is its own"""
    import uvhttp_amd as U
    e = engines[0]
    rng = random.Random(16)
    stride, n = 264, 50000
    wires = [_batch(rng, n, stride, frag=0.5, tweak=_fail_tweak("rsv", at, 0) if at else None)
             for at in (None, 777, None, 30000)]
    refs = [_oracle.decode_batch(w, n, stride=stride, max_message_size=0) for w in wires]
    for _ in range(2):
        for w, ref in zip(wires, refs):
            d = _to_dev(torch, w)
            _, summ = e.decode_inplace(d, n, stride=stride, max_message_size=0, no_desc=True)
            torch.cuda.synchronize()
            assert e.read_summary(summ) == ref["summary"]
            assert np.array_equal(d[: w.size].cpu().numpy(), ref["wire"])
    # graph: capture one call, replay over each wire copied into the captured buffer
    d = _to_dev(torch, wires[0])
    summ = torch.zeros(64, dtype=torch.uint8, device="cuda")
    e.reserve(n, d.numel())
    cs = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cs):
        e.decode_inplace(d, n, stride=stride, max_message_size=0, wire_len=wires[0].size,
                         summary=summ, no_desc=True, stream=cs)
    for w, ref in zip(wires + wires, refs + refs):
        d[: w.size] = torch.from_numpy(w).to("cuda")
        g.replay()
        torch.cuda.synchronize()
        assert e.read_summary(summ) == ref["summary"]
        assert np.array_equal(d[: w.size].cpu().numpy(), ref["wire"])
    assert GUARD and U


@pytest.mark.parametrize("n", [1, 2, 3])
def test_tiny_batches(torch, engines, n):
    """one to three frames: the last frame's part is the tail's alone"""
    rng = random.Random(200 + n)
    stride = 264
    p, _ = _payload_for(stride)
    for frag in (0.0, 1.0):
        _check(torch, engines, _batch(rng, n, stride, frag=frag), n, stride)
    for kind in ("rsv", "bad_opcode"):
        _check(torch, engines, _batch(rng, n, stride, tweak=_fail_tweak(kind, n - 1, p)), n, stride)
    w = _batch(rng, n - 1, stride, frag=0.0) if n > 1 else np.zeros(0, np.uint8)
    last = np.frombuffer(_frame(8, 1, b"\x03\xe8", rng.randbytes(4)), np.uint8)
    r = _check(torch, engines, np.concatenate([w, last]), n, stride)
    assert r["summary"]["state_closed"] == 1
