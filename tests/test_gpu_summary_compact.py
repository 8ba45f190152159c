"""Summary-only compact decode (uvhttp_ws_gpu_decode_compact with d_desc = NULL, include/
uvhttp_ws_amd.h).  A fixed-stride batch of frames of >= 140 wire bytes whose messages cannot
reach max_message_size and whose arena holds n * P bytes runs the speculative compact pass
writing one info byte per frame instead of a 16-byte record; k_sum_scan (fragment state machine,
speculation check, one summary part per block) and k_sum_msgs (message table; its block 0 the
summary and the last frame's message) finish it.  A batch that breaks the speculation — a delivered frame
that is not a data frame of the uniform length P: a reserved opcode, a non-minimal length, a
control or short last frame — is decoded again by k_plan + k_spec_fix, which return at once
otherwise.  Either way the summary, the message table, the arena up to arena_bytes and the wire
must equal the oracle's compact decode (process_data per frame, src/uvhttp_websocket.c:825-1097,
payloads appended per uvhttp_ws_fragment_append :781-822) and the descriptor path's.

Which way a call went is read off the device stamps: k_spec_fix (kind "fixup") runs only when
the speculation failed (or the summary-only path was not taken)."""
import random

import numpy as np
import pytest

import _oracle
from test_gpu_parity import GUARD, _frame, _guard_ok, _guarded, _to_dev

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
    fast.set_stamps(True)
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


def _uniform_p(stride):
    for h in (2, 4, 10):
        p = stride - h - 4
        if p >= 0 and _hs(p) == h:
            return p
    return None


def _batch(rng, n, stride, frag=0.3, tweak=None):
    """n masked data frames of exactly `stride` wire bytes each (the uniform P); tweak(i, frame,
    open_msg) may replace frame i"""
    p = _uniform_p(stride)
    frames, open_msg = [], False
    for i in range(n):
        op = 0 if open_msg else rng.choice([1, 2])
        fin = rng.random() > frag
        f = _frame(op, fin, rng.randbytes(p), rng.randbytes(4))
        open_msg = not fin
        if tweak:
            f, open_msg = tweak(i, f, open_msg)
        frames.append(f)
    return np.frombuffer(b"".join(frames), np.uint8).copy()


def _check(torch, engines, wire, n, stride, wl=None, mm=0, is_server=1, mf=MF, fast=None,
           cap=None):
    """both engines, summary-only compact, vs the oracle; fast: whether the speculation must
    have held on the fast engine (None: not checked)"""
    wl = wire.size if wl is None else wl
    # an arena short of the batch: the oracle copies the frames that fit whole, the device also
    # the part of the next one that fits (test_gpu_spec_compact::test_arena_smaller_than_the_batch)
    whole = cap // _uniform_p(stride) * _uniform_p(stride) if cap is not None else None
    cap = wire.size + 64 if cap is None else cap
    ref = _oracle.decode_batch(wire, n, stride=stride, wire_len=wl, max_frame_size=mf,
                               max_message_size=mm, is_server=is_server, compact=True,
                               arena_cap=cap)
    if callable(fast):
        fast = fast(ref)
    for k, e in enumerate(engines):
        d = _to_dev(torch, wire)
        arena_all, arena = _guarded(torch, cap)
        msgs_all, msgs = _guarded(torch, max(1, n) * e.MSG_BYTES)
        summ_all, summ = _guarded(torch, 64)
        if k == 0:
            e.read_stamps()  # (drop older calls)
        e.decode_compact(d, n, arena, stride=stride, wire_len=wl, max_frame_size=mf,
                         max_message_size=mm, is_server=is_server, msgs=msgs, summary=summ,
                         no_desc=True)
        torch.cuda.synchronize()
        s = e.read_summary(summ)
        assert s == ref["summary"], (k, s, ref["summary"])
        got = d[: wire.size].cpu().numpy()
        assert np.array_equal(got, ref["wire"]), np.nonzero(got != ref["wire"])[0][:8]
        assert _guard_ok(d, wire.size), "write past the wire"
        ab = s["arena_bytes"] if whole is None else min(whole, s["arena_bytes"])
        assert np.array_equal(arena[:ab].cpu().numpy(), ref["arena"][:ab])
        assert _guard_ok(arena_all, cap), "write past the arena"
        assert _guard_ok(msgs_all, max(1, n) * e.MSG_BYTES), "write past the messages"
        m = e.read_msgs(msgs, s["n_messages"])
        assert np.array_equal(m["arena_off"], ref["msg_off"]), k
        assert np.array_equal(m["len"], ref["msg_len"]), k
        assert np.array_equal(m["opcode"], ref["msg_opcode"]), k
        if k == 0 and fast is not None:
            kinds = {r[1] for r in e.read_stamps()}
            assert ("fixup" not in kinds) == fast, (fast, kinds)
    return ref


@pytest.mark.parametrize("stride", [140, 141, 200, 256, 264, 300, 1000, 1024, 2048, 2560])
def test_strides(torch, engines, stride):
    rng = random.Random(stride)
    n = max(3, min(20000, (3 << 20) // stride))
    for frag in (0.0, 0.3, 1.0):
        _check(torch, engines, _batch(rng, n, stride, frag=frag), n, stride, fast=True)
    wire = _batch(rng, n, stride)
    # trailing bytes after the last frame; the last frame cut short (INCOMPLETE)
    _check(torch, engines, np.concatenate([wire, np.frombuffer(rng.randbytes(37), np.uint8)]), n,
           stride, fast=True)
    _check(torch, engines, wire, n, stride, wl=wire.size - 1 - rng.randrange(min(stride - 1, 60)),
           fast=True)


def test_c4_shape(torch, engines):
    """the C4 layout (264-byte slots, 256-byte payloads), one fragmented message of all frames,
    and all-FIN messages: one message per frame"""
    rng = random.Random(4)
    n, stride = 65536, 264
    frames = [_frame(2 if i == 0 else 0, i == n - 1, rng.randbytes(256), rng.randbytes(4))
              for i in range(n)]
    wire = np.frombuffer(b"".join(frames), np.uint8).copy()
    r = _check(torch, engines, wire, n, stride, mm=256 << 20, fast=True)
    assert r["summary"]["n_messages"] == 1
    r = _check(torch, engines, _batch(rng, n, stride, frag=0.0), n, stride, fast=True)
    assert r["summary"]["n_messages"] == n


def _tweak(kind, at, p):
    def tw(i, f, o):
        if i != at:
            return f, o
        b = bytearray(f)
        if kind == "rsv":
            b[0] |= 0x40
        elif kind == "cont_without_start":
            b[0] = (b[0] & 0xF0) | 0
            return bytes(b), o
        elif kind == "data_inside_fragment":
            b[0] = (b[0] & 0xF0) | 2
        elif kind == "reserved_opcode":  # delivered, but not a data frame: off the speculation
            b[0] = (b[0] & 0xF0) | 3
        elif kind == "unmasked":
            b[1] &= 0x7F
        elif kind == "nonminimal":  # a 64-bit length form: P - 6 bytes of payload, delivered
            pay = bytes(p - 6)
            b = bytearray(_frame(0 if o else 2, 1, pay, bytes(4), len_form=64))
            return bytes(b), False
        return bytes(b), o
    return tw


# (kind, does the speculation hold on the fast engine)
KINDS = [("rsv", True), ("cont_without_start", True), ("data_inside_fragment", True),
         ("unmasked", True), ("reserved_opcode", False), ("nonminimal", False)]


@pytest.mark.parametrize("kind,holds", KINDS)
def test_failures_and_ways_out(torch, engines, kind, holds):
    rng = random.Random(kind)
    for stride, n in ((264, 30000), (1000, 5000)):
        p = _uniform_p(stride)
        for at in (0, 1, n // 2, n - 1):
            wire = _batch(rng, n, stride, frag=0.4, tweak=_tweak(kind, at, p))
            # a failing frame ends the batch where it stands; a frame off the speculation sends
            # the batch to the full decode only when it is delivered (before the first failure)
            _check(torch, engines, wire, n, stride,
                   fast=lambda r, at=at: holds or r["summary"]["n_delivered"] <= at)


def test_last_frame_off_the_layout(torch, engines):
    """a control frame (CLOSE sets state_closed) or a short data frame as the last frame: the
    full decode; the same frame not delivered (an earlier failure): the fast path"""
    rng = random.Random(11)
    stride, n = 300, 4000
    for op, payload, frag in ((8, b"\x03\xe8bye", 0.0), (9, b"ping", 0.5), (2, b"short", 0.0)):
        wire = _batch(rng, n - 1, stride, frag=frag)
        last = np.frombuffer(_frame(op, 1, payload, rng.randbytes(4)), np.uint8)
        w = np.concatenate([wire, last])
        r = _check(torch, engines, w, n, stride, fast=False)
        if r["summary"]["n_delivered"] == n:
            assert r["summary"]["state_closed"] == (1 if op == 8 else 0)
    wire = _batch(rng, n - 1, stride, frag=0.0, tweak=_tweak("rsv", 10, 0))
    last = np.frombuffer(_frame(8, 1, b"", rng.randbytes(4)), np.uint8)
    _check(torch, engines, np.concatenate([wire, last]), n, stride, fast=True)


def test_paths_not_taken(torch, engines):
    """a message limit that can bind, an arena smaller than n * P, a stride below 140: the
    descriptor paths with the engine's scratch, same results (no k_sum_msgs)"""
    rng = random.Random(14)
    stride, n = 264, 10000
    wire = _batch(rng, n, stride, frag=0.9)
    for mm in (256 * 10, 256 * n - 1):
        _check(torch, engines, wire, n, stride, mm=mm, fast=False)
    _check(torch, engines, wire, n, stride, mm=256 * n, fast=True)
    _check(torch, engines, wire, n, stride, cap=256 * n - 1, fast=False)
    wire = _batch(rng, 5000, 131, frag=0.3)
    _check(torch, engines, wire, 5000, 131, fast=False)


def test_repeated_calls_and_graph(torch, engines):
    """calls alternating between the fast path and the fall-back on one engine (the gate word is
    per call) and a captured graph replayed over bytes that take either way"""
    import uvhttp_amd as U
    e = engines[0]
    rng = random.Random(16)
    stride, n = 264, 50000
    p = _uniform_p(stride)
    wires = [_batch(rng, n, stride, frag=0.5, tweak=_tweak(k, at, p) if k else None)
             for k, at in ((None, 0), ("reserved_opcode", 777), (None, 0), ("rsv", 30000),
                           ("nonminimal", 49999))]
    for w in wires + wires[::-1]:
        _check(torch, (e,), w, n, stride)
    refs = [_oracle.decode_batch(w, n, stride=stride, max_message_size=0, compact=True,
                                 arena_cap=w.size + 64) for w in wires]
    # graph: one uncaptured call sizes the scratch the fall-back needs, then capture and replay
    d = _to_dev(torch, wires[0])
    arena = torch.zeros(wires[0].size + 64, dtype=torch.uint8, device="cuda")
    msgs = torch.zeros(n * e.MSG_BYTES, dtype=torch.uint8, device="cuda")
    summ = torch.zeros(64, dtype=torch.uint8, device="cuda")
    e.decode_compact(d, n, arena, stride=stride, max_message_size=0, wire_len=wires[0].size,
                     msgs=msgs, summary=summ, no_desc=True)
    torch.cuda.synchronize()
    cs = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cs):
        e.decode_compact(d, n, arena, stride=stride, max_message_size=0, wire_len=wires[0].size,
                         msgs=msgs, summary=summ, no_desc=True, stream=cs)
    for w, ref in zip(wires + wires, refs + refs):
        d[: w.size] = torch.from_numpy(w).to("cuda")
        g.replay()
        torch.cuda.synchronize()
        s = e.read_summary(summ)
        assert s == ref["summary"]
        assert np.array_equal(d[: w.size].cpu().numpy(), ref["wire"])
        ab = s["arena_bytes"]
        assert np.array_equal(arena[:ab].cpu().numpy(), ref["arena"][:ab])
        m = e.read_msgs(msgs, s["n_messages"])
        assert np.array_equal(m["arena_off"], ref["msg_off"])
        assert np.array_equal(m["len"], ref["msg_len"])
    assert GUARD and U


@pytest.mark.parametrize("n", [1, 2, 3])
def test_tiny_batches(torch, engines, n):
    """one to three frames: the last frame's part and message are block 0's alone (fragments
    open or closed, a failure at frame 0, a control or reserved-opcode last frame)"""
    rng = random.Random(100 + n)
    stride = 264
    p = _uniform_p(stride)
    for frag in (0.0, 1.0):
        _check(torch, engines, _batch(rng, n, stride, frag=frag), n, stride, fast=True)
    _check(torch, engines, _batch(rng, n, stride, tweak=_tweak("rsv", 0, p)), n, stride, fast=True)
    _check(torch, engines, _batch(rng, n, stride, tweak=_tweak("reserved_opcode", n - 1, p)), n, stride,
           fast=False)
    w = _batch(rng, n - 1, stride, frag=0.0) if n > 1 else np.zeros(0, np.uint8)
    last = np.frombuffer(_frame(9, 1, b"pi", rng.randbytes(4)), np.uint8)
    _check(torch, engines, np.concatenate([w, last]), n, stride, fast=False)
