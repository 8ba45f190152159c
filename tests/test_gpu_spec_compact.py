"""The speculative compact decode of fixed-stride batches (ws_gpu.hip run_decode):
the payload pass writes every locally uniform frame's payload to frame * P before the state
machine runs; k_plan checks that each delivered frame is where the pass put it and k_spec_fix
redoes the batch with the full scatter when one is not.  Both outcomes must equal the oracle's
compact decode (process_data per frame, payloads appended to an arena): statuses, summary,
message table, the wire (only control payloads unmasked there) and the arena up to arena_bytes.

Batches cover the fast path (uniform frames, failures part-way, fragmented messages over the
max_message_size limit, incomplete last frames) and every way out of it (control frames, a
non-minimal length encoding, a short last frame, unmasked frames, strides with no uniform
payload length)."""
import random
import zlib

import numpy as np
import pytest

from test_gpu_parity import _compare, _frame, _run_both

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def eng(torch):
    import uvhttp_amd as U
    e = U.GpuEngine(0)
    yield e
    e.close()


def _hs(p):
    return 2 if p < 126 else 4 if p < 65536 else 10


def _uniform_p(stride):
    for h in (2, 4, 10):
        p = stride - h - 4
        if p >= 0 and _hs(p) == h:
            return p
    return None


def _stride_batch(rng, n, stride, frag=0.3, tweak=None):
    """n masked data frames of exactly `stride` wire bytes each (uniform P); tweak(i, frames,
    open_msg) may replace frame i (it must keep `stride` bytes unless it is the last)."""
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


STRIDES = [64, 100, 131, 135, 136, 264, 1000, 2560]


@pytest.mark.parametrize("stride", STRIDES)
@pytest.mark.parametrize("seed", range(3))
def test_uniform_batches(torch, eng, stride, seed):
    rng = random.Random(stride * 10 + seed)
    n = rng.choice([1, 2, 63, 64, 65, 500, 5000])
    wire = _stride_batch(rng, n, stride)
    for mm in (0, 64 << 20, 3 * stride):  # unlimited, default, tight (ERR_MESSAGE part-way)
        ref, got = _run_both(torch, eng, wire, n, stride=stride, mm=mm, compact=True)
        _compare(ref, got, compact=True)


def _local_error(kind):
    def tweak(i, f, open_msg):
        if i != tweak.at:
            return f, open_msg
        b = bytearray(f)
        if kind == "rsv":
            b[0] |= 0x40
        elif kind == "cont_without_start":
            b[0] = (b[0] & 0xF0) | 0
            return bytes(b), open_msg
        elif kind == "data_inside_fragment":
            b[0] = (b[0] & 0xF0) | 2
        elif kind == "too_big_opcode":
            b[0] = (b[0] & 0xF0) | 3
        return bytes(b), open_msg
    return tweak


@pytest.mark.parametrize("kind", ["rsv", "cont_without_start", "data_inside_fragment",
                                  "too_big_opcode"])
@pytest.mark.parametrize("where", ["first", "middle", "last"])
def test_failures_part_way(torch, eng, kind, where):
    rng = random.Random(zlib.crc32(f"{kind}/{where}".encode()))
    n, stride = 3000, 264
    tw = _local_error(kind)
    tw.at = {"first": 0, "middle": 1777, "last": n - 1}[where]
    wire = _stride_batch(rng, n, stride, frag=0.5, tweak=tw)
    ref, got = _run_both(torch, eng, wire, n, stride=stride, mm=0, compact=True)
    _compare(ref, got, compact=True)


def test_out_of_speculation(torch, eng):
    """frames that do not sit at frame * P: a control frame, a non-minimal 16-bit length, a short
    last frame, an incomplete last frame — each sends the batch through the full scatter (or,
    for the incomplete frame, simply is not delivered); results equal the oracle's"""
    rng = random.Random(99)
    stride, n = 100, 700
    p = _uniform_p(stride)
    cases = {
        "ping": lambda i, f, o: (_frame(9, 1, rng.randbytes(p), rng.randbytes(4)), o) if i == 300 else (f, o),
        "close": lambda i, f, o: (_frame(8, 1, b"\x03\xe8" + rng.randbytes(p - 2), rng.randbytes(4)), o)
        if i == 10 else (f, o),
        "nonminimal": lambda i, f, o: (_frame(2 if not o else 0, 1, rng.randbytes(p - 2),
                                              rng.randbytes(4), len_form=16), False) if i == 450 else (f, o),
    }
    for name, tw in cases.items():
        wire = _stride_batch(rng, n, stride, frag=0.0, tweak=tw)
        assert wire.size == n * stride, name
        ref, got = _run_both(torch, eng, wire, n, stride=stride, mm=0, compact=True)
        _compare(ref, got, compact=True)
    # last frame shorter than the stride (delivered at a non-uniform length)
    wire = _stride_batch(rng, n - 1, stride, frag=0.0)
    last = np.frombuffer(_frame(2, 1, rng.randbytes(17), rng.randbytes(4)), np.uint8)
    wire2 = np.concatenate([wire, last])
    ref, got = _run_both(torch, eng, wire2, n, stride=stride, mm=0, compact=True)
    _compare(ref, got, compact=True)
    # last frame cut short (INCOMPLETE: not delivered, nothing of it in the arena)
    wire3 = _stride_batch(rng, n, stride, frag=0.0)[: n * stride - 37]
    ref, got = _run_both(torch, eng, wire3, n, stride=stride, mm=0, compact=True)
    _compare(ref, got, compact=True)


@pytest.mark.parametrize("stride", [132, 133, 6, 70000])
def test_no_uniform_length_or_large(torch, eng, stride):
    """strides with no uniform masked payload (132, 133) or outside the speculative range take
    the k_plan-first compact decode"""
    rng = random.Random(stride)
    if stride in (132, 133):
        p = stride - 8  # 16-bit length form (non-minimal)
        frames = [_frame(2, 1, rng.randbytes(p), rng.randbytes(4), len_form=16) for _ in range(300)]
    elif stride == 6:
        frames = [_frame(2, 1, b"", rng.randbytes(4)) for _ in range(1000)]
    else:
        frames = [_frame(2, 1, rng.randbytes(stride - 14), rng.randbytes(4)) for _ in range(20)]
    wire = np.frombuffer(b"".join(frames), np.uint8).copy()
    assert wire.size == len(frames) * stride
    ref, got = _run_both(torch, eng, wire, len(frames), stride=stride, mm=0, compact=True)
    _compare(ref, got, compact=True)


def test_client_unmasked_frames(torch):
    """is_server = 0 with unmasked frames: never uniform (P assumes the 4 key bytes), decoded by
    the full scatter; the oracle agrees"""
    import uvhttp_amd as U
    import _oracle
    rng = random.Random(5)
    stride = 264
    frames = [_frame(2, 1, rng.randbytes(stride - 4), masked=False, len_form=16) for _ in range(400)]
    wire = np.frombuffer(b"".join(frames), np.uint8).copy()
    n = len(frames)
    e = U.GpuEngine(0)
    try:
        ref = _oracle.decode_batch(wire, n, stride=stride, max_message_size=0, is_server=0,
                                   compact=True, arena_cap=wire.size + 64)
        dw = torch.from_numpy(wire.copy()).to("cuda")
        arena = torch.zeros(wire.size + 64, dtype=torch.uint8, device="cuda")
        desc, msgs, summ = e.decode_compact(dw, n, arena, stride=stride, max_message_size=0,
                                            is_server=0, wire_len=wire.size)
        torch.cuda.synchronize()
        s = e.read_summary(summ)
        assert s == ref["summary"]
        ab = s["arena_bytes"]
        assert np.array_equal(arena[:ab].cpu().numpy(), ref["arena"][:ab])
    finally:
        e.close()


def test_speculation_off_matches(torch, eng, monkeypatch):
    """UVHTTP_WS_SPEC=0 (k_plan-first compact decode) and the speculative decode agree"""
    import uvhttp_amd as U
    rng = random.Random(7)
    wire = _stride_batch(rng, 4096, 264, frag=0.4)
    monkeypatch.setenv("UVHTTP_WS_SPEC", "0")
    e0 = U.GpuEngine(0)
    monkeypatch.delenv("UVHTTP_WS_SPEC")
    try:
        for e in (e0, eng):
            ref, got = _run_both(torch, e, wire, 4096, stride=264, mm=5000, compact=True)
            _compare(ref, got, compact=True)
    finally:
        e0.close()


@pytest.mark.parametrize("stride", [64, 264, 1000])
def test_arena_smaller_than_the_batch(torch, eng, stride):
    """an arena that ends part-way through a uniform batch (caps that are not a
    multiple of 16 too).  The speculative pass clamps its writes at arena_cap: statuses, summary
    and messages equal the oracle's (which copies only the frames that fit), every frame that
    fits whole is in the arena, and nothing is written past arena_cap."""
    from test_gpu_parity import GUARD, _guard_ok, _guarded, _to_dev
    import _oracle
    rng = random.Random(stride)
    n = 2000
    p = _uniform_p(stride)
    wire = _stride_batch(rng, n, stride, frag=0.3)
    for cap in (p * n // 2 + 5, (p * n // 3) & ~15, p * 3 + 1, 17, p * n - 1):
        ref = _oracle.decode_batch(wire, n, stride=stride, max_message_size=0, compact=True,
                                   arena_cap=cap)
        dw = _to_dev(torch, wire)
        arena_all, arena = _guarded(torch, cap)
        desc, msgs, summ = eng.decode_compact(dw, n, arena, stride=stride, max_message_size=0,
                                              wire_len=wire.size)
        torch.cuda.synchronize()
        s = eng.read_summary(summ)
        assert s == ref["summary"], (cap, s, ref["summary"])
        assert np.array_equal(eng.read_desc(desc, n)["status"], ref["status"])
        assert np.array_equal(dw[: wire.size].cpu().numpy(), ref["wire"])
        m = eng.read_msgs(msgs, s["n_messages"])
        assert np.array_equal(m["arena_off"], ref["msg_off"]) and np.array_equal(m["len"], ref["msg_len"])
        whole = (cap // p) * p  # the frames that fit whole
        got = arena.cpu().numpy()
        assert np.array_equal(got[:whole], ref["arena"][:whole]), cap
        assert _guard_ok(arena_all, cap), f"write past arena_cap {cap}"
        assert GUARD == 0xA5
