"""k_desc_emit (ws_gpu.hip): stride batches decoded in place WITH descriptors under the
summary-only bounds (stride >= 140, no message able to reach max_message_size) take the payload
pass leaving records + info bytes, the info-byte scan (k_sum_scan) and one fully parallel
descriptor pass — no k_plan look-back, no k_fixup.  Every descriptor field,
the summary and the wire must equal the oracle's batch decode (src/uvhttp_websocket.c:825-1097
per frame) and both other device paths: k_plan on the records (UVHTTP_WS_DESC_EMIT=0) and the
k_plan-first path (UVHTTP_WS_FUSED=0), including the descriptors of frames after a failure
(SKIPPED, no message id, no MSG_END on every path)."""
import random

import numpy as np
import pytest

import _oracle
from test_gpu_fused import _batch, _decode, _engine
from test_gpu_parity import _frame

pytestmark = pytest.mark.gpu
MF = 16 * 1024 * 1024


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module", params=["2", "1"])
def engines(torch, request):
    """k_desc_emit with info bytes from the payload pass (1) or rebuilt from the records (2),
    k_plan on the records, the k_plan-first path"""
    e = [_engine({"UVHTTP_WS_DESC_EMIT": request.param}), _engine({"UVHTTP_WS_DESC_EMIT": "0"}),
         _engine({"UVHTTP_WS_FUSED": "0"})]
    e[0].set_stamps(True)
    yield e
    for x in e:
        x.close()


FUSED_MAX = 2560  # (ws_gpu.hip kFusedMaxAvg: wire bytes per frame the fused stride path takes)


def _check(torch, engines, wire, n, stride, wl=None, mm=0, is_server=1, emit=None):
    wl = wire.size if wl is None else wl
    if emit is None:
        emit = wl // n <= FUSED_MAX
    ref = _oracle.decode_batch(wire, n, stride=stride, wire_len=wl, max_frame_size=MF,
                               max_message_size=mm, is_server=is_server)
    engines[0].read_stamps()
    outs = [_decode(torch, e, wire, n, stride, wl, mm=mm, is_server=is_server) for e in engines]
    kinds = {r[1] for r in engines[0].read_stamps()}
    assert ("desc_emit" in kinds) == emit, kinds
    for k, got in enumerate(outs):
        assert got["summary"] == ref["summary"], (k, got["summary"], ref["summary"])
        assert np.array_equal(got["desc"]["status"], ref["status"]), k
        assert np.array_equal(got["wire"], ref["wire"]), (k, np.nonzero(got["wire"] != ref["wire"])[0][:8])
    for k in range(1, len(outs)):
        diff = np.nonzero(outs[0]["desc"] != outs[k]["desc"])[0]
        assert diff.size == 0, (k, diff[:4], outs[0]["desc"][diff[:2]], outs[k]["desc"][diff[:2]])
    return ref


@pytest.mark.parametrize("plen", [132, 133, 200, 250, 258, 1000, 2000, 4090, 16370, 70000])
def test_strides(torch, engines, plen):
    rng = random.Random(plen)
    n = max(3, min(20000, (8 << 20) // (plen + 14)))
    wire, _ = _batch(rng, n, plen)
    stride = wire.size // n
    _check(torch, engines, wire, n, stride)
    _check(torch, engines, np.concatenate([wire, np.frombuffer(rng.randbytes(37), np.uint8)]), n, stride)
    _check(torch, engines, wire, n, stride, wl=wire.size - 1 - rng.randrange(min(stride, 40)))


def _frag_batch(rng, n, plen, p_frag, tweak=None):
    frames, open_msg = [], False
    for i in range(n):
        op = 0 if open_msg else rng.choice([1, 2])
        fin = rng.random() > p_frag
        f = _frame(op, fin, rng.randbytes(plen), rng.randbytes(4))
        if tweak:
            f, fin = tweak(i, f, fin, open_msg)
        open_msg = not fin
        frames.append(f)
    return np.frombuffer(b"".join(frames), np.uint8).copy()


@pytest.mark.parametrize("p_frag", [0.0, 0.3, 0.9, 1.0])
def test_fragmented_messages(torch, engines, p_frag):
    """message ids and MSG_END across scan blocks (1024 frames each): long fragmented runs"""
    rng = random.Random(int(p_frag * 10))
    for plen, n in ((256, 70000), (1000, 9000)):
        wire = _frag_batch(rng, n, plen, p_frag)
        _check(torch, engines, wire, n, len(wire) // n)


@pytest.mark.parametrize("kind", ["cont", "new_in_frag", "rsv", "unmasked", "reserved_op", "control_last",
                                  "ping_last_open"])
def test_failures_and_odd_frames(torch, engines, kind):
    """a failure at the first, a block-boundary, a middle and the last frame: statuses, the
    re-mask of everything the payload pass unmasked from it on, SKIPPED descriptors; reserved
    opcodes (delivered, no state change); a control frame as the last frame"""
    rng = random.Random(kind)
    for plen, n in ((256, 5000), (3000, 700)):
        for where in (0, 1, 1023, 1024, n // 2, n - 1):
            if kind in ("control_last", "ping_last_open") and where != n - 1:
                continue

            def tw(i, f, fin, open_msg, where=where):
                if i != where:
                    return f, fin
                b = bytearray(f)
                if kind == "cont":
                    b[0] = (b[0] & 0xF0) | (0 if not open_msg else 1)
                elif kind == "new_in_frag":
                    b[0] = (b[0] & 0xF0) | (2 if open_msg else 0)
                elif kind == "rsv":
                    b[0] |= 0x20
                elif kind == "unmasked":
                    b[1] &= 0x7F
                elif kind == "reserved_op":
                    b[0] = 0x80 | 3
                    return bytes(b), not open_msg  # (no state change: keep what was open)
                elif kind in ("control_last", "ping_last_open"):
                    return _frame(8 if kind == "control_last" else 9, 1, b"\x03\xe8", rng.randbytes(4)), True
                return bytes(b), fin
            wire = _frag_batch(rng, n, plen, 0.4 if kind != "ping_last_open" else 1.0, tw)
            stride = (2 if plen < 126 else 4) + 4 + plen  # (the uniform frames' size)
            _check(torch, engines, wire, n, stride)


def test_paths_not_taken(torch, engines):
    """a message limit that can bind, a stride below 140, client frames: the other paths"""
    rng = random.Random(5)
    wire = _frag_batch(rng, 5000, 256, 0.5)
    _check(torch, engines, wire, 5000, len(wire) // 5000, mm=256 * 100, emit=False)
    _check(torch, engines, wire, 5000, len(wire) // 5000, mm=256 * 5000)
    wire = _frag_batch(rng, 5000, 120, 0.5)
    _check(torch, engines, wire, 5000, len(wire) // 5000, emit=False)


def test_c4_full_size(torch, engines):
    """C4: 1 048 576 x 256-byte fragments of one message, every descriptor against the
    k_plan-on-records path, statuses and summary against the oracle; and C4 with a failure at
    frame 700 000 (re-mask of 348 576 frames)"""
    import uvhttp_amd as U
    n, plen = 1048576, 256
    stride = U.gen_frame_stride(plen)
    wl = stride * n
    ow, _ = _oracle.gen_frames(n, plen, 7, fragmented=True, opcode0=2)
    for bad in (None, 700000):
        w = ow.copy()
        if bad is not None:
            w[bad * stride] |= 0x40  # RSV1
        _check(torch, engines[:2], w, n, stride, mm=256 << 20)


@pytest.fixture(scope="module", params=["2", "1"])
def compact_engines(torch, request):
    """compact decodes with descriptors: k_sum_msgs writing them (info bytes rebuilt from the
    records, 2, or left by the pass, 1), the speculative pass + k_plan on records + k_spec_fix
    (UVHTTP_WS_DESC_EMIT=0), k_plan first + the scatter (UVHTTP_WS_SPEC=0)"""
    e = [_engine({"UVHTTP_WS_DESC_EMIT": request.param}), _engine({"UVHTTP_WS_DESC_EMIT": "0"}),
         _engine({"UVHTTP_WS_SPEC": "0"})]
    e[0].set_stamps(True)
    yield e
    for x in e:
        x.close()


def _compact_all(torch, engines, wire, n, stride, mm=0, fast=None):
    ref = _oracle.decode_batch(wire, n, stride=stride, max_frame_size=MF, max_message_size=mm,
                               compact=True, arena_cap=wire.size + 64)
    outs = []
    engines[0].read_stamps()
    for e in engines:
        d = torch.from_numpy(np.concatenate([wire, np.zeros(64, np.uint8)])).to("cuda")
        arena = torch.zeros(wire.size + 64, dtype=torch.uint8, device="cuda")
        desc, msgs, summ = e.decode_compact(d, n, arena, stride=stride, wire_len=wire.size,
                                            max_frame_size=MF, max_message_size=mm)
        torch.cuda.synchronize()
        s = e.read_summary(summ)
        outs.append(dict(s=s, desc=e.read_desc(desc, n), msgs=e.read_msgs(msgs, s["n_messages"]),
                         arena=arena[: s["arena_bytes"]].cpu().numpy(), wire=d[: wire.size].cpu().numpy()))
    kinds = {r[1] for r in engines[0].read_stamps()}
    if fast is not None:
        assert (("fixup" not in kinds) and ("sum_scan" in kinds)) == fast, kinds
    for k, o in enumerate(outs):
        assert o["s"] == ref["summary"], (k, o["s"], ref["summary"])
        assert np.array_equal(o["desc"]["status"], ref["status"]), k
        assert np.array_equal(o["wire"], ref["wire"]), k
        assert np.array_equal(o["arena"], ref["arena"][: o["s"]["arena_bytes"]]), k
        assert np.array_equal(o["msgs"]["arena_off"], ref["msg_off"]), k
        assert np.array_equal(o["msgs"]["len"], ref["msg_len"]), k
    for k in (1, 2):
        diff = np.nonzero(outs[0]["desc"] != outs[k]["desc"])[0]
        assert diff.size == 0, (k, diff[:4], outs[0]["desc"][diff[:2]], outs[k]["desc"][diff[:2]])
        assert np.array_equal(outs[0]["msgs"], outs[k]["msgs"]), k
    return ref


@pytest.mark.parametrize("plen", [132, 200, 256, 1000, 2000])
def test_compact_with_descriptors(torch, compact_engines, plen):
    """uniform batches (fast: the speculation holds), failures part-way (the frames after them
    keep their wire payload offsets on every path), a control frame last (the fall-back)"""
    rng = random.Random(plen + 1)
    n = max(3, min(20000, (4 << 20) // (plen + 8)))
    stride = (2 if plen < 126 else 4) + 4 + plen
    for p_frag in (0.0, 0.5, 1.0):
        _compact_all(torch, compact_engines, _frag_batch(rng, n, plen, p_frag), n, stride, fast=True)
    for where in (0, 1023, n // 2, n - 1):
        def tw(i, f, fin, open_msg, where=where):
            if i != where:
                return f, fin
            b = bytearray(f)
            b[0] |= 0x20  # RSV2
            return bytes(b), fin
        _compact_all(torch, compact_engines, _frag_batch(rng, n, plen, 0.4, tw), n, stride, fast=True)

    def ctl_last(i, f, fin, open_msg):
        return (_frame(9, 1, b"ping", rng.randbytes(4)), True) if i == n - 1 else (f, fin)
    _compact_all(torch, compact_engines, _frag_batch(rng, n, plen, 0.4, ctl_last), n, stride, fast=False)


def test_compact_c4_full_size(torch, compact_engines):
    """C4 compact with descriptors: one 256 MiB message of 1 048 576 fragments"""
    import uvhttp_amd as U
    n, plen = 1048576, 256
    stride = U.gen_frame_stride(plen)
    ow, _ = _oracle.gen_frames(n, plen, 7, fragmented=True, opcode0=2)
    _compact_all(torch, compact_engines[:2] + compact_engines[1:2], ow, n, stride, mm=256 << 20, fast=True)
