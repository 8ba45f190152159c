"""The fused stride path (ws_gpu.hip: k_unmask_stride -> k_plan on records -> k_fixup): the
payload pass parses the headers from the tile it loaded, unmasks speculatively, and k_fixup
re-masks everything from the first failure on.  Checked bit-exact against the oracle and
against the k_plan-first path (UVHTTP_WS_FUSED=0) on the same inputs:

* strides around the tile geometry (headers straddling a tile end, frames starting before
  the tile, 64-byte minimum, 64 KiB+ frames) under every payload tile shape;
* failures the speculative unmask must undo: state-machine failures (CONTINUATION with
  nothing open, data inside a fragment, message over the limit), header violations, a wrong-
  sized frame (LAYOUT), a cut last frame, client-side unmasked frames, trailing bytes;
* a look-back give-up (UVHTTP_WS_MAX_POLLS=0): nothing may stay unmasked.
"""
import os
import random

import numpy as np
import pytest

import _oracle
from test_gpu_parity import _frame

pytestmark = pytest.mark.gpu
MF, MM = 16 * 1024 * 1024, 64 * 1024 * 1024


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


@pytest.fixture(scope="module", params=["3pass", "lookback", "lookback256"])
def engines(torch, request):
    """the fused path (records scanned by reduce-then-scan, or by k_plan's look-back in
    1024- or 256-thread blocks) and the k_plan-first path; the fused path is forced for every
    frame size"""
    fused = _engine({"UVHTTP_WS_REC_SCAN": request.param[:8], "UVHTTP_WS_FUSED_MAX": str(1 << 40),
                     "UVHTTP_WS_PLAN_WIDE": "0" if request.param.endswith("256") else "1",
                     "UVHTTP_WS_DESC_EMIT": "0"})  # (k_desc_emit: test_gpu_desc_emit.py)
    plain = _engine({"UVHTTP_WS_FUSED": "0"})
    yield fused, plain
    fused.close()
    plain.close()


def _decode(torch, eng, wire, n, stride, wl, mf=MF, mm=MM, is_server=1):
    d = torch.from_numpy(np.concatenate([wire, np.full(64, 0xA5, np.uint8)])).to("cuda")
    desc, summ = eng.decode_inplace(d, n, stride=stride, wire_len=wl, max_frame_size=mf,
                                    max_message_size=mm, is_server=is_server)
    torch.cuda.synchronize()
    out = d.cpu().numpy()
    assert (out[wire.size:] == 0xA5).all(), "write past the wire"
    return dict(summary=eng.read_summary(summ), desc=eng.read_desc(desc, n), wire=out[:wire.size])


def _check_all(torch, engines, wire, n, stride, wl=None, **kw):
    wl = wire.size if wl is None else wl
    ref = _oracle.decode_batch(wire, n, stride=stride, wire_len=wl,
                               max_frame_size=kw.get("mf", MF), max_message_size=kw.get("mm", MM),
                               is_server=kw.get("is_server", 1))
    outs = [_decode(torch, e, wire, n, stride, wl, **kw) for e in engines]
    for got in outs:
        assert got["summary"] == ref["summary"], (got["summary"], ref["summary"])
        assert np.array_equal(got["desc"]["status"], ref["status"])
        assert np.array_equal(got["wire"], ref["wire"]), np.nonzero(got["wire"] != ref["wire"])[0][:8]
    # the two device paths agree on every descriptor field too
    assert np.array_equal(outs[0]["desc"], outs[1]["desc"])
    return ref


def _batch(rng, n, plen, kind="ok", where=0, masked=True):
    k = lambda: rng.randbytes(4)  # noqa: E731
    frames = [_frame(2, 1, rng.randbytes(plen), k(), masked) for _ in range(n)]
    mm = MM
    if kind == "cont":
        frames[where] = _frame(0, 1, rng.randbytes(plen), k(), masked)
    elif kind == "new_in_frag" and where > 0:
        frames[where - 1] = _frame(1, 0, rng.randbytes(plen), k(), masked)
    elif kind == "too_big":
        frames = [_frame(2 if i == 0 else 0, 0, rng.randbytes(plen), k(), masked) for i in range(n)]
        mm = plen * (where + 1) - 1 or 1
    elif kind == "rsv":
        frames[where] = _frame(2, 1, rng.randbytes(plen), k(), masked, rsv=4)
    elif kind == "unmasked":
        frames[where] = _frame(2, 1, rng.randbytes(plen), None, False) + bytes(4)
        frames[where] = frames[where][:len(frames[0])]
    return np.frombuffer(b"".join(frames), np.uint8).copy(), mm


@pytest.mark.parametrize("plen", [56, 57, 60, 120, 250, 258, 1000, 4090, 16370, 70000])
def test_strides_around_tiles(torch, engines, plen):
    """payloads chosen so strides (>= 64) put headers on and across tile boundaries"""
    rng = random.Random(plen)
    n = max(3, min(3000, (4 << 20) // (plen + 14)))
    wire, _ = _batch(rng, n, plen)
    stride = wire.size // n
    _check_all(torch, engines, wire, n, stride)
    # trailing bytes after the last frame, and the last frame cut short
    _check_all(torch, engines, np.concatenate([wire, np.frombuffer(rng.randbytes(37), np.uint8)]),
               n, stride)
    _check_all(torch, engines, wire, n, stride, wl=wire.size - 1 - rng.randrange(min(stride, 40)))


@pytest.mark.parametrize("shape", [(64, 1), (64, 2), (64, 4), (128, 1), (128, 2), (256, 1),
                                   (256, 2), (256, 4)])
def test_tile_shapes(torch, engines, shape):
    rng = random.Random(shape[0] * 10 + shape[1])
    for plen in (60, 200, 3000):
        wire, mm = _batch(rng, 700, plen, "cont", 350)
        stride = wire.size // 700
        fused, plain = engines
        fused.set_tile(*shape)
        try:
            _check_all(torch, engines, wire, 700, stride, mm=mm)
        finally:
            fused.set_tile(0, 0)


@pytest.mark.parametrize("kind", ["cont", "new_in_frag", "too_big", "rsv", "unmasked"])
def test_failures_are_undone(torch, engines, kind):
    """frames from the first failure on are unmasked speculatively by the payload pass and
    must end exactly as the oracle leaves them (masked)"""
    rng = random.Random(["cont", "new_in_frag", "too_big", "rsv", "unmasked"].index(kind))
    for plen, n in ((60, 2000), (250, 5000), (3000, 300), (70000, 20)):
        for where in (0, 1, n // 3, n - 1):
            wire, mm = _batch(rng, n, plen, kind, where)
            stride = wire.size // n
            ref = _check_all(torch, engines, wire, n, stride, mm=mm)
            if kind != "new_in_frag" or where > 0:
                assert ref["summary"]["status"] == -1


def test_layout_and_client_frames(torch, engines):
    rng = random.Random(3)
    n, plen = 4000, 200
    frames = [_frame(1, 1, rng.randbytes(plen), rng.randbytes(4)) for _ in range(n)]
    stride = len(frames[0])
    frames[1234] = _frame(1, 1, rng.randbytes(plen - 2), rng.randbytes(4)) + b"zz"  # LAYOUT
    wire = np.frombuffer(b"".join(frames), np.uint8).copy()
    _check_all(torch, engines, wire, n, stride)
    # client side: unmasked frames are legal (nothing to XOR; 4 more payload bytes keep the
    # stride), masked ones still unmask
    frames = [_frame(2, 1, rng.randbytes(plen + 4), None, False) if i % 3 else
              _frame(2, 1, rng.randbytes(plen), rng.randbytes(4)) for i in range(n)]
    assert {len(f) for f in frames} == {stride}
    wire = np.frombuffer(b"".join(frames), np.uint8).copy()
    _check_all(torch, engines, wire, n, stride, is_server=0)


def test_lookback_give_up_restores_everything(torch):
    """UVHTTP_WS_MAX_POLLS=0 with the look-back scan over the records (UVHTTP_WS_REC_SCAN=
    lookback; the default reduce-then-scan never waits): the scan gives up, first_bad = 0, and
    k_fixup re-masks every frame the payload pass had unmasked — the wire is byte-identical to
    the input"""
    import uvhttp_amd as U
    rng = random.Random(9)
    n, plen = 300000, 250  # k_plan runs many blocks
    wire, _ = _batch(rng, n, plen)
    stride = wire.size // n
    eng = _engine({"UVHTTP_WS_MAX_POLLS": "0", "UVHTTP_WS_REC_SCAN": "lookback", "UVHTTP_WS_DESC_EMIT": "0"})
    try:
        got = _decode(torch, eng, wire, n, stride, wire.size)
        s = got["summary"]
        assert s["status"] == -1 and s["first_status"] == -11 and s["n_delivered"] == 0, s
        assert (got["desc"]["status"] == 2).all()
        assert np.array_equal(got["wire"], wire)
        with pytest.raises(U.GpuError):
            eng.sync()
    finally:
        eng.close()
