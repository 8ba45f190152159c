"""GPU parity: the gfx950 batch decode (through the C-ABI) against the CPU oracle.

Every comparison is bit-exact: decoded wire bytes (in place), arena bytes (compact), per-frame
status, message table and batch summary.  Small randomized batches cover every error path of
src/uvhttp_websocket.c:825-1097; the BASELINE configs (C2 4 KiB, C3 64 KiB, C4 fragmented
256 B) run at full size with the oracle checking every frame.
"""
import random

import numpy as np
import pytest

import _oracle

pytestmark = pytest.mark.gpu

SEED = 0x5EED0001
MF, MM = 16 * 1024 * 1024, 64 * 1024 * 1024


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module", params=["gather", "scatter"])
def eng(torch, request):
    """Both compact-decode kernels (arena-driven gather, wire-driven scatter; the engine picks
    by average frame size) must produce the same arena; in-place runs are unaffected."""
    import os
    import uvhttp_amd as U
    old = os.environ.get("UVHTTP_WS_COMPACT")
    os.environ["UVHTTP_WS_COMPACT"] = request.param
    try:
        e = U.GpuEngine(0)
    finally:
        if old is None:
            os.environ.pop("UVHTTP_WS_COMPACT", None)
        else:
            os.environ["UVHTTP_WS_COMPACT"] = old
    yield e
    e.close()


def _frame(op, fin, payload, key=None, masked=True, rsv=0, len_form=None):
    n = len(payload)
    b0 = (0x80 if fin else 0) | (rsv << 4) | (op & 0xF)
    mb = 0x80 if masked else 0
    form = len_form or (7 if n < 126 else 16 if n < 65536 else 64)
    if form == 7:
        head = bytes([b0, mb | n])
    elif form == 16:
        head = bytes([b0, mb | 126, n >> 8, n & 0xFF])
    else:
        head = bytes([b0, mb | 127]) + n.to_bytes(8, "big")
    if not masked:
        return head + payload
    key = key if key is not None else bytes(4)
    body = (np.frombuffer(payload, np.uint8) ^ np.resize(np.frombuffer(key, np.uint8), n)).tobytes() if n else b""
    return head + key + body


def _rand_batch(rng, n, sizes, p_ctrl=0.1, p_frag=0.3, p_bad=0.0):
    frames = []
    open_msg = False
    for i in range(n):
        key = bytes(rng.getrandbits(8) for _ in range(4))
        r = rng.random()
        if r < p_ctrl:
            op = rng.choice([8, 9, 10])
            plen = rng.choice([0, 1, 2, 5, 125])
            fin = 1
        else:
            plen = rng.choice(sizes)
            if open_msg:
                op = 0
                fin = rng.random() < 0.4
            else:
                op = rng.choice([1, 2])
                fin = rng.random() > p_frag
            open_msg = not fin
        payload = rng.randbytes(plen) if hasattr(rng, "randbytes") else \
            bytes(rng.getrandbits(8) for _ in range(plen))
        rsv, masked = 0, True
        if p_bad and rng.random() < p_bad:
            kind = rng.choice(["rsv", "unmasked", "cont", "ctrl_big", "ctrl_nofin", "op3"])
            if kind == "rsv":
                rsv = 4
            elif kind == "unmasked":
                masked = False
            elif kind == "cont":
                op = 0
            elif kind == "ctrl_big":
                op, payload, fin = 9, bytes(126), 1
            elif kind == "ctrl_nofin":
                op, fin = 8, 0
            else:
                op = 3
        frames.append(_frame(op, fin, payload, key, masked, rsv))
    offs = np.zeros(len(frames), dtype=np.uint64)
    pos = 0
    for i, f in enumerate(frames):
        offs[i] = pos
        pos += len(f)
    wire = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    return wire, offs


GUARD = 0xA5  # fill of the bytes around every buffer a decode may not write


def _to_dev(torch, arr, pad=64):
    t = torch.full((arr.size + pad,), GUARD, dtype=torch.uint8, device="cuda")
    if arr.size:
        t[: arr.size] = torch.from_numpy(arr).to("cuda")
    return t


def _guarded(torch, nbytes, pad=256):
    """(whole, view): an output buffer of nbytes followed by `pad` guard bytes"""
    t = torch.full((nbytes + pad,), GUARD, dtype=torch.uint8, device="cuda")
    return t, t[:nbytes]


def _guard_ok(t, start):
    return bool((t[start:] == GUARD).all())


def _run_both(torch, eng, wire, n, offs=None, stride=None, mf=MF, mm=MM, compact=False,
              wire_len=None):
    import ctypes as C
    import uvhttp_amd as U
    wl = wire.size if wire_len is None else wire_len
    ref = _oracle.decode_batch(wire, n, stride=stride, offsets=offs, wire_len=wl,
                               max_frame_size=mf, max_message_size=mm, compact=compact,
                               arena_cap=wire.size + 64)
    dw = _to_dev(torch, wire)
    doff = torch.from_numpy(offs.astype(np.int64)).to("cuda") if offs is not None else None
    doff_before = doff.clone() if doff is not None else None
    # every output in a guarded buffer: descriptors / messages for n frames, the summary
    nd = max(1, n) * eng.DESC_BYTES
    desc_all, desc = _guarded(torch, nd)
    summ_all, summ = _guarded(torch, 64)
    if compact:
        arena_all, arena = _guarded(torch, wire.size + 64)
        msgs_all, msgs = _guarded(torch, max(1, n) * eng.MSG_BYTES)
        eng.decode_compact(dw, n, arena, stride=stride, offsets=doff, max_frame_size=mf,
                           max_message_size=mm, wire_len=wl, desc=desc, msgs=msgs, summary=summ)
    else:
        eng.decode_inplace(dw, n, stride=stride, offsets=doff, max_frame_size=mf,
                           max_message_size=mm, wire_len=wl, desc=desc, summary=summ)
    torch.cuda.synchronize()
    got = dict(summary=eng.read_summary(summ), desc=eng.read_desc(desc, n),
               wire=dw[: wire.size].cpu().numpy())
    # nothing written past the wire, the descriptors, the summary (or the arena / messages)
    assert _guard_ok(dw, wire.size), "write past the wire buffer"
    assert _guard_ok(desc_all, nd), "write past the descriptors"
    assert _guard_ok(summ_all, C.sizeof(U.BatchSummary)), "write past the summary"
    if doff is not None:
        assert torch.equal(doff, doff_before), "offset table modified"
    if compact:
        assert _guard_ok(msgs_all, max(1, n) * eng.MSG_BYTES), "write past the messages"
        a = arena.cpu().numpy()
        ab = got["summary"]["arena_bytes"]
        # past the delivered payload the arena is scratch for stride batches (the speculative
        # pass may have placed the frames after a failure there, include/uvhttp_ws_amd.h);
        # offset-table batches never write it
        if offs is not None:
            assert (a[ab:] == GUARD).all(), "arena written past the delivered payload"
        assert _guard_ok(arena_all, wire.size + 64)
        got["arena"] = a
        got["msgs"] = eng.read_msgs(msgs, got["summary"]["n_messages"])
    return ref, got


def _compare(ref, got, compact=False):
    rs, gs = ref["summary"], got["summary"]
    assert gs == rs, (gs, rs)
    assert np.array_equal(got["desc"]["status"], ref["status"]), \
        (np.nonzero(got["desc"]["status"] != ref["status"])[0][:10])
    assert np.array_equal(got["wire"], ref["wire"]), np.nonzero(got["wire"] != ref["wire"])[0][:10]
    if compact:
        nb = rs["arena_bytes"]
        assert np.array_equal(got["arena"][:nb], ref["arena"][:nb])
        m = got["msgs"]
        assert np.array_equal(m["arena_off"], ref["msg_off"])
        assert np.array_equal(m["len"], ref["msg_len"])
        assert np.array_equal(m["opcode"], ref["msg_opcode"])


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("seed", range(8))
def test_random_valid_batches(torch, eng, seed, compact):
    rng = random.Random(seed)
    sizes = [[0, 1, 3, 7, 16, 31, 125, 126, 200], [1000, 4096, 5000],
             [65535, 65536, 70000], [0, 2, 100, 4096, 65536]][seed % 4]
    n = rng.choice([1, 2, 17, 300, 1000])
    wire, offs = _rand_batch(rng, n, sizes, p_ctrl=0.15, p_frag=0.4)
    ref, got = _run_both(torch, eng, wire, n, offs=offs, mm=0, compact=compact)
    _compare(ref, got, compact)


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("seed", range(12))
def test_random_error_batches(torch, eng, seed, compact):
    rng = random.Random(1000 + seed)
    n = rng.choice([5, 50, 400])
    wire, offs = _rand_batch(rng, n, [0, 1, 5, 130, 3000, 70000], p_ctrl=0.2, p_frag=0.5,
                             p_bad=0.02)
    mf = rng.choice([MF, 65536, 3000])
    mm = rng.choice([MM, 5000, 0])
    ref, got = _run_both(torch, eng, wire, n, offs=offs, mf=mf, mm=mm, compact=compact)
    _compare(ref, got, compact)


@pytest.mark.parametrize("compact", [False, True])
def test_edge_cases(torch, eng, compact):
    k = bytes([1, 2, 3, 4])
    cases = []
    # zero-length first fragment does not open a message (fragmented_message stays NULL)
    cases.append([_frame(1, 0, b"", k), _frame(0, 1, b"abc", k)])
    cases.append([_frame(1, 0, b"", k), _frame(2, 1, b"abc", k)])
    # control frames inside a fragmented message; CLOSE keeps processing afterwards
    cases.append([_frame(1, 0, b"Hel", k), _frame(9, 1, b"p", k), _frame(0, 0, b"", k),
                  _frame(8, 1, b"\x03\xe8bye", k), _frame(0, 1, b"lo", k), _frame(2, 1, b"x", k)])
    # 64-bit length with MSB set
    cases.append([_frame(2, 1, b"ok", k), bytes([0x82, 0xFF] + [0x80] + [0] * 7) + k])
    # 16-bit form used for a tiny payload (legal, non-minimal encoding)
    cases.append([_frame(2, 1, b"tiny", k, len_form=16), _frame(1, 1, b"z" * 300, k, len_form=64)])
    # reserved opcodes are ignored; PONG ignored
    cases.append([_frame(3, 1, b"r", k), _frame(0xB, 1, b"", k), _frame(0xA, 1, b"q", k)])
    for frames in cases:
        wire = np.frombuffer(b"".join(frames), np.uint8).copy()
        offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
        ref, got = _run_both(torch, eng, wire, len(frames), offs=offs, compact=compact)
        _compare(ref, got, compact)


@pytest.mark.parametrize("compact", [False, True])
def test_incomplete_and_layout(torch, eng, compact):
    k = bytes([9, 8, 7, 6])
    frames = [_frame(2, 1, bytes(range(200)), k) for _ in range(5)]
    full = b"".join(frames)
    offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
    # last frame cut short at every possible length (header partial, key partial, payload)
    for cut in [1, 2, 3, 4, 5, 7, 8, 50, len(frames[-1]) - 1]:
        wl = len(full) - len(frames[-1]) + cut
        wire = np.frombuffer(full, np.uint8).copy()
        ref, got = _run_both(torch, eng, wire, 5, offs=offs, wire_len=wl, compact=compact)
        assert ref["summary"]["first_status"] == 1
        _compare(ref, got, compact)
    # offset table that disagrees with the frames
    bad = offs.copy()
    bad[2] += 3
    wire = np.frombuffer(full, np.uint8).copy()
    ref, got = _run_both(torch, eng, wire, 5, offs=bad, compact=compact)
    assert ref["summary"]["first_status"] == -9
    _compare(ref, got, compact)


@pytest.mark.parametrize("compact", [False, True])
def test_limits(torch, eng, compact):
    k = bytes([0xAA, 0xBB, 0xCC, 0xDD])
    # max_frame_size boundary and the 64 KiB receive-buffer cap
    for mf in [100, 65521, 65522, 65530, 65536, 70000]:
        frames = [_frame(2, 1, bytes(99), k), _frame(2, 1, bytes(100), k),
                  _frame(2, 1, bytes(101), k), _frame(2, 1, bytes(65522), k),
                  _frame(2, 1, bytes(65536), k)]
        wire = np.frombuffer(b"".join(frames), np.uint8).copy()
        offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
        for i in range(len(frames)):
            sub = frames[i:i + 1]
            w = np.frombuffer(b"".join(sub), np.uint8).copy()
            ref, got = _run_both(torch, eng, w, 1, offs=np.zeros(1, np.uint64), mf=mf,
                                 compact=compact)
            _compare(ref, got, compact)
        ref, got = _run_both(torch, eng, wire, len(frames), offs=offs, mf=mf, compact=compact)
        _compare(ref, got, compact)
    # max_message_size exactly reached / exceeded by the accumulated fragments
    for mm in [10, 11, 12]:
        frames = [_frame(1, 0, b"abcd", k), _frame(0, 0, b"efg", k), _frame(0, 1, b"hij", k)]
        wire = np.frombuffer(b"".join(frames), np.uint8).copy()
        offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
        ref, got = _run_both(torch, eng, wire, 3, offs=offs, mm=mm, compact=compact)
        _compare(ref, got, compact)


def test_empty_batch(torch, eng):
    wire = np.zeros(16, np.uint8)
    ref, got = _run_both(torch, eng, wire, 0, offs=np.zeros(0, np.uint64))
    assert got["summary"]["n_delivered"] == 0 and got["summary"]["status"] == 0
    _compare(ref, got)


def test_misaligned_wire_rejected(torch, eng):
    import uvhttp_amd as U
    buf = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    with pytest.raises(U.GpuError):
        eng.decode_inplace(buf[1:], 1, stride=100)


@pytest.mark.parametrize("plen", [0, 1, 125, 126, 256, 4096, 65535, 65536, 100000])
def test_generator_matches_oracle(torch, eng, plen):
    n = 33
    wire, stride = _oracle.gen_frames(n, plen, SEED, force_keys=True, fragmented=plen == 256)
    import uvhttp_amd as U
    assert U.gen_frame_stride(plen) == stride
    d = torch.zeros(stride * n + 16, dtype=torch.uint8, device="cuda")
    eng.gen_frames(d, n, plen, SEED, force_keys=True, fragmented=plen == 256)
    torch.cuda.synchronize()
    assert np.array_equal(d[: stride * n].cpu().numpy(), wire)


@pytest.mark.parametrize("plen", [0, 125, 256, 4096, 70000])
def test_generator_range_matches_oracle(torch, eng, plen):
    """frames [first, first + count) of a larger batch (bench.py's rank shards: rank r decodes
    frames lo.. of the whole C5 batch, bench.gen_plan) equal the oracle's same range — and
    the same frames of the whole batch generated at once"""
    import uvhttp_amd as U
    total, first, count = 101, 57, 44
    frag = plen == 256
    exp, stride = _oracle.gen_frames(total, plen, SEED, fragmented=frag, force_keys=True,
                                     first=first, count=count, total=total)
    whole, _ = _oracle.gen_frames(total, plen, SEED, fragmented=frag, force_keys=True)
    assert np.array_equal(exp, whole[first * stride:(first + count) * stride])
    d = torch.zeros(stride * count + 16, dtype=torch.uint8, device="cuda")
    eng.gen_frames(d, count, plen, SEED, fragmented=frag, force_keys=True, first=first,
                   count=count, total=total)
    torch.cuda.synchronize()
    assert np.array_equal(d[: stride * count].cpu().numpy(), exp)
    with pytest.raises(U.GpuError):
        eng.gen_frames(d, count, plen, SEED, first=first, count=count, total=first + count - 1)


@pytest.mark.parametrize("off", [0, 1, 3, 15])
def test_device_apply_mask(torch, eng, off):
    rng = np.random.default_rng(off)
    for n in [0, 1, 5, 16, 17, 1000, 65537]:
        host = rng.integers(0, 256, n + off, dtype=np.uint8)
        key = bytes(rng.integers(0, 256, 4, dtype=np.uint8))
        d = _to_dev(torch, host)
        eng.apply_mask(d, key, length=n, offset=off)
        torch.cuda.synchronize()
        exp = bytearray(host.tobytes())
        seg = _oracle.apply_mask(bytearray(exp[off:off + n]), key)
        exp[off:off + n] = seg
        assert bytes(d[: n + off].cpu().numpy().tobytes()) == bytes(exp)


def _full_config(torch, eng, n, plen, fragmented, compact, chunk=4096, no_desc=False):
    """Full-size BASELINE config: device-generated, device-decoded, every frame checked
    against the oracle's decode of the identical oracle-generated frames (no_desc: the
    summary-only decode, d_desc = NULL)."""
    import uvhttp_amd as U
    stride = U.gen_frame_stride(plen)
    wl = stride * n
    d = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
    eng.gen_frames(d, n, plen, SEED, opcode0=2, fragmented=fragmented, force_keys=True)
    mm = 256 * 1024 * 1024 if fragmented else MM
    if compact:
        arena = torch.empty(n * plen + 64, dtype=torch.uint8, device="cuda")
        desc, msgs, summ = eng.decode_compact(d, n, arena, stride=stride, max_message_size=mm,
                                              wire_len=wl, no_desc=no_desc)
    else:
        desc, summ = eng.decode_inplace(d, n, stride=stride, max_message_size=mm, wire_len=wl,
                                        no_desc=no_desc)
    torch.cuda.synchronize()
    s = eng.read_summary(summ)
    assert s["n_delivered"] == n and s["status"] == 0
    assert s["payload_bytes"] == n * plen and s["consumed_bytes"] == wl
    assert s["n_messages"] == (1 if fragmented else n) and s["pending_bytes"] == 0
    if not no_desc:
        st = eng.read_desc(desc, n)["status"]
        assert not st.any()
    hs = stride - 4 - plen
    for first in range(0, n, chunk):
        cnt = min(chunk, n - first)
        ow, _ = _oracle.gen_frames(n, plen, SEED, fragmented=fragmented, force_keys=True,
                                   first=first, count=cnt, total=n)
        # oracle decode of this chunk (frame by frame; the fragment state machine is
        # checked by the summary above and by the small fragmented batches)
        _oracle.load().oracle_unmask_frames(_oracle._ptr(ow), cnt, stride)
        if compact:
            got = arena[first * plen:(first + cnt) * plen].cpu().numpy()
            exp = ow.reshape(cnt, stride)[:, hs + 4:].reshape(-1)
        else:
            got = d[first * stride:(first + cnt) * stride].cpu().numpy()
            exp = ow
        assert np.array_equal(got, exp), first
    if compact:
        m = eng.read_msgs(msgs, s["n_messages"])
        assert int(m["len"].sum()) == n * plen


@pytest.mark.parametrize("compact", [False, True])
def test_config_c2_full(torch, eng, compact):
    _full_config(torch, eng, 65536, 4096, False, compact)


@pytest.mark.parametrize("compact", [False, True])
def test_config_c3_full(torch, eng, compact):
    _full_config(torch, eng, 65536, 65536, False, compact, chunk=1024)


@pytest.mark.parametrize("compact", [False, True])
def test_config_c4_full(torch, eng, compact):
    _full_config(torch, eng, 1048576, 256, True, compact, chunk=131072)


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("cfg", ["c2", "c4"])
def test_config_full_summary_only(torch, eng, cfg, compact):
    """d_desc = NULL at full size: C4 takes the summary-only decode (in place: one payload pass
    + scan + tail; compact: the speculative pass + scan + tail + message table), C2 (4 KiB
    frames, above the fused range) the descriptor paths with the engine's scratch"""
    if cfg == "c4":
        _full_config(torch, eng, 1048576, 256, True, compact, chunk=131072, no_desc=True)
    else:
        _full_config(torch, eng, 65536, 4096, False, compact, no_desc=True)


def test_config_c4_default_limit_rejects(torch, eng):
    """With the default 64 MiB max_message_size the reference rejects C4 at frame 262 144
    (SURVEY §0); the device path reports the same frame and reason."""
    import uvhttp_amd as U
    n, plen = 1048576, 256
    stride = U.gen_frame_stride(plen)
    d = torch.empty(stride * n + 64, dtype=torch.uint8, device="cuda")
    eng.gen_frames(d, n, plen, SEED, opcode0=2, fragmented=True)
    desc, summ = eng.decode_inplace(d, n, stride=stride, max_message_size=MM,
                                    wire_len=stride * n)
    torch.cuda.synchronize()
    s = eng.read_summary(summ)
    assert s["n_delivered"] == 262144 and s["first_status"] == -8 and s["status"] == -1
    assert s["pending_bytes"] == 262144 * 256
    # summary-only (the limit can bind, so not the one-pass decode): the same summary, and the
    # wire as before (the second decode delivers nothing new: it re-masks nothing it did not
    # unmask, so run it on a fresh copy)
    d2 = torch.empty(stride * n + 64, dtype=torch.uint8, device="cuda")
    eng.gen_frames(d2, n, plen, SEED, opcode0=2, fragmented=True)
    _, summ2 = eng.decode_inplace(d2, n, stride=stride, max_message_size=MM, wire_len=stride * n,
                                  no_desc=True)
    torch.cuda.synchronize()
    assert eng.read_summary(summ2) == s
    assert torch.equal(d2[: stride * n], d[: stride * n])
    del d2
    # frames before the rejected one unmasked, it and every later frame left masked
    for i in (0, 262143, 262144, 262145, n - 1):
        got = d[i * stride:(i + 1) * stride].cpu().numpy()
        ow, _ = _oracle.gen_frames(n, plen, SEED, fragmented=True, first=i, count=1, total=n)
        if i < 262144:
            _oracle.load().oracle_unmask_frames(_oracle._ptr(ow), 1, stride)
        assert np.array_equal(got, ow), i


@pytest.mark.parametrize("shape", [(64, 1), (64, 2), (64, 4), (128, 1), (128, 2), (256, 1),
                                   (256, 2), (256, 4)])
def test_tile_shapes_identical(torch, eng, shape):
    """Every payload-kernel workgroup shape gives the oracle's bytes (tuning knob only)."""
    rng = random.Random(77)
    eng.set_tile(*shape)
    try:
        for sizes in ([0, 3, 17, 126, 300], [5000, 65536, 70000]):
            wire, offs = _rand_batch(rng, 200, sizes, p_ctrl=0.1, p_frag=0.4)
            for compact in (False, True):
                ref, got = _run_both(torch, eng, wire, 200, offs=offs, mm=0, compact=compact)
                _compare(ref, got, compact)
    finally:
        eng.set_tile(0, 0)


@pytest.mark.parametrize("depth", [3, 5, 8])
def test_pipeline_and_delivery(torch, eng, depth):
    """Host-memory pipeline: batches written into pinned slots, decoded on the device with
    overlapped copies, delivered to a connection; bytes, statuses, summaries and the callback
    transcript equal the oracle's per-frame process_data.  Depths above 3 keep three
    submissions in flight (submit waits for the one three back)."""
    import uvhttp_amd as U
    pipe = U.GpuPipeline(0, depth=depth, slot_bytes=4 << 20, slot_frames=4096)
    rng = random.Random(4242)
    batches = []
    for b in range(7 + depth):
        sizes = [[0, 5, 125, 126, 1000], [4096, 20000], [65536, 70000]][b % 3]
        n = rng.choice([1, 40, 300]) if b % 3 == 0 else rng.choice([1, 20, 50])
        wire, offs = _rand_batch(rng, n, sizes, p_ctrl=0.1, p_frag=0.3,
                                 p_bad=0.01 if b == 5 else 0.0)
        assert wire.size <= (4 << 20)
        batches.append((wire, offs))
    inflight = {}
    for k, (wire, offs) in enumerate(batches):
        slot = k % depth
        if slot in inflight:
            _check_slot(pipe, *inflight.pop(slot))
        buf = pipe.buffer(slot)
        buf[: wire.size] = wire
        pipe.offsets(slot)[: offs.size] = offs
        pipe.submit(slot, wire.size, offs.size, use_offsets=True, max_message_size=0)
        inflight[slot] = (slot, wire, offs)
    for v in inflight.values():
        _check_slot(pipe, *v)
    pipe.close()


def _check_slot(pipe, slot, wire, offs):
    import uvhttp_amd as U
    dp, sp, summ = pipe.wait(slot)
    n = offs.size
    ref = _oracle.decode_batch(wire, n, offsets=offs, max_message_size=0)
    assert summ == ref["summary"]
    if n:
        assert np.array_equal(pipe.desc_array(dp, n)["status"], ref["status"])
    assert np.array_equal(pipe.buffer(slot)[: wire.size], ref["wire"])
    # delivery transcript vs the oracle fed the same frames one by one
    conn = U.WsConnection(1, max_message_size=0)
    rc = pipe.deliver(conn, slot, dp, sp)
    oc = _oracle.OracleConn(1, max_message_size=0, record=1)
    orc_rc = 0
    for i in range(summ["n_delivered"]):
        end = offs[i + 1] if i + 1 < n else wire.size
        assert oc.process_data(wire[offs[i]:end].tobytes()) == 0
    if summ["status"]:
        orc_rc = -1
    assert rc == orc_rc
    got = [(k, a, p) for k, a, p in conn.events if k in ("message", "close")]
    exp = [(k, a, p if k == "message" else None) for k, a, p in oc.events() if k in ("message", "close")]
    assert got == exp


def test_config_c5_chunk(torch, eng):
    """One C5 pass: 1 048 576 x 64 KiB frames (68.7 GB of wire, > 2^32 work-items of payload
    tiles; each rank's pass at N = 8).  Summary and statuses exact; sampled frames checked byte
    for byte against the oracle here, and EVERY byte of the decoded wire through the sha256 of
    each 4096-frame chunk, against the oracle's digests committed in
    tests/golden/config_digests.json (tests/golden/make_config_digests.py)."""
    import uvhttp_amd as U
    n, plen = 1048576, 65536
    stride = U.gen_frame_stride(plen)
    wl = stride * n
    d = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
    eng.gen_frames(d, n, plen, SEED, opcode0=2, force_keys=True)
    desc, summ = eng.decode_inplace(d, n, stride=stride, wire_len=wl)
    torch.cuda.synchronize()
    s = eng.read_summary(summ)
    assert s["n_delivered"] == n and s["status"] == 0 and s["payload_bytes"] == n * plen
    assert s["consumed_bytes"] == wl and s["n_messages"] == n
    assert not eng.read_desc(desc, n)["status"].any()
    for i in list(range(0, n, 4099)) + [n - 1]:
        got = d[i * stride:(i + 1) * stride].cpu().numpy()
        ow, _ = _oracle.gen_frames(n, plen, SEED, force_keys=True, first=i, count=1, total=n)
        _oracle.load().oracle_unmask_frames(_oracle._ptr(ow), 1, stride)
        assert np.array_equal(got, ow), i
    import hashlib
    import json
    import os
    from concurrent.futures import ThreadPoolExecutor
    with open(os.path.join(os.path.dirname(__file__), "golden", "config_digests.json")) as fh:
        c5 = json.load(fh)["c5_pass"]
    cf = c5["chunk_frames"]
    assert c5["frames"] == n and len(c5["decoded_chunks"]) * cf == n

    def chunk_digest(k):  # (the copy and sha256 run outside the GIL)
        return hashlib.sha256(d[k * cf * stride:(k + 1) * cf * stride].cpu().numpy()).hexdigest()
    with ThreadPoolExecutor(8) as ex:
        got = list(ex.map(chunk_digest, range(n // cf)))
    bad = [k for k, (g, w) in enumerate(zip(got, c5["decoded_chunks"])) if g != w]
    assert not bad, f"decoded chunks differ from the oracle's: {bad[:8]}"
    assert hashlib.sha256("".join(got).encode()).hexdigest() == c5["decoded"]
    del d
    torch.cuda.empty_cache()


@pytest.mark.parametrize("fpt", [1, 2, 4, 8, 16])
def test_plan_frames_per_lane_identical(torch, fpt, monkeypatch):
    """k_plan's frames-per-lane variants (and multi-window look-back: 40 000 frames are 157
    blocks at one frame per lane) give the oracle's statuses, bytes, summaries and messages,
    for valid batches and batches with a failure deep inside."""
    import uvhttp_amd as U
    monkeypatch.setenv("UVHTTP_WS_PLAN_FPT", str(fpt))
    e = U.GpuEngine(0)
    try:
        rng = random.Random(1000 + fpt)
        for p_bad in (0.0, 0.00005):
            wire, offs = _rand_batch(rng, 40000, [0, 1, 7, 125, 126, 300], p_ctrl=0.05,
                                     p_frag=0.3, p_bad=p_bad)
            for compact in (False, True):
                ref, got = _run_both(torch, e, wire, 40000, offs=offs, mm=0, compact=compact)
                _compare(ref, got, compact)
    finally:
        e.close()


def test_epoch_wraparound(torch, monkeypatch):
    """Decode calls on both sides of the epoch wrap (the workspace is cleared when the 30-bit
    call tag runs out) decode like the oracle: big and small batches alternate so stale map
    entries of an earlier call would show."""
    import uvhttp_amd as U
    monkeypatch.setenv("UVHTTP_WS_EPOCH_START", str((1 << 30) - 4))
    e = U.GpuEngine(0)
    try:
        rng = random.Random(31337)
        for k in range(8):
            n = 3000 if k % 2 == 0 else 40
            sizes = [70000, 5000, 125] if k % 2 == 0 else [0, 3, 300]
            wire, offs = _rand_batch(rng, n, sizes, p_ctrl=0.1, p_frag=0.3,
                                     p_bad=0.002 if k % 3 == 2 else 0.0)
            for compact in (False, True):
                ref, got = _run_both(torch, e, wire, n, offs=offs, mm=0, compact=compact)
                _compare(ref, got, compact)
    finally:
        e.close()


@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("plen", [0, 3, 60, 200, 1000])
def test_stride_layouts(torch, eng, plen, compact):
    """Fixed-stride batches of small frames (the payload kernels find a vector's frame by
    arithmetic there): uniform frames, a longer last frame, a wrong-sized frame (LAYOUT), a cut
    last frame, a failing frame in the middle, mixed opcodes of the same wire size."""
    rng = random.Random(plen)
    k = lambda: rng.randbytes(4)  # noqa: E731
    n = 600
    base = [_frame(rng.choice([1, 2]), 1, rng.randbytes(plen), k()) for _ in range(n)]
    stride = len(base[0])
    variants = {"uniform": base,
                "long_last": base[:-1] + [_frame(2, 1, rng.randbytes(plen + 777), k())],
                "layout": base[:300] + [_frame(2, 1, rng.randbytes(plen + 1), k())] + base[301:],
                "rsv": base[:200] + [_frame(2, 1, rng.randbytes(plen), k(), rsv=4)] + base[201:]}
    if plen <= 125:  # same wire size: PING / CONT fragments / TEXT mixed
        mix = []
        for i in range(n):
            # PING, TEXT start, CONT end, BINARY, PONG
            mix.append(_frame([9, 1, 0, 2, 10][i % 5], 0 if i % 5 == 1 else 1,
                              rng.randbytes(plen), k()))
        variants["mixed"] = mix
    for name, frames in variants.items():
        wire = np.frombuffer(b"".join(frames), np.uint8).copy()
        for wl in (wire.size, wire.size - 1 - rng.randrange(min(stride, 30))):
            ref, got = _run_both(torch, eng, wire, len(frames), stride=stride, wire_len=wl,
                                 compact=compact)
            _compare(ref, got, compact)


def test_stride_state_machine_failures(torch):
    """Stride batches with failures only the state machine sees — a CONTINUATION with nothing
    open, a new data frame inside a fragmented message, a message over max_message_size — at
    the first, a middle and the last frame, and deep in a batch of 60 000 frames: bytes,
    statuses and summaries equal the oracle's (frames from the failing one on stay masked)."""
    import uvhttp_amd as U
    e = U.GpuEngine(0)
    try:
        rng = random.Random(55)
        k = lambda: rng.randbytes(4)  # noqa: E731
        for plen, n in ((60, 600), (200, 600), (3000, 200), (1, 60000)):
            for where in (0, 1, n // 2, n - 1):
                for kind in ("cont", "new_in_frag", "too_big", "ok"):
                    frames = [_frame(2, 1, rng.randbytes(plen), k()) for _ in range(n)]
                    mm = MM
                    if kind == "cont":
                        frames[where] = _frame(0, 1, rng.randbytes(plen), k())
                    elif kind == "new_in_frag":
                        if where == 0:
                            continue
                        frames[where - 1] = _frame(1, 0, rng.randbytes(plen), k())
                        frames[where] = _frame(2, 1, rng.randbytes(plen), k())
                    elif kind == "too_big":
                        # a fragmented message from frame 0 that passes the limit at `where`
                        frames = [_frame(2 if i == 0 else 0, 0, rng.randbytes(plen), k())
                                  for i in range(n)]
                        mm = plen * (where + 1) - 1
                        if mm == 0:  # (0 means no limit)
                            continue
                    wire = np.frombuffer(b"".join(frames), np.uint8).copy()
                    stride = len(frames[0])
                    ref, got = _run_both(torch, e, wire, n, stride=stride, mm=mm)
                    if kind != "ok":
                        assert ref["summary"]["status"] == -1
                    _compare(ref, got)
    finally:
        e.close()


def test_stride_random_batches(torch):
    """Random stride batches (every frame the same wire size: PING/PONG/CLOSE/TEXT/BINARY/CONT
    mixed, header violations, cut last frames, frames past the end of the wire), in place,
    against the oracle."""
    import uvhttp_amd as U
    e = U.GpuEngine(0)
    try:
        rng = random.Random(808)
        for it in range(24):
            plen = rng.choice([0, 1, 5, 60, 125, 200, 1000, 3000, 9000])
            n = rng.choice([2, 3, 64, 500, 3000])
            frames, open_msg = [], False
            for i in range(n):
                r = rng.random()
                if r < 0.1 and plen <= 125:
                    op, fin = rng.choice([8, 9, 10]), 1
                elif open_msg:
                    op, fin = 0, rng.random() < 0.3
                else:
                    op, fin = rng.choice([1, 2]), rng.random() < 0.7
                if op <= 2:
                    open_msg = not fin
                rsv = 4 if rng.random() < 0.002 else 0
                frames.append(_frame(op, fin, rng.randbytes(plen), rng.randbytes(4), True, rsv))
            wire = np.frombuffer(b"".join(frames), np.uint8).copy()
            stride = len(frames[0])
            wl = wire.size
            if it % 4 == 1:
                wl -= rng.randint(1, min(stride, 40))            # last frame cut short
            elif it % 4 == 2 and n > 2:
                wl -= stride + rng.randint(0, stride - 1)         # last frame(s) past the end
            mm = rng.choice([MM, 0, plen * 3 + 1])
            ref, got = _run_both(torch, e, wire, n, stride=stride, wire_len=wl, mm=mm)
            _compare(ref, got)
    finally:
        e.close()
