"""uvhttp_ws_deliver_messages over the DEVICE's compact output (the fast
summary-only compact decode, d_desc = NULL, must be deliverable to a reference connection):
decode_compact on the GPU, host copies of the arena, the message table (with the open
message's entry) and the summary, then delivery — callbacks, control-sink calls, CLOSED state
and the open fragment must equal OracleConn fed the delivered frames one process_data call each
(src/uvhttp_websocket.c:825-1097; on_message through src/uvhttp_connection.c:1234-1263)."""
import random

import numpy as np
import pytest

import _deliver as D

pytestmark = pytest.mark.gpu
MF, MM = 16 * 1024 * 1024, 0


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
    e.set_stamps(True)
    yield e
    e.close()


def _device_compact(torch, eng, frames, stride=None, no_desc=True, mm=MM):
    """decode_compact on the device -> host (arena, msgs with the open entry, summary, wire,
    desc or None, the path taken: 'fast' when k_spec_fix did not run)"""
    wire = np.frombuffer(b"".join(f.bytes for f in frames), np.uint8).copy()
    n = len(frames)
    d = torch.zeros(wire.size + 64, dtype=torch.uint8, device="cuda")
    d[: wire.size] = torch.from_numpy(wire).to("cuda")
    arena = torch.zeros(wire.size + 64, dtype=torch.uint8, device="cuda")
    kw = dict(stride=stride)
    if stride is None:
        offs = np.cumsum([0] + [len(f.bytes) for f in frames[:-1]]).astype(np.uint64)
        kw = dict(offsets=torch.from_numpy(offs.view(np.int64)).to("cuda"))
    eng.read_stamps()
    desc, msgs, summ = eng.decode_compact(d, n, arena, wire_len=wire.size, max_frame_size=MF,
                                          max_message_size=mm, no_desc=no_desc, **kw)
    torch.cuda.synchronize()
    s = eng.read_summary(summ)
    fast = "fixup" not in {r[1] for r in eng.read_stamps()}
    m = msgs[: (s["n_messages"] + 1) * 32].cpu().numpy().view(D.MSG_DT)
    hd = None if desc is None else desc[: n * 32].cpu().numpy().view(D.DESC_DT)
    return (arena[: max(1, s["arena_bytes"])].cpu().numpy(), m, s, d[: wire.size].cpu().numpy(),
            hd, fast)


def _deliver_and_check(frames, arena, msgs, s, wire, desc, stride=0, mm=MM):
    import uvhttp_amd as U
    conn = U.WsConnection(1, MF, mm, user_data=True)
    with D.control_sink() as sink:
        rc = U.deliver_messages(conn, arena, msgs, s, wire=wire, desc=desc, stride=stride)
        orc = D.expected(frames, s["n_delivered"], MF, mm)
        D.check(conn, sink, orc, rc, s["status"])
        return conn


def _uniform(rng, n, stride, frag):
    p = stride - (2 if stride - 6 < 126 else 4) - 4
    frames, open_msg = [], False
    for _ in range(n):
        op = 0 if open_msg else rng.choice([1, 2])
        fin = rng.random() > frag
        frames.append(D.Frame(op, fin, rng.randbytes(p), key=rng.randbytes(4)))
        open_msg = not fin
    return frames


@pytest.mark.parametrize("stride", [140, 200, 264, 1000, 2048, 2560])
def test_summary_only_stride_batches(torch, eng, stride):
    """the random stride batches of test_gpu_summary_compact: every message and the open one
    from the fast path's table"""
    rng = random.Random(stride)
    n = max(3, min(6000, (1 << 20) // stride))
    for frag in (0.0, 0.3, 1.0):
        frames = _uniform(rng, n, stride, frag)
        arena, msgs, s, wire, _, fast = _device_compact(torch, eng, frames, stride=stride)
        assert fast and s["n_delivered"] == n
        _deliver_and_check(frames, arena, msgs, s, wire, None, stride=stride)


@pytest.mark.parametrize("last", ["close", "ping", "pong", "reserved", "open"])
def test_summary_only_last_frame(torch, eng, last):
    """a control frame as the last frame sends the call to the full decode (k_spec_fix): the
    table and summary are the same, the control frame is read from the wire"""
    rng = random.Random(last)
    stride = 300
    frames = _uniform(rng, 3000, stride, 0.4)
    open_msg = not frames[-1].fin
    tail = {"close": D.Frame(8, 1, b"\x03\xe8bye"), "ping": D.Frame(9, 1, b"ping"),
            "pong": D.Frame(10, 1, b"pong"), "reserved": D.Frame(11, 1, b""),
            "open": D.Frame(0 if open_msg else 2, 0, rng.randbytes(292))}[last]
    frames.append(tail)
    arena, msgs, s, wire, _, fast = _device_compact(torch, eng, frames, stride=stride)
    assert fast == (last == "open")
    # only the last frame's slot is needed from the wire
    part = np.zeros_like(wire)
    part[(len(frames) - 1) * stride:] = wire[(len(frames) - 1) * stride:]
    _deliver_and_check(frames, arena, msgs, s, part, None, stride=stride)


@pytest.mark.parametrize("seed", range(8))
def test_descriptor_mode_mixed(torch, eng, seed):
    """offset-table batches with control frames anywhere (between fragments too), reserved
    opcodes, failures: delivered from the descriptors + arena + table"""
    rng = random.Random(seed)
    n = rng.randint(1, 400)
    bad = rng.randrange(n) if seed % 2 else None
    frames = D.mixed(rng, n, bad_at=bad)
    arena, msgs, s, wire, desc, _ = _device_compact(torch, eng, frames, no_desc=False)
    assert s["n_delivered"] == (bad if bad is not None else n)
    _deliver_and_check(frames, arena, msgs, s, wire, desc)


def test_message_limit_open_entry(torch, eng):
    """a fragment over max_message_size: the open message's entry holds what was appended"""
    rng = random.Random(9)
    frames = [D.Frame(2, 0, rng.randbytes(300)), D.Frame(9, 1, b"hi"), D.Frame(0, 0, rng.randbytes(300)),
              D.Frame(0, 1, rng.randbytes(600))]
    arena, msgs, s, wire, desc, _ = _device_compact(torch, eng, frames, no_desc=False, mm=1000)
    assert s["pending_bytes"] == 600 and msgs[s["n_messages"]]["reserved"] == 300
    _deliver_and_check(frames, arena, msgs, s, wire, desc, mm=1000)


def test_c4_full_size(torch, eng):
    """C4 (1 048 576 x 256-byte fragments of one 256 MiB message) through the fast summary-only
    compact decode and delivery; then C4-shaped all-FIN frames (one message each, 65 536)"""
    import uvhttp_amd as U
    n, plen = 1048576, 256
    stride = U.gen_frame_stride(plen)
    wl = stride * n
    d = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
    eng.gen_frames(d, n, plen, 7, opcode0=2, fragmented=True)
    host_in = d[:wl].cpu().numpy().copy()
    arena = torch.empty(wl, dtype=torch.uint8, device="cuda")
    eng.read_stamps()
    _, msgs, summ = eng.decode_compact(d, n, arena, stride=stride, wire_len=wl,
                                       max_message_size=256 << 20, no_desc=True)
    torch.cuda.synchronize()
    s = eng.read_summary(summ)
    assert "fixup" not in {r[1] for r in eng.read_stamps()}
    assert s["n_delivered"] == n and s["n_messages"] == 1 and s["pending_bytes"] == 0
    m = msgs[:64].cpu().numpy().view(D.MSG_DT)
    conn = U.WsConnection(1, MF, 256 << 20)
    rc = U.deliver_messages(conn, arena[: s["arena_bytes"]], m, s, stride=stride)
    assert rc == 0 and len(conn.events) == 1
    # the message = the oracle's reassembly: every frame's payload unmasked, in order
    import _oracle
    _oracle.load().oracle_unmask_frames(_oracle._ptr(host_in), n, stride)
    pay = host_in.reshape(n, stride)[:, stride - plen:].reshape(-1)
    ev = conn.events[0]
    assert ev[0] == "message" and ev[1] == 2 and ev[2] == pay.tobytes()
    # all-FIN C4-shaped frames: one message per frame, against the oracle connection
    rng = random.Random(4)
    frames = _uniform(rng, 65536, stride, 0.0)
    arena, msgs, s, wire, _, fast = _device_compact(torch, eng, frames, stride=stride)
    assert fast and s["n_messages"] == 65536
    _deliver_and_check(frames, arena, msgs, s, wire, None, stride=stride)


@pytest.mark.parametrize("depth", [2, 3, 5])
def test_pipeline_compact(torch, depth):
    """the host-memory pipeline's compact submissions (summary-only stride batches with a
    control frame or an open message at the end; offset-table batches with descriptors),
    interleaved with in-place submissions on the same slots, delivered with
    uvhttp_ws_deliver_messages from the slots' host results"""
    import uvhttp_amd as U
    pipe = U.GpuPipeline(0, depth=depth, slot_bytes=4 << 20, slot_frames=8192)
    rng = random.Random(77 + depth)
    jobs = []
    for b in range(9 + depth):
        kind = b % 3
        if kind == 0:  # summary-only stride batch
            stride = rng.choice([140, 264, 1000])
            frames = _uniform(rng, rng.randint(1, 3000), stride, rng.choice([0.0, 0.4, 1.0]))
            if rng.random() < 0.5:
                frames.append(rng.choice([D.Frame(8, 1, b"\x03\xe8x"), D.Frame(9, 1, b"p")]))
            jobs.append(("sum", frames, stride))
        elif kind == 1:  # descriptors
            bad = rng.randrange(40) if b == 4 else None
            jobs.append(("desc", D.mixed(rng, 40, bad_at=bad), 0))
        else:  # in place, same slots
            jobs.append(("inplace", D.mixed(rng, 30), 0))
    inflight = {}

    def finish(slot, job):
        kind, frames, stride = job
        if kind == "inplace":
            dp, sp, s = pipe.wait(slot)
            conn = U.WsConnection(1, MF, MM, user_data=True)
            with D.control_sink() as sink:
                rc = pipe.deliver(conn, slot, dp, sp)
                D.check(conn, sink, D.expected(frames, s["n_delivered"], MF, MM), rc, s["status"])
            return
        ap, mp, dp, sp, s = pipe.wait_compact(slot)
        assert (dp is None) == (kind == "sum")
        conn = U.WsConnection(1, MF, MM, user_data=True)
        with D.control_sink() as sink:
            rc = pipe.deliver_messages(conn, slot, ap, mp, dp, sp, stride=stride)
            D.check(conn, sink, D.expected(frames, s["n_delivered"], MF, MM), rc, s["status"])

    for k, job in enumerate(jobs):
        slot = k % depth
        if slot in inflight:
            finish(slot, inflight.pop(slot))
        kind, frames, stride = job
        wire = np.frombuffer(b"".join(f.bytes for f in frames), np.uint8)
        pipe.buffer(slot)[: wire.size] = wire
        if kind == "sum":
            pipe.submit_compact(slot, wire.size, len(frames), stride=stride, max_message_size=MM)
        else:
            offs = np.cumsum([0] + [len(f.bytes) for f in frames[:-1]]).astype(np.uint64)
            pipe.offsets(slot)[: offs.size] = offs
            sub = pipe.submit if kind == "inplace" else pipe.submit_compact
            sub(slot, wire.size, len(frames), use_offsets=True, max_message_size=MM)
        inflight[slot] = job
    for slot, job in inflight.items():
        finish(slot, job)
    pipe.close()
