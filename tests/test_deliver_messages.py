"""uvhttp_ws_deliver_messages on the host (no GPU): a compact decode's arena, message table and
summary — here the oracle's compact decode of the same bytes (oracle/ws_oracle.c, the batch
contract over src/uvhttp_websocket.c:825-1097) — delivered to a product connection must leave
the callbacks, the control-sink calls (pong / close echo, :1016-1084), the CLOSED state and the
open fragment (size, capacity, opcode, bytes: :781-822) exactly as process_data fed the same
frames one call each.  The device's own outputs go through the same checks in
test_gpu_deliver_messages.py."""
import random

import numpy as np
import pytest

import _deliver as D
import _oracle

MF, MM = 16 * 1024 * 1024, 64 * 1024 * 1024


def _run(frames, mf=MF, mm=MM, summary_only=False, stride=0, drop_wire=False):
    import uvhttp_amd as U
    wire = np.frombuffer(b"".join(f.bytes for f in frames), np.uint8).copy()
    offs = np.cumsum([0] + [len(f.bytes) for f in frames[:-1]]).astype(np.uint64)
    n = len(frames)
    kw = dict(stride=stride) if stride else dict(offsets=offs)
    ref = _oracle.decode_batch(wire, n, max_frame_size=mf, max_message_size=mm, compact=True,
                               arena_cap=wire.size + 64, **kw)
    s = ref["summary"]
    msgs, desc = D.tables(frames, ref, offs)
    conn = U.WsConnection(1, mf, mm, user_data=True)
    with D.control_sink() as sink:
        rc = U.deliver_messages(conn, ref["arena"][: max(1, s["arena_bytes"])], msgs, s,
                                wire=None if drop_wire else ref["wire"],
                                desc=None if summary_only else desc, stride=stride)
        orc = D.expected(frames, s["n_delivered"], mf, mm)
        D.check(conn, sink, orc, rc, s["status"])
    return s


@pytest.mark.parametrize("seed", range(24))
def test_mixed_batches_with_descriptors(seed):
    """data messages, fragments, CLOSE / PING / PONG anywhere (between fragments too), reserved
    opcodes; a third of the batches fail part-way"""
    rng = random.Random(seed)
    n = rng.randint(1, 60)
    bad = rng.randrange(n) if seed % 3 == 2 else None
    s = _run(D.mixed(rng, n, bad_at=bad))
    assert s["n_delivered"] == (bad if bad is not None else n)


def test_message_limit_failure_leaves_open_message():
    """a fragment over max_message_size fails the batch: the message open before it stays
    open with the bytes it had (append_fragment fails without appending, :786-791)"""
    rng = random.Random(7)
    frames = [D.Frame(2, 0, rng.randbytes(300)), D.Frame(9, 1, b"hi"), D.Frame(0, 0, rng.randbytes(300)),
              D.Frame(0, 1, rng.randbytes(600))]
    s = _run(frames, mm=1000)
    assert s["n_delivered"] == 3 and s["pending_bytes"] == 600 and s["status"] == -1


@pytest.mark.parametrize("last", ["close", "ping", "pong", "reserved", "data", "open", "zero_start"])
def test_summary_only_stride_layout(last):
    """summary-only (no descriptors): uniform data frames of a >= 140-byte stride, the last
    frame anything; only the last frame is read from the wire"""
    rng = random.Random(last)
    stride, p = 264, 256
    frames, open_msg = [], False
    for i in range(200):
        op = 0 if open_msg else rng.choice([1, 2])
        fin = rng.random() > 0.5
        frames.append(D.Frame(op, fin, rng.randbytes(p)))
        open_msg = not fin
    tail = {"close": D.Frame(8, 1, b"\x03\xe9bye"), "ping": D.Frame(9, 1, b"ping!"),
            "pong": D.Frame(10, 1, b"pong"), "reserved": D.Frame(11, 1, b"r"),
            "data": D.Frame(0 if open_msg else 2, 1, rng.randbytes(p)),
            "open": D.Frame(0 if open_msg else 1, 0, rng.randbytes(p)),
            "zero_start": D.Frame(2, 0, b"")}[last]
    if last == "zero_start" and open_msg:
        tail = D.Frame(0, 0, b"")  # (an empty middle fragment)
    frames.append(tail)
    _run(frames, summary_only=True, stride=stride)


def test_summary_only_refusals():
    """summary-only with a last frame outside every message and no wire, or a stride a control
    frame could fill: INVALID_PARAM before any callback; a connection with a message already
    open: refused too"""
    import uvhttp_amd as U
    rng = random.Random(3)
    frames = [D.Frame(2, 1, rng.randbytes(256)) for _ in range(5)] + [D.Frame(9, 1, b"x")]
    wire = np.frombuffer(b"".join(f.bytes for f in frames), np.uint8).copy()
    ref = _oracle.decode_batch(wire, 6, stride=264, compact=True, arena_cap=wire.size + 64)
    msgs, desc = D.tables(frames, ref, np.arange(6, dtype=np.uint64) * 264)
    s = ref["summary"]
    conn = U.WsConnection(1)
    assert U.deliver_messages(conn, ref["arena"], msgs, s, wire=None, desc=None, stride=264) == -1
    assert U.deliver_messages(conn, ref["arena"], msgs, s, wire=ref["wire"], desc=None, stride=100) == -1
    assert conn.events == []
    # a message open on the connection: the batch was decoded from a fresh state
    assert conn.process_data(D.frame(1, 0, b"open")) == 0
    assert U.deliver_messages(conn, ref["arena"], msgs, s, wire=ref["wire"], desc=desc) == -1
    assert conn.events == []


def test_malformed_tables_refused():
    """a message outside the arena, out of frame order, or an open entry that disagrees with
    the summary: INVALID_PARAM, nothing delivered"""
    import uvhttp_amd as U
    rng = random.Random(5)
    frames = [D.Frame(2, 1, rng.randbytes(100)) for _ in range(4)] + [D.Frame(1, 0, rng.randbytes(50))]
    wire = np.frombuffer(b"".join(f.bytes for f in frames), np.uint8).copy()
    offs = np.cumsum([0] + [len(f.bytes) for f in frames[:-1]]).astype(np.uint64)
    ref = _oracle.decode_batch(wire, 5, offsets=offs, compact=True, arena_cap=wire.size + 64)
    msgs, desc = D.tables(frames, ref, offs)
    s = ref["summary"]
    for field, val in (("len", 10 ** 9), ("first_frame", 3), ("last_frame", 99)):
        bad = msgs.copy()
        bad[1][field] = val
        conn = U.WsConnection(1)
        assert U.deliver_messages(conn, ref["arena"], bad, s, wire=ref["wire"], desc=desc) == -1
        assert conn.events == []
    bad = msgs.copy()
    bad[4]["reserved"] = 0
    conn = U.WsConnection(1)
    assert U.deliver_messages(conn, ref["arena"], bad, s, wire=ref["wire"], desc=desc) == -1
