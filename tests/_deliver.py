"""Shared pieces of the uvhttp_ws_deliver_messages tests (test_deliver_messages.py on the host
with the oracle's compact decode as input, test_gpu_deliver_messages.py with the device's):
batches of mixed frames, the message table's frame ranges and open-message entry, host
descriptors for the control frames, and the transcript check against OracleConn fed the
delivered frames one process_data call each (the batch contract, include/uvhttp_ws_amd.h)."""
import ctypes as C
import random
from contextlib import contextmanager

import numpy as np

import _oracle

MSG_DT = np.dtype([("arena_off", "<u8"), ("len", "<u8"), ("first_frame", "<u4"),
                   ("last_frame", "<u4"), ("opcode", "<i4"), ("reserved", "<u4")])
DESC_DT = np.dtype([("payload_off", "<u8"), ("payload_len", "<u8"), ("masking_key", "<u4"),
                    ("message", "<u4"), ("opcode", "u1"), ("flags", "u1"),
                    ("header_size", "u1"), ("status", "i1"), ("wire_len", "<u4")])
assert MSG_DT.itemsize == 32 and DESC_DT.itemsize == 32


def frame(op, fin, payload, key=b"\x01\x02\x03\x04", masked=True, len_form=None, rsv=0):
    n = len(payload)
    b0 = (0x80 if fin else 0) | (rsv << 4) | (op & 0xF)
    mb = 0x80 if masked else 0
    form = len_form or (7 if n < 126 else 16 if n < 65536 else 64)
    head = bytes([b0, mb | n]) if form == 7 else \
        bytes([b0, mb | 126, n >> 8, n & 0xFF]) if form == 16 else \
        bytes([b0, mb | 127]) + n.to_bytes(8, "big")
    if not masked:
        return head + payload
    body = (np.frombuffer(payload, np.uint8) ^ np.resize(np.frombuffer(key, np.uint8), n)).tobytes() if n else b""
    return head + key + body


class Frame:
    """one generated frame: its bytes and what it is"""

    def __init__(self, op, fin, payload, bad=False, **kw):
        self.op, self.fin, self.payload = op, fin, payload
        self.bytes = frame(op, fin, payload, **kw)
        self.bad = bad


def mixed(rng, n, sizes=(0, 1, 7, 100, 300, 5000), p_ctrl=0.15, p_frag=0.4, p_res=0.03,
          bad_at=None):
    """n frames: data messages (fragmented or not, zero-length fragments included), CLOSE /
    PING / PONG with payloads of 0-125 bytes, reserved opcodes 3 and 11; bad_at: a frame that
    fails (CONT with no message / data inside a message / RSV bit)"""
    out, open_msg = [], False
    for i in range(n):
        key = rng.randbytes(4)
        r = rng.random()
        if i == bad_at:
            kind = rng.choice(["rsv", "frag"])
            if kind == "rsv":
                out.append(Frame(2, 1, rng.randbytes(10), bad=True, key=key, rsv=4))
            else:  # a CONT with nothing open, or a start inside a message
                out.append(Frame(1 if open_msg else 0, 1, rng.randbytes(10), bad=True, key=key))
            continue
        if r < p_ctrl:
            op = rng.choice([8, 9, 10])
            pl = rng.choice([0, 1, 2, 5, 125])
            payload = rng.randbytes(pl)
            if op == 8 and pl >= 2:
                payload = (1000 + rng.randrange(20)).to_bytes(2, "big") + payload[2:]
            out.append(Frame(op, 1, payload, key=key))
        elif r < p_ctrl + p_res:
            out.append(Frame(rng.choice([3, 11]), 1, rng.randbytes(rng.choice([0, 3, 50])), key=key))
        else:
            pl = rng.choice(sizes)
            if open_msg:
                op, fin = 0, rng.random() < 0.4
            else:
                op, fin = rng.choice([1, 2]), rng.random() > p_frag
                if not fin and pl == 0:
                    pl = 1  # (a zero-length start opens nothing; its CONT would fail)
            open_msg = not fin
            out.append(Frame(op, fin, rng.randbytes(pl), key=key))
    return out


def message_ranges(frames, nd):
    """the data messages of the first nd frames: [(first, last)] of the complete ones and the
    open one (first, last, opcode, first fragment's length) or None"""
    done, cur = [], None
    for i, f in enumerate(frames[:nd]):
        if f.op in (1, 2):
            if f.fin:
                done.append((i, i))
            elif len(f.payload):
                cur = [i, i, f.op, len(f.payload)]
        elif f.op == 0 and cur is not None:
            cur[1] = i
            if f.fin:
                done.append((cur[0], i))
                cur = None
    return done, cur


def tables(frames, ref, offsets):
    """host message table (n_messages + the open entry) and descriptors of the delivered
    frames (only opcode / payload_off / payload_len matter) from an oracle compact decode"""
    s = ref["summary"]
    nd, nm = s["n_delivered"], s["n_messages"]
    done, cur = message_ranges(frames, nd)
    assert len(done) == nm
    msgs = np.zeros(nm + 1, MSG_DT)
    msgs["arena_off"][:nm] = ref["msg_off"]
    msgs["len"][:nm] = ref["msg_len"]
    msgs["opcode"][:nm] = ref["msg_opcode"]
    for k, (a, b) in enumerate(done):
        msgs["first_frame"][k], msgs["last_frame"][k] = a, b
    if s["pending_bytes"]:
        assert cur is not None
        msgs[nm] = (s["arena_bytes"] - s["pending_bytes"], s["pending_bytes"], cur[0], cur[1], cur[2], cur[3])
    desc = np.zeros(max(1, nd + 1), DESC_DT)
    for i, f in enumerate(frames[:nd + 1]):
        hs = len(f.bytes) - len(f.payload) - 4
        desc[i] = (offsets[i] + hs + 4, len(f.payload), 0, 0, f.op, 0, hs, 0, len(f.bytes))
    return msgs, desc


_SINK = []


@contextmanager
def control_sink():
    """the product's control hooks record pongs / close echoes in _SINK while active"""
    import uvhttp_amd as U

    @U.CONTEXT_RESOLVER
    def resolver(conn):
        return 0x5E

    @U.CONTROL_SINK
    def sink(ctx, conn, op, p, n):
        _SINK.append(("pong" if op == 0xA else "close_echo", C.string_at(p, n) if n else b""))

    _SINK.clear()
    U.lib().uvhttp_ws_amd_set_control_hooks(resolver, sink)
    try:
        yield _SINK
    finally:
        U.lib().uvhttp_ws_amd_set_control_hooks(U.CONTEXT_RESOLVER(), U.CONTROL_SINK())


def expected(frames, nd, mf, mm):
    """OracleConn fed the delivered frames one process_data call each"""
    orc = _oracle.OracleConn(1, mf, mm, record=1, wrapper=True)
    for f in frames[:nd]:
        assert orc.process_data(f.bytes) == 0
    return orc


def check(conn, sink, orc, rc, status):
    """the product connection after deliver_messages against the oracle's"""
    assert rc == (0 if status == 0 else -1)
    oev = orc.events()
    assert [e for e in conn.events if e[0] in ("message", "close")] == \
        [(k, a, p if k == "message" else None) for k, a, p in oev if k in ("message", "close")]
    assert list(sink) == [(k, p) for k, a, p in oev if k in ("pong", "close_echo")]
    s = conn.struct
    assert bool(s.fragmented_message) == orc.frag_pending
    if orc.frag_pending:
        assert s.fragmented_size == orc.frag_size
        assert s.fragmented_capacity == orc.frag_capacity
        assert s.fragmented_opcode == orc.frag_opcode
    assert (s.state == 3) == (orc.state == 3)
    assert s.recv_buffer_pos == 0
    # the connection's next process_data call continues where the batch left it: a final
    # fragment completes the open message (its bytes and opcode) or fails like the reference's
    tail = frame(0, 1, b"-tail-", key=b"\x09\x08\x07\x06")
    n0, k0 = len(conn.events), len(orc.events())
    assert conn.process_data(tail) == orc.process_data(tail)
    assert [e for e in conn.events[n0:] if e[0] == "message"] == \
        [(k, a, p) for k, a, p in orc.events()[k0:] if k == "message"]


def seeds(k):
    return [random.Random(1000 + i) for i in range(k)]
