"""The product's drop-in host surface (uvhttp_amd/csrc/ws_host.c) against the reference's
known-answer tests and, on randomized frame streams, against the oracle."""
import ctypes as C
import random

import pytest

import _known
import _oracle
import uvhttp_amd as U


def test_parse_known_answers(known_answers):
    for case in known_answers["parse_frame_header"]:
        _known.check_parse_case(case, U.parse_frame_header)


def test_mask_known_answers(known_answers):
    for case in known_answers["apply_mask"]:
        _known.check_mask_case(case, U.apply_mask)


class _ProductAdapter:
    def __init__(self, cfg, callbacks):
        self.c = U.WsConnection(1, cfg["max_frame_size"], cfg["max_message_size"],
                                callbacks=callbacks)

    def process(self, data):
        return self.c.process_data(data)

    def events(self):
        return [(k, a, p) for k, a, p in self.c.events]

    def set_recv_state(self, size, fill, pos):
        s = self.c.struct
        C.memmove(s.recv_buffer, fill, pos)
        s.recv_buffer_size = size
        s.recv_buffer_pos = pos

    @property
    def state(self):
        return self.c.struct.state

    @property
    def recv_size(self):
        return self.c.struct.recv_buffer_size


@pytest.mark.parametrize("idx", range(31))
def test_process_known_answers(known_answers, idx):
    cases = known_answers["process_data"]
    if idx >= len(cases):
        pytest.skip("no case")
    _known.check_process_case(cases[idx], _ProductAdapter)


def test_struct_abi():
    """Struct layouts match the reference ABI (16 / 48 / 248 bytes)."""
    assert C.sizeof(U.FrameHeader) == 16
    assert U.FrameHeader.payload_length.offset == 8
    assert C.sizeof(U.WsConnectionStruct) == 248
    assert U.WsConnectionStruct.recv_buffer.offset == 112
    assert U.WsConnectionStruct.recv_buffer_pos.offset == 128
    assert U.WsConnectionStruct.fragmented_message.offset == 152
    assert U.WsConnectionStruct.on_message.offset == 184
    assert U.WsConnectionStruct.user_data.offset == 208
    assert U.WsConnectionStruct.frames_received.offset == 240
    assert U.UvhttpConfig.websocket_max_frame_size.offset == 64
    assert C.sizeof(U.FrameDesc) == 32 and C.sizeof(U.MessageDesc) == 32
    # batcher structs (include/uvhttp_ws_amd.h, checked against gcc's layout)
    assert C.sizeof(U.BatcherConfig) == 72 and U.BatcherConfig.on_ready.offset == 48
    assert U.BatcherConfig.on_tls_handback.offset == 64
    assert C.sizeof(U.BatcherStats) == 256 and U.BatcherStats.blocked_ms.offset == 112
    assert U.BatcherStats.zero_copy_reads.offset == 248
    assert U.BatcherStats.blocked_p50_ms.offset == 208


def test_null_and_empty():
    c = U.WsConnection()
    assert c.process_data(b"", null=True) == -1
    assert c.process_data(b"") == 0
    rc, _, _ = U.parse_frame_header(b"", 0, "data")
    assert rc == -1


def _rand_frame(rng, allow_bad):
    ops = [0, 1, 2, 8, 9, 10] + ([3, 11] if allow_bad else [])
    op = rng.choice(ops)
    fin = 1 if op >= 8 else rng.random() < 0.6
    n = rng.choice([0, 1, 2, 3, 5, 125, 126, 127, 200, 1000, 4096, 65535, 65536, 70000])
    if op >= 8 and not allow_bad:
        n = min(n, 125)
    payload = bytes(rng.getrandbits(8) for _ in range(min(n, 64))) * (n // 64 + 1)
    payload = payload[:n]
    key = bytes(rng.getrandbits(8) for _ in range(4))
    b0 = (0x80 if fin else 0) | op
    if allow_bad and rng.random() < 0.03:
        b0 |= 0x40  # RSV1
    masked = not (allow_bad and rng.random() < 0.03)
    mb = 0x80 if masked else 0
    if n < 126:
        head = bytes([b0, mb | n])
    elif n < 65536:
        head = bytes([b0, mb | 126, n >> 8, n & 0xFF])
    else:
        head = bytes([b0, mb | 127]) + n.to_bytes(8, "big")
    if masked:
        body = bytes(p ^ key[i & 3] for i, p in enumerate(payload))
        return head + key + body
    return head + payload


@pytest.mark.parametrize("seed", range(12))
def test_random_streams_match_oracle(seed):
    """Random frame streams cut into random read sizes: identical return codes, callback
    transcripts, state and buffer sizes in the product host path and the oracle."""
    rng = random.Random(seed)
    allow_bad = seed % 3 == 2
    mfs = rng.choice([16 * 1024 * 1024, 70000, 65536, 4096])
    mms = rng.choice([64 * 1024 * 1024, 100000, 3000, 0])
    stream = b"".join(_rand_frame(rng, allow_bad) for _ in range(rng.randint(5, 40)))
    prod = U.WsConnection(1, mfs, mms, user_data=True)
    orc = _oracle.OracleConn(1, mfs, mms, record=1, wrapper=True)
    sink_events = []

    @U.CONTEXT_RESOLVER
    def resolver(conn):
        return 0x5E  # stands for wrapper->conn->server->context

    @U.CONTROL_SINK
    def sink(ctx, conn, op, p, n):
        assert ctx == 0x5E
        sink_events.append(("pong" if op == 0xA else "close_echo", op, C.string_at(p, n) if n else b""))

    U.lib().uvhttp_ws_amd_set_control_hooks(resolver, sink)
    try:
        pos = 0
        while pos < len(stream):
            cut = rng.choice([1, 2, 7, 100, 4096, 16384, 70000])
            chunk = stream[pos:pos + cut]
            pos += cut
            r1 = prod.process_data(chunk)
            r2 = orc.process_data(chunk)
            assert r1 == r2
            s = prod.struct
            assert s.recv_buffer_size == orc.recv_size
            assert s.state == (orc.state if orc.state == 3 else 0)
            if r1 != 0:
                break
        oev = orc.events()
        pev = list(prod.events)
        # interleave the product's callback events with its control-sink calls in order:
        # compare per kind (each kind is ordered)
        for kind in ("message", "close"):
            assert [e for e in pev if e[0] == kind] == \
                [(k, a, p if kind == "message" else None) for k, a, p in oev if k == kind]
        for kind in ("pong", "close_echo"):
            assert [e[2] for e in sink_events if e[0] == kind] == \
                [p for k, a, p in oev if k == kind]
    finally:
        U.lib().uvhttp_ws_amd_set_control_hooks(U.CONTEXT_RESOLVER(), U.CONTROL_SINK())
