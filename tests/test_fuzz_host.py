"""Frame-stream fuzzer (the reference has none for WebSocket frames: SURVEY §2, fuzz row):
hypothesis-generated streams — valid frames, corrupted headers, random garbage, odd limits,
arbitrary read boundaries — fed to the product's drop-in uvhttp_ws_process_data and to the
oracle; return codes, callback transcripts, control-hook calls, state and buffer sizes must
agree after every read."""
import ctypes as C

from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import _oracle
import uvhttp_amd as U


def _frame(op, fin, rsv, masked, key, payload, form):
    n = len(payload)
    b0 = (0x80 if fin else 0) | (rsv << 4) | (op & 0xF)
    mb = 0x80 if masked else 0
    if form == 0 and n < 126:
        head = bytes([b0, mb | n])
    elif form <= 1 and n < 65536:
        head = bytes([b0, mb | 126, n >> 8, n & 0xFF])
    else:
        head = bytes([b0, mb | 127]) + n.to_bytes(8, "big")
    if not masked:
        return head + payload
    return head + key + bytes(b ^ key[i & 3] for i, b in enumerate(payload))


frames = st.builds(
    _frame,
    op=st.sampled_from([0, 1, 2, 3, 8, 9, 10, 11]),
    fin=st.booleans(),
    rsv=st.sampled_from([0, 0, 0, 0, 1, 4]),
    masked=st.sampled_from([True, True, True, False]),
    key=st.binary(min_size=4, max_size=4),
    payload=st.one_of(st.binary(max_size=140), st.binary(min_size=126, max_size=600)),
    form=st.sampled_from([0, 0, 0, 1, 2]),
)
chunks = st.one_of(frames, st.binary(min_size=1, max_size=20))


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(parts=st.lists(chunks, min_size=1, max_size=12),
       cuts=st.lists(st.integers(min_value=1, max_value=700), min_size=1, max_size=30),
       mf=st.sampled_from([16 * 1024 * 1024, 65536, 300, 100]),
       mm=st.sampled_from([64 * 1024 * 1024, 500, 0, 64]),
       server=st.sampled_from([1, 1, 0]))
def test_fuzz_stream_product_vs_oracle(parts, cuts, mf, mm, server):
    stream = b"".join(parts)
    prod = U.WsConnection(server, mf, mm, user_data=True)
    orc = _oracle.OracleConn(server, mf, mm, record=1, wrapper=True)
    sink = []

    @U.CONTEXT_RESOLVER
    def resolver(conn):
        return 1

    @U.CONTROL_SINK
    def hook(ctx, conn, op, p, n):
        sink.append(("pong" if op == 0xA else "close_echo", C.string_at(p, n) if n else b""))

    U.lib().uvhttp_ws_amd_set_control_hooks(resolver, hook)
    try:
        pos, k = 0, 0
        while pos < len(stream):
            n = cuts[k % len(cuts)]
            k += 1
            piece = stream[pos:pos + n]
            pos += n
            r1, r2 = prod.process_data(piece), orc.process_data(piece)
            assert r1 == r2
            s = prod.struct
            assert s.recv_buffer_size == orc.recv_size
            assert s.recv_buffer_pos == _oracle.load().oracle_conn_recv_pos(orc.c)
            frag = s.fragmented_size if s.fragmented_message else 0
            assert frag == _oracle.load().oracle_conn_frag_size(orc.c)
            if r1 != 0:
                break
        oev = orc.events()
        assert [(t, a, p) for t, a, p in prod.events if t == "message"] == \
            [e for e in oev if e[0] == "message"]
        assert [(t, a) for t, a, p in prod.events if t == "close"] == \
            [(t, a) for t, a, p in oev if t == "close"]
        assert sink == [(t, p) for t, a, p in oev if t in ("pong", "close_echo")]
    finally:
        U.lib().uvhttp_ws_amd_set_control_hooks(U.CONTEXT_RESOLVER(), U.CONTROL_SINK())
