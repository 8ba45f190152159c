"""The oracle's stream driver (oracle_decode_streams, the checker of the device stream decode at
BASELINE sizes) against the oracle connection fed the same reads one process_data call at a
time (on_websocket_read, src/uvhttp_connection.c:1128-1164).  CPU only.

Every connection: return code, calls that ran, failure reason, recv-buffer position/size,
fragment state and the delivered messages (digest and count) must agree; the driver's frame
list must tile the consumed bytes, and the wire it decodes in place must hold exactly the
delivered payloads unmasked.
"""
import random

import numpy as np

import _oracle
from test_gpu_parity import _frame


def _conn_bytes(rng, bad):
    frames, open_msg = [], False
    for _ in range(rng.randint(0, 12)):
        key = rng.randbytes(4)
        if rng.random() < 0.15:
            op, fin, payload = rng.choice([8, 9, 10]), 1, rng.randbytes(rng.choice([0, 2, 7, 125]))
        else:
            payload = rng.randbytes(rng.choice([0, 1, 125, 126, 1000, 5000, 70000]))
            op = 0 if open_msg else rng.choice([1, 2])
            fin = rng.random() < 0.5
            open_msg = not fin
        rsv, masked = 0, True
        if bad and rng.random() < 0.08:
            kind = rng.choice(["rsv", "unmasked", "cont"])
            rsv = 2 if kind == "rsv" else 0
            masked = kind != "unmasked"
            op = 0 if kind == "cont" else op
        frames.append(_frame(op, fin, payload, key, masked, rsv))
    data = b"".join(frames)
    if data and rng.random() < 0.3:
        data = data[: rng.randint(0, len(data))]
    return data


def _fnv(data, h=1469598103934665603):
    for b in data:
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def test_oracle_stream_driver_matches_per_read_process_data():
    rng = random.Random(31337)
    for trial in range(6):
        n = rng.choice([1, 7, 40])
        chunks, pos = [], 0
        st = np.zeros(n, _oracle.STREAM_DT)
        read_end, per_conn_reads = [], []
        for k in range(n):
            data = _conn_bytes(rng, bad=trial % 2 == 1)
            pos = (pos + 15) & ~15
            st[k]["begin"], st[k]["len"] = pos, len(data)
            st[k]["recv_buffer_size"] = 65536
            st[k]["max_frame_size"] = rng.choice([16 << 20, 65536, 6000])
            st[k]["max_message_size"] = rng.choice([64 << 20, 9000, 0])
            st[k]["is_server"] = 1
            reads, e = [], 0
            while e < len(data):
                step = rng.choice([1, 3, 100, 4096, 16384, 70000])
                reads.append(data[e:e + step])
                e += len(reads[-1])
            if trial >= 3:  # read tables
                st[k]["first_read"], st[k]["n_reads"] = len(read_end), max(1, len(reads))
                if not reads:
                    reads = [b""]
                acc = 0
                for r in reads:
                    acc += len(r)
                    read_end.append(acc)
            else:
                reads = [data]
            per_conn_reads.append(reads)
            chunks.append((pos, data))
            pos += len(data)
        wire = np.zeros(pos + 16, np.uint8)
        for p, d in chunks:
            wire[p:p + len(d)] = np.frombuffer(d, np.uint8)
        masked = wire.copy()
        out, frames, total = _oracle.decode_streams(
            wire, st, np.array(read_end, np.uint64) if read_end else None, max_frames=100000,
            digest=True)
        assert total == frames.size
        expect = masked.copy()
        fi = 0
        for k in range(n):
            mf, mm = int(st[k]["max_frame_size"]), int(st[k]["max_message_size"])
            orc = _oracle.OracleConn(1, mf, mm, record=1)
            rc, calls = orc.process_reads(per_conn_reads[k])
            o = out[k]
            assert (o["rc"], o["calls"]) == (rc, calls), (trial, k)
            assert o["reason"] == (orc.last_reason if rc else 0)
            assert o["recv_pos"] == orc.recv_pos and o["recv_size"] == orc.recv_size
            assert o["frag_size"] == orc.frag_size
            msgs = [p for t, _, p in orc.events() if t == "message"]
            assert o["n_messages"] == len(msgs)
            assert o["digest"] == _fnv(b"".join(msgs))
            # the frames tile the consumed bytes of the stream, in order
            mine = frames[fi:fi + o["n_frames"]]
            fi += o["n_frames"]
            assert (mine["conn"] == k).all()
            at = int(st[k]["begin"])
            for f in mine:
                start = int(f["payload_off"]) - int(f["header_size"]) - (4 if f["flags"] & 2 else 0)
                assert start == at
                at += int(f["wire_len"])
                if f["flags"] & 2 and f["payload_len"]:
                    key = int(f["key"]).to_bytes(4, "little")
                    a, b = int(f["payload_off"]), int(f["payload_off"] + f["payload_len"])
                    seg = bytearray(expect[a:b].tobytes())
                    _oracle.apply_mask(seg, key)
                    expect[a:b] = np.frombuffer(bytes(seg), np.uint8)
            assert at - int(st[k]["begin"]) == o["consumed"]
            assert o["consumed"] + o["recv_pos"] <= st[k]["len"]
        assert fi == frames.size
        assert np.array_equal(wire, expect)


def test_oracle_stream_driver_pending_message():
    """A connection continuing an open fragmented message (pending_bytes, as the device's
    uvhttp_ws_stream_t carries it): the message completes with the pending prefix counted
    against max_message_size, and over the limit it fails with ERR_MESSAGE."""
    body = b"".join(_frame(0, i == 3, bytes([i]) * 100, b"\x01\x02\x03\x04") for i in range(4))
    for pending, mm, want_rc in ((50, 1000, 0), (700, 1000, -1), (0, 0, -1)):
        st = np.zeros(1, _oracle.STREAM_DT)
        st[0]["len"], st[0]["recv_buffer_size"] = len(body), 65536
        st[0]["pending_bytes"], st[0]["pending_opcode"] = pending, 1
        st[0]["max_frame_size"], st[0]["max_message_size"], st[0]["is_server"] = 1 << 24, mm, 1
        wire = np.frombuffer(body, np.uint8).copy()
        out, frames, _ = _oracle.decode_streams(wire, st, max_frames=16, digest=True)
        assert out[0]["rc"] == want_rc
        if pending == 0:  # a continuation with nothing open
            assert out[0]["reason"] == -7 and out[0]["n_frames"] == 0
        elif want_rc == 0:
            assert out[0]["n_messages"] == 1 and out[0]["frag_size"] == 0
            msg = bytes(pending) + b"".join(bytes([i]) * 100 for i in range(4))
            assert out[0]["digest"] == _fnv(msg)
            assert frames[-1]["flags"] & 0x20 and not frames[0]["flags"] & 0x20
        else:
            assert out[0]["reason"] == -8 and out[0]["n_frames"] == 3
