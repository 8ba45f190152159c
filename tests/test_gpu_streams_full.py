"""Stream decode at BASELINE sizes against the oracle (VERDICT r03 "next" item 1).

The reference decodes every connection's reads with uvhttp_ws_process_data
(src/uvhttp_websocket.c:825-1097), called once per read by on_websocket_read
(src/uvhttp_connection.c:1128-1164).  Here the BASELINE configs run through the device stream
decode (uvhttp_ws_gpu_decode_streams / _decode_reads) at full size:

* C2 / C3 as 65 536 connections of one 4 KiB / 64 KiB frame each (the lane walk, which the
  engine picks above 16 384 connections; C2 also forced onto the wave walk);
* C4 as 4 096 connections x 256 frames, every connection continuing the one 256 MiB message
  (pending_bytes carried: the speculative decode, k_sspec_*; also with it off on the lane walk
  and, in 16 KiB reads, the wave walk);
* each as ONE process_data call per connection and cut into 16 KiB libuv reads (C2 also into
  1000-byte reads, so headers straddle calls).

The checker is oracle_decode_streams (tests/_oracle.py; itself checked against per-read
process_data in tests/test_oracle_streams.py): per connection every result field, per frame
every descriptor field, and the whole decoded wire byte for byte.  Sampled connections are
then delivered through the product's uvhttp_ws_deliver_stream and their on_message payloads
compared with the oracle's.
"""
import ctypes as C
import os

import numpy as np
import pytest

import _oracle

pytestmark = pytest.mark.gpu

SEED = 0x5EED0001
FULL = {  # frames, payload bytes, connections, fragmented (one message over all connections)
    "c2": (65536, 4096, 65536, False),
    "c3": (65536, 65536, 65536, False),
    "c4": (1048576, 256, 4096, True),
}
CASES = [
    ("c2", "auto", None), ("c2", "auto", 16384), ("c2", "auto", 1000), ("c2", "wave", None),
    ("c3", "auto", None), ("c3", "auto", 16384),
    ("c4", "auto", None), ("c4", "auto", 16384), ("c4", "lane", None), ("c4", "wave", 16384),
]


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _engine(walk):
    """auto: the default engine (C4's connections go to the speculative decode); a named walk
    runs with the speculation off, so that the walk decodes every call"""
    import uvhttp_amd as U
    env = {} if walk == "auto" else {"UVHTTP_WS_WALK": walk, "UVHTTP_WS_STREAM_SPEC": "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return U.GpuEngine(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _layout(cfg, read):
    import uvhttp_amd as U
    n, plen, conns, frag = FULL[cfg]
    stride = U.gen_frame_stride(plen)
    per = n // conns
    ln = per * stride
    st = np.zeros(conns, _oracle.STREAM_DT)
    st["begin"] = np.arange(conns, dtype=np.uint64) * ln
    st["len"] = ln
    st["recv_buffer_size"] = 65536  # a fresh connection's buffer (grows per call)
    st["max_frame_size"] = 16 << 20
    st["max_message_size"] = (256 << 20) if frag else (64 << 20)
    st["is_server"] = 1
    if frag:  # connection k continues the message its predecessors started
        st["pending_bytes"] = np.arange(conns, dtype=np.uint64) * per * plen
        st["pending_opcode"] = 2
    read_end = None
    if read:
        nr = -(-ln // read)
        st["first_read"] = np.arange(conns, dtype=np.uint32) * nr
        st["n_reads"] = nr
        one = np.minimum(np.arange(1, nr + 1, dtype=np.uint64) * read, ln)
        read_end = np.tile(one, conns)
    assert U.STREAM_DT.itemsize == _oracle.STREAM_DT.itemsize
    return n, plen, stride, conns, frag, st, read_end


@pytest.mark.parametrize("cfg,walk,read", CASES,
                         ids=[f"{c}-{w}-{r or 'onecall'}" for c, w, r in CASES])
def test_stream_decode_full_size(torch, cfg, walk, read):
    import uvhttp_amd as U
    n, plen, stride, conns, frag, st, read_end = _layout(cfg, read)
    wl = stride * n
    eng = _engine(walk)
    try:
        d = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
        eng.gen_frames(d, n, plen, SEED, opcode0=2, fragmented=frag, force_keys=True)
        tail = torch.randint(0, 256, (64,), dtype=torch.uint8, device="cuda")
        d[wl:] = tail
        dev_st = torch.from_numpy(st.view(np.uint8).copy()).to("cuda")
        re_dev = None if read_end is None else \
            torch.from_numpy(read_end.view(np.int64).copy()).to("cuda")
        desc_t = torch.full(((n + 1) * 32,), 0xA5, dtype=torch.uint8, device="cuda")
        desc, res = eng.decode_streams(d, dev_st, conns, n, desc=desc_t, wire_len=wl,
                                       read_end=re_dev,
                                       n_reads=0 if read_end is None else read_end.size)
        torch.cuda.synchronize()
        eng.sync()
        got_res = res[: conns * U.STREAM_RESULT_BYTES].cpu().numpy().view(U.STREAM_RESULT_DT)
        got_desc = eng.read_desc(desc, n)
        assert (desc_t[n * 32:] == 0xA5).all()
        got_wire = d.cpu().numpy()
    finally:
        eng.close()
    assert np.array_equal(got_wire[wl:], tail.cpu().numpy())  # nothing written past the wire

    # the oracle: every connection fed its process_data calls over the same bytes
    host, _ = _oracle.gen_frames(n, plen, SEED, fragmented=frag, force_keys=True, total=n)
    out, frames, total = _oracle.decode_streams(host, st, read_end, max_frames=n)
    assert total == n  # every frame of the config is delivered

    # per connection: the result record
    r, o = got_res, out
    assert np.array_equal(r["n_delivered"], o["n_frames"])
    assert np.array_equal(r["n_frames"], o["n_frames"] + (o["rc"] != 0))
    assert np.array_equal(r["status"], o["rc"]) and np.array_equal(r["first_status"], o["reason"])
    assert np.array_equal(r["calls"], o["calls"])
    assert np.array_equal(r["consumed_bytes"], o["consumed"])
    assert np.array_equal(r["recv_buffer_size"], o["recv_size"])
    assert np.array_equal(r["pending_bytes"], o["frag_size"])
    assert np.array_equal(r["buffered_end"], o["consumed"] + o["recv_pos"])
    first = np.concatenate([[0], np.cumsum(r["n_frames"].astype(np.uint64))[:-1]])
    assert np.array_equal(r["first_frame"].astype(np.uint64), first)

    # per frame: every descriptor field (connections' frames are contiguous in both lists)
    g = got_desc
    assert np.array_equal(g["payload_off"], frames["payload_off"])
    assert np.array_equal(g["payload_len"], frames["payload_len"])
    assert np.array_equal(g["masking_key"], frames["key"])
    assert np.array_equal(g["opcode"], frames["opcode"])
    assert np.array_equal(g["flags"] & 0x23, frames["flags"])
    assert np.array_equal(g["header_size"], frames["header_size"])
    assert np.array_equal(g["wire_len"], frames["wire_len"])
    assert not g["status"].any()

    # the decoded wire, byte for byte
    assert np.array_equal(got_wire[:wl], host)

    # sampled connections through the product's host delivery (uvhttp_ws_deliver_stream)
    hd = got_desc.view(np.uint8)
    for k in sorted({0, 1, conns // 2, conns - 1}):
        _deliver_one(U, got_wire, hd, st, got_res, host, frames, first, k, frag, plen)


def _deliver_one(U, wire, desc_bytes, st, res, host, frames, first, k, frag, plen):
    conn = U.WsConnection(1, int(st[k]["max_frame_size"]), int(st[k]["max_message_size"]))
    pend = int(st[k]["pending_bytes"])
    if pend:  # the open message the earlier reads left in conn->fragmented_message
        libc = C.CDLL(None)
        libc.malloc.restype = C.c_void_p
        libc.malloc.argtypes = [C.c_size_t]
        p = libc.malloc(pend)
        assert p
        C.memset(p, 0, pend)
        s = conn.struct
        s.fragmented_message, s.fragmented_size, s.fragmented_capacity = p, pend, pend
        s.fragmented_opcode = int(st[k]["pending_opcode"])
    sk = U.Stream.from_buffer_copy(st[k].tobytes())
    rk = U.StreamResult.from_buffer_copy(res[k].tobytes())
    hw = wire.ctypes.data_as(C.POINTER(C.c_uint8))
    hdp = desc_bytes.ctypes.data_as(C.POINTER(C.c_uint8))
    rc = U.lib().uvhttp_ws_deliver_stream(conn.ptr, hw, hdp, C.byref(sk), C.byref(rk))
    assert rc == 0
    mine = frames[int(first[k]):int(first[k]) + int(rk.n_frames)]
    msgs = [e for e in conn.events if e[0] == "message"]
    if not frag:
        assert len(msgs) == len(mine)
        for (_, op, payload), f in zip(msgs, mine):
            a = int(f["payload_off"])
            assert op == 2 and payload == host[a:a + int(f["payload_len"])].tobytes()
    elif k == len(st) - 1:  # the last connection completes the 256 MiB message
        assert len(msgs) == 1 and msgs[0][1] == 2
        body = msgs[0][2]
        assert len(body) == pend + len(mine) * plen
        assert body[:pend] == bytes(pend)
        exp = np.concatenate([host[int(f["payload_off"]):int(f["payload_off"]) + plen]
                              for f in mine])
        assert body[pend:] == exp.tobytes()
    else:
        assert not msgs
        assert conn.struct.fragmented_size == pend + len(mine) * plen
    conn.close()
