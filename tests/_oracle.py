"""ctypes binding of the CPU oracle (oracle/ws_oracle.c) — test infrastructure only.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the
product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "_build", "libws_oracle.so")


class OrcHeader(C.Structure):
    _fields_ = [("fin", C.c_uint8), ("rsv1", C.c_uint8), ("rsv2", C.c_uint8),
                ("rsv3", C.c_uint8), ("opcode", C.c_uint8), ("mask", C.c_uint8),
                ("len_code", C.c_uint8), ("payload_length", C.c_uint64)]


class OrcSummary(C.Structure):
    _fields_ = [("n_frames", C.c_uint32), ("n_delivered", C.c_uint32), ("status", C.c_int32),
                ("first_status", C.c_int32), ("consumed_bytes", C.c_uint64),
                ("payload_bytes", C.c_uint64), ("n_messages", C.c_uint32),
                ("state_closed", C.c_uint32), ("arena_bytes", C.c_uint64),
                ("pending_bytes", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_L = None


def load():
    global _L
    if _L is not None:
        return _L
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True,
                       stdout=subprocess.DEVNULL)
    L = C.CDLL(ORACLE_SO)
    vp, u32, u64, i32, sz = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32, C.c_size_t
    sig = {
        "oracle_parse_frame_header": (C.c_int, [vp, sz, C.POINTER(OrcHeader), C.POINTER(sz)]),
        "oracle_apply_mask": (None, [vp, sz, vp]),
        "oracle_conn_new": (vp, [C.c_int, C.c_int, C.c_int, C.c_int]),
        "oracle_conn_free": (None, [vp]),
        "oracle_conn_set_wrapper": (None, [vp, C.c_int]),
        "oracle_conn_set_digest": (None, [vp, C.c_int]),
        "oracle_conn_set_recv_state": (C.c_int, [vp, sz, vp, sz]),
        "oracle_conn_state": (C.c_int, [vp]),
        "oracle_conn_last_reason": (C.c_int, [vp]),
        "oracle_conn_n_events": (u64, [vp]),
        "oracle_conn_n_messages": (u64, [vp]),
        "oracle_conn_digest": (u64, [vp]),
        "oracle_conn_recv_pos": (sz, [vp]),
        "oracle_conn_recv_size": (sz, [vp]),
        "oracle_conn_frag_size": (sz, [vp]),
        "oracle_conn_frag_opcode": (C.c_int, [vp]),
        "oracle_conn_frag_pending": (C.c_int, [vp]),
        "oracle_conn_frag_capacity": (sz, [vp]),
        "oracle_conn_recv_bytes": (sz, [vp, vp, sz]),
        "oracle_conn_events": (sz, [vp, vp, sz]),
        "oracle_process_data": (C.c_int, [vp, vp, sz]),
        "oracle_decode_batch": (C.c_int, [vp, u64, vp, u64, u32, C.c_int, C.c_int, C.c_int, vp,
                                          u64, vp, vp, vp, vp, C.POINTER(OrcSummary)]),
        "oracle_gen_stride": (u64, [u64]),
        "oracle_build_frame": (C.c_long, [vp, sz, vp, sz, C.c_int, C.c_int, C.c_int, vp]),
        "oracle_gen_key": (u32, [u64, u32, C.c_int]),
        "oracle_gen_frames": (None, [vp, u32, u32, u32, u64, u64, C.c_int, C.c_int, C.c_int]),
        "oracle_gen_plain": (None, [vp, u32, u64, u64]),
        "oracle_unmask_frames": (u64, [vp, u32, u64]),
        "oracle_stream_decode": (u64, [vp, u64, sz, C.c_int, C.c_int, C.POINTER(u64)]),
        "oracle_decode_streams": (u64, [vp, vp, u32, vp, vp, vp, u64, C.c_int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _ = i32
    _L = L
    return L


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else None


def parse_frame_header(data: bytes, length=None, null=None):
    L = load()
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
    n = len(data) if length is None else length
    h, hs = OrcHeader(), C.c_size_t(0)
    rc = L.oracle_parse_frame_header(None if null == "data" else buf, n,
                                     None if null == "header" else C.byref(h),
                                     None if null == "header_size" else C.byref(hs))
    return rc, h, hs.value


def apply_mask(data: bytearray, key, length=None, null=None):
    L = load()
    n = len(data) if length is None else length
    buf = (C.c_uint8 * max(1, len(data))).from_buffer(data) if len(data) else None
    kb = (C.c_uint8 * 4).from_buffer_copy(bytes(key)) if key else None
    L.oracle_apply_mask(None if null == "data" else buf, n, None if null == "key" else kb)
    return data


EV_MESSAGE, EV_CLOSE, EV_PONG, EV_CLOSE_ECHO = 1, 2, 3, 4


class OracleConn:
    def __init__(self, is_server=1, max_frame_size=16 * 1024 * 1024,
                 max_message_size=64 * 1024 * 1024, record=1, wrapper=False):
        self.L = load()
        self.c = self.L.oracle_conn_new(is_server, max_frame_size, max_message_size, record)
        if wrapper:
            self.L.oracle_conn_set_wrapper(self.c, 1)

    def set_recv_state(self, size, fill: bytes, pos):
        buf = (C.c_uint8 * max(1, pos)).from_buffer_copy(fill[:pos] + b"\0" * (pos - len(fill[:pos])) if pos else b"\0")
        return self.L.oracle_conn_set_recv_state(self.c, size, buf, pos)

    def process_data(self, data: bytes, length=None, null=False):
        buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(bytes(data) or b"\0")
        n = len(data) if length is None else length
        return self.L.oracle_process_data(self.c, None if null else buf, n)

    @property
    def state(self):
        return self.L.oracle_conn_state(self.c)

    @property
    def recv_size(self):
        return self.L.oracle_conn_recv_size(self.c)

    @property
    def recv_pos(self):
        return self.L.oracle_conn_recv_pos(self.c)

    def recv_bytes(self) -> bytes:
        n = self.L.oracle_conn_recv_pos(self.c)
        buf = (C.c_uint8 * max(1, n))()
        self.L.oracle_conn_recv_bytes(self.c, buf, n)
        return bytes(buf)[:n]

    @property
    def frag_size(self):
        return self.L.oracle_conn_frag_size(self.c)

    @property
    def frag_opcode(self):
        return self.L.oracle_conn_frag_opcode(self.c)

    @property
    def frag_capacity(self):
        return self.L.oracle_conn_frag_capacity(self.c)

    @property
    def frag_pending(self):
        return bool(self.L.oracle_conn_frag_pending(self.c))

    def process_reads(self, reads):
        """The reference's on_websocket_read loop: process_data per read until a call fails
        (src/uvhttp_connection.c:1128-1164).  -> (rc of the last call, calls that ran)."""
        rc, calls = 0, 0
        for r in reads:
            calls += 1
            rc = self.process_data(r)
            if rc != 0:
                break
        return rc, calls

    @property
    def last_reason(self):
        return self.L.oracle_conn_last_reason(self.c)

    def events(self):
        n = self.L.oracle_conn_events(self.c, None, 0)
        raw = (C.c_uint8 * max(1, n))()
        self.L.oracle_conn_events(self.c, raw, n)
        b = bytes(raw)[:n]
        out, i = [], 0
        while i < n:
            typ = b[i]
            a = int.from_bytes(b[i + 1:i + 5], "little", signed=True)
            ln = int.from_bytes(b[i + 5:i + 13], "little")
            payload = b[i + 13:i + 13 + ln]
            i += 13 + ln
            name = {EV_MESSAGE: "message", EV_CLOSE: "close", EV_PONG: "pong",
                    EV_CLOSE_ECHO: "close_echo"}[typ]
            out.append((name, a, payload))
        return out

    def __del__(self):
        try:
            self.L.oracle_conn_free(self.c)
        except Exception:
            pass


def decode_batch(wire: np.ndarray, n_frames, stride=None, offsets=None, wire_len=None,
                 max_frame_size=16 * 1024 * 1024, max_message_size=64 * 1024 * 1024,
                 is_server=1, compact=False, arena_cap=None):
    """Oracle batch decode; returns dict(wire=…, arena=…, status=…, summary=…, msgs=…).
    `wire` is copied (the caller's array is not modified)."""
    L = load()
    w = np.array(wire, dtype=np.uint8, copy=True)
    wl = w.size if wire_len is None else wire_len
    status = np.zeros(max(1, n_frames), dtype=np.int8)
    msg_off = np.zeros(max(1, n_frames), dtype=np.uint64)
    msg_len = np.zeros(max(1, n_frames), dtype=np.uint64)
    msg_op = np.zeros(max(1, n_frames), dtype=np.int32)
    arena = None
    if compact:
        cap = w.size if arena_cap is None else arena_cap
        arena = np.zeros(max(1, cap), dtype=np.uint8)
    offs = None if offsets is None else np.ascontiguousarray(offsets, dtype=np.uint64)
    s = OrcSummary()
    L.oracle_decode_batch(_ptr(w), wl, _ptr(offs), stride or 0, n_frames, max_frame_size,
                          max_message_size, is_server, _ptr(arena),
                          0 if arena is None else arena.size, _ptr(status), _ptr(msg_off),
                          _ptr(msg_len), _ptr(msg_op), C.byref(s))
    sd = s.as_dict()
    nm = sd["n_messages"]
    return dict(wire=w, arena=arena, status=status[:n_frames], summary=sd,
                msg_off=msg_off[:nm], msg_len=msg_len[:nm], msg_opcode=msg_op[:nm])


STREAM_DT = np.dtype([("begin", "<u8"), ("len", "<u8"), ("recv_buffer_size", "<u8"),
                      ("pending_bytes", "<u8"), ("pending_opcode", "<i4"),
                      ("max_frame_size", "<i4"), ("max_message_size", "<i4"),
                      ("is_server", "<i4"), ("first_read", "<u4"), ("n_reads", "<u4"),
                      ("reserved", "<u8")])
STREAM_OUT_DT = np.dtype([("n_frames", "<u4"), ("calls", "<u4"), ("rc", "<i4"), ("reason", "<i4"),
                          ("consumed", "<u8"), ("recv_pos", "<u8"), ("recv_size", "<u8"),
                          ("frag_size", "<u8"), ("frag_opcode", "<i4"), ("n_messages", "<u4"),
                          ("digest", "<u8")])
STREAM_FRAME_DT = np.dtype([("payload_off", "<u8"), ("payload_len", "<u8"), ("key", "<u4"),
                            ("opcode", "u1"), ("flags", "u1"), ("header_size", "u1"),
                            ("reserved", "u1"), ("conn", "<u4"), ("wire_len", "<u4")])
assert STREAM_DT.itemsize == 64 and STREAM_OUT_DT.itemsize == 64
assert STREAM_FRAME_DT.itemsize == 32


def decode_streams(wire: np.ndarray, streams: np.ndarray, read_end=None, max_frames=None,
                   digest=False):
    """Oracle of uvhttp_ws_gpu_decode_streams / _decode_reads: every connection fed its
    process_data calls (one per read, until a call fails).  `wire` (uint8) is decoded IN
    PLACE (completed frames' payloads unmasked).  -> (per-connection outcomes STREAM_OUT_DT,
    completed frames STREAM_FRAME_DT in connection order)."""
    L = load()
    assert wire.dtype == np.uint8 and wire.flags.c_contiguous
    st = np.ascontiguousarray(streams).view(STREAM_DT)
    n = st.size
    re = None if read_end is None else np.ascontiguousarray(read_end, dtype=np.uint64)
    out = np.zeros(max(1, n), STREAM_OUT_DT)
    cap = max_frames if max_frames is not None else 0
    frames = np.zeros(max(1, cap), STREAM_FRAME_DT)
    total = L.oracle_decode_streams(_ptr(wire), _ptr(st), n, _ptr(re), _ptr(out),
                                    _ptr(frames) if cap else None, cap, 1 if digest else 0)
    return out[:n], frames[:min(total, cap)], int(total)


def gen_frames(n_frames, payload_len, seed, opcode0=2, fragmented=False, force_keys=False,
               first=0, count=None, total=None):
    L = load()
    stride = int(L.oracle_gen_stride(payload_len))
    count = n_frames if count is None else count
    total = n_frames if total is None else total
    out = np.empty(stride * count, dtype=np.uint8)
    L.oracle_gen_frames(_ptr(out), first, count, total, payload_len, seed, opcode0,
                        1 if fragmented else 0, 1 if force_keys else 0)
    return out, stride


def gen_plain(i, payload_len, seed):
    L = load()
    out = np.empty(max(1, payload_len), dtype=np.uint8)
    L.oracle_gen_plain(_ptr(out), i, payload_len, seed)
    return out[:payload_len]


def build_frame(payload: bytes, opcode, mask, fin, key=b"\x00\x00\x00\x00", cap=None):
    """oracle_build_frame -> (rc, bytes)"""
    L = load()
    cap = len(payload) + 14 if cap is None else cap
    out = (C.c_uint8 * max(1, cap))()
    src = (C.c_uint8 * max(1, len(payload))).from_buffer_copy(payload or b"\0")
    kb = (C.c_uint8 * 4).from_buffer_copy(bytes(key))
    rc = L.oracle_build_frame(out, cap, src if payload else None, len(payload), opcode, mask,
                              fin, kb)
    return rc, bytes(out)[: max(rc, 0)]


# ---- TLS record layer (oracle/tls_oracle.c), layouts of include/uvhttp_tls_amd.h ----------

TLS_KEY_DT = np.dtype([("key", "u1", 32), ("iv", "u1", 12), ("key_len", "<u4"),
                       ("version", "<u4"), ("cipher", "<u4"), ("reserved", "<u4", 2)])
TLS_STREAM_DT = np.dtype([("begin", "<u8"), ("len", "<u8"), ("seq", "<u8"), ("key", "<u4"),
                          ("ws_prefix", "<u4")])
TLS_RECORD_DT = np.dtype([("rec_off", "<u8"), ("out_off", "<u8"), ("content_len", "<u4"),
                          ("stream", "<u4"), ("type", "u1"), ("status", "i1"),
                          ("reserved", "<u2"), ("reserved2", "<u4")])
TLS_RESULT_DT = np.dtype([("first_record", "<u4"), ("n_records", "<u4"),
                          ("n_delivered", "<u4"), ("status", "<i4"), ("first_status", "<i4"),
                          ("reserved", "<u4"), ("consumed_bytes", "<u8"), ("next_seq", "<u8"),
                          ("out_off", "<u8"), ("plain_len", "<u8"), ("reserved3", "<u8")])
TLS_SEAL_DT = np.dtype([("src_off", "<u8"), ("out_off", "<u8"), ("seq", "<u8"),
                        ("plain_len", "<u4"), ("key", "<u2"), ("type", "u1"),
                        ("reserved", "u1")])
assert TLS_KEY_DT.itemsize == 64 and TLS_STREAM_DT.itemsize == 32
assert TLS_RECORD_DT.itemsize == 32 and TLS_RESULT_DT.itemsize == 64
assert TLS_SEAL_DT.itemsize == 32

TLS12, TLS13 = 0x0303, 0x0304
AES_GCM, CHACHA = 0, 1
REC_OK, REC_SKIPPED, REC_CONTROL = 0, 2, 3
REC_OVERFLOW, REC_BAD_MAC, REC_BAD_TYPE, REC_VERSION = -1, -2, -3, -4
REC_EMPTY, REC_CAPACITY, REC_KEY = -5, -6, -7


def _tls_sigs(L):
    vp, u32, u64, sz = C.c_void_p, C.c_uint32, C.c_uint64, C.c_size_t
    for name, res, args in [
        ("oracle_aes_encrypt_block", C.c_int, [vp, C.c_int, vp, vp]),
        ("oracle_aes_sbox", C.c_uint8, [C.c_uint8]),
        ("oracle_gf_mult", None, [vp, vp, vp]),
        ("oracle_gcm", C.c_int, [vp, C.c_int, vp, vp, sz, vp, sz, vp, vp, C.c_int]),
        ("oracle_tls_open_batch", u64, [vp, u64, vp, u32, vp, u32, vp, u32, vp, vp, u64]),
        ("oracle_tls_seal_record", u64, [vp, u64, C.c_uint8, vp, u32, u32, vp]),
        ("oracle_tls_open_stream_bytes", u64, [vp, u64, vp, u64, vp]),
        ("oracle_chacha20_block", None, [vp, u32, vp, vp]),
        ("oracle_poly1305", None, [vp, vp, sz, vp]),
        ("oracle_chachapoly", C.c_int, [vp, vp, vp, sz, vp, sz, vp, vp, C.c_int]),
    ]:
        fn = getattr(L, name)
        fn.restype, fn.argtypes = res, args
    return L


def _buf(b: bytes):
    return (C.c_uint8 * max(1, len(b))).from_buffer_copy(bytes(b) or b"\0")


def aes_encrypt_block(key: bytes, block: bytes) -> bytes:
    L = _tls_sigs(load())
    out = (C.c_uint8 * 16)()
    assert L.oracle_aes_encrypt_block(_buf(key), len(key), _buf(block), out) == 0
    return bytes(out)


def gcm(key: bytes, iv: bytes, aad: bytes, data: bytes, tag: bytes = None, decrypt=False):
    """AES-GCM: encrypt -> (ct, tag); decrypt -> (rc, pt) (rc -2 on a tag mismatch)"""
    L = _tls_sigs(load())
    out = (C.c_uint8 * max(1, len(data)))()
    t = _buf(tag or bytes(16))
    rc = L.oracle_gcm(_buf(key), len(key), _buf(iv), _buf(aad), len(aad), _buf(data),
                      len(data), out, t, 1 if decrypt else 0)
    if decrypt:
        return rc, bytes(out)[:len(data)]
    return bytes(out)[:len(data)], bytes(t)


def tls_key(key: bytes, iv: bytes, version, cipher=AES_GCM):
    k = np.zeros(1, TLS_KEY_DT)
    k[0]["key"][:len(key)] = np.frombuffer(key, np.uint8)
    k[0]["iv"][:] = np.frombuffer(iv.ljust(12, b"\0"), np.uint8)
    k[0]["key_len"] = len(key)
    k[0]["version"] = version
    k[0]["cipher"] = cipher
    return k


def chacha20_block(key: bytes, counter: int, nonce: bytes) -> bytes:
    L = _tls_sigs(load())
    out = (C.c_uint8 * 64)()
    L.oracle_chacha20_block(_buf(key), counter, _buf(nonce), out)
    return bytes(out)


def poly1305(key: bytes, msg: bytes) -> bytes:
    L = _tls_sigs(load())
    out = (C.c_uint8 * 16)()
    L.oracle_poly1305(_buf(key), _buf(msg), len(msg), out)
    return bytes(out)


def chachapoly(key: bytes, nonce: bytes, aad: bytes, data: bytes, tag: bytes = None,
               decrypt=False):
    """AEAD_CHACHA20_POLY1305: encrypt -> (ct, tag); decrypt -> (rc, pt)"""
    L = _tls_sigs(load())
    out = (C.c_uint8 * max(1, len(data)))()
    t = _buf(tag or bytes(16))
    rc = L.oracle_chachapoly(_buf(key), _buf(nonce), _buf(aad), len(aad), _buf(data), len(data),
                             out, t, 1 if decrypt else 0)
    if decrypt:
        return rc, bytes(out)[:len(data)]
    return bytes(out)[:len(data)], bytes(t)


def tls_seal(keyrec, seq, type_, content: bytes, pad=0) -> bytes:
    L = _tls_sigs(load())
    out = (C.c_uint8 * (len(content) + pad + 64))()
    n = L.oracle_tls_seal_record(_ptr(keyrec), seq, type_, _buf(content), len(content), pad, out)
    assert n > 0
    return bytes(out)[:n]


def tls_open_batch(wire: np.ndarray, keys: np.ndarray, streams: np.ndarray, max_records=None,
                   out_cap=None):
    """Oracle of uvhttp_tls_gpu_open_records -> (records, results, out)"""
    L = _tls_sigs(load())
    w = np.ascontiguousarray(wire, dtype=np.uint8)
    max_records = max(1, w.size // 5 + 1) if max_records is None else max_records
    out_cap = w.size if out_cap is None else out_cap
    recs = np.zeros(max(1, max_records), TLS_RECORD_DT)
    res = np.zeros(max(1, len(streams)), TLS_RESULT_DT)
    out = np.zeros(max(1, out_cap), np.uint8)
    n = L.oracle_tls_open_batch(_ptr(w), w.size, _ptr(keys), len(keys), _ptr(streams),
                                len(streams), _ptr(recs), max_records, _ptr(res), _ptr(out),
                                out_cap)
    return recs[:n], res[:len(streams)], out


def tls_open_stream_bytes(keyrec, seq, wire: np.ndarray, out: np.ndarray) -> int:
    L = _tls_sigs(load())
    return int(L.oracle_tls_open_stream_bytes(_ptr(keyrec), seq, _ptr(wire), wire.size,
                                              _ptr(out)))
