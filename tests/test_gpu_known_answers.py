"""The HIP path pinned directly to the reference's own known answers
(tests/golden/reference_known_answers.json, transcribed from test/unit/test_websocket_*.cpp),
not only through the oracle:

* every process_data scenario (including the recv-buffer `pre` pokes and config limits)
  through the device batcher: each feed is one device flush (uvhttp_ws_gpu_decode_reads),
  the reference test's expected return codes, callbacks, close codes, payloads and buffer
  growth are asserted on what the flush delivered;
* the scenarios whose feeds are each exactly one frame, as ONE decode_inplace batch (frame k
  = feed k, the batch contract), delivered with uvhttp_ws_deliver_batch;
* the parse_frame_header cases through decode_inplace (one-frame batches: the descriptor's
  header fields) and the apply_mask cases through uvhttp_ws_gpu_apply_mask;
* the full-size C2 / C4 batches: the device summary and every frame status field by field
  against the oracle's process_data-per-frame batch decode (decode_batch), not only bytes.
"""
import ctypes as C

import numpy as np
import pytest

import _known
import _oracle

pytestmark = pytest.mark.gpu


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
    yield e
    e.close()


class _BatcherAdapter:
    """check_process_case adapter: every feed is one device flush of a batcher."""

    def __init__(self, cfg, callbacks):
        import uvhttp_amd as U
        self.c = U.WsConnection(1, cfg["max_frame_size"], cfg["max_message_size"],
                                callbacks=callbacks)
        self.b = U.Batcher(device=0, min_device_bytes=0)
        self.feeds = 0

    def process(self, data):
        rc = self.b.submit(self.c, data)
        assert self.b.flush() == 0
        self.feeds += 1
        key = C.addressof(self.c.ptr.contents)
        return -1 if key in self.b.failures else rc

    def events(self):
        return list(self.c.events)

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
def test_process_known_answers_device_batcher(torch, known_answers, idx):
    cases = known_answers["process_data"]
    if idx >= len(cases):
        pytest.skip("no case")
    made = []

    def make(cfg, callbacks):
        a = _BatcherAdapter(cfg, callbacks)
        made.append(a)
        return a

    _known.check_process_case(cases[idx], make)
    st = made[0].b.stats()
    # every feed was decoded by the device (no host decoder involved)
    assert st["device_flushes"] == made[0].feeds and st["host_reads"] == 0, st
    made[0].b.close()


def _one_frame_feeds(case):
    """the case's feeds when each is exactly one complete frame (else None)"""
    import uvhttp_amd as U
    out = []
    for fd in case["feeds"]:
        data = bytes.fromhex(fd["hex"])
        rc, h, hs = U.parse_frame_header(data, None, None)
        if rc != 0:
            return None
        if hs + (4 if h.mask else 0) + h.payload_length != len(data):
            return None
        out.append(data)
    return out


def test_process_known_answers_decode_inplace(torch, eng, known_answers):
    """feeds of one frame each -> one batch; the batch contract (process_data per frame, in
    order, on one connection) makes the device's delivery the reference test's outcome"""
    import uvhttp_amd as U
    ran = 0
    for case in known_answers["process_data"]:
        if case.get("pre"):
            continue  # a poked recv buffer is not a batch input (covered by the batcher test)
        feeds = _one_frame_feeds(case)
        if not feeds:
            continue
        cfg = dict(_known.DEFAULTS)
        cfg.update(case.get("config") or {})
        wire = b"".join(feeds)
        offs = np.cumsum([0] + [len(f) for f in feeds[:-1]]).astype(np.uint64)
        d = torch.from_numpy(np.frombuffer(wire + bytes(64 - len(wire) % 16 + 16), np.uint8).copy()).to("cuda")
        o = torch.from_numpy(offs.view(np.int64)).to("cuda")
        desc, summ = eng.decode_inplace(d, len(feeds), offsets=o, wire_len=len(wire),
                                        max_frame_size=cfg["max_frame_size"],
                                        max_message_size=cfg["max_message_size"])
        torch.cuda.synchronize()
        s = eng.read_summary(summ)
        # the first feed the reference test expects to fail is the batch's first failure
        bad = [k for k, fd in enumerate(case["feeds"]) if fd["expect_rc"] != 0]
        assert s["n_delivered"] == (bad[0] if bad else len(feeds)), case["id"]
        assert s["status"] == (-1 if bad else 0), case["id"]
        # deliver to a product connection and check the test's expectations
        conn = U.WsConnection(1, cfg["max_frame_size"], cfg["max_message_size"],
                              callbacks=not case.get("no_callbacks"))
        hw = (C.c_uint8 * len(wire)).from_buffer_copy(d[:len(wire)].cpu().numpy().tobytes())
        hd = (C.c_uint8 * (32 * len(feeds))).from_buffer_copy(desc[:32 * len(feeds)].cpu().numpy().tobytes())
        hs = (C.c_uint8 * C.sizeof(U.BatchSummary)).from_buffer_copy(summ.cpu().numpy().tobytes())
        rc = U.lib().uvhttp_ws_deliver_batch(conn.ptr, C.cast(hw, C.c_void_p),
                                             C.cast(hd, C.c_void_p), C.cast(hs, C.c_void_p))
        assert rc == (-1 if bad else 0), case["id"]
        _known.check_expectations(case, list(conn.events), conn.struct.state,
                                  lambda: conn.struct.recv_buffer_size)
        ran += 1
    assert ran >= 15, ran


def test_parse_known_answers_device(torch, eng, known_answers):
    """each parse case as a one-frame batch (client side, so unmasked frames are legal): the
    descriptor carries the parsed header; rc -1 <-> the device could not parse the header
    (too short: no wire length; 64-bit length with the MSB set: ERR_PARSE)"""
    ran = 0
    for case in known_answers["parse_frame_header"]:
        if case.get("null"):
            continue  # NULL-pointer arguments are host-API cases
        data = bytes.fromhex(case["bytes"])
        n = case.get("length", len(data))
        d = torch.from_numpy(np.frombuffer(data + bytes(64), np.uint8).copy()).to("cuda")
        desc, summ = eng.decode_inplace(d, 1, stride=max(1, n), wire_len=n, is_server=0,
                                        max_frame_size=2 ** 31 - 1)
        torch.cuda.synchronize()
        r = eng.read_desc(desc, 1)[0]
        parsed = int(r["status"]) != -1 and int(r["wire_len"]) > 0
        exp = case["expect"]
        assert (0 if parsed else -1) == exp["rc"], case["id"]
        ran += 1
        if not parsed:
            continue
        hsz = int(r["header_size"])
        got = {"fin": int(r["flags"]) & 1, "mask": (int(r["flags"]) >> 1) & 1,
               "opcode": int(r["opcode"]), "header_size": hsz,
               "payload_length": int(r["payload_len"]),
               "len_code": int(r["payload_len"]) if hsz == 2 else (126 if hsz == 4 else 127)}
        for k, v in exp.items():
            if k != "rc":
                assert got[k] == v, (case["id"], k)
    assert ran == 16, ran  # every case but the three NULL-argument ones


@pytest.mark.parametrize("offset", [0, 1, 7])
def test_mask_known_answers_device(torch, eng, known_answers, offset):
    """uvhttp_ws_gpu_apply_mask on each case's bytes (at several alignments)"""
    for case in known_answers["apply_mask"]:
        if case.get("null"):
            continue
        data = bytes.fromhex(case["data"])
        n = case.get("length", len(data))
        key = bytes.fromhex(case["key"])
        buf = torch.from_numpy(np.frombuffer(bytes(offset) + data + bytes(32), np.uint8).copy()).to("cuda")
        if n:
            eng.apply_mask(buf, key, length=n, offset=offset)
        torch.cuda.synchronize()
        out = bytes(buf[offset:offset + len(data)].cpu().numpy())
        if "expect_after" in case:
            assert out == bytes.fromhex(case["expect_after"]), case["id"]
        if case.get("differs"):
            assert out != data, case["id"]
        for i, v in case.get("checks", {}).items():
            assert out[int(i)] == v, case["id"]
        if case.get("roundtrip"):
            eng.apply_mask(buf, key, length=n, offset=offset)
            torch.cuda.synchronize()
            assert bytes(buf[offset:offset + len(data)].cpu().numpy()) == data, case["id"]


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4"])
def test_full_config_summary_vs_oracle_decode_batch(torch, eng, cfg):
    """BASELINE C2 / C3 / C4 at full size: the device summary and all frame statuses equal the
    oracle's process_data-per-frame decode of the identical frames, field by field (C4 also
    with the default 64 MiB max_message_size, where the reference rejects frame 262 144)."""
    import uvhttp_amd as U
    n, plen, frag = {"c2": (65536, 4096, False), "c3": (65536, 65536, False),
                     "c4": (1048576, 256, True)}[cfg]
    stride = U.gen_frame_stride(plen)
    wl = stride * n
    host, _ = _oracle.gen_frames(n, plen, 0x5EED0001, fragmented=frag, force_keys=True, total=n)
    for mm in ([256 << 20, 64 << 20] if frag else [64 << 20]):
        d = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
        eng.gen_frames(d, n, plen, 0x5EED0001, opcode0=2, fragmented=frag, force_keys=True)
        desc, summ = eng.decode_inplace(d, n, stride=stride, max_message_size=mm, wire_len=wl)
        torch.cuda.synchronize()
        ref = _oracle.decode_batch(host, n, stride=stride, max_message_size=mm)
        got = eng.read_summary(summ)
        assert got == ref["summary"], (cfg, mm)
        st = eng.read_desc(desc, n)["status"]
        assert np.array_equal(st, ref["status"]), (cfg, mm)
        if mm == 64 << 20 and frag:
            assert got["n_delivered"] == 262144
        assert np.array_equal(d[:wl].cpu().numpy(), ref["wire"]), (cfg, mm)
