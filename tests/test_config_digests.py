"""BASELINE configs pinned by committed SHA-256 digests (tests/golden/config_digests.json,
made by tests/golden/make_config_digests.py from the oracle).

CPU: the oracle still reproduces the committed digests (C2, C4, the C5 sample).
GPU: the device generator and both device decodes reproduce them with no oracle in the loop:
masked wire, in-place decoded wire, and the compact payload stream (for C4 the reassembled
256 MiB message)."""
import hashlib
import json
import os

import pytest

import _oracle

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "config_digests.json")) as _fh:
    DIG = json.load(_fh)


def _mk():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "make_config_digests", os.path.join(HERE, "golden", "make_config_digests.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("cfg", ["c2", "c4"])
def test_oracle_reproduces_digests(cfg):
    m = _mk()
    d = DIG[cfg]
    got = m.config_digests(d["frames"], d["payload_len"], d["fragmented"])
    assert got == d


def test_oracle_reproduces_c5_sample():
    want = {k: DIG["c5_pass"][k] for k in ("frames", "payload_len", "sample", "payload_sample")}
    assert _mk().c5_digest() == want
    _ = _oracle  # oracle library built by the fixture chain


def test_oracle_reproduces_c5_chunks():
    """three of the 256 chunk digests of the whole C5 pass (the GPU test checks all of them)"""
    import hashlib
    m = _mk()
    c5 = DIG["c5_pass"]
    chunks = c5["decoded_chunks"]
    assert len(chunks) * c5["chunk_frames"] == c5["frames"]
    assert hashlib.sha256("".join(chunks).encode()).hexdigest() == c5["decoded"]
    for k in (0, 127, len(chunks) - 1):
        assert m.c5_chunk_digest(k) == chunks[k], k


def _sha_dev(t, nbytes, chunk=256 << 20):
    h = hashlib.sha256()
    for o in range(0, nbytes, chunk):
        h.update(t[o:min(nbytes, o + chunk)].cpu().numpy())
    return h.hexdigest()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["c2", "c3", "c4"])
def test_device_reproduces_digests(cfg):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import uvhttp_amd as U
    d = DIG[cfg]
    n, plen, frag, stride = d["frames"], d["payload_len"], d["fragmented"], d["stride"]
    assert U.gen_frame_stride(plen) == stride
    eng = U.GpuEngine(0)
    try:
        wl = stride * n
        mm = 256 << 20
        wire = torch.empty(wl + 64, dtype=torch.uint8, device="cuda")
        eng.gen_frames(wire, n, plen, DIG["seed"], opcode0=2, fragmented=frag, force_keys=True)
        torch.cuda.synchronize()
        assert _sha_dev(wire, wl) == d["wire"]
        arena = torch.empty(n * plen + 64, dtype=torch.uint8, device="cuda")
        _, _, summ = eng.decode_compact(wire, n, arena, stride=stride, max_message_size=mm,
                                        wire_len=wl)
        torch.cuda.synchronize()
        s = eng.read_summary(summ)
        assert s["n_delivered"] == n and s["status"] == 0
        assert _sha_dev(arena, n * plen) == d["payload"]
        assert _sha_dev(wire, wl) == d["wire"]  # compact leaves the wire untouched
        _, summ = eng.decode_inplace(wire, n, stride=stride, max_message_size=mm, wire_len=wl)
        torch.cuda.synchronize()
        assert eng.read_summary(summ)["n_delivered"] == n
        assert _sha_dev(wire, wl) == d["decoded"]
    finally:
        eng.close()
