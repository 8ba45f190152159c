"""Batched send-side framing: uvhttp_ws_gpu_build_frames against the
oracle's restatement of uvhttp_ws_build_frame (src/uvhttp_websocket.c:204-285), the reference
tests' known answers, and build -> decode round trips."""
import random

import numpy as np
import pytest

import _oracle

pytestmark = pytest.mark.gpu

BUILD_DT = np.dtype([("payload_off", "<u8"), ("payload_len", "<u8"), ("key", "<u4"),
                     ("opcode", "u1"), ("fin", "u1"), ("mask", "u1"), ("r0", "u1"),
                     ("r1", "<u8")])


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


# emit path: the engine's automatic choice, the frame-grouped LDS kernel (kb_emit_frames) for
# every batch (including frames far larger than its LDS window), or the output-tile kernels
# (kb_emit) for every batch; UVHTTP_WS_BUILD_FRAMES is read when the engine is created
_PATHS = {"auto": None, "grouped": str(1 << 62), "tiles": "0"}


@pytest.fixture(scope="module", params=list(_PATHS))
def eng(torch, request):
    import os
    import uvhttp_amd as U
    old = os.environ.get("UVHTTP_WS_BUILD_FRAMES")
    if _PATHS[request.param] is None:
        os.environ.pop("UVHTTP_WS_BUILD_FRAMES", None)
    else:
        os.environ["UVHTTP_WS_BUILD_FRAMES"] = _PATHS[request.param]
    try:
        e = U.GpuEngine(0)
    finally:
        if old is None:
            os.environ.pop("UVHTTP_WS_BUILD_FRAMES", None)
        else:
            os.environ["UVHTTP_WS_BUILD_FRAMES"] = old
    yield e
    e.close()


GUARD = 256


def _build(torch, eng, src, frames, cap_extra=64, cap=None):
    total = 0
    exp = []
    for f in frames:
        payload = src[f["payload_off"]:f["payload_off"] + f["payload_len"]].tobytes()
        key = int(f["key"]).to_bytes(4, "little")
        rc, b = _oracle.build_frame(payload, int(f["opcode"]), int(f["mask"]), int(f["fin"]), key)
        assert rc == len(b)
        exp.append(b)
        total += rc
    cap = total + cap_extra if cap is None else cap
    dsrc = torch.from_numpy(src.copy()).to("cuda") if src.size else \
        torch.zeros(16, dtype=torch.uint8, device="cuda")
    dfr = torch.from_numpy(frames.view(np.uint8).copy()).to("cuda") if len(frames) else \
        torch.zeros(32, dtype=torch.uint8, device="cuda")
    size = max(16, cap)
    out = torch.zeros(size + GUARD, dtype=torch.uint8, device="cuda")
    out[size:] = 0xA5  # guard: nothing may be written past the caller's buffer
    src_before, fr_before = dsrc.clone(), dfr.clone()
    off = eng.build_frames(dsrc, dfr, len(frames), out[:cap] if cap else out[:0])
    torch.cuda.synchronize()
    host = out.cpu().numpy()
    assert (host[size:] == 0xA5).all(), "write past the output buffer"
    assert torch.equal(dsrc, src_before) and torch.equal(dfr, fr_before), "inputs modified"
    return exp, total, host[:size], off.cpu().numpy()


def _rand_frames(rng, src_len, n, sizes):
    fr = np.zeros(n, BUILD_DT)
    for i in range(n):
        p = min(rng.choice(sizes), src_len)
        fr[i]["payload_len"] = p
        fr[i]["payload_off"] = rng.randint(0, src_len - p) if src_len > p else 0
        fr[i]["key"] = rng.getrandbits(32)
        fr[i]["opcode"] = rng.choice([0, 1, 2, 8, 9, 10, 0x13])
        fr[i]["fin"] = rng.choice([0, 1])
        fr[i]["mask"] = rng.choice([0, 1])
    return fr


# cap_extra moves the caller's capacity per frame, which picks the emit shape and the output
# map granularity: every shape must handle frames much smaller and much larger than its map tile
@pytest.mark.parametrize("cap_extra", [64, 1 << 22])
@pytest.mark.parametrize("seed", range(8))
def test_build_matches_oracle(torch, eng, seed, cap_extra):
    rng = random.Random(seed)
    src = np.frombuffer(rng.randbytes(300000), np.uint8).copy()
    sizes = [[0, 1, 5, 125, 126, 127, 200], [1000, 4095, 65535, 65536, 70000],
             [0, 3, 300, 65536]][seed % 3]
    frames = _rand_frames(rng, src.size, rng.choice([1, 17, 300, 2000]), sizes)
    exp, total, out, off = _build(torch, eng, src, frames, cap_extra=cap_extra)
    assert int(off[len(frames)]) == total
    assert np.array_equal(off[:len(frames)], np.cumsum([0] + [len(b) for b in exp[:-1]]))
    assert out[:total].tobytes() == b"".join(exp)
    assert not out[total:].any()  # nothing past the frames


def test_build_capacity(torch, eng):
    rng = random.Random(5)
    src = np.frombuffer(rng.randbytes(5000), np.uint8).copy()
    frames = _rand_frames(rng, src.size, 40, [10, 100, 1000])
    exp, total, out, off = _build(torch, eng, src, frames, cap=100)
    assert int(off[len(frames)]) == total > 100
    assert not out.any()  # all-or-nothing, like build_frame's size check


def test_build_known_answers(torch, eng, known_answers):
    for case in known_answers["build_frame"]:
        if case["expect"]["rc"] < 0:
            continue
        fill = case["fill"].encode().decode("unicode_escape").encode("latin-1")
        payload = (fill * (case["length"] // len(fill) + 1))[: case["length"]]
        src = np.frombuffer(payload, np.uint8).copy()
        fr = np.zeros(1, BUILD_DT)
        fr[0]["payload_len"] = len(payload)
        fr[0]["key"] = 0x44332211
        fr[0]["opcode"], fr[0]["fin"], fr[0]["mask"] = case["opcode"], case["fin"], case["mask"]
        exp, total, out, off = _build(torch, eng, src, fr)
        assert total == case["expect"]["rc"], case["id"]
        head = bytes.fromhex(case["expect"]["head"])
        assert out[: len(head)].tobytes() == head, case["id"]
        assert out[:total].tobytes() == exp[0], case["id"]


def test_build_then_decode_roundtrip(torch, eng):
    """Client (masked) frames built on the device decode back to their payloads."""
    rng = random.Random(11)
    src = np.frombuffer(rng.randbytes(1 << 20), np.uint8).copy()
    frames = _rand_frames(rng, src.size, 500, [0, 7, 126, 4096, 65536])
    frames["mask"] = 1
    frames["opcode"] = 2
    frames["fin"] = 1
    exp, total, out, off = _build(torch, eng, src, frames)
    wire = torch.from_numpy(out.copy()).to("cuda")
    offs = torch.from_numpy(off[:len(frames)].astype(np.int64)).to("cuda")
    desc, summ = eng.decode_inplace(wire, len(frames), offsets=offs, wire_len=total)
    torch.cuda.synchronize()
    s = eng.read_summary(summ)
    assert s["n_delivered"] == len(frames) and s["status"] == 0
    d = eng.read_desc(desc, len(frames))
    w = wire.cpu().numpy()
    for i, f in enumerate(frames):
        got = w[d[i]["payload_off"]:d[i]["payload_off"] + d[i]["payload_len"]]
        assert np.array_equal(got, src[f["payload_off"]:f["payload_off"] + f["payload_len"]])


# uvhttp_server_ws_broadcast (src/uvhttp_server.c:1626-1657) sends ONE payload to every open
# connection through uvhttp_ws_send_text -> uvhttp_ws_send_frame (src/uvhttp_websocket.c:
# 509-531, 595-600): a TEXT frame, FIN set, masked only when the connection is a client's.
# As a batch that is n descriptors over the same source bytes.
@pytest.mark.parametrize("plen,n", [(1, 5000), (125, 2048), (126, 3000), (1000, 4096),
                                    (4096, 16384), (65535, 300), (65536, 257), (70000, 64)])
def test_broadcast_shared_payload(torch, eng, plen, n):
    rng = random.Random(plen * 7 + n)
    src = np.frombuffer(rng.randbytes(plen + 37), np.uint8).copy()
    for masked in (0, 1):  # server connections; client connections (each its own key)
        frames = np.zeros(n, BUILD_DT)
        frames["payload_off"], frames["payload_len"] = 37, plen
        frames["opcode"], frames["fin"], frames["mask"] = 1, 1, masked
        frames["key"] = [rng.getrandbits(32) for _ in range(n)]
        exp, total, out, off = _build(torch, eng, src, frames)
        assert int(off[n]) == total
        assert out[:total].tobytes() == b"".join(exp)
        if not masked:  # every connection receives the identical frame
            one = len(exp[0])
            assert total == n * one
            assert (out[:total].reshape(n, one) == np.frombuffer(exp[0], np.uint8)).all()
