"""Device-side kernel stamps (uvhttp_ws_gpu_engine_set_stamps / _read_stamps, include/
uvhttp_ws_amd.h): with stamps on, every kernel of a call leaves one (call, kernel, begin, end)
record on the GPU's wall clock; calls come back in order, kernels of a call in start order and
never overlapping (one stream), and the ring keeps the last 128 calls.  Stamps change nothing
in the results (the decode is checked against the summary the oracle expects)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


def _wire(torch, U, eng, n, plen, frag=False):
    stride = U.gen_frame_stride(plen)
    wire = torch.empty(stride * n + 64, dtype=torch.uint8, device="cuda")
    eng.gen_frames(wire, n, plen, 11, opcode0=2, fragmented=frag)
    return wire, stride


def _check_calls(recs, kernels_expected, calls):
    by_call = {}
    for call, kern, b, e in recs:
        assert e >= b, (call, kern, b, e)
        by_call.setdefault(call, []).append((b, e, kern))
    assert len(by_call) == calls
    order = list(by_call)  # read_stamps returns the oldest call first (tags wrap at 2^24 - 1)
    assert all(1 <= c < (1 << 24) for c in order)
    assert [(c - order[0]) % ((1 << 24) - 1) for c in order] == list(range(calls))  # consecutive
    prev_end = 0
    for c in order:
        ks = sorted(by_call[c])
        assert {k for _, _, k in ks} >= kernels_expected, ks
        for (b0, e0, _), (b1, _, _) in zip(ks, ks[1:]):
            assert b1 >= e0 - 2000, ks  # one stream: a kernel starts after the previous ends
        assert ks[0][0] >= prev_end - 2000
        prev_end = ks[-1][1]


@pytest.mark.parametrize("calls", [1, 5, 130])
def test_stamps_batch_in_place(torch, calls):
    import uvhttp_amd as U
    eng = U.GpuEngine(0)
    try:
        for plen, kern in ((65536, {"plan", "payload"}), (256, {"payload", "sum_scan", "desc_emit"})):
            n = 4096 if plen == 65536 else 65536
            wire, stride = _wire(torch, U, eng, n, plen, frag=plen == 256)
            desc, summ = eng.alloc_outputs(n)
            eng.set_stamps(True)
            eng.read_stamps()
            for _ in range(calls):
                eng.decode_inplace(wire, n, stride=stride, max_message_size=0, wire_len=n * stride,
                                   desc=desc, summary=summ)
            torch.cuda.synchronize()
            recs = eng.read_stamps()
            eng.set_stamps(False)
            _check_calls(recs, kern, min(calls, 128))
            assert eng.read_summary(summ)["n_delivered"] == n
            assert eng.read_stamps() == []  # read_stamps cleared the ring
    finally:
        eng.close()


@pytest.mark.parametrize("fuse", ["1", "0"])
def test_stamps_stream_decode(torch, fuse):
    """the wave walk, its scan and k_stream_desc, or with UVHTTP_WS_WALK_FUSE=1 the one
    launch of k_swalk_fused (stamped as "walk")"""
    import os
    import numpy as np
    import uvhttp_amd as U
    old = os.environ.get("UVHTTP_WS_WALK_FUSE")
    os.environ["UVHTTP_WS_WALK_FUSE"] = fuse
    try:
        eng = U.GpuEngine(0)
    finally:
        if old is None:
            os.environ.pop("UVHTTP_WS_WALK_FUSE", None)
        else:
            os.environ["UVHTTP_WS_WALK_FUSE"] = old
    try:
        n, plen = 8192, 4096
        wire, stride = _wire(torch, U, eng, n, plen)
        st = np.zeros(n, dtype=U.STREAM_DT)
        st["begin"] = np.arange(n, dtype=np.uint64) * stride
        st["len"] = stride
        st["recv_buffer_size"] = 65536
        st["max_frame_size"], st["max_message_size"], st["is_server"] = 16 << 20, 0, 1
        sdev = torch.from_numpy(st.view(np.uint8).copy()).to("cuda")
        eng.set_stamps(True)
        eng.read_stamps()
        for _ in range(3):
            desc, res = eng.decode_streams(wire, sdev, n, n, wire_len=n * stride)
        torch.cuda.synchronize()
        recs = eng.read_stamps()
        eng.set_stamps(False)
        _check_calls(recs, {"walk", "payload"} if fuse == "1" else
                     {"walk", "walk_scan", "stream_desc", "payload"}, 3)
        r = eng.read_stream_results(res, n)
        assert all(x.status == 0 and x.n_delivered == 1 for x in r)
    finally:
        eng.close()


def test_stamps_send_side(torch):
    """the send side stamps its kernels too: kb_size, the block scan and the emit kernel (as
    "payload"; the tile emit adds kb_offsets), one call after another"""
    import numpy as np
    import uvhttp_amd as U
    eng = U.GpuEngine(0)
    try:
        for n, plen, kinds in ((65536, 256, {"build_size", "build_scan", "payload"}),
                               (2048, 16384, {"build_size", "build_scan", "build_offsets", "payload"})):
            fr = np.zeros(n, dtype=[("po", "<u8"), ("pl", "<u8"), ("key", "<u4"), ("op", "u1"),
                                    ("fin", "u1"), ("mask", "u1"), ("r0", "u1"), ("r1", "<u8")])
            fr["po"] = np.arange(n, dtype=np.uint64) * plen
            fr["pl"], fr["op"], fr["fin"] = plen, 2, 1
            d = torch.from_numpy(fr.view(np.uint8).copy()).to("cuda")
            src = torch.randint(0, 256, (n * plen + 64,), dtype=torch.uint8, device="cuda")
            out = torch.zeros(n * (plen + 14) + 64, dtype=torch.uint8, device="cuda")
            eng.set_stamps(True)
            eng.read_stamps()
            for _ in range(3):
                off = eng.build_frames(src, d, n, out)
            torch.cuda.synchronize()
            recs = eng.read_stamps()
            eng.set_stamps(False)
            _check_calls(recs, kinds, 3)
            assert int(off[n].item()) == n * (plen + (2 if plen < 126 else 4 if plen < 65536 else 10))
    finally:
        eng.close()
