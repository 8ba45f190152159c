"""Pins the oracle (oracle/ws_oracle.c) against the reference's own known-answer tests."""
import pytest

import _known
import _oracle


def test_oracle_parse_known_answers(known_answers):
    for case in known_answers["parse_frame_header"]:
        _known.check_parse_case(case, _oracle.parse_frame_header)


def test_oracle_mask_known_answers(known_answers):
    for case in known_answers["apply_mask"]:
        _known.check_mask_case(case, _oracle.apply_mask)


class _OracleAdapter:
    def __init__(self, cfg, callbacks):
        self.c = _oracle.OracleConn(1, cfg["max_frame_size"], cfg["max_message_size"], record=1)
        self.callbacks = callbacks

    def process(self, data):
        return self.c.process_data(data)

    def events(self):
        ev = self.c.events()
        return ev if self.callbacks else []

    def set_recv_state(self, size, fill, pos):
        assert self.c.set_recv_state(size, fill, pos) == 0

    @property
    def state(self):
        return self.c.state

    @property
    def recv_size(self):
        return self.c.recv_size


@pytest.mark.parametrize("idx", range(31))
def test_oracle_process_known_answers(known_answers, idx):
    cases = known_answers["process_data"]
    if idx >= len(cases):
        pytest.skip("no case")
    _known.check_process_case(cases[idx], _OracleAdapter)


def test_oracle_null_inputs():
    c = _oracle.OracleConn()
    assert c.process_data(b"", null=True) == -1  # test_websocket_boost_coverage.cpp:968-976


def test_oracle_generator_roundtrip():
    """Synthetic frames unmask to the documented plaintext (SURVEY §8(d) generator)."""
    import numpy as np
    for plen in (0, 5, 125, 126, 4096, 65535, 65536):
        wire, stride = _oracle.gen_frames(4, plen, 0x5EED0001, force_keys=True)
        out = _oracle.decode_batch(wire, 4, stride=stride)
        assert out["summary"]["n_delivered"] == 4
        hs = 2 if plen < 126 else 4 if plen < 65536 else 10
        for i in range(4):
            got = out["wire"][i * stride + hs + 4: i * stride + hs + 4 + plen]
            assert np.array_equal(got, _oracle.gen_plain(i, plen, 0x5EED0001)), (plen, i)


def test_oracle_build_frame_known_answers(known_answers):
    for case in known_answers["build_frame"]:
        fill = case["fill"].encode().decode("unicode_escape").encode("latin-1")
        payload = (fill * (case["length"] // len(fill) + 1))[: case["length"]]
        key = b"\x11\x22\x33\x44"
        rc, out = _oracle.build_frame(payload, case["opcode"], case["mask"], case["fin"], key,
                                      cap=case["cap"])
        exp = case["expect"]
        assert rc == exp["rc"] if exp["rc"] >= 0 else rc < 0, case["id"]
        if rc < 0:
            continue
        head = bytes.fromhex(exp["head"])
        assert out[: len(head)] == head, case["id"]
        hs = len(head)
        if case["mask"]:
            assert out[hs:hs + 4] == key
            body = bytes(b ^ key[i & 3] for i, b in enumerate(out[hs + 4:]))
            assert body == payload, case["id"]
        elif exp.get("payload_plain"):
            assert out[hs:] == payload, case["id"]
