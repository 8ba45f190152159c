"""Replays the reference's known-answer tests (tests/golden/reference_known_answers.json)
against an implementation adapter: the oracle or the product's drop-in host API."""
DEFAULTS = dict(max_frame_size=16 * 1024 * 1024, max_message_size=64 * 1024 * 1024)


def check_parse_case(case, parse):
    data = bytes.fromhex(case["bytes"])
    rc, h, hs = parse(data, case.get("length"), case.get("null"))
    exp = case["expect"]
    assert rc == exp["rc"], case["id"]
    names = {"fin": "fin", "opcode": "opcode", "mask": "mask", "payload_length": "payload_length"}
    for k, v in exp.items():
        if k == "rc":
            continue
        if k == "header_size":
            assert hs == v, case["id"]
        elif k == "len_code":
            got = getattr(h, "len_code", None)
            if got is None:
                got = h.payload_len
            assert got == v, case["id"]
        else:
            assert getattr(h, names[k]) == v, (case["id"], k)


def check_mask_case(case, mask):
    data = bytearray(bytes.fromhex(case["data"]))
    key = bytes.fromhex(case["key"]) if case["key"] else None
    orig = bytes(data)
    mask(data, key, case.get("length"), case.get("null"))
    if "expect_after" in case:
        assert bytes(data) == bytes.fromhex(case["expect_after"]), case["id"]
    if case.get("differs"):
        assert bytes(data) != orig, case["id"]
    for idx, val in case.get("checks", {}).items():
        assert data[int(idx)] == val, case["id"]
    if case.get("roundtrip"):
        mask(data, key, case.get("length"), case.get("null"))
        assert bytes(data) == orig, case["id"]
    if case.get("null") == "data":
        assert bytes(data) == orig


def check_process_case(case, make_conn):
    """make_conn(cfg, callbacks) -> adapter with .process(bytes)->rc, .events() list of
    (kind, a, payload), .state, .recv_size, .set_recv_state(size, fill, pos)."""
    cfg = dict(DEFAULTS)
    if case.get("config"):
        cfg.update(case["config"])
    conn = make_conn(cfg, not case.get("no_callbacks"))
    pre = case.get("pre")
    if pre:
        fill_to = pre.get("fill_to", 0)
        pat = bytes.fromhex(pre.get("fill", "00"))
        fill = bytearray()
        while len(fill) + len(pat) <= fill_to:
            fill += pat
        fill += bytes(fill_to - len(fill))
        conn.set_recv_state(pre.get("recv_buffer_size", 64 * 1024), bytes(fill), fill_to)
    after = case.get("expect_after_feed")
    for k, fd in enumerate(case["feeds"]):
        rc = conn.process(bytes.fromhex(fd["hex"]))
        assert rc == fd["expect_rc"], (case["id"], k, rc)
        if after:
            called = any(e[0] == "message" for e in conn.events())
            assert called == after[k]["message_called"], (case["id"], k)
    check_expectations(case, conn.events(), conn.state, lambda: conn.recv_size)


def check_expectations(case, ev, state, recv_size):
    """the reference test's assertions on what the feeds left: callbacks, state, buffer"""
    msgs = [e for e in ev if e[0] == "message"]
    closes = [e for e in ev if e[0] == "close"]
    exp = case["expect"]
    if "message_called" in exp:
        assert bool(msgs) == exp["message_called"], case["id"]
    if "close_called" in exp:
        assert bool(closes) == exp["close_called"], case["id"]
    if "last_opcode" in exp:
        assert msgs[-1][1] == exp["last_opcode"], case["id"]
    if "last_message" in exp:
        assert msgs[-1][2] == bytes.fromhex(exp["last_message"]), case["id"]
    if "last_message_len" in exp:
        assert len(msgs[-1][2]) == exp["last_message_len"], case["id"]
    if "close_code" in exp:
        assert closes[-1][1] == exp["close_code"], case["id"]
    if "state" in exp:
        assert state == 3, case["id"]
    if "recv_buffer_size_gt" in exp:
        assert recv_size() > exp["recv_buffer_size_gt"], case["id"]
