"""Transcribe the reference's own known-answer tests into tests/golden/reference_known_answers.json.

Every case below is DATA taken from a test of adam-ikari/uvhttp v2.7.0 (file:line cited in
`src`): the wire bytes that test feeds and the results that test asserts.  Nothing here is
computed by this repository's code — the expected values are the reference tests' own
assertions (plus RFC 6455 §5.7, the published example the reference test quotes), so they
pin both the oracle (oracle/ws_oracle.c) and the product library.

Frame builders restate the two test helpers the reference tests use:
  build_raw_frame     test/unit/test_websocket_boost_coverage.cpp:39-81   (mask bit, all-zero key)
  build_masked_frame  test/unit/test_websocket_boost_coverage2.cpp:89-130 (mask bit, given key)

Run:  python tests/golden/make_known_answers.py   (rewrites the JSON next to this file)
"""
import json
import os

UT = "test/unit/"
AUTO = UT + "test_websocket_automated.cpp"
FIX = UT + "test_websocket_frame_fixes.cpp"
BOOST = UT + "test_websocket_boost_coverage.cpp"
BOOST2 = UT + "test_websocket_boost_coverage2.cpp"
API = UT + "test_websocket_api_coverage.cpp"

CONT, TEXT, BINARY, CLOSE, PING, PONG = 0x0, 0x1, 0x2, 0x8, 0x9, 0xA
DEFAULT_MAX_FRAME = 16 * 1024 * 1024  # include/uvhttp_defaults.h:171-173


def _len_bytes(n):
    if n < 126:
        return bytes([0x80 | n])
    if n < 65536:
        return bytes([0x80 | 126, (n >> 8) & 0xFF, n & 0xFF])
    return bytes([0x80 | 127]) + n.to_bytes(8, "big")


def masked_frame(payload, opcode, fin, key=b"\x00\x00\x00\x00"):
    head = bytes([(0x80 if fin else 0) | (opcode & 0x0F)]) + _len_bytes(len(payload)) + key
    body = bytes(b ^ key[i % 4] for i, b in enumerate(payload))
    return head + body


def raw_frame(payload, opcode, fin):  # build_raw_frame: zero key
    return masked_frame(payload, opcode, fin)


def h(b):
    return bytes(b).hex()


parse_cases = [
    dict(id="text_unmasked", src=AUTO + ":102-115", bytes=h([0x81, 0x05]) + b"Hello".hex(),
         expect=dict(rc=0, fin=1, opcode=TEXT, mask=0, len_code=5, header_size=2)),
    dict(id="rfc6455_masked_hello", src=AUTO + ":117-130",
         bytes="818537fa213d7f9f4d5158",
         expect=dict(rc=0, fin=1, opcode=TEXT, mask=1, len_code=5, header_size=2)),
    dict(id="close", src=AUTO + ":147-158", bytes="8800",
         expect=dict(rc=0, fin=1, opcode=CLOSE, header_size=2)),
    dict(id="ping", src=AUTO + ":160-172", bytes="890401020304",
         expect=dict(rc=0, fin=1, opcode=PING, len_code=4, header_size=2)),
    dict(id="pong", src=AUTO + ":174-185", bytes="8a00",
         expect=dict(rc=0, fin=1, opcode=PONG, header_size=2)),
    dict(id="fragmented", src=AUTO + ":187-198", bytes="0105" + b"Hello".hex(),
         expect=dict(rc=0, fin=0, opcode=TEXT, len_code=5)),
    dict(id="ext16_256", src=AUTO + ":200-209", bytes="827e0100",
         expect=dict(rc=0, header_size=4)),
    dict(id="ext64_65536", src=AUTO + ":211-220", bytes="827f0000000000010000",
         expect=dict(rc=0, header_size=10)),
    dict(id="null_data", src=AUTO + ":226-231", bytes="", length=2, null="data",
         expect=dict(rc=-1)),
    dict(id="null_header", src=AUTO + ":233-238", bytes="8100", null="header",
         expect=dict(rc=-1)),
    dict(id="null_header_size", src=AUTO + ":240-245", bytes="8100", null="header_size",
         expect=dict(rc=-1)),
    dict(id="one_byte", src=AUTO + ":247-254", bytes="81", expect=dict(rc=-1)),
    dict(id="zero_len_null", src=AUTO + ":256-261", bytes="", length=0, null="data",
         expect=dict(rc=-1)),
    dict(id="small_masked", src=FIX + ":26-37", bytes="818500000000" + b"ab".hex(),
         expect=dict(rc=0, fin=1, opcode=TEXT, mask=1, len_code=5, payload_length=5,
                     header_size=2)),
    dict(id="ext16_200", src=FIX + ":39-49", bytes="81fe00c800000000",
         expect=dict(rc=0, opcode=TEXT, len_code=126, payload_length=200, header_size=4)),
    dict(id="ext16_max", src=FIX + ":51-59", bytes="81feffff000000000000",
         expect=dict(rc=0, len_code=126, payload_length=65535, header_size=4)),
    dict(id="ext64_70000", src=FIX + ":61-72", bytes="81ff0000000000011170000000000000",
         expect=dict(rc=0, opcode=TEXT, len_code=127, payload_length=70000, header_size=10)),
    dict(id="ext64_msb_rejected", src=FIX + ":74-84", bytes="82ffffffffffffffffff000000000000",
         expect=dict(rc=-1)),
    dict(id="ext64_max_legal", src=FIX + ":86-96", bytes="82ff7fffffffffffffff000000000000",
         expect=dict(rc=0, len_code=127, payload_length=(1 << 63) - 1, header_size=10)),
    dict(id="ext16_too_short", src=FIX + ":98-103", bytes="81fe00", expect=dict(rc=-1)),
]

mask_cases = [
    dict(id="roundtrip_hello", src=AUTO + ":267-280", data=b"Hello".hex(), key="37fa213d",
         roundtrip=True, differs=True),
    dict(id="single_byte", src=AUTO + ":282-289", data="ff", key="12345678",
         expect_after=h([0xFF ^ 0x12]), roundtrip=True),
    dict(id="large_1024", src=AUTO + ":291-305", data=h([i & 0xFF for i in range(1024)]),
         key="12345678", roundtrip=True, differs=True),
    dict(id="null_data", src=AUTO + ":307-312", data="", key="12345678", null="data",
         length=5),
    dict(id="null_key", src=AUTO + ":314-319", data="010203", key="", null="key",
         expect_after="010203"),
    dict(id="zero_length", src=AUTO + ":321-329", data="010203", key="12345678", length=0,
         expect_after="010203"),
    dict(id="two_bytes", src=BOOST2 + ":893-906", data="4142", key="12345678",
         roundtrip=True, differs=True),
    dict(id="five_bytes_key_wrap", src=BOOST2 + ":911-926", data="4142434445", key="12345678",
         checks={"0": 0x41 ^ 0x12, "4": 0x45 ^ 0x12}, roundtrip=True, differs=True),
    dict(id="six_bytes", src=BOOST2 + ":931-942", data="414243444546", key="12345678",
         roundtrip=True, differs=True),
    # RFC 6455 §5.7: the masked "Hello" example; the reference test quotes the bytes
    # (test_websocket_automated.cpp:119) and the RFC gives the plaintext.
    dict(id="rfc6455_5_7_hello", src="RFC 6455 §5.7; " + AUTO + ":119", data="7f9f4d5158",
         key="37fa213d", expect_after=b"Hello".hex()),
]


def feed(frame_bytes, rc=0):
    return dict(hex=bytes(frame_bytes).hex(), expect_rc=rc)


K1234 = bytes([0x12, 0x34, 0x56, 0x78])
process_cases = [
    dict(id="text_frame", src=BOOST + ":576-600",
         feeds=[feed(raw_frame(b"Hello", TEXT, 1))],
         expect=dict(message_called=True, last_opcode=TEXT, last_message=b"Hello".hex())),
    dict(id="binary_frame", src=BOOST + ":602-626",
         feeds=[feed(raw_frame(bytes([1, 2, 3, 4]), BINARY, 1))],
         expect=dict(message_called=True, last_opcode=BINARY)),
    dict(id="close_frame_reason", src=BOOST + ":628-656",
         feeds=[feed(raw_frame(bytes([0x03, 0xE8]) + b"Normal", CLOSE, 1))],
         expect=dict(close_called=True, close_code=1000, state="CLOSED")),
    dict(id="close_frame_empty", src=BOOST + ":658-681",
         feeds=[feed(raw_frame(b"", CLOSE, 1))],
         expect=dict(close_called=True, close_code=1000, state="CLOSED")),
    dict(id="close_frame_code_only", src=BOOST + ":683-712",
         feeds=[feed(raw_frame(bytes([0x03, 0xE9]), CLOSE, 1))],
         expect=dict(close_called=True, close_code=1001, state="CLOSED")),
    dict(id="ping_no_wrapper", src=BOOST + ":714-738",
         feeds=[feed(raw_frame(b"ping!", PING, 1))],
         expect=dict(message_called=False, close_called=False)),
    dict(id="ping_empty", src=BOOST + ":740-761", feeds=[feed(raw_frame(b"", PING, 1))],
         expect=dict()),
    dict(id="pong_ignored", src=BOOST + ":763-785", feeds=[feed(raw_frame(b"pong", PONG, 1))],
         expect=dict(message_called=False, close_called=False)),
    dict(id="fragmented_text", src=BOOST + ":789-829",
         feeds=[feed(raw_frame(b"Hel", TEXT, 0)), feed(raw_frame(b"lo", CONT, 1))],
         expect_after_feed=[dict(message_called=False), dict(message_called=True)],
         expect=dict(message_called=True, last_opcode=TEXT, last_message=b"Hello".hex())),
    dict(id="fragmented_binary", src=BOOST + ":831-864",
         feeds=[feed(raw_frame(bytes([0xAA, 0xBB]), BINARY, 0)),
                feed(raw_frame(bytes([0xCC, 0xDD]), CONT, 1))],
         expect_after_feed=[dict(message_called=False), dict(message_called=True)],
         expect=dict(message_called=True, last_opcode=BINARY, last_message_len=4)),
    dict(id="single_text", src=BOOST + ":866-890",
         feeds=[feed(raw_frame(b"single", TEXT, 1))],
         expect=dict(message_called=True, last_message_len=6)),
    dict(id="two_frames_one_buffer", src=BOOST + ":892-928",
         feeds=[feed(raw_frame(b"first", TEXT, 1) + raw_frame(b"second", TEXT, 1))],
         expect=dict(message_called=True, last_message=b"second".hex())),
    dict(id="partial_header", src=BOOST + ":930-960",
         feeds=[feed([0x81]), feed(bytes([0x85, 0, 0, 0, 0]) + b"Hello")],
         expect_after_feed=[dict(message_called=False), dict(message_called=True)],
         expect=dict(message_called=True, last_message_len=5)),
    dict(id="close_no_callback", src=BOOST + ":981-1002",
         feeds=[feed(raw_frame(bytes([0x03, 0xE8]), CLOSE, 1))], no_callbacks=True,
         expect=dict(state="CLOSED")),
    dict(id="text_no_callback", src=BOOST + ":1004-1024",
         feeds=[feed(raw_frame(b"test", TEXT, 1))], no_callbacks=True, expect=dict()),
    dict(id="buffer_expansion", src=BOOST + ":1026-1070",
         config=dict(max_frame_size=1024 * 1024, max_message_size=0),
         pre=dict(fill="8a8000000000", fill_to=64 * 1024 - 4),
         feeds=[feed(raw_frame(b"expansion!", TEXT, 1))],
         expect=dict(recv_buffer_size_gt=64 * 1024 - 4)),
    dict(id="masked_text_real_key", src=BOOST + ":1072-1107",
         feeds=[feed(masked_frame(b"masked!", TEXT, 1, K1234))],
         expect=dict(message_called=True, last_message=b"masked!".hex(),
                     last_message_len=7)),
    dict(id="expansion_capped_at_max_frame", src=BOOST + ":1243-1284",
         config=dict(max_frame_size=12, max_message_size=0), pre=dict(recv_buffer_size=8),
         feeds=[feed(raw_frame(b"test", TEXT, 1))],
         expect=dict(message_called=True, last_message=b"test".hex(), last_message_len=4)),
    dict(id="expansion_exceeds_max_frame", src=BOOST + ":1286-1320",
         config=dict(max_frame_size=10, max_message_size=0),
         pre=dict(recv_buffer_size=8, fill="000000000000", fill_to=6),
         feeds=[feed(raw_frame(b"12345678", TEXT, 1), rc=-1)], expect=dict()),
    dict(id="fragments_realloc_intermediate", src=BOOST + ":1322-1377",
         feeds=[feed(raw_frame(b"AB", TEXT, 0)), feed(raw_frame(b"CDE", CONT, 0)),
                feed(raw_frame(b"FG", CONT, 1))],
         expect_after_feed=[dict(message_called=False), dict(message_called=False),
                            dict(message_called=True)],
         expect=dict(last_opcode=TEXT, last_message=b"ABCDEFG".hex(), last_message_len=7)),
    dict(id="fragments_realloc_final", src=BOOST + ":1379-1417",
         feeds=[feed(raw_frame(b"AB", TEXT, 0)), feed(raw_frame(b"CDEFG", CONT, 1))],
         expect=dict(message_called=True, last_opcode=TEXT, last_message=b"ABCDEFG".hex())),
    dict(id="fragments_binary_realloc_final", src=BOOST + ":1419-1450",
         feeds=[feed(raw_frame(bytes([1, 2]), BINARY, 0)),
                feed(raw_frame(bytes([3, 4, 5, 6, 7]), CONT, 1))],
         expect=dict(message_called=True, last_opcode=BINARY, last_message_len=7)),
    dict(id="continuation_without_start", src=BOOST + ":1452-1472",
         feeds=[feed(raw_frame(b"x", CONT, 1), rc=-1)], expect=dict(message_called=False)),
    dict(id="data_frame_inside_fragment", src=BOOST + ":1474-1499",
         feeds=[feed(raw_frame(b"ab", TEXT, 0)), feed(raw_frame(b"cd", TEXT, 1), rc=-1)],
         expect=dict()),
    dict(id="fragment_exceeds_max_message", src=BOOST + ":1501-1536",
         config=dict(max_frame_size=DEFAULT_MAX_FRAME, max_message_size=4),
         feeds=[feed(raw_frame(b"abc", TEXT, 0)), feed(raw_frame(b"de", CONT, 1), rc=-1)],
         expect=dict()),
    dict(id="masked_close_1000_ok", src=BOOST2 + ":612-643",
         feeds=[feed(masked_frame(bytes([0x03, 0xE8]) + b"OK", CLOSE, 1,
                                  bytes([0x37, 0xFA, 0x21, 0x3D])))],
         expect=dict(close_called=True, close_code=1000, state="CLOSED")),
    dict(id="masked_text_Masked", src=BOOST2 + ":645-675",
         feeds=[feed(masked_frame(b"Masked!", TEXT, 1, K1234))],
         expect=dict(message_called=True, last_opcode=TEXT, last_message=b"Masked!".hex())),
    dict(id="masked_close_1002", src=BOOST2 + ":677-706",
         feeds=[feed(masked_frame(bytes([0x03, 0xEA]), CLOSE, 1,
                                  bytes([0xAA, 0xBB, 0xCC, 0xDD])))],
         expect=dict(close_called=True, close_code=1002)),
    dict(id="four_fragments", src=BOOST2 + ":1068-1112",
         feeds=[feed(raw_frame(p, TEXT if i == 0 else CONT, 1 if i == 3 else 0))
                for i, p in enumerate([b"AB", b"CD", b"EF", b"GH"])],
         expect_after_feed=[dict(message_called=False)] * 3 + [dict(message_called=True)],
         expect=dict(last_message=b"ABCDEFGH".hex(), last_message_len=8)),
    dict(id="huge_64bit_length_rejected", src=FIX + ":183-200",
         feeds=[feed(bytes([0x81, 0xFF] + [0xFF] * 8 + [0, 0, 0, 0]), rc=-1)], expect=dict()),
    dict(id="length_over_max_frame_rejected", src=FIX + ":202-220",
         feeds=[feed(bytes([0x81, 0xFF]) + (DEFAULT_MAX_FRAME + 1).to_bytes(8, "big")
                     + bytes(4), rc=-1)], expect=dict()),
]


def bcase(id, src, fill, n, opcode, mask, fin, cap, expect):
    return dict(id=id, src=src, fill=fill, length=n, opcode=opcode, mask=mask, fin=fin, cap=cap,
                expect=expect)


build_cases = [
    bcase("small_hello", FIX + ":105-115", "hello", 5, TEXT, 0, 1, 64,
          dict(rc=7, head="8105", payload_plain=True)),
    bcase("ext16_200", FIX + ":117-131", "x", 200, TEXT, 0, 1, 256,
          dict(rc=204, head="817e00c8", payload_plain=True)),
    bcase("ext16_boundary", FIX + ":133-145", "y", 65535, BINARY, 0, 1, 65536 + 16,
          dict(rc=4 + 65535, head="827effff")),
    bcase("ext64_70000", FIX + ":147-166", "z", 70000, BINARY, 0, 1, 70016,
          dict(rc=10 + 70000, head="827f0000000000011170", payload_plain=True)),
    bcase("insufficient_buffer", FIX + ":168-175", "\0", 200, TEXT, 0, 1, 8, dict(rc=-1)),
    bcase("masked_ext64", BOOST2 + ":719-747", "D", 70000, TEXT, 1, 1, 70014,
          dict(rc=70014, head="81ff0000000000011170")),
    bcase("masked_ext16", BOOST2 + ":752-777", "E", 300, BINARY, 1, 1, 308,
          dict(rc=308, head="82fe012c")),
    bcase("server_short", BOOST + ":217-230", "Hello", 5, TEXT, 0, 1, 64,
          dict(rc=7, head="8105", payload_plain=True)),
    bcase("server_medium", BOOST + ":232-254", "B", 300, TEXT, 0, 1, 304,
          dict(rc=304, head="817e012c", payload_plain=True)),
]


def main():
    out = dict(
        reference="adam-ikari/uvhttp v2.7.0",
        note="inputs and assertions transcribed from the reference unit tests (see src)",
        parse_frame_header=parse_cases,
        apply_mask=mask_cases,
        process_data=process_cases,
        build_frame=build_cases,
    )
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)),
                        "reference_known_answers.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print(path, len(parse_cases), len(mask_cases), len(process_cases), len(build_cases))


if __name__ == "__main__":
    main()
