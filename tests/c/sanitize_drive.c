/*
 * sanitize_drive.c — differential run of the product's host decoder (uvhttp_amd/csrc/ws_host.c)
 * against the oracle (oracle/ws_oracle.c), built with -fsanitize=address,undefined
 * (tests/c/Makefile).  The reference ships ASan/UBSan/TSan build options
 * (CMakeLists.txt:73-75, 273-287) and has no WebSocket fuzzer (.github/workflows/ci-fuzz.yml
 * covers HTTP only); this is that fuzzer for the host side of this path.
 *
 * Per iteration: a random frame stream (every opcode, fragments, control frames, 7/16/64-bit
 * length forms, empty payloads, header violations — RSV bits, unmasked, oversized control,
 * 64-bit lengths with the MSB set, lengths over max_frame_size — and random limits) cut into
 * random reads; both decoders get the same reads, process_data by process_data, until one
 * fails.  Return codes, transcripts (messages, closes, pongs, close echoes), recv-buffer
 * bytes / size and fragment state must agree after every call.  Also parse_frame_header and
 * apply_mask on random inputs at every alignment, and TLS seal -> open round trips of the
 * TLS oracle (oracle/tls_oracle.c).  Any sanitizer report aborts the run (non-zero exit).
 *
 *   sanitize_drive ITERATIONS SEED
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "uvhttp_ws_amd.h"

/* ---- oracle entry points (oracle/ws_oracle.c, tls_oracle.c) ----------------------------- */
typedef struct orc_conn orc_conn_t;
typedef struct {
    uint8_t fin, rsv1, rsv2, rsv3, opcode, mask, len_code;
    uint64_t payload_length;
} orc_header_t;
int oracle_parse_frame_header(const uint8_t* d, size_t n, orc_header_t* h, size_t* hs);
void oracle_apply_mask(uint8_t* data, size_t len, const uint8_t* key);
orc_conn_t* oracle_conn_new(int is_server, int max_frame_size, int max_message_size, int record);
void oracle_conn_free(orc_conn_t* c);
void oracle_conn_set_wrapper(orc_conn_t* c, int has_wrapper);
int oracle_process_data(orc_conn_t* c, const uint8_t* data, size_t len);
size_t oracle_conn_events(const orc_conn_t* c, uint8_t* out, size_t cap);
size_t oracle_conn_recv_pos(const orc_conn_t* c);
size_t oracle_conn_recv_size(const orc_conn_t* c);
size_t oracle_conn_recv_bytes(const orc_conn_t* c, uint8_t* out, size_t cap);
size_t oracle_conn_frag_size(const orc_conn_t* c);
int oracle_conn_frag_pending(const orc_conn_t* c);
int oracle_conn_frag_opcode(const orc_conn_t* c);
int oracle_conn_state(const orc_conn_t* c);

typedef struct {
    uint8_t key[32];
    uint8_t iv[12];
    uint32_t key_len, version, cipher, reserved[2];
} tls_key_t;
typedef struct {
    uint64_t begin, len, seq;
    uint32_t key, ws_prefix;
} tls_stream_t;
typedef struct {
    uint64_t rec_off, out_off;
    uint32_t content_len, stream;
    uint8_t type;
    int8_t status;
    uint16_t reserved;
    uint32_t reserved2;
} tls_record_t;
typedef struct {
    uint32_t first_record, n_records, n_delivered;
    int32_t status, first_status;
    uint32_t reserved;
    uint64_t consumed_bytes, next_seq, out_off, plain_len, reserved3;
} tls_result_t;
uint64_t oracle_tls_seal_record(const tls_key_t* k, uint64_t seq, uint8_t type,
                                const uint8_t* content, uint32_t n, uint32_t pad, uint8_t* rec);
uint64_t oracle_tls_open_batch(const uint8_t* wire, uint64_t wire_len, const tls_key_t* keys,
                               uint32_t n_keys, const tls_stream_t* streams, uint32_t n_streams,
                               tls_record_t* records, uint32_t max_records, tls_result_t* results,
                               uint8_t* out, uint64_t out_cap);

/* ---- helpers ------------------------------------------------------------------------------- */
static uint64_t g_state;
static uint64_t rnd(void) {
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static uint64_t rn(uint64_t n) { return n ? rnd() % n : 0; }

#define CHECK(cond, ...)                                             \
    do {                                                             \
        if (!(cond)) {                                               \
            fprintf(stderr, "iteration %llu: ", (unsigned long long)g_iter); \
            fprintf(stderr, __VA_ARGS__);                            \
            fprintf(stderr, "\n");                                   \
            exit(1);                                                 \
        }                                                            \
    } while (0)

static unsigned long long g_iter;

/* product transcript, same record format as the oracle's: u8 type | i32 a | u64 len | bytes */
typedef struct {
    uint8_t* p;
    size_t n, cap;
} buf_t;
static buf_t g_tr;
static void tr_push(uint8_t type, int32_t a, const uint8_t* p, uint64_t len) {
    const size_t need = 13 + (size_t)len;
    if (g_tr.n + need > g_tr.cap) {
        size_t nc = g_tr.cap ? g_tr.cap : 4096;
        while (nc < g_tr.n + need) nc *= 2;
        g_tr.p = (uint8_t*)realloc(g_tr.p, nc);
        g_tr.cap = nc;
    }
    uint8_t* w = g_tr.p + g_tr.n;
    w[0] = type;
    memcpy(w + 1, &a, 4);
    memcpy(w + 5, &len, 8);
    if (len) memcpy(w + 13, p, (size_t)len);
    g_tr.n += need;
}
static int on_message(uvhttp_ws_connection_t* c, const char* d, size_t n, int op) {
    (void)c;
    tr_push(1, op, (const uint8_t*)d, n);
    return 0;
}
/* the close reason is the payload after the code, not NUL-terminated (as the reference
 * passes it); its length comes from the CLOSE frame, which sits at the front of recv_buffer
 * while process_data dispatches it */
static int on_close(uvhttp_ws_connection_t* c, int code, const char* reason) {
    uvhttp_ws_frame_header_t h;
    size_t hs = 0;
    uint64_t rl = 0;
    if (uvhttp_ws_parse_frame_header(c->recv_buffer, c->recv_buffer_pos, &h, &hs) == UVHTTP_OK &&
        h.payload_length >= 2)
        rl = h.payload_length - 2;
    tr_push(2, code, rl ? (const uint8_t*)reason : NULL, rl);
    return 0;
}
static void* resolver(uvhttp_ws_connection_t* c) {
    (void)c;
    return (void*)0x1;
}
static void sink(void* ctx, uvhttp_ws_connection_t* c, int op, const uint8_t* p, size_t n) {
    (void)ctx;
    (void)c;
    tr_push(op == 0xA ? 3 : 4, op, p, n);
}

/* one frame into out; returns its size */
static size_t make_frame(uint8_t* out, int op, int fin, const uint8_t* payload, uint64_t n,
                         int masked, int rsv, int form, uint64_t len_field) {
    size_t h = 0;
    out[h++] = (uint8_t)((fin ? 0x80 : 0) | (rsv << 4) | (op & 0xF));
    const uint8_t m = masked ? 0x80 : 0;
    if (form == 7) {
        out[h++] = m | (uint8_t)len_field;
    } else if (form == 16) {
        out[h++] = m | 126;
        out[h++] = (uint8_t)(len_field >> 8);
        out[h++] = (uint8_t)len_field;
    } else {
        out[h++] = m | 127;
        for (int k = 7; k >= 0; --k) out[h++] = (uint8_t)(len_field >> (8 * k));
    }
    uint8_t key[4] = {0, 0, 0, 0};
    if (masked) {
        const uint64_t kw = rnd();
        memcpy(key, &kw, 4);
        memcpy(out + h, key, 4);
        h += 4;
    }
    for (uint64_t b = 0; b < n; ++b) out[h + b] = payload[b] ^ (masked ? key[b & 3] : 0);
    return h + (size_t)n;
}

static size_t make_stream(uint8_t* out, size_t cap, int n_frames, int bad) {
    static uint8_t payload[70000];
    size_t pos = 0;
    int open = 0;
    for (int f = 0; f < n_frames; ++f) {
        static const uint64_t sizes[] = {0, 1, 2, 3, 7, 64, 125, 126, 127, 300, 1000, 4000, 65535, 65536, 69999};
        uint64_t n = sizes[rn(sizeof(sizes) / sizeof(sizes[0]))];
        if (n > 5000 && rn(4)) n = rn(200);
        int op, fin = 1;
        const uint64_t r = rn(100);
        if (r < 12) {
            op = (int)(0x8 + rn(3));
            if (n > 125) n = rn(126);
            if (op == 0x8 && n == 1) n = 2;
        } else if (r < 14) {
            op = (int)(0x3 + rn(5)); /* reserved non-control opcodes 3..7 */
        } else {
            op = open ? 0 : (int)(1 + rn(2));
            fin = rn(10) < 6;
            open = !fin;
        }
        for (uint64_t b = 0; b < n; ++b) payload[b] = (uint8_t)rnd();
        int masked = 1, rsv = 0;
        int form = n < 126 ? 7 : n < 65536 ? 16 : 64;
        uint64_t len_field = n;
        if (rn(20) == 0) form = n < 65536 ? (rn(2) ? 16 : 64) : 64; /* non-minimal forms */
        if (bad && rn(30) == 0) {
            switch (rn(6)) {
                case 0: rsv = (int)(1 + rn(7)); break;
                case 1: masked = 0; break;
                case 2: op = (int)(0x8 + rn(3)); fin = (int)rn(2); break; /* control, maybe !FIN */
                case 3: form = 64; len_field = (1ull << 63) | rnd(); n = 0; break;
                case 4: form = 64; len_field = 1ull << 40; n = 0; break;   /* > max_frame_size */
                default: op = 0; break;                                  /* stray continuation */
            }
        }
        if (pos + n + 14 > cap) break;
        pos += make_frame(out + pos, op, fin, payload, n, masked, rsv, form, len_field);
    }
    return pos;
}

static void compare_state(uvhttp_ws_connection_t* p, orc_conn_t* o, const char* where) {
    CHECK(p->recv_buffer_pos == oracle_conn_recv_pos(o), "%s: recv_buffer_pos %zu vs %zu", where,
          p->recv_buffer_pos, oracle_conn_recv_pos(o));
    CHECK(p->recv_buffer_size == oracle_conn_recv_size(o), "%s: recv_buffer_size", where);
    static uint8_t tmp[1 << 22];
    const size_t n = oracle_conn_recv_bytes(o, tmp, sizeof(tmp));
    CHECK(n <= sizeof(tmp) && (!n || !memcmp(tmp, p->recv_buffer, n)), "%s: recv bytes", where);
    const size_t fs = p->fragmented_message ? p->fragmented_size : 0;
    CHECK(fs == oracle_conn_frag_size(o), "%s: fragment size", where);
    CHECK((p->fragmented_message != NULL) == oracle_conn_frag_pending(o), "%s: pending", where);
    CHECK((int)p->fragmented_opcode == oracle_conn_frag_opcode(o), "%s: fragment opcode", where);
    CHECK((p->state == 3) == (oracle_conn_state(o) == 3), "%s: state", where);
    const size_t ol = oracle_conn_events(o, NULL, 0);
    uint8_t* ev = (uint8_t*)malloc(ol ? ol : 1);
    oracle_conn_events(o, ev, ol);
    CHECK(ol == g_tr.n && (!ol || !memcmp(ev, g_tr.p, ol)), "%s: transcript (%zu vs %zu bytes)",
          where, g_tr.n, ol);
    free(ev);
}

static void one_stream(int bad) {
    static uint8_t stream[1 << 21];
    const int n_frames = (int)(1 + rn(rn(4) ? 20 : 200));
    const size_t len = make_stream(stream, sizeof(stream), n_frames, bad);
    static const int mfs[] = {16 * 1024 * 1024, 65536, 4000, 100000, 200};
    static const int mms[] = {64 * 1024 * 1024, 9000, 0, 1000};
    const int mf = mfs[rn(5)], mm = mms[rn(4)];
    const int is_server = rn(10) != 0;
    uvhttp_config_t cfg;
    memset(&cfg, 0, sizeof(cfg));
    cfg.websocket_max_frame_size = mf;
    cfg.websocket_max_message_size = mm;
    uvhttp_ws_connection_t* p = uvhttp_ws_connection_create(0, NULL, is_server, &cfg);
    uvhttp_ws_set_callbacks(p, on_message, on_close, NULL);
    p->user_data = (void*)0x1;
    orc_conn_t* o = oracle_conn_new(is_server, mf, mm, 1);
    oracle_conn_set_wrapper(o, 1);
    g_tr.n = 0;
    size_t pos = 0;
    while (pos < len) {
        static const size_t cuts[] = {1, 2, 3, 7, 100, 1000, 4096, 16384};
        size_t n = rn(5) ? cuts[rn(8)] : (size_t)rn(70000);
        if (n > len - pos) n = len - pos;
        const int rp = uvhttp_ws_process_data(p, stream + pos, n);
        const int ro = oracle_process_data(o, stream + pos, n);
        CHECK(rp == ro, "process_data rc %d vs %d at byte %zu", rp, ro, pos);
        pos += n;
        if (rp) break;
    }
    compare_state(p, o, "stream");
    uvhttp_ws_connection_free(p);
    oracle_conn_free(o);
}

/* parse_frame_header and apply_mask on random bytes / alignments */
static void headers_and_masks(void) {
    uint8_t b[32];
    for (int k = 0; k < 32; ++k) b[k] = (uint8_t)rnd();
    if (rn(3) == 0) b[1] = (uint8_t)((b[1] & 0x80) | (126 + rn(2)));
    const size_t n = (size_t)rn(15);
    uvhttp_ws_frame_header_t h;
    size_t hs = 0, ohs = 0;
    orc_header_t oh;
    const int rp = uvhttp_ws_parse_frame_header(b, n, &h, &hs);
    const int ro = oracle_parse_frame_header(b, n, &oh, &ohs);
    CHECK(rp == ro, "parse rc");
    if (!rp) {
        CHECK(hs == ohs && h.payload_length == oh.payload_length && h.opcode == oh.opcode &&
                  h.fin == oh.fin && h.mask == oh.mask && h.payload_len == oh.len_code,
              "parse fields");
    }
    static uint8_t m1[4200], m2[4200];
    const size_t off = (size_t)rn(16), ln = (size_t)rn(4096);
    uint8_t key[4];
    const uint64_t kw = rnd();
    memcpy(key, &kw, 4);
    for (size_t k = 0; k < off + ln + 16; ++k) m1[k] = m2[k] = (uint8_t)rnd();
    uvhttp_ws_apply_mask(m1 + off, ln, key);
    oracle_apply_mask(m2 + off, ln, key);
    CHECK(!memcmp(m1, m2, off + ln + 16), "apply_mask off %zu len %zu", off, ln);
}

/* TLS oracle: seal records then open them as a batch (ASan coverage of tls_oracle.c) */
static void tls_round_trip(void) {
    tls_key_t k;
    memset(&k, 0, sizeof(k));
    for (int i = 0; i < 32; ++i) k.key[i] = (uint8_t)rnd();
    for (int i = 0; i < 12; ++i) k.iv[i] = (uint8_t)rnd();
    const int kind = (int)rn(3);
    k.cipher = kind == 2 ? 1u : 0u;
    k.key_len = kind == 0 ? 16u : 32u;
    k.version = rn(2) ? 0x0304u : 0x0303u;
    static uint8_t wire[8 * (16384 + 300)], content[16384], out[8 * (16384 + 300)];
    size_t pos = 0;
    const int n = (int)(1 + rn(6));
    const uint64_t seq = rnd() >> 16;
    for (int r = 0; r < n; ++r) {
        const uint32_t cl = (uint32_t)(rn(3) ? rn(300) : rn(16385));
        for (uint32_t b = 0; b < cl; ++b) content[b] = (uint8_t)rnd();
        const uint32_t pad = k.version == 0x0304u ? (uint32_t)rn(3) * 20 : 0;
        pos += oracle_tls_seal_record(&k, seq + (uint64_t)r, 23, content, cl, pad, wire + pos);
    }
    if (rn(4) == 0 && pos) wire[rn(pos)] ^= (uint8_t)(1 + rn(255)); /* corrupt one byte */
    const size_t cut = rn(5) == 0 ? (size_t)rn(pos + 1) : pos;
    tls_stream_t st = {0, cut, seq, 0, (uint32_t)rn(40)};
    tls_record_t recs[16];
    tls_result_t res;
    oracle_tls_open_batch(wire, cut, &k, 1, &st, 1, recs, 16, &res, out, sizeof(out));
    CHECK(res.n_delivered <= res.n_records && res.n_records <= 16, "tls counts");
}

int main(int argc, char** argv) {
    const unsigned long long iters = argc > 1 ? strtoull(argv[1], NULL, 10) : 2000;
    g_state = argc > 2 ? strtoull(argv[2], NULL, 10) : 1;
    uvhttp_ws_amd_set_control_hooks(resolver, sink);
    for (g_iter = 0; g_iter < iters; ++g_iter) {
        one_stream((int)(g_iter & 1));
        for (int k = 0; k < 8; ++k) headers_and_masks();
        if (g_iter % 4 == 0) tls_round_trip();
    }
    free(g_tr.p);
    printf("sanitize_drive: %llu iterations clean\n", iters);
    return 0;
}
