/*
 * oracle/ws_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference decode path of adam-ikari/uvhttp v2.7.0,
 * src/uvhttp_websocket.c, used as the parity checker for the MI355X path and as the
 * `cpu_baseline` ("port") timed by bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product library (uvhttp_amd/) never
 * links, loads or calls anything in this directory.
 *
 * Pinning: the reference cannot be built in this image without writing stand-in headers
 * for mbedtls/llhttp/uthash (absent, un-vendored submodules), so it is treated as
 * unbuildable.  This restatement is pinned instead by the
 * known-answer vectors held in the reference's own unit tests, transcribed as data into
 * tests/golden/reference_known_answers.json and checked by tests/test_oracle_golden.py.
 *
 * Restated functions (each follows the cited reference lines statement by statement):
 *   oracle_parse_frame_header  <- uvhttp_ws_parse_frame_header  :133-185
 *   oracle_apply_mask          <- uvhttp_ws_apply_mask          :188-197
 *   oracle_fragment_append     <- uvhttp_ws_fragment_append     :781-822
 *   oracle_process_data        <- uvhttp_ws_process_data        :825-1097
 *   oracle_conn_new            <- uvhttp_ws_connection_create   :71-109
 * Harness additions (not reference code): an event transcript, an "unmasked payload"
 * instrumentation hook, the batch driver that mirrors the device batch contract of
 * include/uvhttp_ws_amd.h, and the synthetic frame generator.
 *
 * Build: oracle/Makefile (gcc -O2 -DNDEBUG, the reference release flags,
 * CMakeLists.txt:129,144).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_ERR (-1)

/* failure reasons, numerically identical to UVHTTP_WS_FRAME_* in include/uvhttp_ws_amd.h */
enum {
    R_OK = 0,
    R_INCOMPLETE = 1,
    R_SKIPPED = 2,
    R_PARSE = -1,
    R_RSV = -2,
    R_CONTROL = -3,
    R_UNMASKED = -4,
    R_TOO_BIG = -5,
    R_BUFFER = -6,
    R_FRAGMENT = -7,
    R_MESSAGE = -8,
    R_LAYOUT = -9,
};

/* ---- header ------------------------------------------------------------------------ */

typedef struct {
    uint8_t fin, rsv1, rsv2, rsv3, opcode, mask, len_code;
    uint64_t payload_length;
} orc_header_t;

/* :133-185 */
int oracle_parse_frame_header(const uint8_t* d, size_t n, orc_header_t* h, size_t* hs) {
    if (!d || !h || !hs || n < 2) return ORC_ERR;
    memset(h, 0, sizeof(*h));
    h->fin = (d[0] >> 7) & 1;
    h->rsv1 = (d[0] >> 6) & 1;
    h->rsv2 = (d[0] >> 5) & 1;
    h->rsv3 = (d[0] >> 4) & 1;
    h->opcode = d[0] & 0x0F;
    h->mask = (d[1] >> 7) & 1;
    h->len_code = d[1] & 0x7F;
    h->payload_length = h->len_code;
    *hs = 2;
    if (h->len_code == 126) {
        if (n < 4) return ORC_ERR;
        h->payload_length = ((uint64_t)d[2] << 8) | (uint64_t)d[3];
        *hs = 4;
    } else if (h->len_code == 127) {
        if (n < 10) return ORC_ERR;
        uint64_t v = 0;
        for (int k = 2; k < 10; ++k) v = (v << 8) | (uint64_t)d[k];
        h->payload_length = v;
        if (v >> 63) return ORC_ERR; /* RFC 6455 §5.2, :178-180 */
        *hs = 10;
    }
    return ORC_OK;
}

/* :188-197 — the per-byte loop, kept scalar on purpose (it is the CPU baseline). */
void oracle_apply_mask(uint8_t* data, size_t len, const uint8_t* key) {
    if (!data || !key) return;
    for (size_t i = 0; i < len; i++) data[i] ^= key[i % 4];
}

/* ---- connection + transcript --------------------------------------------------------- */

enum { EV_MESSAGE = 1, EV_CLOSE = 2, EV_PONG = 3, EV_CLOSE_ECHO = 4 };

typedef void (*orc_unmask_hook)(void* ctx, const uint8_t* payload, uint64_t len, int opcode);
struct orc_conn_frame;

typedef struct {
    int is_server;
    int max_frame_size;   /* config.max_frame_size (int, as the reference) */
    int max_message_size; /* config.max_message_size */
    int state;            /* 1 OPEN, 3 CLOSED */
    int has_wrapper;      /* stands for conn->user_data != NULL */
    uint8_t* rbuf;
    size_t rbuf_size, rbuf_pos;
    uint8_t* frag;
    size_t frag_size, frag_cap;
    int frag_opcode;
    int last_reason;      /* harness: why the last call failed */
    int frame_completed;  /* harness: a frame was fully processed in the last call */
    /* transcript */
    int record;           /* 0: count only, 1: keep payload bytes */
    int digest_on;        /* fold delivered message bytes into `digest` */
    uint8_t* ev;
    size_t ev_len, ev_cap;
    uint64_t n_events, n_messages, message_bytes;
    uint64_t digest;      /* FNV-1a 64 over delivered message payloads */
    uint64_t last_msg_len;
    int last_msg_opcode;
    orc_unmask_hook hook;
    void* hook_ctx;
    /* harness: bytes drained from the front of recv_buffer by completed frames over the
     * connection's life (stream offset of recv_buffer[0]) and a per-completed-frame hook */
    uint64_t consumed;
    void (*frame_hook)(void* ctx, struct orc_conn_frame* f);
    void* frame_ctx;
} orc_conn_t;

/* harness: one completed frame as the frame hook sees it (before recv_buffer is drained) */
typedef struct orc_conn_frame {
    uint64_t stream_off;     /* stream offset of the frame's first header byte */
    uint64_t payload_len;
    const uint8_t* payload;  /* unmasked payload inside recv_buffer (NULL if empty) */
    uint32_t key;            /* masking key bytes k0..k3, k0 = low byte (0 if unmasked) */
    uint8_t opcode, fin, mask, header_size;
    int msg_end;             /* this data frame delivered a message (on_message fired) */
} orc_conn_frame_t;

/* :71-109 (defaults include/uvhttp_defaults.h:171-194) */
orc_conn_t* oracle_conn_new(int is_server, int max_frame_size, int max_message_size,
                            int record) {
    orc_conn_t* c = (orc_conn_t*)calloc(1, sizeof(*c));
    if (!c) return NULL;
    c->is_server = is_server;
    c->max_frame_size = max_frame_size;
    c->max_message_size = max_message_size;
    c->state = 1;
    c->record = record;
    c->rbuf_size = 64 * 1024;
    c->rbuf = (uint8_t*)malloc(c->rbuf_size);
    c->digest = 1469598103934665603ull;
    if (!c->rbuf) {
        free(c);
        return NULL;
    }
    return c;
}

void oracle_conn_free(orc_conn_t* c) {
    if (!c) return;
    free(c->rbuf);
    free(c->frag);
    free(c->ev);
    free(c);
}

void oracle_conn_set_wrapper(orc_conn_t* c, int has_wrapper) { c->has_wrapper = has_wrapper; }
void oracle_conn_set_digest(orc_conn_t* c, int on) { c->digest_on = on; }
void oracle_conn_set_hook(orc_conn_t* c, orc_unmask_hook h, void* ctx) {
    c->hook = h;
    c->hook_ctx = ctx;
}
/* Tests of the reference poke recv_buffer_size / recv_buffer_pos directly
 * (test_websocket_boost_coverage.cpp:1026-1070, 1243-1320); this mirrors that. */
int oracle_conn_set_recv_state(orc_conn_t* c, size_t size, const uint8_t* fill, size_t pos) {
    size_t alloc = size > pos ? size : pos;
    if (alloc > c->rbuf_size) {
        uint8_t* nb = (uint8_t*)realloc(c->rbuf, alloc);
        if (!nb) return ORC_ERR;
        c->rbuf = nb;
    }
    if (pos && fill) memcpy(c->rbuf, fill, pos);
    c->rbuf_size = size;
    c->rbuf_pos = pos;
    return ORC_OK;
}
int oracle_conn_state(const orc_conn_t* c) { return c->state; }
int oracle_conn_last_reason(const orc_conn_t* c) { return c->last_reason; }
uint64_t oracle_conn_n_events(const orc_conn_t* c) { return c->n_events; }
uint64_t oracle_conn_n_messages(const orc_conn_t* c) { return c->n_messages; }
uint64_t oracle_conn_digest(const orc_conn_t* c) { return c->digest; }
size_t oracle_conn_recv_pos(const orc_conn_t* c) { return c->rbuf_pos; }
size_t oracle_conn_recv_size(const orc_conn_t* c) { return c->rbuf_size; }
size_t oracle_conn_frag_size(const orc_conn_t* c) { return c->frag ? c->frag_size : 0; }
int oracle_conn_frag_pending(const orc_conn_t* c) { return c->frag != NULL; }
size_t oracle_conn_frag_capacity(const orc_conn_t* c) { return c->frag ? c->frag_cap : 0; }
int oracle_conn_frag_opcode(const orc_conn_t* c) { return c->frag_opcode; }
/* harness: copy of recv_buffer[0, rbuf_pos) (tests compare the bytes left buffered) */
size_t oracle_conn_recv_bytes(const orc_conn_t* c, uint8_t* out, size_t cap) {
    const size_t n = c->rbuf_pos < cap ? c->rbuf_pos : cap;
    if (n && out) memcpy(out, c->rbuf, n);
    return c->rbuf_pos;
}

/* transcript record: u8 type | i32 a | u64 len | len bytes (only when record) */
static void ev_push(orc_conn_t* c, uint8_t type, int32_t a, const uint8_t* p, uint64_t len) {
    c->n_events++;
    if (!c->record) return;
    size_t need = 1 + 4 + 8 + (size_t)len;
    if (c->ev_len + need > c->ev_cap) {
        size_t nc = c->ev_cap ? c->ev_cap : 4096;
        while (nc < c->ev_len + need) nc *= 2;
        uint8_t* nb = (uint8_t*)realloc(c->ev, nc);
        if (!nb) abort();
        c->ev = nb;
        c->ev_cap = nc;
    }
    uint8_t* w = c->ev + c->ev_len;
    w[0] = type;
    memcpy(w + 1, &a, 4);
    memcpy(w + 5, &len, 8);
    if (len) memcpy(w + 13, p, (size_t)len);
    c->ev_len += need;
}

size_t oracle_conn_events(const orc_conn_t* c, uint8_t* out, size_t cap) {
    if (out && cap >= c->ev_len && c->ev_len) memcpy(out, c->ev, c->ev_len);
    return c->ev_len;
}

static void deliver_message(orc_conn_t* c, const uint8_t* p, uint64_t len, int opcode) {
    c->n_messages++;
    c->message_bytes += len;
    c->last_msg_len = len;
    c->last_msg_opcode = opcode;
    if (c->digest_on) {
        for (uint64_t i = 0; i < len; ++i) {
            c->digest ^= p[i];
            c->digest *= 1099511628211ull;
        }
    }
    ev_push(c, EV_MESSAGE, opcode, p, len);
}

/* :781-822 */
static int oracle_fragment_append(orc_conn_t* c, const uint8_t* p, size_t n) {
    size_t cap_msg = (size_t)c->max_message_size;
    if (cap_msg > 0 && (c->frag_size > cap_msg || n > cap_msg - c->frag_size)) return ORC_ERR;
    if (n > c->frag_cap - c->frag_size) {
        size_t required = c->frag_size + n;
        size_t nc = c->frag_cap;
        if (nc == 0) {
            nc = required;
        } else {
            while (nc < required) {
                if (nc > SIZE_MAX / 2) return ORC_ERR;
                nc *= 2;
            }
        }
        uint8_t* nb = (uint8_t*)realloc(c->frag, nc);
        if (!nb) return ORC_ERR;
        c->frag = nb;
        c->frag_cap = nc;
    }
    if (n) memcpy(c->frag + c->frag_size, p, n);
    c->frag_size += n;
    return ORC_OK;
}

#define FAIL(reason)             \
    do {                         \
        c->last_reason = reason; \
        return ORC_ERR;          \
    } while (0)

/* :825-1097 */
int oracle_process_data(orc_conn_t* c, const uint8_t* data, size_t len) {
    if (!c) return ORC_ERR;
    c->last_reason = R_OK;
    c->frame_completed = 0;
    if (!data) return ORC_ERR;

    /* append into the receive buffer, growing x2 up to max_frame_size (:832-869) */
    if (c->rbuf_pos + len > c->rbuf_size) {
        size_t ns = c->rbuf_size;
        if (ns > SIZE_MAX / 2) FAIL(R_BUFFER);
        ns *= 2;
        while (c->rbuf_pos + len > ns) {
            if (ns > SIZE_MAX / 2) FAIL(R_BUFFER);
            ns *= 2;
        }
        if (ns > (size_t)c->max_frame_size) {
            ns = (size_t)c->max_frame_size;
            if (c->rbuf_pos + len > ns) FAIL(R_BUFFER);
        }
        uint8_t* nb = (uint8_t*)realloc(c->rbuf, ns);
        if (!nb) FAIL(R_BUFFER);
        c->rbuf = nb;
        c->rbuf_size = ns;
    }
    if (len) memcpy(c->rbuf + c->rbuf_pos, data, len);
    c->rbuf_pos += len;

    while (c->rbuf_pos >= 2) {
        orc_header_t h;
        size_t hs;
        if (oracle_parse_frame_header(c->rbuf, c->rbuf_pos, &h, &hs) != ORC_OK) {
            uint8_t code = c->rbuf[1] & 0x7F; /* :884-890 */
            size_t need = code == 126 ? 4 : code == 127 ? 10 : 2;
            if (c->rbuf_pos < need) break;
            FAIL(R_PARSE);
        }
        if (h.rsv1 || h.rsv2 || h.rsv3) FAIL(R_RSV);                           /* :895 */
        if (h.opcode >= 0x8 && (h.payload_length > 125 || !h.fin)) FAIL(R_CONTROL); /* :902 */
        if (c->is_server && !h.mask) FAIL(R_UNMASKED);                          /* :910 */
        if (h.payload_length > (uint64_t)c->max_frame_size) FAIL(R_TOO_BIG);    /* :919 */

        size_t total = hs + (size_t)h.payload_length + (h.mask ? 4 : 0); /* :925-932 */
        if (c->rbuf_pos < total) break;

        uint8_t* payload = NULL; /* :935-947 */
        if (h.payload_length > 0) {
            payload = c->rbuf + hs;
            if (h.mask) {
                uint8_t key[4];
                memcpy(key, c->rbuf + hs, 4);
                payload += 4;
                oracle_apply_mask(payload, (size_t)h.payload_length, key);
            }
        }
        if (c->hook) c->hook(c->hook_ctx, payload, h.payload_length, h.opcode);
        const uint64_t msgs_before = c->n_messages; /* harness (frame hook) */

        if (h.opcode <= 0x2) { /* TEXT / BINARY / CONTINUATION, :950-1015 */
            if (c->frag == NULL) {
                if (h.opcode == 0x0) FAIL(R_FRAGMENT);
                if (!h.fin) {
                    c->frag_opcode = h.opcode;
                    c->frag_size = 0;
                    c->frag_cap = 0;
                    c->frag = NULL;
                    if (oracle_fragment_append(c, payload, (size_t)h.payload_length) != ORC_OK)
                        FAIL(R_MESSAGE);
                } else {
                    deliver_message(c, payload, h.payload_length, h.opcode);
                }
            } else {
                if (h.opcode != 0x0) FAIL(R_FRAGMENT);
                if (oracle_fragment_append(c, payload, (size_t)h.payload_length) != ORC_OK)
                    FAIL(R_MESSAGE);
                if (h.fin) {
                    deliver_message(c, c->frag, c->frag_size, c->frag_opcode);
                    free(c->frag);
                    c->frag = NULL;
                    c->frag_size = 0;
                    c->frag_cap = 0;
                }
            }
        } else if (h.opcode == 0x8) { /* CLOSE, :1016-1069 */
            int code = 1000;
            uint64_t rlen = 0;
            if (h.payload_length >= 2) {
                code = (payload[0] << 8) | payload[1];
                rlen = h.payload_length - 2;
            }
            ev_push(c, EV_CLOSE, code, payload ? payload + 2 : NULL, rlen);
            if (c->has_wrapper) {
                uint8_t echo[2 + 125];
                size_t elen = 0;
                if (h.payload_length >= 2) {
                    echo[0] = payload[0];
                    echo[1] = payload[1];
                    elen = 2;
                    size_t r = (size_t)h.payload_length - 2;
                    if (r > 125) r = 125;
                    if (r) {
                        memcpy(echo + 2, payload + 2, r);
                        elen += r;
                    }
                }
                ev_push(c, EV_CLOSE_ECHO, 0x8, echo, elen);
            }
            c->state = 3;
        } else if (h.opcode == 0x9) { /* PING -> PONG, :1070-1084 */
            if (c->has_wrapper) ev_push(c, EV_PONG, 0xA, payload, h.payload_length);
        }
        /* PONG and reserved opcodes: nothing (:1085) */

        if (c->frame_hook) { /* harness: the frame is complete; recv_buffer not yet drained */
            orc_conn_frame_t f;
            f.stream_off = c->consumed;
            f.payload_len = h.payload_length;
            f.payload = payload;
            f.key = h.mask ? (uint32_t)c->rbuf[hs] | (uint32_t)c->rbuf[hs + 1] << 8 |
                                 (uint32_t)c->rbuf[hs + 2] << 16 | (uint32_t)c->rbuf[hs + 3] << 24
                           : 0;
            f.opcode = h.opcode;
            f.fin = h.fin;
            f.mask = h.mask;
            f.header_size = (uint8_t)hs;
            f.msg_end = c->n_messages != msgs_before;
            c->frame_hook(c->frame_ctx, &f);
        }
        c->consumed += total;

        size_t rem = c->rbuf_pos - total; /* :1087-1093 */
        if (rem) memmove(c->rbuf, c->rbuf + total, rem);
        c->rbuf_pos = rem;
        c->frame_completed++;
    }
    return ORC_OK;
}

/* ---- batch driver: the device batch contract of include/uvhttp_ws_amd.h ----------------- */

typedef struct {
    uint32_t n_frames, n_delivered;
    int32_t status, first_status;
    uint64_t consumed_bytes, payload_bytes;
    uint32_t n_messages, state_closed;
    uint64_t arena_bytes, pending_bytes;
} orc_summary_t; /* == uvhttp_ws_batch_summary_t */

typedef struct {
    uint8_t* tmp;        /* unmasked payload of the frame being fed (copied out on success) */
    uint64_t tmp_len;
    int tmp_opcode;
    int seen;
} orc_batch_ctx_t;

static void batch_hook(void* vctx, const uint8_t* payload, uint64_t len, int opcode) {
    orc_batch_ctx_t* b = (orc_batch_ctx_t*)vctx;
    b->seen = 1;
    b->tmp_len = len;
    b->tmp_opcode = opcode;
    if (len) memcpy(b->tmp, payload, (size_t)len);
}

static uint64_t frame_start(const uint64_t* off, uint64_t stride, uint32_t i) {
    return off ? off[i] : (uint64_t)i * stride;
}

/* Decode n frames exactly as the device entry points promise (include/uvhttp_ws_amd.h):
 * each frame is fed alone to a fresh-buffered server connection, frames before the first
 * failure are delivered, the failing frame and all later ones are left untouched.
 * wire is updated in place (delivered payloads unmasked) unless arena != NULL, in which
 * case data payloads are appended to the arena and only control payloads are unmasked in
 * the wire.  status[n] receives per-frame status; msg_* (may be NULL, room for n)
 * receive the delivered messages. */
int oracle_decode_batch(uint8_t* wire, uint64_t wire_len, const uint64_t* off, uint64_t stride,
                        uint32_t n, int max_frame_size, int max_message_size, int is_server,
                        uint8_t* arena, uint64_t arena_cap, int8_t* status,
                        uint64_t* msg_off, uint64_t* msg_len, int32_t* msg_opcode,
                        orc_summary_t* sum) {
    orc_conn_t* c = oracle_conn_new(is_server, max_frame_size, max_message_size, 0);
    if (!c) return -1;
    orc_batch_ctx_t bc;
    memset(&bc, 0, sizeof(bc));
    memset(sum, 0, sizeof(*sum));
    sum->n_frames = n;
    uint64_t arena_pos = 0, msg_start = 0, tmp_cap = 0;
    uint32_t i = 0;
    int first_reason = R_OK;
    oracle_conn_set_hook(c, batch_hook, &bc);
    for (; i < n; ++i) {
        uint64_t o = frame_start(off, stride, i);
        uint64_t end = (i + 1 < n) ? frame_start(off, stride, i + 1) : wire_len;
        if (end > wire_len) end = wire_len;
        uint64_t slot = end > o ? end - o : 0;
        int last = (i + 1 == n);
        const uint8_t* p = wire + o;
        orc_header_t h;
        size_t hs = 0;
        int parsable = 0, msb = 0;
        uint64_t wlen = 0;
        memset(&h, 0, sizeof(h));
        if (slot >= 2) {
            uint8_t code = p[1] & 0x7F;
            size_t need = code == 126 ? 4 : code == 127 ? 10 : 2;
            if (slot >= need) {
                parsable = 1;
                if (oracle_parse_frame_header(p, (size_t)slot, &h, &hs) != ORC_OK) msb = 1;
                else wlen = hs + (h.mask ? 4 : 0) + h.payload_length;
            }
        }
        uint64_t fed;
        if (!last) {
            if (!parsable || (!msb && wlen != slot)) {
                first_reason = R_LAYOUT;
                break;
            }
            fed = slot;
        } else {
            fed = (parsable && !msb && wlen < slot) ? wlen : slot;
        }
        if (fed > tmp_cap) {
            tmp_cap = fed;
            bc.tmp = (uint8_t*)realloc(bc.tmp, (size_t)tmp_cap);
            if (!bc.tmp) abort();
        }
        bc.seen = 0;
        int pending_before = oracle_conn_frag_pending(c);
        uint64_t msgs_before = c->n_messages;
        if (oracle_process_data(c, p, (size_t)fed) != ORC_OK) {
            first_reason = oracle_conn_last_reason(c);
            break;
        }
        if (!c->frame_completed) {
            first_reason = R_INCOMPLETE;
            break;
        }
        /* delivered: publish the unmasked payload */
        uint64_t pay_off = o + hs + (h.mask ? 4 : 0);
        if (h.opcode <= 0x2 && arena) {
            if (!pending_before) msg_start = arena_pos;
            if (arena_pos + h.payload_length <= arena_cap && h.payload_length)
                memcpy(arena + arena_pos, bc.tmp, (size_t)h.payload_length);
            arena_pos += h.payload_length;
        } else if (h.payload_length) {
            memcpy(wire + pay_off, bc.tmp, (size_t)h.payload_length);
        }
        sum->consumed_bytes += fed;
        sum->payload_bytes += h.payload_length;
        if (h.opcode == 0x8) sum->state_closed = 1;
        if (c->n_messages != msgs_before) {
            uint64_t k = msgs_before;
            if (msg_off) msg_off[k] = msg_start;
            if (msg_len) msg_len[k] = c->last_msg_len;
            if (msg_opcode) msg_opcode[k] = c->last_msg_opcode;
        }
    }
    sum->n_delivered = i;
    sum->first_status = first_reason;
    sum->status = (first_reason < 0) ? -1 : 0;
    sum->n_messages = (uint32_t)c->n_messages;
    sum->arena_bytes = arena ? arena_pos : 0;
    sum->pending_bytes = oracle_conn_frag_size(c);
    if (status) {
        for (uint32_t k = 0; k < n; ++k)
            status[k] = k < i ? R_OK : (k == i ? (int8_t)first_reason : R_SKIPPED);
    }
    free(bc.tmp);
    oracle_conn_free(c);
    return 0;
}

/* ---- synthetic frames (definition shared with uvhttp_ws_gpu_gen_frames) ---------------- */

static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

uint64_t oracle_gen_stride(uint64_t payload_len) {
    uint64_t hs = payload_len < 126 ? 2 : payload_len < 65536 ? 4 : 10;
    return hs + 4 + payload_len;
}

uint32_t oracle_gen_key(uint64_t seed, uint32_t i, int force_keys) {
    if (force_keys && i == 0) return 0x00000000u;
    if (force_keys && i == 1) return 0xFFFFFFFFu;
    return (uint32_t)splitmix64(seed ^ (uint64_t)i);
}

/* Writes frames [first, first+count) of the synthetic batch into out (frame `first` at
 * out[0]); the full batch has n_frames frames. */
void oracle_gen_frames(uint8_t* out, uint32_t first, uint32_t count, uint32_t n_frames,
                       uint64_t payload_len, uint64_t seed, int opcode0, int fragmented,
                       int force_keys) {
    uint64_t stride = oracle_gen_stride(payload_len);
    for (uint32_t f = 0; f < count; ++f) {
        uint32_t i = first + f;
        uint8_t* w = out + (uint64_t)f * stride;
        int fin = !fragmented || i + 1 == n_frames;
        int op = (i == 0 || !fragmented) ? opcode0 : 0;
        w[0] = (uint8_t)((fin ? 0x80 : 0) | (op & 0x0F));
        size_t hs;
        if (payload_len < 126) {
            w[1] = (uint8_t)(0x80 | payload_len);
            hs = 2;
        } else if (payload_len < 65536) {
            w[1] = 0x80 | 126;
            w[2] = (uint8_t)(payload_len >> 8);
            w[3] = (uint8_t)payload_len;
            hs = 4;
        } else {
            w[1] = 0x80 | 127;
            for (int k = 0; k < 8; ++k) w[2 + k] = (uint8_t)(payload_len >> (56 - 8 * k));
            hs = 10;
        }
        uint32_t key = oracle_gen_key(seed, i, force_keys);
        uint8_t kb[4] = {(uint8_t)key, (uint8_t)(key >> 8), (uint8_t)(key >> 16),
                         (uint8_t)(key >> 24)};
        memcpy(w + hs, kb, 4);
        uint8_t* pl = w + hs + 4;
        uint64_t base = seed + ((uint64_t)i << 32);
        for (uint64_t b = 0; b < payload_len; b += 8) {
            uint64_t r = splitmix64(base + (b >> 3));
            for (int k = 0; k < 8 && b + k < payload_len; ++k)
                pl[b + k] = (uint8_t)(r >> (8 * k)) ^ kb[(b + k) & 3];
        }
    }
}

/* plaintext of frame i (what a correct unmask must produce) */
void oracle_gen_plain(uint8_t* out, uint32_t i, uint64_t payload_len, uint64_t seed) {
    uint64_t base = seed + ((uint64_t)i << 32);
    for (uint64_t b = 0; b < payload_len; b += 8) {
        uint64_t r = splitmix64(base + (b >> 3));
        for (int k = 0; k < 8 && b + k < payload_len; ++k) out[b + k] = (uint8_t)(r >> (8 * k));
    }
}

/* ---- CPU baseline kernels (bench.py cpu_baseline leg) ----------------------------------- */

/* apply_mask-only over n frames of a fixed-stride batch (per-frame key from the wire). */
uint64_t oracle_unmask_frames(uint8_t* wire, uint32_t n, uint64_t stride) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint8_t* w = wire + (uint64_t)i * stride;
        orc_header_t h;
        size_t hs;
        if (oracle_parse_frame_header(w, (size_t)stride, &h, &hs) != ORC_OK) break;
        oracle_apply_mask(w + hs + 4, (size_t)h.payload_length, w + hs);
        total += h.payload_length;
    }
    return total;
}

/* process_data fed in `chunk`-byte reads (the live-server shape, 16 KiB reads). */
uint64_t oracle_stream_decode(const uint8_t* wire, uint64_t len, size_t chunk,
                              int max_frame_size, int max_message_size, uint64_t* digest) {
    orc_conn_t* c = oracle_conn_new(1, max_frame_size, max_message_size, 0);
    if (!c) return 0;
    c->digest_on = digest != NULL;
    for (uint64_t o = 0; o < len; o += chunk) {
        size_t n = (size_t)((len - o) < chunk ? (len - o) : chunk);
        if (oracle_process_data(c, wire + o, n) != ORC_OK) break;
    }
    uint64_t bytes = c->message_bytes;
    if (digest) *digest = c->digest;
    oracle_conn_free(c);
    return bytes;
}

/* ---- stream driver: the device stream contract of include/uvhttp_ws_amd.h ---------------- */
/* Many connections, each fed its process_data calls (src/uvhttp_connection.c:1128-1164:
 * one call per read until a call fails) — the checker of uvhttp_ws_gpu_decode_streams /
 * _decode_reads at any size.  Layouts == uvhttp_ws_stream_t (64 B). */
typedef struct {
    uint64_t begin, len, recv_buffer_size, pending_bytes;
    int32_t pending_opcode, max_frame_size, max_message_size, is_server;
    uint32_t first_read, n_reads;
    uint64_t reserved;
} orc_stream_t;

/* per connection: what its process_data calls returned and left (64 B) */
typedef struct {
    uint32_t n_frames;      /* frames completed (delivered) */
    uint32_t calls;         /* calls that ran, a failing one included */
    int32_t rc;             /* the last call's return */
    int32_t reason;         /* R_* of the failure (0 if none) */
    uint64_t consumed;      /* bytes drained by completed frames */
    uint64_t recv_pos;      /* bytes left in recv_buffer */
    uint64_t recv_size;
    uint64_t frag_size;     /* open fragmented message (0 = none) */
    int32_t frag_opcode;
    uint32_t n_messages;
    uint64_t digest;        /* FNV-1a 64 over delivered message bytes (pending prefix = zeros;
                               only when asked: it is a byte-serial loop) */
} orc_stream_out_t;

/* per completed frame, connections in order (32 B) */
typedef struct {
    uint64_t payload_off;   /* absolute wire offset of the payload */
    uint64_t payload_len;
    uint32_t key;
    uint8_t opcode, flags, header_size, reserved; /* flags: 1 FIN, 2 MASK, 0x20 MSG_END */
    uint32_t conn;
    uint32_t wire_len;
} orc_stream_frame_t;

typedef struct {
    uint8_t* wire;          /* delivered payloads are written back unmasked here */
    uint64_t begin;
    orc_stream_frame_t* frames;
    uint64_t cap, n;
    uint32_t conn;
} orc_stream_ctx_t;

static void stream_frame_hook(void* vctx, orc_conn_frame_t* f) {
    orc_stream_ctx_t* x = (orc_stream_ctx_t*)vctx;
    const uint64_t poff = x->begin + f->stream_off + f->header_size + (f->mask ? 4 : 0);
    if (f->payload_len && f->payload) memcpy(x->wire + poff, f->payload, (size_t)f->payload_len);
    if (x->n < x->cap) {
        orc_stream_frame_t* o = &x->frames[x->n];
        o->payload_off = poff;
        o->payload_len = f->payload_len;
        o->key = f->key;
        o->opcode = f->opcode;
        o->flags = (uint8_t)((f->fin ? 1 : 0) | (f->mask ? 2 : 0) | (f->msg_end ? 0x20 : 0));
        o->header_size = f->header_size;
        o->reserved = 0;
        o->conn = x->conn;
        uint64_t wl = f->header_size + (f->mask ? 4 : 0) + f->payload_len;
        o->wire_len = wl > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)wl;
    }
    x->n++;
}

/* Returns the number of completed frames over all connections (frames beyond max_frames
 * are counted, not stored).  wire is decoded in place like the device's stream decode. */
uint64_t oracle_decode_streams(uint8_t* wire, const orc_stream_t* s, uint32_t n,
                               const uint64_t* read_end, orc_stream_out_t* out,
                               orc_stream_frame_t* frames, uint64_t max_frames, int digest) {
    orc_stream_ctx_t x;
    memset(&x, 0, sizeof(x));
    x.wire = wire;
    x.frames = frames;
    x.cap = frames ? max_frames : 0;
    for (uint32_t k = 0; k < n; ++k) {
        const orc_stream_t* st = &s[k];
        orc_stream_out_t* o = &out[k];
        memset(o, 0, sizeof(*o));
        orc_conn_t* c = oracle_conn_new(st->is_server, st->max_frame_size, st->max_message_size, 0);
        if (!c) abort();
        c->digest_on = digest;
        if (oracle_conn_set_recv_state(c, (size_t)st->recv_buffer_size, NULL, 0) != ORC_OK) abort();
        if (st->pending_bytes) { /* an open fragmented message from earlier calls (zeros) */
            c->frag = (uint8_t*)calloc(1, (size_t)st->pending_bytes);
            if (!c->frag) abort();
            c->frag_size = c->frag_cap = (size_t)st->pending_bytes;
            c->frag_opcode = st->pending_opcode;
        }
        x.begin = st->begin;
        x.conn = k;
        uint64_t before = x.n;
        c->frame_hook = stream_frame_hook;
        c->frame_ctx = &x;
        uint32_t nr = st->n_reads ? st->n_reads : 1;
        uint64_t pos = 0;
        for (uint32_t r = 0; r < nr; ++r) {
            uint64_t end = st->n_reads ? read_end[st->first_read + r] : st->len;
            o->calls++;
            o->rc = oracle_process_data(c, wire + st->begin + pos, (size_t)(end - pos));
            pos = end;
            if (o->rc != ORC_OK) {
                o->reason = c->last_reason;
                break;
            }
        }
        o->n_frames = (uint32_t)(x.n - before);
        o->consumed = c->consumed;
        o->recv_pos = c->rbuf_pos;
        o->recv_size = c->rbuf_size;
        o->frag_size = oracle_conn_frag_size(c);
        o->frag_opcode = c->frag_opcode;
        o->n_messages = (uint32_t)c->n_messages;
        o->digest = c->digest;
        oracle_conn_free(c);
    }
    return x.n;
}

/* ---- send side: uvhttp_ws_build_frame (:204-285) --------------------------------------- */
/* The reference draws the client masking key from the context DRBG (:257-266, :55-68);
 * here the key is an argument (the DRBG is host-side mbedtls, outside this path). */
long oracle_build_frame(uint8_t* buf, size_t cap, const uint8_t* payload, size_t plen,
                        int opcode, int mask, int fin, const uint8_t* key) {
    if (!buf) return -1;
    size_t hs = plen < 126 ? 2 : plen < 65536 ? 4 : 10;
    if (plen > SIZE_MAX - hs - (mask ? 4 : 0)) return -1;
    size_t total = hs + plen + (mask ? 4 : 0);
    if (cap < total) return -1;
    buf[0] = (uint8_t)((fin ? 0x80 : 0x00) | (opcode & 0x0F));
    if (plen < 126) {
        buf[1] = (uint8_t)((mask ? 0x80 : 0x00) | plen);
    } else if (plen < 65536) {
        buf[1] = (uint8_t)((mask ? 0x80 : 0x00) | 126);
        buf[2] = (uint8_t)((plen >> 8) & 0xFF);
        buf[3] = (uint8_t)(plen & 0xFF);
    } else {
        uint64_t l = (uint64_t)plen;
        buf[1] = (uint8_t)((mask ? 0x80 : 0x00) | 127);
        for (int k = 0; k < 8; ++k) buf[2 + k] = (uint8_t)((l >> (56 - 8 * k)) & 0xFF);
    }
    if (mask) {
        for (int k = 0; k < 4; ++k) buf[hs + k] = key[k];
        if (payload && plen > 0) {
            memcpy(buf + hs + 4, payload, plen);
            oracle_apply_mask(buf + hs + 4, plen, key);
        }
    } else if (payload && plen > 0) {
        memcpy(buf + hs, payload, plen);
    }
    return (long)total;
}
