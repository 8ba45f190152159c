/*
 * ws_host.c — drop-in host side of the decode surface (include/uvhttp_ws_amd.h §1b).
 *
 * These are the functions src/uvhttp_connection.c links against
 * (on_websocket_read -> uvhttp_ws_process_data, src/uvhttp_connection.c:1154-1164).  A live
 * libuv read is <= 16 KiB (include/uvhttp_constants.h:207-208), far below what pays for a
 * device round trip, so the per-connection stream path runs here on the host; batches of
 * frames resident in HBM go through the gfx950 kernels in ws_gpu.hip instead.
 *
 * Structure: process_data = append (grow_recv) -> repeat { scan_frame -> unmask ->
 * dispatch_frame -> drain } until the buffered bytes hold no complete frame.  The observable
 * behaviour — return codes, callback order and arguments, recv/fragment buffer sizes, state —
 * matches src/uvhttp_websocket.c:825-1097; tests/test_host_dropin.py replays the reference's
 * own known-answer tests and a randomized stream against the oracle to check it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "uvhttp_ws_amd.h"

static uvhttp_ws_amd_context_resolver g_resolver = NULL;
static uvhttp_ws_amd_control_sink g_control_sink = NULL;

void uvhttp_ws_amd_set_control_hooks(uvhttp_ws_amd_context_resolver resolver,
                                     uvhttp_ws_amd_control_sink sink) {
    g_resolver = resolver;
    g_control_sink = sink;
}

/* the server context the reference reaches through conn->user_data, or NULL */
static void* server_context(uvhttp_ws_connection_t* c) {
    return (c->user_data != NULL && g_resolver != NULL) ? g_resolver(c) : NULL;
}

/* ---- connection lifetime (src/uvhttp_websocket.c:71-130, 1100-1111) ------------------- */

struct uvhttp_ws_connection* uvhttp_ws_connection_create(int fd, mbedtls_ssl_context* ssl,
                                                         int is_server,
                                                         const uvhttp_config_t* config) {
    uvhttp_ws_connection_t* c = (uvhttp_ws_connection_t*)calloc(1, sizeof(*c));
    if (c == NULL) return NULL;
    c->fd = fd;
    c->ssl = ssl;
    c->is_server = is_server;
    c->state = UVHTTP_WS_STATE_CONNECTING;
    c->config.max_frame_size =
        config ? config->websocket_max_frame_size : UVHTTP_WS_AMD_DEFAULT_MAX_FRAME_SIZE;
    c->config.max_message_size =
        config ? config->websocket_max_message_size : UVHTTP_WS_AMD_DEFAULT_MAX_MESSAGE_SIZE;
    c->config.ping_interval =
        config ? config->websocket_ping_interval : UVHTTP_WS_AMD_DEFAULT_PING_INTERVAL;
    c->config.ping_timeout =
        config ? config->websocket_ping_timeout : UVHTTP_WS_AMD_DEFAULT_PING_TIMEOUT;
    c->recv_buffer_size = UVHTTP_WS_AMD_DEFAULT_RECV_BUFFER_SIZE;
    c->recv_buffer = (uint8_t*)malloc(c->recv_buffer_size);
    if (c->recv_buffer == NULL) {
        free(c);
        return NULL;
    }
    return c;
}

void uvhttp_ws_connection_free(struct uvhttp_ws_connection* c) {
    if (c == NULL) return;
    free(c->recv_buffer);
    free(c->send_buffer);
    free(c->fragmented_message);
    free(c);
}

void uvhttp_ws_set_callbacks(struct uvhttp_ws_connection* c,
                             uvhttp_ws_on_message_callback on_message,
                             uvhttp_ws_on_close_callback on_close,
                             uvhttp_ws_on_error_callback on_error) {
    if (c == NULL) return;
    c->on_message = on_message;
    c->on_close = on_close;
    c->on_error = on_error;
}

/* ---- header + mask --------------------------------------------------------------------- */

/* Length code -> bytes of header before the mask key (RFC 6455 §5.2). */
static size_t header_span(uint8_t second_byte) {
    uint8_t code = second_byte & 0x7F;
    return code == 126 ? 4 : code == 127 ? 10 : 2;
}

uvhttp_error_t uvhttp_ws_parse_frame_header(const uint8_t* data, size_t len,
                                            uvhttp_ws_frame_header_t* header,
                                            size_t* header_size) {
    if (data == NULL || header == NULL || header_size == NULL || len < 2)
        return UVHTTP_ERROR_INVALID_PARAM;
    memset(header, 0, sizeof(*header));
    const uint8_t b0 = data[0], b1 = data[1];
    header->fin = b0 >> 7;
    header->rsv1 = (b0 >> 6) & 1;
    header->rsv2 = (b0 >> 5) & 1;
    header->rsv3 = (b0 >> 4) & 1;
    header->opcode = b0 & 0x0F;
    header->mask = b1 >> 7;
    header->payload_len = b1 & 0x7F;
    const size_t span = header_span(b1);
    uint64_t length = b1 & 0x7F;
    header->payload_length = length;
    *header_size = 2;
    if (span > 2) {
        if (len < span) return UVHTTP_ERROR_INVALID_PARAM;
        length = 0;
        for (size_t k = 2; k < span; ++k) length = (length << 8) | data[k];
        header->payload_length = length;
        if (span == 10 && (length >> 63)) return UVHTTP_ERROR_INVALID_PARAM;
        *header_size = span;
    }
    header->payload_length = length;
    return UVHTTP_OK;
}

/* Word-at-a-time XOR: the key rotated to the first aligned byte is replicated into a
 * 64-bit word; head and tail bytes use the plain byte rule. */
void uvhttp_ws_apply_mask(uint8_t* data, size_t len, const uint8_t* key) {
    if (data == NULL || key == NULL) return;
    size_t i = 0;
    while (i < len && ((uintptr_t)(data + i) & 7u)) {
        data[i] ^= key[i & 3];
        ++i;
    }
    if (len - i >= 8) {
        uint8_t rot[8];
        for (int b = 0; b < 8; ++b) rot[b] = key[(i + (size_t)b) & 3];
        uint64_t k64;
        memcpy(&k64, rot, 8);
        uint64_t* w = (uint64_t*)(void*)(data + i);
        size_t nw = (len - i) / 8;
        for (size_t j = 0; j < nw; ++j) w[j] ^= k64;
        i += nw * 8;
    }
    for (; i < len; ++i) data[i] ^= key[i & 3];
}

/* ---- stream decode ----------------------------------------------------------------------- */

enum scan_outcome { SCAN_FRAME, SCAN_NEED_MORE, SCAN_REJECT };

typedef struct {
    uvhttp_ws_frame_header_t hdr;
    size_t head;  /* header bytes before the key */
    size_t total; /* header + key + payload */
} frame_view_t;

/* Recv-buffer growth (src/uvhttp_websocket.c:832-866): double until the new bytes fit,
 * never beyond config.max_frame_size. */
static int grow_recv(uvhttp_ws_connection_t* c, size_t extra) {
    const size_t want = c->recv_buffer_pos + extra;
    if (want <= c->recv_buffer_size) return 0;
    size_t cap = c->recv_buffer_size;
    do {
        if (cap > SIZE_MAX / 2) return -1;
        cap *= 2;
    } while (want > cap);
    const size_t ceiling = (size_t)c->config.max_frame_size;
    if (cap > ceiling) {
        cap = ceiling;
        if (want > cap) return -1;
    }
    uint8_t* nb = (uint8_t*)realloc(c->recv_buffer, cap);
    if (nb == NULL) return -1;
    c->recv_buffer = nb;
    c->recv_buffer_size = cap;
    return 0;
}

/* Decide what the head of the receive buffer holds (src/uvhttp_websocket.c:876-932). */
static enum scan_outcome scan_frame(const uvhttp_ws_connection_t* c, frame_view_t* v) {
    const uint8_t* buf = c->recv_buffer;
    const size_t have = c->recv_buffer_pos;
    if (uvhttp_ws_parse_frame_header(buf, have, &v->hdr, &v->head) != UVHTTP_OK)
        return have < header_span(buf[1]) ? SCAN_NEED_MORE : SCAN_REJECT;
    const uvhttp_ws_frame_header_t* h = &v->hdr;
    if (h->rsv1 | h->rsv2 | h->rsv3) return SCAN_REJECT;
    if (h->opcode >= UVHTTP_WS_OPCODE_CLOSE && (h->payload_length > 125 || !h->fin))
        return SCAN_REJECT;
    if (c->is_server && !h->mask) return SCAN_REJECT;
    if (h->payload_length > (uint64_t)c->config.max_frame_size) return SCAN_REJECT;
    v->total = v->head + (h->mask ? 4u : 0u) + (size_t)h->payload_length;
    return have < v->total ? SCAN_NEED_MORE : SCAN_FRAME;
}

/* uvhttp_ws_fragment_append semantics (src/uvhttp_websocket.c:781-822). */
static int append_fragment(uvhttp_ws_connection_t* c, const uint8_t* p, size_t n) {
    const size_t limit = (size_t)c->config.max_message_size;
    if (limit != 0 && (c->fragmented_size > limit || n > limit - c->fragmented_size)) return -1;
    if (n > c->fragmented_capacity - c->fragmented_size) {
        const size_t need = c->fragmented_size + n;
        size_t cap = c->fragmented_capacity;
        if (cap == 0) {
            cap = need;
        } else {
            while (cap < need) {
                if (cap > SIZE_MAX / 2) return -1;
                cap *= 2;
            }
        }
        uint8_t* nb = (uint8_t*)realloc(c->fragmented_message, cap);
        if (nb == NULL) return -1;
        c->fragmented_message = nb;
        c->fragmented_capacity = cap;
    }
    if (n) memcpy(c->fragmented_message + c->fragmented_size, p, n);
    c->fragmented_size += n;
    return 0;
}

static void drop_fragment(uvhttp_ws_connection_t* c) {
    free(c->fragmented_message);
    c->fragmented_message = NULL;
    c->fragmented_size = 0;
    c->fragmented_capacity = 0;
}

/* Data frames: RFC 6455 §5.4 reassembly (src/uvhttp_websocket.c:950-1015). */
static int on_data_frame(uvhttp_ws_connection_t* c, const uvhttp_ws_frame_header_t* h,
                         const uint8_t* payload) {
    const size_t n = (size_t)h->payload_length;
    const int is_cont = h->opcode == UVHTTP_WS_OPCODE_CONTINUATION;
    if (c->fragmented_message != NULL) { /* a message is open */
        if (!is_cont) return -1;
        if (append_fragment(c, payload, n) != 0) return -1;
        if (h->fin) {
            if (c->on_message)
                c->on_message(c, (const char*)c->fragmented_message, c->fragmented_size,
                              c->fragmented_opcode);
            drop_fragment(c);
        }
        return 0;
    }
    if (is_cont) return -1;
    if (h->fin) {
        if (c->on_message) c->on_message(c, (const char*)payload, n, h->opcode);
        return 0;
    }
    c->fragmented_opcode = (uvhttp_ws_opcode_t)h->opcode;
    c->fragmented_size = 0;
    c->fragmented_capacity = 0;
    c->fragmented_message = NULL;
    return append_fragment(c, payload, n);
}

/* CLOSE (src/uvhttp_websocket.c:1016-1069). */
static void on_close_frame(uvhttp_ws_connection_t* c, const uint8_t* payload, size_t n) {
    int code = 1000;
    const char* reason = "";
    if (n >= 2) {
        code = (payload[0] << 8) | payload[1];
        if (n > 2) reason = (const char*)(payload + 2);
    }
    void* ctx = server_context(c); /* captured before on_close frees the wrapper */
    if (c->on_close) c->on_close(c, code, reason);
    if (ctx != NULL && g_control_sink != NULL) {
        uint8_t echo[2 + 125];
        size_t elen = 0;
        if (n >= 2) {
            size_t r = n - 2 > 125 ? 125 : n - 2;
            memcpy(echo, payload, 2 + r);
            elen = 2 + r;
        }
        g_control_sink(ctx, c, UVHTTP_WS_OPCODE_CLOSE, echo, elen);
    }
    c->state = UVHTTP_WS_STATE_CLOSED;
}

static int dispatch_frame(uvhttp_ws_connection_t* c, const uvhttp_ws_frame_header_t* h,
                          const uint8_t* payload) {
    switch (h->opcode) {
        case UVHTTP_WS_OPCODE_CONTINUATION:
        case UVHTTP_WS_OPCODE_TEXT:
        case UVHTTP_WS_OPCODE_BINARY:
            return on_data_frame(c, h, payload);
        case UVHTTP_WS_OPCODE_CLOSE:
            on_close_frame(c, payload, (size_t)h->payload_length);
            return 0;
        case UVHTTP_WS_OPCODE_PING: { /* src/uvhttp_websocket.c:1070-1084 */
            void* ctx = server_context(c);
            if (ctx != NULL && g_control_sink != NULL)
                g_control_sink(ctx, c, UVHTTP_WS_OPCODE_PONG, payload, (size_t)h->payload_length);
            return 0;
        }
        default: /* PONG and reserved opcodes are ignored (:1085) */
            return 0;
    }
}

uvhttp_error_t uvhttp_ws_process_data(struct uvhttp_ws_connection* c, const uint8_t* data,
                                      size_t len) {
    if (c == NULL || data == NULL) return UVHTTP_ERROR_INVALID_PARAM;
    if (grow_recv(c, len) != 0) return UVHTTP_ERROR_INVALID_PARAM;
    if (len) memcpy(c->recv_buffer + c->recv_buffer_pos, data, len);
    c->recv_buffer_pos += len;

    while (c->recv_buffer_pos >= 2) {
        frame_view_t v;
        const enum scan_outcome s = scan_frame(c, &v);
        if (s == SCAN_NEED_MORE) break;
        if (s == SCAN_REJECT) return UVHTTP_ERROR_INVALID_PARAM;

        uint8_t* payload = NULL;
        if (v.hdr.payload_length > 0) {
            payload = c->recv_buffer + v.head;
            if (v.hdr.mask) {
                uint8_t key[4];
                memcpy(key, payload, 4);
                payload += 4;
                uvhttp_ws_apply_mask(payload, (size_t)v.hdr.payload_length, key);
            }
        }
        if (dispatch_frame(c, &v.hdr, payload) != 0) return UVHTTP_ERROR_INVALID_PARAM;

        const size_t rest = c->recv_buffer_pos - v.total;
        if (rest) memmove(c->recv_buffer, c->recv_buffer + v.total, rest);
        c->recv_buffer_pos = rest;
    }
    return UVHTTP_OK;
}

/* ---- delivery of a device-decoded batch (include/uvhttp_ws_amd.h) ----------------------- */

uvhttp_error_t uvhttp_ws_deliver_batch(struct uvhttp_ws_connection* c, const uint8_t* wire,
                                       const uvhttp_ws_frame_desc_t* desc,
                                       const uvhttp_ws_batch_summary_t* summary) {
    if (c == NULL || summary == NULL || (summary->n_delivered && (wire == NULL || desc == NULL)))
        return UVHTTP_ERROR_INVALID_PARAM;
    for (uint32_t i = 0; i < summary->n_delivered; ++i) {
        const uvhttp_ws_frame_desc_t* d = &desc[i];
        uvhttp_ws_frame_header_t h;
        memset(&h, 0, sizeof(h));
        h.fin = (d->flags & UVHTTP_WS_FLAG_FIN) ? 1 : 0;
        h.mask = (d->flags & UVHTTP_WS_FLAG_MASK) ? 1 : 0;
        h.opcode = d->opcode & 0x0F;
        h.payload_length = d->payload_len;
        const uint8_t* payload = d->payload_len ? wire + d->payload_off : NULL;
        if (dispatch_frame(c, &h, payload) != 0) return UVHTTP_ERROR_INVALID_PARAM;
    }
    return summary->status == 0 ? UVHTTP_OK : UVHTTP_ERROR_INVALID_PARAM;
}

/* A control frame of a compact decode (payload unmasked in place in the wire) through the
 * same dispatch as process_data; data frames of reserved opcodes fall through to its default. */
static void dispatch_control(uvhttp_ws_connection_t* c, int opcode, const uint8_t* payload,
                             uint64_t len) {
    uvhttp_ws_frame_header_t h;
    memset(&h, 0, sizeof(h));
    h.fin = 1;
    h.opcode = (uint8_t)(opcode & 0x0F);
    h.payload_length = len;
    (void)dispatch_frame(c, &h, len ? payload : NULL);
}

/* The delivered frames of a compact decode are its messages (each fires at its last frame) and
 * its non-data frames, merged in frame order (include/uvhttp_ws_amd.h). */
uvhttp_error_t uvhttp_ws_deliver_messages(struct uvhttp_ws_connection* c, const uint8_t* arena,
                                          const uvhttp_ws_message_desc_t* msgs,
                                          const uvhttp_ws_batch_summary_t* summary,
                                          const uint8_t* wire, const uvhttp_ws_frame_desc_t* desc,
                                          uint64_t frame_stride) {
    if (c == NULL || summary == NULL || c->fragmented_message != NULL)
        return UVHTTP_ERROR_INVALID_PARAM;
    const uint32_t nd = summary->n_delivered, nm = summary->n_messages;
    const int open = summary->pending_bytes != 0;
    if (nd > summary->n_frames || nm > nd || ((nm || open) && (msgs == NULL || arena == NULL)))
        return UVHTTP_ERROR_INVALID_PARAM;
    /* every message inside the arena, in frame order, ending at a delivered frame */
    for (uint32_t m = 0; m < nm + (uint32_t)open; ++m) {
        const uvhttp_ws_message_desc_t* d = &msgs[m];
        if (d->arena_off > summary->arena_bytes || d->len > summary->arena_bytes - d->arena_off ||
            d->first_frame > d->last_frame || d->last_frame >= nd ||
            (m && d->first_frame <= msgs[m - 1].last_frame))
            return UVHTTP_ERROR_INVALID_PARAM;
    }
    if (open && (msgs[nm].len != summary->pending_bytes || msgs[nm].reserved == 0))
        return UVHTTP_ERROR_INVALID_PARAM;
    /* summary-only: only the last delivered frame can be a non-data frame (frames of a
     * >= 140-byte stride are too long to be control frames); find out whether it is one */
    const uint8_t* last_ctl = NULL;
    uvhttp_ws_frame_header_t lh;
    size_t lhead = 0;
    if (desc == NULL && nd > 0) {
        if (frame_stride < 140) return UVHTTP_ERROR_INVALID_PARAM;
        const uint32_t last = nd - 1;
        const int covered = (nm && msgs[nm - 1].last_frame == last) || (open && msgs[nm].last_frame == last);
        if (!covered) {
            if (wire == NULL) return UVHTTP_ERROR_INVALID_PARAM;
            last_ctl = wire + (size_t)last * frame_stride;
            if (uvhttp_ws_parse_frame_header(last_ctl, (size_t)frame_stride, &lh, &lhead) != UVHTTP_OK)
                return UVHTTP_ERROR_INVALID_PARAM;
            if (lh.opcode < UVHTTP_WS_OPCODE_CLOSE) last_ctl = NULL; /* a data frame that completes
                                                                      nothing: a zero-length start */
        }
    }
    if (desc != NULL && nd > 0 && wire == NULL) {
        for (uint32_t i = 0; i < nd; ++i)
            if (desc[i].opcode >= UVHTTP_WS_OPCODE_CLOSE && desc[i].payload_len)
                return UVHTTP_ERROR_INVALID_PARAM;
    }

    uint32_t m = 0;
    if (desc != NULL) {
        for (uint32_t i = 0; i < nd; ++i) {
            const uvhttp_ws_frame_desc_t* d = &desc[i];
            if (d->opcode < UVHTTP_WS_OPCODE_CLOSE) continue; /* data frames: their messages */
            for (; m < nm && msgs[m].last_frame < i; ++m)
                if (c->on_message)
                    c->on_message(c, (const char*)arena + msgs[m].arena_off, (size_t)msgs[m].len,
                                  msgs[m].opcode);
            dispatch_control(c, d->opcode, wire ? wire + d->payload_off : NULL, d->payload_len);
        }
    }
    for (; m < nm; ++m)
        if (c->on_message)
            c->on_message(c, (const char*)arena + msgs[m].arena_off, (size_t)msgs[m].len,
                          msgs[m].opcode);
    if (last_ctl != NULL)
        dispatch_control(c, lh.opcode, last_ctl + lhead + (lh.mask ? 4u : 0u), lh.payload_length);
    if (open) { /* the open message as append_fragment left it: capacity = first fragment
                   doubled until it holds everything appended (src/uvhttp_websocket.c:794-816) */
        const uvhttp_ws_message_desc_t* d = &msgs[nm];
        size_t cap = (size_t)d->reserved;
        while (cap < (size_t)d->len) {
            if (cap > SIZE_MAX / 2) return UVHTTP_ERROR_INVALID_PARAM;
            cap *= 2;
        }
        uint8_t* buf = (uint8_t*)malloc(cap);
        if (buf == NULL) return UVHTTP_ERROR_INVALID_PARAM;
        memcpy(buf, arena + d->arena_off, (size_t)d->len);
        c->fragmented_message = buf;
        c->fragmented_size = (size_t)d->len;
        c->fragmented_capacity = cap;
        c->fragmented_opcode = (uvhttp_ws_opcode_t)d->opcode;
    }
    return summary->status == 0 ? UVHTTP_OK : UVHTTP_ERROR_INVALID_PARAM;
}

/* ---- stream decode, host side (include/uvhttp_ws_amd.h) ---------------------------------- */

void uvhttp_ws_stream_init(const struct uvhttp_ws_connection* c, uint64_t begin, uint64_t len,
                           uvhttp_ws_stream_t* out) {
    if (c == NULL || out == NULL) return;
    memset(out, 0, sizeof(*out));
    out->begin = begin;
    out->len = len;
    out->recv_buffer_size = c->recv_buffer_size;
    out->pending_bytes = c->fragmented_message != NULL ? c->fragmented_size : 0;
    out->pending_opcode = (int32_t)c->fragmented_opcode;
    out->max_frame_size = c->config.max_frame_size;
    out->max_message_size = c->config.max_message_size;
    out->is_server = c->is_server;
}

uvhttp_error_t uvhttp_ws_deliver_stream(struct uvhttp_ws_connection* c, const uint8_t* wire,
                                        const uvhttp_ws_frame_desc_t* desc,
                                        const uvhttp_ws_stream_t* s,
                                        const uvhttp_ws_stream_result_t* r) {
    if (c == NULL || s == NULL || r == NULL || (s->len && wire == NULL))
        return UVHTTP_ERROR_INVALID_PARAM;
    /* nothing ran on the connection: a malformed descriptor, too many frames for the batch,
     * a device fault, or the first call failed its growth check and returned before touching
     * the buffer (src/uvhttp_websocket.c:836-857) */
    if (r->first_status == UVHTTP_WS_FRAME_ERR_CAPACITY ||
        r->first_status == UVHTTP_WS_FRAME_ERR_LAYOUT ||
        r->first_status == UVHTTP_WS_FRAME_ERR_DEVICE ||
        (r->first_status == UVHTTP_WS_FRAME_ERR_BUFFER && r->calls <= 1))
        return UVHTTP_ERROR_INVALID_PARAM;
    if (r->consumed_bytes > r->buffered_end || r->buffered_end > s->len ||
        (r->n_delivered && desc == NULL))
        return UVHTTP_ERROR_INVALID_PARAM;
    if (r->recv_buffer_size != c->recv_buffer_size) {
        uint8_t* nb = (uint8_t*)realloc(c->recv_buffer, (size_t)r->recv_buffer_size);
        if (nb == NULL) return UVHTTP_ERROR_INVALID_PARAM;
        c->recv_buffer = nb;
        c->recv_buffer_size = (size_t)r->recv_buffer_size;
    }
    const uint8_t* base = wire + s->begin;
    for (uint32_t k = 0; k < r->n_delivered; ++k) {
        const uvhttp_ws_frame_desc_t* d = &desc[r->first_frame + k];
        uvhttp_ws_frame_header_t h;
        memset(&h, 0, sizeof(h));
        h.fin = (d->flags & UVHTTP_WS_FLAG_FIN) ? 1 : 0;
        h.mask = (d->flags & UVHTTP_WS_FLAG_MASK) ? 1 : 0;
        h.opcode = d->opcode & 0x0F;
        h.payload_length = d->payload_len;
        const uint8_t* payload = d->payload_len ? wire + d->payload_off : NULL;
        if (dispatch_frame(c, &h, payload) != 0) break; /* cannot happen after a clean decode */
    }
    /* what the calls leave buffered: the stream bytes after the delivered frames, up to the
     * end of the last call that ran */
    const size_t rest = (size_t)(r->buffered_end - r->consumed_bytes);
    if (rest) memmove(c->recv_buffer, base + r->consumed_bytes, rest);
    c->recv_buffer_pos = rest;
    /* a complete data frame rejected by the fragment state machine: the reference unmasked it
     * in recv_buffer (:944) before its fragment checks failed (:964-1000), and those checks
     * may already have changed the fragment state (a start records its opcode before the
     * size check) — replay that frame's unmask and dispatch, which fails the same way */
    if ((r->first_status == UVHTTP_WS_FRAME_ERR_FRAGMENT ||
         r->first_status == UVHTTP_WS_FRAME_ERR_MESSAGE) && desc != NULL) {
        const uvhttp_ws_frame_desc_t* d = &desc[r->first_frame + r->n_delivered];
        const size_t at = (size_t)(d->payload_off - s->begin - r->consumed_bytes);
        if (d->payload_len && at + d->payload_len <= rest) {
            uint8_t* payload = c->recv_buffer + at;
            if (d->flags & UVHTTP_WS_FLAG_MASK) {
                uint8_t key[4];
                memcpy(key, &d->masking_key, 4); /* k0 = low byte */
                uvhttp_ws_apply_mask(payload, (size_t)d->payload_len, key);
            }
            uvhttp_ws_frame_header_t h;
            memset(&h, 0, sizeof(h));
            h.fin = (d->flags & UVHTTP_WS_FLAG_FIN) ? 1 : 0;
            h.mask = (d->flags & UVHTTP_WS_FLAG_MASK) ? 1 : 0;
            h.opcode = d->opcode & 0x0F;
            h.payload_length = d->payload_len;
            (void)dispatch_frame(c, &h, payload);
        } else if (!d->payload_len) {
            uvhttp_ws_frame_header_t h;
            memset(&h, 0, sizeof(h));
            h.fin = (d->flags & UVHTTP_WS_FLAG_FIN) ? 1 : 0;
            h.opcode = d->opcode & 0x0F;
            (void)dispatch_frame(c, &h, NULL);
        }
    }
    return r->status == 0 ? UVHTTP_OK : UVHTTP_ERROR_INVALID_PARAM;
}

/* Copy of a read into the batcher's pinned arena (ws_batcher.hip; internal).  The arena is
 * only read again by the DMA engine, so whole vectors go out with non-temporal stores: no
 * read-for-ownership of the destination lines, no cache pollution (glibc memcpy switches to
 * streaming stores only far above libuv's 16 KiB reads).  32-byte AVX2 streaming stores where
 * the CPU has them: 91 GB/s into pinned memory on the MI355X box's EPYC 9575F against 54-59 GB/s
 * for 16-byte SSE2 ones and 45 GB/s for memcpy (tools/copy_probe.cpp,
 * profiles/r03p42_copy_probe.jsonl).  Other targets (the host decoder builds anywhere) copy
 * with memcpy and fence with a full barrier. */
#if defined(__x86_64__) || defined(__i386__)
#include <immintrin.h>

__attribute__((target("avx2"))) static void copy_stream_avx2(uint8_t* d, const uint8_t* s, size_t len) {
    const size_t head = (32u - ((uintptr_t)d & 31u)) & 31u;
    memcpy(d, s, head);
    d += head;
    s += head;
    len -= head;
    size_t i = 0;
    for (; i + 128 <= len; i += 128) {
        const __m256i a = _mm256_loadu_si256((const __m256i*)(s + i));
        const __m256i b = _mm256_loadu_si256((const __m256i*)(s + i + 32));
        const __m256i c = _mm256_loadu_si256((const __m256i*)(s + i + 64));
        const __m256i e = _mm256_loadu_si256((const __m256i*)(s + i + 96));
        _mm256_stream_si256((__m256i*)(d + i), a);
        _mm256_stream_si256((__m256i*)(d + i + 32), b);
        _mm256_stream_si256((__m256i*)(d + i + 64), c);
        _mm256_stream_si256((__m256i*)(d + i + 96), e);
    }
    for (; i + 32 <= len; i += 32)
        _mm256_stream_si256((__m256i*)(d + i), _mm256_loadu_si256((const __m256i*)(s + i)));
    memcpy(d + i, s + i, len - i);
}

static void copy_stream_sse2(uint8_t* d, const uint8_t* s, size_t len) {
    const size_t head = (16u - ((uintptr_t)d & 15u)) & 15u;
    memcpy(d, s, head);
    d += head;
    s += head;
    len -= head;
    size_t i = 0;
    for (; i + 64 <= len; i += 64) {
        const __m128i a = _mm_loadu_si128((const __m128i*)(s + i));
        const __m128i b = _mm_loadu_si128((const __m128i*)(s + i + 16));
        const __m128i c = _mm_loadu_si128((const __m128i*)(s + i + 32));
        const __m128i e = _mm_loadu_si128((const __m128i*)(s + i + 48));
        _mm_stream_si128((__m128i*)(d + i), a);
        _mm_stream_si128((__m128i*)(d + i + 16), b);
        _mm_stream_si128((__m128i*)(d + i + 32), c);
        _mm_stream_si128((__m128i*)(d + i + 48), e);
    }
    for (; i + 16 <= len; i += 16)
        _mm_stream_si128((__m128i*)(d + i), _mm_loadu_si128((const __m128i*)(s + i)));
    memcpy(d + i, s + i, len - i);
}

/* The streaming stores of copy_stream are weakly ordered: make them visible before a DMA engine
 * reads the arena (the batcher calls this before each H2D of it).  One fence per upload, not one
 * per 16 KiB read: a fence per call cost a third of the copy rate (58.8 vs 91 GB/s,
 * profiles/r03p44_numa_copy_e2e.txt). */
__attribute__((visibility("hidden"))) void uvhttp_ws_amd_copy_fence(void) { _mm_sfence(); }
#else
__attribute__((visibility("hidden"))) void uvhttp_ws_amd_copy_fence(void) {
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
}
#endif

__attribute__((visibility("hidden"))) void uvhttp_ws_amd_copy_stream(void* dst, const void* src,
                                                                     size_t len) {
#if defined(__x86_64__) || defined(__i386__)
    static int have_avx2 = -1;
    if (len < 1024) {
        memcpy(dst, src, len);
        return;
    }
    if (have_avx2 < 0) {
#ifdef UVWS_EXPERIMENTS  /* UVHTTP_WS_COPY_SSE2=1: the SSE2 path, for tests on AVX2 machines */
        const char* f = getenv("UVHTTP_WS_COPY_SSE2");
        have_avx2 = (__builtin_cpu_supports("avx2") && !(f && f[0] == '1')) ? 1 : 0;
#else
        have_avx2 = __builtin_cpu_supports("avx2") ? 1 : 0;
#endif
    }
    if (have_avx2)
        copy_stream_avx2((uint8_t*)dst, (const uint8_t*)src, len);
    else
        copy_stream_sse2((uint8_t*)dst, (const uint8_t*)src, len);
#else
    memcpy(dst, src, len);
#endif
}
