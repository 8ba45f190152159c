/*
 * c1_echo.c — BASELINE config C1 as a self-checking program: the reference's
 * examples/05_websocket echo server (websocket_echo_server.c:12-23) on a real libuv loop,
 * with the product's drop-in decode surface (include/uvhttp_ws_amd.h) where the reference
 * links src/uvhttp_websocket.c.
 *
 * Server side, per accepted TCP connection (the reference's L2, src/uvhttp_connection.c):
 *   on_alloc_buffer (:128-158)    every read lands in a 16 KiB read_buffer
 *                                 (include/uvhttp_constants.h:207-208)
 *   on_websocket_read (:1098-1175) plain branch: uvhttp_ws_process_data(ws, buf, nread)
 *                                 (:1163-1164); a failure closes with 1002 (:1166-1174)
 *   on_message -> echo            uvhttp_server_ws_send -> uvhttp_ws_send_text -> an
 *                                 unmasked FIN|TEXT server frame (src/uvhttp_server.c:
 *                                 1057-1089; src/uvhttp_websocket.c:204-285, 509-592)
 * In --batch mode the read callback hands the read to the batcher instead
 * (uvhttp_ws_amd_batcher_submit_read) and a libuv check handle flushes it once per loop
 * iteration — the same callbacks then fire from the flush.
 *
 * Client side (same loop): N clients each send M masked BINARY frames of S payload bytes
 * (keys and payload from a seeded generator), written in C-byte pieces so frames straddle
 * reads, then read their echoes and compare them with the frames they expect.
 *
 * Output: one JSON line (per-client echo digests, read statistics) for tests/test_c1_echo.py.
 * Exit status 0 only if every client received exactly its expected echo stream.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <uv.h>

#include "uvhttp_ws_amd.h"

#define READ_BUFFER_SIZE 16384 /* include/uvhttp_constants.h:207-208 */
#define MAX_CLIENTS 256

typedef struct server_conn server_conn_t;
struct server_conn {
    uv_tcp_t tcp;
    uvhttp_ws_connection_t* ws;
    char read_buffer[READ_BUFFER_SIZE];
    int closing;
};

typedef struct {
    uv_tcp_t tcp;
    uv_connect_t connect;
    int id;
    uint8_t* tx;       /* masked frames to send */
    size_t tx_len, tx_pos;
    uint8_t* expect;   /* echo frames expected back */
    size_t expect_len;
    uint8_t* rx;       /* echo bytes received */
    size_t rx_len;
    uint64_t rx_digest;
    int done;
} client_t;

static uv_loop_t* g_loop;
static uv_tcp_t g_server;
static uv_check_t g_flush_check;
static server_conn_t* g_conns[MAX_CLIENTS];
static int g_n_conns;
static client_t g_clients[MAX_CLIENTS];
static int g_n_clients, g_done_clients;
static uint64_t g_reads, g_read_bytes, g_max_read, g_messages, g_errors;
static int g_batch, g_async;
static uv_async_t g_ready;
#ifndef C1_HOST_ONLY
static uvhttp_ws_amd_batcher_t* g_batcher;
#endif

static uint64_t splitmix64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint64_t fnv1a(uint64_t h, const uint8_t* p, size_t n) {
    for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
    return h;
}

/* frame header bytes per RFC 6455 §5.2 (the reference's build_frame, :204-285) */
static size_t put_header(uint8_t* out, uint8_t b0, int masked, uint64_t n) {
    size_t h = 0;
    out[h++] = b0;
    const uint8_t m = masked ? 0x80 : 0;
    if (n < 126) {
        out[h++] = m | (uint8_t)n;
    } else if (n < 65536) {
        out[h++] = m | 126;
        out[h++] = (uint8_t)(n >> 8);
        out[h++] = (uint8_t)n;
    } else {
        out[h++] = m | 127;
        for (int k = 7; k >= 0; --k) out[h++] = (uint8_t)(n >> (8 * k));
    }
    return h;
}

static server_conn_t* conn_of(const uvhttp_ws_connection_t* ws) {
    for (int i = 0; i < g_n_conns; ++i)
        if (g_conns[i] && g_conns[i]->ws == ws) return g_conns[i];
    return NULL;
}

static void on_write_done(uv_write_t* req, int status) {
    if (status) g_errors++;
    free(req->data);
    free(req);
}

/* uvhttp_server_ws_send(ws_conn, data, len): an unmasked FIN|TEXT frame */
static int ws_message_handler(uvhttp_ws_connection_t* ws, const char* data, size_t len,
                              int opcode) {
    (void)opcode;
    server_conn_t* c = conn_of(ws);
    g_messages++;
    if (!c || c->closing) return 0;
    uint8_t* frame = (uint8_t*)malloc(len + 10);
    const size_t h = put_header(frame, 0x81, 0, len);
    if (len) memcpy(frame + h, data, len);
    uv_write_t* req = (uv_write_t*)malloc(sizeof(*req));
    req->data = frame;
    uv_buf_t b = uv_buf_init((char*)frame, (unsigned)(h + len));
    if (uv_write(req, (uv_stream_t*)&c->tcp, &b, 1, on_write_done) != 0) {
        g_errors++;
        free(frame);
        free(req);
    }
    return 0;
}

static void on_server_close(uv_handle_t* h) {
    server_conn_t* c = (server_conn_t*)h->data;
    for (int i = 0; i < g_n_conns; ++i)
        if (g_conns[i] == c) g_conns[i] = NULL;
    uvhttp_ws_connection_free(c->ws);
    free(c);
}

static void server_close(server_conn_t* c) {
    if (c->closing) return;
    c->closing = 1;
#ifndef C1_HOST_ONLY
    if (g_batcher) uvhttp_ws_amd_batcher_forget(g_batcher, c->ws);
#endif
    uv_close((uv_handle_t*)&c->tcp, on_server_close);
}

/* on_alloc_buffer: every read goes to the connection's 16 KiB read buffer */
static void on_alloc(uv_handle_t* h, size_t suggested, uv_buf_t* buf) {
    (void)suggested;
    server_conn_t* c = (server_conn_t*)h->data;
    *buf = uv_buf_init(c->read_buffer, READ_BUFFER_SIZE);
}

/* on_websocket_read, plain branch (src/uvhttp_connection.c:1098-1175) */
static void on_server_read(uv_stream_t* s, ssize_t nread, const uv_buf_t* buf) {
    server_conn_t* c = (server_conn_t*)s->data;
    if (nread < 0) {
        server_close(c);
        return;
    }
    if (nread == 0) return;
    g_reads++;
    g_read_bytes += (uint64_t)nread;
    if ((uint64_t)nread > g_max_read) g_max_read = (uint64_t)nread;
    int result;
#ifndef C1_HOST_ONLY
    if (g_batch)
        result = uvhttp_ws_amd_batcher_submit_read(g_batcher, c->ws, (const uint8_t*)buf->base,
                                                   (size_t)nread);
    else
#endif
        result = uvhttp_ws_process_data(c->ws, (const uint8_t*)buf->base, (size_t)nread);
    if (result != 0) {
        g_errors++;
        server_close(c);
    }
}

#ifndef C1_HOST_ONLY
/* batcher results: a connection whose deferred reads failed is closed like :1166-1174 */
static void on_batch_failure(void* ctx, uvhttp_ws_connection_t* ws, int rc) {
    (void)ctx;
    (void)rc;
    server_conn_t* c = conn_of(ws);
    g_errors++;
    if (c) server_close(c);
}

static void on_flush_check(uv_check_t* h) {
    (void)h;
    if (!g_batcher) return;
    if ((g_async ? uvhttp_ws_amd_batcher_flush_async(g_batcher)
                 : uvhttp_ws_amd_batcher_flush(g_batcher)) != 0)
        g_errors++;
}

/* --async 1: a device queue's results are back (HIP runtime thread): wake the loop */
static void on_batch_ready(void* ctx) {
    (void)ctx;
    uv_async_send(&g_ready);
}
/* ... and deliver them on the loop thread */
static void on_ready_async(uv_async_t* h) {
    (void)h;
    if (g_batcher && uvhttp_ws_amd_batcher_poll(g_batcher) < 0) g_errors++;
}
#endif

static void on_connection(uv_stream_t* server, int status) {
    if (status < 0) return;
    server_conn_t* c = (server_conn_t*)calloc(1, sizeof(*c));
    uv_tcp_init(g_loop, &c->tcp);
    c->tcp.data = c;
    if (uv_accept(server, (uv_stream_t*)&c->tcp) != 0) {
        free(c);
        return;
    }
    /* uvhttp_connection_handle_websocket_handshake (:1343-1368): a server-side decoder
     * with the server config, callbacks installed, then reads switched to it */
    c->ws = uvhttp_ws_connection_create(-1, NULL, 1, NULL);
    uvhttp_ws_set_callbacks(c->ws, ws_message_handler, NULL, NULL);
    g_conns[g_n_conns++] = c;
    uv_read_start((uv_stream_t*)&c->tcp, on_alloc, on_server_read);
}

/* ---- clients ---------------------------------------------------------------------------- */

static void client_alloc(uv_handle_t* h, size_t suggested, uv_buf_t* buf) {
    (void)h;
    *buf = uv_buf_init((char*)malloc(suggested), (unsigned)suggested);
}

static void on_client_closed(uv_handle_t* h) {
    (void)h;
    if (++g_done_clients == g_n_clients) {
        uv_close((uv_handle_t*)&g_server, NULL);
        if (g_batch) uv_close((uv_handle_t*)&g_flush_check, NULL);
        if (g_async) uv_close((uv_handle_t*)&g_ready, NULL);
        for (int i = 0; i < g_n_conns; ++i)
            if (g_conns[i]) server_close(g_conns[i]);
    }
}

static void on_client_read(uv_stream_t* s, ssize_t nread, const uv_buf_t* buf) {
    client_t* cl = (client_t*)s->data;
    if (nread > 0) {
        if (cl->rx_len + (size_t)nread <= cl->expect_len)
            memcpy(cl->rx + cl->rx_len, buf->base, (size_t)nread);
        cl->rx_len += (size_t)nread;
    }
    free(buf->base);
    if ((nread < 0 || cl->rx_len >= cl->expect_len) && !cl->done) {
        cl->done = 1;
        uv_close((uv_handle_t*)&cl->tcp, on_client_closed);
    }
}

static size_t g_chunk = 1000;

static void client_write_next(client_t* cl);

static void on_client_write(uv_write_t* req, int status) {
    client_t* cl = (client_t*)req->data;
    free(req);
    if (status) {
        g_errors++;
        return;
    }
    client_write_next(cl);
}

static void client_write_next(client_t* cl) {
    if (cl->tx_pos >= cl->tx_len) return;
    size_t n = cl->tx_len - cl->tx_pos;
    if (n > g_chunk) n = g_chunk;
    uv_write_t* req = (uv_write_t*)malloc(sizeof(*req));
    req->data = cl;
    uv_buf_t b = uv_buf_init((char*)cl->tx + cl->tx_pos, (unsigned)n);
    cl->tx_pos += n;
    uv_write(req, (uv_stream_t*)&cl->tcp, &b, 1, on_client_write);
}

static void on_client_connect(uv_connect_t* req, int status) {
    client_t* cl = (client_t*)req->data;
    if (status) {
        g_errors++;
        return;
    }
    uv_read_start((uv_stream_t*)&cl->tcp, client_alloc, on_client_read);
    client_write_next(cl);
}

/* M masked BINARY frames of S bytes: what the client sends and the echo it expects */
static void client_make(client_t* cl, int id, int frames, size_t size, uint64_t seed) {
    uint64_t s = seed * 1000003u + (uint64_t)id;
    cl->id = id;
    cl->tx = (uint8_t*)malloc((size + 14) * (size_t)frames + 1);
    cl->expect = (uint8_t*)malloc((size + 10) * (size_t)frames + 1);
    cl->tx_len = cl->expect_len = 0;
    for (int f = 0; f < frames; ++f) {
        const uint64_t kw = splitmix64(&s);
        const uint8_t key[4] = {(uint8_t)kw, (uint8_t)(kw >> 8), (uint8_t)(kw >> 16),
                                (uint8_t)(kw >> 24)};
        uint8_t* fr = cl->tx + cl->tx_len;
        size_t h = put_header(fr, 0x82, 1, size);
        memcpy(fr + h, key, 4);
        h += 4;
        uint8_t* ex = cl->expect + cl->expect_len;
        const size_t eh = put_header(ex, 0x81, 0, size);
        for (size_t b = 0; b < size; ++b) {
            const uint8_t p = (uint8_t)splitmix64(&s);
            fr[h + b] = p ^ key[b & 3];
            ex[eh + b] = p;
        }
        cl->tx_len += h + size;
        cl->expect_len += eh + size;
    }
    cl->rx = (uint8_t*)malloc(cl->expect_len + 1);
}

int main(int argc, char** argv) {
    int clients = 1, frames = 1, device = 0;
    size_t size = 1024;
    uint64_t seed = 1, threshold = 0;
    const char* dump = NULL;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--clients")) clients = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--frames")) frames = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--size")) size = (size_t)strtoull(argv[i + 1], NULL, 10);
        else if (!strcmp(argv[i], "--chunk")) g_chunk = (size_t)strtoull(argv[i + 1], NULL, 10);
        else if (!strcmp(argv[i], "--seed")) seed = strtoull(argv[i + 1], NULL, 10);
        else if (!strcmp(argv[i], "--batch")) g_batch = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--async")) g_async = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--device")) device = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--threshold")) threshold = strtoull(argv[i + 1], NULL, 10);
        else if (!strcmp(argv[i], "--dump")) dump = argv[i + 1];
    }
    if (clients < 1 || clients > MAX_CLIENTS || frames < 0 || g_chunk == 0) return 2;
    g_loop = uv_default_loop();
#ifdef C1_HOST_ONLY
    (void)device;
    (void)threshold;
    if (g_batch || g_async) return 2;
#else
    if (g_async && !g_batch) return 2;
    if (g_batch) {
        uvhttp_ws_amd_batcher_config_t bc;
        uvhttp_ws_amd_batcher_config_init(&bc);
        bc.device = device;
        bc.min_device_bytes = threshold;
        bc.on_failure = on_batch_failure;
        if (g_async) {
            uv_async_init(g_loop, &g_ready, on_ready_async);
            bc.on_ready = on_batch_ready;
        }
        if (uvhttp_ws_amd_batcher_create(&bc, &g_batcher) != 0) {
            fprintf(stderr, "batcher_create failed\n");
            return 3;
        }
        uv_check_init(g_loop, &g_flush_check);
        uv_check_start(&g_flush_check, on_flush_check);
    }
#endif
    uv_tcp_init(g_loop, &g_server);
    struct sockaddr_in addr;
    uv_ip4_addr("127.0.0.1", 0, &addr);
    if (uv_tcp_bind(&g_server, (const struct sockaddr*)&addr, 0) ||
        uv_listen((uv_stream_t*)&g_server, 128, on_connection))
        return 4;
    int namelen = sizeof(addr);
    uv_tcp_getsockname(&g_server, (struct sockaddr*)&addr, &namelen);
    g_n_clients = clients;
    for (int i = 0; i < clients; ++i) {
        client_t* cl = &g_clients[i];
        client_make(cl, i, frames, size, seed);
        uv_tcp_init(g_loop, &cl->tcp);
        cl->tcp.data = cl;
        cl->connect.data = cl;
        uv_tcp_connect(&cl->connect, &cl->tcp, (const struct sockaddr*)&addr, on_client_connect);
    }
    uv_run(g_loop, UV_RUN_DEFAULT);
    int ok = 1;
    printf("{\"clients\": [");
    for (int i = 0; i < clients; ++i) {
        client_t* cl = &g_clients[i];
        const int match = cl->rx_len == cl->expect_len && !memcmp(cl->rx, cl->expect, cl->expect_len);
        ok &= match;
        printf("%s{\"id\": %d, \"sent\": %zu, \"echoed\": %zu, \"expected\": %zu, \"match\": %d, "
               "\"echo_fnv\": \"%016llx\"}",
               i ? ", " : "", cl->id, cl->tx_len, cl->rx_len, cl->expect_len, match,
               (unsigned long long)fnv1a(1469598103934665603ull, cl->rx,
                                         cl->rx_len < cl->expect_len ? cl->rx_len : cl->expect_len));
    }
    struct {
        unsigned long long device_flushes, host_reads, device_reads, device_frames;
    } st = {0, 0, 0, 0};
#ifndef C1_HOST_ONLY
    if (g_batcher) {
        uvhttp_ws_amd_batcher_stats_t bs;
        uvhttp_ws_amd_batcher_stats(g_batcher, &bs);
        st.device_flushes = bs.device_flushes;
        st.host_reads = bs.host_reads;
        st.device_reads = bs.device_reads;
        st.device_frames = bs.device_frames;
    }
#endif
    printf("], \"reads\": %llu, \"read_bytes\": %llu, \"max_read\": %llu, \"messages\": %llu, "
           "\"errors\": %llu, \"batch\": %d, \"device_flushes\": %llu, \"host_reads\": %llu, "
           "\"device_reads\": %llu, \"device_frames\": %llu}\n",
           (unsigned long long)g_reads, (unsigned long long)g_read_bytes,
           (unsigned long long)g_max_read, (unsigned long long)g_messages,
           (unsigned long long)g_errors, g_batch, st.device_flushes, st.host_reads,
           st.device_reads, st.device_frames);
#ifndef C1_HOST_ONLY
    if (g_batcher) uvhttp_ws_amd_batcher_free(g_batcher);
#endif
    /* --dump PREFIX: each client's sent bytes and received echo, for the oracle check */
    for (int i = 0; dump && i < clients; ++i) {
        char path[4096];
        snprintf(path, sizeof(path), "%s.tx.%d", dump, i);
        FILE* f = fopen(path, "wb");
        if (f) {
            fwrite(g_clients[i].tx, 1, g_clients[i].tx_len, f);
            fclose(f);
        }
        snprintf(path, sizeof(path), "%s.rx.%d", dump, i);
        f = fopen(path, "wb");
        if (f) {
            const size_t n = g_clients[i].rx_len < g_clients[i].expect_len ? g_clients[i].rx_len
                                                                            : g_clients[i].expect_len;
            fwrite(g_clients[i].rx, 1, n, f);
            fclose(f);
        }
    }
    uv_loop_close(g_loop);
    for (int i = 0; i < clients; ++i) {
        free(g_clients[i].tx);
        free(g_clients[i].expect);
        free(g_clients[i].rx);
    }
    return ok && !g_errors ? 0 : 1;
}
