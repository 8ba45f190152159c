/*
 * batcher_e2e.c — end-to-end rate of the live shape (measurement only): libuv-
 * sized reads of many connections start and end in host memory; each flush stages them,
 * copies them to the MI355X, decodes them there (uvhttp_ws_gpu_decode_reads), copies the
 * result back and delivers on_message per connection (uvhttp_ws_amd_batcher_*).  The same
 * reads through the host decoder (--device -1: process_data per read on this core) give the
 * reference-shaped CPU rate.  Prints one JSON line.
 *
 * --async 1: one flush_async per round (the loop's uv_check), so the device decodes round k
 * while the loop takes the reads of round k+1; the last round is flushed synchronously.  The
 * batcher's on_ready (a HIP host callback once a flush's results are in host memory) sets a
 * flag the loop checks between connections' reads — what a uv_async_t does in a libuv loop,
 * whose async handles run in the same poll phase as the read callbacks — and poll() then
 * delivers that flush and starts the one flush_async asked for meanwhile.
 *
 *   batcher_e2e --conns N --frames M --size S --read R --flushes F --device D [--async 1]
 *               [--pin 1: loop thread on the GPU's NUMA node] [--trace 1] [--reads MODEL]
 *
 * --reads: how a socket read reaches the batcher.  "submit" (default): the bytes are already in
 * libuv's buffer (the stream itself) and submit_read copies them into the staging arena — the
 * socket's own copy is not modelled.  "kcopy": the socket read is modelled as a memcpy into a
 * 16 KiB libuv buffer, then submit_read copies again (the reference shape, src/uvhttp_connection.c:
 * 128-158 + 1163).  "zc": alloc_read hands out arena space, the socket read (memcpy) lands there,
 * commit_read queues it — one copy, the socket's own.
 */
#define _GNU_SOURCE
#include <sched.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "uvhttp_ws_amd.h"

static uint64_t g_msgs, g_bytes;
static int on_message(uvhttp_ws_connection_t* c, const char* d, size_t n, int op) {
    (void)c;
    (void)d;
    (void)op;
    g_msgs++;
    g_bytes += n;
    return 0;
}

static atomic_int g_ready;
/* --trace 1: a timeline of the loop's batcher calls and the on_ready wake-ups (stderr) */
static int g_trace;
static double g_t0;
static double now_s(void);
#define TRACE_MAX 4096
static struct { double t; char what; int a, b; } g_ev[TRACE_MAX];
static atomic_int g_nev;
static void trace(char what, int a, int b) {
    if (!g_trace) return;
    const int k = atomic_fetch_add(&g_nev, 1);
    if (k < TRACE_MAX) {
        g_ev[k].t = now_s();
        g_ev[k].what = what;
        g_ev[k].a = a;
        g_ev[k].b = b;
    }
}
static void on_ready(void* ctx) {
    (void)ctx;
    atomic_store(&g_ready, 1);
    trace('R', 0, 0);
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int main(int argc, char** argv) {
    int conns = 1024, frames = 4, flushes = 20, device = 0, async = 0, pin = 0;
    const char* reads_model = "submit";
    double cap_rounds = 1.0;
    size_t size = 65536, rd = 16384;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!strcmp(argv[i], "--conns")) conns = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--frames")) frames = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--size")) size = (size_t)strtoull(argv[i + 1], NULL, 10);
        else if (!strcmp(argv[i], "--read")) rd = (size_t)strtoull(argv[i + 1], NULL, 10);
        else if (!strcmp(argv[i], "--flushes")) flushes = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--device")) device = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--async")) async = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--trace")) g_trace = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--pin")) pin = atoi(argv[i + 1]);
        else if (!strcmp(argv[i], "--cap")) cap_rounds = atof(argv[i + 1]);
        else if (!strcmp(argv[i], "--reads")) reads_model = argv[i + 1];
    }
    /* one connection's stream: M masked BINARY frames of S bytes (every connection sends
     * the same bytes; keys differ per frame) */
    const size_t hs = size < 126 ? 2 : size < 65536 ? 4 : 10;
    const size_t flen = hs + 4 + size, slen = flen * (size_t)frames;
    uint8_t* stream = (uint8_t*)malloc(slen);
    uint64_t s = 12345;
    for (int f = 0; f < frames; ++f) {
        uint8_t* p = stream + (size_t)f * flen;
        p[0] = 0x82;
        if (hs == 2) p[1] = 0x80 | (uint8_t)size;
        else if (hs == 4) { p[1] = 0x80 | 126; p[2] = (uint8_t)(size >> 8); p[3] = (uint8_t)size; }
        else { p[1] = 0x80 | 127; for (int k = 0; k < 8; ++k) p[2 + k] = (uint8_t)(size >> (56 - 8 * k)); }
        for (size_t b = 0; b < 4 + size; ++b) {
            s = s * 6364136223846793005ull + 1442695040888963407ull;
            p[hs + b] = (uint8_t)(s >> 33);
        }
    }
    uvhttp_ws_connection_t** cs = (uvhttp_ws_connection_t**)calloc((size_t)conns, sizeof(*cs));
    for (int c = 0; c < conns; ++c) {
        cs[c] = uvhttp_ws_connection_create(-1, NULL, 1, NULL);
        uvhttp_ws_set_callbacks(cs[c], on_message, NULL, NULL);
    }
    uvhttp_ws_amd_batcher_config_t cfg;
    uvhttp_ws_amd_batcher_config_init(&cfg);
    cfg.device = device;
    cfg.min_device_bytes = 0;
    /* staging capacity in rounds (--cap, default 1): with 1 a read that arrives while the
     * previous flush is still on the device waits for it at the round boundary (backpressure),
     * so every flush carries one round; above 1 the waiting queue absorbs the next round's
     * first reads, and when the loop outruns PCIe the flushes grow, each D2H gets longer and
     * the queue overflows mid-round anyway (1.4: 21.5 vs 24+ GiB/s, r03p45).  decode_reads'
     * frame bound (max_bytes / 6 + connections < 2^26) caps a flush near 384 MiB. */
    const uint64_t round = (uint64_t)conns * (slen + 64);
    cfg.max_bytes = (uint64_t)((double)round * cap_rounds) + (1u << 20);
    cfg.max_connections = (uint32_t)conns;
    cfg.max_reads = (uint32_t)((size_t)(async ? 2 : 1) * conns * (slen / rd + 2));
    if (async) cfg.on_ready = on_ready;
    uvhttp_ws_amd_batcher_t* b = NULL;
    if (uvhttp_ws_amd_batcher_create(&cfg, &b) != 0) {
        fprintf(stderr, "batcher_create failed\n");
        return 1;
    }
    /* --pin 1: the loop thread onto the GPU's NUMA node (uvhttp_ws_amd_batcher_numa_node), as
     * INTEGRATION.md §3 asks of a server */
    const int node = uvhttp_ws_amd_batcher_numa_node(b);
    int pinned = -1;
    if (pin && node >= 0) {
        char path[96], list[4096];
        snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
        FILE* f = fopen(path, "r");
        if (f && fgets(list, sizeof(list), f)) {
            cpu_set_t set;
            CPU_ZERO(&set);
            for (char* p = list; *p && *p != '\n';) {
                char* e;
                long lo = strtol(p, &e, 10), hi = lo;
                if (*e == '-') hi = strtol(e + 1, &e, 10);
                for (long c = lo; c <= hi && c < CPU_SETSIZE; ++c) CPU_SET((int)c, &set);
                p = (*e == ',') ? e + 1 : e;
            }
            if (sched_setaffinity(0, sizeof(set), &set) == 0) pinned = node;
        }
        if (f) fclose(f);
    }
    const int zc = !strcmp(reads_model, "zc"), kcopy = !strcmp(reads_model, "kcopy");
    uint8_t* rbuf = (uint8_t*)malloc(rd);  /* kcopy: libuv's read buffer */
    double t0 = 0, t_submit = 0, t_flush = 0;
    uvhttp_ws_amd_batcher_stats_t st0;
    memset(&st0, 0, sizeof(st0));
    for (int it = -2; it < flushes; ++it) {  /* two warm-up flushes */
        if (it == 0) {
            if (async && uvhttp_ws_amd_batcher_flush(b) != 0) return 3;  /* drain the warm-up */
            g_msgs = g_bytes = 0;
            /* the timed flushes only: every counter, percentile and maximum from here on */
            uvhttp_ws_amd_batcher_reset_stats(b);
            uvhttp_ws_amd_batcher_stats(b, &st0);
            t0 = now_s();
            g_t0 = t0;
        }
        const double ts = now_s();
        uvhttp_ws_amd_batcher_stats_t sx;
        uvhttp_ws_amd_batcher_stats(b, &sx);
        trace('S', it, (int)sx.async_flushes);
        for (int c = 0; c < conns; ++c) {
            for (size_t o = 0; o < slen; o += rd) {
                const size_t len = o + rd <= slen ? rd : slen - o;
                if (zc) {  /* uv_alloc_cb -> the socket read into the arena -> uv_read_cb */
                    for (size_t got = 0; got < len;) {
                        uint8_t* buf = NULL;
                        size_t cap = 0;
                        if (uvhttp_ws_amd_batcher_alloc_read(b, cs[c], len - got, &buf, &cap)) return 2;
                        const size_t k = cap < len - got ? cap : len - got;
                        memcpy(buf, stream + o + got, k);
                        if (uvhttp_ws_amd_batcher_commit_read(b, cs[c], k)) return 2;
                        got += k;
                    }
                } else if (kcopy) {
                    memcpy(rbuf, stream + o, len);
                    if (uvhttp_ws_amd_batcher_submit_read(b, cs[c], rbuf, len)) return 2;
                } else if (uvhttp_ws_amd_batcher_submit_read(b, cs[c], stream + o, len)) {
                    return 2;
                }
            }
            /* the loop's uv_async handle: a finished flush is delivered between reads */
            if (async && atomic_load_explicit(&g_ready, memory_order_relaxed)) {
                atomic_store(&g_ready, 0);
                const int pr = uvhttp_ws_amd_batcher_poll(b);
                uvhttp_ws_amd_batcher_stats(b, &sx);
                trace('P', pr, (int)sx.async_flushes);
                if (pr < 0) return 3;
            }
        }
        const double tf = now_s();
        trace('E', it, 0);
        /* async: the loop's uv_async wake-up (poll) and uv_check (flush_async) */
        if (async) {
            const int pr = uvhttp_ws_amd_batcher_poll(b);
            uvhttp_ws_amd_batcher_stats(b, &sx);
            trace('p', pr, (int)sx.async_flushes);
            if (pr < 0) return 3;
        }
        if ((async ? uvhttp_ws_amd_batcher_flush_async(b) : uvhttp_ws_amd_batcher_flush(b)) != 0) return 3;
        uvhttp_ws_amd_batcher_stats(b, &sx);
        trace('F', (int)sx.device_flushes, (int)sx.async_flushes);
        if (it >= 0) {
            t_submit += tf - ts;
            t_flush += now_s() - tf;
        }
    }
    const double tl = now_s();
    if (async && uvhttp_ws_amd_batcher_flush(b) != 0) return 3;
    t_flush += now_s() - tl;
    const double el = now_s() - t0;
    uvhttp_ws_amd_batcher_stats_t st;
    uvhttp_ws_amd_batcher_stats(b, &st);
    const double payload = (double)size * frames * conns * flushes;
    printf("{\"path\": \"%s\", \"reads\": \"%s\", \"zero_copy_reads\": %llu, \"value\": %.3f, \"unit\": \"GiB/s\", \"conns\": %d, "
           "\"frames_per_conn\": %d, \"payload\": %zu, \"read\": %zu, \"flushes\": %d, "
           "\"ms_per_flush\": %.3f, \"messages_ok\": %d, \"device_flushes\": %llu, "
           "\"device_ms_total\": %.1f, \"async\": %d, \"submit_ms_per_flush\": %.3f, "
           "\"flush_call_ms_per_flush\": %.3f, \"blocked_ms_per_flush\": %.3f, \"gpu_numa_node\": %d, \"pinned_node\": %d, "
           "\"host_flushes\": %llu, \"fallback_flushes\": %llu, \"capacity_flushes\": %llu, \"device_errors\": %llu, "
           "\"max_blocked_ms\": %.3f, \"blocked_calls\": %llu, \"blocked_p50_ms\": %.3f, "
           "\"blocked_p99_ms\": %.3f, \"max_blocked_split_ms\": {\"wait\": %.3f, \"stage\": %.3f, "
           "\"deliver\": %.3f}, \"desc_refetches\": %llu, "
           "\"per_flush_ms\": {\"copy\": %.3f, \"upload\": %.3f, "
           "\"stage\": %.3f, \"wait\": %.3f, \"deliver\": %.3f}}\n",
           device >= 0 ? "device batcher (stage, H2D, decode_reads, D2H, deliver)"
                       : "host decoder (process_data per read, 1 core)",
           reads_model, (unsigned long long)(st.zero_copy_reads - st0.zero_copy_reads), payload / el / (1024.0 * 1024 * 1024), conns, frames, size, rd, flushes,
           el * 1e3 / flushes, g_msgs == (uint64_t)conns * frames * flushes,
           (unsigned long long)(st.device_flushes - st0.device_flushes), st.device_ms - st0.device_ms,
           async, t_submit * 1e3 / flushes, t_flush * 1e3 / flushes,
           (st.blocked_ms - st0.blocked_ms) / flushes, node, pinned,
           (unsigned long long)(st.host_flushes - st0.host_flushes),
           (unsigned long long)(st.fallback_flushes - st0.fallback_flushes),
           (unsigned long long)(st.capacity_flushes - st0.capacity_flushes),
           (unsigned long long)(st.device_errors - st0.device_errors), st.max_blocked_ms,
           (unsigned long long)st.blocked_calls, st.blocked_p50_ms, st.blocked_p99_ms,
           st.max_blocked_wait_ms, st.max_blocked_stage_ms, st.max_blocked_deliver_ms,
           (unsigned long long)st.desc_refetches,
           (st.copy_ms - st0.copy_ms) / flushes, (st.upload_ms - st0.upload_ms) / flushes,
           (st.stage_ms - st0.stage_ms) / flushes, (st.wait_ms - st0.wait_ms) / flushes,
           (st.deliver_ms - st0.deliver_ms) / flushes);
    if (g_trace) {
        /* S = round starts (round, flushes started), E = its reads queued, P / p = poll on
         * on_ready / after the round (result, flushes started), F = flush_async returned
         * (flushes delivered, started), R = on_ready fired (HIP callback thread) */
        const int ne = atomic_load(&g_nev) < TRACE_MAX ? atomic_load(&g_nev) : TRACE_MAX;
        for (int k = 0; k < ne; ++k)
            fprintf(stderr, "%9.3f ms  %c %d %d\n", (g_ev[k].t - g_t0) * 1e3, g_ev[k].what, g_ev[k].a, g_ev[k].b);
    }
    uvhttp_ws_amd_batcher_free(b);
    for (int c = 0; c < conns; ++c) uvhttp_ws_connection_free(cs[c]);
    free(cs);
    free(stream);
    free(rbuf);
    return 0;
}
