// ws_batcher_group.cpp — the live path over several GPUs (include/uvhttp_ws_amd.h,
// uvhttp_ws_amd_batcher_group_*).
//
// The reference decodes every read of a connection on the loop thread that owns it
// (on_websocket_read, src/uvhttp_connection.c:1098-1175, one loop per server,
// src/uvhttp_connection.c:160-164).  A batcher binds one GPU, and the live shape is bound by
// that GPU's PCIe link, so a server on an 8-GPU node spreads its connections
// over a group of batchers, one per device.  A connection is pinned to one member for its
// lifetime: its reads go to that member's queues only, so each connection still sees exactly
// its own sequence of process_data calls (the member guarantees that), while different
// connections flush over different PCIe links in parallel.  Each member owns its pinned arenas
// (placed next to its GPU) and its streams; the group only routes and fans the loop's flush /
// poll calls out.  Host code only.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <unordered_map>
#include <vector>

#include "uvhttp_ws_amd.h"

// ws_batcher.hip (library-internal): 1 while the batcher holds anything of `conn` (queued
// reads, a failure mark, TLS state)
extern "C" int uvhttp_ws_amd_batcher_holds_conn(const uvhttp_ws_amd_batcher_t* b,
                                                const uvhttp_ws_connection_t* conn);

struct uvhttp_ws_amd_batcher_group {
    std::vector<uvhttp_ws_amd_batcher_t*> members;
    std::vector<int> devices;    // each member's device (-1: host decoder)
    std::vector<uint64_t> live;  // connections pinned to each member
    std::unordered_map<uvhttp_ws_connection_t*, uint32_t> member_of;
    uint32_t next = 0;  // round-robin start among equally loaded members
};

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

// pin a new connection to the member with the fewest live connections (ties: round robin),
// among the device members only when device_only; kNone if there is no such member
uint32_t pin(uvhttp_ws_amd_batcher_group_t* g, uvhttp_ws_connection_t* conn, bool device_only) {
    const uint32_t n = (uint32_t)g->members.size();
    uint32_t best = kNone;
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t m = (g->next + k) % n;
        if (device_only && g->devices[m] < 0) continue;
        if (best == kNone || g->live[m] < g->live[best]) best = m;
    }
    if (best == kNone) return kNone;
    g->next = best + 1;
    g->live[best]++;
    g->member_of.emplace(conn, best);
    return best;
}

// the member a connection belongs to (pinned on its first read, until forget)
uint32_t member_for(uvhttp_ws_amd_batcher_group_t* g, uvhttp_ws_connection_t* conn) {
    auto it = g->member_of.find(conn);
    if (it != g->member_of.end()) return it->second;
    return pin(g, conn, false);
}

// fold a member's flush / poll result into the group's: the first error wins, else the sum
int fold(int acc, int rc) {
    if (acc < 0) return acc;
    return rc < 0 ? rc : acc + rc;
}

}  // namespace

extern "C" {

int uvhttp_ws_amd_batcher_group_create(const uvhttp_ws_amd_batcher_config_t* cfg, const int* devices,
                                       int n_devices, uvhttp_ws_amd_batcher_group_t** out) {
    if (!cfg || !devices || n_devices <= 0 || !out) return UVHTTP_WS_GPU_EINVAL;
    *out = nullptr;
    uvhttp_ws_amd_batcher_group_t* g = new (std::nothrow) uvhttp_ws_amd_batcher_group_t();
    if (!g) return UVHTTP_WS_GPU_ENOMEM;
    for (int k = 0; k < n_devices; ++k) {
        uvhttp_ws_amd_batcher_config_t c = *cfg;
        c.device = devices[k];
        uvhttp_ws_amd_batcher_t* b = nullptr;
        const int rc = uvhttp_ws_amd_batcher_create(&c, &b);
        if (rc != UVHTTP_WS_GPU_OK) {
            uvhttp_ws_amd_batcher_group_free(g);
            return rc;
        }
        g->members.push_back(b);
        g->devices.push_back(devices[k]);
        g->live.push_back(0);
    }
    *out = g;
    return UVHTTP_WS_GPU_OK;
}

void uvhttp_ws_amd_batcher_group_free(uvhttp_ws_amd_batcher_group_t* g) {
    if (!g) return;
    for (uvhttp_ws_amd_batcher_t* b : g->members) uvhttp_ws_amd_batcher_free(b);
    delete g;
}

int uvhttp_ws_amd_batcher_group_size(const uvhttp_ws_amd_batcher_group_t* g) {
    return g ? (int)g->members.size() : 0;
}

uvhttp_ws_amd_batcher_t* uvhttp_ws_amd_batcher_group_batcher(uvhttp_ws_amd_batcher_group_t* g, int i) {
    return g && i >= 0 && i < (int)g->members.size() ? g->members[(size_t)i] : nullptr;
}

int uvhttp_ws_amd_batcher_group_member(uvhttp_ws_amd_batcher_group_t* g, struct uvhttp_ws_connection* conn) {
    if (!g || !conn) return -1;
    auto it = g->member_of.find(conn);  // a query: never pins
    return it == g->member_of.end() ? -1 : (int)it->second;
}

uvhttp_error_t uvhttp_ws_amd_batcher_group_submit_read(uvhttp_ws_amd_batcher_group_t* g,
                                                       struct uvhttp_ws_connection* conn,
                                                       const uint8_t* data, size_t len) {
    if (!g || !conn) return UVHTTP_ERROR_INVALID_PARAM;
    return uvhttp_ws_amd_batcher_submit_read(g->members[member_for(g, conn)], conn, data, len);
}

int uvhttp_ws_amd_batcher_group_set_tls(uvhttp_ws_amd_batcher_group_t* g, struct uvhttp_ws_connection* conn,
                                        const void* tls_key, uint64_t read_seq) {
    if (!g || !conn) return UVHTTP_WS_GPU_EINVAL;
    // TLS records open only on a device member (a host decoder has no AEAD): a new connection
    // is pinned among the device members; one pinned to a host member moves when that member
    // holds nothing of it yet (its reads so far were all delivered)
    auto it = g->member_of.find(conn);
    uint32_t m = it == g->member_of.end() ? kNone : it->second;
    if (m != kNone && g->devices[m] < 0) {
        if (uvhttp_ws_amd_batcher_holds_conn(g->members[m], conn)) return UVHTTP_WS_GPU_ENODEV;
        g->live[m]--;
        g->member_of.erase(it);
        m = kNone;
    }
    if (m == kNone) m = pin(g, conn, true);
    if (m == kNone) return UVHTTP_WS_GPU_ENODEV;
    return uvhttp_ws_amd_batcher_set_tls(g->members[m], conn, tls_key, read_seq);
}

uvhttp_error_t uvhttp_ws_amd_batcher_group_alloc_read(uvhttp_ws_amd_batcher_group_t* g,
                                                      struct uvhttp_ws_connection* conn, size_t suggested,
                                                      uint8_t** buf, size_t* len) {
    if (!g || !conn) return UVHTTP_ERROR_INVALID_PARAM;
    return uvhttp_ws_amd_batcher_alloc_read(g->members[member_for(g, conn)], conn, suggested, buf, len);
}

uvhttp_error_t uvhttp_ws_amd_batcher_group_commit_read(uvhttp_ws_amd_batcher_group_t* g,
                                                       struct uvhttp_ws_connection* conn, size_t nread) {
    if (!g || !conn) return UVHTTP_ERROR_INVALID_PARAM;
    auto it = g->member_of.find(conn);
    if (it == g->member_of.end()) return UVHTTP_ERROR_INVALID_PARAM;  // (no alloc_read before)
    return uvhttp_ws_amd_batcher_commit_read(g->members[it->second], conn, nread);
}

uvhttp_error_t uvhttp_ws_amd_batcher_group_submit_tls_read(uvhttp_ws_amd_batcher_group_t* g,
                                                           struct uvhttp_ws_connection* conn,
                                                           const uint8_t* ciphertext, size_t len) {
    if (!g || !conn) return UVHTTP_ERROR_INVALID_PARAM;
    return uvhttp_ws_amd_batcher_submit_tls_read(g->members[member_for(g, conn)], conn, ciphertext, len);
}

int uvhttp_ws_amd_batcher_group_flush_async(uvhttp_ws_amd_batcher_group_t* g) {
    if (!g) return UVHTTP_WS_GPU_EINVAL;
    int acc = 0;
    for (uvhttp_ws_amd_batcher_t* b : g->members) acc = fold(acc, uvhttp_ws_amd_batcher_flush_async(b));
    return acc < 0 ? acc : 0;
}

int uvhttp_ws_amd_batcher_group_poll(uvhttp_ws_amd_batcher_group_t* g) {
    if (!g) return UVHTTP_WS_GPU_EINVAL;
    int acc = 0;
    for (uvhttp_ws_amd_batcher_t* b : g->members) acc = fold(acc, uvhttp_ws_amd_batcher_poll(b));
    return acc;
}

int uvhttp_ws_amd_batcher_group_flush(uvhttp_ws_amd_batcher_group_t* g) {
    if (!g) return UVHTTP_WS_GPU_EINVAL;
    // every member's queue goes to its device before any is waited for, so the links overlap
    int acc = 0;
    for (uvhttp_ws_amd_batcher_t* b : g->members) acc = fold(acc, uvhttp_ws_amd_batcher_flush_async(b));
    for (uvhttp_ws_amd_batcher_t* b : g->members) acc = fold(acc, uvhttp_ws_amd_batcher_flush(b));
    return acc < 0 ? acc : 0;
}

int uvhttp_ws_amd_batcher_group_in_flight(const uvhttp_ws_amd_batcher_group_t* g) {
    if (!g) return 0;
    for (const uvhttp_ws_amd_batcher_t* b : g->members)
        if (uvhttp_ws_amd_batcher_in_flight(b)) return 1;
    return 0;
}

void uvhttp_ws_amd_batcher_group_forget(uvhttp_ws_amd_batcher_group_t* g, struct uvhttp_ws_connection* conn) {
    if (!g || !conn) return;
    auto it = g->member_of.find(conn);
    if (it == g->member_of.end()) return;
    uvhttp_ws_amd_batcher_forget(g->members[it->second], conn);
    g->live[it->second]--;
    g->member_of.erase(it);
}

int uvhttp_ws_amd_batcher_group_stats(const uvhttp_ws_amd_batcher_group_t* g,
                                      uvhttp_ws_amd_batcher_stats_t* out) {
    if (!g || !out) return UVHTTP_WS_GPU_EINVAL;
    memset(out, 0, sizeof(*out));
    for (const uvhttp_ws_amd_batcher_t* b : g->members) {
        uvhttp_ws_amd_batcher_stats_t s;
        const int rc = uvhttp_ws_amd_batcher_stats(b, &s);
        if (rc) return rc;
        out->flushes += s.flushes;
        out->device_flushes += s.device_flushes;
        out->host_flushes += s.host_flushes;
        out->host_reads += s.host_reads;
        out->device_reads += s.device_reads;
        out->device_frames += s.device_frames;
        out->device_bytes += s.device_bytes;
        out->failures += s.failures;
        out->capacity_flushes += s.capacity_flushes;
        out->device_ms += s.device_ms;
        out->async_flushes += s.async_flushes;
        out->fallback_flushes += s.fallback_flushes;
        out->device_errors += s.device_errors;
        out->direct_reads += s.direct_reads;
        out->blocked_ms += s.blocked_ms;
        out->wait_ms += s.wait_ms;
        out->copy_ms += s.copy_ms;
        out->upload_ms += s.upload_ms;
        out->stage_ms += s.stage_ms;
        out->deliver_ms += s.deliver_ms;
        out->tls_records += s.tls_records;
        out->tls_bytes += s.tls_bytes;
        out->tls_handbacks += s.tls_handbacks;
        out->desc_refetches += s.desc_refetches;
        out->blocked_calls += s.blocked_calls;
        out->zero_copy_reads += s.zero_copy_reads;
        // per-call distributions do not add up: the worst member's
        if (s.max_blocked_ms > out->max_blocked_ms) {
            out->max_blocked_ms = s.max_blocked_ms;
            out->max_blocked_wait_ms = s.max_blocked_wait_ms;
            out->max_blocked_stage_ms = s.max_blocked_stage_ms;
            out->max_blocked_deliver_ms = s.max_blocked_deliver_ms;
        }
        if (s.blocked_p50_ms > out->blocked_p50_ms) out->blocked_p50_ms = s.blocked_p50_ms;
        if (s.blocked_p99_ms > out->blocked_p99_ms) out->blocked_p99_ms = s.blocked_p99_ms;
    }
    return UVHTTP_WS_GPU_OK;
}

void uvhttp_ws_amd_batcher_group_reset_stats(uvhttp_ws_amd_batcher_group_t* g) {
    if (!g) return;
    for (uvhttp_ws_amd_batcher_t* b : g->members) uvhttp_ws_amd_batcher_reset_stats(b);
}

}  // extern "C"
