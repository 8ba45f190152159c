// ws_batcher.hip — the batcher (include/uvhttp_ws_amd.h): live libuv reads of many
// connections, queued by the loop thread and decoded together at flush().
//
// It sits where the reference's on_websocket_read calls uvhttp_ws_process_data once per read
// (src/uvhttp_connection.c:1098-1175).  Per connection the queued reads are exactly the
// process_data calls the reference would have made, so a flush must leave every connection
// as those calls would: the device path stages recv_buffer[0, recv_buffer_pos) + the reads
// per connection with a read table (one entry per call) and runs uvhttp_ws_gpu_decode_reads;
// uvhttp_ws_deliver_stream replays the callbacks and the buffer / fragment state.  Small
// flushes run the host decoder (the product's ws_host.c) read by read.
// With a device, reads are queued straight into a pinned arena in arrival order; a flush
// uploads the arena once and k_batcher_gather lays every connection's bytes out contiguously
// in device memory (the host never re-copies the reads into the decode layout: that staging
// memcpy, 256 MiB per flush on the loop thread, was most of a flush's time).
#include <hip/hip_runtime.h>

#include <chrono>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "uvhttp_ws_amd.h"

namespace {

struct QueuedRead {
    uint64_t off;  // in the arena
    uint64_t len;
};

struct ConnSlot {
    uvhttp_ws_connection_t* conn;
    std::vector<uint32_t> reads;  // indices into reads_, arrival order
    uint64_t bytes;               // queued read bytes
    uint64_t prefix;              // recv_buffer_pos when the slot opened
    bool dropped;                 // forgotten (or failed) during this flush
};

inline uint64_t align16(uint64_t x) { return (x + 15) & ~(uint64_t)15; }

struct GatherSeg {  // arena[src, src + len) -> wire[dst, dst + len)
    uint64_t src, dst, len;
};

// one workgroup per segment (a read, or a connection's recv-buffer prefix); byte copies with
// consecutive lanes on consecutive bytes (source and destination alignments differ per read)
__global__ __launch_bounds__(256) void k_batcher_gather(const uint8_t* __restrict__ arena,
                                                        uint8_t* __restrict__ wire,
                                                        const GatherSeg* __restrict__ seg) {
    const GatherSeg g = seg[blockIdx.x];
    for (uint64_t i = threadIdx.x; i < g.len; i += 256) wire[g.dst + i] = arena[g.src + i];
}

}  // namespace

struct uvhttp_ws_amd_batcher {
    uvhttp_ws_amd_batcher_config_t cfg;
    // queue of the current flush
    std::vector<uint8_t> arena;  // host-only batcher: the queued reads
    uint8_t* h_arena;            // device batcher: the queued reads, pinned (wire_cap bytes),
    uint64_t arena_len;          // then (scratch of each device flush) the recv-buffer prefixes
    uint64_t reads_end;          // end of the queued reads in h_arena
    std::vector<QueuedRead> reads;
    std::vector<ConnSlot> slots;
    std::unordered_map<uvhttp_ws_connection_t*, uint32_t> slot_of;
    uint64_t staged;  // bytes the device layout needs (prefixes + reads + alignment)
    std::unordered_set<uvhttp_ws_connection_t*> failed;
    bool in_flush;
    // device path
    uvhttp_ws_gpu_engine_t* eng;
    hipStream_t stream;
    uint32_t max_frames;
    uint64_t wire_cap;
    uint8_t *h_wire, *d_wire;
    uvhttp_ws_stream_t *h_streams, *d_streams;
    uvhttp_ws_stream_result_t *h_results, *d_results;
    uint64_t *h_read_end, *d_read_end;
    uvhttp_ws_frame_desc_t *h_desc, *d_desc;
    uint8_t* d_arena;
    GatherSeg *h_seg, *d_seg;
    uvhttp_ws_amd_batcher_stats_t st;
};

static uint8_t* arena_data(uvhttp_ws_amd_batcher_t* b) {
    return b->h_arena ? b->h_arena : b->arena.data();
}

// append len bytes to the queue's arena; returns their offset
static uint64_t arena_append(uvhttp_ws_amd_batcher_t* b, const uint8_t* data, size_t len) {
    if (!b->h_arena) {
        const uint64_t off = b->arena.size();
        b->arena.insert(b->arena.end(), data, data + len);
        return off;
    }
    const uint64_t off = b->arena_len;
    if (len) memcpy(b->h_arena + off, data, len);
    b->arena_len += len;
    return off;
}

static void release(uvhttp_ws_amd_batcher_t* b) {
    if (b->eng) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(b->cfg.device);
        if (b->stream) (void)hipStreamSynchronize(b->stream);
        (void)hipHostFree(b->h_wire);
        (void)hipHostFree(b->h_streams);
        (void)hipHostFree(b->h_results);
        (void)hipHostFree(b->h_read_end);
        (void)hipHostFree(b->h_desc);
        (void)hipHostFree(b->h_arena);
        (void)hipHostFree(b->h_seg);
        (void)hipFree(b->d_arena);
        (void)hipFree(b->d_seg);
        (void)hipFree(b->d_wire);
        (void)hipFree(b->d_streams);
        (void)hipFree(b->d_results);
        (void)hipFree(b->d_read_end);
        (void)hipFree(b->d_desc);
        if (b->stream) (void)hipStreamDestroy(b->stream);
        uvhttp_ws_gpu_engine_free(b->eng);
        (void)hipSetDevice(prev);
    }
    delete b;
}

static void clear_queue(uvhttp_ws_amd_batcher_t* b) {
    b->arena.clear();
    b->arena_len = b->reads_end = 0;
    b->reads.clear();
    b->slots.clear();
    b->slot_of.clear();
    b->staged = 0;
}

static void report_failure(uvhttp_ws_amd_batcher_t* b, ConnSlot& s, int rc) {
    b->failed.insert(s.conn);
    b->st.failures++;
    s.dropped = true;
    if (b->cfg.on_failure) b->cfg.on_failure(b->cfg.ctx, s.conn, rc);
}

// the reference's path: process_data per read, until one fails
static void flush_host(uvhttp_ws_amd_batcher_t* b) {
    b->st.host_flushes++;
    for (size_t k = 0; k < b->slots.size(); ++k) {
        ConnSlot& s = b->slots[k];
        for (uint32_t r : s.reads) {
            if (s.dropped) break;
            const QueuedRead& q = b->reads[r];
            const uvhttp_error_t rc =
                uvhttp_ws_process_data(s.conn, arena_data(b) + q.off, (size_t)q.len);
            b->st.host_reads++;
            if (rc != UVHTTP_OK) report_failure(b, s, rc);
        }
    }
}

// stage -> H2D -> decode_reads -> D2H -> deliver.  Returns 1 when the flush must run on
// the host instead (frame capacity), 0 when delivered, < 0 on a device error (nothing
// delivered).
static int flush_device(uvhttp_ws_amd_batcher_t* b) {
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t pos = 0;
    uint32_t nr = 0, nk = 0, nseg = 0;
    std::vector<uint32_t> slot_k(b->slots.size(), UINT32_MAX);
    // prefixes go after the reads; a flush that failed (queue kept) and is retried starts over
    b->arena_len = b->reads_end;
    for (size_t k = 0; k < b->slots.size(); ++k) {
        ConnSlot& s = b->slots[k];
        if (s.dropped) continue;
        uvhttp_ws_connection_t* c = s.conn;
        pos = align16(pos);
        const uint64_t begin = pos;
        if (c->recv_buffer_pos) {  // the bytes recv_buffer already holds come first
            const uint64_t off = arena_append(b, c->recv_buffer, c->recv_buffer_pos);
            b->h_seg[nseg++] = GatherSeg{off, pos, c->recv_buffer_pos};
        }
        pos += c->recv_buffer_pos;
        const uint32_t r0 = nr;
        for (uint32_t r : s.reads) {
            const QueuedRead& q = b->reads[r];
            if (q.len) b->h_seg[nseg++] = GatherSeg{q.off, pos, q.len};
            pos += q.len;
            b->h_read_end[nr++] = pos - begin;
        }
        uvhttp_ws_stream_init(c, begin, pos - begin, &b->h_streams[nk]);
        b->h_streams[nk].first_read = r0;
        b->h_streams[nk].n_reads = nr - r0;
        slot_k[k] = nk++;
    }
    if (!nk) return 0;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != b->cfg.device) (void)hipSetDevice(b->cfg.device);
    // frames this flush can hold: a server connection's frames are >= 6 bytes except a
    // failing last one, so bytes / 6 + connections never overflows for servers; the
    // descriptor buffers grow to that bound on demand
    const uint64_t bound = pos / 6 + nk + 1;
    if (bound > b->max_frames) {
        const uint64_t nf = bound > 2ull * b->max_frames ? bound : 2ull * b->max_frames;
        (void)hipHostFree(b->h_desc);
        (void)hipFree(b->d_desc);
        b->h_desc = nullptr;
        b->d_desc = nullptr;
        b->max_frames = 0;
        if (nf > 0xFFFFFFFFull ||
            hipHostMalloc((void**)&b->h_desc, nf * sizeof(uvhttp_ws_frame_desc_t), hipHostMallocDefault) != hipSuccess ||
            hipMalloc((void**)&b->d_desc, nf * sizeof(uvhttp_ws_frame_desc_t)) != hipSuccess ||
            uvhttp_ws_gpu_engine_reserve(b->eng, (uint32_t)nf, b->wire_cap, 0) != 0) {
            if (prev != b->cfg.device) (void)hipSetDevice(prev);
            return UVHTTP_WS_GPU_ENOMEM;
        }
        b->max_frames = (uint32_t)nf;
    }
    hipStream_t s = b->stream;
    int rc = UVHTTP_WS_GPU_OK;
    hipError_t h = hipMemcpyAsync(b->d_arena, b->h_arena, b->arena_len, hipMemcpyHostToDevice, s);
    if (h == hipSuccess && nseg)
        h = hipMemcpyAsync(b->d_seg, b->h_seg, nseg * sizeof(GatherSeg), hipMemcpyHostToDevice, s);
    if (h == hipSuccess && nseg) {
        hipLaunchKernelGGL(k_batcher_gather, dim3(nseg), dim3(256), 0, s, b->d_arena, b->d_wire,
                           b->d_seg);
        h = hipGetLastError();
    }
    if (h == hipSuccess)
        h = hipMemcpyAsync(b->d_streams, b->h_streams, nk * sizeof(uvhttp_ws_stream_t),
                           hipMemcpyHostToDevice, s);
    if (h == hipSuccess && nr)
        h = hipMemcpyAsync(b->d_read_end, b->h_read_end, nr * sizeof(uint64_t),
                           hipMemcpyHostToDevice, s);
    if (h == hipSuccess)
        rc = uvhttp_ws_gpu_decode_reads(b->eng, b->d_wire, pos, b->d_streams, nk, b->d_read_end,
                                        nr, b->max_frames, b->d_desc, b->d_results, s);
    if (h == hipSuccess && rc == UVHTTP_WS_GPU_OK)
        h = hipMemcpyAsync(b->h_results, b->d_results, nk * sizeof(uvhttp_ws_stream_result_t),
                           hipMemcpyDeviceToHost, s);
    if (h == hipSuccess && rc == UVHTTP_WS_GPU_OK)
        h = hipMemcpyAsync(b->h_wire, b->d_wire, pos, hipMemcpyDeviceToHost, s);
    if (h == hipSuccess && rc == UVHTTP_WS_GPU_OK) rc = uvhttp_ws_gpu_engine_sync(b->eng, s);
    uint64_t frames = 0;
    bool capacity = false;
    if (h == hipSuccess && rc == UVHTTP_WS_GPU_OK) {
        for (uint32_t k = 0; k < nk; ++k) {
            const uvhttp_ws_stream_result_t& r = b->h_results[k];
            if (r.first_status == UVHTTP_WS_FRAME_ERR_CAPACITY) capacity = true;
            const uint64_t e = (uint64_t)r.first_frame + r.n_frames;
            if (r.n_frames && e > frames) frames = e;
        }
        if (!capacity && frames) {
            h = hipMemcpyAsync(b->h_desc, b->d_desc, frames * sizeof(uvhttp_ws_frame_desc_t),
                               hipMemcpyDeviceToHost, s);
            if (h == hipSuccess) h = hipStreamSynchronize(s);
        }
    }
    if (prev != b->cfg.device) (void)hipSetDevice(prev);
    if (h != hipSuccess) return UVHTTP_WS_GPU_ELAUNCH;
    if (rc != UVHTTP_WS_GPU_OK) return rc;
    if (capacity) {
        b->st.capacity_flushes++;
        return 1;
    }
    b->st.device_flushes++;
    b->st.device_bytes += pos;
    b->st.device_frames += frames;
    // deliver, connection by connection (callbacks may forget connections as we go)
    for (size_t k = 0; k < b->slots.size(); ++k) {
        ConnSlot& sl = b->slots[k];
        if (slot_k[k] == UINT32_MAX || sl.dropped) continue;
        const uint32_t j = slot_k[k];
        const uvhttp_error_t dr = uvhttp_ws_deliver_stream(sl.conn, b->h_wire, b->h_desc,
                                                           &b->h_streams[j], &b->h_results[j]);
        b->st.device_reads += b->h_results[j].calls;
        if (dr != UVHTTP_OK) report_failure(b, sl, dr);
    }
    b->st.device_ms +=
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

extern "C" {

void uvhttp_ws_amd_batcher_config_init(uvhttp_ws_amd_batcher_config_t* c) {
    if (!c) return;
    memset(c, 0, sizeof(*c));
    c->device = -1;
    c->min_device_bytes = 256 * 1024;
    c->max_bytes = 32ull << 20;
    c->max_connections = 16384;
    c->max_reads = 1u << 18;
}

int uvhttp_ws_amd_batcher_create(const uvhttp_ws_amd_batcher_config_t* cfg,
                                 uvhttp_ws_amd_batcher_t** out) {
    if (!cfg || !out || !cfg->max_bytes || !cfg->max_connections || !cfg->max_reads)
        return UVHTTP_WS_GPU_EINVAL;
    *out = nullptr;
    uvhttp_ws_amd_batcher_t* b = new (std::nothrow) uvhttp_ws_amd_batcher_t();
    if (!b) return UVHTTP_WS_GPU_ENOMEM;
    b->cfg = *cfg;
    memset(&b->st, 0, sizeof(b->st));
    if (cfg->device < 0) b->arena.reserve(cfg->max_bytes < (64ull << 20) ? cfg->max_bytes : (64ull << 20));
    if (cfg->device >= 0) {
        int rc = uvhttp_ws_gpu_engine_create(cfg->device, &b->eng);
        if (rc) {
            b->eng = nullptr;
            delete b;
            return rc;
        }
        // descriptor capacity starts small and grows with the flushes (flush_device)
        b->wire_cap = cfg->max_bytes + 16ull * cfg->max_connections + 64;
        b->max_frames = 65536;
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(cfg->device);
        const size_t ns = cfg->max_connections;
        bool ok = hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) == hipSuccess &&
                  hipHostMalloc((void**)&b->h_wire, b->wire_cap, hipHostMallocDefault) == hipSuccess &&
                  hipHostMalloc((void**)&b->h_streams, ns * sizeof(uvhttp_ws_stream_t), hipHostMallocDefault) == hipSuccess &&
                  hipHostMalloc((void**)&b->h_results, ns * sizeof(uvhttp_ws_stream_result_t), hipHostMallocDefault) == hipSuccess &&
                  hipHostMalloc((void**)&b->h_read_end, cfg->max_reads * sizeof(uint64_t), hipHostMallocDefault) == hipSuccess &&
                  hipHostMalloc((void**)&b->h_desc, (size_t)b->max_frames * sizeof(uvhttp_ws_frame_desc_t), hipHostMallocDefault) == hipSuccess &&
                  hipMalloc((void**)&b->d_wire, b->wire_cap) == hipSuccess &&
                  hipMalloc((void**)&b->d_streams, ns * sizeof(uvhttp_ws_stream_t)) == hipSuccess &&
                  hipMalloc((void**)&b->d_results, ns * sizeof(uvhttp_ws_stream_result_t)) == hipSuccess &&
                  hipMalloc((void**)&b->d_read_end, cfg->max_reads * sizeof(uint64_t)) == hipSuccess &&
                  hipMalloc((void**)&b->d_desc, (size_t)b->max_frames * sizeof(uvhttp_ws_frame_desc_t)) == hipSuccess &&
                  hipHostMalloc((void**)&b->h_arena, b->wire_cap, hipHostMallocDefault) == hipSuccess &&
                  hipMalloc((void**)&b->d_arena, b->wire_cap) == hipSuccess &&
                  hipHostMalloc((void**)&b->h_seg, ((size_t)cfg->max_reads + ns) * sizeof(GatherSeg), hipHostMallocDefault) == hipSuccess &&
                  hipMalloc((void**)&b->d_seg, ((size_t)cfg->max_reads + ns) * sizeof(GatherSeg)) == hipSuccess;
        if (ok) ok = uvhttp_ws_gpu_engine_reserve(b->eng, b->max_frames, b->wire_cap, 0) == 0;
        (void)hipSetDevice(prev);
        if (!ok) {
            release(b);
            return UVHTTP_WS_GPU_ENOMEM;
        }
    }
    *out = b;
    return UVHTTP_WS_GPU_OK;
}

void uvhttp_ws_amd_batcher_free(uvhttp_ws_amd_batcher_t* b) {
    if (b) release(b);
}

int uvhttp_ws_amd_batcher_flush(uvhttp_ws_amd_batcher_t* b) {
    if (!b) return UVHTTP_WS_GPU_EINVAL;
    if (b->in_flush || b->reads.empty()) return UVHTTP_WS_GPU_OK;
    b->in_flush = true;
    b->st.flushes++;
    int rc = UVHTTP_WS_GPU_OK;
    uint64_t queued = 0;
    for (const ConnSlot& s : b->slots) queued += s.bytes;
    if (b->eng && queued >= b->cfg.min_device_bytes) {
        rc = flush_device(b);
        if (rc == 1) {  // frame capacity (client-side connections only): the host decodes it
            flush_host(b);
            rc = UVHTTP_WS_GPU_OK;
        }
    } else {
        flush_host(b);
    }
    b->in_flush = false;
    if (rc == UVHTTP_WS_GPU_OK) clear_queue(b);
    return rc;
}

uvhttp_error_t uvhttp_ws_amd_batcher_submit_read(uvhttp_ws_amd_batcher_t* b,
                                                 struct uvhttp_ws_connection* conn,
                                                 const uint8_t* data, size_t len) {
    if (!b || !conn || (!data && len)) return UVHTTP_ERROR_INVALID_PARAM;
    if (b->failed.count(conn)) return UVHTTP_ERROR_INVALID_PARAM;
    auto it = b->slot_of.find(conn);
    const bool fresh = it == b->slot_of.end();
    const uint64_t need = (uint64_t)len + (fresh ? align16(conn->recv_buffer_pos) + 16 : 0);
    if (b->staged + need > b->cfg.max_bytes || b->reads.size() + 1 > b->cfg.max_reads ||
        (fresh && b->slots.size() + 1 > b->cfg.max_connections)) {
        if (b->in_flush) return UVHTTP_ERROR_INVALID_PARAM;  // (not from a flush callback)
        if (uvhttp_ws_amd_batcher_flush(b) != UVHTTP_WS_GPU_OK) return UVHTTP_ERROR_INVALID_PARAM;
        if (b->failed.count(conn)) return UVHTTP_ERROR_INVALID_PARAM;
        it = b->slot_of.end();
        if (align16(conn->recv_buffer_pos) + 16 + len > b->cfg.max_bytes) {
            // larger than a whole flush: decode it here, in order (nothing of it is queued)
            const uvhttp_error_t rc = uvhttp_ws_process_data(conn, data, len);
            b->st.host_reads++;
            if (rc != UVHTTP_OK) b->failed.insert(conn);
            return rc;
        }
        return uvhttp_ws_amd_batcher_submit_read(b, conn, data, len);
    }
    uint32_t k;
    if (fresh) {
        k = (uint32_t)b->slots.size();
        b->slots.push_back(ConnSlot{conn, {}, 0, conn->recv_buffer_pos, false});
        b->slot_of[conn] = k;
        b->staged += align16(conn->recv_buffer_pos) + 16;
    } else {
        k = it->second;
    }
    const uint64_t off = arena_append(b, data, len);
    b->reads_end = b->arena_len;
    b->reads.push_back(QueuedRead{off, len});
    b->slots[k].reads.push_back((uint32_t)(b->reads.size() - 1));
    b->slots[k].bytes += len;
    b->staged += len;
    return UVHTTP_OK;
}

void uvhttp_ws_amd_batcher_forget(uvhttp_ws_amd_batcher_t* b, struct uvhttp_ws_connection* conn) {
    if (!b || !conn) return;
    b->failed.erase(conn);
    auto it = b->slot_of.find(conn);
    if (it == b->slot_of.end()) return;
    b->slots[it->second].dropped = true;  // the flush in progress (if any) skips it
    if (!b->in_flush) {                   // (a new connection at this address gets a new slot)
        b->slots[it->second].reads.clear();
        b->slot_of.erase(it);
    }
}

int uvhttp_ws_amd_batcher_stats(const uvhttp_ws_amd_batcher_t* b,
                                uvhttp_ws_amd_batcher_stats_t* out) {
    if (!b || !out) return UVHTTP_WS_GPU_EINVAL;
    *out = b->st;
    return UVHTTP_WS_GPU_OK;
}

}  // extern "C"
