// ws_batcher.hip — the batcher (include/uvhttp_ws_amd.h): live libuv reads of many
// connections, queued by the loop thread and decoded together.
//
// It sits where the reference's on_websocket_read calls uvhttp_ws_process_data once per read
// (src/uvhttp_connection.c:1098-1175).  Per connection the queued reads are exactly the
// process_data calls the reference would have made, so a flush must leave every connection
// as those calls would: the device path stages recv_buffer[0, recv_buffer_pos) + the reads
// per connection with a read table (one entry per call) and runs uvhttp_ws_gpu_decode_reads;
// uvhttp_ws_deliver_stream replays the callbacks and the buffer / fragment state.  Small
// flushes run the host decoder (the product's ws_host.c) read by read.
//
// Two queues, so the loop thread never waits for PCIe or the GPU while it has reads to take:
//   * the accumulating queue takes submit_read's bytes into its pinned arena; once the queue
//     is large enough for the device, the arena streams to HBM in 8 MiB pieces on the upload
//     stream while reads keep arriving (the H2D overlaps the loop's own work);
//   * flush_async hands the accumulating queue to the device (the recv-buffer prefixes and
//     read tables are staged then, from the connections' state at that moment, so they see
//     every earlier flush) and switches submit_read to the other queue: gather, decode and
//     D2H run on the compute stream while the loop returns to libuv;
//   * poll (or the next flush) delivers the finished queue: callbacks, recv-buffer and
//     fragment state per connection, exactly what process_data per read would have left.
// A connection's reads in the accumulating queue are staged only after the in-flight queue
// has been delivered (flush_async completes it first), so its state is always current.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unordered_map>
#include <unordered_set>
#include <memory>
#include <utility>
#include <vector>

#include "uvhttp_tls_amd.h"
#include "uvhttp_ws_amd.h"

extern "C" void uvhttp_ws_amd_copy_stream(void* dst, const void* src, size_t len);  // ws_host.c
extern "C" void uvhttp_ws_amd_copy_fence(void);  // ws_host.c: streaming stores -> visible to DMA

// TLS connections (uvhttp_ws_amd_batcher_set_tls): a queue's TLS connections are laid out
// after the plain ones in the device wire as ciphertext (the previous flushes' unconsumed
// bytes, then the new reads); the flush opens their records (uvhttp_tls_gpu_open_records),
// turns every delivered record into one process_data call (uvhttp_tls_gpu_ws_streams: the
// chunks mbedtls_ssl_read returns, src/uvhttp_connection.c:1128-1158) and decodes the
// plaintext with decode_reads, next to the plain connections' decode.

namespace {

constexpr uint32_t kMaxFramesPerFlush = 1u << 26;  // decode_reads' frame limit (ws_gpu.hip)
constexpr uint64_t kUploadPiece = 8ull << 20;        // arena bytes per early H2D
constexpr uint32_t kMinFrames = 65536;              // initial descriptor capacity per queue
// room a TLS connection's carry may need when the queue is staged: at most one incomplete
// record (5-byte header + 2^14 content + 256 bytes of AEAD expansion, RFC 8446 §5.2)
constexpr uint64_t kTlsCarryMax = 5 + 16384 + 256 + 16;

struct QueuedRead {
    uint64_t off;  // in the queue's arena
    uint64_t len;
};

struct ConnSlot {
    uvhttp_ws_connection_t* conn;
    std::vector<uint32_t> reads;  // indices into Queue::reads, arrival order
    uint64_t bytes;               // queued read bytes
    bool dropped;                 // forgotten, or failed in an earlier queue
    bool tls;                     // ciphertext reads of a TLS connection
};

// a TLS connection's read side: its key, the sequence number of its next record and the
// ciphertext a flush did not consume (an incomplete record: it waits for more bytes, as in
// mbedtls's input buffer)
struct TlsConn {
    uvhttp_tls_key_t key;
    uint64_t seq;
    std::vector<uint8_t> carry;
};

inline uint64_t align16(uint64_t x) { return (x + 15) & ~(uint64_t)15; }

// the host-only arena grows by resize() without zero-filling: alloc_read hands the new bytes
// to the socket read, which writes them
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) {}
    template <class U>
    void construct(U* p) { ::new ((void*)p) U; }
    template <class U, class... A>
    void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
};

struct GatherSeg {  // arena[src, src + len) -> wire[dst, dst + len)
    uint64_t src, dst, len;
};

// one workgroup per segment (a read, or a connection's recv-buffer prefix): 16-byte windows,
// consecutive lanes on consecutive windows (source and destination alignments differ per read,
// so the windows are unaligned loads and stores — gfx950 serves them in one access), bytes for
// the segment's last partial window.  Byte-wise copies took 0.30-0.34 ms per 256 MiB flush
// (profiles/r03_e2e_async_timeline.txt).
__global__ __launch_bounds__(256) void k_batcher_gather(const uint8_t* __restrict__ arena,
                                                        uint8_t* __restrict__ wire,
                                                        const GatherSeg* __restrict__ seg) {
    const GatherSeg g = seg[blockIdx.x];
    const uint8_t* src = arena + g.src;
    uint8_t* dst = wire + g.dst;
    const uint64_t full = g.len & ~(uint64_t)15;
    for (uint64_t i = (uint64_t)threadIdx.x * 16; i < full; i += 256 * 16) {
        uint32_t w[4];
        __builtin_memcpy(w, src + i, 16);
        __builtin_memcpy(dst + i, w, 16);
    }
    for (uint64_t i = full + threadIdx.x; i < g.len; i += 256) dst[i] = src[i];
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

// One queue: the reads of one flush, and (device batcher) the buffers its decode uses.
struct BatchQueue {
    std::vector<uint8_t, NoInitAlloc<uint8_t>> arena;  // host-only batcher: the queued reads
    uint64_t gen = 0;            // bumped whenever the queue is cleared (zero-copy reads check it)
    uint8_t* h_arena = nullptr;  // device batcher: the reads, pinned (wire_cap bytes), then
    uint64_t arena_len = 0;      // the recv-buffer prefixes staged at flush time
    uint64_t uploaded = 0;       // h_arena[0, uploaded) is already on its way to d_arena
    std::vector<QueuedRead> reads;
    std::vector<ConnSlot> slots;
    std::unordered_map<uvhttp_ws_connection_t*, uint32_t> slot_of;
    uint64_t staged = 0;  // estimate of the device layout (reads + prefixes + alignment)
    uint64_t bytes = 0;   // queued read bytes
    // device buffers
    uint8_t *d_arena = nullptr, *h_wire = nullptr, *d_wire = nullptr;
    uvhttp_ws_stream_t *h_streams = nullptr, *d_streams = nullptr;
    uvhttp_ws_stream_result_t *h_results = nullptr, *d_results = nullptr;
    uint64_t *h_read_end = nullptr, *d_read_end = nullptr;
    uvhttp_ws_frame_desc_t *h_desc = nullptr, *d_desc = nullptr;
    GatherSeg *h_seg = nullptr, *d_seg = nullptr;
    uint32_t max_frames = 0;
    uint64_t desc_copied = 0, wdesc_copied = 0;  // descriptors the launch copies back
    hipEvent_t up_ev = nullptr, done_ev = nullptr;
    // TLS connections (allocated with the first set_tls)
    bool tls_ready = false;
    uint32_t n_tls_slots = 0;       // TLS slots queued
    uint8_t *d_plain = nullptr, *h_plain = nullptr;  // opened plaintext (wire_cap bytes)
    uvhttp_tls_key_t *h_keys = nullptr, *d_keys = nullptr;
    uvhttp_tls_stream_t *h_tst = nullptr, *d_tst = nullptr;
    uvhttp_tls_result_t *h_tres = nullptr, *d_tres = nullptr;
    uvhttp_tls_record_t* d_trecs = nullptr;
    uint64_t* d_wread_end = nullptr;
    uint32_t trec_cap = 0;
    uvhttp_ws_stream_t *h_wst = nullptr, *d_wst = nullptr;
    uvhttp_ws_stream_result_t *h_wres = nullptr, *d_wres = nullptr;
    uvhttp_ws_frame_desc_t *h_wdesc = nullptr, *d_wdesc = nullptr;
    uint32_t wdesc_cap = 0;
    uint64_t *h_poff = nullptr, *d_poff = nullptr;
    // the flush in flight
    bool in_flight = false;
    int launch_rc = 0;
    uint32_t nk = 0;               // plain connections staged
    uint64_t pos = 0;              // wire bytes staged
    uint32_t nt = 0;               // TLS connections staged
    uint32_t nr = 0;               // plain reads staged
    uint64_t max_records = 0;      // TLS record capacity of the launch
    uint64_t tls_base = 0, tls_bytes = 0, plain_cap = 0;
    std::vector<uint32_t> slot_k;  // slot -> stream index (UINT32_MAX: not staged)
    std::vector<uint64_t> carry_off;  // TLS slot -> its staged carry in h_arena (offset, len)
    std::vector<uint64_t> carry_len;
    std::chrono::steady_clock::time_point t_submit;
};

struct uvhttp_ws_amd_batcher {
    uvhttp_ws_amd_batcher_config_t cfg;
    BatchQueue q[2];
    int cur = 0;  // the accumulating queue; q[cur ^ 1] is idle or in flight
    std::unordered_set<uvhttp_ws_connection_t*> failed;
    int delivering = 0;  // callbacks of a delivery are running (no nested flushes)
    bool want_flush = false;  // flush_async asked while a queue was in flight: poll starts it
    // device path
    uvhttp_ws_gpu_engine_t* eng = nullptr;
    hipStream_t up = nullptr;  // H2D of the arenas
    hipStream_t cs = nullptr;  // gather, decode, D2H
    uint64_t wire_cap = 0;
#ifdef UVWS_TEST_HOOKS
    // fault injection, compiled only into the test build (libuvhttp_ws_amd_testhooks.so):
    // UVHTTP_WS_BATCHER_FAIL_EVERY=k makes every k-th device launch report ELAUNCH before
    // enqueueing anything
    uint32_t fail_every = 0;
    uint32_t launches = 0;
#endif
    uvhttp_tls_gpu_engine_t* teng = nullptr;  // record open (first set_tls)
    std::unordered_map<uvhttp_ws_connection_t*, TlsConn> tls;
    // descriptors a launch copies back: a high-water mark of recent flushes' frame counts (the
    // count itself is only known on the device); a flush with more fetches the rest after it
    // completes (desc_refetches)
    uint64_t desc_hint = 4096, wdesc_hint = 4096;
    uvhttp_ws_amd_batcher_stats_t st;
    // the zero-copy read handed out by alloc_read and not yet committed: space at arena offset
    // `off` of queue `qi` (generation `gen`), `cap` bytes, for `conn`
    struct {
        uvhttp_ws_connection_t* conn = nullptr;
        int qi = 0;
        uint64_t gen = 0, off = 0, cap = 0;
        bool tls = false;
        bool direct = false;  // the space is `direct` below: decoded at commit (submit_read's
                              // path for a read no flush can hold)
    } pend;
    std::vector<uint8_t, NoInitAlloc<uint8_t>> direct;
    std::vector<float> blocked;  // ms of each blocked call (ring of the last kBlockedKeep)
    uint64_t blocked_n = 0;
};

namespace {

uint8_t* arena_data(uvhttp_ws_amd_batcher_t* b, BatchQueue& q) {
    return b->eng ? q.h_arena : q.arena.data();
}

void free_queue(BatchQueue& q) {
    (void)hipHostFree(q.h_arena);
    (void)hipHostFree(q.h_wire);
    (void)hipHostFree(q.h_streams);
    (void)hipHostFree(q.h_results);
    (void)hipHostFree(q.h_read_end);
    (void)hipHostFree(q.h_desc);
    (void)hipHostFree(q.h_seg);
    (void)hipFree(q.d_arena);
    (void)hipFree(q.d_wire);
    (void)hipFree(q.d_streams);
    (void)hipFree(q.d_results);
    (void)hipFree(q.d_read_end);
    (void)hipFree(q.d_desc);
    (void)hipFree(q.d_seg);
    if (q.up_ev) (void)hipEventDestroy(q.up_ev);
    if (q.done_ev) (void)hipEventDestroy(q.done_ev);
    (void)hipHostFree(q.h_plain);
    (void)hipHostFree(q.h_keys);
    (void)hipHostFree(q.h_tst);
    (void)hipHostFree(q.h_tres);
    (void)hipHostFree(q.h_wst);
    (void)hipHostFree(q.h_wres);
    (void)hipHostFree(q.h_wdesc);
    (void)hipHostFree(q.h_poff);
    (void)hipFree(q.d_plain);
    (void)hipFree(q.d_keys);
    (void)hipFree(q.d_tst);
    (void)hipFree(q.d_tres);
    (void)hipFree(q.d_trecs);
    (void)hipFree(q.d_wread_end);
    (void)hipFree(q.d_wst);
    (void)hipFree(q.d_wres);
    (void)hipFree(q.d_wdesc);
    (void)hipFree(q.d_poff);
}

// the TLS side of a queue: per-connection tables (max_connections), the plaintext buffer;
// records and their descriptors grow per flush (grow_tls)
bool alloc_tls(uvhttp_ws_amd_batcher_t* b, BatchQueue& q) {
    if (q.tls_ready) return true;
    const size_t ns = b->cfg.max_connections;
    q.tls_ready =
        hipHostMalloc((void**)&q.h_plain, b->wire_cap, hipHostMallocDefault) == hipSuccess &&
        hipHostMalloc((void**)&q.h_keys, ns * sizeof(uvhttp_tls_key_t), hipHostMallocDefault) == hipSuccess &&
        hipHostMalloc((void**)&q.h_tst, ns * sizeof(uvhttp_tls_stream_t), hipHostMallocDefault) == hipSuccess &&
        hipHostMalloc((void**)&q.h_tres, ns * sizeof(uvhttp_tls_result_t), hipHostMallocDefault) == hipSuccess &&
        hipHostMalloc((void**)&q.h_wst, ns * sizeof(uvhttp_ws_stream_t), hipHostMallocDefault) == hipSuccess &&
        hipHostMalloc((void**)&q.h_wres, ns * sizeof(uvhttp_ws_stream_result_t), hipHostMallocDefault) == hipSuccess &&
        hipHostMalloc((void**)&q.h_poff, ns * sizeof(uint64_t), hipHostMallocDefault) == hipSuccess &&
        hipMalloc((void**)&q.d_plain, b->wire_cap) == hipSuccess &&
        hipMalloc((void**)&q.d_keys, ns * sizeof(uvhttp_tls_key_t)) == hipSuccess &&
        hipMalloc((void**)&q.d_tst, ns * sizeof(uvhttp_tls_stream_t)) == hipSuccess &&
        hipMalloc((void**)&q.d_tres, ns * sizeof(uvhttp_tls_result_t)) == hipSuccess &&
        hipMalloc((void**)&q.d_wst, ns * sizeof(uvhttp_ws_stream_t)) == hipSuccess &&
        hipMalloc((void**)&q.d_wres, ns * sizeof(uvhttp_ws_stream_result_t)) == hipSuccess &&
        hipMalloc((void**)&q.d_poff, ns * sizeof(uint64_t)) == hipSuccess;
    return q.tls_ready;
}

// records (and the read table, one entry per record) for nr records, plaintext frame
// descriptors for nf frames
int grow_tls(uvhttp_ws_amd_batcher_t* b, BatchQueue& q, uint64_t nr, uint64_t nf) {
    if (nr > q.trec_cap) {
        uint64_t want = 2ull * q.trec_cap > nr ? 2ull * q.trec_cap : nr;
        if (want > (1u << 28)) want = 1u << 28;
        if (want < nr) return UVHTTP_WS_GPU_ENOMEM;
        (void)hipFree(q.d_trecs);
        (void)hipFree(q.d_wread_end);
        q.d_trecs = nullptr;
        q.d_wread_end = nullptr;
        q.trec_cap = 0;
        if (hipMalloc((void**)&q.d_trecs, want * sizeof(uvhttp_tls_record_t)) != hipSuccess ||
            hipMalloc((void**)&q.d_wread_end, want * sizeof(uint64_t)) != hipSuccess)
            return UVHTTP_WS_GPU_ENOMEM;
        q.trec_cap = (uint32_t)want;
    }
    if (nf > q.wdesc_cap) {
        uint64_t want = 2ull * q.wdesc_cap > nf ? 2ull * q.wdesc_cap : nf;
        if (want > kMaxFramesPerFlush) want = kMaxFramesPerFlush;
        if (want < nf) return UVHTTP_WS_GPU_ENOMEM;
        (void)hipHostFree(q.h_wdesc);
        (void)hipFree(q.d_wdesc);
        q.h_wdesc = nullptr;
        q.d_wdesc = nullptr;
        q.wdesc_cap = 0;
        if (hipHostMalloc((void**)&q.h_wdesc, want * sizeof(uvhttp_ws_frame_desc_t), hipHostMallocDefault) != hipSuccess ||
            hipMalloc((void**)&q.d_wdesc, want * sizeof(uvhttp_ws_frame_desc_t)) != hipSuccess ||
            uvhttp_ws_gpu_engine_reserve(b->eng, (uint32_t)want, b->wire_cap, 0) != 0)
            return UVHTTP_WS_GPU_ENOMEM;
        q.wdesc_cap = (uint32_t)want;
    }
    return 0;
}

bool alloc_queue(uvhttp_ws_amd_batcher_t* b, BatchQueue& q) {
    const size_t ns = b->cfg.max_connections, nr = b->cfg.max_reads;
    q.max_frames = kMinFrames;
    return hipHostMalloc((void**)&q.h_arena, b->wire_cap, hipHostMallocDefault) == hipSuccess &&
           hipHostMalloc((void**)&q.h_wire, b->wire_cap, hipHostMallocDefault) == hipSuccess &&
           hipHostMalloc((void**)&q.h_streams, ns * sizeof(uvhttp_ws_stream_t), hipHostMallocDefault) == hipSuccess &&
           hipHostMalloc((void**)&q.h_results, ns * sizeof(uvhttp_ws_stream_result_t), hipHostMallocDefault) == hipSuccess &&
           hipHostMalloc((void**)&q.h_read_end, nr * sizeof(uint64_t), hipHostMallocDefault) == hipSuccess &&
           hipHostMalloc((void**)&q.h_desc, (size_t)q.max_frames * sizeof(uvhttp_ws_frame_desc_t), hipHostMallocDefault) == hipSuccess &&
           hipHostMalloc((void**)&q.h_seg, (nr + ns) * sizeof(GatherSeg), hipHostMallocDefault) == hipSuccess &&
           hipMalloc((void**)&q.d_arena, b->wire_cap) == hipSuccess &&
           hipMalloc((void**)&q.d_wire, b->wire_cap) == hipSuccess &&
           hipMalloc((void**)&q.d_streams, ns * sizeof(uvhttp_ws_stream_t)) == hipSuccess &&
           hipMalloc((void**)&q.d_results, ns * sizeof(uvhttp_ws_stream_result_t)) == hipSuccess &&
           hipMalloc((void**)&q.d_read_end, nr * sizeof(uint64_t)) == hipSuccess &&
           hipMalloc((void**)&q.d_desc, (size_t)q.max_frames * sizeof(uvhttp_ws_frame_desc_t)) == hipSuccess &&
           hipMalloc((void**)&q.d_seg, (nr + ns) * sizeof(GatherSeg)) == hipSuccess &&
           hipEventCreateWithFlags(&q.up_ev, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&q.done_ev, hipEventDisableTiming) == hipSuccess;
}

void release(uvhttp_ws_amd_batcher_t* b) {
    if (b->eng) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(b->cfg.device);
        if (b->up) (void)hipStreamSynchronize(b->up);
        if (b->cs) (void)hipStreamSynchronize(b->cs);
        free_queue(b->q[0]);
        free_queue(b->q[1]);
        if (b->up) (void)hipStreamDestroy(b->up);
        if (b->cs) (void)hipStreamDestroy(b->cs);
        uvhttp_ws_gpu_engine_free(b->eng);
        if (b->teng) uvhttp_tls_gpu_engine_free(b->teng);
        (void)hipSetDevice(prev);
    }
    delete b;
}

void clear_queue(BatchQueue& q) {
    q.gen++;
    q.arena.clear();
    q.arena_len = q.uploaded = 0;
    q.reads.clear();
    q.slots.clear();
    q.slot_of.clear();
    q.staged = q.bytes = 0;
    q.in_flight = false;
    q.launch_rc = 0;
    q.nk = 0;
    q.pos = 0;
    q.nt = 0;
    q.n_tls_slots = 0;
    q.tls_bytes = q.plain_cap = 0;
    q.slot_k.clear();
    q.carry_off.clear();
    q.carry_len.clear();
}

// device batcher: the arena bytes not yet sent go to HBM on the upload stream
void upload_tail(uvhttp_ws_amd_batcher_t* b, BatchQueue& q) {
    if (q.arena_len > q.uploaded) {
        uvhttp_ws_amd_copy_fence();  // the reads' streaming stores before the DMA engine reads them
        (void)hipMemcpyAsync(q.d_arena + q.uploaded, q.h_arena + q.uploaded,
                             q.arena_len - q.uploaded, hipMemcpyHostToDevice, b->up);
        q.uploaded = q.arena_len;
    }
}

void report_failure(uvhttp_ws_amd_batcher_t* b, uvhttp_ws_connection_t* conn, int rc) {
    b->failed.insert(conn);
    b->st.failures++;
    if (b->cfg.on_failure) b->cfg.on_failure(b->cfg.ctx, conn, rc);
}

// the reference's path: process_data per read, until one fails.  Slots are addressed by
// index and re-read after every callback (forget() may mark one dropped meanwhile); reads
// submitted from callbacks go to the other queue, so this queue does not change under us.
void flush_host(uvhttp_ws_amd_batcher_t* b, BatchQueue& q) {
    b->st.host_flushes++;
    b->delivering++;
    for (size_t k = 0; k < q.slots.size(); ++k) {
        if (q.slots[k].tls) continue;  // ciphertext: only the device opens records
        for (size_t j = 0; j < q.slots[k].reads.size(); ++j) {
            if (q.slots[k].dropped || b->failed.count(q.slots[k].conn)) break;
            const QueuedRead r = q.reads[q.slots[k].reads[j]];
            uvhttp_ws_connection_t* conn = q.slots[k].conn;
            const uvhttp_error_t rc =
                uvhttp_ws_process_data(conn, arena_data(b, q) + r.off, (size_t)r.len);
            b->st.host_reads++;
            if (rc != UVHTTP_OK) {
                q.slots[k].dropped = true;
                report_failure(b, conn, rc);
            }
        }
    }
    b->delivering--;
}

// grow a queue's descriptor capacity to nf frames (device + pinned host copy)
int grow_desc(uvhttp_ws_amd_batcher_t* b, BatchQueue& q, uint64_t nf) {
    if (nf <= q.max_frames) return 0;
    uint64_t want = 2ull * q.max_frames;
    if (want < nf) want = nf;
    if (want > kMaxFramesPerFlush) want = kMaxFramesPerFlush;
    if (want < nf) return 1;  // more frames than one decode takes: the host decodes it
    (void)hipHostFree(q.h_desc);
    (void)hipFree(q.d_desc);
    q.h_desc = nullptr;
    q.d_desc = nullptr;
    q.max_frames = 0;
    if (hipHostMalloc((void**)&q.h_desc, want * sizeof(uvhttp_ws_frame_desc_t), hipHostMallocDefault) != hipSuccess ||
        hipMalloc((void**)&q.d_desc, want * sizeof(uvhttp_ws_frame_desc_t)) != hipSuccess ||
        uvhttp_ws_gpu_engine_reserve(b->eng, (uint32_t)want, b->wire_cap, 0) != 0)
        return UVHTTP_WS_GPU_ENOMEM;
    q.max_frames = (uint32_t)want;
    return 0;
}

// Stage q's connections (recv-buffer prefixes from their current state, read tables) and
// enqueue H2D -> gather -> decode_reads -> D2H (and, for TLS connections, open_records ->
// ws_streams -> decode_reads on the plaintext).  Returns 0 when launched, 1 when the queue
// must be decoded on the host instead (it does not fit the device layout), < 0 on an error.
int launch_device(uvhttp_ws_amd_batcher_t* b, BatchQueue& q) {
    uint64_t pos = 0;
    uint32_t nr = 0, nk = 0, nt = 0, nseg = 0;
    q.slot_k.assign(q.slots.size(), UINT32_MAX);
    q.carry_off.assign(q.slots.size(), 0);
    q.carry_len.assign(q.slots.size(), 0);
    auto live = [&](const ConnSlot& s) {
        return !s.dropped && !b->failed.count(s.conn) && (!s.tls || b->tls.count(s.conn));
    };
    // room check first: prefixes (and TLS carries) go after the reads in the arena, and the
    // device layout (16-byte aligned connections) must fit the device wire; a TLS
    // connection's plaintext reservation (prefix + at most its ciphertext) must fit d_plain
    uint64_t extra = 0, layout = 0, plain_need = 0;
    for (const ConnSlot& s : q.slots) {
        if (!live(s)) continue;
        const uint64_t carry = s.tls ? b->tls[s.conn].carry.size() : 0;
        extra += s.conn->recv_buffer_pos + carry;
        layout = align16(layout) + (s.tls ? carry : s.conn->recv_buffer_pos) + s.bytes + 16;
        if (s.tls) plain_need = align16(plain_need) + s.conn->recv_buffer_pos + carry + s.bytes + 16;
    }
    if (q.arena_len + extra > b->wire_cap || layout > b->wire_cap || plain_need > b->wire_cap)
        return 1;
    // plain connections first
    for (size_t k = 0; k < q.slots.size(); ++k) {
        ConnSlot& s = q.slots[k];
        if (s.tls || !live(s)) continue;
        uvhttp_ws_connection_t* c = s.conn;
        pos = align16(pos);
        const uint64_t begin = pos;
        if (c->recv_buffer_pos) {  // the bytes recv_buffer already holds come first
            const uint64_t off = q.arena_len;
            memcpy(q.h_arena + off, c->recv_buffer, c->recv_buffer_pos);
            q.arena_len += c->recv_buffer_pos;
            q.h_seg[nseg++] = GatherSeg{off, pos, c->recv_buffer_pos};
        }
        pos += c->recv_buffer_pos;
        const uint32_t r0 = nr;
        for (uint32_t r : s.reads) {
            const QueuedRead& qr = q.reads[r];
            if (qr.len) q.h_seg[nseg++] = GatherSeg{qr.off, pos, qr.len};
            pos += qr.len;
            q.h_read_end[nr++] = pos - begin;
        }
        uvhttp_ws_stream_init(c, begin, pos - begin, &q.h_streams[nk]);
        q.h_streams[nk].first_read = r0;
        q.h_streams[nk].n_reads = nr - r0;
        q.slot_k[k] = nk++;
    }
    q.nk = nk;
    q.pos = pos;
    // TLS connections: ciphertext (carry, then reads) after the plain layout; their
    // recv-buffer prefixes stay in the arena, where ws_streams copies them from
    const uint64_t tls_base = align16(pos);
    uint64_t tpos = tls_base, plain_cap = 0;
    for (size_t k = 0; k < q.slots.size(); ++k) {
        ConnSlot& s = q.slots[k];
        if (!s.tls || !live(s)) continue;
        uvhttp_ws_connection_t* c = s.conn;
        TlsConn& t = b->tls[c];
        tpos = align16(tpos);
        const uint64_t cbegin = tpos;
        if (!t.carry.empty()) {
            const uint64_t off = q.arena_len;
            memcpy(q.h_arena + off, t.carry.data(), t.carry.size());
            q.arena_len += t.carry.size();
            q.h_seg[nseg++] = GatherSeg{off, tpos, (uint64_t)t.carry.size()};
            q.carry_off[k] = off;
            q.carry_len[k] = t.carry.size();
            tpos += t.carry.size();
        }
        for (uint32_t r : s.reads) {
            const QueuedRead& qr = q.reads[r];
            if (qr.len) q.h_seg[nseg++] = GatherSeg{qr.off, tpos, qr.len};
            tpos += qr.len;
        }
        q.h_poff[nt] = q.arena_len;
        if (c->recv_buffer_pos) {
            memcpy(q.h_arena + q.arena_len, c->recv_buffer, c->recv_buffer_pos);
            q.arena_len += c->recv_buffer_pos;
        }
        uvhttp_tls_stream_t ts;
        memset(&ts, 0, sizeof(ts));
        ts.begin = cbegin - tls_base;
        ts.len = tpos - cbegin;
        ts.seq = t.seq;
        ts.key = nt;
        ts.ws_prefix = (uint32_t)c->recv_buffer_pos;
        q.h_tst[nt] = ts;
        q.h_keys[nt] = t.key;
        uvhttp_ws_stream_init(c, 0, 0, &q.h_wst[nt]);  // ws_streams sets begin / len / reads
        plain_cap = align16(plain_cap) + c->recv_buffer_pos + (tpos - cbegin) + 16;
        q.slot_k[k] = nt++;
    }
    q.nt = nt;
    q.tls_base = tls_base;
    q.tls_bytes = tpos - tls_base;
    q.plain_cap = plain_cap;
    if (!nk && !nt) return 1;  // nothing left to decode (all dropped): the host path is a no-op
    // descriptors: the decode runs with the capacity the queue has (grown by earlier
    // flushes); a decode with more frames reports ERR_CAPACITY without touching a byte and
    // complete_device re-runs it with more (pre-sizing for the worst case — 6-byte frames —
    // pinned GiBs of host memory per queue and stalled the loop for 100s of ms)
    // records: every counted record but a connection's stopping one has >= 5 + 16 bytes
    const uint64_t max_records = q.tls_bytes / 21 + nt + 1;
    q.nr = nr;
    q.max_records = max_records;
    if (nt) {
        const int gt = grow_tls(b, q, max_records, q.wdesc_cap ? q.wdesc_cap : kMinFrames);
        if (gt) return gt;
    }
#ifdef UVWS_TEST_HOOKS
    if (b->fail_every && ++b->launches % b->fail_every == 0) return UVHTTP_WS_GPU_ELAUNCH;
#endif
    hipStream_t s = b->cs;
    // UVHTTP_WS_BATCHER_TRACE=1 (experiment builds): host time of each enqueue step on stderr
#ifdef UVWS_EXPERIMENTS
    static const bool trace = getenv("UVHTTP_WS_BATCHER_TRACE") != nullptr;
#else
    constexpr bool trace = false;
#endif
    auto tp = std::chrono::steady_clock::now();
    auto mark = [&](const char* what) {
        if (!trace) return;
        fprintf(stderr, "[batcher] %-12s %8.3f ms\n", what, ms_since(tp));
        tp = std::chrono::steady_clock::now();
    };
    upload_tail(b, q);
    mark("upload_tail");
    hipError_t h = hipEventRecord(q.up_ev, b->up);
    if (h == hipSuccess) h = hipStreamWaitEvent(s, q.up_ev, 0);
    mark("up_event");
    if (h == hipSuccess && nseg)
        h = hipMemcpyAsync(q.d_seg, q.h_seg, nseg * sizeof(GatherSeg), hipMemcpyHostToDevice, s);
    mark("seg_h2d");
    if (h == hipSuccess && nseg) {
        hipLaunchKernelGGL(k_batcher_gather, dim3(nseg), dim3(256), 0, s, q.d_arena, q.d_wire, q.d_seg);
        h = hipGetLastError();
    }
    mark("gather");
    int rc = UVHTTP_WS_GPU_OK;
    if (nk) {
        if (h == hipSuccess)
            h = hipMemcpyAsync(q.d_streams, q.h_streams, nk * sizeof(uvhttp_ws_stream_t),
                               hipMemcpyHostToDevice, s);
        if (h == hipSuccess && nr)
            h = hipMemcpyAsync(q.d_read_end, q.h_read_end, nr * sizeof(uint64_t), hipMemcpyHostToDevice, s);
        mark("tables_h2d");
        if (h == hipSuccess)
            rc = uvhttp_ws_gpu_decode_reads(b->eng, q.d_wire, pos, q.d_streams, nk, q.d_read_end, nr,
                                            q.max_frames, q.d_desc, q.d_results, s);
        mark("decode_reads");
        if (h == hipSuccess && rc == UVHTTP_WS_GPU_OK)
            h = hipMemcpyAsync(q.h_results, q.d_results, nk * sizeof(uvhttp_ws_stream_result_t),
                               hipMemcpyDeviceToHost, s);
        if (h == hipSuccess && rc == UVHTTP_WS_GPU_OK)
            h = hipMemcpyAsync(q.h_wire, q.d_wire, pos, hipMemcpyDeviceToHost, s);
        // the descriptors too, as many as recent flushes used (the frame count is only known
        // on the device): a synchronous copy of all of them after completion queued behind the
        // next queue's uploads on the copy engine and blocked the loop for milliseconds, and
        // copying the whole capacity moved up to bytes / 6 descriptors per flush
        q.desc_copied = b->desc_hint < q.max_frames ? b->desc_hint : q.max_frames;
        if (h == hipSuccess && rc == UVHTTP_WS_GPU_OK)
            h = hipMemcpyAsync(q.h_desc, q.d_desc, (size_t)q.desc_copied * sizeof(uvhttp_ws_frame_desc_t),
                               hipMemcpyDeviceToHost, s);
        mark("d2h");
    }
    if (nt && h == hipSuccess && rc == UVHTTP_WS_GPU_OK) {
        h = hipMemcpyAsync(q.d_keys, q.h_keys, nt * sizeof(uvhttp_tls_key_t), hipMemcpyHostToDevice, s);
        if (h == hipSuccess)
            h = hipMemcpyAsync(q.d_tst, q.h_tst, nt * sizeof(uvhttp_tls_stream_t), hipMemcpyHostToDevice, s);
        if (h == hipSuccess)
            h = hipMemcpyAsync(q.d_wst, q.h_wst, nt * sizeof(uvhttp_ws_stream_t), hipMemcpyHostToDevice, s);
        if (h == hipSuccess)
            h = hipMemcpyAsync(q.d_poff, q.h_poff, nt * sizeof(uint64_t), hipMemcpyHostToDevice, s);
        if (h == hipSuccess) {
            rc = uvhttp_tls_gpu_open_records(b->teng, q.d_wire + tls_base, q.tls_bytes, q.d_keys, nt,
                                             q.d_tst, nt, q.d_trecs, (uint32_t)max_records, q.d_tres,
                                             q.d_plain, plain_cap, s);
            if (!rc)
                rc = uvhttp_tls_gpu_ws_streams(b->teng, q.d_tres, q.d_trecs, nt, q.d_tst, q.d_arena,
                                               q.d_poff, q.d_plain, q.d_wst, q.d_wread_end, s);
            if (!rc)
                rc = uvhttp_ws_gpu_decode_reads(b->eng, q.d_plain, plain_cap, q.d_wst, nt,
                                                q.d_wread_end, (uint32_t)max_records, q.wdesc_cap,
                                                q.d_wdesc, q.d_wres, s);
            if (rc) rc = UVHTTP_WS_GPU_ELAUNCH;
        }
        if (h == hipSuccess && !rc)
            h = hipMemcpyAsync(q.h_tres, q.d_tres, nt * sizeof(uvhttp_tls_result_t), hipMemcpyDeviceToHost, s);
        if (h == hipSuccess && !rc)
            h = hipMemcpyAsync(q.h_wres, q.d_wres, nt * sizeof(uvhttp_ws_stream_result_t),
                               hipMemcpyDeviceToHost, s);
        if (h == hipSuccess && !rc)
            h = hipMemcpyAsync(q.h_wst, q.d_wst, nt * sizeof(uvhttp_ws_stream_t), hipMemcpyDeviceToHost, s);
        if (h == hipSuccess && !rc)
            h = hipMemcpyAsync(q.h_plain, q.d_plain, plain_cap, hipMemcpyDeviceToHost, s);
        q.wdesc_copied = b->wdesc_hint < q.wdesc_cap ? b->wdesc_hint : q.wdesc_cap;
        if (h == hipSuccess && !rc)
            h = hipMemcpyAsync(q.h_wdesc, q.d_wdesc, (size_t)q.wdesc_copied * sizeof(uvhttp_ws_frame_desc_t),
                               hipMemcpyDeviceToHost, s);
    }
    if (h == hipSuccess && rc == UVHTTP_WS_GPU_OK) h = hipEventRecord(q.done_ev, s);
    if (h == hipSuccess && rc == UVHTTP_WS_GPU_OK && b->cfg.on_ready)
        h = hipLaunchHostFunc(s, b->cfg.on_ready, b->cfg.ready_ctx);
    if (h != hipSuccess) return UVHTTP_WS_GPU_ELAUNCH;
    return rc;
}

// bytes [from, end) of a TLS slot's staged ciphertext (its carry, then its reads)
std::vector<uint8_t> tls_tail(const BatchQueue& q, size_t k, uint64_t from) {
    std::vector<uint8_t> out;
    uint64_t at = 0;
    auto take = [&](const uint8_t* p, uint64_t n) {
        if (at + n > from) {
            const uint64_t skip = from > at ? from - at : 0;
            out.insert(out.end(), p + skip, p + n);
        }
        at += n;
    };
    take(q.h_arena + q.carry_off[k], q.carry_len[k]);
    for (uint32_t r : q.slots[k].reads) take(q.h_arena + q.reads[r].off, q.reads[r].len);
    return out;
}

// the connection's TLS handling ends here (CONTROL record): everything from that record on,
// including ciphertext it has queued in the accumulating queue since, goes back to the caller
void tls_handback(uvhttp_ws_amd_batcher_t* b, uvhttp_ws_connection_t* conn,
                  std::vector<uint8_t> bytes, uint64_t next_seq, int status) {
    BatchQueue& acc = b->q[b->cur];
    auto it = acc.slot_of.find(conn);
    if (it != acc.slot_of.end() && acc.slots[it->second].tls) {
        ConnSlot& s = acc.slots[it->second];
        for (uint32_t r : s.reads)
            bytes.insert(bytes.end(), acc.h_arena + acc.reads[r].off,
                         acc.h_arena + acc.reads[r].off + acc.reads[r].len);
        s.dropped = true;
        acc.slot_of.erase(it);
    }
    b->tls.erase(conn);
    b->st.tls_handbacks++;
    if (b->cfg.on_tls_handback)
        b->cfg.on_tls_handback(b->cfg.ctx, conn, bytes.data(), bytes.size(), next_seq, status);
}

// A queue's TLS slots could not be opened on the device (a device or launch error, or a queue
// that did not fit the device layout).  Nothing of them was delivered and their ciphertext is
// intact — the connection's carry plus its reads in this queue — so it goes back to the caller
// from the connection's next record on (on_tls_handback, status
// UVHTTP_WS_BATCHER_HANDBACK_DEVICE): mbedtls reads it on the host, as it would have without the
// batcher.  Only with no handback callback does the connection fail (the host has no AEAD).
void handback_tls_slots(uvhttp_ws_amd_batcher_t* b, BatchQueue& q) {
    b->delivering++;  // (the callback runs as a delivery's: no nested flushes)
    for (size_t k = 0; k < q.slots.size(); ++k) {
        ConnSlot& s = q.slots[k];
        if (!s.tls || s.dropped || b->failed.count(s.conn)) continue;
        s.dropped = true;
        auto ti = b->tls.find(s.conn);
        if (ti == b->tls.end()) continue;  // (forgotten meanwhile)
        if (!b->cfg.on_tls_handback) {
            b->tls.erase(ti);
            report_failure(b, s.conn, UVHTTP_ERROR_INVALID_PARAM);
            continue;
        }
        std::vector<uint8_t> bytes = ti->second.carry;
        for (uint32_t r : s.reads)
            bytes.insert(bytes.end(), q.h_arena + q.reads[r].off, q.h_arena + q.reads[r].off + q.reads[r].len);
        tls_handback(b, s.conn, std::move(bytes), ti->second.seq, UVHTTP_WS_BATCHER_HANDBACK_DEVICE);
    }
    b->delivering--;
}

// A decode whose frames did not fit its descriptors reported ERR_CAPACITY and unmasked
// nothing: grow the descriptors (up to the bytes / 6 + connections bound of server frames)
// and run it again on the device, synchronously (rare: capacities only grow).
int rerun_over_capacity(uvhttp_ws_amd_batcher_t* b, BatchQueue& q) {
    auto over = [](const uvhttp_ws_stream_result_t* r, uint32_t n) {
        for (uint32_t k = 0; k < n; ++k)
            if (r[k].first_status == UVHTTP_WS_FRAME_ERR_CAPACITY) return true;
        return false;
    };
    hipStream_t s = b->cs;
    const uint64_t bound = q.pos / 6 + q.nk + 1;
    while (q.nk && over(q.h_results, q.nk) && q.max_frames < bound) {
        const uint64_t want = 8ull * q.max_frames < bound ? 8ull * q.max_frames : bound;
        if (grow_desc(b, q, want)) break;  // (left over capacity: the host decodes it)
        int rc = uvhttp_ws_gpu_decode_reads(b->eng, q.d_wire, q.pos, q.d_streams, q.nk, q.d_read_end,
                                            q.nr, q.max_frames, q.d_desc, q.d_results, s);
        if (!rc && (hipMemcpyAsync(q.h_results, q.d_results, q.nk * sizeof(uvhttp_ws_stream_result_t),
                                   hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipMemcpyAsync(q.h_wire, q.d_wire, q.pos, hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipMemcpyAsync(q.h_desc, q.d_desc, (size_t)q.max_frames * sizeof(uvhttp_ws_frame_desc_t),
                                   hipMemcpyDeviceToHost, s) != hipSuccess))
            rc = UVHTTP_WS_GPU_ELAUNCH;
        q.desc_copied = q.max_frames;
        if (!rc) rc = uvhttp_ws_gpu_engine_sync(b->eng, s);
        if (rc) return rc;
    }
    const uint64_t wbound = q.plain_cap / 6 + q.nt + 1;
    while (q.nt && over(q.h_wres, q.nt) && q.wdesc_cap < wbound) {
        const uint64_t want = 8ull * q.wdesc_cap < wbound ? 8ull * q.wdesc_cap : wbound;
        if (grow_tls(b, q, q.max_records, want)) break;
        int rc = uvhttp_ws_gpu_decode_reads(b->eng, q.d_plain, q.plain_cap, q.d_wst, q.nt,
                                            q.d_wread_end, (uint32_t)q.max_records, q.wdesc_cap,
                                            q.d_wdesc, q.d_wres, s);
        if (!rc && (hipMemcpyAsync(q.h_wres, q.d_wres, q.nt * sizeof(uvhttp_ws_stream_result_t),
                                   hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipMemcpyAsync(q.h_plain, q.d_plain, q.plain_cap, hipMemcpyDeviceToHost, s) != hipSuccess ||
                    hipMemcpyAsync(q.h_wdesc, q.d_wdesc, (size_t)q.wdesc_cap * sizeof(uvhttp_ws_frame_desc_t),
                                   hipMemcpyDeviceToHost, s) != hipSuccess))
            rc = UVHTTP_WS_GPU_ELAUNCH;
        q.wdesc_copied = q.wdesc_cap;
        if (!rc) rc = uvhttp_ws_gpu_engine_sync(b->eng, s);
        if (rc) return rc;
    }
    return UVHTTP_WS_GPU_OK;
}

// descriptors [copied, used) of a finished decode, when the launch copied back fewer than it
// produced (synchronous; rare once the high-water mark has seen the flush shape)
int fetch_rest(uvhttp_ws_amd_batcher_t* b, const uvhttp_ws_frame_desc_t* d, uvhttp_ws_frame_desc_t* h,
               uint64_t copied, uint64_t used) {
    if (used <= copied) return 0;
    b->st.desc_refetches++;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != b->cfg.device) (void)hipSetDevice(b->cfg.device);
    const hipError_t h2 = hipMemcpy(h + copied, d + copied,
                                    (size_t)(used - copied) * sizeof(uvhttp_ws_frame_desc_t),
                                    hipMemcpyDeviceToHost);
    if (prev != b->cfg.device) (void)hipSetDevice(prev);
    return h2 == hipSuccess ? 0 : UVHTTP_WS_GPU_ELAUNCH;
}

// the next launches' copy-back: a quarter above this flush's frames, decaying by 1/8 per flush
uint64_t next_hint(uint64_t hint, uint64_t frames) {
    const uint64_t want = frames + frames / 4 + 256;
    const uint64_t decayed = hint - hint / 8;
    return want > decayed ? want : decayed;
}

// q's decode has finished (or failed): deliver it, or decode it on the host when the
// device could not (nothing of q has been delivered before this point; TLS connections,
// which the host cannot open, fail instead).
// the batcher's device is current for the scope (a group's members live on different GPUs, and
// a re-run grows device buffers: they must land on this batcher's device)
struct DeviceScope {
    int prev = -1, dev;
    explicit DeviceScope(int d) : dev(d) {
        if (dev < 0) return;
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceScope() {
        if (dev >= 0 && prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
};

int complete_device(uvhttp_ws_amd_batcher_t* b, BatchQueue& q) {
    DeviceScope ds(b->cfg.device);
    int rc = q.launch_rc;
    if (!rc) {
        const auto tw = std::chrono::steady_clock::now();
        if (hipEventSynchronize(q.done_ev) != hipSuccess) rc = UVHTTP_WS_GPU_ELAUNCH;
        else rc = uvhttp_ws_gpu_engine_sync(b->eng, b->cs);  // device-side give-ups
        b->st.wait_ms += ms_since(tw);
    }
    uint64_t frames = 0, wframes = 0;
    bool capacity = false;
    if (!rc) rc = rerun_over_capacity(b, q);
    if (!rc) {
        for (uint32_t k = 0; k < q.nk; ++k) {
            const uvhttp_ws_stream_result_t& r = q.h_results[k];
            if (r.first_status == UVHTTP_WS_FRAME_ERR_CAPACITY) capacity = true;
            const uint64_t e = (uint64_t)r.first_frame + r.n_frames;
            if (r.n_frames && e > frames) frames = e;
        }
        for (uint32_t k = 0; k < q.nt; ++k) {
            const uvhttp_ws_stream_result_t& r = q.h_wres[k];
            const uint64_t e = (uint64_t)r.first_frame + r.n_frames;
            if (r.first_status != UVHTTP_WS_FRAME_ERR_CAPACITY && r.n_frames && e > wframes) wframes = e;
        }
        // the descriptors came back with the results (launch_device / rerun_over_capacity)
        // up to the high-water mark; a flush with more frames fetches the rest now
        rc = fetch_rest(b, q.d_desc, q.h_desc, q.desc_copied, capacity ? 0 : frames);
        if (!rc) rc = fetch_rest(b, q.d_wdesc, q.h_wdesc, q.wdesc_copied, wframes);
        b->desc_hint = next_hint(b->desc_hint, frames);
        if (q.nt) b->wdesc_hint = next_hint(b->wdesc_hint, wframes);
    }
    if (rc) {
        // the host decodes the plain connections instead (their reads are still in the
        // pinned arena and no connection has seen any of them); a device error is counted
        // and returned
        b->st.device_errors++;
        flush_host(b, q);
        handback_tls_slots(b, q);
        return rc;
    }
    if (capacity) {  // more plain frames than the descriptors hold (client connections)
        b->st.capacity_flushes++;
        flush_host(b, q);
    } else {
        b->st.device_bytes += q.pos;
        b->st.device_frames += frames;
    }
    b->st.device_flushes++;
    b->st.device_bytes += q.tls_bytes;
    b->st.device_frames += wframes;
    // deliver, connection by connection (callbacks may forget connections as we go)
    const auto td = std::chrono::steady_clock::now();
    b->delivering++;
    for (size_t k = 0; k < q.slots.size(); ++k) {
        if (q.slot_k[k] == UINT32_MAX || q.slots[k].dropped) continue;
        const uint32_t j = q.slot_k[k];
        uvhttp_ws_connection_t* conn = q.slots[k].conn;
        if (!q.slots[k].tls) {
            if (capacity) continue;  // (decoded by the host above)
            const uvhttp_error_t dr =
                uvhttp_ws_deliver_stream(conn, q.h_wire, q.h_desc, &q.h_streams[j], &q.h_results[j]);
            b->st.device_reads += q.h_results[j].calls;
            if (dr != UVHTTP_OK) {
                q.slots[k].dropped = true;
                report_failure(b, conn, dr);
            }
            continue;
        }
        // TLS: the records delivered, each one process_data call on its content
        const uvhttp_tls_result_t tr = q.h_tres[j];
        if (tr.first_status == UVHTTP_TLS_REC_ERR_KEY || tr.first_status == UVHTTP_TLS_REC_ERR_CAPACITY ||
            q.h_wres[j].first_status == UVHTTP_WS_FRAME_ERR_CAPACITY) {
            q.slots[k].dropped = true;
            b->tls.erase(conn);
            report_failure(b, conn, UVHTTP_ERROR_INVALID_PARAM);
            continue;
        }
        bool ws_failed = false;
        if (tr.n_delivered) {  // (no complete record: mbedtls_ssl_read returned WANT_READ)
            const uvhttp_error_t dr =
                uvhttp_ws_deliver_stream(conn, q.h_plain, q.h_wdesc, &q.h_wst[j], &q.h_wres[j]);
            b->st.device_reads += q.h_wres[j].calls;
            b->st.tls_records += tr.n_delivered;
            b->st.tls_bytes += tr.consumed_bytes;
            if (dr != UVHTTP_OK) {
                q.slots[k].dropped = true;
                b->tls.erase(conn);
                report_failure(b, conn, dr);
                ws_failed = true;
            }
        }
        if (ws_failed || q.slots[k].dropped) continue;  // (forgotten from a callback)
        auto ti = b->tls.find(conn);
        if (ti == b->tls.end()) continue;
        std::vector<uint8_t> rest = tls_tail(q, k, tr.consumed_bytes);
        if (tr.first_status == UVHTTP_TLS_REC_CONTROL) {
            tls_handback(b, conn, std::move(rest), tr.next_seq, tr.first_status);
        } else if (tr.status != 0) {  // bad MAC / overflow / bad type / version: close
            q.slots[k].dropped = true;
            b->tls.erase(ti);
            report_failure(b, conn, UVHTTP_ERROR_INVALID_PARAM);
        } else {  // an incomplete record (or none) waits for the next reads
            ti->second.seq = tr.next_seq;
            ti->second.carry.swap(rest);
        }
    }
    b->delivering--;
    b->st.deliver_ms += ms_since(td);
    b->st.device_ms += ms_since(q.t_submit);
    return 0;
}

// Finish the queue in flight, if any.  wait = false: only when its results are already back.
// Returns 1 when a queue was delivered, 0 when none (or not ready), < 0 a device error (the
// queue was then decoded on the host).
int finish_inflight(uvhttp_ws_amd_batcher_t* b, bool wait) {
    BatchQueue& q = b->q[b->cur ^ 1];
    if (!q.in_flight) return 0;
    if (!wait && !q.launch_rc && hipEventQuery(q.done_ev) == hipErrorNotReady) return 0;
    const int rc = complete_device(b, q);
    clear_queue(q);
    return rc < 0 ? rc : 1;
}

// Hand the accumulating queue over: finish the one in flight (its connections' state must be
// final before this queue is staged), switch submit_read to the other queue, then decode this
// one on the host (small) or start its device decode.  wait = false: when the queue in flight
// is not finished yet, only note the request (poll starts the queue once it has delivered).
int start_flush(uvhttp_ws_amd_batcher_t* b, bool wait) {
    const BatchQueue& other = b->q[b->cur ^ 1];
    if (other.in_flight && !wait && !other.launch_rc && hipEventQuery(other.done_ev) == hipErrorNotReady) {
        b->want_flush = true;
        return 0;
    }
    int rc = finish_inflight(b, true);
    rc = rc < 0 ? rc : 0;
    b->want_flush = false;
    BatchQueue& q = b->q[b->cur];
    if (q.reads.empty()) return rc;
    b->st.flushes++;
    b->cur ^= 1;  // reads submitted from now on (callbacks included) queue in the other one
    if (b->eng && (q.bytes >= b->cfg.min_device_bytes || q.n_tls_slots)) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        if (prev != b->cfg.device) (void)hipSetDevice(b->cfg.device);
        q.t_submit = std::chrono::steady_clock::now();
        const auto tl = std::chrono::steady_clock::now();
        const int lr = launch_device(b, q);
        b->st.stage_ms += ms_since(tl);
        if (prev != b->cfg.device) (void)hipSetDevice(prev);
        if (lr == 1) {
            b->st.fallback_flushes++;
            flush_host(b, q);
            handback_tls_slots(b, q);
            clear_queue(q);
        } else {
            // launched, or a launch error that complete_device turns into a host decode
            q.in_flight = true;
            q.launch_rc = lr;
            b->st.async_flushes++;
        }
    } else {
        flush_host(b, q);
        clear_queue(q);
    }
    return rc;
}

constexpr size_t kBlockedKeep = 65536;

// loop-thread time spent inside one batcher call (waiting, staging, delivering): summed, kept
// per call for the percentiles, and the longest call's split by phase
struct Blocked {
    uvhttp_ws_amd_batcher_t* b;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    double wait0 = b->st.wait_ms, stage0 = b->st.stage_ms, deliver0 = b->st.deliver_ms;
    ~Blocked() {
        const double ms = ms_since(t0);
        b->st.blocked_ms += ms;
        b->st.blocked_calls++;
        if (b->blocked.size() < kBlockedKeep) b->blocked.push_back((float)ms);
        else b->blocked[b->blocked_n % kBlockedKeep] = (float)ms;
        b->blocked_n++;
        if (ms > b->st.max_blocked_ms) {
            b->st.max_blocked_ms = ms;
            b->st.max_blocked_wait_ms = b->st.wait_ms - wait0;
            b->st.max_blocked_stage_ms = b->st.stage_ms - stage0;
            b->st.max_blocked_deliver_ms = b->st.deliver_ms - deliver0;
        }
    }
};

}  // namespace

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
    // one flush's device layout must stay addressable by decode_reads (its frame bound is
    // bytes / 6 + connections <= 2^26; larger flushes would always fall back to the host)
    if (cfg->device >= 0 && cfg->max_bytes / 6 + cfg->max_connections + 1 > kMaxFramesPerFlush)
        return UVHTTP_WS_GPU_EINVAL;
    uvhttp_ws_amd_batcher_t* b = new (std::nothrow) uvhttp_ws_amd_batcher_t();
    if (!b) return UVHTTP_WS_GPU_ENOMEM;
    b->cfg = *cfg;
    memset(&b->st, 0, sizeof(b->st));
    if (cfg->device < 0) {
        const size_t r = cfg->max_bytes < (64ull << 20) ? cfg->max_bytes : (64ull << 20);
        b->q[0].arena.reserve(r);
        b->q[1].arena.reserve(r);
    } else {
        int rc = uvhttp_ws_gpu_engine_create(cfg->device, &b->eng);
        if (rc) {
            b->eng = nullptr;
            delete b;
            return rc;
        }
        b->wire_cap = cfg->max_bytes + 16ull * cfg->max_connections + 64;
#ifdef UVWS_TEST_HOOKS
        if (const char* fe = getenv("UVHTTP_WS_BATCHER_FAIL_EVERY")) b->fail_every = (uint32_t)atoi(fe);
#endif
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(cfg->device);
        bool ok = hipStreamCreateWithFlags(&b->up, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamCreateWithFlags(&b->cs, hipStreamNonBlocking) == hipSuccess &&
                  alloc_queue(b, b->q[0]) && alloc_queue(b, b->q[1]);
        if (ok) ok = uvhttp_ws_gpu_engine_reserve(b->eng, kMinFrames, b->wire_cap, 0) == 0;
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

int uvhttp_ws_amd_batcher_flush_async(uvhttp_ws_amd_batcher_t* b) {
    if (!b) return UVHTTP_WS_GPU_EINVAL;
    if (b->delivering) return UVHTTP_WS_GPU_OK;  // (from a callback: the caller flushes later)
    Blocked bl{b};
    return start_flush(b, false);
}

int uvhttp_ws_amd_batcher_poll(uvhttp_ws_amd_batcher_t* b) {
    if (!b) return UVHTTP_WS_GPU_EINVAL;
    if (b->delivering) return 0;
    if (!b->q[b->cur ^ 1].in_flight) return 0;
    Blocked bl{b};
    const int rc = finish_inflight(b, false);
    if (rc != 0 && b->want_flush) {  // delivered: start what flush_async asked for meanwhile
        const int r2 = start_flush(b, false);
        if (r2 < 0 && rc > 0) return r2;
    }
    return rc;
}

int uvhttp_ws_amd_batcher_in_flight(const uvhttp_ws_amd_batcher_t* b) {
    return b && b->q[b->cur ^ 1].in_flight ? 1 : 0;
}

int uvhttp_ws_amd_batcher_flush(uvhttp_ws_amd_batcher_t* b) {
    if (!b) return UVHTTP_WS_GPU_EINVAL;
    if (b->delivering) return UVHTTP_WS_GPU_OK;
    Blocked bl{b};
    int rc = start_flush(b, true);            // finishes the queue in flight, starts this one
    const int r2 = finish_inflight(b, true);  // and waits for it
    if (!rc && r2 < 0) rc = r2;
    return rc;
}

}  // extern "C"

namespace {

// The recv-buffer prefix a connection will have when the accumulating queue is staged: what it
// holds now, plus — while the queue in flight still has reads of it — at most those bytes (its
// delivery leaves their unconsumed tail in recv_buffer).  Accounting with the current size alone
// let a queue outgrow the device layout once a flush had cut a frame in two (the async live shape
// then fell back to the host decoder for 3-6 of 20 flushes, r03p47).
uint64_t prefix_bound(const uvhttp_ws_amd_batcher_t* b, const uvhttp_ws_connection_t* conn) {
    uint64_t pos = conn->recv_buffer_pos;
    const BatchQueue& other = b->q[b->cur ^ 1];
    if (other.in_flight) {
        const auto it = other.slot_of.find(const_cast<uvhttp_ws_connection_t*>(conn));
        if (it != other.slot_of.end()) pos += other.slots[it->second].bytes;
    }
    return pos;
}

// The device layout a fresh slot of conn reserves in a queue: its recv-buffer prefix (aligned)
// + 16, and room for a TLS connection's carried incomplete record
uint64_t slot_prefix(const uvhttp_ws_amd_batcher_t* b, const uvhttp_ws_connection_t* conn, bool tls) {
    return align16(prefix_bound(b, conn)) + 16 + (tls ? kTlsCarryMax : 0);
}

// Bytes a read of conn may have in the accumulating queue without handing it over (0: none)
uint64_t read_room(const uvhttp_ws_amd_batcher_t* b, uvhttp_ws_connection_t* conn, bool tls) {
    const BatchQueue& q = b->q[b->cur];
    const bool fresh = q.slot_of.find(conn) == q.slot_of.end();
    const uint64_t used = q.staged + (fresh ? slot_prefix(b, conn, tls) : 0);
    if (used >= b->cfg.max_bytes || q.reads.size() + 1 > b->cfg.max_reads ||
        (fresh && q.slots.size() + 1 > b->cfg.max_connections))
        return 0;
    return b->cfg.max_bytes - used;
}

// Make room in the accumulating queue for a read of `len` bytes of conn: a full queue is handed
// to the decoder first.  0: it fits now; 1: it is larger than a whole flush (the queue before it
// was handed over and, if it held reads of conn, delivered); -1: refused (inside a callback, where
// no flush can run, or conn failed / was handed back meanwhile).
int make_room(uvhttp_ws_amd_batcher_t* b, uvhttp_ws_connection_t* conn, uint64_t len, bool tls) {
    if (read_room(b, conn, tls) >= len) return 0;
    // the queue is full: hand it to the decoder first (not from inside a callback, where
    // the flush being delivered cannot be finished: the read is refused there)
    if (b->delivering) return -1;
    Blocked bl{b};
    (void)start_flush(b, true);  // (a device error there was decoded on the host and counted)
    if (b->failed.count(conn)) return -1;
    if (tls && !b->tls.count(conn)) return -1;  // handed back
    if (slot_prefix(b, conn, tls) + len > b->cfg.max_bytes && b->q[b->cur ^ 1].in_flight) {
        // too large only because the queue just handed over still holds reads of this
        // connection (prefix_bound counts them): deliver it, then the prefix is exact
        (void)finish_inflight(b, true);
        if (b->failed.count(conn)) return -1;
        if (tls && !b->tls.count(conn)) return -1;
    }
    return slot_prefix(b, conn, tls) + len > b->cfg.max_bytes ? 1 : 0;
}

// Record a read of `len` bytes already at arena offset `off` of the accumulating queue (the
// queue has room: make_room / read_room)
void record_read(uvhttp_ws_amd_batcher_t* b, uvhttp_ws_connection_t* conn, uint64_t off, uint64_t len,
                 bool tls) {
    BatchQueue* q = &b->q[b->cur];
    auto it = q->slot_of.find(conn);
    uint32_t k;
    if (it == q->slot_of.end()) {
        k = (uint32_t)q->slots.size();
        q->slots.push_back(ConnSlot{conn, {}, 0, false, tls});
        q->slot_of[conn] = k;
        q->staged += slot_prefix(b, conn, tls);
        if (tls) q->n_tls_slots++;
    } else {
        k = it->second;
    }
    if (b->eng) {
        q->arena_len = off + len;
        // a queue large enough for the device streams to HBM while it fills
        if ((q->bytes + len >= b->cfg.min_device_bytes || q->n_tls_slots) &&
            q->arena_len - q->uploaded >= kUploadPiece) {
            int prev = 0;
            (void)hipGetDevice(&prev);
            if (prev != b->cfg.device) (void)hipSetDevice(b->cfg.device);
            const auto tu = std::chrono::steady_clock::now();
            upload_tail(b, *q);
            b->st.upload_ms += ms_since(tu);
            if (prev != b->cfg.device) (void)hipSetDevice(prev);
        }
    }
    q->reads.push_back(QueuedRead{off, len});
    q->slots[k].reads.push_back((uint32_t)(q->reads.size() - 1));
    q->slots[k].bytes += len;
    q->staged += len;
    q->bytes += len;
}

// queue one read (plain bytes, or a TLS connection's ciphertext)
uvhttp_error_t queue_read(uvhttp_ws_amd_batcher_t* b, uvhttp_ws_connection_t* conn,
                          const uint8_t* data, size_t len, bool tls) {
    // any other queueing call between alloc_read and commit_read voids the allocation: this read
    // would take the arena bytes the socket read is landing in
    b->pend.conn = nullptr;
    if (b->failed.count(conn)) return UVHTTP_ERROR_INVALID_PARAM;
    {
        const BatchQueue& q = b->q[b->cur];
        auto it = q.slot_of.find(conn);
        if (it != q.slot_of.end() && q.slots[it->second].tls != tls) return UVHTTP_ERROR_INVALID_PARAM;
    }
    const int room = make_room(b, conn, len, tls);
    if (room < 0) return UVHTTP_ERROR_INVALID_PARAM;
    if (room == 1) {
        if (tls) {
            // ciphertext can be cut anywhere (records reassemble across flushes): queue it
            // in halves of a flush
            const size_t piece = (size_t)(b->cfg.max_bytes / 2);
            if (piece == 0 || slot_prefix(b, conn, true) + piece > b->cfg.max_bytes)
                return UVHTTP_ERROR_INVALID_PARAM;
            for (size_t o = 0; o < len; o += piece) {
                const uvhttp_error_t rc = queue_read(b, conn, data + o, len - o < piece ? len - o : piece, true);
                if (rc != UVHTTP_OK) return rc;
            }
            return UVHTTP_OK;
        }
        // larger than a whole flush: every earlier read of the connection must be
        // delivered first, then the read is decoded here (nothing of it is queued)
        (void)finish_inflight(b, true);
        if (b->failed.count(conn)) return UVHTTP_ERROR_INVALID_PARAM;
        const uvhttp_error_t rc = uvhttp_ws_process_data(conn, data, len);
        b->st.host_reads++;
        b->st.direct_reads++;
        if (rc != UVHTTP_OK) b->failed.insert(conn);
        return rc;
    }
    BatchQueue* q = &b->q[b->cur];
    uint64_t off;
    if (!b->eng) {
        off = q->arena.size();
        q->arena.insert(q->arena.end(), data, data + len);
    } else {
        off = q->arena_len;
        if (off + len > b->wire_cap) return UVHTTP_ERROR_INVALID_PARAM;  // (cannot happen)
        const auto tc = std::chrono::steady_clock::now();
        if (len) uvhttp_ws_amd_copy_stream(q->h_arena + off, data, len);
        b->st.copy_ms += ms_since(tc);
    }
    record_read(b, conn, off, len, tls);
    return UVHTTP_OK;
}

}  // namespace

extern "C" {

uvhttp_error_t uvhttp_ws_amd_batcher_submit_read(uvhttp_ws_amd_batcher_t* b,
                                                 struct uvhttp_ws_connection* conn,
                                                 const uint8_t* data, size_t len) {
    if (!b || !conn || (!data && len)) return UVHTTP_ERROR_INVALID_PARAM;
    if (b->tls.count(conn)) return UVHTTP_ERROR_INVALID_PARAM;  // a TLS connection's reads are ciphertext
    return queue_read(b, conn, data, len, false);
}

uvhttp_error_t uvhttp_ws_amd_batcher_alloc_read(uvhttp_ws_amd_batcher_t* b,
                                                struct uvhttp_ws_connection* conn, size_t suggested,
                                                uint8_t** buf, size_t* len) {
    if (!b || !conn || !buf || !len) return UVHTTP_ERROR_INVALID_PARAM;
    *buf = nullptr;
    *len = 0;
    b->pend.conn = nullptr;  // (an allocation never committed is dropped)
    if (b->failed.count(conn)) return UVHTTP_ERROR_INVALID_PARAM;
    const bool tls = b->tls.count(conn) != 0;
    {
        const BatchQueue& q = b->q[b->cur];
        auto it = q.slot_of.find(conn);
        if (it != q.slot_of.end() && q.slots[it->second].tls != tls) return UVHTTP_ERROR_INVALID_PARAM;
    }
    uint64_t want = suggested ? suggested : 65536;
    uint64_t room = read_room(b, conn, tls);
    if (room == 0) {
        // only a queue with no room left is handed over (libuv always suggests 64 KiB: a
        // queue with some room hands out that room instead of waiting for the queue in flight,
        // and the socket delivers the rest to the next read)
        if (make_room(b, conn, want, tls) < 0) return UVHTTP_ERROR_INVALID_PARAM;
        room = read_room(b, conn, tls);
        if (room == 0) {
            // not even one byte fits a flush beside the connection's recv-buffer prefix: the
            // read is decoded at commit, after the connection's earlier reads (submit_read's
            // direct path; make_room delivered them if they were in flight).  The buffer is
            // bounded whatever the caller suggests, and an allocation failure is an error code,
            // not an exception through the C ABI.
            if (tls) return UVHTTP_ERROR_INVALID_PARAM;
            const uint64_t bound = b->cfg.max_bytes > 65536 ? b->cfg.max_bytes : 65536;
            if (want > bound) want = bound;
            try {
                b->direct.resize(want);
            } catch (...) {
                return UVHTTP_ERROR_INVALID_PARAM;
            }
            b->pend.conn = conn;
            b->pend.cap = want;
            b->pend.tls = false;
            b->pend.direct = true;
            *buf = b->direct.data();
            *len = (size_t)want;
            return UVHTTP_OK;
        }
    }
    if (room < want) want = room;
    BatchQueue& q = b->q[b->cur];
    uint64_t off;
    uint8_t* base;
    if (!b->eng) {
        off = q.arena.size();
        q.arena.resize(off + want);  // (no fill: the read writes it)
        base = q.arena.data();
    } else {
        off = q.arena_len;
        if (off + want > b->wire_cap) return UVHTTP_ERROR_INVALID_PARAM;  // (cannot happen)
        base = q.h_arena;
    }
    b->pend.conn = conn;
    b->pend.qi = b->cur;
    b->pend.gen = q.gen;
    b->pend.off = off;
    b->pend.cap = want;
    b->pend.tls = tls;
    b->pend.direct = false;
    *buf = base + off;
    *len = (size_t)want;
    return UVHTTP_OK;
}

uvhttp_error_t uvhttp_ws_amd_batcher_commit_read(uvhttp_ws_amd_batcher_t* b,
                                                 struct uvhttp_ws_connection* conn, size_t nread) {
    if (!b || !conn) return UVHTTP_ERROR_INVALID_PARAM;
    const auto p = b->pend;
    b->pend.conn = nullptr;
    if (p.conn != conn || nread > p.cap) return UVHTTP_ERROR_INVALID_PARAM;
    if (p.direct) {
        if (nread == 0) return UVHTTP_OK;
        if (b->delivering) return UVHTTP_ERROR_INVALID_PARAM;  // (alloc_read refused there already)
        (void)finish_inflight(b, true);
        if (b->failed.count(conn)) return UVHTTP_ERROR_INVALID_PARAM;
        const uvhttp_error_t rc = uvhttp_ws_process_data(conn, b->direct.data(), nread);
        b->st.host_reads++;
        b->st.direct_reads++;
        b->st.zero_copy_reads++;
        if (rc != UVHTTP_OK) b->failed.insert(conn);
        return rc;
    }
    // the allocation must be in the queue still accumulating (no flush since)
    if (p.qi != b->cur || b->q[p.qi].gen != p.gen) return UVHTTP_ERROR_INVALID_PARAM;
    BatchQueue& q = b->q[b->cur];
    if (!b->eng) q.arena.resize(p.off + nread);
    if (nread == 0) return UVHTTP_OK;  // nothing read (EAGAIN, or EOF / an error the caller handles)
    if (b->failed.count(conn)) return UVHTTP_ERROR_INVALID_PARAM;  // (forgotten meanwhile: cannot happen)
    record_read(b, conn, p.off, nread, p.tls);
    b->st.zero_copy_reads++;
    return UVHTTP_OK;
}

int uvhttp_ws_amd_batcher_set_tls(uvhttp_ws_amd_batcher_t* b, struct uvhttp_ws_connection* conn,
                                  const void* tls_key, uint64_t read_seq) {
    if (!b || !conn || !tls_key) return UVHTTP_WS_GPU_EINVAL;
    b->pend.conn = nullptr;  // (an outstanding alloc_read is void: commit_read refuses it)
    if (!b->eng) return UVHTTP_WS_GPU_ENODEV;  // no host AEAD: TLS needs the device
    // plain reads of this connection still queued would be decoded after ciphertext that
    // follows them: flush them first
    for (int i = 0; i < 2; ++i) {
        auto it = b->q[i].slot_of.find(conn);
        if (it != b->q[i].slot_of.end() && !b->q[i].slots[it->second].tls) {
            // (inside a batcher callback no flush can run: refuse rather than register a TLS
            // connection whose queued plain reads would then be unreachable)
            if (b->delivering) return UVHTTP_WS_GPU_EINVAL;
            Blocked bl{b};
            (void)start_flush(b, true);
            (void)finish_inflight(b, true);
            break;
        }
    }
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != b->cfg.device) (void)hipSetDevice(b->cfg.device);
    bool ok = true;
    if (!b->teng) ok = uvhttp_tls_gpu_engine_create(b->cfg.device, &b->teng) == UVHTTP_TLS_GPU_OK;
    if (ok) ok = alloc_tls(b, b->q[0]) && alloc_tls(b, b->q[1]);
    if (prev != b->cfg.device) (void)hipSetDevice(prev);
    if (!ok) return UVHTTP_WS_GPU_ENOMEM;
    TlsConn& t = b->tls[conn];
    memcpy(&t.key, tls_key, sizeof(t.key));
    t.seq = read_seq;
    t.carry.clear();
    return UVHTTP_WS_GPU_OK;
}

uvhttp_error_t uvhttp_ws_amd_batcher_submit_tls_read(uvhttp_ws_amd_batcher_t* b,
                                                     struct uvhttp_ws_connection* conn,
                                                     const uint8_t* ciphertext, size_t len) {
    if (!b || !conn || (!ciphertext && len)) return UVHTTP_ERROR_INVALID_PARAM;
    if (!b->tls.count(conn)) return UVHTTP_ERROR_INVALID_PARAM;  // not (or no longer) TLS here
    return queue_read(b, conn, ciphertext, len, true);
}

void uvhttp_ws_amd_batcher_forget(uvhttp_ws_amd_batcher_t* b, struct uvhttp_ws_connection* conn) {
    if (!b || !conn) return;
    b->pend.conn = nullptr;  // an uncommitted allocation (of any connection) is void
    b->failed.erase(conn);
    b->tls.erase(conn);
    for (int i = 0; i < 2; ++i) {
        BatchQueue& q = b->q[i];
        auto it = q.slot_of.find(conn);
        if (it == q.slot_of.end()) continue;
        q.slots[it->second].dropped = true;  // a delivery in progress skips it
        // (a new connection at this address gets a new slot; the old slot's reads stay in
        // the arena, unreferenced)
        if (i == b->cur) q.slot_of.erase(it);
    }
}

// library-internal (the batcher group): 1 while the batcher holds anything of `conn` — reads
// queued or in flight, a failure mark, TLS state — so the group may move it to another member
__attribute__((visibility("hidden"))) int uvhttp_ws_amd_batcher_holds_conn(
    const uvhttp_ws_amd_batcher_t* b, const uvhttp_ws_connection_t* conn) {
    uvhttp_ws_connection_t* c = const_cast<uvhttp_ws_connection_t*>(conn);
    if (b->failed.count(c) || b->tls.count(c)) return 1;
    for (int i = 0; i < 2; ++i) {
        const BatchQueue& q = b->q[i];
        auto it = q.slot_of.find(c);
        if (it != q.slot_of.end() && !q.slots[it->second].dropped) return 1;
    }
    return 0;
}

int uvhttp_ws_amd_batcher_numa_node(const uvhttp_ws_amd_batcher_t* b) {
    if (!b || !b->eng) return -1;
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, b->cfg.device) != hipSuccess) return -1;
    for (char* c = bus; *c; ++c)
        if (*c >= 'A' && *c <= 'F') *c = (char)(*c - 'A' + 'a');  // sysfs spells hex in lower case
    char path[160];
    snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
    FILE* f = fopen(path, "r");
    if (!f) return -1;
    int node = -1;
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
    return node;
}

void uvhttp_ws_amd_batcher_reset_stats(uvhttp_ws_amd_batcher_t* b) {
    if (!b) return;
    memset(&b->st, 0, sizeof(b->st));
    b->blocked.clear();
    b->blocked_n = 0;
}

int uvhttp_ws_amd_batcher_stats(const uvhttp_ws_amd_batcher_t* b,
                                uvhttp_ws_amd_batcher_stats_t* out) {
    if (!b || !out) return UVHTTP_WS_GPU_EINVAL;
    *out = b->st;
    if (!b->blocked.empty()) {
        std::vector<float> v(b->blocked);
        const size_t i50 = (v.size() - 1) / 2, i99 = (v.size() - 1) * 99 / 100;
        std::nth_element(v.begin(), v.begin() + i50, v.end());
        out->blocked_p50_ms = v[i50];
        std::nth_element(v.begin(), v.begin() + i99, v.end());
        out->blocked_p99_ms = v[i99];
    }
    return UVHTTP_WS_GPU_OK;
}

}  // extern "C"
