// ws_gpu.hip — MI355X (gfx950) batched WebSocket frame decode + payload unmask.
//
// Replaces, for frames already resident in HBM, the per-frame work of
// src/uvhttp_websocket.c (adam-ikari/uvhttp v2.7.0):
//   uvhttp_ws_parse_frame_header  :133-185   -> parse_one (one lane per frame)
//   validation in process_data    :851-932   -> parse_one (local) + resolve_one (state machine)
//   fragment state machine        :950-1015  -> resolve_one (segmented scan, no serial walk)
//   uvhttp_ws_fragment_append     :781-822   -> prefix offsets + k_gather_compact
//   uvhttp_ws_apply_mask          :188-197   -> k_unmask_inplace / k_gather_compact
//
// Pipeline per decode call (one stream, no host sync, two launches):
//   k_plan     frames -> desc[] (header, key, status), single-pass decoupled look-back scan,
//              state machine, message ids, arena offsets, first failure, tile -> first-frame
//              maps; its last block writes the batch summary
//   k_unmask_inplace / k_gather_compact   the HBM-bound payload pass (the roofline kernel);
//              its first lanes also mark frames after the first failure SKIPPED
//
// The payload pass is pure streaming integer work: 16-byte loads/stores per lane, the
// 4-byte key rotated once per (vector, frame) into a 32-bit word, no LDS on the fast path,
// no MFMA (nothing here is matrix-shaped).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "uvhttp_ws_amd.h"

namespace {

constexpr int kBlock = 256;                 // threads per workgroup (4 waves of 64)
constexpr uint64_t kMapTile = 16384;        // granularity of the tile -> first-frame maps
// compact decode: wire-driven (k_scatter_compact) below this average frame size, arena-driven
// gather above.  (Same-process A/B, scatter vs gather: 16 KiB frames 97.0 vs 102.2 us per
// 256 MiB step, 24 KiB 96.8 vs 102.8, 32 KiB 109.8 vs 101.2, 64 KiB 1775 vs 1338 per 4 GiB;
// profiles/r06zd_*, r06ze_*.  16 KiB until round 6.)
constexpr uint64_t kScatterAvg = 26624;
constexpr uint32_t kMaxFrames = 1u << 26;   // k_scan handles <= 2^18 block aggregates
constexpr uint32_t kNoFrame = 0xFFFFFFFFu;  // tile map entry no frame claimed this call
constexpr uint32_t kMaxEpoch = (1u << 30) - 1;  // decode-call tags run 1 .. kMaxEpoch

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------
// scan element: everything the fragment state machine needs about frames [0, i)
// ------------------------------------------------------------------------------------
struct ScanElem {
    int32_t last_data;   // max: index of the latest data frame (-1 none)
    int32_t last_start;  // max: index of the latest non-CONT data frame (-1 none)
    uint64_t data_pay;   // sum: payload bytes of data frames (arena offset)
    uint64_t all_pay;    // sum: payload bytes of all frames
    uint64_t seg_pay;    // segmented sum: data payload since the latest start
    uint32_t n_fin;      // sum: data frames with FIN (completed messages)
    uint32_t n_close;    // sum: CLOSE frames
    uint32_t bits;       // kSegFlag | kHead | kLastOpen | start opcode << 4
};
// bits: the segment contains a start; a connection starts here (the scan restarts); the
// latest data frame leaves a message open (FIN=0 and not a zero-length start, whose empty
// first fragment allocates nothing: src/uvhttp_websocket.c:794-816 + :964); the opcode of
// the latest start (the message's opcode)
constexpr uint32_t kSegFlag = 1u, kHead = 2u, kLastOpen = 4u, kOpShift = 4u, kOpMask = 0xF0u;

__device__ __host__ inline ScanElem scan_identity() {
    ScanElem e;
    e.last_data = -1;
    e.last_start = -1;
    e.data_pay = 0;
    e.all_pay = 0;
    e.seg_pay = 0;
    e.n_fin = 0;
    e.n_close = 0;
    e.bits = 0;
    return e;
}

// segmented: a connection start in b discards everything before it
__device__ __host__ inline ScanElem scan_combine(const ScanElem& a, const ScanElem& b) {
    if (b.bits & kHead) return b;
    ScanElem r;
    r.last_data = a.last_data > b.last_data ? a.last_data : b.last_data;
    r.last_start = a.last_start > b.last_start ? a.last_start : b.last_start;
    r.data_pay = a.data_pay + b.data_pay;
    r.all_pay = a.all_pay + b.all_pay;
    r.seg_pay = (b.bits & kSegFlag) ? b.seg_pay : a.seg_pay + b.seg_pay;
    r.n_fin = a.n_fin + b.n_fin;
    r.n_close = a.n_close + b.n_close;
    const uint32_t open = (b.last_data >= 0 ? b.bits : a.bits) & kLastOpen;
    const uint32_t op = (b.last_start >= 0 ? b.bits : a.bits) & kOpMask;
    r.bits = ((a.bits | b.bits) & kSegFlag) | (a.bits & kHead) | open | op;
    return r;
}

__device__ inline bool is_data_op(uint32_t op) { return op <= 2u; }

// element of frame i, rebuilt from its descriptor (local status must be OK for the
// state machine to consider it; invalid frames never precede a delivered frame)
__device__ inline ScanElem scan_elem_of(const uvhttp_ws_frame_desc_t& d, int32_t i, bool head) {
    ScanElem e = scan_identity();
    const uint32_t op = d.opcode;
    const bool fin = d.flags & UVHTTP_WS_FLAG_FIN;
    e.all_pay = d.payload_len;
    if (is_data_op(op)) {
        e.last_data = i;
        e.data_pay = d.payload_len;
        e.seg_pay = d.payload_len;
        if (op != 0) {
            e.last_start = i;
            e.bits |= kSegFlag | (op << kOpShift);
        }
        if (!fin && !(op != 0 && d.payload_len == 0)) e.bits |= kLastOpen;
        e.n_fin = fin ? 1u : 0u;
    } else if (op == 8) {
        e.n_close = 1;
    }
    if (head) e.bits |= kHead;
    return e;
}

__device__ inline ScanElem shfl_up_elem(const ScanElem& e, int delta) {
    ScanElem r;
    r.last_data = __shfl_up(e.last_data, delta, 64);
    r.last_start = __shfl_up(e.last_start, delta, 64);
    r.data_pay = __shfl_up(e.data_pay, delta, 64);
    r.all_pay = __shfl_up(e.all_pay, delta, 64);
    r.seg_pay = __shfl_up(e.seg_pay, delta, 64);
    r.n_fin = __shfl_up(e.n_fin, delta, 64);
    r.n_close = __shfl_up(e.n_close, delta, 64);
    r.bits = __shfl_up(e.bits, delta, 64);
    return r;
}

__device__ inline ScanElem shfl_down_elem(const ScanElem& e, int delta) {
    ScanElem r;
    r.last_data = __shfl_down(e.last_data, delta, 64);
    r.last_start = __shfl_down(e.last_start, delta, 64);
    r.data_pay = __shfl_down(e.data_pay, delta, 64);
    r.all_pay = __shfl_down(e.all_pay, delta, 64);
    r.seg_pay = __shfl_down(e.seg_pay, delta, 64);
    r.n_fin = __shfl_down(e.n_fin, delta, 64);
    r.n_close = __shfl_down(e.n_close, delta, 64);
    r.bits = __shfl_down(e.bits, delta, 64);
    return r;
}

// One DPP move of every word of a scan element: lanes the pattern gives no source (or whose
// row the row mask leaves out) get the identity, which scan_combine(identity, x) ignores.
// DPP moves are VALU operations: no LDS round trip per word as with ds_bpermute (__shfl_up).
template <int CTRL, int RMASK>
__device__ inline ScanElem dpp_elem(const ScanElem& e) {
    auto mv = [](uint32_t old, uint32_t x) -> uint32_t {
        return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, RMASK, 0xF, false);
    };
    auto mv64 = [&](uint64_t x) -> uint64_t {
        return (uint64_t)mv(0u, (uint32_t)x) | ((uint64_t)mv(0u, (uint32_t)(x >> 32)) << 32);
    };
    ScanElem r;
    r.last_data = (int32_t)mv(0xFFFFFFFFu, (uint32_t)e.last_data);
    r.last_start = (int32_t)mv(0xFFFFFFFFu, (uint32_t)e.last_start);
    r.data_pay = mv64(e.data_pay);
    r.all_pay = mv64(e.all_pay);
    r.seg_pay = mv64(e.seg_pay);
    r.n_fin = mv(0u, e.n_fin);
    r.n_close = mv(0u, e.n_close);
    r.bits = mv(0u, e.bits);
    return r;
}

// inclusive wave scan (lane i ends with v[0] (+) ... (+) v[i]): within rows of 16 by row_shr
// 1, 2, 4, 8, then across rows by row_bcast:15 (rows 1 and 3 take the row before's total) and
// row_bcast:31 (rows 2 and 3 take rows 0-1's)
__device__ inline ScanElem wave_inclusive_scan(ScanElem v) {
    v = scan_combine(dpp_elem<0x111, 0xF>(v), v);
    v = scan_combine(dpp_elem<0x112, 0xF>(v), v);
    v = scan_combine(dpp_elem<0x114, 0xF>(v), v);
    v = scan_combine(dpp_elem<0x118, 0xF>(v), v);
    v = scan_combine(dpp_elem<0x142, 0xA>(v), v);
    v = scan_combine(dpp_elem<0x143, 0xC>(v), v);
    return v;
}

// ordered wave reduction: lane 0 ends with v[63] (+) ... (+) v[0] — lane 63 is the OLDEST
__device__ inline ScanElem wave_reduce_newest_first(ScanElem v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const ScanElem o = shfl_down_elem(v, d);
        if (lane + d < 64) v = scan_combine(o, v);
    }
    return v;
}

// Block-wide exclusive scan (NT threads = NT / 64 waves): wave-level Hillis-Steele over the
// 64 lanes with __shfl_up, then the wave totals through LDS.  Returns the exclusive prefix
// for this thread; *total receives the block aggregate.
template <int NT = kBlock>
__device__ ScanElem block_exclusive_scan(ScanElem v, ScanElem* total) {
    __shared__ ScanElem wave_tot[NT / 64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
#ifdef UVWS_SCAN_BPERMUTE
    ScanElem inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        ScanElem o = shfl_up_elem(inc, d);
        if (lane >= d) inc = scan_combine(o, inc);
    }
#else
    const ScanElem inc = wave_inclusive_scan(v);
#endif
    if (lane == 63) wave_tot[wave] = inc;
    __syncthreads();
    ScanElem wave_pre = scan_identity();
    ScanElem all = scan_identity();
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        if (w < wave) wave_pre = scan_combine(wave_pre, wave_tot[w]);
        all = scan_combine(all, wave_tot[w]);
    }
    ScanElem exc = shfl_up_elem(inc, 1);
    if (lane == 0) exc = scan_identity();
    __syncthreads();
    *total = all;
    return scan_combine(wave_pre, exc);
}

// ------------------------------------------------------------------------------------
// workspace layout (device), carved from one allocation
// ------------------------------------------------------------------------------------
struct alignas(16) LbRec {
    uint32_t w[16];
};

struct Workspace {
    ScanElem* block_agg;   // [n_blocks]: k_plan block aggregates (build: u64 block sums)
    ScanElem* group_agg;   // build only: u64 group sums
    ScanElem* block_incl;  // [n_blocks]: k_plan inclusive prefixes (look-back "P" values)
    ScanElem* block_excl;  // [n_blocks]: k_plan exclusive prefixes (summary)
    LbRec* rec_a;          // [n_blocks]: look-back aggregate records
    LbRec* rec_p;          // [n_blocks]: look-back inclusive-prefix records
    uint32_t* counters;    // [0] block ticket, [1] blocks done; reset by the last block
    uint64_t* tile_first;  // [n_tiles]: tagged first frame whose slot contains the tile start
    uint64_t* first_bad;   // [1]: tagged first failing frame of the batch
    uint64_t* spec_bad;    // [1]: tagged first delivered frame the speculative compact pass
                           // did not place (its arena offset or layout is not the uniform one)
    uint64_t* arena_first; // [n_arena_tiles]: tagged first data frame of the arena tile
    uint32_t* ctl;         // control words outside the clearable workspace (see kCtl*)
    void* recs;            // [n_frames] FrameRec8: the payload passes' records, or info bytes
    void* parts;           // [n_frames / 1024 + 2] TilePart: per k_sum_scan block (4 frames a thread)
    uint8_t* info;         // [n_frames + 64]: info bytes beside the records (k_desc_emit's decode)
};

// ctl words (their own allocation, never cleared with the workspace)
constexpr int kCtlEpoch = 0;     // device epoch of graph-captured calls
constexpr int kCtlDone = 1;      // k_epoch's last-block counter
constexpr int kCtlFaultEp = 2;   // epoch of the latest call whose look-back gave up
constexpr int kCtlFaults = 3;    // running count of such calls (engine_sync compares it)
constexpr int kCtlGate = 4;      // epoch of the latest summary-only compact call whose speculation
                                 // failed (its k_plan + k_spec_fix then run, k_sum_msgs does not)
// speculative stream decode (k_sspec_*): epoch of the latest call whose connections k_sspec_plan
// (or the capacity check in k_sspec_tiles) found ineligible — the walk decodes it — and of the
// latest whose speculation a later kernel broke (undone, then the walk)
constexpr int kCtlSpecOff = 5;
constexpr int kCtlSpecBreak = 6;
constexpr int kCtlWords = 7;
// epochs: host-issued tags run 1 .. kMaxHostEpoch, device-issued ones (captured calls)
// kMaxHostEpoch + 1 .. kMaxEpoch, so a replayed graph never meets a tag a host call left
constexpr uint32_t kMaxHostEpoch = kMaxEpoch / 2;

// Epoch tags.  Every decode call gets a fresh 32-bit epoch; map entries and first_bad are
// stored as (epoch << 32) | ~frame and claimed with atomicMax, so within a call the smallest
// frame wins and entries left by earlier calls read as "unclaimed" — no reset pass.
__device__ inline uint64_t tag_of(uint32_t epoch, uint32_t frame) {
    return ((uint64_t)epoch << 32) | (uint32_t)~frame;
}
// A host call after graph replays meets entries the replays tagged with their (larger, device)
// epochs, which a max never displaces: on an engine that has captured calls (cas: BatchArgs /
// WalkArgs cas_claims) such an entry is replaced by compare-and-swap, then this call's claims
// order by max again — one returning atomicMax in the common case.  Engines that never captured
// a call cannot meet one and keep the fire-and-forget atomicMax.
__device__ inline void tag_claim(uint64_t* p, uint32_t epoch, uint32_t frame, uint32_t cas) {
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    const unsigned long long mine = tag_of(epoch, frame);
    if (!cas) {
        atomicMax(q, mine);
        return;
    }
    unsigned long long cur = atomicMax(q, mine);
    while ((uint32_t)(cur >> 32) > epoch) {  // a later epoch's entry
        const unsigned long long seen = atomicCAS(q, cur, mine);
        if (seen == cur) return;
        cur = seen;
        if ((uint32_t)(cur >> 32) <= epoch) {  // another claim of this call replaced it first
            atomicMax(q, mine);
            return;
        }
    }
}
__device__ inline uint32_t tag_get(uint64_t v, uint32_t epoch, uint32_t none) {
    return (uint32_t)(v >> 32) == epoch ? ~(uint32_t)v : none;
}

// k_swalk_fused runs for the wave walk only (at most 16 384 connections, 4 per block)
constexpr uint32_t kSwalkFusedMaxBlocks = 16384 / 4;

// extra scratch of the stream decode (one allocation per engine, grown on demand)
struct StreamScratch {
    uint64_t* frame_off;   // [max_frames] two-pass walk: frame starts
    uint32_t* n_total;     // [1] frames found (0 on capacity overflow)
    uint64_t* read_size;   // [n_reads_total] recv-buffer size after each call
    uint32_t* walk_tmp;    // single pass: per-connection slices of 32-bit frame starts
    uint2* walk_rec;       // single pass, wave walk (or null): per start, the frame's key and
                           // header bytes when the walk's fast path parsed them (kNoRec: not)
    uint32_t* agg;         // [n_streams / 256 + 1] lane walk block counts -> prefixes
    uint32_t* ctr;         // [4] k_swalk_fused: [0] block ticket, [1] connections done (both
                           // reset by their last taker), [2] epoch of a call over capacity
    void* srec;            // [2 kSwalkFusedMaxBlocks] k_swalk_fused look-back records (A, P per block)
};

// parse_hdr's result for one frame, 16 bytes: the in-register form of a frame record (the
// payload passes store it packed, FrameRec8 below; k_plan, k_fixup, the scans and the
// descriptor passes read those instead of the headers).  flags bit 7 (kRecHasLen): the header
// parsed to a wire length (then payload_off / wire_len follow from header_size and the mask).
struct alignas(16) FrameRec {
    uint64_t payload_len;
    uint32_t masking_key;
    uint8_t opcode, flags, header_size;
    int8_t status;  // before the state machine
};
static_assert(sizeof(FrameRec) == 16, "one 16-byte load per record");
constexpr uint8_t kRecHasLen = 0x80;

// What the payload passes actually write per frame: 8 bytes — the masking key and one packed
// word — for a frame that parsed OK to a wire length with a payload under 2^23 bytes (every
// delivered frame of a fused stride batch or of a speculated connection).  Any other frame is
// written as kR8Esc and its reader parses the header from the wire again (rec_at: stride
// batches leave headers untouched; the speculative stream decode never reads one — such a
// frame breaks the speculation).  Packed word: payload_len [0, 23), opcode [23, 27), FIN [27],
// MASK [28], header-size code [29, 31) (hs >> 2: 2 / 4 / 10 bytes), kR8Esc [31].  (16-byte
// records cost C4 in place 50 MB of its 643 MB step traffic — written by the pass, read by the
// scan and the descriptor pass; 8-byte ones: whole-step traffic 1.181 -> 1.135 x in place,
// 1.150 -> 1.119 compact, 1.163 -> 1.132 streams, step times within 1 % either way,
// profiles/r06x7_*, traffic_c4_*.json.  A 16-byte side record stored by the pass for escaped
// frames — one conditional store in the parse loop — cost the speculative stream pass 11 us
// on C4: profiles/r06x5_*, r06x_*.)
struct alignas(8) FrameRec8 {
    uint32_t key;
    uint32_t w;
};
static_assert(sizeof(FrameRec8) == 8, "one 8-byte load per record");
constexpr uint32_t kR8Esc = 1u << 31, kR8LenBits = 23;

__device__ inline FrameRec8 rec8_pack(const FrameRec& r) {
    const bool simple = r.status == UVHTTP_WS_FRAME_OK && (r.flags & kRecHasLen) &&
                        !(r.flags & ~(kRecHasLen | UVHTTP_WS_FLAG_FIN | UVHTTP_WS_FLAG_MASK)) &&
                        r.payload_len < (1ull << kR8LenBits) && r.opcode < 16 &&
                        (r.header_size == 2 || r.header_size == 4 || r.header_size == 10);
    FrameRec8 p;
    p.key = r.masking_key;
    p.w = simple ? ((uint32_t)r.payload_len | ((uint32_t)r.opcode << 23) | ((uint32_t)(r.flags & 3u) << 27) |
                    ((uint32_t)(r.header_size >> 2) << 29))
                 : kR8Esc;
    return p;
}

// a simple record's fields (false: escaped, the caller re-parses the header)
__device__ inline bool rec8_unpack(const FrameRec8& p, FrameRec& r) {
    r.payload_len = p.w & ((1u << kR8LenBits) - 1);
    r.masking_key = p.key;
    r.opcode = (uint8_t)((p.w >> 23) & 0xF);
    r.flags = (uint8_t)(kRecHasLen | ((p.w >> 27) & 3u));
    const uint32_t hc = (p.w >> 29) & 3u;
    r.header_size = (uint8_t)(hc == 0 ? 2 : hc == 1 ? 4 : 10);
    r.status = UVHTTP_WS_FRAME_OK;
    return !(p.w & kR8Esc);
}

__device__ inline void rec8_store(FrameRec8* r8, uint32_t i, const FrameRec& r) { r8[i] = rec8_pack(r); }

// Summary-only decode (uvhttp_ws_gpu_decode_inplace with d_desc == NULL, stride batches): what
// the batch summary needs from a run of consecutive frames, in frame order, up to the run's
// first failure — one per k_sum_scan block, combined by k_sum_tail.
struct alignas(16) TilePart {
    uint64_t pay;   // payload bytes of the frames (src/uvhttp_websocket.c: all delivered frames)
    uint64_t seg;   // data payload since the latest start (all of it when the run has no start)
    uint32_t nfin;  // data frames with FIN: completed messages
    uint32_t ls;    // latest start (non-CONT data frame), kNoFrame if none
    uint32_t last;  // latest data frame, kNoFrame if none
    uint32_t bits;  // kPartOpen: `last` leaves a message open; kPartClosed: a CLOSE was delivered;
                    // kPartBin: `ls` is a BINARY start (compact: the message's opcode)
    uint32_t ff;    // the run's first failing frame (the run stops before it), kNoFrame if none
    uint32_t pad[3];
};
static_assert(sizeof(TilePart) == 48, "three 16-byte words");
constexpr uint32_t kPartOpen = 1u, kPartClosed = 2u, kPartBin = 4u;

__device__ __host__ inline TilePart part_identity() {
    TilePart p;
    p.pay = 0;
    p.seg = 0;
    p.nfin = 0;
    p.ls = kNoFrame;
    p.last = kNoFrame;
    p.bits = 0;
    p.ff = kNoFrame;
    p.pad[0] = p.pad[1] = p.pad[2] = 0;
    return p;
}


// a followed by b: a run that failed ends the combined run there
__device__ __host__ inline TilePart part_combine(const TilePart& a, const TilePart& b) {
    if (a.ff != kNoFrame) return a;
    TilePart r;
    r.ff = b.ff;
    r.pad[0] = r.pad[1] = r.pad[2] = 0;
    r.pay = a.pay + b.pay;
    r.nfin = a.nfin + b.nfin;
    r.ls = b.ls != kNoFrame ? b.ls : a.ls;
    r.seg = b.ls != kNoFrame ? b.seg : a.seg + b.seg;
    r.last = b.last != kNoFrame ? b.last : a.last;
    r.bits = ((b.last != kNoFrame ? b.bits : a.bits) & kPartOpen) | ((a.bits | b.bits) & kPartClosed) |
             ((b.ls != kNoFrame ? b.bits : a.bits) & kPartBin);
    return r;
}

struct BatchArgs {
    uint8_t* wire;
    uint64_t wire_len;
    const uint64_t* frame_off;
    uint64_t frame_stride;
    double stride_inv;        // 1 / frame_stride (stride batches: frame index by multiply)
    FrameRec8* recs;          // stride batches decoded by the fused path (else null); summary-only: info bytes
    uint32_t n;
    int32_t max_frame_size;
    int32_t max_message_size;
    int32_t is_server;
    uint64_t n_tiles;        // in-place tiles over the wire
    uint8_t* arena;          // compact mode (nullptr: in-place)
    uint64_t arena_cap;
    uint64_t n_arena_tiles;
    // stream mode (streams != nullptr; only the claims and payload kernels run): frames come
    // from the walk, n is the capacity and the real count is *n_dev; a frame is delivered iff
    // its descriptor says OK
    const uvhttp_ws_stream_t* streams;
    const uint32_t* n_dev;
    uvhttp_ws_stream_result_t* s_results;  // after k_swalk_fused: results stream_fix may rewrite
    const uint32_t* s_over;  //   (StreamScratch::ctr[2]: epoch of a call over capacity)
    uint32_t n_streams;
    uint32_t epoch;          // tag of this call's map / first_bad entries
    uint32_t dev_epoch;      // 1: a captured call, the epoch is ws.ctl[kCtlEpoch]
    uint32_t max_polls;      // look-back wait bound (0: give up at the first wait; tests)
    uvhttp_ws_batch_summary_t* summary;  // batch mode: written by k_finalize
    uint32_t plan_frames;    // frames per k_plan block (kBlock * FPT)
    uint32_t no_ticket;      // k_plan orders blocks by blockIdx (experiment: UVHTTP_WS_PLAN_TICKET=0)
    uint64_t* stamp;         // device-side kernel stamps (diagnostics), or null
    uint64_t spec_P;         // compact stride batch, speculative pass: the uniform payload length
                             // (frame i's payload at arena offset i * spec_P); 0 = none
    uint32_t gate;           // k_plan / k_spec_fix run only when ws.ctl[kCtlGate] holds this call's
                             // epoch (the summary-only compact decode's fallback)
    uint32_t cas_claims;     // the engine has captured calls: tag_claim displaces later epochs
    uvhttp_ws_message_desc_t* msgs;  // compact decode: the message table (the summary writer
                                     // adds the open message's entry at msgs[n_messages])
};

// ------------------------------------------------------------------------------------
// Device-side kernel stamps (diagnostics, uvhttp_ws_gpu_engine_set_stamps).  With stamps
// on, each kernel records when its first workgroups started and when its waves ended on the
// GPU's constant wall clock, so the gaps between the kernels of a call and between
// consecutive calls are read off the device timeline.  Plain vector stores only — atomics on
// one address from every wave of a 262 144-workgroup payload kernel serialise across the XCDs
// (a C3 kernel took 11 ms with them): the first 256 workgroups store their start into their own
// word, a sample of the waves (below) its end into one of 4096 words, so the latest of those
// words is within a few workgroups of the kernel's end.  Slots form a ring keyed by the call's
// epoch and every word is tagged (epoch << 40) | t, so the reader keeps the newest call of each
// slot without a reset.
// ------------------------------------------------------------------------------------
constexpr uint32_t kStampRing = 128, kStampKinds = 16, kStampBegin = 256, kStampEnd = 4096;
constexpr uint64_t kStampPer = kStampBegin + kStampEnd;
constexpr uint64_t kStampLow = (1ull << 40) - 1;
constexpr uint32_t kStampTagPeriod = (1u << 24) - 1;
constexpr uint64_t kStampWords = (uint64_t)kStampRing * kStampKinds * kStampPer;
// experiment builds (-DUVWS_PLAN_PHASES, tools/build_variant.sh): k_plan's per-block phase
// times follow the ring, 8 words per block (uvhttp_ws_gpu_engine_debug_phases)
constexpr uint64_t kPhaseWords = 8 * 8192;
constexpr uint64_t kStampAlloc = kStampWords + kPhaseWords;

// a stamp word's call tag: 1 .. 2^24 - 1, never 0 (0 marks an unused word), one more per call
__host__ __device__ inline uint32_t stamp_tag(uint32_t epoch) { return epoch % kStampTagPeriod + 1u; }
__device__ inline uint64_t* stamp_slot(uint64_t* st, uint32_t epoch, uint32_t kind) {
    return st + ((uint64_t)(epoch % kStampRing) * kStampKinds + kind) * kStampPer;
}
// which workgroups (by index g in the whole pass) store an end word, and which end word wave w
// of workgroup g stores (shared with the host-side simulation the stamp tests drive)
__host__ __device__ inline bool stamp_sampled(uint64_t g) {
    return g < 1024 || (g < 65536 ? (g & 63) == 63 : (g & 1023) == 1023);
}
__host__ __device__ inline uint32_t stamp_end_word(uint64_t g, uint32_t wave) {
    const uint64_t blk = g < 1024 ? g : g < 65536 ? 1024 + (g >> 6) : 2048 + (g >> 10);
    return (uint32_t)((blk * 4 + (wave & 3)) % kStampEnd);
}
// the constant-rate wall clock (100 MHz).  Inline asm without a memory clobber: the builtin
// counts as a memory access, so a clock read at a kernel's start turned every later uniform
// workspace load into a vector load (the compiler could no longer prove them unclobbered)
__device__ inline uint64_t stamp_clock() {
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
    return t;
}

// One per kernel; both words are stored when the workgroup's threads return (no store may come
// first: a global store ahead of the payload kernels' uniform workspace loads — tile map,
// first_bad, descriptors — turns them into vector loads, and so does a clock read, which the
// compiler must treat as a memory access: C3's payload kernel took 1.92 ms instead of 1.25
// with stamps off, profiles/r04_ab_stampoff2.txt).  So the kernels whose uniform loads matter
// (payload kernels, walks, descriptors: at_start = false) read no clock at their start; their
// "begin" is the earliest END among their first 256 workgroups — late by one workgroup's
// duration — unless the kernel reads it through anchor_s / anchor_v (the payload kernels, the
// walks and k_stream_desc do).  The others (k_plan, scans, fix-ups) read the clock when they start.
//
// A pass too large for one dispatch packet is launched as pieces of <= 2^24 workgroups
// (run_decode, build_frames); each piece passes its first workgroup's index in the whole pass
// (`base`, the tile_base argument), and the words are placed by that global index, so only
// the first piece stores begins and every piece's ends land in the same slot: the reader's
// earliest begin / latest end then span the whole pass (blockIdx.x alone restarted in every
// piece, and the slot kept the last piece: a C5 pass read as 6.7 us).
struct StampScope {
    uint64_t* st;
    uint32_t epoch, kind;
    uint64_t t0;
    uint64_t base;
    __device__ StampScope(uint64_t* st_, uint32_t epoch_, uint32_t kind_, bool at_start = true,
                          uint64_t base_ = 0)
        : st(st_), epoch(epoch_), kind(kind_), t0(at_start && st_ ? stamp_clock() : 0), base(base_) {}
    // The start clock of a kernel whose uniform loads must stay scalar: read by an asm that is
    // not a memory access (so it clobbers nothing) and is pinned before the kernel's first
    // loads by passing the index they are computed from through it (v is returned unchanged).
    __device__ uint32_t anchor_s(uint32_t v) {
        uint64_t t;
        asm("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t), "+s"(v));
        t0 = t;
        return v;
    }
    __device__ uint32_t anchor_v(uint32_t v) {
        uint64_t t;
        asm("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t), "+v"(v));
        t0 = t;
        return v;
    }
    // runs at every return of the kernel: thread 0 of the first workgroups stores the start,
    // the first active lane of each wave its end
    __device__ ~StampScope() {
        if (!st) return;
        // ends: every wave of the first 1024 workgroups (all of them in the walk, plan and scan
        // launches), then one workgroup in 64 up to workgroup 65 536 and one in 1024 past it —
        // the last of those to finish ends within 64 (1024) workgroups' time of the kernel.
        // Each end store costs: one in 64 of a C3 payload kernel's 4.2 M workgroups slowed it
        // by 6 %, one in 1024 by 0.2 % (profiles/r04_stamps_runtime_ab.txt).  Nothing from the
        // dispatch packet (grid or block size): a load of it in each wave cost as much.
        const uint64_t g = base + blockIdx.x;  // the workgroup's index in the whole pass
        const bool first = threadIdx.x == 0 && g < kStampBegin;
        const bool sample = stamp_sampled(g);
        if (!first && !sample) return;
        uint64_t* sl = stamp_slot(st, epoch, kind);
        const uint64_t tag = (uint64_t)stamp_tag(epoch) << 40;
        const uint64_t now = stamp_clock();
        if (first) sl[g] = tag | ((t0 ? t0 : now) & kStampLow);
        if (!sample) return;
        const uint64_t act = __ballot(1);
        if ((threadIdx.x & 63) != (uint32_t)__builtin_ctzll(act)) return;
        sl[kStampBegin + stamp_end_word(g, threadIdx.x >> 6)] = tag | (now & kStampLow);
    }
};

// every kernel of a call resolves its epoch: a captured call reads the one the replay's
// k_epoch set (a plain load: written by an earlier kernel of the stream, so visible, and
// uniform, so it stays a scalar load — a volatile load here turned every tag test of the
// payload kernel into vector code, +6 us on C2)
__device__ inline void resolve_epoch(BatchArgs& a, const Workspace& ws) {
    if (a.dev_epoch) a.epoch = ws.ctl[kCtlEpoch];
}

// the call's look-back gave up (k_plan recorded this epoch): nothing of it may be delivered
__device__ inline bool device_fault(const BatchArgs& a, const Workspace& ws) {
    return *reinterpret_cast<volatile const uint32_t*>(ws.ctl + kCtlFaultEp) == a.epoch;
}

__device__ inline uint32_t first_bad_of(const BatchArgs& a, const Workspace& ws, uint32_t n) {
    return tag_get(*ws.first_bad, a.epoch, n);
}

__device__ inline uint64_t frame_start(const BatchArgs& a, uint32_t i) {
    return a.frame_off ? a.frame_off[i] : (uint64_t)i * a.frame_stride;
}

__device__ inline uint32_t nframes(const BatchArgs& a) { return a.n_dev ? *a.n_dev : a.n; }

// what frame i needs to know about its connection (batch mode: one implicit connection)
struct SegInfo {
    uint32_t seg;
    bool head, last;         // first / last frame of its connection
    uint64_t end;            // end of the bytes this frame may use
    int32_t max_frame_size, max_message_size, is_server;
    uint64_t init_pending;   // open fragmented message when the call starts
    int32_t init_opcode;
};

__device__ inline SegInfo seg_info(const BatchArgs& a, uint32_t i, uint32_t n) {
    SegInfo g;
    g.seg = 0;
    g.head = (i == 0);
    g.last = (i + 1 == n);
    g.end = g.last ? a.wire_len : frame_start(a, i + 1);
    g.max_frame_size = a.max_frame_size;
    g.max_message_size = a.max_message_size;
    g.is_server = a.is_server;
    g.init_pending = 0;
    g.init_opcode = 0;
    if (g.end > a.wire_len) g.end = a.wire_len;
    return g;
}

__device__ inline uint32_t rotr32(uint32_t x, uint32_t s) {
    return s ? (x >> s) | (x << (32u - s)) : x;
}

// ------------------------------------------------------------------------------------
// parse_one: frame i's header parse + every check process_data makes before the state
// machine (src/uvhttp_websocket.c:832-932), in the reference's order, on the bytes the
// batch contract feeds (include/uvhttp_ws_amd.h "Batch semantics").  Writes desc[i] and
// returns the frame's scan element.
// ------------------------------------------------------------------------------------
// the at most 14 header bytes (2 + 8 length + 4 key) of the frame at o in one 16-byte load;
// bytes past the frame's slot are loaded but never used (only the last 16 bytes of the wire
// go bytewise)
// The 16 bytes at wire[o, o + 16) (zeros past `len`).  Away from the end of the buffer they
// come from the two ALIGNED 16-byte vectors around them and a byte funnel shift: an unaligned
// 16-byte copy compiles to sixteen byte loads on gfx950 (k_plan spent most of its time there).
// The last 32 bytes of the buffer go bytewise so nothing past `len` is read.
template <bool NT = false>
__device__ inline u32x4 load16_at(const uint8_t* base, uint64_t len, uint64_t o) {
    const uint64_t lo = o & ~(uint64_t)15;
    if (len >= 32 && lo <= len - 32) {  // (cannot wrap for o near 2^64)
        const u32x4 v0 = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + lo))
                            : *reinterpret_cast<const u32x4*>(base + lo);
        const u32x4 v1 = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + lo + 16))
                            : *reinterpret_cast<const u32x4*>(base + lo + 16);
        uint64_t x0 = v0.x | ((uint64_t)v0.y << 32), x1 = v0.z | ((uint64_t)v0.w << 32);
        uint64_t x2 = v1.x | ((uint64_t)v1.y << 32);
        const uint64_t x3 = v1.z | ((uint64_t)v1.w << 32);
        const uint32_t d = (uint32_t)(o & 15);
        if (d & 8) {
            x0 = x1;
            x1 = x2;
            x2 = x3;
        }
        const uint32_t s = (d & 7) * 8;
        const uint64_t r0 = s ? (x0 >> s) | (x1 << (64 - s)) : x0;
        const uint64_t r1 = s ? (x1 >> s) | (x2 << (64 - s)) : x1;
        return u32x4{(uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32)};
    }
    const uint64_t avail = len > o ? len - o : 0;
    uint32_t t[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < 16 && k < avail; ++k) t[k >> 2] |= (uint32_t)base[o + k] << (8 * (k & 3));
    return u32x4{t[0], t[1], t[2], t[3]};
}

__device__ inline u32x4 load_header(const BatchArgs& a, uint64_t o) {
    return load16_at(a.wire, a.wire_len, o);
}

__device__ inline ScanElem parse_hdr(const BatchArgs& a, uint32_t i, const SegInfo& g, uint64_t o,
                                     u32x4 hv, uvhttp_ws_frame_desc_t& d) {
    const uint64_t slot = g.end > o ? g.end - o : 0;
    const bool last = g.last;

    d.payload_off = o;  // frames that do not parse keep a monotonic (empty) payload
    d.payload_len = 0;
    d.masking_key = 0;
    d.message = 0;
    d.opcode = 0;
    d.flags = 0;
    d.header_size = 0;
    d.status = UVHTTP_WS_FRAME_OK;
    d.wire_len = 0;

    const uint32_t hw0 = hv.x, hw1 = hv.y, hw2 = hv.z, hw3 = hv.w;
    const uint64_t hlo = (uint64_t)hw0 | ((uint64_t)hw1 << 32);
    const uint64_t hhi = (uint64_t)hw2 | ((uint64_t)hw3 << 32);
    auto hb = [&](int k) -> uint32_t {  // header byte k (k is a constant after inlining)
        return (uint32_t)((k < 8 ? hlo >> (8 * k) : hhi >> (8 * (k - 8))) & 0xFF);
    };

    bool parsable = false, msb = false;
    uint64_t plen = 0, wlen = 0;
    uint32_t hsz = 2, b0 = 0, b1 = 0;
    if (slot >= 2) {
        b0 = hb(0);
        b1 = hb(1);
        const uint32_t code = b1 & 0x7F;
        const uint32_t need = code == 126 ? 4 : code == 127 ? 10 : 2;
        if (slot >= need) {
            parsable = true;
            if (need == 2) {
                plen = code;
            } else if (need == 4) {
                plen = ((uint64_t)hb(2) << 8) | hb(3);
            } else {
                plen = ((uint64_t)hb(2) << 56) | ((uint64_t)hb(3) << 48) | ((uint64_t)hb(4) << 40) |
                       ((uint64_t)hb(5) << 32) | ((uint64_t)hb(6) << 24) | ((uint64_t)hb(7) << 16) |
                       ((uint64_t)hb(8) << 8) | (uint64_t)hb(9);
            }
            msb = (need == 10) && (plen >> 63);
            hsz = need;
            if (!msb) {
                const uint32_t m = (b1 >> 7) ? 4u : 0u;
                wlen = hsz + m + plen;
                if (m && slot >= hsz + 4) {
                    d.masking_key = need == 2 ? (uint32_t)(hlo >> 16)
                                  : need == 4 ? (uint32_t)(hlo >> 32)
                                              : (uint32_t)(hhi >> 16);
                }
                d.payload_off = o + hsz + m;
            }
        }
    }
    d.opcode = (uint8_t)(b0 & 0x0F);
    d.flags = (uint8_t)(((b0 >> 7) & 1) | (((b1 >> 7) & 1) << 1) | (((b0 >> 6) & 1) << 2) |
                        (((b0 >> 5) & 1) << 3) | (((b0 >> 4) & 1) << 4));
    d.header_size = (uint8_t)hsz;
    d.payload_len = plen;
    d.wire_len = wlen > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)wlen;

    int st = UVHTTP_WS_FRAME_OK;
    uint64_t fed;
    if (!a.streams && !last && (!parsable || (!msb && wlen != slot))) {
        st = UVHTTP_WS_FRAME_ERR_LAYOUT;  // batch mode only: streams are walked
        fed = slot;
    } else {
        fed = (last && parsable && !msb && wlen < slot) ? wlen : slot;
    }
    if (st == UVHTTP_WS_FRAME_OK) {
        // recv buffer cap (:851-857): an empty buffer grows to max(max_frame, 64 KiB);
        // a stream decode checks it once per connection in k_walk instead
        const uint64_t mf = (uint64_t)(int64_t)g.max_frame_size;
        const uint64_t cap = mf > 65536u ? mf : 65536u;
        if (!a.streams && fed > cap) st = UVHTTP_WS_FRAME_ERR_BUFFER;
        else if (!parsable) st = UVHTTP_WS_FRAME_INCOMPLETE;
        else if (msb) st = UVHTTP_WS_FRAME_ERR_PARSE;
        else if (d.flags & (UVHTTP_WS_FLAG_RSV1 | UVHTTP_WS_FLAG_RSV2 | UVHTTP_WS_FLAG_RSV3))
            st = UVHTTP_WS_FRAME_ERR_RSV;
        else if (d.opcode >= 8 && (plen > 125 || !(d.flags & UVHTTP_WS_FLAG_FIN)))
            st = UVHTTP_WS_FRAME_ERR_CONTROL;
        else if (g.is_server && !(d.flags & UVHTTP_WS_FLAG_MASK))
            st = UVHTTP_WS_FRAME_ERR_UNMASKED;
        else if (plen > mf) st = UVHTTP_WS_FRAME_ERR_TOO_BIG;
        else if (fed < wlen) st = UVHTTP_WS_FRAME_INCOMPLETE;
    }
    d.status = (int8_t)st;
    ScanElem elem = scan_identity();
    if (st == UVHTTP_WS_FRAME_OK) elem = scan_elem_of(d, (int32_t)i, g.head);
    else if (g.head) elem.bits = kHead;
    return elem;
}

__device__ inline ScanElem parse_one(const BatchArgs& a, uint32_t i, const SegInfo& g,
                                     uvhttp_ws_frame_desc_t& d) {
    const uint64_t o = frame_start(a, i);
    return parse_hdr(a, i, g, o, load_header(a, o), d);
}

__device__ inline FrameRec rec_of(const uvhttp_ws_frame_desc_t& d) {
    FrameRec r;
    r.payload_len = d.payload_len;
    r.masking_key = d.masking_key;
    r.opcode = d.opcode;
    r.flags = (uint8_t)(d.flags | (d.wire_len ? kRecHasLen : 0));  // wire_len >= 2 iff parsed
    r.header_size = d.header_size;
    r.status = d.status;
    return r;
}

// the 8-byte record straight from a parsed descriptor (rec8_pack(rec_of(d)), fewer steps in
// the payload pass's parse loop)
__device__ inline FrameRec8 rec8_of_desc(const uvhttp_ws_frame_desc_t& d) {
    const uint32_t hs = d.header_size;
    const bool simple = d.status == UVHTTP_WS_FRAME_OK && d.wire_len && !(d.flags & ~3u) &&
                        d.payload_len < (1ull << kR8LenBits) && (hs == 2 || hs == 4 || hs == 10);
    FrameRec8 p;
    p.key = d.masking_key;
    p.w = simple ? ((uint32_t)d.payload_len | ((uint32_t)d.opcode << 23) | ((uint32_t)d.flags << 27) | ((hs >> 2) << 29))
                 : kR8Esc;
    return p;
}

// frame i's record in a stride batch: the payload pass's, or — escaped — its header parsed again
// from the wire (the pass's parse_hdr on the same bytes)
__device__ inline FrameRec rec_at(const BatchArgs& a, const FrameRec8& p, uint32_t i) {
    FrameRec r;
    if (rec8_unpack(p, r)) return r;
    uvhttp_ws_frame_desc_t d;
    (void)parse_one(a, i, seg_info(a, i, a.n), d);
    return rec_of(d);
}

// the descriptor parse_hdr wrote for the frame at o, rebuilt from its record
__device__ inline void desc_of_rec(const FrameRec& r, uint64_t o, uvhttp_ws_frame_desc_t& d) {
    const bool has_len = r.flags & kRecHasLen;
    const uint64_t m = (r.flags & UVHTTP_WS_FLAG_MASK) ? 4u : 0u;
    d.payload_len = r.payload_len;
    d.masking_key = r.masking_key;
    d.message = 0;
    d.opcode = r.opcode;
    d.flags = (uint8_t)(r.flags & ~kRecHasLen);
    d.header_size = r.header_size;
    d.status = r.status;
    d.payload_off = has_len ? o + r.header_size + m : o;
    const uint64_t wlen = has_len ? r.header_size + m + r.payload_len : 0;
    d.wire_len = wlen > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)wlen;
}

// the frame's scan element from its parsed descriptor (what parse_hdr returns)
__device__ inline ScanElem elem_of_parsed(const uvhttp_ws_frame_desc_t& d, uint32_t i, bool head) {
    ScanElem e = scan_identity();
    if (d.status == UVHTTP_WS_FRAME_OK) e = scan_elem_of(d, (int32_t)i, head);
    else if (head) e.bits = kHead;
    return e;
}

// x / frame_stride for a stride batch (x < 2^53): a double multiply, then one correction
__device__ inline uint64_t div_stride(const BatchArgs& a, uint64_t x) {
    uint64_t q = (uint64_t)((double)x * a.stride_inv);
    if (q * a.frame_stride > x) --q;
    else if ((q + 1) * a.frame_stride <= x) ++q;
    return q;
}

// resolve_one: frame i's state-machine step.  With E = scan over the frames of the same
// connection before i, the state before frame i follows from the latest data frame p alone
// (all frames before a delivered frame are valid): PENDING iff p exists, p has FIN=0, and p
// is not a zero-length start (a zero-length first fragment allocates nothing, so
// fragmented_message stays NULL, src/uvhttp_websocket.c:794-816 + :964).  With no data
// frame before i in its connection, the state is the connection's initial one.
// d: the frame's parsed descriptor (registers), completed here; the caller stores it once
__device__ inline void resolve_one(const BatchArgs& a, uvhttp_ws_message_desc_t* msgs,
                                   const Workspace& ws, uint32_t i, uint32_t n, const SegInfo& g,
                                   ScanElem ex, uvhttp_ws_frame_desc_t& d) {
    if (g.head) ex = scan_identity();  // nothing of this connection precedes its first frame

    // in-place tiles whose start byte lies in this frame's span up to the next frame (frame
    // 0 also owns the bytes before its start); the max-of-tag claim keeps the smallest frame
    // when a bad offset table makes slots overlap.  (The fused stride path's payload pass
    // finds frames by arithmetic: no tile map.)
    // (the speculative compact decode claims none: its fallback scatter finds a stride batch's
    // frames by arithmetic, tile_first_of)
    if ((!a.recs || a.arena) && !a.spec_P) {  // (compact decodes: k_scatter_compact reads this map too)
        const uint64_t o = frame_start(a, i);
        uint64_t end = (i + 1 < n) ? frame_start(a, i + 1) : a.wire_len;
        if (end > a.wire_len) end = a.wire_len;
        const uint64_t lo = (i == 0) ? 0 : o;
        // (a start past the end claims nothing; the guard also keeps lo + kMapTile from
        // wrapping for an offset-table entry near 2^64)
        for (uint64_t t = lo < end ? lo / kMapTile + (lo % kMapTile != 0) : a.n_tiles;
             t * kMapTile < end && t < a.n_tiles; ++t)
            tag_claim(&ws.tile_first[t], a.epoch, i, a.cas_claims);
    }

    // fragment state before this frame: the latest data frame of the connection, carried
    // in the scan (no other block's descriptors are read)
    const bool pending = ex.last_data >= 0 ? (ex.bits & kLastOpen) != 0 : g.init_pending > 0;
    // bytes of the open message so far (the connection's carried part when no start yet)
    const uint64_t acc = (ex.bits & kSegFlag) ? ex.seg_pay : g.init_pending + ex.seg_pay;

    int st = d.status;
    if (st == UVHTTP_WS_FRAME_OK && is_data_op(d.opcode)) {
        const uint64_t lim = (uint64_t)(int64_t)g.max_message_size;
        const bool is_cont = d.opcode == 0;
        const bool fin = d.flags & UVHTTP_WS_FLAG_FIN;
        if (!pending) {
            if (is_cont) st = UVHTTP_WS_FRAME_ERR_FRAGMENT;
            else if (!fin && lim != 0 && d.payload_len > lim) st = UVHTTP_WS_FRAME_ERR_MESSAGE;
        } else {
            if (!is_cont) st = UVHTTP_WS_FRAME_ERR_FRAGMENT;
            else if (lim != 0 && (acc > lim || d.payload_len > lim - acc))
                st = UVHTTP_WS_FRAME_ERR_MESSAGE;
        }
        if (st == UVHTTP_WS_FRAME_OK) {
            d.message = ex.n_fin;
            if (a.arena) d.payload_off = ex.data_pay;
            if (fin) {
                d.flags |= UVHTTP_WS_FLAG_MSG_END;
                if (msgs) {
                    uvhttp_ws_message_desc_t m;
                    const uint64_t before = pending ? ex.seg_pay : 0;
                    m.arena_off = a.arena ? ex.data_pay - before : 0;
                    m.len = before + d.payload_len;
                    m.first_frame = pending ? (uint32_t)ex.last_start : i;
                    m.last_frame = i;
                    m.opcode = pending ? (uint8_t)((ex.bits & kOpMask) >> kOpShift) : d.opcode;
                    m.reserved = 0;
                    msgs[ex.n_fin] = m;
                }
            }
            // arena tiles whose first byte lies in this data frame's payload
            if (a.arena && d.payload_len && !a.spec_P) {  // (only k_gather_compact reads them)
                const uint64_t lo = ex.data_pay, hi = ex.data_pay + d.payload_len;
                for (uint64_t t = (lo + kMapTile - 1) / kMapTile; t * kMapTile < hi && t < a.n_arena_tiles;
                     ++t)
                    tag_claim(&ws.arena_first[t], a.epoch, i, a.cas_claims);
            }
        }
        d.status = (int8_t)st;
    }
    if (st != UVHTTP_WS_FRAME_OK) tag_claim(ws.first_bad, a.epoch, i, a.cas_claims);
    // speculative compact pass (stride batches): it placed frame i's payload at i * spec_P when
    // the frame looked uniform locally; a delivered frame anywhere else (a control frame, another
    // length, an offset moved by an earlier frame) sends the call to the full scatter (k_spec_fix)
    else if (a.spec_P && (!is_data_op(d.opcode) || d.payload_len != a.spec_P ||
                          ex.data_pay != (uint64_t)i * a.spec_P ||
                          d.header_size + ((d.flags & UVHTTP_WS_FLAG_MASK) ? 4u : 0u) !=
                              a.frame_stride - a.spec_P))
        tag_claim(ws.spec_bad, a.epoch, i, a.cas_claims);
}

// ------------------------------------------------------------------------------------
// Single-pass decoupled look-back (one launch for parse + scan + state machine).
// Blocks take tickets in launch order, so a block only ever waits on blocks that already
// run.  A block publishes its aggregate ("A" record), then all 256 lanes look back at 256
// predecessors at a time, combining aggregates until they meet a published inclusive
// prefix ("P" record).  A record is 64 bytes: four 16-byte chunks, each 12 bytes of the
// scan value + a 4-byte tag (epoch << 2 | kind), written and read as single device-coherent
// (sc1) 16-byte accesses.  A reader accepts a record only when all four tags carry this
// call's epoch and kind, so one round trip both polls and fetches — no flags, no L2
// writeback or invalidate.  Polls are bounded so a defect cannot hang the device: on
// exhaustion the block still publishes (so its successors finish) but records the call's
// epoch in ws.ctl[kCtlFaultEp] and bumps ws.ctl[kCtlFaults]; the call then delivers nothing
// (first_bad = frame 0 / every stream ERR_DEVICE) and engine_sync reports ELAUNCH.
// ------------------------------------------------------------------------------------
constexpr uint32_t kRecAgg = 1, kRecPrefix = 2;
constexpr uint32_t kMaxPolls = 1u << 20;
constexpr int kAuxSc1 = 16;  // buffer-op cache policy: device scope (sc1)
static_assert(sizeof(ScanElem) == 48, "scan value packs into 11 of the record's 12 data words");

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

__device__ inline __amdgpu_buffer_rsrc_t rec_rsrc(const LbRec* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<LbRec*>(base), 0, 0x7FFFFFFF, 0x00020000);
}

// the scan value as 11 words, in record order
#define UVWS_ELEM_WORDS(e)                                                                   \
    (uint32_t)(e).last_data, (uint32_t)(e).last_start, (uint32_t)(e).data_pay,               \
        (uint32_t)((e).data_pay >> 32), (uint32_t)(e).all_pay, (uint32_t)((e).all_pay >> 32), \
        (uint32_t)(e).seg_pay, (uint32_t)((e).seg_pay >> 32), (e).n_fin, (e).n_close, (e).bits

__device__ inline void rec_store(LbRec* recs, uint32_t j, const ScanElem& v, uint32_t tag) {
    const uint32_t w[12] = {UVWS_ELEM_WORDS(v), 0u};
    const __amdgpu_buffer_rsrc_t rs = rec_rsrc(recs);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const u32x4v x = {w[3 * c], w[3 * c + 1], w[3 * c + 2], tag};
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, j * 64u + 16u * c, 0, kAuxSc1);
    }
}

__device__ inline void rec_fetch(const LbRec* recs, uint32_t j, u32x4v x[4]) {
    const __amdgpu_buffer_rsrc_t rs = rec_rsrc(recs);
#pragma unroll
    for (int c = 0; c < 4; ++c) x[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, j * 64u + 16u * c, 0, kAuxSc1);
}

__device__ inline bool rec_valid(const u32x4v x[4], uint32_t tag) {
    return x[0].w == tag && x[1].w == tag && x[2].w == tag && x[3].w == tag;
}

__device__ inline ScanElem rec_value(const u32x4v x[4]) {
    ScanElem e;
    e.last_data = (int32_t)x[0].x;
    e.last_start = (int32_t)x[0].y;
    e.data_pay = (uint64_t)x[0].z | ((uint64_t)x[1].x << 32);
    e.all_pay = (uint64_t)x[1].y | ((uint64_t)x[1].z << 32);
    e.seg_pay = (uint64_t)x[2].x | ((uint64_t)x[2].y << 32);
    e.n_fin = x[2].z;
    e.n_close = x[3].x;
    e.bits = x[3].y;
    return e;
}

// exclusive prefix of block b (all threads call; the value is broadcast through LDS)
template <int NT = kBlock>
__device__ ScanElem lookback_prefix(const Workspace& ws, uint32_t b, const ScanElem& agg,
                                    uint32_t epoch, uint32_t max_polls) {
    __shared__ ScanElem s_wave[NT / 64];
    __shared__ ScanElem s_pre;
    __shared__ int s_kstar;
    __shared__ int s_go;
    const uint32_t tag_a = (epoch << 2) | kRecAgg, tag_p = (epoch << 2) | kRecPrefix;
    if (threadIdx.x == 0) {
        if (b == 0) {
            rec_store(ws.rec_p, 0, agg, tag_p);
            s_pre = scan_identity();
            ws.block_excl[0] = scan_identity();
            ws.block_incl[0] = agg;
        } else {
            rec_store(ws.rec_a, b, agg, tag_a);
        }
    }
    if (b == 0) {
        __syncthreads();
        return s_pre;
    }
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    ScanElem run = scan_identity();  // thread 0: combination of the predecessors seen so far
    int64_t end = b;                 // window: blocks [end - NT, end)
    uint32_t polls = 0;              // uniform: every thread counts the same rounds
    bool gave_up = false;
    for (;;) {
#ifdef UVWS_LOOKBACK_BPERMUTE
        const int64_t j = end - 1 - t;  // larger t = older block
#else
        const int64_t j = end - NT + t;  // larger t = newer block (window order = lane order)
#endif
        ScanElem v = scan_identity();
        bool is_p = j < 0, ready = j < 0;  // lanes before block 0: identity "P"
        for (;;) {
            if (!ready) {  // both records in one round trip
                u32x4v xp[4], xa[4];
                rec_fetch(ws.rec_p, (uint32_t)j, xp);
                rec_fetch(ws.rec_a, (uint32_t)j, xa);
                if (rec_valid(xp, tag_p)) {
                    v = rec_value(xp), is_p = true, ready = true;
                } else if (rec_valid(xa, tag_a)) {
                    v = rec_value(xa), ready = true;
                }
            }
            if (__syncthreads_and(ready) && max_polls) break;
            if (++polls > max_polls) {
                gave_up = true;
                break;
            }
            // back off so waiting blocks do not flood memory while predecessors still parse
            __builtin_amdgcn_s_sleep(8);
        }
#ifdef UVWS_LOOKBACK_BPERMUTE
        // nearest published prefix (smallest t with P)
        if (t == 0) s_kstar = NT;
        __syncthreads();
        const uint64_t pm = __ballot(is_p);
        if (lane == 0 && pm) atomicMin(&s_kstar, wave * 64 + __builtin_ctzll(pm));
        __syncthreads();
        const int kstar = s_kstar;
        if (t > kstar || j < 0) v = scan_identity();
        v = wave_reduce_newest_first(v);
        if (lane == 0) s_wave[wave] = v;
        __syncthreads();
        if (t == 0) {
            ScanElem w = scan_identity();
#pragma unroll
            for (int k = NT / 64 - 1; k >= 0; --k) w = scan_combine(w, s_wave[k]);
            run = scan_combine(w, run);
            s_go = (kstar < NT || gave_up) ? 0 : 1;
        }
#else
        // nearest published prefix: the largest t with P; the window from it to the newest
        // block, combined in lane order by the DPP wave scan (lane 63 holds the wave's part)
        if (t == 0) s_kstar = -1;
        __syncthreads();
        const uint64_t pm = __ballot(is_p);
        if (lane == 0 && pm) atomicMax(&s_kstar, wave * 64 + 63 - __builtin_clzll(pm));
        __syncthreads();
        const int kstar = s_kstar;
        if (t < kstar || j < 0) v = scan_identity();
        v = wave_inclusive_scan(v);
        if (lane == 63) s_wave[wave] = v;
        __syncthreads();
        if (t == 0) {
            ScanElem w = scan_identity();
#pragma unroll
            for (int k = 0; k < NT / 64; ++k) w = scan_combine(w, s_wave[k]);
            run = scan_combine(w, run);
            s_go = (kstar >= 0 || gave_up) ? 0 : 1;
        }
#endif
        __syncthreads();
        if (!s_go) break;
        end -= NT;
    }
    if (t == 0) {
        s_pre = run;
        const ScanElem incl = scan_combine(run, agg);
        ws.block_excl[b] = run;
        ws.block_incl[b] = incl;
        rec_store(ws.rec_p, b, incl, tag_p);
        if (gave_up) {
            __hip_atomic_store(&ws.ctl[kCtlFaultEp], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&ws.ctl[kCtlFaults], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            tag_claim(ws.first_bad, epoch, 0, 1u);  // batch mode: the payload pass unmasks nothing (rare: always displaces)
        }
    }
    __syncthreads();
    return s_pre;
}

// fused stride path: the lane's FPT records (one contiguous 16 * FPT-byte run) -> the
// frames' descriptors in registers and the lane's scan aggregate
template <int FPT>
__device__ inline ScanElem rec_pass1(const BatchArgs& a, uint32_t i0, uint32_t n,
                                     uvhttp_ws_frame_desc_t (&dv)[FPT]) {
    ScanElem tagg = scan_identity();
    FrameRec8 r[FPT];
    const uint32_t ilast = n ? n - 1 : 0;
#pragma unroll
    for (int k = 0; k < FPT; ++k) r[k] = a.recs[i0 + k < n ? i0 + k : ilast];
#pragma unroll
    for (int k = 0; k < FPT; ++k) {
        const uint32_t i = i0 + k;
        if (i < n) {
            desc_of_rec(rec_at(a, r[k], i), (uint64_t)i * a.frame_stride, dv[k]);
            tagg = scan_combine(tagg, elem_of_parsed(dv[k], i, i == 0));
        }
    }
    return tagg;
}

// one descriptor store (UVWS_DESC_NT, experiment: two streaming 16-byte stores)
__device__ inline void store_desc(uvhttp_ws_frame_desc_t* desc, uint32_t i, const uvhttp_ws_frame_desc_t& d) {
#ifdef UVWS_DESC_NT
    const u32x4* w = reinterpret_cast<const u32x4*>(&d);
    __builtin_nontemporal_store(w[0], reinterpret_cast<u32x4*>(desc + i));
    __builtin_nontemporal_store(w[1], reinterpret_cast<u32x4*>(desc + i) + 1);
#else
    desc[i] = d;
#endif
}

// pass 2: the state machine in frame order from the lane's exclusive prefix `run`; each
// descriptor is stored once.  (Staging a wave's descriptors in LDS to store them as whole
// streaming lines measured 2.5 % slower on C4: the LDS round trip costs more than the partial
// lines it saves.)
template <int FPT>
__device__ inline void plan_pass2(const BatchArgs& a, uvhttp_ws_frame_desc_t* desc,
                                  uvhttp_ws_message_desc_t* msgs, const Workspace& ws, uint32_t i0,
                                  uint32_t n, ScanElem run, uvhttp_ws_frame_desc_t (&dv)[FPT]) {
#pragma unroll
    for (int k = 0; k < FPT; ++k) {
        const uint32_t i = i0 + k;
        if (i < n) {
            const SegInfo g = seg_info(a, i, n);
            ScanElem e = scan_identity();
            if (dv[k].status == UVHTTP_WS_FRAME_OK) e = scan_elem_of(dv[k], (int32_t)i, g.head);
            else if (g.head) e.bits = kHead;
            resolve_one(a, msgs, ws, i, n, g, run, dv[k]);
            store_desc(desc, i, dv[k]);
            run = scan_combine(run, e);
        }
    }
}

// k_plan: one launch per decode: parse -> block scan -> look-back -> state machine.  Each
// lane owns FPT consecutive frames (FPT > 1 keeps the block count, and with it the look-back
// chain, short for large batches): pass 1 parses them and reduces their scan elements,
// pass 2 (after the block's prefix is known) re-reads their descriptors and runs the state
// machine in frame order.  The block holding the last ticket resets the counter for the
// next call.
template <int FPT, int NT = kBlock, bool REC = false>
__global__ __launch_bounds__(NT) void k_plan(BatchArgs a, uvhttp_ws_frame_desc_t* desc,
                                                 uvhttp_ws_message_desc_t* msgs, Workspace ws) {
    resolve_epoch(a, ws);
    if (a.gate && ws.ctl[kCtlGate] != a.epoch) return;  // (summary-only compact: speculation held)
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_PLAN);
    __shared__ uint32_t s_ticket;
    if (threadIdx.x == 0) {
        uint32_t t = blockIdx.x;
        if (!a.no_ticket) {
            t = __hip_atomic_fetch_add(&ws.counters[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t + 1 == gridDim.x)
                __hip_atomic_store(&ws.counters[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_ticket = t;
    }
    __syncthreads();
    const uint32_t b = s_ticket;
    const uint32_t n = nframes(a);
    const uint32_t i0 = (b * NT + threadIdx.x) * FPT;
#ifdef UVWS_PLAN_PHASES
    // per block: [0] start (after the ticket) [1] thread 0's pass 1 done [2] block scan done
    // [3] look-back done [4] thread 0's pass 2 done [5] latest wave end, [6] blockIdx, [7] CU id
    unsigned long long* ph = a.stamp && b < 8192 ? reinterpret_cast<unsigned long long*>(a.stamp + kStampWords + 8ull * b) : nullptr;
    auto phase = [&](int k) {
        if (ph && threadIdx.x == 0) ph[k] = (unsigned long long)wall_clock64();
    };
    phase(0);
    if (ph && threadIdx.x == 0) {
        ph[6] = blockIdx.x;
        ph[7] = __smid();
    }
    struct PhaseEnd {
        unsigned long long* p;
        __device__ ~PhaseEnd() {
            if (p && (threadIdx.x & 63) == 0) atomicMax(p + 5, (unsigned long long)wall_clock64());
        }
    } phase_end_{ph};
#else
    auto phase = [](int) {};
#endif
    if constexpr (REC) {
        // records path: the lane's 8-byte records stay in registers across the scan (the
        // 32-byte descriptors built from them took 128 registers and spilled at 16 frames per
        // lane) and pass 2 rebuilds each descriptor from its record.  (Coalesced record loads
        // handed to their owner lanes through LDS measured no faster: profiles/r03p49_*.)
        ScanElem tagg = scan_identity();
        FrameRec8 r[FPT];
        const uint32_t ilast = n ? n - 1 : 0;
#pragma unroll
        for (int k = 0; k < FPT; ++k) r[k] = a.recs[i0 + k < n ? i0 + k : ilast];
#pragma unroll
        for (int k = 0; k < FPT; ++k) {
            const uint32_t i = i0 + k;
            if (i < n) {
                uvhttp_ws_frame_desc_t d;
                desc_of_rec(rec_at(a, r[k], i), (uint64_t)i * a.frame_stride, d);
                tagg = scan_combine(tagg, elem_of_parsed(d, i, i == 0));
            }
        }
        phase(1);
        ScanElem agg;
        const ScanElem local = block_exclusive_scan<NT>(tagg, &agg);
        phase(2);
        ScanElem run = scan_combine(lookback_prefix<NT>(ws, b, agg, a.epoch, a.max_polls), local);
        phase(3);
#pragma unroll
        for (int k = 0; k < FPT; ++k) {
            const uint32_t i = i0 + k;
            if (i < n) {
                uvhttp_ws_frame_desc_t d;
                desc_of_rec(rec_at(a, r[k], i), (uint64_t)i * a.frame_stride, d);
                const SegInfo g = seg_info(a, i, n);
                const ScanElem e = elem_of_parsed(d, i, g.head);
                resolve_one(a, msgs, ws, i, n, g, run, d);
                store_desc(desc, i, d);
                run = scan_combine(run, e);
            }
        }
        phase(4);
        return;
    }
    if (FPT == 1) {
        SegInfo g;
        uvhttp_ws_frame_desc_t d;
        ScanElem elem = scan_identity();
        if (i0 < n) {
            g = seg_info(a, i0, n);
            if (a.recs) {  // fused stride path: the payload pass parsed the header already
                desc_of_rec(rec_at(a, a.recs[i0], i0), frame_start(a, i0), d);
                elem = elem_of_parsed(d, i0, g.head);
            } else {
                elem = parse_one(a, i0, g, d);
            }
        }
        phase(1);
        ScanElem agg;
        const ScanElem local = block_exclusive_scan<NT>(elem, &agg);
        phase(2);
        const ScanElem pre = lookback_prefix<NT>(ws, b, agg, a.epoch, a.max_polls);
        phase(3);
        if (i0 < n) {
            resolve_one(a, msgs, ws, i0, n, g, scan_combine(pre, local), d);
            desc[i0] = d;
        }
        phase(4);
        return;
    }
    // pass 1: all header loads of the lane's frames in flight together, then parse into
    // registers (descriptors are stored once, after the state machine)
    ScanElem tagg = scan_identity();
    uvhttp_ws_frame_desc_t dv[FPT];
    if (a.recs) {
        tagg = rec_pass1<FPT>(a, i0, n, dv);
    } else {
        // every load unconditional (indices clamped to the last frame, header windows to the
        // last 16 wire bytes) so all of them are in flight together: under per-frame branches
        // the compiler waited for each load before issuing the next (32 round trips per lane)
        uint64_t o[FPT];
        u32x4 hv[FPT];
        const uint32_t ilast = n ? n - 1 : 0;
        if (a.frame_off) {
#pragma unroll
            for (int k = 0; k < FPT; ++k) o[k] = a.frame_off[i0 + k < n ? i0 + k : ilast];
        } else {
#pragma unroll
            for (int k = 0; k < FPT; ++k) o[k] = (uint64_t)(i0 + k < n ? i0 + k : ilast) * a.frame_stride;
        }
        // two aligned 16-byte loads per frame, all issued before any is used
#pragma unroll
        for (int k = 0; k < FPT; ++k) hv[k] = load_header(a, o[k]);
#pragma unroll
        for (int k = 0; k < FPT; ++k) {
            const uint32_t i = i0 + k;
            if (i < n) tagg = scan_combine(tagg, parse_hdr(a, i, seg_info(a, i, n), o[k], hv[k], dv[k]));
        }
    }
    phase(1);
    ScanElem agg;
    const ScanElem local = block_exclusive_scan<NT>(tagg, &agg);
    phase(2);
    ScanElem run = scan_combine(lookback_prefix<NT>(ws, b, agg, a.epoch, a.max_polls), local);
    phase(3);
    plan_pass2<FPT>(a, desc, msgs, ws, i0, n, run, dv);
    phase(4);
}

// ------------------------------------------------------------------------------------
// Reduce-then-scan over the fused path's records (no tickets, no look-back waits): the
// records are 16 contiguous bytes per frame, so reading them twice is cheaper than making
// 256 blocks wait on each other (tools/ab_lib.py).
//   k_rec_reduce   block b: the scan aggregate of its kBlock * FPT frames -> block_agg[b]
//   k_rec_scan     one 1024-thread block: exclusive / inclusive prefixes of the aggregates
//   k_rec_resolve  block b: its frames' descriptors, the block scan from block_excl[b], the
//                  state machine and the descriptor stores (k_plan's pass 2)
// ------------------------------------------------------------------------------------
template <int FPT>
__global__ __launch_bounds__(kBlock) void k_rec_reduce(BatchArgs a, Workspace ws) {
    const uint32_t n = a.n;
    const uint32_t i0 = (blockIdx.x * kBlock + threadIdx.x) * FPT;
    uvhttp_ws_frame_desc_t dv[FPT];
    const ScanElem tagg = rec_pass1<FPT>(a, i0, n, dv);
    ScanElem agg;
    (void)block_exclusive_scan(tagg, &agg);
    if (threadIdx.x == 0) ws.block_agg[blockIdx.x] = agg;
}

constexpr int kScanBlock = 1024;
__global__ __launch_bounds__(kScanBlock) void k_rec_scan(Workspace ws, uint32_t nblocks) {
    const uint32_t per = (nblocks + kScanBlock - 1) / kScanBlock;
    const uint32_t j0 = threadIdx.x * per;
    ScanElem mine = scan_identity();
    for (uint32_t j = j0; j < j0 + per && j < nblocks; ++j) mine = scan_combine(mine, ws.block_agg[j]);
    ScanElem tot;
    ScanElem run = block_exclusive_scan<kScanBlock>(mine, &tot);
    for (uint32_t j = j0; j < j0 + per && j < nblocks; ++j) {
        ws.block_excl[j] = run;
        run = scan_combine(run, ws.block_agg[j]);
        ws.block_incl[j] = run;
    }
}

template <int FPT>
__global__ __launch_bounds__(kBlock) void k_rec_resolve(BatchArgs a, uvhttp_ws_frame_desc_t* desc,
                                                        uvhttp_ws_message_desc_t* msgs, Workspace ws) {
    resolve_epoch(a, ws);
    const uint32_t n = a.n;
    const uint32_t i0 = (blockIdx.x * kBlock + threadIdx.x) * FPT;
    uvhttp_ws_frame_desc_t dv[FPT];
    const ScanElem tagg = rec_pass1<FPT>(a, i0, n, dv);
    ScanElem agg;
    const ScanElem local = block_exclusive_scan(tagg, &agg);
    plan_pass2<FPT>(a, desc, msgs, ws, i0, n, scan_combine(ws.block_excl[blockIdx.x], local), dv);
}

// A frame the call did not deliver (after the first failure, or every frame after a device
// fault): SKIPPED, and no message id or MSG_END — the scan carries state past the first failure,
// but nothing of it belongs to a delivered message, so every decode path leaves the same
// descriptor (k_desc_emit never computes that state).  Word 5 = message, word 6 = opcode | flags
// << 8 | header_size << 16 | status << 24.
// A compact decode's data frame keeps its payload in the wire then too (payload_off = the wire
// offset parse_hdr gives; the scan past the failure may have assigned an arena offset).
__device__ inline void skip_desc(const BatchArgs& a, uvhttp_ws_frame_desc_t* desc, uint64_t i) {
    uint32_t* w = reinterpret_cast<uint32_t*>(desc + i);
    const uint32_t w6 = w[6];
    w[5] = 0u;
    w[6] = (w6 & 0x00FFFFFFu & ~((uint32_t)UVHTTP_WS_FLAG_MSG_END << 8)) |
           ((uint32_t)(uint8_t)UVHTTP_WS_FRAME_SKIPPED << 24);
    if (a.arena) {
        const uint64_t o = frame_start(a, (uint32_t)i);
        const uint64_t po = w[7] ? o + ((w6 >> 16) & 0xFFu) + (((w6 >> 8) & UVHTTP_WS_FLAG_MASK) ? 4u : 0u) : o;
        w[0] = (uint32_t)po;
        w[1] = (uint32_t)(po >> 32);
    }
}

// summary of a batch decode, after k_plan (one wave of k_finalize): E(nb) is
// the exclusive scan value at the first failing frame (or the total)
__device__ void write_summary(const BatchArgs& a, const uvhttp_ws_frame_desc_t* desc,
                              const Workspace& ws, uint32_t nb) {
    const uint32_t n = a.n;
    const int lane = threadIdx.x & 63;
    ScanElem e;
    if (nb >= n) {
        e = ws.block_incl[n ? (n - 1) / a.plan_frames : 0];
    } else {
        const uint32_t b = nb / a.plan_frames;
        e = ws.block_excl[b];
        for (uint32_t f0 = b * a.plan_frames; f0 < nb; f0 += 64) {
            const uint32_t f = f0 + (63 - lane);  // lane 63 holds the oldest frame
            ScanElem el = scan_identity();
            if (f < nb) el = scan_elem_of(desc[f], (int32_t)f, f == 0);
            el = wave_reduce_newest_first(el);
            e = scan_combine(e, el);
        }
    }
    if (lane != 0) return;
    uvhttp_ws_batch_summary_t s;
    s.n_frames = n;
    s.n_delivered = nb < n ? nb : n;
    s.first_status = nb < n ? desc[nb].status : 0;
    s.status = s.first_status < 0 ? -1 : 0;
    const uint64_t start0 = n ? frame_start(a, 0) : 0;
    if (n == 0) {
        s.consumed_bytes = 0;
    } else if (nb < n) {
        s.consumed_bytes = frame_start(a, nb) - start0;
    } else {
        s.consumed_bytes = frame_start(a, n - 1) + desc[n - 1].wire_len - start0;
    }
    s.payload_bytes = e.all_pay;
    s.n_messages = e.n_fin;
    s.state_closed = e.n_close ? 1u : 0u;
    s.arena_bytes = a.arena ? e.data_pay : 0;
    s.pending_bytes = (e.last_data >= 0 && (e.bits & kLastOpen)) ? e.seg_pay : 0;
    *a.summary = s;
    // compact: the message a fragmented start left open (the arena's last pending_bytes), so a
    // caller can leave conn->fragmented_message as process_data does (uvhttp_ws_deliver_messages);
    // reserved = its first fragment's length, from which the reference's capacity follows
    // (src/uvhttp_websocket.c:794-816).  n_messages < n_frames here: the open start is no FIN.
    if (a.msgs && s.pending_bytes && e.last_start >= 0) {
        uvhttp_ws_message_desc_t m;
        m.arena_off = e.data_pay - e.seg_pay;
        m.len = e.seg_pay;
        m.first_frame = (uint32_t)e.last_start;
        m.last_frame = (uint32_t)e.last_data;
        m.opcode = (int32_t)((e.bits & kOpMask) >> kOpShift);
        m.reserved = (uint32_t)desc[e.last_start].payload_len;
        a.msgs[s.n_messages] = m;
    }
}

// k_finalize (batch mode, after the payload pass, one lane per frame): statuses after the
// first failure become SKIPPED; a compact decode unmasks control payloads (<= 125 B) in
// place; wave 0 of block 0 writes the batch summary
// (block `blk` of a grid of `nthr`-thread blocks, one frame per thread, `a` with its epoch
// resolved and nb = first_bad_of(a, ws, a.n); no workgroup barrier, so the in-place payload
// kernel runs it at the end of its first blocks and the decode needs no third launch)
__device__ inline void finalize_frames(const BatchArgs& a, uvhttp_ws_frame_desc_t* desc,
                                       const Workspace& ws, uint32_t blk, uint32_t nthr,
                                       uint32_t nb, bool controls = true) {
    const uint32_t i = blk * nthr + threadIdx.x;
    if (device_fault(a, ws)) {  // nothing was delivered (the payload pass saw first_bad = 0)
        if (i < a.n) skip_desc(a, desc, i);
        if (blk == 0 && threadIdx.x == 0) {
            uvhttp_ws_batch_summary_t s;
            memset(&s, 0, sizeof(s));
            s.n_frames = a.n;
            s.status = -1;
            s.first_status = UVHTTP_WS_FRAME_ERR_DEVICE;
            *a.summary = s;
        }
        return;
    }
    if (i < a.n) {
        if (i > nb) skip_desc(a, desc, i);
        if (a.arena && i < nb && controls) {
            const uvhttp_ws_frame_desc_t d = desc[i];
            if (d.opcode > 2 && d.payload_len) {
                const uint32_t key = d.masking_key;
                for (uint64_t q = 0; q < d.payload_len; ++q)
                    a.wire[d.payload_off + q] ^= (uint8_t)(key >> (8 * (q & 3)));
            }
        }
    }
    if (blk == 0 && threadIdx.x < 64) write_summary(a, desc, ws, nb);
}

__global__ __launch_bounds__(kBlock) void k_finalize(BatchArgs a, uvhttp_ws_frame_desc_t* desc,
                                                     Workspace ws) {
    resolve_epoch(a, ws);
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_FINALIZE);
    finalize_frames(a, desc, ws, blockIdx.x, kBlock, first_bad_of(a, ws, a.n));
}

// ------------------------------------------------------------------------------------
// payload helpers
// ------------------------------------------------------------------------------------

// bytes [lo, hi) of dword m (0..3) of a 16-byte vector as a 32-bit byte-lane mask
__device__ inline uint32_t lane_bytes(int lo, int hi, int m) {
    int l = lo - 4 * m, h = hi - 4 * m;
    l = l < 0 ? 0 : (l > 4 ? 4 : l);
    h = h < 0 ? 0 : (h > 4 ? 4 : h);
    if (h <= l) return 0u;
    const uint32_t up = h == 4 ? 0xFFFFFFFFu : ((1u << (8 * h)) - 1u);
    return up & ~((1u << (8 * l)) - 1u);
}

// mask vector contribution of one payload range [ps, pe) with key `key` (payload byte j
// uses key byte j & 3) to the 16-byte vector at address `va`.
__device__ inline void add_mask(u32x4& m, uint64_t va, uint64_t ps, uint64_t pe, uint32_t key) {
    if (pe <= va || ps >= va + 16) return;
    const uint32_t rk = rotr32(key, 8u * (uint32_t)((va - ps) & 3u));
    if (ps <= va && va + 16 <= pe) {
        m = u32x4{rk, rk, rk, rk};
        return;
    }
    const int lo = ps > va ? (int)(ps - va) : 0;
    const int hi = pe < va + 16 ? (int)(pe - va) : 16;
    m.x |= rk & lane_bytes(lo, hi, 0);
    m.y |= rk & lane_bytes(lo, hi, 1);
    m.z |= rk & lane_bytes(lo, hi, 2);
    m.w |= rk & lane_bytes(lo, hi, 3);
}

__device__ inline bool any_bits(const u32x4& m) { return (m.x | m.y | m.z | m.w) != 0u; }

// ------------------------------------------------------------------------------------
// k_unmask_inplace: the roofline kernel of the in-place decode.
// One workgroup per BLOCK*VPT*16-byte tile of the wire buffer (default 64 threads x 1
// vector = 1 KiB: on MI355X many small workgroups with one 16-byte load per lane stream
// read+write at 6.7 TB/s against 5.9 TB/s for 16 KiB workgroups — tools/stream_probe.hip,
// profiles/r01_stream_probe.txt).  Lane t handles the vectors tile + (v*BLOCK + t)*16.
// The payload loads are issued first — they depend only on the tile index — and the frame
// lookup (coarse map -> descriptors) runs while they are in flight.  Every byte of the
// wire belongs to exactly one tile, so whole-vector stores never race: bytes outside any
// delivered payload are XORed with 0 and vectors with no payload byte are not stored.
// ------------------------------------------------------------------------------------
// store-path cache policy of the payload pass: 0 = global_store nt; 18 = buffer_store with
// sc1|nt (write-through, not kept in L2), measured 1.7 % faster for the 64x1 shape
// (tools/stream_probe.hip, profiles/r01_stream_probe_policy.txt)
// the in-place payload kernel's tile shape by average wire bytes per frame (tools/ab_lib.py
// UVHTTP_WS_TILE sweeps, profiles/r04_tile_sizes_ab.txt): since the scalar-descriptor path takes
// up to kFastFrames frames per tile, small tiles win from 2.5 KiB frames up — 2 KiB tiles
// (64 x 2) at 2.5-12 KiB frames (C2 +1.5-2.5 %, 8 KiB +4 %), 1 KiB tiles (64 x 1) above (16 KiB
// +7 %, 64 KiB as before); 256 x 2 / 256 x 4 below
__host__ inline void inplace_tile_shape(uint64_t avg, int& blk, int& vpt) {
    if (avg >= 12288) blk = 64, vpt = 1;
    else if (avg >= 2560) blk = 64, vpt = 2;
    else blk = 256, vpt = avg >= 2048 ? 2 : 4;
}

#ifndef UVWS_FAST_FRAMES
#define UVWS_FAST_FRAMES 8
#endif
constexpr uint32_t kFastFrames = UVWS_FAST_FRAMES;  // scalar-descriptor path up to this many frames
template <int BLOCK, int VPT, int STORE_AUX>
__device__ __forceinline__ void unmask_tile(BatchArgs a,
                                            const uvhttp_ws_frame_desc_t* __restrict__ desc,
                                            const Workspace& ws, uint64_t tile_base,
                                            uint32_t& n_out, uint32_t& nb_out, StampScope& ss) {
    constexpr uint64_t kT = (uint64_t)BLOCK * VPT * 16;
    __shared__ uint64_t s_ps[BLOCK];
    __shared__ uint64_t s_pe[BLOCK];
    __shared__ uint32_t s_key[BLOCK];

    const uint64_t t0 = (tile_base + ss.anchor_s(blockIdx.x)) * kT;
    const uint64_t vend = a.wire_len;
    // loads are clamped to the last whole vector so they can be issued unconditionally;
    // the one vector straddling the end of the wire is finished bytewise
    const uint64_t full_end = vend & ~(uint64_t)15;
    const uint64_t clamp_va = full_end ? full_end - 16 : 0;

    u32x4 data[VPT];
    uint64_t va[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        va[v] = t0 + ((uint64_t)v * BLOCK + threadIdx.x) * 16u;
        const uint64_t la = va[v] < full_end ? va[v] : clamp_va;
        data[v] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.wire + la));
    }

    // batch mode: frames >= nb are not delivered (read after the loads are issued, like the
    // epoch of a captured call)
    resolve_epoch(a, ws);
    const uint32_t n = nframes(a);
    const uint32_t nb = first_bad_of(a, ws, n);
    n_out = n;
    nb_out = nb;
    if (nb == 0 || n == 0 || t0 >= vend) return;
    const uint32_t last = (nb < n ? nb : n) - 1;
    // frames overlapping [t0, t0 + kT): from the first frame of the coarse map tile holding
    // t0 to the first frame of the coarse tile after the one holding the tile's last byte
    // (loading the two map entries ahead of the test above changed nothing, r04_hoist_ab.txt)
    const uint64_t c0 = t0 / kMapTile, c1 = (t0 + kT - 1) / kMapTile + 1;
    const uint32_t f0 = tag_get(ws.tile_first[c0], a.epoch, kNoFrame);
    uint32_t f1 = (c1 < a.n_tiles) ? tag_get(ws.tile_first[c1], a.epoch, kNoFrame) : last;
    if (f0 > last) return;  // the tile starts past the delivered frames (or is unclaimed)
    if (f1 > last || f1 < f0) f1 = last;

    u32x4 m[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) m[v] = u32x4{0, 0, 0, 0};

    // (a stride-layout variant that finds a vector's frame by arithmetic and loads its
    // descriptor per lane measured slower than staging the tile's frames in LDS: C4 96 -> 117
    // us, C2 89 -> 96 us — many lanes re-loading the same 32-byte descriptors)
    if (f1 - f0 < kFastFrames) {
        // fast path: a few frames touch the tile; their descriptors are uniform scalar loads
        // (lgkmcnt: the mask work starts when they arrive, not behind the tile's data loads,
        // which a per-lane descriptor load would wait for on the in-order vmcnt)
        if (a.streams) {
            // stream decode: a delivered frame's payload only (undelivered: an empty range), no
            // branch on the status (r04_streams_desc_load_ab.txt)
            for (uint32_t f = f0; f <= f1; ++f) {
                const uint64_t ps = desc[f].payload_off;
                const uint64_t len = desc[f].payload_len;
                const uint32_t key = desc[f].masking_key;
                // the status byte through its 32-bit word (opcode, flags, header_size, status):
                // a byte field cannot be a scalar load, and as a vector load its wait also waited
                // for the tile's data loads, serialising the mask work behind them
                const uint32_t w6 = reinterpret_cast<const uint32_t*>(desc + f)[6];
                const uint64_t pe = ps + ((int8_t)(w6 >> 24) == UVHTTP_WS_FRAME_OK ? len : 0);
#pragma unroll
                for (int v = 0; v < VPT; ++v) add_mask(m[v], va[v], ps, pe, key);
            }
        } else {
            // batch decode: frames below nb are delivered; the three fields only (loading the
            // whole 32-byte descriptor here cost C3 in place 7 %, profiles/r04_desc_load_ab.txt)
            for (uint32_t f = f0; f <= f1; ++f) {
                const uint64_t ps = desc[f].payload_off;
                const uint64_t pe = ps + desc[f].payload_len;
                const uint32_t key = desc[f].masking_key;
#pragma unroll
                for (int v = 0; v < VPT; ++v) add_mask(m[v], va[v], ps, pe, key);
            }
        }
    } else {
        // general path: stage BLOCK frame ranges per round in LDS, binary-search per vector
        for (uint32_t base = f0; base <= f1; base += BLOCK) {
            const uint32_t cnt = (f1 - base + 1) < (uint32_t)BLOCK ? (f1 - base + 1) : BLOCK;
            // skip rounds that end before the tile or start after it
            __syncthreads();
            if (threadIdx.x < cnt) {
                const uvhttp_ws_frame_desc_t d = desc[base + threadIdx.x];
                const bool ok = !a.streams || d.status == UVHTTP_WS_FRAME_OK;  // undelivered: empty
                s_ps[threadIdx.x] = d.payload_off;
                s_pe[threadIdx.x] = d.payload_off + (ok ? d.payload_len : 0);
                s_key[threadIdx.x] = d.masking_key;
            }
            __syncthreads();
            if (s_ps[0] >= t0 + kT) break;  // this and later rounds start past the tile
#pragma unroll
            for (int v = 0; v < VPT; ++v) {
                // last staged frame whose payload starts before the vector's end
                int lo = 0, hi = (int)cnt - 1, j = -1;
                while (lo <= hi) {
                    const int mid = (lo + hi) >> 1;
                    if (s_ps[mid] < va[v] + 16) {
                        j = mid;
                        lo = mid + 1;
                    } else {
                        hi = mid - 1;
                    }
                }
                for (; j >= 0; --j) {
                    if (s_pe[j] <= va[v]) {
                        if (s_pe[j] != s_ps[j]) break;  // empty payloads don't end the walk
                        continue;
                    }
                    add_mask(m[v], va[v], s_ps[j], s_pe[j], s_key[j]);
                }
            }
        }
    }

    if (STORE_AUX == 0) {
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            if (any_bits(m[v]) && va[v] + 16 <= vend)
                __builtin_nontemporal_store(data[v] ^ m[v], reinterpret_cast<u32x4*>(a.wire + va[v]));
        }
    } else {
        // buffer resource over this tile (wave-uniform: built from kernel args + blockIdx)
        const uint64_t room = vend > t0 ? vend - t0 : 0;
        const uint32_t nrec = (uint32_t)(room < kT ? room : kT);
        __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(a.wire + t0, 0, (int)nrec, 0x00020000);
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            if (any_bits(m[v]) && va[v] + 16 <= vend) {
                const u32x4 x = data[v] ^ m[v];
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, x), rs,
                    (uint32_t)(va[v] - t0), 0, STORE_AUX);
            }
        }
    }
    // the single vector that straddles the end of the wire: byte stores
    if (full_end != vend && full_end >= t0 && full_end < t0 + kT) {
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            if (va[v] == full_end && any_bits(m[v])) {
                const uint32_t mw[4] = {m[v].x, m[v].y, m[v].z, m[v].w};
                for (uint64_t bq = 0; full_end + bq < vend; ++bq) {
                    const uint8_t mb = (uint8_t)(mw[bq >> 2] >> (8 * (bq & 3)));
                    if (mb) a.wire[full_end + bq] ^= mb;
                }
            }
        }
    }
}

// After k_swalk_fused: a call over capacity (ws_over = its epoch) or whose look-back gave up
// has every connection's result rewritten — ERR_CAPACITY for those with frames, as
// k_stream_desc; ERR_DEVICE for all (nothing was unmasked: first_bad 0).  One workgroup.
__device__ inline void device_result(uvhttp_ws_stream_result_t& r);
__device__ inline void capacity_result(uvhttp_ws_stream_result_t& r);
__device__ inline void stream_fix(const BatchArgs& a, const Workspace& ws) {
    const bool fault = ws.ctl[kCtlFaultEp] == a.epoch;
    if (!fault && *a.s_over != a.epoch) return;
    for (uint32_t j = threadIdx.x; j < a.n_streams; j += blockDim.x) {
        uvhttp_ws_stream_result_t o = a.s_results[j];
        if (fault) device_result(o);
        else if (o.n_frames) capacity_result(o);
        a.s_results[j] = o;
    }
}

template <int BLOCK, int VPT, int STORE_AUX = 0>
__global__ __launch_bounds__(BLOCK) void k_unmask_inplace(
    BatchArgs a, const uvhttp_ws_frame_desc_t* __restrict__ desc, Workspace ws,
    uint64_t tile_base) {
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_PAYLOAD, false, tile_base);
    uint32_t n, nb;
    unmask_tile<BLOCK, VPT, STORE_AUX>(a, desc, ws, tile_base, n, nb, stamp_);  // resolves the epoch
    // batch in-place decode: the first ceil(n / BLOCK) workgroups then do k_finalize's work
    // (statuses after the first failure become SKIPPED — frames no tile reads — and the
    // summary); the launch covers max(tiles, those blocks).  After the tile, so the tile's
    // workspace and descriptor reads stay scalar loads no store of this kernel precedes.
    if (!a.streams && tile_base + blockIdx.x < (a.n + BLOCK - 1) / BLOCK) {
        resolve_epoch(a, ws);
        finalize_frames(a, const_cast<uvhttp_ws_frame_desc_t*>(desc), ws,
                        (uint32_t)(tile_base + blockIdx.x), BLOCK, nb);
    }
    if (a.s_results && tile_base + blockIdx.x == 0) {
        resolve_epoch(a, ws);
        stream_fix(a, ws);
    }
}

// ------------------------------------------------------------------------------------
// Stride batches (frame i at i * stride, stride >= kFusedMinStride), in place: the fused
// path.  k_plan's header gather reads one scattered 16-byte window per frame; from cold HBM
// that costs as much as streaming the whole wire (tools/hdr_probe.hip: 1 048 576 headers of
// 264-byte frames 52-60 us, the 277 MB wire read linearly 43 us).  The payload pass reads
// every byte anyway, so here it parses the headers itself:
//   k_unmask_stride  each workgroup stages its tile in LDS, parses the frames whose header
//                    starts in it (parse_hdr: every pre-state-machine check), writes their
//                    16-byte records, and unmasks every locally valid frame (speculatively:
//                    the state machine has not run yet);
//   k_plan (recs)    the scan + state machine from the records (contiguous, just written);
//   k_fixup          statuses after the first failure, the summary, and — only when a frame
//                    failed — the re-mask of the frames from the first failure on, which
//                    restores their bytes (XOR is its own inverse): the batch contract's
//                    "failing frame and everything after it are left untouched".
// ------------------------------------------------------------------------------------
constexpr uint64_t kFusedMinStride = 64;
// above this many wire bytes per frame the headers are few and the k_plan-first path is
// faster (its payload pass overlaps the descriptor lookup with the loads; tools/fused_sweep.py,
// profiles/r03p8_fused_sweep.txt: fused wins by 7 us at 2 KiB frames, loses by 4 at 3 KiB).
// 16 KiB fused tiles made the sweep favour fusing up to 8 KiB (r03p35_fused_tiles.txt), but
// the C2 bench itself (4 KiB frames) lost 5 % fused: 2217-2255 vs 2357-2367 GiB/s (r03p36)
constexpr uint64_t kFusedMaxAvg = 2560;
// k_unmask_stride's third role (AUX == kSpecCompact): the speculative pass of a compact stride
// batch (run_decode)
constexpr int kSpecCompact = 100;

// 16 bytes at byte offset r of an LDS-staged tile, from the two aligned vectors around it
__device__ inline u32x4 lds_window(const u32x4* tile, uint32_t r) {
    const u32x4 v0 = tile[r >> 4], v1 = tile[(r >> 4) + 1];
    uint64_t x0 = v0.x | ((uint64_t)v0.y << 32), x1 = v0.z | ((uint64_t)v0.w << 32);
    uint64_t x2 = v1.x | ((uint64_t)v1.y << 32);
    const uint64_t x3 = v1.z | ((uint64_t)v1.w << 32);
    const uint32_t dd = r & 15;
    if (dd & 8) {
        x0 = x1;
        x1 = x2;
        x2 = x3;
    }
    const uint32_t sh = (dd & 7) * 8;
    const uint64_t r0 = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
    const uint64_t r1 = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
    return u32x4{(uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32)};
}

// x / s for x < 2^24 (tile-relative offsets): a float reciprocal and one correction step
__device__ inline uint32_t div_small(uint32_t x, uint32_t s, float inv_s) {
    uint32_t q = (uint32_t)((float)x * inv_s);
    if (q * s > x) --q;
    else if ((q + 1) * s <= x) ++q;
    return q;
}

// a payload bound relative to the tile start t0 as int32: far bounds are clamped to
// [-64, kT + 64], a start keeping its value mod 4 (the key's byte phase for the tile's vectors)
__device__ inline int32_t rel_clamp(uint64_t x, uint64_t t0, uint64_t kT, bool keep_phase) {
    if (x < t0 && t0 - x > 64) {
        const int32_t ph = keep_phase ? (int32_t)((t0 - x) & 3u) : 0;
        return -64 - ph;  // (x - t0) mod 4 == (-ph) mod 4
    }
    if (x >= t0 + kT + 64) return (int32_t)(kT + 64);
    return (int32_t)((int64_t)x - (int64_t)t0);
}

// summary-only decode: what the fragment state machine and the summary need of one parsed frame
constexpr uint64_t kSumMinStride = 140;  // a control frame (<= 125 B of payload, header <= 10 B
                                         // even non-minimal, + key) is shorter than any slot
constexpr uint32_t kSiOk = 1u, kSiData = 2u, kSiFin = 4u, kSiStart = 8u, kSiZero = 16u, kSiClose = 32u;
constexpr uint32_t kSiHmShift = 8;  // header + key bytes in bits 8..15 (payload = slot - them)
__device__ constexpr uint32_t kHm[6] = {2u, 4u, 6u, 8u, 10u, 14u};  // every header + key size
__device__ inline uint32_t sum_info(const uvhttp_ws_frame_desc_t& d) {
    uint32_t x = ((uint32_t)d.header_size + ((d.flags & UVHTTP_WS_FLAG_MASK) ? 4u : 0u)) << kSiHmShift;
    if (d.status == UVHTTP_WS_FRAME_OK) x |= kSiOk;
    if (d.opcode <= 2) x |= kSiData;
    if (d.opcode == 1 || d.opcode == 2) x |= kSiStart;
    if (d.flags & UVHTTP_WS_FLAG_FIN) x |= kSiFin;
    if (d.payload_len == 0) x |= kSiZero;
    if (d.opcode == 8) x |= kSiClose;
    return x;
}
// the data frame leaves a message open: FIN = 0 and not a zero-length start, whose empty first
// fragment allocates nothing (src/uvhttp_websocket.c:794-816 + :964; kLastOpen in the scan)
__device__ inline bool si_open(uint32_t x) {
    return (x & kSiData) && !(x & kSiFin) && !((x & kSiStart) && (x & kSiZero));
}
// the one byte per frame the summary-only payload pass leaves for k_sum_scan: locally valid,
// data frame, FIN, start, BINARY (a compact decode's message opcode), and the header + key size
// class (kHm)
constexpr uint32_t kI8Ok = 1u, kI8Data = 2u, kI8Fin = 4u, kI8Start = 8u, kI8Bin = 16u, kI8HmShift = 5;
// a data frame that is not the batch's last leaves a message open iff it has no FIN: its payload
// fills a slot of >= kSumMinStride bytes, so it is never a zero-length start (si_open)
__device__ inline bool i8_open(uint32_t x) { return (x & kI8Data) && !(x & kI8Fin); }
__device__ inline uint8_t info8_of(const uvhttp_ws_frame_desc_t& d) {
    const uint32_t x = sum_info(d);
    const uint32_t hm = x >> kSiHmShift;
    const uint32_t c = hm == 2 ? 0u : hm == 4 ? 1u : hm == 6 ? 2u : hm == 8 ? 3u : hm == 10 ? 4u : 5u;
    return (uint8_t)(((x & kSiOk) ? kI8Ok : 0u) | ((x & kSiData) ? kI8Data : 0u) |
                     ((x & kSiFin) ? kI8Fin : 0u) | ((x & kSiStart) ? kI8Start : 0u) |
                     (d.opcode == 2 ? kI8Bin : 0u) | (c << kI8HmShift));
}
// add_mask on tile-relative int32 positions (vector at r, payload [ps, pe))
__device__ inline void add_mask_rel(u32x4& m, int32_t r, int32_t ps, int32_t pe, uint32_t key) {
    if (pe <= r || ps >= r + 16) return;
    const uint32_t rk = rotr32(key, 8u * (uint32_t)((r - ps) & 3));
    if (ps <= r && r + 16 <= pe) {
        m = u32x4{rk, rk, rk, rk};
        return;
    }
    const int lo = ps > r ? ps - r : 0;
    const int hi = pe < r + 16 ? pe - r : 16;
    m.x |= rk & lane_bytes(lo, hi, 0);
    m.y |= rk & lane_bytes(lo, hi, 1);
    m.z |= rk & lane_bytes(lo, hi, 2);
    m.w |= rk & lane_bytes(lo, hi, 3);
}

// what the payload pass leaves per frame: a 16-byte record (k_plan on records), an info byte
// (the summary-only scan), or both (records for k_desc_emit, info bytes for its scan)
constexpr int kLeaveRec = 0, kLeaveInfo = 1, kLeaveBoth = 2;
template <int BLOCK, int VPT, int AUX = 18, int SUM = kLeaveRec>
__global__ __launch_bounds__(BLOCK) void k_unmask_stride(BatchArgs a, Workspace ws, uint64_t tile_base) {
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_PAYLOAD, false, tile_base);
    constexpr uint64_t kT = (uint64_t)BLOCK * VPT * 16;
    constexpr int kMaxF = (int)(kT / kFusedMinStride) + 2;  // frames touching one tile
    __shared__ u32x4 s_tile[BLOCK * VPT + 1];               // the tile + the 16 bytes after
    // each frame's payload [ps, pe) relative to t0, clamped to int32 keeping ps mod 4 (the
    // key's byte phase), and key: one 16-byte LDS entry, read with one ds_read_b128
    __shared__ int4 s_fr[kMaxF];
    __shared__ u32x4 s_h0;                                  // header of the frame covering t0

    const uint64_t t0 = (tile_base + stamp_.anchor_s(blockIdx.x)) * kT;
    const uint64_t vend = a.wire_len;
    const uint64_t full_end = vend & ~(uint64_t)15;
    const uint64_t clamp_va = full_end ? full_end - 16 : 0;
    const uint64_t S = a.frame_stride;
    const uint32_t n = a.n;

    u32x4 data[VPT];
    uint64_t va[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        va[v] = t0 + ((uint64_t)v * BLOCK + threadIdx.x) * 16u;
        const uint64_t la = va[v] < full_end ? va[v] : clamp_va;
        data[v] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.wire + la));
    }
    // frames of this tile: fbase covers t0 (or is the last frame), fb starts last in it
    const uint64_t q0 = div_stride(a, t0);
    const uint32_t fbase = (uint32_t)(q0 < n ? q0 : n - 1);
    const uint64_t qb = div_stride(a, t0 + kT - 1);
    const uint32_t fb = (uint32_t)(qb < n ? qb : n - 1);
    const uint64_t obase = (uint64_t)fbase * S;
    // the two windows outside the tile, issued with the tile's loads: the header of the frame
    // that started before t0, and the 16 bytes after the tile (a header near the tile's end)
    u32x4 extra = u32x4{0, 0, 0, 0};
    if (threadIdx.x == 0 && obase < t0) extra = load16_at(a.wire, vend, obase);
    if (threadIdx.x == 1) extra = load16_at(a.wire, vend, t0 + kT);

#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        u32x4 x = data[v];
        // the vector straddling the end of the wire: its real bytes (zeros past the end)
        if (va[v] == full_end && full_end < vend) x = load16_at(a.wire, vend, full_end);
        s_tile[v * BLOCK + threadIdx.x] = x;
    }
    if (threadIdx.x == 0) s_h0 = extra;
    if (threadIdx.x == 1) s_tile[BLOCK * VPT] = extra;
    __syncthreads();

    // parse: thread j takes frame fbase + j (loops for frames smaller than kT / BLOCK);
    // consecutive lanes on consecutive frames keep the LDS header reads and the record stores
    // dense (spreading the frames over all four waves measured 5 us slower on C4, r03p7)
    const uint32_t nf = fb - fbase + 1;
    for (uint32_t j = threadIdx.x; j < nf; j += BLOCK) {
        const uint32_t f = fbase + j;
        const uint64_t o = (uint64_t)f * S;
        // (a header starting in the tile: 16 bytes at its tile offset from LDS)
        const u32x4 hv = o < t0 ? s_h0 : lds_window(s_tile, (uint32_t)(o - t0));
        uvhttp_ws_frame_desc_t d;
        (void)parse_hdr(a, f, seg_info(a, f, n), o, hv, d);
        if (o >= t0) {  // (a frame that started earlier: its own tile's)
            // summary-only decode: one info byte per frame (k_sum_scan runs the state machine
            // on them); else the frame's 16-byte record for k_plan
            if constexpr (SUM == kLeaveInfo) {
                reinterpret_cast<uint8_t*>(a.recs)[f] = info8_of(d);
            } else {
                a.recs[f] = rec8_of_desc(d);
                if constexpr (SUM == kLeaveBoth) ws.info[f] = info8_of(d);
            }
        }
        const bool ok = d.status == UVHTTP_WS_FRAME_OK;
        // speculative compact pass: the frame is uniform (a locally valid data frame with the
        // batch's uniform payload length and header + key bytes), so it goes to f * spec_P
        const bool uniform = AUX == kSpecCompact && ok && d.opcode <= 2 && d.payload_len == a.spec_P &&
                             d.header_size + ((d.flags & UVHTTP_WS_FLAG_MASK) ? 4u : 0u) == S - a.spec_P;
        s_fr[j] = int4{rel_clamp(d.payload_off, t0, kT, true),
                       rel_clamp(d.payload_off + (ok ? d.payload_len : 0), t0, kT, false),
                       (int32_t)d.masking_key, uniform ? 1 : 0};
    }
    // AUX < 0: the records-only pass of a compact stride decode (the wire stays masked)
    if constexpr (AUX < 0) return;
    __syncthreads();
    if constexpr (AUX == kSpecCompact) {
        // The speculative compact pass: the tile's payload bytes of uniform frames go to arena
        // offset f * P + q (P = spec_P, q = byte within the payload) — where the compact decode
        // puts them when every frame before f is uniform and delivered, which k_plan checks
        // (ws.spec_bad; k_spec_fix redoes the call with the full scatter otherwise).  The bytes
        // of wire [t0, e) land in one contiguous arena range [X0, X1), written as aligned
        // 16-byte vectors assembled from the tile in LDS (streaming stores: no dirty lines left
        // for the next kernel's reads), bytewise only at the range's two ends and around a
        // frame that is not uniform.  The wire itself stays masked, as in every compact decode.
        const uint64_t P = a.spec_P, D = S - P;  // D: header + key bytes of a uniform frame
        const uint64_t e = t0 + kT < vend ? t0 + kT : vend;
        if (e <= t0) return;
        const uint64_t pa = (uint64_t)fbase * S + D;  // fbase's payload start
        const uint64_t X0 = (uint64_t)fbase * P + (t0 > pa ? t0 - pa : 0);
        const uint64_t qe = div_stride(a, e - 1);
        const uint64_t fe = qe < n ? qe : n - 1;
        const uint64_t pe = fe * S + D;
        uint64_t X1 = fe * P + (e > pe ? (e - pe < P ? e - pe : P) : 0);
        if (X1 > a.arena_cap) X1 = a.arena_cap;
        if (X0 >= X1) return;
        const uint64_t base = X0 & ~(uint64_t)15;
        const uint32_t nvec = (uint32_t)((X1 - base + 15) >> 4);
        const uint32_t P32 = (uint32_t)P;
        const float inv_p = 1.0f / (float)P32;
        const uint64_t room = a.arena_cap - base;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            a.arena + base, 0, (int)(room < kT + 64 ? room : kT + 64), 0x00020000);
        for (uint32_t k = threadIdx.x; k < nvec; k += BLOCK) {
            const uint64_t ov = base + 16ull * k;
            const uint64_t lo = ov > X0 ? ov : X0, hi = ov + 16 < X1 ? ov + 16 : X1;
            // the common vector: inside the range and inside one uniform frame's payload (every
            // vector when P is a multiple of 16) — one window of the tile XOR the rotated key
            if (lo == ov && hi == ov + 16) {
                const uint32_t rx = (uint32_t)(ov - (uint64_t)fbase * P);
                const uint32_t jr = div_small(rx, P32, inv_p);
                const uint32_t q = rx - jr * P32;
                const int4 fr = s_fr[jr];
                if (q + 16 <= P32 && fr.w) {
                    const uint32_t rw = (uint32_t)(((uint64_t)fbase + jr) * S + D + q - t0);
                    const uint32_t rk = rotr32((uint32_t)fr.z, 8u * (q & 3u));
                    const u32x4 outv = lds_window(s_tile, rw) ^ u32x4{rk, rk, rk, rk};
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, outv), rs,
                        (uint32_t)(ov - base), 0, 18);
                    continue;
                }
            }
            unsigned __int128 acc = 0;
            uint32_t valid = 0;
            for (uint64_t x = lo; x < hi;) {
                // frame of arena byte x relative to fbase (x - fbase * P < kT + 2 P: 32-bit)
                const uint32_t rx = (uint32_t)(x - (uint64_t)fbase * P);
                const uint32_t jr = div_small(rx, P32, inv_p);
                const uint32_t q = rx - jr * P32;
                uint64_t run_end = x + (P32 - q);
                if (run_end > hi) run_end = hi;
                const int4 fr = s_fr[jr];
                if (fr.w) {
                    const uint32_t len = (uint32_t)(run_end - x), off = (uint32_t)(x - ov);
                    const uint32_t rw = (uint32_t)(((uint64_t)fbase + jr) * S + D + q - t0);
                    const uint32_t rk = rotr32((uint32_t)fr.z, 8u * (q & 3u));
                    const u32x4 w = lds_window(s_tile, rw) ^ u32x4{rk, rk, rk, rk};
                    const unsigned __int128 v = ((unsigned __int128)(((uint64_t)w.w << 32) | w.z) << 64) |
                                                (((uint64_t)w.y << 32) | w.x);
                    const unsigned __int128 m = len >= 16 ? ~(unsigned __int128)0
                                                          : (((unsigned __int128)1 << (8 * len)) - 1);
                    acc |= (v & m) << (8 * off);
                    valid |= ((1u << len) - 1u) << off;
                }
                x = run_end;
            }
            if (valid == 0xFFFFu) {
                const u32x4 outv = {(uint32_t)acc, (uint32_t)(acc >> 32), (uint32_t)(acc >> 64),
                                    (uint32_t)(acc >> 96)};
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, outv), rs,
                    (uint32_t)(ov - base), 0, 18);
            } else if (valid) {
                for (uint32_t bq = 0; bq < 16; ++bq)
                    if (valid & (1u << bq)) a.arena[ov + bq] = (uint8_t)(acc >> (8 * bq));
            }
        }
        return;
    }

    // a payload lies inside its frame's slot, so only frames jl..jh (relative to fbase) can
    // touch the vector at tile offset r: frame of byte r = (r + d0) / S, d0 = t0 - obase.
    // 32-bit tile-relative arithmetic (r + d0 + 15 < kT + 2 S; a tile at or past the last
    // frame's start holds that frame alone, however far it reaches)
    const bool last_only = fbase + 1 >= n;
    const uint32_t S32 = (uint32_t)S;
    const uint32_t d0 = last_only ? 0u : (uint32_t)(t0 - obase);
    const float inv_s = 1.0f / (float)S32;
    const uint32_t jmax = fb - fbase;
    u32x4 m[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        m[v] = u32x4{0, 0, 0, 0};
        if (va[v] >= vend) continue;
        const uint32_t r = (uint32_t)((v * BLOCK + threadIdx.x) * 16);
        uint32_t jl = 0, jh = 0;
        if (!last_only) {
            jl = div_small(r + d0, S32, inv_s);
            jh = div_small(r + 15 + d0, S32, inv_s);
            jl = jl < jmax ? jl : jmax;
            jh = jh < jmax ? jh : jmax;
        }
        for (uint32_t j = jl; j <= jh; ++j) {
            const int4 fr = s_fr[j];
            add_mask_rel(m[v], (int32_t)r, fr.x, fr.y, (uint32_t)fr.z);
        }
    }
    const uint64_t room = vend > t0 ? vend - t0 : 0;
    const uint32_t nrec = (uint32_t)(room < kT ? room : kT);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.wire + t0, 0, (int)nrec, 0x00020000);
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        if (any_bits(m[v]) && va[v] + 16 <= vend) {
            const u32x4 x = data[v] ^ m[v];
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, x), rs,
                (uint32_t)(va[v] - t0), 0, AUX < 0 ? 0 : AUX);
        }
    }
    if (full_end != vend && full_end >= t0 && full_end < t0 + kT) {
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            if (va[v] == full_end && any_bits(m[v])) {
                const uint32_t mw[4] = {m[v].x, m[v].y, m[v].z, m[v].w};
                for (uint64_t bq = 0; full_end + bq < vend; ++bq) {
                    const uint8_t mb = (uint8_t)(mw[bq >> 2] >> (8 * (bq & 3)));
                    if (mb) a.wire[full_end + bq] ^= mb;
                }
            }
        }
    }
}

// XOR frame payload bytes [ps, pe) with the key again (one wave; 16-byte vectors inside,
// single bytes at the two ends, so no byte outside the payload is rewritten)
__device__ inline void remask_range(uint8_t* wire, uint64_t ps, uint64_t pe, uint32_t key) {
    const int lane = threadIdx.x & 63;
    const uint64_t a0 = (ps + 15) & ~(uint64_t)15, a1 = pe & ~(uint64_t)15;
    if (a0 >= a1) {
        for (uint64_t b = ps + lane; b < pe; b += 64) wire[b] ^= (uint8_t)(key >> (8 * ((b - ps) & 3)));
        return;
    }
    for (uint64_t b = ps + lane; b < a0; b += 64) wire[b] ^= (uint8_t)(key >> (8 * ((b - ps) & 3)));
    for (uint64_t b = a1 + lane; b < pe; b += 64) wire[b] ^= (uint8_t)(key >> (8 * ((b - ps) & 3)));
    const uint32_t rk = rotr32(key, 8u * (uint32_t)((a0 - ps) & 3u));
    for (uint64_t v = a0 + 16ull * lane; v < a1; v += 16ull * 64) {
        u32x4* p = reinterpret_cast<u32x4*>(wire + v);
        *p = *p ^ u32x4{rk, rk, rk, rk};
    }
}

// After the fused path's k_plan: statuses after the first failure become SKIPPED, block 0
// writes the summary, and every frame the payload pass unmasked from the first failure on is
// masked again.  A look-back give-up (device fault) claimed first_bad = 0: all is restored.
__global__ __launch_bounds__(kBlock) void k_fixup(BatchArgs a, uvhttp_ws_frame_desc_t* desc,
                                                  Workspace ws) {
    resolve_epoch(a, ws);
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_FIXUP);
    const uint32_t n = a.n;
    const uint32_t nb = first_bad_of(a, ws, n);
    const bool fault = device_fault(a, ws);
    const uint64_t tid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t nthreads = (uint64_t)gridDim.x * kBlock;
    if (blockIdx.x == 0 && threadIdx.x < 64) {
        if (fault) {
            if (threadIdx.x == 0) {
                uvhttp_ws_batch_summary_t s;
                memset(&s, 0, sizeof(s));
                s.n_frames = n;
                s.status = -1;
                s.first_status = UVHTTP_WS_FRAME_ERR_DEVICE;
                *a.summary = s;
            }
        } else {
            write_summary(a, desc, ws, nb);
        }
    }
    if (nb >= n) return;  // every frame delivered: nothing to undo
    for (uint64_t i = tid; i < n; i += nthreads)
        if (i > nb || fault) skip_desc(a, desc, i);
    const uint64_t wave = tid >> 6, nwaves = nthreads >> 6;
    for (uint64_t i = nb + wave; i < n; i += nwaves) {
        const FrameRec r = rec_at(a, a.recs[i], (uint32_t)i);
        if (r.status != UVHTTP_WS_FRAME_OK || r.payload_len == 0) continue;  // not unmasked
        uvhttp_ws_frame_desc_t d;
        desc_of_rec(r, i * a.frame_stride, d);
        remask_range(a.wire, d.payload_off, d.payload_off + d.payload_len, d.masking_key);
    }
}

// ------------------------------------------------------------------------------------
// Summary-only decode, after k_unmask_stride<..., SUM = true> (which left one info byte per
// frame and unmasked every locally valid frame):
//   k_sum_scan  4 frames per thread (kScanFpt): the fragment state machine — with every frame before a
//               delivered one delivered, no control frame filling a slot but the last (stride >=
//               kSumMinStride) and no max_message_size check able to fire (run_decode's bound),
//               the state before frame f is "the latest data frame before f left a message
//               open" (src/uvhttp_websocket.c:950-1015: CONT needs an open message, a start must
//               not meet one) — then the summary's sums up to the first failure, per block
//               (ordered); a block with a failure claims first_bad;
//   k_sum_tail  with first_bad final: every block re-masks the frames the payload pass
//               unmasked from the first failure on (headers intact: parsed again from the wire);
//               block 0 combines the scan blocks' parts in order, adds the last frame's (the
//               scan leaves it out: its slot may be longer than the stride) and writes the
//               summary (write_summary's fields).
// No block waits for another: nothing here can give up.  (Computing the parts inside the
// payload pass, one per tile, cost that bandwidth-bound kernel 7 us on C4: 91.8 -> 99.2.)
// ------------------------------------------------------------------------------------
__device__ inline TilePart shfl_down_part(const TilePart& p, int d) {
    TilePart r;
    r.pay = __shfl_down(p.pay, d, 64);
    r.seg = __shfl_down(p.seg, d, 64);
    r.nfin = __shfl_down(p.nfin, d, 64);
    r.ls = __shfl_down(p.ls, d, 64);
    r.last = __shfl_down(p.last, d, 64);
    r.bits = __shfl_down(p.bits, d, 64);
    r.ff = __shfl_down(p.ff, d, 64);
    r.pad[0] = r.pad[1] = r.pad[2] = 0;
    return r;
}

// ordered reduction over the block's NT threads (thread t holds element t): thread 0 gets all
template <int NT>
__device__ TilePart block_reduce_parts(const TilePart& v) {
    __shared__ TilePart s_p[NT];
    s_p[threadIdx.x] = v;
    __syncthreads();
    TilePart r = part_identity();
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
#pragma unroll
        for (int k = 0; k < NT / 64; ++k) r = part_combine(r, s_p[lane * (NT / 64) + k]);
        // lane l holds [l, l + 2d) after step d
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const TilePart o = shfl_down_part(r, d);
            if (lane + d < 64) r = part_combine(r, o);
        }
    }
    __syncthreads();
    return r;
}

// frames per k_sum_scan thread: one 4-byte load of info bytes.  (16 per thread — one 16-byte
// load — left one wave per SIMD walking its frames serially: 10.4 us on C4; rocprofv3, r05k)
constexpr uint32_t kScanFpt = 4;

// a frame the speculative compact pass placed at f * P: a data frame whose header + key take
// the slot's D = stride - P bytes (the payload then fills the rest: P bytes)
__device__ inline bool i8_uniform(uint32_t x, uint64_t D) {
    return (x & kI8Data) && kHm[x >> kI8HmShift] == D;
}

// the info byte of frame f from its record (k_desc_emit's scan over the records)
__device__ inline uint32_t info_of_rec(const FrameRec& r, uint64_t S, uint32_t f) {
    uvhttp_ws_frame_desc_t d;
    desc_of_rec(r, (uint64_t)f * S, d);
    return info8_of(d);
}
__device__ inline uint32_t info_of_rec(const BatchArgs& a, const FrameRec8& p, uint64_t S, uint32_t f) {
    return info_of_rec(rec_at(a, p, f), S, f);
}

template <bool COMPACT, uint32_t KIND = UVHTTP_WS_STAMP_PLAN, bool FROM_REC = false>
__global__ __launch_bounds__(kBlock) void k_sum_scan(BatchArgs a, Workspace ws) {
    resolve_epoch(a, ws);
    StampScope stamp_(a.stamp, a.epoch, KIND);
    const uint32_t n = a.n;
    const uint64_t S = a.frame_stride;
    const uint64_t D = S - a.spec_P;
    const uint8_t* info = reinterpret_cast<const uint8_t*>(a.recs);
    const uint32_t F0 = (blockIdx.x * kBlock + threadIdx.x) * kScanFpt;
    uint32_t w = 0u;
    if constexpr (FROM_REC) {  // the info bytes rebuilt from the thread's 4 records (64 B)
        FrameRec8 r[kScanFpt];
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k) r[k] = a.recs[F0 + k < n ? F0 + k : n - 1];
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k)
            if (F0 + k < n) w |= info_of_rec(a, r[k], S, F0 + k) << (8 * k);
    } else {
        // (info bytes past n are never used; the buffer holds at least n + 16)
        w = F0 < n ? *reinterpret_cast<const uint32_t*>(info + F0) : 0u;
    }
    // the frame before this thread's first: the previous lane's last byte (lane 0: a load)
    const uint32_t up = __shfl_up(w, 1, 64);
    uint32_t pb = (threadIdx.x & 63) ? up >> 24
                                     : (F0 > 0 && F0 < n ? (FROM_REC ? info_of_rec(a, a.recs[F0 - 1], S, F0 - 1)
                                                                     : (uint32_t)info[F0 - 1])
                                                         : 0u);
    TilePart acc = part_identity();
    uint32_t sb = kNoFrame;  // compact: the thread's first delivered frame not at f * P
#pragma unroll
    for (uint32_t k = 0; k < kScanFpt; ++k) {
        const uint32_t f = F0 + k;
        if (f >= n) break;
        const uint32_t x = (w >> (8 * k)) & 0xFF;
        uint32_t p = f ? pb : 0u;  // (nothing before frame 0: no message open)
        // frames that are not data frames — reserved opcodes 3-7, which the reference delivers
        // leaving the fragment state as it was — may sit between f and the data frame that
        // decides: walk back to it; each such frame is walked over by one data frame at most
        if ((x & kI8Ok) && (x & kI8Data) && f > 0 && (p & kI8Ok) && !(p & kI8Data)) {
            for (uint32_t g = f - 1;;) {
                if (g == 0) {
                    p = 0u;
                    break;
                }
                --g;
                const uint32_t gi = g >= F0 ? (w >> (8 * (g - F0))) & 0xFF
                                            : FROM_REC ? info_of_rec(a, a.recs[g], S, g) : (uint32_t)info[g];
                if (!(gi & kI8Ok)) {  // a failure before f decides the batch anyway
                    p = 0u;
                    break;
                }
                if (gi & kI8Data) {
                    p = gi;
                    break;
                }
            }
        }
        if (!(x & kI8Ok) || ((x & kI8Data) && i8_open(p) == ((x & kI8Start) != 0))) {
            acc.ff = f;
            break;
        }
        if (f + 1 < n) {  // (the last frame's part is the tail's)
            const uint64_t plen = S - kHm[x >> kI8HmShift];
            acc.pay += plen;
            if (x & kI8Data) {
                if (x & kI8Start) {
                    acc.ls = f;
                    acc.seg = plen;
                    acc.bits = (x & kI8Bin) ? kPartBin : 0u;
                } else {
                    acc.seg += plen;
                }
                acc.nfin += (x & kI8Fin) ? 1u : 0u;
                acc.last = f;
                acc.bits = (acc.bits & ~kPartOpen) | (i8_open(x) ? kPartOpen : 0u);
            }
            if constexpr (COMPACT) {
                if (sb == kNoFrame && !i8_uniform(x, D)) sb = f;
            }
        }
        pb = x;
    }
    if constexpr (COMPACT) {
        if (sb != kNoFrame) tag_claim(ws.spec_bad, a.epoch, sb, a.cas_claims);  // (rare: a batch off the fast path)
    }
    const TilePart bp = block_reduce_parts<kBlock>(acc);
    if (threadIdx.x == 0) {
        reinterpret_cast<TilePart*>(ws.parts)[blockIdx.x] = bp;
        if (bp.ff != kNoFrame) tag_claim(ws.first_bad, a.epoch, bp.ff, a.cas_claims);
    }
}

constexpr uint32_t kSumTailGrid = 128;  // k_sum_tail blocks (all re-mask after a failure)

// the combination of parts [0, hi) in order, in every thread of the block (each thread a run
// of consecutive parts, kU loads in flight)
// (kU parts in flight per thread: 8 for k_sum_tail; k_desc_emit takes 2 — with 8 its block 0's
// summary set the whole kernel's registers, 146 VGPRs and 3 waves per SIMD, against 62)
template <uint32_t kU = 8>
__device__ TilePart parts_prefix(const TilePart* parts, uint32_t hi) {
    __shared__ TilePart s_res;
    const uint32_t per = (hi + kBlock - 1) / kBlock;
    const uint32_t p0 = threadIdx.x * per;
    TilePart acc = part_identity();
    for (uint32_t pb = p0; pb < p0 + per && pb < hi; pb += kU) {
        TilePart r[kU];
#pragma unroll
        for (uint32_t k = 0; k < kU; ++k) r[k] = pb + k < p0 + per && pb + k < hi ? parts[pb + k] : part_identity();
#pragma unroll
        for (uint32_t k = 0; k < kU; ++k) acc = part_combine(acc, r[k]);
    }
    const TilePart tot = block_reduce_parts<kBlock>(acc);
    if (threadIdx.x == 0) s_res = tot;
    __syncthreads();
    return s_res;
}

// the summary of a summary-only decode from the parts of frames [0, n - 1) combined (tot), the
// last frame's header (dl) and the first failure nb (thread 0)
__device__ void sum_summary(const BatchArgs& a, TilePart tot, const uvhttp_ws_frame_desc_t& dl,
                            uint32_t nb, bool compact) {
    const uint32_t n = a.n;
    const uint64_t S = a.frame_stride;
    uvhttp_ws_batch_summary_t sm;
    sm.n_frames = n;
    sm.n_delivered = nb < n ? nb : n;
    sm.first_status = 0;
    sm.state_closed = 0;
    if (nb < n) {  // its local status, or (locally valid) the fragment check's
        uvhttp_ws_frame_desc_t d;
        (void)parse_one(a, nb, seg_info(a, nb, n), d);
        sm.first_status = d.status != UVHTTP_WS_FRAME_OK ? d.status : UVHTTP_WS_FRAME_ERR_FRAGMENT;
        sm.consumed_bytes = (uint64_t)nb * S;
    } else {  // the last frame was delivered: its part
        const uint32_t x = sum_info(dl);
        TilePart lp = part_identity();
        lp.pay = dl.payload_len;
        if (x & kSiData) {
            lp.seg = dl.payload_len;
            lp.nfin = (x & kSiFin) ? 1u : 0u;
            lp.ls = (x & kSiStart) ? n - 1 : kNoFrame;
            lp.last = n - 1;
            lp.bits = si_open(x) ? kPartOpen : 0u;
        }
        tot = part_combine(tot, lp);
        sm.state_closed = (x & kSiClose) ? 1u : 0u;
        sm.consumed_bytes = (uint64_t)(n - 1) * S + dl.wire_len;
    }
    sm.status = sm.first_status < 0 ? -1 : 0;
    sm.payload_bytes = tot.pay;
    sm.n_messages = tot.nfin;
    sm.arena_bytes = compact ? tot.pay : 0;  // (compact: every delivered frame is a data frame)
    sm.pending_bytes = (tot.last != kNoFrame && (tot.bits & kPartOpen)) ? tot.seg : 0;
    *a.summary = sm;
}

__global__ __launch_bounds__(kBlock) void k_sum_tail(BatchArgs a, Workspace ws, uint32_t n_parts) {
    resolve_epoch(a, ws);
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_FIXUP);
    const uint32_t n = a.n;
    // the last frame's header (its part of the summary), read first
    uvhttp_ws_frame_desc_t dl;
    if (blockIdx.x == 0 && threadIdx.x == 0) (void)parse_one(a, n - 1, seg_info(a, n - 1, n), dl);
    const uint32_t nb = first_bad_of(a, ws, n);
    if (nb < n) {  // a failure: restore the frames the payload pass unmasked from it on
        const uint64_t wave = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
        const uint64_t nwaves = (uint64_t)gridDim.x * (kBlock / 64);
        for (uint64_t i = nb + wave; i < n; i += nwaves) {
            uvhttp_ws_frame_desc_t d;
            (void)parse_one(a, (uint32_t)i, seg_info(a, (uint32_t)i, n), d);
            if (d.status == UVHTTP_WS_FRAME_OK && d.payload_len)
                remask_range(a.wire, d.payload_off, d.payload_off + d.payload_len, d.masking_key);
        }
    }
    if (blockIdx.x != 0) return;
    // block 0: the scan blocks' parts in order
    const TilePart tot = parts_prefix(reinterpret_cast<const TilePart*>(ws.parts), n_parts);
    if (threadIdx.x == 0) sum_summary(a, tot, dl, nb, false);
}

// block-wide exclusive scans of one count (sum) and one frame mark (max) per thread
__device__ inline void block_exscan_sum_max(uint32_t c, uint32_t l, uint32_t& ec, uint32_t& el) {
    __shared__ uint32_t s_c[kBlock / 64], s_l[kBlock / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t ic = c, il = l;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t oc = __shfl_up(ic, d, 64), ol = __shfl_up(il, d, 64);
        if (lane >= d) {
            ic += oc;
            il = ol > il ? ol : il;
        }
    }
    uint32_t xl = __shfl_up(il, 1, 64);
    if (lane == 0) xl = 0;
    if (lane == 63) {
        s_c[wv] = ic;
        s_l[wv] = il;
    }
    __syncthreads();
    uint32_t bc = 0, bl = 0;
    for (int k = 0; k < wv; ++k) {
        bc += s_c[k];
        bl = s_l[k] > bl ? s_l[k] : bl;
    }
    ec = bc + ic - c;
    el = xl > bl ? xl : bl;
}

// block-wide exclusive scan of a sum (uint64: four 16-bit counters packed, no carries between
// them while each stays below 2^16) -> the thread's exclusive prefix and the block's total
__device__ inline void block_exscan_u64(uint64_t v, uint64_t& ex, uint64_t& tot) {
    __shared__ uint64_t s_w[kBlock / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; ++k) {
        before += k < wv ? s_w[k] : 0u;
        all += s_w[k];
    }
    ex = before + inc - v;
    tot = all;
}

// what a block of k_sum_msgs needs of the scan parts before it: FIN frames (sum) and the
// latest start with its BINARY bit as ((ls + 1) << 1 | bin) (max; 0 = none) — commutative, so
// each thread loads the parts t, t + kBlock, ... (one 16-byte load each: nfin, ls, last, bits)
__device__ inline void parts_fin_start(const TilePart* parts, uint32_t hi, uint32_t& nfin, uint32_t& key) {
    __shared__ uint32_t s_c[kBlock / 64], s_k[kBlock / 64];
    uint32_t c = 0, k = 0;
    for (uint32_t pb = threadIdx.x; pb < hi; pb += kBlock) {
        const u32x4 q = *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint8_t*>(parts + pb) + 16);
        c += q.x;
        const uint32_t kk = q.y == kNoFrame ? 0u : ((q.y + 1) << 1) | ((q.w & kPartBin) ? 1u : 0u);
        k = kk > k ? kk : k;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        c += __shfl_xor(c, d, 64);
        const uint32_t o = __shfl_xor(k, d, 64);
        k = o > k ? o : k;
    }
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        s_c[wv] = c;
        s_k[wv] = k;
    }
    __syncthreads();
    nfin = 0;
    key = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        nfin += s_c[w];
        key = s_k[w] > key ? s_k[w] : key;
    }
}

// Summary-only compact decode, after k_sum_scan<true> (the parts of its blocks in ws.parts):
// the message table and the summary.  With every frame before the first failure a uniform
// data frame (the speculation held), message m ends at the m-th FIN frame f and starts at the
// latest start s <= f: arena [s P, (f + 1) P), frames s..f.  Block b takes the frames of scan
// block b again; the messages and the latest start before it come from parts [0, b) (sums and
// maxima, so no ordered combine).  Block 0 decides the speculation — a delivered frame off the
// uniform layout (k_sum_scan claimed spec_bad) or a last frame that is not uniform sets
// ctl[kCtlGate] = epoch and k_plan + k_spec_fix decode the call again (messages written here
// are then overwritten or past n_messages) — and otherwise writes the last frame's message and
// the summary, which with every delivered frame P bytes of data needs no more than the FIN
// count, the latest start and whether the last delivered frame left its message open.
// (One launch after the scan; a single-block tail leaving ordered prefixes + this kernel took
// 6.4 + 2.0 us and a boundary on C4, every block combining full parts in order 9.2 us.)
// DESC (compact decode with descriptors, the payload pass leaving 16-byte records: FROM_REC):
// every block also writes its 1024 frames' descriptors as k_desc_emit does, data frames at their
// arena offset f * P; a call whose speculation failed has them rewritten by the fall-back.
template <bool FROM_REC = false, bool DESC = false>
__global__ __launch_bounds__(kBlock) void k_sum_msgs(BatchArgs a, Workspace ws, uint32_t n_parts,
                                                     uvhttp_ws_message_desc_t* msgs,
                                                     uvhttp_ws_frame_desc_t* desc = nullptr) {
    resolve_epoch(a, ws);
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_FINALIZE);
    const uint32_t n = a.n;
    const uint64_t S = a.frame_stride;
    const uint64_t P = a.spec_P;
    const bool head = blockIdx.x == 0;
    uvhttp_ws_frame_desc_t dl;
    if (head && threadIdx.x == 0) (void)parse_one(a, n - 1, seg_info(a, n - 1, n), dl);
    const uint32_t nb = first_bad_of(a, ws, n);
    const uint32_t sb = tag_get(*ws.spec_bad, a.epoch, n);
    const uint32_t end = nb < n - 1 ? nb : n - 1;  // frames [0, end) here, the last one is block 0's
    // (DESC without FROM_REC: records in a.recs, the payload pass's info bytes in ws.info)
    const uint8_t* info_b = (DESC && !FROM_REC) ? ws.info : reinterpret_cast<const uint8_t*>(a.recs);
    auto info_at = [&](uint32_t f) -> uint32_t {
        if constexpr (FROM_REC) return info_of_rec(a, a.recs[f], S, f);
        else return info_b[f];
    };
    const uint32_t F0 = (blockIdx.x * kBlock + threadIdx.x) * kScanFpt;
    uint32_t w = 0u;
    if constexpr (FROM_REC) {
        FrameRec8 r4[kScanFpt];
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k) r4[k] = a.recs[F0 + k < n ? F0 + k : n - 1];
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k)
            if (F0 + k < n) w |= info_of_rec(a, r4[k], S, F0 + k) << (8 * k);
    } else {
        w = F0 < n ? *reinterpret_cast<const uint32_t*>(info_b + F0) : 0u;
    }
    constexpr uint32_t kPartFrames = kBlock * kScanFpt;
    // block 0: the parts of every frame before `end` (a part stops at its first failure)
    const uint32_t hi = head ? (end / kPartFrames + 1 < n_parts ? end / kPartFrames + 1 : n_parts) : blockIdx.x;
    uint32_t pre_fin, pre_key;
    parts_fin_start(reinterpret_cast<const TilePart*>(ws.parts), hi, pre_fin, pre_key);
    const uint32_t tot_fin = pre_fin, tot_key = pre_key;
    if (head) pre_fin = pre_key = 0;
    uint32_t cnt = 0, ls1 = 0;  // FIN frames; latest start + 1 (0: none)
#pragma unroll
    for (uint32_t k = 0; k < kScanFpt; ++k) {
        const uint32_t f = F0 + k, x = (w >> (8 * k)) & 0xFF;
        if (f < end) {
            cnt += (x & kI8Fin) ? 1u : 0u;
            if (x & kI8Start) ls1 = f + 1;
        }
    }
    uint32_t ec, el;
    block_exscan_sum_max(cnt, ls1, ec, el);
    if (cnt) {
        uint32_t m = pre_fin + ec;
        const uint32_t pre_ls = pre_key ? (pre_key >> 1) - 1 : kNoFrame;
        uint32_t ls = el ? el - 1 : pre_ls;
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k) {
            const uint32_t f = F0 + k, x = (w >> (8 * k)) & 0xFF;
            if (f >= end) break;
            if (x & kI8Start) ls = f;
            if (x & kI8Fin) {
                // the start's opcode: its info byte, or — before the block — the prefix's bit
                const uint32_t xs = ls >= F0 ? (w >> (8 * (ls - F0))) & 0xFF
                                    : ls == pre_ls ? ((pre_key & 1u) ? kI8Bin : 0u) : info_at(ls);
                uvhttp_ws_message_desc_t md;
                md.arena_off = (uint64_t)ls * P;
                md.len = (uint64_t)(f - ls + 1) * P;
                md.first_frame = ls;
                md.last_frame = f;
                md.opcode = (xs & kI8Bin) ? 2 : 1;
                md.reserved = 0;
                msgs[m++] = md;
            }
        }
    }
    if constexpr (DESC) {  // (strided rounds, as k_desc_emit: contiguous loads and stores)
        const uint32_t B0 = blockIdx.x * kBlock * kScanFpt;
        FrameRec r[kScanFpt];
        uint32_t x[kScanFpt];
        {
            FrameRec8 p[kScanFpt];
#pragma unroll
            for (uint32_t k = 0; k < kScanFpt; ++k) {
                const uint32_t f = B0 + k * kBlock + threadIdx.x;
                p[k] = a.recs[f < n ? f : n - 1];
            }
#pragma unroll
            for (uint32_t k = 0; k < kScanFpt; ++k) {
                const uint32_t f = B0 + k * kBlock + threadIdx.x;
                r[k] = rec_at(a, p[k], f < n ? f : n - 1);
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k) {
            const uint32_t f = B0 + k * kBlock + threadIdx.x;
            x[k] = f < n ? (FROM_REC ? info_of_rec(r[k], S, f) : (uint32_t)info_b[f]) : 0u;
        }
        uint64_t v = 0;
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k) {
            const uint32_t f = B0 + k * kBlock + threadIdx.x;
            if (f < nb && f < n && (x[k] & kI8Data) && (x[k] & kI8Fin)) v += 1ull << (16 * k);
        }
        uint64_t ex, tot;
        block_exscan_u64(v, ex, tot);
        uint32_t round_base = head ? 0u : tot_fin;  // (tot_fin: FIN frames of parts [0, b))
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k) {
            const uint32_t f = B0 + k * kBlock + threadIdx.x;
            if (f < n) {
                uvhttp_ws_frame_desc_t d;
                desc_of_rec(r[k], (uint64_t)f * S, d);
                if (f < nb) {
                    if (is_data_op(d.opcode)) {
                        d.message = round_base + (uint32_t)((ex >> (16 * k)) & 0xFFFFu);
                        d.payload_off = (uint64_t)f * P;
                        if (d.flags & UVHTTP_WS_FLAG_FIN) d.flags |= UVHTTP_WS_FLAG_MSG_END;
                    }
                } else if (f == nb) {
                    if (d.status == UVHTTP_WS_FRAME_OK) d.status = UVHTTP_WS_FRAME_ERR_FRAGMENT;
                } else {
                    d.status = UVHTTP_WS_FRAME_SKIPPED;
                }
                store_desc(desc, f, d);
            }
            round_base += (uint32_t)((tot >> (16 * k)) & 0xFFFFu);
        }
    }
    if (!head || threadIdx.x != 0) return;
    const bool last_off = nb >= n && !(dl.opcode <= 2 && dl.payload_len == P &&
                                       dl.header_size + ((dl.flags & UVHTTP_WS_FLAG_MASK) ? 4u : 0u) == S - P);
    if (sb < nb || last_off) {
        ws.ctl[kCtlGate] = a.epoch;
        return;
    }
    uint32_t nfin = tot_fin;
    uint32_t ls = tot_key ? (tot_key >> 1) - 1 : kNoFrame;
    bool bin = tot_key & 1u;
    uvhttp_ws_batch_summary_t sm;
    sm.n_frames = n;
    sm.state_closed = 0;
    uint32_t nd;  // frames delivered, every one P bytes of data
    bool open;    // the last of them leaves its message open
    if (nb < n) {  // its local status, or (locally valid) the fragment check's
        nd = nb;
        uvhttp_ws_frame_desc_t d;
        (void)parse_one(a, nb, seg_info(a, nb, n), d);
        sm.first_status = d.status != UVHTTP_WS_FRAME_OK ? d.status : UVHTTP_WS_FRAME_ERR_FRAGMENT;
        sm.consumed_bytes = (uint64_t)nb * S;
        open = nb > 0 && !(info_at(nb - 1) & kI8Fin);
    } else {  // every frame, the last one (a uniform data frame) included
        nd = n;
        sm.first_status = 0;
        sm.consumed_bytes = (uint64_t)(n - 1) * S + dl.wire_len;
        if (dl.opcode != 0) {
            ls = n - 1;
            bin = dl.opcode == 2;
        }
        open = !(dl.flags & UVHTTP_WS_FLAG_FIN);
        if (!open) {  // the last frame's message
            uvhttp_ws_message_desc_t md;
            md.arena_off = (uint64_t)ls * P;
            md.len = (uint64_t)(n - ls) * P;
            md.first_frame = ls;
            md.last_frame = n - 1;
            md.opcode = bin ? 2 : 1;
            md.reserved = 0;
            msgs[nfin++] = md;
        }
    }
    sm.n_delivered = nd;
    sm.status = sm.first_status < 0 ? -1 : 0;
    sm.payload_bytes = (uint64_t)nd * P;
    sm.n_messages = nfin;
    sm.arena_bytes = sm.payload_bytes;
    sm.pending_bytes = open ? (uint64_t)(nd - ls) * P : 0;
    *a.summary = sm;
    if (open) {  // the open message (write_summary's entry; every fragment is P bytes)
        uvhttp_ws_message_desc_t md;
        md.arena_off = (uint64_t)ls * P;
        md.len = sm.pending_bytes;
        md.first_frame = ls;
        md.last_frame = nd - 1;
        md.opcode = bin ? 2 : 1;
        md.reserved = (uint32_t)P;
        msgs[nfin] = md;
    }
}

// ------------------------------------------------------------------------------------
// Descriptor decode of a stride batch in place (d_desc != NULL, the summary-only bounds: stride
// >= kSumMinStride, no message able to reach max_message_size), after k_unmask_stride<...,
// kLeaveBoth> (16-byte record + info byte per frame, every locally valid frame unmasked) and
// k_sum_scan (state machine on the info bytes, one part per 1024 frames, first_bad claimed):
// k_desc_emit is fully parallel — no look-back, no block waits for another.  Block b takes the
// 1024 frames of scan block b: message ids are the FIN data frames before a frame, i.e. the FIN
// counts of parts [0, b) (a sum: each thread loads a few parts, as k_sum_msgs does) plus a block
// scan; frames before first_bad are delivered (status OK, message id, MSG_END on a FIN data
// frame), first_bad keeps its local status or fails the fragment check (src/uvhttp_websocket.c:
// 964-996 — ERR_MESSAGE cannot fire under the bound), later frames are SKIPPED (skip_desc's
// form).  Then k_fixup's work: block 0 the summary (parts in order, as k_sum_tail), and after a
// failure each block re-masks its frames from first_bad on.  Replaces k_plan on the records + 
// k_fixup for these batches (C4: 27 + 2 us and a look-back).
// ------------------------------------------------------------------------------------
template <bool FROM_REC>
__global__ __launch_bounds__(kBlock) void k_desc_emit(BatchArgs a, Workspace ws, uint32_t n_parts,
                                                      uvhttp_ws_frame_desc_t* desc) {
    resolve_epoch(a, ws);
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_DESC_EMIT);
    const uint32_t n = a.n;
    const uint64_t S = a.frame_stride;
    const bool head = blockIdx.x == 0;
    const uint32_t nb = first_bad_of(a, ws, n);
    // the block's 1024 frames (scan block b's) in four rounds of 256: thread t takes frame
    // B0 + 256 k + t, so every record load and descriptor store of a wave is contiguous (a
    // thread per 4 consecutive frames stored 128-byte-strided descriptors: 15.6 us on C4)
    const uint32_t B0 = blockIdx.x * kBlock * kScanFpt;
    FrameRec r[kScanFpt];
    uint32_t x[kScanFpt];
    const uint32_t ilast = n - 1;
    {
        FrameRec8 p[kScanFpt];
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k) {
            const uint32_t f = B0 + k * kBlock + threadIdx.x;
            p[k] = a.recs[f < n ? f : ilast];
            if constexpr (!FROM_REC) x[k] = f < n ? ws.info[f] : 0u;
        }
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k) {
            const uint32_t f = B0 + k * kBlock + threadIdx.x;
            r[k] = rec_at(a, p[k], f < n ? f : ilast);
        }
    }
    if constexpr (FROM_REC) {
#pragma unroll
        for (uint32_t k = 0; k < kScanFpt; ++k) x[k] = info_of_rec(r[k], S, B0 + k * kBlock + threadIdx.x);
    }
    uint32_t pre_fin = 0, pre_key = 0;
    parts_fin_start(reinterpret_cast<const TilePart*>(ws.parts), blockIdx.x, pre_fin, pre_key);
    // FIN data frames among the delivered ones, per round (16-bit fields)
    uint64_t v = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanFpt; ++k) {
        const uint32_t f = B0 + k * kBlock + threadIdx.x;
        if (f < nb && f < n && (x[k] & kI8Data) && (x[k] & kI8Fin)) v += 1ull << (16 * k);
    }
    uint64_t ex, tot;
    block_exscan_u64(v, ex, tot);
    uint32_t round_base = pre_fin;
#pragma unroll
    for (uint32_t k = 0; k < kScanFpt; ++k) {
        const uint32_t f = B0 + k * kBlock + threadIdx.x;
        if (f < n) {
            uvhttp_ws_frame_desc_t d;
            desc_of_rec(r[k], (uint64_t)f * S, d);
            if (f < nb) {
                if (is_data_op(d.opcode)) {
                    d.message = round_base + (uint32_t)((ex >> (16 * k)) & 0xFFFFu);
                    if (d.flags & UVHTTP_WS_FLAG_FIN) d.flags |= UVHTTP_WS_FLAG_MSG_END;
                }
            } else if (f == nb) {
                if (d.status == UVHTTP_WS_FRAME_OK) d.status = UVHTTP_WS_FRAME_ERR_FRAGMENT;
            } else {
                d.status = UVHTTP_WS_FRAME_SKIPPED;
            }
            store_desc(desc, f, d);
        }
        round_base += (uint32_t)((tot >> (16 * k)) & 0xFFFFu);
    }
    if (head) {  // the summary (every block's part, in order), as k_sum_tail's block 0
        const TilePart tp = parts_prefix<2>(reinterpret_cast<const TilePart*>(ws.parts), n_parts);
        if (threadIdx.x == 0) {  // (the last frame parsed here: not live across the kernel)
            uvhttp_ws_frame_desc_t dl;
            (void)parse_one(a, n - 1, seg_info(a, n - 1, n), dl);
            sum_summary(a, tp, dl, nb, false);
        }
    }
    if (nb >= n) return;
    // a failure: restore this block's frames the payload pass unmasked from first_bad on (a
    // wave per frame, the records say which were locally valid)
    const uint32_t b1 = B0 + kBlock * kScanFpt < n ? B0 + kBlock * kScanFpt : n;
    const uint32_t wave = threadIdx.x >> 6;
    for (uint32_t i = (nb > B0 ? nb : B0) + wave; i < b1; i += kBlock / 64) {
        const FrameRec rr = rec_at(a, a.recs[i], i);
        if (rr.status != UVHTTP_WS_FRAME_OK || rr.payload_len == 0) continue;
        uvhttp_ws_frame_desc_t d;
        desc_of_rec(rr, (uint64_t)i * S, d);
        remask_range(a.wire, d.payload_off, d.payload_off + d.payload_len, d.masking_key);
    }
}

// ------------------------------------------------------------------------------------
// k_gather_compact: the roofline kernel of the compact decode.  One workgroup per
// BLOCK*VPT*16-byte tile of the message arena; lane t produces the aligned arena vectors of
// its tile.  Each vector's bytes come from the delivered data frame(s) covering it:
// out[o] = wire[ps_f + (o - aoff_f)] ^ key_f[(o - aoff_f) & 3].  The source window is
// unaligned (payload starts at header+key offsets) and read as one 16-byte load.
// ------------------------------------------------------------------------------------
__device__ inline u32x4 load16_any(const uint8_t* base, int64_t addr, uint64_t limit) {
    if (addr >= 0 && (uint64_t)addr + 16 <= limit) {
        u32x4 r;
        __builtin_memcpy(&r, base + addr, 16);
        return r;
    }
    uint32_t w[4] = {0, 0, 0, 0};
    for (int b = 0; b < 16; ++b) {
        const int64_t x = addr + b;
        if (x >= 0 && (uint64_t)x < limit) w[b >> 2] |= (uint32_t)base[x] << (8 * (b & 3));
    }
    return u32x4{w[0], w[1], w[2], w[3]};
}

// block-wide inclusive max-scan of one u64 per thread
template <int BLOCK>
__device__ uint64_t block_inclusive_max(uint64_t v) {
    __shared__ uint64_t wave_max[BLOCK / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(v, d, 64);
        if (lane >= d && o > v) v = o;
    }
    if (BLOCK > 64) {
        if (lane == 63) wave_max[wave] = v;
        __syncthreads();
        for (int w = 0; w < wave; ++w)
            if (wave_max[w] > v) v = wave_max[w];
        __syncthreads();
    }
    return v;
}

template <int BLOCK, int VPT>
__device__ __forceinline__ void gather_tile(const BatchArgs& a,
                                            const uvhttp_ws_frame_desc_t* __restrict__ desc,
                                            const Workspace& ws, uint64_t arena_bytes_cap,
                                            uint64_t tile_base, uint32_t n, uint32_t nb) {
    constexpr uint64_t kT = (uint64_t)BLOCK * VPT * 16;
    __shared__ uint64_t s_as[BLOCK];  // arena start of the data payload
    __shared__ uint64_t s_ae[BLOCK];  // arena end (== start for control frames)
    __shared__ uint64_t s_ps[BLOCK];  // wire offset of the payload
    __shared__ uint32_t s_key[BLOCK];

    const uint64_t t0 = (tile_base + blockIdx.x) * kT;
    if (nb == 0 || n == 0 || t0 >= a.n_arena_tiles * kMapTile) return;
    const uint32_t last = (nb < n ? nb : n) - 1;
    const uint64_t c0 = t0 / kMapTile, c1 = (t0 + kT - 1) / kMapTile + 1;
    const uint32_t f0 = tag_get(ws.arena_first[c0], a.epoch, kNoFrame);
    if (f0 > last) return;
    uint32_t f1 = (c1 < a.n_arena_tiles) ? tag_get(ws.arena_first[c1], a.epoch, kNoFrame) : last;
    if (f1 > last || f1 < f0) f1 = last;

    uint64_t oa[VPT];
    u32x4 out[VPT];
    bool touched[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        oa[v] = t0 + ((uint64_t)v * BLOCK + threadIdx.x) * 16u;
        out[v] = u32x4{0, 0, 0, 0};
        touched[v] = false;
    }
    uint64_t arena_end = 0;  // end of the delivered data payload staged so far

    // fast path (data frames of ~4 KiB and up): at most two data frames cover the tile; their
    // descriptors are uniform scalar loads, no LDS staging
    bool fast = false;
    if (f1 - f0 < 2) {
        const uvhttp_ws_frame_desc_t d0 = desc[f0];
        const uvhttp_ws_frame_desc_t d1 = desc[f1];
        if (d0.opcode <= 2 && d1.opcode <= 2) {
            fast = true;
            for (uint32_t f = f0; f <= f1; ++f) {
                const uvhttp_ws_frame_desc_t& d = f == f0 ? d0 : d1;
                const uint64_t fa = d.payload_off, fe = fa + d.payload_len;
                const uint64_t ps = frame_start(a, f) + d.header_size + ((d.flags & UVHTTP_WS_FLAG_MASK) ? 4u : 0u);
#pragma unroll
                for (int v = 0; v < VPT; ++v) {
                    if (fe <= oa[v] || fa >= oa[v] + 16) continue;
                    const int lo_b = fa > oa[v] ? (int)(fa - oa[v]) : 0;
                    const int hi_b = fe < oa[v] + 16 ? (int)(fe - oa[v]) : 16;
                    const int64_t wstart = (int64_t)ps + (int64_t)(oa[v] - fa);
                    const u32x4 w = load16_any(a.wire, wstart, a.wire_len);
                    const uint32_t rk = rotr32(d.masking_key, 8u * (uint32_t)((oa[v] - fa) & 3u));
                    const u32x4 sel{lane_bytes(lo_b, hi_b, 0), lane_bytes(lo_b, hi_b, 1),
                                    lane_bytes(lo_b, hi_b, 2), lane_bytes(lo_b, hi_b, 3)};
                    out[v] |= (w ^ u32x4{rk, rk, rk, rk}) & sel;
                    touched[v] = true;
                }
                if (fe > arena_end) arena_end = fe;
            }
        }
    }

    for (uint32_t base = f0; !fast && base <= f1; base += BLOCK) {
        const uint32_t cnt = (f1 - base + 1) < (uint32_t)BLOCK ? (f1 - base + 1) : BLOCK;
        uint64_t as = 0, ae = 0, ps = 0;
        uint32_t key = 0;
        bool data = false;
        if (threadIdx.x < cnt) {
            const uint32_t f = base + threadIdx.x;
            const uvhttp_ws_frame_desc_t d = desc[f];
            data = d.opcode <= 2;
            if (data) {
                as = d.payload_off;
                ae = as + d.payload_len;
                ps = frame_start(a, f) + d.header_size + ((d.flags & UVHTTP_WS_FLAG_MASK) ? 4u : 0u);
            }
            key = d.masking_key;
        }
        // control frames take the running arena end so s_as stays sorted
        uint64_t run = block_inclusive_max<BLOCK>(data ? ae : 0);
        if (run < arena_end) run = arena_end;
        __syncthreads();
        if (threadIdx.x < cnt) {
            s_as[threadIdx.x] = data ? as : run;
            s_ae[threadIdx.x] = data ? ae : run;
            s_ps[threadIdx.x] = ps;
            s_key[threadIdx.x] = key;
        }
        __syncthreads();
        if (cnt && s_ae[cnt - 1] > arena_end) arena_end = s_ae[cnt - 1];
        if (s_as[0] >= t0 + kT) break;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            // last staged frame starting before the vector's end
            int lo = 0, hi = (int)cnt - 1, j = -1;
            while (lo <= hi) {
                const int mid = (lo + hi) >> 1;
                if (s_as[mid] < oa[v] + 16) {
                    j = mid;
                    lo = mid + 1;
                } else {
                    hi = mid - 1;
                }
            }
            for (; j >= 0; --j) {
                const uint64_t fa = s_as[j], fe = s_ae[j];
                if (fe == fa) continue;  // control frame or empty payload
                if (fe <= oa[v]) break;
                const int lo_b = fa > oa[v] ? (int)(fa - oa[v]) : 0;
                const int hi_b = fe < oa[v] + 16 ? (int)(fe - oa[v]) : 16;
                // window byte b <- wire[ps + (oa + b - fa)]
                const int64_t wstart = (int64_t)s_ps[j] + (int64_t)(oa[v] - fa);
                const u32x4 w = load16_any(a.wire, wstart, a.wire_len);
                const uint32_t rk = rotr32(s_key[j], 8u * (uint32_t)((oa[v] - fa) & 3u));
                const u32x4 sel{lane_bytes(lo_b, hi_b, 0), lane_bytes(lo_b, hi_b, 1),
                                lane_bytes(lo_b, hi_b, 2), lane_bytes(lo_b, hi_b, 3)};
                out[v] |= (w ^ u32x4{rk, rk, rk, rk}) & sel;
                touched[v] = true;
            }
        }
    }

    const uint64_t lim = arena_end < arena_bytes_cap ? arena_end : arena_bytes_cap;
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        if (!touched[v] || oa[v] >= lim) continue;
        if (oa[v] + 16 <= lim) {
            __builtin_nontemporal_store(out[v], reinterpret_cast<u32x4*>(a.arena + oa[v]));
        } else {
            const uint32_t ow[4] = {out[v].x, out[v].y, out[v].z, out[v].w};
            for (uint64_t b = 0; b < 16 && oa[v] + b < lim; ++b)
                a.arena[oa[v] + b] = (uint8_t)(ow[b >> 2] >> (8 * (b & 3)));
        }
    }
}

template <int BLOCK, int VPT>
__global__ __launch_bounds__(BLOCK) void k_gather_compact(
    BatchArgs a, const uvhttp_ws_frame_desc_t* __restrict__ desc, Workspace ws,
    uint64_t arena_bytes_cap, uint64_t tile_base) {
    resolve_epoch(a, ws);
    // (no device stamp here: a StampScope in this kernel cost 2.6-2.8 % on C3 compact even with
    // stamps off, profiles/r04_gather_stamp_ab.txt — its timeline shows plan and finalize only)
    const uint32_t n = nframes(a);
    gather_tile<BLOCK, VPT>(a, desc, ws, arena_bytes_cap, tile_base, n, first_bad_of(a, ws, n));
    // (k_finalize stays a launch of its own here: folding it in like k_scatter_compact cost
    // 3 % on C3 compact — 1.330 -> 1.372 ms per step)
}

// ------------------------------------------------------------------------------------
// k_scatter_compact: the compact decode for small frames, driven by the WIRE instead of the
// arena.  The arena-driven gather must find a tile's frames before it knows what to load (map
// -> descriptors -> source loads: three dependent round trips per workgroup), which leaves
// frames of a few hundred bytes at ~4 TB/s.  Here each workgroup takes a wire tile like the
// in-place kernel: its loads are issued first, the frames come from the in-place tile map
// (staged in LDS, binary search per vector) while they are in flight, and each vector's
// payload bytes of a delivered data frame are unmasked and stored at the frame's arena offset
// (unaligned 16-byte stores; the bytes at a payload's edges by 8/4/2/1-byte pieces).
// ------------------------------------------------------------------------------------
// bytes [0, n) of v (little-endian) to p, n <= 16
__device__ inline void store_lo_bytes(uint8_t* p, unsigned __int128 v, int n) {
#ifdef UVWS_SCATTER_NT
    // (experiment: streaming stores, so no dirty arena lines are left behind in the caches)
    if (n == 16) {
        const u32x4 x = {(uint32_t)v, (uint32_t)(v >> 32), (uint32_t)(v >> 64), (uint32_t)(v >> 96)};
        __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
        return;
    }
    if (n & 8) {
        __builtin_nontemporal_store((uint64_t)v, reinterpret_cast<uint64_t*>(p));
        p += 8;
        v >>= 64;
    }
    if (n & 4) {
        __builtin_nontemporal_store((uint32_t)v, reinterpret_cast<uint32_t*>(p));
        p += 4;
        v >>= 32;
    }
    if (n & 2) {
        __builtin_nontemporal_store((uint16_t)v, reinterpret_cast<uint16_t*>(p));
        p += 2;
        v >>= 16;
    }
    if (n & 1) __builtin_nontemporal_store((uint8_t)v, p);
    return;
#endif
    if (n == 16) {
        __builtin_memcpy(p, &v, 16);
        return;
    }
    if (n & 8) {
        const uint64_t w = (uint64_t)v;
        __builtin_memcpy(p, &w, 8);
        p += 8;
        v >>= 64;
    }
    if (n & 4) {
        const uint32_t w = (uint32_t)v;
        __builtin_memcpy(p, &w, 4);
        p += 4;
        v >>= 32;
    }
    if (n & 2) {
        const uint16_t w = (uint16_t)v;
        __builtin_memcpy(p, &w, 2);
        p += 2;
        v >>= 16;
    }
    if (n & 1) *p = (uint8_t)v;
}

// the first frame whose slot holds map tile c's first byte (k_plan's claims, resolve_one);
// the speculative compact decode claims nothing — its frames sit at i * stride, so the frame
// is found by arithmetic (frame n - 1's slot runs to the end of the wire)
__device__ inline uint32_t tile_first_of(const BatchArgs& a, const Workspace& ws, uint64_t c) {
    if (a.spec_P) {
        const uint64_t x = c * kMapTile;
        if (x >= a.wire_len || a.n == 0) return kNoFrame;
        const uint64_t q = div_stride(a, x);
        return q < a.n ? (uint32_t)q : a.n - 1;
    }
    return tag_get(ws.tile_first[c], a.epoch, kNoFrame);
}

template <int BLOCK, int VPT>
__device__ __forceinline__ void scatter_tile(
    BatchArgs a, const uvhttp_ws_frame_desc_t* __restrict__ desc, const Workspace& ws,
    uint64_t arena_bytes_cap, uint64_t tile) {
    constexpr uint64_t kT = (uint64_t)BLOCK * VPT * 16;
    __shared__ uint64_t s_ps[BLOCK];  // wire offset of the payload
    __shared__ uint64_t s_pe[BLOCK];  // its end (== start: not a delivered data frame)
    __shared__ uint64_t s_ao[BLOCK];  // arena offset
    __shared__ uint32_t s_key[BLOCK];

    const uint64_t t0 = tile * kT;
    const uint64_t vend = a.wire_len;
    const uint64_t full_end = vend & ~(uint64_t)15;
    const uint64_t clamp_va = full_end ? full_end - 16 : 0;
    u32x4 data[VPT];
    uint64_t va[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        va[v] = t0 + ((uint64_t)v * BLOCK + threadIdx.x) * 16u;
        const uint64_t la = va[v] < full_end ? va[v] : clamp_va;
        data[v] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.wire + la));
    }
    // the one vector straddling the end of the wire: its bytes individually (the clamped
    // load above read the previous vector)
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        if (va[v] == full_end && full_end < vend) {
            uint32_t t[4] = {0, 0, 0, 0};
            for (uint64_t q = 0; full_end + q < vend; ++q)
                t[q >> 2] |= (uint32_t)a.wire[full_end + q] << (8 * (q & 3));
            data[v] = u32x4{t[0], t[1], t[2], t[3]};
        }
    }
    resolve_epoch(a, ws);  // after the loads are issued
    const uint32_t n = nframes(a);
    const uint32_t nb = first_bad_of(a, ws, n);
    if (nb == 0 || n == 0 || t0 >= vend) return;
    const uint32_t last = (nb < n ? nb : n) - 1;
    const uint64_t c0 = t0 / kMapTile, c1 = (t0 + kT - 1) / kMapTile + 1;
    const uint32_t f0 = tile_first_of(a, ws, c0);
    uint32_t f1 = (c1 < a.n_tiles) ? tile_first_of(a, ws, c1) : last;
    if (f0 > last) return;
    if (f1 > last || f1 < f0) f1 = last;

    for (uint32_t base = f0; base <= f1; base += BLOCK) {
        const uint32_t cnt = (f1 - base + 1) < (uint32_t)BLOCK ? (f1 - base + 1) : BLOCK;
        __syncthreads();
        if (threadIdx.x < cnt) {
            const uint32_t f = base + threadIdx.x;
            const uvhttp_ws_frame_desc_t d = desc[f];
            const uint64_t ps = frame_start(a, f) + d.header_size + ((d.flags & UVHTTP_WS_FLAG_MASK) ? 4u : 0u);
            const bool data_frame = d.opcode <= 2;
            s_ps[threadIdx.x] = ps;
            s_pe[threadIdx.x] = ps + (data_frame ? d.payload_len : 0);
            s_ao[threadIdx.x] = d.payload_off;
            s_key[threadIdx.x] = d.masking_key;
        }
        __syncthreads();
        if (s_ps[0] >= t0 + kT) break;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            if (va[v] >= vend) continue;
            int lo = 0, hi = (int)cnt - 1, j = -1;
            while (lo <= hi) {
                const int mid = (lo + hi) >> 1;
                if (s_ps[mid] < va[v] + 16) {
                    j = mid;
                    lo = mid + 1;
                } else {
                    hi = mid - 1;
                }
            }
            for (; j >= 0; --j) {
                const uint64_t ps = s_ps[j], pe = s_pe[j];
                if (pe <= va[v]) {
                    if (pe != ps) break;  // empty / control payloads don't end the walk
                    continue;
                }
                const int b0 = ps > va[v] ? (int)(ps - va[v]) : 0;
                int b1 = pe < va[v] + 16 ? (int)(pe - va[v]) : 16;
                if (va[v] + b1 > vend) b1 = (int)(vend - va[v]);
                const uint64_t dst = s_ao[j] + (va[v] + b0 - ps);
                if (dst >= arena_bytes_cap || b1 <= b0) continue;
                const int len = (int)(dst + (b1 - b0) <= arena_bytes_cap ? b1 - b0 : arena_bytes_cap - dst);
                const uint32_t rk = rotr32(s_key[j], 8u * (uint32_t)((va[v] - ps) & 3u));
                const u32x4 x = data[v] ^ u32x4{rk, rk, rk, rk};
                unsigned __int128 w = ((unsigned __int128)(((uint64_t)x.w << 32) | x.z) << 64) |
                                      (((uint64_t)x.y << 32) | x.x);
                w >>= 8 * b0;
                store_lo_bytes(a.arena + dst, w, len);
            }
        }
    }
}

__device__ inline uint64_t block_exclusive_sum_u64(uint64_t v, uint64_t* total) {
    __shared__ uint64_t wsum[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint64_t pre = 0, all = 0;
    for (int k = 0; k < kBlock / 64; ++k) {
        if (k < wave) pre += wsum[k];
        all += wsum[k];
    }
    __syncthreads();
    *total = all;
    return pre + inc - v;
}


template <int BLOCK, int VPT>
__global__ __launch_bounds__(BLOCK) void k_scatter_compact(
    BatchArgs a, const uvhttp_ws_frame_desc_t* __restrict__ desc, Workspace ws,
    uint64_t arena_bytes_cap, uint64_t tile_base) {
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_PAYLOAD, false, tile_base);
    scatter_tile<BLOCK, VPT>(a, desc, ws, arena_bytes_cap, tile_base + stamp_.anchor_s(blockIdx.x));
    // k_finalize's work at the end of the first ceil(n / BLOCK) workgroups, as the in-place
    // kernel does (statuses after the first failure, control payloads unmasked in the wire —
    // bytes no tile reads —, the summary): one launch fewer, C4 compact 1274 -> 1293 GiB/s,
    // C2 2226 -> 2256
    if (tile_base + blockIdx.x < (a.n + BLOCK - 1) / BLOCK) {
        resolve_epoch(a, ws);
        finalize_frames(a, const_cast<uvhttp_ws_frame_desc_t*>(desc), ws,
                        (uint32_t)(tile_base + blockIdx.x), BLOCK, first_bad_of(a, ws, a.n));
    }
}

// After k_plan on the speculative compact pass's records: when every delivered frame sat where
// the pass put it (ws.spec_bad past the first failure) only the summary remains (and SKIPPED
// statuses after a failure); otherwise the whole batch is scattered again from the wire by the
// same workgroups (grid-stride over the wire tiles; the tile map k_plan claimed), control
// payloads unmasked in the wire, as a k_plan-first compact decode does.
__global__ __launch_bounds__(kBlock) void k_spec_fix(BatchArgs a, uvhttp_ws_frame_desc_t* desc,
                                                     Workspace ws, uint64_t n_tiles) {
    resolve_epoch(a, ws);
    if (a.gate && ws.ctl[kCtlGate] != a.epoch) return;  // (summary-only compact: speculation held)
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_FIXUP);
    const uint32_t n = a.n;
    const uint32_t nb = first_bad_of(a, ws, n);
    const bool slow = tag_get(*ws.spec_bad, a.epoch, n) < nb && !device_fault(a, ws);
    if (slow) {
        for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x)
            scatter_tile<kBlock, 4>(a, desc, ws, a.arena_cap, t);
    }
    const uint32_t nblk = (n + kBlock - 1) / kBlock;
    for (uint32_t blk = blockIdx.x; blk < (nblk ? nblk : 1); blk += gridDim.x)
        finalize_frames(a, desc, ws, blk, kBlock, nb, slow);
}
// ------------------------------------------------------------------------------------
// Stream decode (uvhttp_ws_gpu_decode_streams / _decode_reads): many connections, each with
// its own state, limits and one process_data call per read.  Frames of one connection depend
// on each other only through the sequential header chain and the fragment state machine, and
// connections are the parallelism: one wave (few, long connections) or one lane (many short
// ones) runs a connection's whole process_data sequence (src/uvhttp_websocket.c:825-1097):
//   per call: the recv-buffer growth check (:832-857) on what the call holds;
//   per frame: header parse + the checks before unmasking (:876-932) — a rejected frame fails
//     the call in which its header bytes arrive — and, once the call holds the whole frame,
//     the fragment state machine and max_message_size (:950-1015, :781-822);
//   the calls after a failing call never run (the caller closes).
// The walk records each counted frame's start (the failing frame is the last one counted)
// and writes the connection's whole result except its first descriptor index.  Then:
//   k_swalk_scan    first frame of every connection, total, capacity
//   k_stream_desc   a wave per connection rebuilds its headers from the walk's frame records
//                   (or re-reads them: two aligned 16-byte loads each), writes the descriptors
//                   and message ids, and claims the 16 KiB tiles of the payload kernel's map
//                   (k_stream_desc_lane: a lane per connection, the same)
//   payload kernel  (k_unmask_inplace) unmasks every delivered frame in place
// No look-back, no bounded waits: nothing here can give up (k_swalk_fused, an opt-in that
// folds the walk, the scan and k_stream_desc into one launch, has a bounded look-back).
// ------------------------------------------------------------------------------------
struct WalkArgs {
    const uint8_t* wire;
    uint64_t wire_len;
    const uvhttp_ws_stream_t* streams;
    uint32_t n_streams;
    uint32_t max_frames;
    const uint64_t* read_end;  // [n_reads_total] read boundaries (relative), or null
    uint32_t n_reads_total;
    uint32_t single;           // 1: frame starts go to per-connection slices of walk_tmp
    uint32_t* agg;             // lane walk: frame counts per 256-connection block -> prefixes
    uvhttp_ws_stream_result_t* results;
    uvhttp_ws_frame_desc_t* desc;
    StreamScratch sc;
    // k_stream_desc (wave mode) claims the payload kernel's tile map itself
    uint64_t* tile_first;      // Workspace::tile_first
    uint64_t n_tiles;
    uint32_t epoch;            // this call's tag (dev_epoch: ctl[kCtlEpoch])
    uint32_t dev_epoch;
    const uint32_t* ctl;
    uint64_t* stamp;           // device-side kernel stamps (diagnostics), or null
    uint32_t cas_claims;       // the engine has captured calls (tag_claim)
    uint32_t max_polls;        // k_swalk_fused look-back wait bound (BatchArgs::max_polls)
    uint32_t no_ticket;        // k_swalk_fused: blocks in blockIdx order (UVHTTP_WS_PLAN_TICKET=0)
    uint64_t* first_bad;       // Workspace::first_bad (k_swalk_fused: a look-back give-up)
    uint32_t nt_stores;        // UVHTTP_WS_STREAM_NT=1: frame records and descriptors as streaming stores
    uint32_t desc_scan;        // k_stream_desc finds first frames itself (no k_swalk_scan)
    uint32_t nt_loads;         // UVHTTP_WS_WALK_NT_LOAD=1: the wave walk's header loads non-temporal (A/B)
    uint32_t spec;             // the speculative decode ran first: walk only if it gave way (spec_slow)
};

// Did the speculative stream decode give the call to the walk?  (Kernels of the walk path
// launched behind k_sspec_* return at once otherwise.)
__device__ inline bool spec_slow(const uint32_t* ctl, uint32_t epoch) {
    return ctl[kCtlSpecOff] == epoch || ctl[kCtlSpecBreak] == epoch;
}
__device__ inline bool walk_skip(const WalkArgs& w) {
    return w.spec && !spec_slow(w.ctl, w.dev_epoch ? w.ctl[kCtlEpoch] : w.epoch);
}

// process_data's buffer growth: returns false on failure (*out = size then), else the size
// after the call
__device__ inline bool grow_recv(uint64_t have, uint64_t size, int32_t max_frame, uint64_t* out) {
    *out = size;
    if (have <= size) return true;
    uint64_t ns = size;
    if (ns > (~0ull) / 2) return false;
    ns *= 2;
    while (have > ns) {
        if (ns > (~0ull) / 2) return false;
        ns *= 2;
    }
    const uint64_t ceiling = (uint64_t)(int64_t)max_frame;
    if (ns > ceiling) {
        ns = ceiling;
        if (have > ns) return false;
    }
    *out = ns;
    return true;
}

// Is connection s's descriptor usable?  In range of the wire (a test that cannot wrap for a
// begin near 2^64), after the previous connection (streams are ordered and disjoint), under
// 4 GiB (frame starts are kept as 32-bit offsets), and its read table — when it has one — in
// range, non-decreasing and ending at len.  Lanes [lane, lane + step, ...) check the read
// entries; the caller combines the lanes' answers.
__device__ inline bool stream_ok_part(const WalkArgs& w, uint32_t s, const uvhttp_ws_stream_t& st,
                                      uint32_t lane, uint32_t step) {
    if (!(st.len <= w.wire_len && st.begin <= w.wire_len - st.len) || (st.len >> 32)) return false;
    if (s > 0 && lane == 0) {
        const uvhttp_ws_stream_t pv = w.streams[s - 1];
        if (st.begin < pv.begin || st.begin - pv.begin < pv.len) return false;
    }
    if (st.n_reads == 0) return true;
    if (!w.read_end || st.first_read > w.n_reads_total ||
        st.n_reads > w.n_reads_total - st.first_read)
        return false;
    const uint64_t* re = w.read_end + st.first_read;
    bool ok = lane != 0 || re[st.n_reads - 1] == st.len;
    for (uint32_t k = lane; k < st.n_reads && ok; k += step) {
        const uint64_t prev = k ? re[k - 1] : 0;
        ok = re[k] >= prev && re[k] <= st.len;
    }
    return ok;
}

// per-connection decoder state carried by the walk (wave-uniform in the wave walk)
struct ConnState {
    uint64_t pos;        // stream offset of the next undecided frame
    uint64_t end;        // stream bytes the current call holds
    uint64_t size;       // recv_buffer_size after the current call's growth
    uint64_t acc;        // bytes of the open fragmented message (pending)
    uint32_t k;          // current call
    uint32_t count;      // frames counted
    uint32_t pending;    // a fragmented message is open (fragmented_message != NULL)
    int32_t fail;        // UVHTTP_WS_FRAME_* of the failure (0: none)
    uint32_t grow_fail;  // the current call failed its growth check
};

// One connection's process_data calls, frame by frame.  hdr(pos, hb) yields the ten header
// bytes at stream offset pos; emit(pos, idx) records counted frame idx.  Returns the state at
// the stop; the caller turns it into the result.
// fast(c) may first take any run of frames it can decide alone (complete, valid, accepted by
// the state machine) and advance c; everything else goes through the general code below.
struct NoFast {
    __device__ void operator()(struct ConnState&) const {}
};

template <typename Hdr, typename Emit, typename Fast = NoFast>
__device__ inline ConnState walk_calls(const WalkArgs& w, const uvhttp_ws_stream_t& st, Hdr&& hdr,
                                       Emit&& emit, Fast&& fast = NoFast()) {
    const uint64_t mf = (uint64_t)(int64_t)st.max_frame_size;
    const uint64_t lim = (uint64_t)(int64_t)st.max_message_size;
    const uint32_t K = st.n_reads ? st.n_reads : 1;
    const uint64_t* re = st.n_reads ? w.read_end + st.first_read : nullptr;
    ConnState c;
    c.pos = 0;
    c.k = 0;
    c.count = 0;
    c.fail = 0;
    c.pending = st.pending_bytes ? 1u : 0u;
    c.acc = st.pending_bytes;
    c.end = re ? re[0] : st.len;
    c.grow_fail = grow_recv(c.end, st.recv_buffer_size, st.max_frame_size, &c.size) ? 0u : 1u;
    if (re) w.sc.read_size[st.first_read] = c.size;
    while (!c.grow_fail) {
        fast(c);
        uint64_t need_end;  // the stream offset the next decision needs
        if (c.end - c.pos >= 2) {
            uint32_t hb[10];
            hdr(c.pos, hb);
            const uint32_t b0 = hb[0], b1 = hb[1];
            const uint32_t code = b1 & 0x7F;
            const uint32_t need = code == 126 ? 4 : code == 127 ? 10 : 2;
            if (c.end - c.pos >= need) {
                uint64_t plen = code;
                if (need == 4) {
                    plen = (hb[2] << 8) | hb[3];
                } else if (need == 10) {
                    plen = ((uint64_t)((hb[2] << 24) | (hb[3] << 16) | (hb[4] << 8) | hb[5]) << 32) |
                           (uint32_t)((hb[6] << 24) | (hb[7] << 16) | (hb[8] << 8) | hb[9]);
                }
                const uint32_t op = b0 & 0x0F;
                const bool fin = b0 & 0x80;
                int32_t st_h = UVHTTP_WS_FRAME_OK;  // :876-921, in the reference's order
                if (need == 10 && (plen >> 63)) st_h = UVHTTP_WS_FRAME_ERR_PARSE;
                else if (b0 & 0x70) st_h = UVHTTP_WS_FRAME_ERR_RSV;
                else if (op >= 8 && (plen > 125 || !fin)) st_h = UVHTTP_WS_FRAME_ERR_CONTROL;
                else if (st.is_server && !(b1 & 0x80)) st_h = UVHTTP_WS_FRAME_ERR_UNMASKED;
                else if (plen > mf) st_h = UVHTTP_WS_FRAME_ERR_TOO_BIG;
                if (st_h != UVHTTP_WS_FRAME_OK) {  // fails this call, before any unmasking
                    emit(c.pos, c.count);
                    ++c.count;
                    c.fail = st_h;
                    break;
                }
                const uint64_t wl = need + ((b1 & 0x80) ? 4u : 0u) + plen;
                if (c.end - c.pos >= wl) {  // complete: this call unmasks and dispatches it
                    if (op <= 2) {  // the fragment state machine (:950-1015)
                        const bool cont = op == 0;
                        int32_t sm = UVHTTP_WS_FRAME_OK;
                        if (!c.pending) {
                            if (cont) sm = UVHTTP_WS_FRAME_ERR_FRAGMENT;
                            else if (!fin && lim != 0 && plen > lim) sm = UVHTTP_WS_FRAME_ERR_MESSAGE;
                            else if (!fin && plen) {  // an empty first fragment opens nothing
                                c.pending = 1;
                                c.acc = plen;
                            }
                        } else if (!cont) {
                            sm = UVHTTP_WS_FRAME_ERR_FRAGMENT;
                        } else if (lim != 0 && (c.acc > lim || plen > lim - c.acc)) {
                            sm = UVHTTP_WS_FRAME_ERR_MESSAGE;
                        } else if (fin) {
                            c.pending = 0;
                            c.acc = 0;
                        } else {
                            c.acc += plen;
                        }
                        if (sm != UVHTTP_WS_FRAME_OK) {
                            emit(c.pos, c.count);
                            ++c.count;
                            c.fail = sm;
                            break;
                        }
                    }
                    emit(c.pos, c.count);
                    ++c.count;
                    c.pos += wl;
                    continue;
                }
                need_end = c.pos + wl;
            } else {
                need_end = c.pos + need;
            }
        } else {
            need_end = c.pos + 2;
        }
        // the bytes of the next decision come with a later call: run the calls up to it
        // (each one's growth check sees the partial frame plus everything it appended)
        while (c.end < need_end && c.k + 1 < K) {
            ++c.k;
            c.end = re[c.k];
            uint64_t grown;
            c.grow_fail = grow_recv(c.end - c.pos, c.size, st.max_frame_size, &grown) ? 0u : 1u;
            c.size = grown;
            w.sc.read_size[st.first_read + c.k] = grown;
            if (c.grow_fail) break;
        }
        if (c.grow_fail || c.end < need_end) break;  // else every call ran: the rest waits
    }
    return c;
}

// the connection's result from its walk (first_frame is placed by k_swalk_scan)
__device__ inline uvhttp_ws_stream_result_t walk_result(const WalkArgs& w, const uvhttp_ws_stream_t& st,
                                                        const ConnState& c) {
    const uint64_t* re = st.n_reads ? w.read_end + st.first_read : nullptr;
    auto end_of = [&](uint32_t call) { return re ? re[call] : st.len; };
    uvhttp_ws_stream_result_t r;
    r.first_frame = 0;
    r.n_frames = c.count;
    r.n_delivered = c.count - (c.fail ? 1u : 0u);
    r.status = (c.fail || c.grow_fail) ? -1 : 0;
    r.first_status = c.fail ? c.fail : c.grow_fail ? UVHTTP_WS_FRAME_ERR_BUFFER : 0;
    r.calls = c.k + 1;
    r.consumed_bytes = c.pos;  // the end of the last delivered frame
    r.recv_buffer_size = c.size;
    // the fragment state after the last delivered frame (a failing frame changes nothing the
    // device reports; deliver_stream replays its partial effect on the host)
    r.pending_bytes = c.pending ? c.acc : 0;
    // a failing growth check returns before appending: the buffer holds what the calls
    // before it left (the first call: untouched, marked by 0)
    r.buffered_end = c.grow_fail ? (c.k ? end_of(c.k - 1) : 0) : end_of(c.k);
    r.reserved = 0;
    return r;
}

__device__ inline uvhttp_ws_stream_result_t layout_result(const uvhttp_ws_stream_t& st) {
    uvhttp_ws_stream_result_t r;
    memset(&r, 0, sizeof(r));
    r.status = -1;
    r.first_status = UVHTTP_WS_FRAME_ERR_LAYOUT;
    r.recv_buffer_size = st.recv_buffer_size;
    r.pending_bytes = st.pending_bytes;
    return r;
}

// slice of connection s in walk_tmp (single pass): its frames are >= 2 bytes apart and
// connections are disjoint and ordered, so begin / 2 + s leaves room for every start
__device__ inline uint64_t slice_base(const uvhttp_ws_stream_t& st, uint32_t s) {
    return st.begin / 2 + s;
}

// Frame records of the wave walk's fast path (walk_rec, parallel to walk_tmp): the masking key
// and b0 | b1 << 8 | payload length << 16 for a frame with a 7- or 16-bit length, so
// k_stream_desc builds that frame's descriptor without gathering its header from HBM again
// (C4 streams: the gather was most of k_stream_desc).  kNoRec: the header must be re-read.
constexpr uint32_t kNoRec = 0xFFFFFFFFu;

// the 16-byte header image of a recorded frame (what load16_at would return for its header)
__device__ inline u32x4 rec_header(uint2 r) {
    const uint32_t b0 = r.y & 0xFF, b1 = (r.y >> 8) & 0xFF, plen = r.y >> 16;
    const uint32_t key = r.x;
    if ((b1 & 0x7F) == 126) {  // b0 b1 len_hi len_lo key0..3
        return u32x4{b0 | (b1 << 8) | ((plen >> 8) << 16) | ((plen & 0xFF) << 24), key, 0u, 0u};
    }
    return u32x4{b0 | (b1 << 8) | (key << 16), key >> 16, 0u, 0u};  // b0 b1 key0..3
}

// ---- lane walk: one lane per connection, headers straight from global memory -------------
// MODE 0: count; 1: write starts to frame_off from the connection's first frame (two-pass);
// 2: count and write starts into the connection's slice (single pass)
// block-wide sum (256 threads) and exclusive prefix of one u32 per thread
__device__ inline uint32_t block_scan_u32(uint32_t v, uint32_t* total) {
    __shared__ uint32_t wsum[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t pre = 0, all = 0;
    for (int k = 0; k < kBlock / 64; ++k) {
        if (k < wave) pre += wsum[k];
        all += wsum[k];
    }
    __syncthreads();
    *total = all;
    return pre + inc - v;
}

// lane mode: connection s's first frame = its block's prefix (k_swalk_scan) + the counts of
// the block's earlier connections (every thread of the block calls this)
__device__ inline uint32_t lane_first(const WalkArgs& w, uint32_t s) {
    const uint32_t c = s < w.n_streams ? w.results[s].n_frames : 0;
    uint32_t total;
    const uint32_t local = block_scan_u32(c, &total);
    return w.agg[blockIdx.x] + local;
}

template <int MODE>
__device__ inline uint32_t walk_lane(const WalkArgs& w, uint32_t s, uint32_t lf) {
    const uvhttp_ws_stream_t st = w.streams[s];
    if (!stream_ok_part(w, s, st, 0, 1)) {
        if (MODE != 1) w.results[s] = layout_result(st);
        return 0;
    }
    const uint64_t first = MODE == 1 ? lf : slice_base(st, s);
    const ConnState c = walk_calls(
        w, st,
        [&](uint64_t pos, uint32_t hb[10]) {  // (bytes past the stream are never used)
            const u32x4 v = load16_at(w.wire, w.wire_len, st.begin + pos);
            const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 10; ++q) hb[q] = (x[q >> 2] >> (8 * (q & 3))) & 0xFF;
        },
        [&](uint64_t pos, uint32_t idx) {
            if (MODE == 1 && first + idx < w.max_frames) w.sc.frame_off[first + idx] = st.begin + pos;
            if (MODE == 2) w.sc.walk_tmp[first + idx] = (uint32_t)pos;
        });
    if (MODE != 1) w.results[s] = walk_result(w, st, c);
    return c.count;
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void k_swalk_lane(WalkArgs w) {
    if (walk_skip(w)) return;
    StampScope stamp_(w.stamp, w.epoch, MODE == 1 ? UVHTTP_WS_STAMP_WALK2 : UVHTTP_WS_STAMP_WALK, false);
    const uint32_t s = stamp_.anchor_v(blockIdx.x * kBlock + threadIdx.x);
    const uint32_t lf = MODE == 1 ? lane_first(w, s) : 0;  // (before any thread leaves)
    uint32_t count = 0;
    if (s < w.n_streams) count = walk_lane<MODE>(w, s, lf);
    if (MODE == 1) return;
    uint32_t total;
    (void)block_scan_u32(count, &total);
    if (threadIdx.x == 0) w.agg[blockIdx.x] = total;
}

// ---- wave walk: one wave per connection (connections with many frames) -------------------
// The connection's bytes pass through LDS in aligned 4 KiB blocks: a two-slot ring (the block
// of the current header and the next) plus a 16-byte mirror of slot 0 after slot 1, so the
// ten bytes of any header are one run of LDS bytes; the block after those is in flight in
// registers, issued when the walk entered the current block.  Block loads are buffer loads
// bounded by the wire's last 16-byte granule (bytes past it read as 0): no per-lane branches.  Every lane
// reads the same header bytes (broadcast) and readfirstlane makes them scalar, so the header
// decode, the checks and the state machine run on the scalar unit with uniform branches.
// Frame starts are collected one per lane and stored 64 at a time.
constexpr uint32_t kWalkBlk = 4096;
constexpr int kWalkVec = (int)(kWalkBlk / (64u * 16u));  // 16-byte loads per lane per block
constexpr uint32_t kRingBytes = 2 * kWalkBlk + 16;

__device__ inline void walk_load_block(const WalkArgs& w, uint64_t blk, u32x4 v[kWalkVec]) {
    const int lane = threadIdx.x & 63;
    const uint64_t base = blk * kWalkBlk;
    // the range check drops every dword that is not wholly inside num_records (a wire ending
    // two bytes into a 16-bit-length header read as zeros: an "unmasked" frame), so the range is
    // the wire rounded up to its 16-byte granule — the wire is 16-byte aligned, so the granule
    // never crosses a page; its bytes past wire_len are never used (every decision is checked
    // against the call's end)
    const uint64_t room = w.wire_len > base ? ((w.wire_len - base + 15) & ~(uint64_t)15) : 0;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(w.wire + (room ? base : 0)), 0, (int)(room < kWalkBlk ? room : kWalkBlk),
        0x00020000);
#pragma unroll
    for (int k = 0; k < kWalkVec; ++k)
        v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rs, (uint32_t)(k * 64 + lane) * 16u, 0, 0));
}

__device__ inline void walk_store_block(uint8_t* ring, uint64_t blk, const u32x4 v[kWalkVec]) {
    const int lane = threadIdx.x & 63;
    const uint32_t slot = (uint32_t)(blk & 1);
    uint8_t* dst = ring + slot * kWalkBlk;
#pragma unroll
    for (int k = 0; k < kWalkVec; ++k)
        *reinterpret_cast<u32x4*>(dst + (uint32_t)(k * 64 + lane) * 16u) = v[k];
    if (slot == 0 && lane == 0)  // the mirror after slot 1: slot 0's first 16 bytes
        *reinterpret_cast<u32x4*>(ring + 2 * kWalkBlk) = v[0];
}

__device__ inline void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// MODE 0 / 1 / 2 as the lane walk; 3: as 2, the result returned (every lane) instead of
// written (k_swalk_fused)
template <int MODE>
__device__ inline uvhttp_ws_stream_result_t walk_wave(const WalkArgs& w, uint32_t s, uint8_t* ring) {
    const uint32_t lane = threadIdx.x & 63;
    const uvhttp_ws_stream_t st = w.streams[s];
    const bool ok = __all(stream_ok_part(w, s, st, lane, 64));
    if (!ok) {
        const uvhttp_ws_stream_result_t r = layout_result(st);
        if ((MODE == 0 || MODE == 2) && lane == 0) {
            w.results[s] = r;
            w.agg[s] = 0;
        }
        return r;
    }
    // (wave mode: agg[s] holds the connection's frame count for k_swalk_scan, then its first)
    const uint64_t first = MODE == 1 ? w.agg[s] : slice_base(st, s);
    uint64_t cur = ~0ull;  // block of the current header; LDS holds cur and cur + 1
    u32x4 pf[kWalkVec];    // block cur + 2, in flight
    // frame start records: one lane per frame (the fast path below stores a run of frames, one
    // per lane, in one instruction)
    auto emit_lane = [&](uint64_t pos, uint32_t idx, bool on, uint2 rec) {
        if (MODE == 0 || !on) return;
        const uint64_t f = first + idx;
        if (MODE >= 2) {
            if (w.nt_stores) {
                __builtin_nontemporal_store((uint32_t)pos, &w.sc.walk_tmp[f]);
                if (w.sc.walk_rec) {
                    __builtin_nontemporal_store(rec.x, &w.sc.walk_rec[f].x);
                    __builtin_nontemporal_store(rec.y, &w.sc.walk_rec[f].y);
                }
            } else {
                w.sc.walk_tmp[f] = (uint32_t)pos;
                if (w.sc.walk_rec) w.sc.walk_rec[f] = rec;
            }
        } else if (f < w.max_frames) {
            w.sc.frame_off[f] = st.begin + pos;
        }
    };
    auto emit = [&](uint64_t pos, uint32_t idx) { emit_lane(pos, idx, lane == 0, uint2{0u, kNoRec}); };
    const ConnState c = walk_calls(
        w, st,
        [&](uint64_t pos, uint32_t hb[10]) {
            const uint64_t at = st.begin + pos;
            const uint64_t blk = at / kWalkBlk;
            if (blk != cur) {
                if (cur != ~0ull && blk == cur + 1) {
                    walk_store_block(ring, blk + 1, pf);  // the prefetched block joins the ring
                } else {
                    u32x4 t[kWalkVec];
                    walk_load_block(w, blk, t);
                    walk_load_block(w, blk + 1, pf);
                    walk_store_block(ring, blk, t);
                    walk_store_block(ring, blk + 1, pf);
                }
                walk_load_block(w, blk + 2, pf);
                cur = blk;
                wave_sync_lds();
            }
            const uint32_t r = (uint32_t)((blk & 1) * kWalkBlk + at % kWalkBlk);
#pragma unroll
            for (int q = 0; q < 10; ++q) hb[q] = __builtin_amdgcn_readfirstlane(ring[r + q]);
        },
        [&](uint64_t pos, uint32_t idx) { emit(pos, idx); },
        [&](ConnState& c) {
            // The hot loop, on runs of equal frames.  Frame 0 of a step is the one at pos (its
            // header from the LDS ring, or carried from the step before).  When frame 0 has the
            // previous frame's wire length wl0, lane l speculates that frames 0 .. l-1 all have
            // it and loads the header at pos + l * wl0 straight from global memory (one 32-byte
            // window per lane — the payload bytes between headers are never fetched), then
            // checks it: same first byte (opcode and flags), same length, complete in the
            // current call, valid, and accepted by the fragment state machine given the run
            // before it.  The leading accepted lanes (a ballot) are decided at once — up to 64
            // frames per step — and the first rejected lane's header becomes the next step's
            // frame 0.  Runs the state machine cannot take whole (a message start without FIN,
            // a final fragment) stop after their first frame; anything else leaves for the
            // general code.  All lanes compute with vector registers; each step's outcome is
            // made uniform by readfirstlane.
            if (c.grow_fail) return;
            const uint32_t end32 = (uint32_t)c.end;
            const uint64_t mf = (uint64_t)(int64_t)st.max_frame_size;
            const uint64_t lim = (uint64_t)(int64_t)st.max_message_size;
            uint32_t pos = (uint32_t)c.pos, pend = c.pending;
            uint64_t acc = c.acc;
            uint32_t cnt = c.count;
            // header fields from ten bytes hb[0..9]
            auto decode = [&](const uint32_t* hb, uint32_t& b0, uint32_t& wl, uint64_t& plen, bool& bad) {
                b0 = hb[0];
                const uint32_t b1 = hb[1], code = b1 & 0x7F;
                const uint32_t need = code < 126 ? 2u : code == 126 ? 4u : 10u;
                plen = code;
                if (code == 126) plen = (hb[2] << 8) | hb[3];
                if (code == 127)
                    plen = ((uint64_t)((hb[2] << 24) | (hb[3] << 16) | (hb[4] << 8) | hb[5]) << 32) |
                           (uint32_t)((hb[6] << 24) | (hb[7] << 16) | (hb[8] << 8) | hb[9]);
                const uint32_t op = b0 & 0x0F, fin = b0 >> 7, m = b1 >> 7;
                bad = (b0 & 0x70) || (op >= 8 && (plen > 125 || !fin)) || (st.is_server && !m) ||
                      plen > mf || (plen >> 31);  // (a length of 2^31 or more: general code)
                wl = need + 4u * m + (uint32_t)plen;
            };
            // a header's 16 bytes (issued apart from the decode, so several are in flight), then
            // its fields and the frame's record for k_stream_desc: key and header bytes, kNoRec
            // for a 64-bit length
            auto fetch = [&](uint64_t p) {
                return w.nt_loads ? load16_at<true>(w.wire, w.wire_len, st.begin + p)
                                  : load16_at(w.wire, w.wire_len, st.begin + p);
            };
            auto decode16 = [&](const u32x4& v, uint32_t& b0, uint32_t& wl, uint64_t& plen, bool& bad,
                                uint2& rec) {
                const uint32_t x[4] = {v.x, v.y, v.z, v.w};
                uint32_t hb[10];
#pragma unroll
                for (int q = 0; q < 10; ++q) hb[q] = (x[q >> 2] >> (8 * (q & 3))) & 0xFF;
                decode(hb, b0, wl, plen, bad);
                const uint32_t code = hb[1] & 0x7F;
                const uint32_t key = code < 126 ? (v.x >> 16) | (v.y << 16) : v.y;  // bytes 2-5 / 4-7
                rec = code < 127 ? uint2{(hb[1] & 0x80) ? key : 0u, hb[0] | (hb[1] << 8) | ((uint32_t)plen << 16)}
                                 : uint2{0u, kNoRec};
            };
            // kG groups of 64 speculative frames per step: lane l of group g takes frame
            // 1 + l + 64 g, so one step decides up to 64 kG frames with kG loads in flight per
            // lane (64 per step measured 40 us for C4's 4096 x 256 frames: four dependent gathers)
            constexpr uint32_t kG = 4, kRun = 64 * kG;
            uint32_t wlp = 0;          // the previous step's frame length (0: first step)
            bool have0 = false;        // frame 0's header carried from the previous step
            uint32_t cb0 = 0, cwl = 0;  // (its fields)
            uint64_t cplen = 0;
            bool cbad = false;
            uint2 crec{0u, kNoRec};    // (and its record)
            for (;;) {
                if (end32 - pos < 10) break;  // (uniform)
                uint32_t b00, wl0;
                uint64_t plen0;
                bool bad0;
                uint2 rec0{0u, kNoRec};
                if (have0) {
                    b00 = cb0, wl0 = cwl, plen0 = cplen, bad0 = cbad, rec0 = crec;
                } else {
                    // frame 0 straight from global memory (every lane the same 16 bytes): the
                    // general code's LDS ring of 4 KiB blocks is loaded only when it runs
                    decode16(fetch(pos), b00, wl0, plen0, bad0, rec0);
                    b00 = __builtin_amdgcn_readfirstlane(b00);
                    wl0 = __builtin_amdgcn_readfirstlane(wl0);
                    plen0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(plen0 >> 32)) << 32) |
                            __builtin_amdgcn_readfirstlane((uint32_t)plen0);
                    bad0 = __builtin_amdgcn_readfirstlane((uint32_t)bad0) != 0;
                    rec0 = uint2{__builtin_amdgcn_readfirstlane(rec0.x), __builtin_amdgcn_readfirstlane(rec0.y)};
                }
                const uint32_t op0 = b00 & 0x0F, fin0 = b00 >> 7;
                const bool data0 = op0 <= 2;
                const bool smf0 = data0 && (pend ? (op0 != 0 || (lim != 0 && (acc > lim || plen0 > lim - acc)))
                                                 : (op0 == 0 || (!fin0 && lim != 0 && plen0 > lim)));
                if (bad0 || wl0 > end32 - pos || smf0) break;
                // runs: control frames, complete messages (op 1/2 + FIN, nothing open), and
                // middle fragments (CONTINUATION without FIN, a message open)
                const uint32_t kind = !data0 ? 0u : (op0 != 0 && fin0) ? 1u : (op0 == 0 && !fin0) ? 2u : 3u;
                uint32_t n = 1;
                have0 = false;
                uint2 recl[kG];  // lane l of group g: the record of frame 1 + l + 64 g
#pragma unroll
                for (uint32_t g = 0; g < kG; ++g) recl[g] = uint2{0u, kNoRec};
#ifdef UVWS_WALK_SPEC_FIRST_OFF
                const bool spec = wl0 == wlp;
#else
                // (the first step speculates on frame 0's own length: one dependent header
                // round trip fewer per connection; a connection of unequal frames wastes one
                // step's loads)
                const bool spec = wl0 == wlp || wlp == 0;
#endif
                if (kind != 3 && spec) {
                    // speculation: frames 1 .. kRun all have frame 0's length, so the frame after
                    // the run — the next step's frame 0 — was always read, even after a full run
                    u32x4 hv[kG];
                    bool hin[kG];
#pragma unroll
                    for (uint32_t g = 0; g < kG; ++g) {  // every load first
                        const uint64_t pl = (uint64_t)pos + (uint64_t)(lane + 1 + 64 * g) * wl0;
                        hin[g] = pl + 10 <= end32;
                        hv[g] = hin[g] ? fetch(pl) : u32x4{0u, 0u, 0u, 0u};
                    }
                    uint64_t good[kG];
                    uint32_t b0l[kG], wll[kG];
                    uint64_t plenl[kG];
                    bool badl[kG];
#pragma unroll
                    for (uint32_t g = 0; g < kG; ++g) {
                        const uint32_t f = lane + 1 + 64 * g;
                        const uint64_t pl = (uint64_t)pos + (uint64_t)f * wl0;
                        b0l[g] = 0, wll[g] = 0, plenl[g] = 0, badl[g] = true;
                        if (hin[g]) decode16(hv[g], b0l[g], wll[g], plenl[g], badl[g], recl[g]);
                        const bool okl = hin[g] && pl + wl0 <= end32 && !badl[g] && b0l[g] == b00 &&
                                         wll[g] == wl0 && plenl[g] == plen0 &&
                                         (kind != 2 || lim == 0 || acc + (uint64_t)(f + 1) * plen0 <= lim);
                        good[g] = __ballot(okl);
                    }
                    // frame 0 plus the leading accepted frames, at most kRun per step
                    uint32_t m = 0;
#pragma unroll
                    for (uint32_t g = 0; g < kG; ++g) {
                        if (m == 64 * g) m += ~good[g] == 0 ? 64u : (uint32_t)__builtin_ctzll(~good[g]);
                    }
                    n = __builtin_amdgcn_readfirstlane(m + 1 < kRun ? m + 1 : kRun);
                    // frame n (the first not taken) is the next step's frame 0: lane (n - 1) % 64
                    // of group (n - 1) / 64 read it
                    const uint32_t gn = (n - 1) / 64, ln = (n - 1) % 64;
                    uint32_t hsel = 0, b0s = 0, wls = 0, pl0 = 0, pl1 = 0, bads = 0, rx = 0, ry = 0;
#pragma unroll
                    for (uint32_t g = 0; g < kG; ++g) {
                        if (g == gn) {  // (uniform)
                            hsel = __builtin_amdgcn_readlane((uint32_t)hin[g], ln);
                            b0s = __builtin_amdgcn_readlane(b0l[g], ln);
                            wls = __builtin_amdgcn_readlane(wll[g], ln);
                            pl1 = __builtin_amdgcn_readlane((uint32_t)(plenl[g] >> 32), ln);
                            pl0 = __builtin_amdgcn_readlane((uint32_t)plenl[g], ln);
                            bads = __builtin_amdgcn_readlane((uint32_t)badl[g], ln);
                            rx = __builtin_amdgcn_readlane(recl[g].x, ln);
                            ry = __builtin_amdgcn_readlane(recl[g].y, ln);
                        }
                    }
                    if (hsel) {
                        have0 = true;
                        cb0 = b0s, cwl = wls, cplen = ((uint64_t)pl1 << 32) | pl0, cbad = bads != 0;
                        crec = uint2{rx, ry};
                    }
                }
                // lane l emits frames l + 64 g: the record of frame j >= 1 is lane (j - 1) % 64
                // of group (j - 1) / 64 (frame 0's is the carried one)
                uint2 prevg = rec0;  // group g - 1's lane 63 (frame 64 g's record)
#pragma unroll
                for (uint32_t g = 0; g < kG; ++g) {
                    if (64 * g >= n) break;  // (uniform)
                    const uint32_t j = 64 * g + lane;
                    // record of frame j = recl[(j - 1) / 64] at lane (j - 1) % 64: for lane
                    // l >= 1 that is group g's lane l - 1, for lane 0 group g - 1's lane 63 (or,
                    // frame 0, the carried one) — the shuffle runs on every lane
                    const uint2 up{__shfl_up(recl[g].x, 1, 64), __shfl_up(recl[g].y, 1, 64)};
                    const uint2 rj = lane ? up : prevg;
                    emit_lane((uint64_t)pos + (uint64_t)j * wl0, cnt + j, j < n, rj);
                    prevg = uint2{__builtin_amdgcn_readlane(recl[g].x, 63), __builtin_amdgcn_readlane(recl[g].y, 63)};
                }
                if (kind == 2) {
                    acc += (uint64_t)n * plen0;
                } else if (kind == 3) {  // one frame: a start without FIN or a final fragment
                    if (pend) {
                        acc = 0;
                        pend = 0;
                    } else if (plen0) {
                        pend = 1;
                        acc = plen0;
                    }
                }
                pos += n * wl0;
                cnt += n;
                wlp = wl0;
            }
            c.pos = __builtin_amdgcn_readfirstlane(pos);
            c.pending = __builtin_amdgcn_readfirstlane(pend);
            c.acc = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(acc >> 32)) << 32) |
                    __builtin_amdgcn_readfirstlane((uint32_t)acc);
            c.count = cnt;
        });
    const uvhttp_ws_stream_result_t r = walk_result(w, st, c);
    if ((MODE == 0 || MODE == 2) && lane == 0) {
        w.results[s] = r;
        w.agg[s] = c.count;
    }
    return r;
}

// the connections of (virtual) workgroup vb, a wave each
template <int MODE>
__device__ inline void swalk_wave_block(const WalkArgs& w, uint32_t vb, StampScope& stamp_) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[kBlock / 64][kRingBytes];
    // readfirstlane: the connection (and all walk state derived from it) is wave-uniform, so
    // it lives in scalar registers and the walk's branches are scalar branches
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t s = stamp_.anchor_s(vb * (kBlock / 64) + wave);
    if (s >= w.n_streams) return;
    if (MODE == 1 && !w.results[s].n_frames) return;
    (void)walk_wave<MODE>(w, s, ring[wave]);
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void k_swalk_wave(WalkArgs w) {
    if (walk_skip(w)) return;
    StampScope stamp_(w.stamp, w.epoch, MODE == 1 ? UVHTTP_WS_STAMP_WALK2 : UVHTTP_WS_STAMP_WALK, false);
    swalk_wave_block<MODE>(w, blockIdx.x, stamp_);
}

// Behind the speculative decode the walk path is a fall-back that almost never runs, and a
// launch that returns at once costs about its workgroup count: 1024 workgroups per gated
// kernel — three of them — put ~7 us between C4 stream calls (stamps, profiles/r06p_*), 256
// about 1 (the gated compact fall-back's).  So the gated walk kernels stride over the blocks
// with kGatedGrid workgroups.
constexpr uint32_t kGatedGrid = 256;
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_swalk_wave_gated(WalkArgs w, uint32_t n_blocks) {
    if (walk_skip(w)) return;
    StampScope stamp_(w.stamp, w.epoch, MODE == 1 ? UVHTTP_WS_STAMP_WALK2 : UVHTTP_WS_STAMP_WALK, false);
    for (uint32_t vb = blockIdx.x; vb < n_blocks; vb += gridDim.x) swalk_wave_block<MODE>(w, vb, stamp_);
}

// first frames, total, capacity (one workgroup).  Lane mode scans the walk's per-block
// counts (agg, in place; k_stream_desc_lane adds the block-local part); wave mode (at most
// 16384 connections) writes every connection's first frame itself.  Each thread takes a
// contiguous chunk: sum it, scan the sums across the block, then write the chunk's prefixes.
__global__ __launch_bounds__(kBlock) void k_swalk_scan(WalkArgs w, uint32_t lane_mode) {
    if (walk_skip(w)) return;
    StampScope stamp_(w.stamp, w.epoch, UVHTTP_WS_STAMP_WALK_SCAN);
    const uint32_t m = lane_mode ? (w.n_streams + kBlock - 1) / kBlock : w.n_streams;
    const uint32_t per = (m + kBlock - 1) / kBlock;
    const uint32_t beg = threadIdx.x * per;
    const uint32_t fin = beg + per < m ? beg + per : m;
    auto count_of = [&](uint32_t j) { return w.agg[j]; };  // (block counts / connection counts)
    // (unrolled by 8 so each thread's loads are in flight together: a chunk of 16 results read
    // one after another cost ~12 us at 4096 connections)
    uint64_t run = 0;
#pragma unroll 8
    for (uint32_t j = beg; j < fin; ++j) run += count_of(j);
    uint64_t total;
    uint64_t pre = block_exclusive_sum_u64(run, &total);
#pragma unroll 8
    for (uint32_t j = beg; j < fin; ++j) {
        const uint32_t v = count_of(j);
        w.agg[j] = (uint32_t)pre;
        pre += v;
    }
    if (threadIdx.x == 0) *w.sc.n_total = total <= w.max_frames ? (uint32_t)total : 0u;
}

// frame k of connection s (frame start `pos`, stream-relative): its descriptor and end
__device__ inline void stream_frame_desc(const WalkArgs& w, const uvhttp_ws_stream_t& st,
                                         const uvhttp_ws_stream_result_t& r, uint32_t k,
                                         uint64_t pos, const u32x4& hv, uvhttp_ws_frame_desc_t& d,
                                         bool& fin_data, uint64_t& fe) {
    const uint64_t hlo = hv.x | ((uint64_t)hv.y << 32), hhi = hv.z | ((uint64_t)hv.w << 32);
    auto hb = [&](int q) -> uint32_t {
        return (uint32_t)((q < 8 ? hlo >> (8 * q) : hhi >> (8 * (q - 8))) & 0xFF);
    };
    const uint32_t b0 = hb(0), b1 = hb(1), code = b1 & 0x7F;
    const uint32_t hsz = code == 126 ? 4 : code == 127 ? 10 : 2;
    uint64_t plen = code;
    if (hsz == 4) {
        plen = (hb(2) << 8) | hb(3);
    } else if (hsz == 10) {
        plen = 0;
#pragma unroll
        for (int q = 2; q < 10; ++q) plen = (plen << 8) | hb(q);
    }
    const bool msb = hsz == 10 && (plen >> 63);
    const uint32_t m = (b1 >> 7) ? 4u : 0u;
    const uint64_t slot = st.len - pos;
    const bool failing = k + 1 == r.n_frames && r.n_delivered < r.n_frames;
    d.payload_off = st.begin + pos + (msb ? 0 : hsz + m);
    d.payload_len = plen;
    d.masking_key = (m && slot >= hsz + 4)
                        ? (hsz == 2 ? (uint32_t)(hlo >> 16) : hsz == 4 ? (uint32_t)(hlo >> 32)
                                                                      : (uint32_t)(hhi >> 16))
                        : 0u;
    d.message = 0;
    d.opcode = (uint8_t)(b0 & 0x0F);
    d.flags = (uint8_t)(((b0 >> 7) & 1) | ((b1 >> 7) << 1) | (((b0 >> 6) & 1) << 2) |
                        (((b0 >> 5) & 1) << 3) | (((b0 >> 4) & 1) << 4));
    d.header_size = (uint8_t)hsz;
    d.status = (int8_t)(failing ? r.first_status : UVHTTP_WS_FRAME_OK);
    const uint64_t wl = msb ? 0 : hsz + m + plen;
    d.wire_len = wl > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)wl;
    fin_data = !failing && d.opcode <= 2 && (b0 & 0x80);
    if (fin_data) d.flags |= UVHTTP_WS_FLAG_MSG_END;
    // the frame's end for the tile claims, clamped to the connection for a failing frame's
    // declared length
    fe = st.begin + (msb || wl > slot ? st.len : pos + wl);
}

__device__ inline void capacity_result(uvhttp_ws_stream_result_t& r) {
    r.status = -1;
    r.first_status = UVHTTP_WS_FRAME_ERR_CAPACITY;
    r.n_frames = r.n_delivered = 0;
    r.calls = 0;
    r.consumed_bytes = 0;
    r.buffered_end = 0;
}

// The payload kernel's tile map: frame i claims the 16 KiB map tiles whose first byte lies in
// [end of frame i - 1, end of frame i) — the first frame ending after a tile's start, where the
// kernel's frame range for that tile must begin; the max-of-tag claim keeps the smallest frame.
// A connection's frame 0 starts its range at its begin when the previous connection's last
// frame ended exactly there (back to back, nothing undecoded: one claimer per tile), else at
// the tile holding its begin: that tile, when it starts in an earlier connection's frame, is
// claimed by that frame as well (the smaller index wins), and tiles wholly between
// connections' frames (gaps, undecoded tails) hold no payload byte and stay unclaimed, which
// the payload kernel skips.  (Always the tile floor cost C2 streams 8 us: four connections per
// tile claiming it from neighbouring lanes of one instruction.)
__device__ inline uint64_t tile_floor(uint64_t b) { return b / kMapTile * kMapTile; }
__device__ inline uint64_t claim_start(const WalkArgs& w, uint32_t s, const uvhttp_ws_stream_t& st) {
    if (s == 0) return tile_floor(st.begin);
    const uvhttp_ws_stream_result_t& pr = w.results[s - 1];
    const uint64_t pb = w.streams[s - 1].begin;
    const bool exact = pr.n_frames != 0 && pr.status == 0 && pb + pr.consumed_bytes == st.begin;
    return exact ? st.begin : tile_floor(st.begin);
}
__device__ inline void stream_claim_tiles(const WalkArgs& w, uint64_t lo, uint64_t fe, uint32_t frame,
                                          uint32_t epoch) {
    const uint64_t hi = fe < w.wire_len ? fe : w.wire_len;
    for (uint64_t t = lo / kMapTile + (lo % kMapTile != 0); t * kMapTile < hi && t < w.n_tiles; ++t)
        tag_claim(&w.tile_first[t], epoch, frame, w.cas_claims);
}

// (desc_scan, wave path: at most kDescScanMax connections, so each workgroup's pass over the counts is
// 16 loads per thread of a 16 KiB array every XCD's L2 holds)
constexpr uint32_t kDescScanMax = 4096;
constexpr uint32_t kDescScanLaneMax = kBlock * kBlock;  // (k_stream_desc_lane: one block total per thread)

// lane mode: one lane per connection (few frames each) writes its descriptors in order and
// claims the tile map
__global__ __launch_bounds__(kBlock) void k_stream_desc_lane(WalkArgs w) {
    if (walk_skip(w)) return;
    StampScope stamp_(w.stamp, w.epoch, UVHTTP_WS_STAMP_STREAM_DESC, false);
    const uint32_t s = stamp_.anchor_v(blockIdx.x * kBlock + threadIdx.x);
    uint32_t first, n_total;
    if (w.desc_scan) {
        // k_swalk_scan's work here (single pass, at most kDescScanLaneMax connections): the lane
        // walk left each block's frame count in agg, at most one per thread of this block
        const uint32_t nb = (w.n_streams + kBlock - 1) / kBlock;
        const uint32_t v = threadIdx.x < nb ? w.agg[threadIdx.x] : 0u;
        uint64_t pre_b, tot;
        (void)block_exclusive_sum_u64(threadIdx.x < blockIdx.x ? v : 0u, &pre_b);
        (void)block_exclusive_sum_u64(v, &tot);
        const uint32_t c = s < w.n_streams ? w.results[s].n_frames : 0u;
        uint32_t blk_total;
        first = (uint32_t)pre_b + block_scan_u32(c, &blk_total);
        n_total = tot <= w.max_frames ? (uint32_t)tot : 0u;
        if (blockIdx.x == 0 && threadIdx.x == 0) *w.sc.n_total = n_total;
    } else {
        first = lane_first(w, s);
        n_total = s < w.n_streams ? *w.sc.n_total : 0u;
    }
    if (s >= w.n_streams) return;
    uvhttp_ws_stream_result_t r = w.results[s];
    if (n_total == 0 && r.n_frames) {
        capacity_result(r);
        w.results[s] = r;
        return;
    }
    w.results[s].first_frame = first;
    if (!r.n_frames) return;
    r.first_frame = first;
    const uvhttp_ws_stream_t st = w.streams[s];
    const uint64_t sb = slice_base(st, s);
    const uint32_t epoch = w.dev_epoch ? w.ctl[kCtlEpoch] : w.epoch;
    uint64_t lo = claim_start(w, s, st);  // (the claim rule: stream_claim_tiles)
    uint32_t msg = 0;
    for (uint32_t k = 0; k < r.n_frames; ++k) {
        const uint64_t pos = w.single ? w.sc.walk_tmp[sb + k] : w.sc.frame_off[first + k] - st.begin;
        uvhttp_ws_frame_desc_t d;
        bool fin_data;
        uint64_t fe;
        stream_frame_desc(w, st, r, k, pos, load16_at(w.wire, w.wire_len, st.begin + pos), d, fin_data, fe);
        if (d.status == UVHTTP_WS_FRAME_OK && d.opcode <= 2) d.message = msg;
        msg += fin_data ? 1u : 0u;
        w.desc[first + k] = d;
        stream_claim_tiles(w, lo, fe, first + k, epoch);
        lo = fe;
    }
}

// One wave writes connection s's descriptors (the frames' headers rebuilt from the walk's
// records or re-read with two aligned 16-byte loads each), the running message id (FIN data
// frames delivered before the frame in its connection), MSG_END, the failing frame's status,
// and claims the tile map (stream_claim_tiles).  r: the connection's result, first_frame
// placed; prev_end: where frame 0's claim range starts (claim_start;
// k_swalk_fused: the begin of the nearest earlier connection with frames — more claims than
// needed, the smallest frame still wins).
__device__ inline void stream_desc_wave(const WalkArgs& w, uint32_t s, const uvhttp_ws_stream_t& st,
                                        const uvhttp_ws_stream_result_t& r, uint64_t prev_end,
                                        uint32_t epoch) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t sb = slice_base(st, s);
    uint32_t msg = 0;  // FIN data frames delivered before this chunk
    // groups of four 64-frame chunks: every start and header load of a group is issued before
    // any is used (one chunk at a time cost two dependent round trips per 64 frames)
    constexpr int kG = 4;
    for (uint32_t g0 = 0; g0 < r.n_frames; g0 += 64 * kG) {
        uint64_t pos[kG];
        u32x4 hv[kG];
        uint2 rec[kG];
#pragma unroll
        for (int c = 0; c < kG; ++c) {
            const uint32_t k = g0 + 64 * c + lane;
            const bool act = k < r.n_frames;
            pos[c] = !act ? 0 : w.single ? w.sc.walk_tmp[sb + k] : w.sc.frame_off[r.first_frame + k] - st.begin;
            rec[c] = act && w.single && w.sc.walk_rec ? w.sc.walk_rec[sb + k] : uint2{0u, kNoRec};
        }
        // headers the walk recorded are rebuilt from their records; the others are gathered
#pragma unroll
        for (int c = 0; c < kG; ++c)
            hv[c] = rec[c].y != kNoRec ? rec_header(rec[c]) : load16_at(w.wire, w.wire_len, st.begin + pos[c]);
#pragma unroll
        for (int c = 0; c < kG; ++c) {
            if (g0 + 64 * c >= r.n_frames) break;  // (uniform)
            const uint32_t k = g0 + 64 * c + lane;
            const bool act = k < r.n_frames;
            uvhttp_ws_frame_desc_t d;
            bool fin_data = false;
            uint64_t fe = 0;
            if (act) stream_frame_desc(w, st, r, k, pos[c], hv[c], d, fin_data, fe);
            // the previous frame's end: lane - 1, or the last frame of the chunk before
            uint64_t lo = ((uint64_t)__shfl_up((uint32_t)(fe >> 32), 1, 64) << 32) | __shfl_up((uint32_t)fe, 1, 64);
            if (lane == 0) lo = prev_end;
            prev_end = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(fe >> 32), 63) << 32) |
                       __builtin_amdgcn_readlane((uint32_t)fe, 63);
            if (act) stream_claim_tiles(w, lo, fe, r.first_frame + k, epoch);
            // message id: FIN data frames delivered before this one in the connection
            const uint64_t fm = __ballot(fin_data);
            const uint32_t before = msg + (uint32_t)__builtin_popcountll(fm & ((1ull << lane) - 1));
            if (act) {
                if (d.status == UVHTTP_WS_FRAME_OK && d.opcode <= 2) d.message = before;
                if (w.nt_stores) {
                    const u32x4* dw = reinterpret_cast<const u32x4*>(&d);
                    __builtin_nontemporal_store(dw[0], reinterpret_cast<u32x4*>(w.desc + r.first_frame + k));
                    __builtin_nontemporal_store(dw[1], reinterpret_cast<u32x4*>(w.desc + r.first_frame + k) + 1);
                } else {
                    w.desc[r.first_frame + k] = d;
                }
            }
            msg += (uint32_t)__builtin_popcountll(fm);
        }
    }
}

// k_stream_desc: one wave per connection (stream_desc_wave) after k_swalk_scan.  Capacity
// overflow: every result says so, nothing else.

__device__ inline void stream_desc_block(const WalkArgs& w, uint32_t vb, StampScope& stamp_) {
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t s = stamp_.anchor_s(vb * (kBlock / 64) + wave);
    uint32_t first, n_total;
    if (w.desc_scan) {
        // k_swalk_scan's work here: the walk left each connection's frame count in agg; every
        // workgroup sums all of them (the total, capacity) and those before its first
        // connection, then adds its own earlier waves' (one launch and its boundary fewer)
        const uint32_t s0 = vb * (kBlock / 64);
        // (all 16 loads issued before any is used: as a loop they ran one round trip each,
        // 15.7 us for this kernel instead of 11.5)
        uint32_t v[kDescScanMax / kBlock];
#pragma unroll
        for (uint32_t k = 0; k < kDescScanMax / kBlock; ++k) {
            const uint32_t j = threadIdx.x + k * kBlock;
            v[k] = j < w.n_streams ? w.agg[j] : 0u;
        }
        uint64_t tot = 0, pre = 0;
#pragma unroll
        for (uint32_t k = 0; k < kDescScanMax / kBlock; ++k) {
            tot += v[k];
            pre += threadIdx.x + k * kBlock < s0 ? v[k] : 0u;
        }
        uint64_t all_pre, all_tot;
        (void)block_exclusive_sum_u64(pre, &all_pre);
        (void)block_exclusive_sum_u64(tot, &all_tot);
        for (uint32_t k = s0; k < s && k < w.n_streams; ++k) all_pre += w.agg[k];
        first = (uint32_t)all_pre;
        n_total = all_tot <= w.max_frames ? (uint32_t)all_tot : 0u;
        if (vb == 0 && threadIdx.x == 0) *w.sc.n_total = n_total;
        if (s >= w.n_streams) return;
    } else {
        if (s >= w.n_streams) return;
        first = w.agg[s];  // (k_swalk_scan's prefix)
        n_total = *w.sc.n_total;
    }
    // every load of the setup issued together
    uvhttp_ws_stream_result_t r = w.results[s];
    const uvhttp_ws_stream_t st = w.streams[s];
    r.first_frame = first;
    const bool fits = n_total != 0 || r.n_frames == 0;
    if (!fits) {
        if (lane == 0) {
            capacity_result(r);
            w.results[s] = r;
        }
        return;
    }
    if (lane == 0) w.results[s].first_frame = r.first_frame;
    if (!r.n_frames) return;
    stream_desc_wave(w, s, st, r, claim_start(w, s, st), w.dev_epoch ? w.ctl[kCtlEpoch] : w.epoch);
}

__global__ __launch_bounds__(kBlock) void k_stream_desc(WalkArgs w) {
    if (walk_skip(w)) return;
    StampScope stamp_(w.stamp, w.epoch, UVHTTP_WS_STAMP_STREAM_DESC, false);
    stream_desc_block(w, blockIdx.x, stamp_);
}

// (behind the speculative decode: k_swalk_wave_gated's grid)
__global__ __launch_bounds__(kBlock) void k_stream_desc_gated(WalkArgs w, uint32_t n_blocks) {
    if (walk_skip(w)) return;
    StampScope stamp_(w.stamp, w.epoch, UVHTTP_WS_STAMP_STREAM_DESC, false);
    for (uint32_t vb = blockIdx.x; vb < n_blocks; vb += gridDim.x) {
        __syncthreads();  // (the previous block's LDS in the block sums)
        stream_desc_block(w, vb, stamp_);
    }
}

// ---- speculative stream decode (k_sspec_*) ------------------------------------------------
// The walk reads every frame's header on its own — a scattered 128-byte line per frame (C4
// streams: 166 MB moved for 1 M headers, 31.5 us) — before the payload pass reads the same
// lines again.  For a call whose connections' frames all have the wire length of their first
// frame (a client sending equal frames: the C4 stream shape) the payload pass can find and check
// the headers itself:
//   k_sspec_plan   a lane per connection: the growth check (src/uvhttp_websocket.c:832-857),
//                  the first frame's header (its wire length L >= 64 is the speculation: N = len
//                  / L complete frames, the rest an incomplete frame the call buffers), the
//                  message-limit bound, frame counts and first frames (the last block to finish
//                  scans the blocks' counts), and the 16 KiB tiles each connection's frames touch
//                  claimed with its index (max of the tag: the smallest connection wins);
//   k_sspec_pass   a workgroup per 16 KiB tile: the tile's connections (<= 64) from the claim
//                  map, every frame of theirs touching the tile parsed from LDS with every check
//                  before unmasking (:876-921) and its wire length checked against L, a 16-byte
//                  record per frame, each frame that passes unmasked in place;
//   k_sspec_emit   a wave per connection: the fragment state machine (:950-1015) in rounds of 64
//                  frames, descriptors (as k_stream_desc writes them) and the result (as the walk
//                  leaves it).
// The calls of a connection with a read table change nothing of this but the recv-buffer growth
// (checked per call; which call delivers a frame shows in no output), so the plan follows it.
// A connection the plan cannot speculate on (a layout or growth failure in any call, a first
// frame that fails, a complete frame of another length after the N-th, a message limit that could
// bind, frames under 64 bytes) gives the whole call to the walk before anything is unmasked; a
// frame the pass finds off the speculation, or a state-machine failure in the emit, gives it to
// the walk after: k_sspec_pass<UNDO> masks again what the pass unmasked (the same per-frame
// decision, XOR is its own inverse) and the walk path runs (its kernels, launched behind these,
// return at once unless ctl says the call is theirs: walk_skip / spec_gate).
// ------------------------------------------------------------------------------------------
struct SpecConn {   // 64 bytes, written by k_sspec_plan
    uint64_t b;       // begin in the wire
    uint64_t len;
    uint64_t size;    // recv_buffer_size after the call's growth
    uint64_t pending; // pending_bytes in (the open message carried from earlier calls)
    uint32_t L;       // speculated wire length of every frame (0: no complete frame)
    uint32_t N;       // speculated complete frames
    uint32_t local;   // frames of the block's earlier connections
    int32_t mf;       // max_frame_size
    uint32_t is_server;
    uint32_t pad[3];     // [0]: process_data calls (reads; 1 without a read table)
};
static_assert(sizeof(SpecConn) == 64, "one connection per 64 bytes");
constexpr uint32_t kSpecMinL = 64;              // frames of >= 64 bytes: at most kT / 64 start in a tile
constexpr uint32_t kSpecConnsPerTile = 32;      // (the general path's table)
constexpr uint64_t kSpecT = kMapTile;           // k_sspec_pass tile = the claim map's tile
// frames touching a tile: those starting in it (disjoint, >= 64 bytes) and the one covering its
// start — whatever the connections.  (A table sized for 64 connections' edge frames took 24.6 KB
// of LDS: 6 workgroups per CU, the pass 99 us on C4 streams.)
constexpr uint32_t kSpecMaxF = (uint32_t)(kSpecT / kSpecMinL) + 2;
constexpr uint32_t kSpecUndoGrid = 256;         // k_sspec_fallback's grid (kGatedGrid: a gated launch)

struct SpecArgs {
    uint8_t* wire;
    uint64_t wire_len;
    const uvhttp_ws_stream_t* streams;
    uint32_t n_streams;
    uint32_t max_frames;
    const uint64_t* read_end;  // [n_reads_total] or null (decode_streams)
    uint32_t n_reads_total;
    SpecConn* conns;
    uint32_t* blk;            // [plan blocks]: frames per block (k_sspec_plan)
    uint32_t* blk_pre;        // [plan blocks]: their exclusive prefix (k_sspec_tiles)
    uint32_t n_blk;
    uint64_t* conn_tile;      // [n_tiles]: tagged first connection whose frames touch the tile
    struct SpecTile* tiles;   // [n_tiles]: what k_sspec_pass needs of the tile (k_sspec_plan)
    uint64_t n_tiles;
    FrameRec8* recs;          // [max_frames]
    uvhttp_ws_frame_desc_t* desc;
    uvhttp_ws_stream_result_t* results;
    uint32_t* ctl;
    uint32_t epoch, dev_epoch, cas_claims;
    uint64_t* stamp;
};
__device__ inline uint32_t spec_epoch(const SpecArgs& a) { return a.dev_epoch ? a.ctl[kCtlEpoch] : a.epoch; }

// a stream frame's header from its 16-byte window: false if `avail` bytes do not hold the
// header; else the fields and the status of the checks before unmasking (walk_calls' order)
struct SpecHdr {
    uint64_t plen, wl;
    uint32_t hs, m, key, b0, b1;
    int32_t st;
};
__device__ inline bool spec_parse(const u32x4& hv, uint64_t avail, int32_t mf, uint32_t is_server,
                                  SpecHdr& h) {
    const uint64_t hlo = hv.x | ((uint64_t)hv.y << 32), hhi = hv.z | ((uint64_t)hv.w << 32);
    h.b0 = (uint32_t)(hlo & 0xFF);
    h.b1 = (uint32_t)((hlo >> 8) & 0xFF);
    const uint32_t code = h.b1 & 0x7F;
    h.hs = code == 126 ? 4 : code == 127 ? 10 : 2;
    if (avail < h.hs) return false;
    if (h.hs == 2) {
        h.plen = code;
    } else if (h.hs == 4) {
        h.plen = ((hlo >> 16) & 0xFF) << 8 | ((hlo >> 24) & 0xFF);
    } else {
        uint64_t v = 0;
#pragma unroll
        for (int q = 2; q < 10; ++q) v = (v << 8) | ((q < 8 ? hlo >> (8 * q) : hhi >> (8 * (q - 8))) & 0xFF);
        h.plen = v;
    }
    h.m = (h.b1 & 0x80) ? 4u : 0u;
    h.key = h.hs == 2 ? (uint32_t)(hlo >> 16) : h.hs == 4 ? (uint32_t)(hlo >> 32) : (uint32_t)(hhi >> 16);
    if (!h.m) h.key = 0;
    const uint32_t op = h.b0 & 0x0F;
    const bool fin = h.b0 & 0x80;
    int32_t st = UVHTTP_WS_FRAME_OK;
    if (h.hs == 10 && (h.plen >> 63)) st = UVHTTP_WS_FRAME_ERR_PARSE;
    else if (h.b0 & 0x70) st = UVHTTP_WS_FRAME_ERR_RSV;
    else if (op >= 8 && (h.plen > 125 || !fin)) st = UVHTTP_WS_FRAME_ERR_CONTROL;
    else if (is_server && !h.m) st = UVHTTP_WS_FRAME_ERR_UNMASKED;
    else if (h.plen > (uint64_t)(int64_t)mf) st = UVHTTP_WS_FRAME_ERR_TOO_BIG;
    h.st = st;
    h.wl = st == UVHTTP_WS_FRAME_OK ? h.hs + h.m + h.plen : 0;
    return true;
}

// What k_sspec_pass needs of a tile (one 64-byte record, loaded with the tile's bytes: no
// dependent load before the parse), written by k_sspec_tiles: the tile's first connection (the
// one whose frames cover the tile start, or the first beginning inside it) and the next one when
// it begins inside the tile too, each as (begin, L, first frame touching the tile, how many, that
// frame's index in the call), and the parsed header of the frame covering the tile start (it
// began in an earlier tile).  A tile with a third connection takes the general path (the
// connection table read from SpecConn through the claim map).  (The plan's connection threads
// writing these records themselves, with frame records indexed by wire position so that no
// first frame was needed: plan 17 us, pass 105, emit 15 on C4 — scattered records.)
struct SpecTile {
    uint32_t tag;        // the call's epoch (a stale record never matches)
    uint32_t flags;      // kSt*
    uint32_t cover_key;  // the covering frame's masking key
    uint32_t pad;
    struct {
        uint64_t b;
        uint32_t L, ka, cnt, first;
    } c[2];
};
static_assert(sizeof(SpecTile) == 64, "one 64-byte record per tile");
constexpr uint32_t kStConns = 3u, kStMore = 4u, kStCover = 8u, kStCoverGood = 16u, kStHmShift = 8,
                   kStSrv0 = 1u << 12, kStSrv1 = 1u << 13;

// the first-touching frame and count of a connection's frames in the tile at t0
__device__ inline void spec_range(uint64_t b, uint32_t L, uint32_t N, uint64_t t0, uint32_t& ka, uint32_t& cnt) {
    ka = 0;
    cnt = 0;
    if (!N) return;
    const uint64_t reg = (uint64_t)N * L;  // (< 2^32: len < 2^32, the plan's check)
    if (b + reg <= t0) return;
    ka = t0 > b ? (uint32_t)(t0 - b) / L : 0u;
    const uint64_t xl = t0 + kSpecT - 1 - b;
    const uint32_t kb = xl < reg ? (uint32_t)xl / L : N - 1;
    cnt = kb >= ka ? kb - ka + 1 : 0u;
}

__global__ __launch_bounds__(kBlock) void k_sspec_plan(SpecArgs a) {
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_SPEC_PLAN);
    const uint32_t epoch = spec_epoch(a);
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    bool ok = true;
    uint32_t N = 0, L = 0;
    if (s < a.n_streams) {
        const uvhttp_ws_stream_t st = a.streams[s];
        uint64_t size = st.recv_buffer_size;
        // laid out in the wire after the previous connection, its read table (if any) in range
        // and ending at len (else the walk reports ERR_LAYOUT)
        const uint32_t K = st.n_reads;
        ok = st.len <= a.wire_len && st.begin <= a.wire_len - st.len && !(st.len >> 32) &&
             (K == 0 || (a.read_end && st.first_read <= a.n_reads_total && K <= a.n_reads_total - st.first_read &&
                         a.read_end[st.first_read + K - 1] == st.len));
        if (ok && s > 0) {
            const uvhttp_ws_stream_t pv = a.streams[s - 1];
            ok = st.begin >= pv.begin && st.begin - pv.begin >= pv.len;
        }
        // no message can reach max_message_size: what is open plus every byte of the call
        const uint64_t lim = (uint64_t)(int64_t)st.max_message_size;
        ok = ok && (lim == 0 || (st.pending_bytes <= lim && st.len <= lim - st.pending_bytes));
        SpecHdr h;
        if (ok && st.len >= 2 && spec_parse(load16_at(a.wire, a.wire_len, st.begin), st.len, st.max_frame_size,
                                            (uint32_t)st.is_server, h)) {
            if (h.st != UVHTTP_WS_FRAME_OK) {
                ok = false;  // the call fails at its first frame: the walk reports it
            } else if (h.wl <= st.len) {
                L = (uint32_t)h.wl;
                // (L - 2 <= max_frame_size: no frame of this length can fail TOO_BIG, so the
                // pass checks the length alone)
                ok = L >= kSpecMinL && (uint64_t)L - 2 <= (uint64_t)(int64_t)st.max_frame_size &&
                     L <= (1u << kR8LenBits);  // (every payload fits its 8-byte record)
                N = ok ? (uint32_t)(st.len / L) : 0u;
                const uint64_t rem = st.len - (uint64_t)N * L;
                // the middle and the last speculated frame must be frames of length L too: a
                // connection of mixed frame sizes is left to the walk here, before the pass has
                // unmasked anything (otherwise its break costs the call a pass, an undo and the walk)
                const u32x4 hm = load16_at(a.wire, a.wire_len, st.begin + (uint64_t)(N / 2) * L);
                const u32x4 hz = load16_at(a.wire, a.wire_len, st.begin + (uint64_t)(N ? N - 1 : 0) * L);
                const u32x4 hr = load16_at(a.wire, a.wire_len, st.begin + (uint64_t)N * L);
                SpecHdr h1;
                ok = ok && spec_parse(hm, L, INT32_MAX, (uint32_t)st.is_server, h1) && h1.st == UVHTTP_WS_FRAME_OK &&
                     h1.wl == L;
                ok = ok && spec_parse(hz, L, INT32_MAX, (uint32_t)st.is_server, h1) && h1.st == UVHTTP_WS_FRAME_OK &&
                     h1.wl == L;
                SpecHdr h2;
                // what follows the N-th frame must be a frame the call cannot complete
                if (ok && rem >= 2 && spec_parse(hr, rem, st.max_frame_size, (uint32_t)st.is_server, h2))
                    ok = h2.st == UVHTTP_WS_FRAME_OK && h2.wl > rem;
            }
        }
        // the recv-buffer growth of every call (src/uvhttp_websocket.c:832-857): call k holds
        // the bytes from the first frame the earlier calls did not complete to its read's end;
        // a call whose growth fails gives the connection to the walk
        uint32_t calls = 1;
        if (ok && K <= 1) {
            ok = grow_recv(st.len, st.recv_buffer_size, st.max_frame_size, &size);
        } else if (ok) {
            const uint64_t* re = a.read_end + st.first_read;
            uint64_t prev = 0;
            for (uint32_t k = 0; k < K && ok; ++k) {
                const uint64_t end = re[k];
                const uint64_t done = L ? prev / L : 0u;  // frames the earlier calls completed
                const uint64_t pos = (done < N ? done : N) * (uint64_t)L;
                ok = end >= prev && end <= st.len && grow_recv(end - pos, size, st.max_frame_size, &size);
                prev = end;
            }
            calls = K;
        }
        if (!ok) N = L = 0;
        SpecConn c;
        c.b = st.begin;
        c.len = st.len;
        c.size = size;
        c.pending = st.pending_bytes;
        c.L = L;
        c.N = N;
        c.local = 0;
        c.mf = st.max_frame_size;
        c.is_server = (uint32_t)st.is_server;
        c.pad[0] = calls;
        c.pad[1] = c.pad[2] = 0;
        a.conns[s] = c;
        // the tiles this connection's frames touch (the tile of its begin and every tile
        // starting inside its frames)
        if (ok && N) {
            const uint64_t fe = st.begin + (uint64_t)N * L;
            tag_claim(&a.conn_tile[st.begin / kSpecT], epoch, s, a.cas_claims);
            for (uint64_t t = st.begin / kSpecT + 1; t * kSpecT < fe; ++t) tag_claim(&a.conn_tile[t], epoch, s, a.cas_claims);
        }
    }
    if (!ok) a.ctl[kCtlSpecOff] = epoch;
    uint32_t total;
    const uint32_t local = block_scan_u32(N, &total);
    if (s < a.n_streams) a.conns[s].local = local;
    // (the blocks' counts become first frames in k_sspec_tiles, which every later kernel follows:
    // a last-block scan here — a fence and an atomic per block — cost the plan about 3 us)
    if (threadIdx.x == 0) a.blk[blockIdx.x] = total;
}

// exclusive prefixes of the plan blocks' frame counts in LDS (every thread), and their total
__device__ inline uint64_t spec_blk_prefix(const SpecArgs& a, uint32_t* s_pre) {
    uint64_t base = 0;
    for (uint32_t b0 = 0; b0 < a.n_blk; b0 += kBlock) {
        const uint32_t j = b0 + threadIdx.x;
        const uint32_t v = j < a.n_blk ? a.blk[j] : 0u;
        uint64_t tot;
        const uint64_t pre = block_exclusive_sum_u64(v, &tot);
        if (j < a.n_blk) s_pre[j] = (uint32_t)(base + pre);
        base += tot;
        __syncthreads();
    }
    return base;
}
constexpr uint32_t kSpecMaxBlk = 4096;  // plan blocks (1 M connections) the LDS prefix holds

// a thread per claimed tile (after k_sspec_plan: connections and claims); every workgroup scans
// the plan blocks' frame counts (the first frames; workgroup 0 leaves them in blk_pre for the
// pass's general path and k_sspec_emit) and checks the capacity
__global__ __launch_bounds__(kBlock) void k_sspec_tiles(SpecArgs a) {
    const uint32_t epoch = spec_epoch(a);
    if (a.ctl[kCtlSpecOff] == epoch) return;
    __shared__ uint32_t s_pre[kSpecMaxBlk];
    const uint64_t total = spec_blk_prefix(a, s_pre);
    if (total > a.max_frames) {  // (ERR_CAPACITY: the walk reports it)
        if (threadIdx.x == 0) a.ctl[kCtlSpecOff] = epoch;
        return;
    }
    if (blockIdx.x == 0)
        for (uint32_t j = threadIdx.x; j < a.n_blk; j += kBlock) a.blk_pre[j] = s_pre[j];
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= a.n_tiles) return;
    const uint32_t c0 = tag_get(a.conn_tile[t], epoch, kNoFrame);
    if (c0 == kNoFrame) return;
    const uint64_t t0 = t * kSpecT;
    const SpecConn s0 = a.conns[c0];
    SpecConn s1;
    const bool has1 = c0 + 1 < a.n_streams;
    if (has1) s1 = a.conns[c0 + 1];
    const bool in1 = has1 && s1.b < t0 + kSpecT;
    const bool more = in1 && c0 + 2 < a.n_streams && a.conns[c0 + 2].b < t0 + kSpecT;
    SpecTile r;
    r.pad = 0;
    r.cover_key = 0;
    uint32_t flags = (in1 ? 2u : 1u) | (more ? kStMore : 0u) | (s0.is_server ? kStSrv0 : 0u);
    spec_range(s0.b, s0.L, s0.N, t0, r.c[0].ka, r.c[0].cnt);
    r.c[0].b = s0.b;
    r.c[0].L = s0.L;
    r.c[0].first = s_pre[c0 / kBlock] + s0.local + r.c[0].ka;
    r.c[1].b = 0;
    r.c[1].L = r.c[1].ka = r.c[1].cnt = r.c[1].first = 0;
    if (in1) {
        spec_range(s1.b, s1.L, s1.N, t0, r.c[1].ka, r.c[1].cnt);
        r.c[1].b = s1.b;
        r.c[1].L = s1.L;
        r.c[1].first = s_pre[(c0 + 1) / kBlock] + s1.local + r.c[1].ka;
        if (s1.is_server) flags |= kStSrv1;
    }
    if (r.c[0].cnt + r.c[1].cnt > kSpecMaxF) flags |= kStMore;
    const uint64_t o = s0.b + (uint64_t)r.c[0].ka * s0.L;
    if (r.c[0].cnt && o < t0) {  // the frame covering the tile start
        SpecHdr h;
        const bool good = spec_parse(load16_at(a.wire, a.wire_len, o), s0.L, INT32_MAX, s0.is_server, h) &&
                          h.st == UVHTTP_WS_FRAME_OK && h.wl == s0.L;
        flags |= kStCover | (good ? kStCoverGood : 0u) | ((h.hs + h.m) << kStHmShift);
        r.cover_key = h.key;
    }
    r.flags = flags;
    r.tag = epoch;
    a.tiles[t] = r;
}

// One 16 KiB tile of the speculative pass (UNDO: mask again what the pass unmasked, nothing
// else written).  Returns with every thread at the same point (the callers loop over tiles).
template <bool UNDO>
__device__ inline void sspec_tile(const SpecArgs& a, uint64_t tile, uint32_t epoch) {
    constexpr int BLOCK = kBlock, VPT = 4;
    constexpr uint64_t kT = kSpecT;
    static_assert((uint64_t)BLOCK * VPT * 16 == kT, "tile = claim map tile");
    __shared__ u32x4 s_tile[BLOCK * VPT + 1];
    __shared__ int4 s_fr[kSpecMaxF];
    __shared__ uint64_t s_cb[kSpecConnsPerTile];
    __shared__ uint32_t s_cL[kSpecConnsPerTile], s_cka[kSpecConnsPerTile], s_cfirst[kSpecConnsPerTile];
    __shared__ uint32_t s_cpre[kSpecConnsPerTile + 1];
    __shared__ uint32_t s_csrv[kSpecConnsPerTile];
    __shared__ uint32_t s_nc, s_bad, s_cov, s_covkey;  // s_cov: kStCover | kStCoverGood | hm
    const uint64_t t0 = tile * kT;
    const uint64_t vend = a.wire_len;
    const uint64_t full_end = vend & ~(uint64_t)15;
    const uint64_t clamp_va = full_end ? full_end - 16 : 0;
    u32x4 data[VPT];
    uint64_t va[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        va[v] = t0 + ((uint64_t)v * BLOCK + threadIdx.x) * 16u;
        const uint64_t la = va[v] < full_end ? va[v] : clamp_va;
        data[v] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.wire + la));
    }
    u32x4 extra = u32x4{0, 0, 0, 0};
    if (threadIdx.x == 1) extra = load16_at(a.wire, vend, t0 + kT);
    const SpecTile tr = a.tiles[tile];  // (uniform: scalar loads beside the tile's)
    if (!UNDO && a.ctl[kCtlSpecOff] == epoch) return;  // the plan gave the call to the walk
    const bool fast = tr.tag == epoch && !(tr.flags & kStMore);
    if (fast) {
        if (threadIdx.x == 0) {
            const uint32_t nc = tr.flags & kStConns;
            s_nc = nc;
            s_bad = 0;
            s_cpre[0] = 0;
#pragma unroll
            for (uint32_t l = 0; l < 2; ++l) {
                s_cb[l] = tr.c[l].b;
                s_cL[l] = tr.c[l].L;
                s_cka[l] = tr.c[l].ka;
                s_cfirst[l] = tr.c[l].first - tr.c[l].ka;  // (index of the connection's frame 0)
                s_csrv[l] = (tr.flags & (l ? kStSrv1 : kStSrv0)) ? 1u : 0u;
            }
            s_cpre[1] = tr.c[0].cnt;
            s_cpre[2] = tr.c[0].cnt + (nc > 1 ? tr.c[1].cnt : 0u);
            s_cov = tr.flags & (kStCover | kStCoverGood | (0xFu << kStHmShift));
            s_covkey = tr.cover_key;
        }
    } else {
        // the general path: the tile's connections from the claim map and SpecConn
        const uint32_t c0 = tag_get(a.conn_tile[tile], epoch, kNoFrame);
        if (c0 == kNoFrame) return;  // (uniform) no connection's frames touch the tile
        const uint32_t lane = threadIdx.x & 63;
        if (threadIdx.x < 64) {
            // c0 and the connections after it that begin before the tile's end
            const uint32_t c = c0 + lane;
            const bool valid = c < a.n_streams;
            SpecConn sc;
            if (valid) sc = a.conns[c];
            const bool beyond = !valid || sc.b >= t0 + kT || lane >= kSpecConnsPerTile;
            const uint64_t bm = __ballot(beyond);
            const uint32_t nc = (uint32_t)__builtin_ctzll(bm);  // (lane kSpecConnsPerTile is beyond)
            uint32_t cnt = 0, ka = 0;
            if (lane < nc) spec_range(sc.b, sc.L, sc.N, t0, ka, cnt);
            uint32_t inc = cnt;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(inc, d, 64);
                if (lane >= (uint32_t)d) inc += o;
            }
            if (lane < nc) {
                s_cb[lane] = sc.b;
                s_cL[lane] = sc.L;
                s_cka[lane] = ka;
                s_cfirst[lane] = sc.N ? a.blk_pre[c / kBlock] + sc.local : 0u;
                s_csrv[lane] = sc.is_server;
                s_cpre[lane + 1] = inc;
            }
            const uint32_t F = __shfl(inc, 63, 64);
            if (lane == 0) {
                s_cpre[0] = 0;
                s_nc = nc;
                // more connections than one wave reads, or more frames than the table holds:
                // the call goes to the walk (the undo pass decides the same: nothing unmasked)
                s_bad = (nc == kSpecConnsPerTile && c0 + kSpecConnsPerTile < a.n_streams &&
                         a.conns[c0 + kSpecConnsPerTile].b < t0 + kT) || F > kSpecMaxF;
                // the frame covering the tile start (only the first connection's can begin before it)
                s_cov = 0;
                s_covkey = 0;
                if (cnt && sc.b + (uint64_t)ka * sc.L < t0) {
                    SpecHdr h;
                    const bool good = spec_parse(load16_at(a.wire, vend, sc.b + (uint64_t)ka * sc.L), sc.L,
                                                 INT32_MAX, sc.is_server, h) &&
                                      h.st == UVHTTP_WS_FRAME_OK && h.wl == sc.L;
                    s_cov = kStCover | (good ? kStCoverGood : 0u) | ((h.hs + h.m) << kStHmShift);
                    s_covkey = h.key;
                }
            }
        }
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        u32x4 x = data[v];
        if (va[v] == full_end && full_end < vend) x = load16_at(a.wire, vend, full_end);
        s_tile[v * BLOCK + threadIdx.x] = x;
    }
    if (threadIdx.x == 1) s_tile[BLOCK * VPT] = extra;
    __syncthreads();
    if (s_bad) {
        if (!UNDO && threadIdx.x == 0) a.ctl[kCtlSpecBreak] = epoch;
        return;
    }
    const uint32_t nc = s_nc, F = s_cpre[nc];
    for (uint32_t j = threadIdx.x; j < F; j += BLOCK) {
        uint32_t lo = 0, hi = nc - 1;  // the connection: last l with s_cpre[l] <= j
        while (nc > 1 && lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (s_cpre[mid] <= j) lo = mid;
            else hi = mid - 1;
        }
        const uint32_t l = lo;
        const uint32_t k = s_cka[l] + (j - s_cpre[l]);
        const uint32_t L = s_cL[l];
        const uint64_t o = s_cb[l] + (uint64_t)k * L;
        if (o < t0) {  // the covering frame (its header in an earlier tile: parsed before)
            const uint32_t cov = s_cov, hm = (cov >> kStHmShift) & 0xFu;
            const bool good = cov & kStCoverGood;
            if (!UNDO && !good) a.ctl[kCtlSpecBreak] = epoch;
            const uint64_t ps = o + hm;
            s_fr[j] = int4{rel_clamp(ps, t0, kT, true), rel_clamp(good ? o + L : ps, t0, kT, false),
                           (int32_t)s_covkey, 0};
            continue;
        }
        SpecHdr h;
        // (no TOO_BIG check: the plan required L - 2 <= max_frame_size, so no frame of wire
        // length L can be too big, and one claiming a larger length fails wl == L)
        const bool good = spec_parse(lds_window(s_tile, (uint32_t)(o - t0)), L, INT32_MAX, s_csrv[l], h) &&
                          h.st == UVHTTP_WS_FRAME_OK && h.wl == L;
        if (!UNDO) {
            if (!good) a.ctl[kCtlSpecBreak] = epoch;
            FrameRec r;
            r.payload_len = h.plen;
            r.masking_key = h.key;
            r.opcode = (uint8_t)(h.b0 & 0x0F);
            r.flags = (uint8_t)(((h.b0 >> 7) & 1) | ((h.b1 >> 7) << 1) | kRecHasLen);
            r.header_size = (uint8_t)h.hs;
            r.status = (int8_t)(good ? UVHTTP_WS_FRAME_OK : UVHTTP_WS_FRAME_ERR_LAYOUT);
            rec8_store(a.recs, s_cfirst[l] + k, r);
        }
        const uint64_t ps = o + h.hs + h.m;
        s_fr[j] = int4{rel_clamp(ps, t0, kT, true), rel_clamp(good ? ps + h.plen : ps, t0, kT, false),
                       (int32_t)h.key, 0};
    }
    __syncthreads();
    // each vector's mask.  Up to two connections in the tile (every tile of a call of large
    // connections) by arithmetic, as k_unmask_stride: the frames of byte x of connection l are
    // (x - start of its first frame in the tile) / L; more, by a binary search over the table
    // (frames in wire order: payload ranges sorted and disjoint).  (A search per vector cost the
    // pass 124 us on C4 streams.)
    u32x4 m[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) m[v] = u32x4{0, 0, 0, 0};
    if (nc <= 2) {
        for (uint32_t l = 0; l < nc; ++l) {
            const uint32_t Ll = s_cL[l], cnt = s_cpre[l + 1] - s_cpre[l], base = s_cpre[l];
            if (!cnt) continue;
            const int64_t fs = (int64_t)(s_cb[l] + (uint64_t)s_cka[l] * Ll) - (int64_t)t0;  // first frame, tile-relative
            const float inv_l = 1.0f / (float)Ll;
#pragma unroll
            for (int v = 0; v < VPT; ++v) {
                if (va[v] >= vend) continue;
                const int64_t rel = (int64_t)((v * BLOCK + threadIdx.x) * 16) - fs;
                if (rel + 15 < 0) continue;
                uint32_t lo, hi;
                if (Ll < (1u << 20) && rel + 15 < (1 << 24)) {  // (div_small: offsets below 2^24)
                    lo = rel < 0 ? 0u : div_small((uint32_t)rel, Ll, inv_l);
                    hi = div_small((uint32_t)(rel + 15), Ll, inv_l);
                } else {
                    lo = rel < 0 ? 0u : (uint32_t)((uint64_t)rel / Ll);
                    hi = (uint32_t)((uint64_t)(rel + 15) / Ll);
                }
                if (lo >= cnt) continue;
                hi = hi < cnt - 1 ? hi : cnt - 1;
                const int32_t r = (int32_t)((v * BLOCK + threadIdx.x) * 16);
                for (uint32_t j = lo; j <= hi; ++j) {
                    const int4 fr = s_fr[base + j];
                    add_mask_rel(m[v], r, fr.x, fr.y, (uint32_t)fr.z);
                }
            }
        }
    } else {
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            if (va[v] >= vend || F == 0) continue;
            const int32_t r = (int32_t)((v * BLOCK + threadIdx.x) * 16);
            uint32_t lo = 0, hi = F;  // first j with pe > r
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_fr[mid].y > r) hi = mid;
                else lo = mid + 1;
            }
            for (uint32_t j = lo; j < F; ++j) {
                const int4 fr = s_fr[j];
                if (fr.x >= r + 16) break;
                add_mask_rel(m[v], r, fr.x, fr.y, (uint32_t)fr.z);
            }
        }
    }
    const uint64_t room = vend > t0 ? vend - t0 : 0;
    const uint32_t nrec = (uint32_t)(room < kT ? room : kT);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.wire + t0, 0, (int)nrec, 0x00020000);
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        if (any_bits(m[v]) && va[v] + 16 <= vend) {
            const u32x4 x = data[v] ^ m[v];
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, x), rs,
                (uint32_t)(va[v] - t0), 0, 18);
        }
    }
    if (full_end != vend && full_end >= t0 && full_end < t0 + kT) {
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            if (va[v] == full_end && any_bits(m[v])) {
                const uint32_t mw[4] = {m[v].x, m[v].y, m[v].z, m[v].w};
                for (uint64_t bq = 0; full_end + bq < vend; ++bq) {
                    const uint8_t mb = (uint8_t)(mw[bq >> 2] >> (8 * (bq & 3)));
                    if (mb) a.wire[full_end + bq] ^= mb;
                }
            }
        }
    }
}

// the pass: a workgroup per tile; UNDO (only when the speculation broke): a grid-stride loop
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(7))) void k_sspec_pass(SpecArgs a, uint64_t tile_base) {
    const uint32_t epoch = spec_epoch(a);
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_PAYLOAD, false, tile_base);
    sspec_tile<false>(a, tile_base + stamp_.anchor_s(blockIdx.x), epoch);
}


// a wave per connection: the state machine over the pass's records, descriptors, the result
__global__ __launch_bounds__(kBlock) void k_sspec_emit(SpecArgs a) {
    const uint32_t epoch = spec_epoch(a);
    if (a.ctl[kCtlSpecOff] == epoch || a.ctl[kCtlSpecBreak] == epoch) return;
    StampScope stamp_(a.stamp, a.epoch, UVHTTP_WS_STAMP_STREAM_DESC, false);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t s = stamp_.anchor_s(blockIdx.x * (kBlock / 64) + wave);
    if (s >= a.n_streams) return;
    const SpecConn sc = a.conns[s];
    const uint32_t first = a.blk_pre[s / kBlock] + sc.local;
    bool open = sc.pending != 0;
    uint64_t acc = sc.pending;
    uint32_t msg = 0;
    const uint64_t below = (1ull << lane) - 1;
    for (uint32_t r0 = 0; r0 < sc.N; r0 += 64) {
        const uint32_t k = r0 + lane;
        const bool act = k < sc.N;
        FrameRec rec;
        rec.payload_len = 0;
        rec.masking_key = 0;
        rec.opcode = 8;
        rec.flags = 0;
        rec.header_size = 2;
        rec.status = 0;
        // (an escaped record — a payload of 2^23 bytes or more — gives the call to the walk;
        // the plan keeps L <= 2^23, so a speculated frame never has one)
        const bool esc = act && !rec8_unpack(a.recs[first + k], rec);
        const bool data = act && rec.opcode <= 2;
        const bool fin = rec.flags & UVHTTP_WS_FLAG_FIN;
        const bool cont = rec.opcode == 0;
        // the message open after this frame (a data frame): CONT keeps it until FIN; a start
        // opens one unless FIN or empty (an empty first fragment allocates nothing, :794-816)
        const bool oa = cont ? !fin : (!fin && rec.payload_len != 0);
        const uint64_t dm = __ballot(data), om = __ballot(data && oa);
        const uint64_t prior = dm & below;
        const bool open_before = prior ? ((om >> (63 - __builtin_clzll(prior))) & 1) : open;
        const bool fail = esc || (data && (cont ? !open_before : open_before));
        if (__ballot(fail)) {  // the reference stops here: the walk reports it
            if (lane == 0) a.ctl[kCtlSpecBreak] = epoch;
            return;
        }
        const bool fin_data = data && fin;
        const uint64_t fm = __ballot(fin_data);
        if (act) {
            const uint64_t pos = (uint64_t)k * sc.L;
            uvhttp_ws_frame_desc_t d;
            d.payload_off = sc.b + pos + rec.header_size + ((rec.flags & UVHTTP_WS_FLAG_MASK) ? 4u : 0u);
            d.payload_len = rec.payload_len;
            d.masking_key = rec.masking_key;
            d.message = data ? msg + (uint32_t)__builtin_popcountll(fm & below) : 0u;
            d.opcode = rec.opcode;
            d.flags = (uint8_t)((rec.flags & ~kRecHasLen) | (fin_data ? UVHTTP_WS_FLAG_MSG_END : 0u));
            d.header_size = rec.header_size;
            d.status = UVHTTP_WS_FRAME_OK;
            d.wire_len = sc.L;
            a.desc[first + k] = d;
        }
        // what the round leaves open: the latest data frame decides; the bytes since the latest
        // start (a start or a FIN resets them)
        const uint64_t rm = __ballot(data && (!cont || fin));
        const int jr = rm ? 63 - __builtin_clzll(rm) : -1;
        uint64_t add = (data && (int)lane > jr) ? rec.payload_len : 0u;
        if ((int)lane == jr && !cont && !fin) add = rec.payload_len;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) add += __shfl_xor(add, d, 64);
        acc = jr >= 0 ? add : acc + add;
        if (dm) open = (om >> (63 - __builtin_clzll(dm))) & 1;
        msg += (uint32_t)__builtin_popcountll(fm);
    }
    if (lane == 0) {
        uvhttp_ws_stream_result_t r;
        r.first_frame = first;
        r.n_frames = sc.N;
        r.n_delivered = sc.N;
        r.status = 0;
        r.first_status = 0;
        r.calls = sc.pad[0];
        r.consumed_bytes = (uint64_t)sc.N * sc.L;
        r.recv_buffer_size = sc.size;
        r.pending_bytes = open ? acc : 0u;
        r.buffered_end = sc.len;
        r.reserved = 0;
        a.results[s] = r;
    }
}

// The walk path behind a speculative attempt ends here, gated, in a grid-stride loop (a no-op
// launch of one workgroup per tile costs more than the loop): when the pass ran and the
// speculation broke, each tile first gets the pass's unmask undone (k_sspec_pass's decisions
// again — the walk and k_stream_desc before this read only headers, which no pass changes),
// then the in-place payload kernel's work from the walk's descriptors.
__global__ __launch_bounds__(kBlock) void k_sspec_fallback(SpecArgs sa, BatchArgs a,
                                                           const uvhttp_ws_frame_desc_t* __restrict__ desc,
                                                           Workspace ws, uint64_t n_tiles) {
    resolve_epoch(a, ws);
    if (!spec_slow(ws.ctl, a.epoch)) return;
    const bool undo = ws.ctl[kCtlSpecOff] != a.epoch;  // (the pass ran: its unmask is undone)
    StampScope ss(nullptr, 0, 0, false);
    for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
        __syncthreads();  // (the previous tile's LDS)
        if (undo) {
            sspec_tile<true>(sa, t, a.epoch);
            __syncthreads();
        }
        uint32_t n, nb;
        unmask_tile<kBlock, 4, 18>(a, desc, ws, t - blockIdx.x, n, nb, ss);
    }
}

// ---- k_swalk_fused: walk, first frame and descriptors of a connection in one launch -------
// The wave walk in single pass (k_swalk_wave<2>), then k_swalk_scan's prefix by a decoupled
// look-back over connections, then k_stream_desc's work — one launch where there were three
// (C4 streams: the scan and the descriptor pass with their launch gaps were 17 us of 147).
// Blocks take tickets in launch order (connections 4 ticket .. 4 ticket + 3, a wave each), so
// a block only waits on blocks that already run.  Each block publishes the aggregate of its
// four connections (A record), then its 256 threads combine their predecessors' records, 256
// blocks per round, back to the nearest inclusive prefix (P record) — a look-back per
// connection, 64 per round, took n / 64 dependent rounds when the walks end together: C4
// streams 307 us per step instead of 149.  A record is one device-coherent 16-byte access:
// frame count (saturated at 2^32 - 1), begin + 1 of the latest connection with frames (0:
// none — k_stream_desc's prev_end), tag (epoch << 2 | kind).  Polls are bounded as k_plan's: a wave that gives up
// publishes anyway and records the device fault.  The connection whose wave finishes last
// (a counter) rewrites every result when the call overflowed max_frames (ERR_CAPACITY, as
// k_stream_desc) or faulted (ERR_DEVICE: nothing delivered).
constexpr uint32_t kSwAgg = 1, kSwPrefix = 2;

struct SwVal {
    uint32_t count;  // frames (saturated)
    uint64_t hb;     // begin + 1 of the latest connection with frames, 0: none
};

__device__ inline SwVal sw_combine(const SwVal& e, const SwVal& l) {
    const uint64_t c = (uint64_t)e.count + l.count;
    return SwVal{c > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)c, l.hb ? l.hb : e.hb};
}

__device__ inline void sw_store(const WalkArgs& w, uint32_t slot, const SwVal& v, uint32_t tag) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(w.sc.srec, 0, 0x7FFFFFFF, 0x00020000);
    const u32x4v x = {v.count, (uint32_t)v.hb, (uint32_t)(v.hb >> 32), tag};
    __builtin_amdgcn_raw_buffer_store_b128(x, rs, slot * 16u, 0, kAuxSc1);
}

__device__ inline u32x4v sw_fetch(const WalkArgs& w, uint32_t slot) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(w.sc.srec, 0, 0x7FFFFFFF, 0x00020000);
    return __builtin_amdgcn_raw_buffer_load_b128(rs, slot * 16u, 0, kAuxSc1);
}

// block b's exclusive prefix (every thread; records: A at 2 b, P at 2 b + 1), k_plan's
// look-back over SwVal: 256 predecessors per round, thread t taking block end - 256 + t
__device__ inline SwVal sw_lookback(const WalkArgs& w, uint32_t b, const SwVal& agg, uint32_t epoch,
                                    bool& gave_up) {
    __shared__ uint32_t s_cnt[kBlock / 64];
    __shared__ uint64_t s_hb[kBlock / 64];
    __shared__ int s_kstar;
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t ta = (epoch << 2) | kSwAgg, tp = (epoch << 2) | kSwPrefix;
    gave_up = false;
    if (b == 0) {
        if (t == 0) sw_store(w, 1, agg, tp);
        return SwVal{0u, 0ull};
    }
    if (t == 0) sw_store(w, 2 * b, agg, ta);
    SwVal run{0u, 0ull};  // the predecessors combined so far (all newer than the next window)
    int64_t end = b;      // window: blocks [end - 256, end), thread 255 the newest
    uint32_t polls = 0;   // (uniform: every thread counts the same rounds)
    for (;;) {
        const int64_t j = end - kBlock + (int64_t)t;
        SwVal v{0u, 0ull};
        bool is_p = j < 0, ready = j < 0;  // (before block 0: identity "P")
        for (;;) {
            if (!ready) {  // both records in one round trip
                const u32x4v xp = sw_fetch(w, 2 * (uint32_t)j + 1);
                const u32x4v xa = sw_fetch(w, 2 * (uint32_t)j);
                if (xp.w == tp) {
                    v = SwVal{xp.x, xp.y | ((uint64_t)xp.z << 32)}, is_p = true, ready = true;
                } else if (xa.w == ta) {
                    v = SwVal{xa.x, xa.y | ((uint64_t)xa.z << 32)}, ready = true;
                }
            }
            if (__syncthreads_and(ready) && w.max_polls) break;
            if (++polls > w.max_polls) {
                gave_up = true;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
        // from the newest published prefix (the highest thread with P) to the newest block
        if (t == 0) s_kstar = -1;
        __syncthreads();
        const uint64_t pm = __ballot(is_p);
        if (lane == 0 && pm) atomicMax(&s_kstar, (int)(wave * 64 + 63 - __builtin_clzll(pm)));
        __syncthreads();
        const int kstar = s_kstar;
        if ((int)t < kstar) v = SwVal{0u, 0ull};
        uint64_t cnt = v.count;
#pragma unroll
        for (int d = 32; d; d >>= 1) cnt += __shfl_xor(cnt, d, 64);
        const uint64_t hm = __ballot(v.hb != 0);
        uint64_t hb = 0;
        if (hm) {
            const uint32_t hl = 63 - __builtin_clzll(hm);
            hb = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v.hb >> 32), hl) << 32) |
                 __builtin_amdgcn_readlane((uint32_t)v.hb, hl);
        }
        if (lane == 0) {
            s_cnt[wave] = cnt > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cnt;
            s_hb[wave] = hb;
        }
        __syncthreads();
        SwVal win{0u, 0ull};
#pragma unroll
        for (int k = 0; k < kBlock / 64; ++k) win = sw_combine(win, SwVal{s_cnt[k], s_hb[k]});
        run = sw_combine(win, run);
        __syncthreads();  // (s_kstar, s_cnt, s_hb reused by the next round)
        if (kstar >= 0 || gave_up) break;
        end -= kBlock;
    }
    if (t == 0) sw_store(w, 2 * b + 1, sw_combine(run, agg), tp);
    return run;
}

__device__ inline void device_result(uvhttp_ws_stream_result_t& r) {
    capacity_result(r);
    r.first_status = UVHTTP_WS_FRAME_ERR_DEVICE;
}

__global__ __launch_bounds__(kBlock) void k_swalk_fused(WalkArgs w) {
    StampScope stamp_(w.stamp, w.epoch, UVHTTP_WS_STAMP_WALK, false);
    __shared__ __attribute__((aligned(16))) uint8_t ring[kBlock / 64][kRingBytes];
    __shared__ uint32_t s_ticket;
    if (threadIdx.x == 0) {
        uint32_t t = blockIdx.x;
        if (!w.no_ticket) {
            t = __hip_atomic_fetch_add(&w.sc.ctr[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (t + 1 == gridDim.x) __hip_atomic_store(&w.sc.ctr[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        s_ticket = t;
    }
    __syncthreads();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t bt = __builtin_amdgcn_readfirstlane(s_ticket);
    const uint32_t s = stamp_.anchor_s(bt * (kBlock / 64) + wave);
    const uint32_t epoch = w.dev_epoch ? w.ctl[kCtlEpoch] : w.epoch;
    // (a wave past the last connection still joins the block's look-back, with nothing)
    uvhttp_ws_stream_result_t r;
    memset(&r, 0, sizeof(r));
    if (s < w.n_streams) r = walk_wave<3>(w, s, ring[wave]);
    const SwVal mine{s < w.n_streams ? r.n_frames : 0u, s < w.n_streams && r.n_frames ? w.streams[s].begin + 1 : 0ull};
    // the block's four connections in order: each wave's prefix within the block, the block's
    // aggregate; then the block's prefix (the slice stores of each wave are ordered before its
    // own reads by the barriers)
    __shared__ uint32_t s_wc[kBlock / 64];
    __shared__ uint64_t s_wh[kBlock / 64];
    if (lane == 0) {
        s_wc[wave] = mine.count;
        s_wh[wave] = mine.hb;
    }
    __syncthreads();
    SwVal local{0u, 0ull}, agg{0u, 0ull};
#pragma unroll
    for (uint32_t k = 0; k < kBlock / 64; ++k) {
        if (k == wave) local = agg;
        agg = sw_combine(agg, SwVal{s_wc[k], s_wh[k]});
    }
    bool gave_up;
    const SwVal pre = sw_combine(sw_lookback(w, bt, agg, epoch, gave_up), local);
    if (s >= w.n_streams) return;
    r.first_frame = pre.count;
    const uint64_t incl = (uint64_t)pre.count + r.n_frames;
    const bool over = incl > w.max_frames;
    uint32_t* ctl = const_cast<uint32_t*>(w.ctl);
    if (lane == 0) {
        if (gave_up) {  // k_plan's give-up: the payload kernel unmasks nothing (first_bad 0)
            __hip_atomic_store(&ctl[kCtlFaultEp], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&ctl[kCtlFaults], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            tag_claim(w.first_bad, epoch, 0, 1u);
        }
        uvhttp_ws_stream_result_t o = r;
        if (over && r.n_frames) capacity_result(o);
        w.results[s] = o;
        // the total (0 over capacity); a call over capacity, known from the last connection's
        // total only, or with a device fault has every result rewritten by the payload kernel's
        // first workgroup (stream_fix: after this kernel, so with every result visible)
        if (s + 1 == w.n_streams) {
            *w.sc.n_total = over ? 0u : (uint32_t)incl;
            if (over) w.sc.ctr[2] = epoch;
        }
    }
    if (!over && !gave_up && r.n_frames) stream_desc_wave(w, s, w.streams[s], r, pre.hb ? pre.hb - 1 : 0ull, epoch);
}



// ------------------------------------------------------------------------------------
// send side: batched uvhttp_ws_build_frame (:204-285).  kb_size -> two-level u64 scan ->
// kb_offsets -> kb_emit.  kb_emit is an HBM-bound scatter: one workgroup per output tile,
// each 16-byte output vector assembled from the covering frame's header image (staged in
// LDS) and its payload (one unaligned 16-byte source window, XORed with the rotated key
// for client frames).  Bytes per frame: P read + (H + 4m + P) written.
// ------------------------------------------------------------------------------------
// Emit record of one built frame, copied by kb_offsets into every 16 KiB output-map tile whose
// first byte the frame covers (exactly one frame covers a byte, so each tile has one writer
// and no atomics).  64 bytes = one scalar s_load_dwordx16 in kb_emit, so a tile's lookup is a
// single dependent round trip before its payload loads.
struct __attribute__((aligned(64))) BuildRec {
    uint64_t st;     // frame start in out
    uint64_t ps;     // payload start in out
    uint64_t fe;     // frame end in out
    uint64_t src;    // payload offset in src
    u32x4 img;       // header image (<= 14 bytes)
    uint32_t key;    // 0 for server frames (XOR no-op)
    uint32_t frame;  // frame index
    uint32_t tag;    // epoch of the call that wrote it
    uint32_t pad;
};
static_assert(sizeof(BuildRec) == 64, "one s_load_dwordx16");

struct BuildArgs {
    const uint8_t* src;
    uint64_t src_len;
    const uvhttp_ws_build_desc_t* frames;
    uint32_t n;
    uint8_t* out;
    uint64_t out_cap;
    uint64_t* out_off;   // [n + 1]
    uint64_t* blk;       // per-block sums -> prefixes (u64 scratch)
    uint64_t* grp;       // per-group sums -> prefixes, [n_groups] = total
    BuildRec* mrec;      // output map tile -> record of the frame covering its first byte
    uint64_t n_map;
    uint32_t map_shift;  // log2 of the map tile (>= the emit tile; ~ the average frame size)
    uint32_t epoch;      // tag of this call's map records (stale records never match)
    uint32_t group;      // kb_emit_frames: frames per workgroup (<= kEmitF)
    uint32_t n_groups;   // grp[n_groups] = the total output bytes
    const uint32_t* ctl; // captured calls (dev_epoch): the epoch is ctl[kCtlEpoch]
    uint32_t dev_epoch;
    uint64_t* stamp;     // device-side kernel stamps (diagnostics), or null
};

__device__ inline void resolve_epoch(BuildArgs& b) {
    if (b.dev_epoch) b.epoch = b.ctl[kCtlEpoch];
}

__device__ inline uint64_t build_size(const uvhttp_ws_build_desc_t& f) {
    const uint64_t p = f.payload_len;
    return (p < 126 ? 2 : p < 65536 ? 4 : 10) + (f.mask ? 4 : 0) + p;
}


// per 256-frame block: the frames' sizes, their offsets within the block (out_off, made final by
// kb_emit_frames or kb_offsets) and the block's total (blk)
__global__ __launch_bounds__(kBlock) void kb_size(BuildArgs b) {
    StampScope stamp_(b.stamp, b.epoch, UVHTTP_WS_STAMP_BUILD_SIZE);
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint64_t sz = i < b.n ? build_size(b.frames[i]) : 0;
    uint64_t total;
    const uint64_t local = block_exclusive_sum_u64(sz, &total);
    if (i < b.n) b.out_off[i] = local;
    if (threadIdx.x == 0) b.blk[blockIdx.x] = total;
}

// the block totals' exclusive prefixes in one workgroup when there are at most kScanOne of them
// (batches of <= 1 M frames; one launch instead of kb_scan_groups + kb_scan_top): blk[k] becomes
// the prefix, grp[0 .. n_groups) = 0 and grp[n_groups] the total, the two-level layout's meaning
constexpr uint32_t kScanOnePer = 16, kScanOne = kBlock * kScanOnePer;
__global__ __launch_bounds__(kBlock) void kb_scan_one(BuildArgs b, uint32_t n_blocks) {
    StampScope stamp_(b.stamp, b.epoch, UVHTTP_WS_STAMP_BUILD_SCAN);
    uint64_t v[kScanOnePer], run = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanOnePer; ++k) {
        const uint32_t g = threadIdx.x * kScanOnePer + k;
        v[k] = g < n_blocks ? b.blk[g] : 0;
        run += v[k];
    }
    uint64_t total;
    uint64_t pre = block_exclusive_sum_u64(run, &total);
#pragma unroll
    for (uint32_t k = 0; k < kScanOnePer; ++k) {
        const uint32_t g = threadIdx.x * kScanOnePer + k;
        if (g < n_blocks) b.blk[g] = pre;
        pre += v[k];
    }
    for (uint32_t g = threadIdx.x; g < b.n_groups; g += kBlock) b.grp[g] = 0;
    if (threadIdx.x == 0) b.grp[b.n_groups] = total;
}

__global__ __launch_bounds__(kBlock) void kb_scan_groups(BuildArgs b, uint32_t n_blocks) {
    StampScope stamp_(b.stamp, b.epoch, UVHTTP_WS_STAMP_BUILD_SCAN);
    const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
    const uint64_t v = k < n_blocks ? b.blk[k] : 0;
    uint64_t total;
    const uint64_t pre = block_exclusive_sum_u64(v, &total);
    if (k < n_blocks) b.blk[k] = pre;
    if (threadIdx.x == 0) b.grp[blockIdx.x] = total;
}

__global__ __launch_bounds__(kBlock) void kb_scan_top(BuildArgs b, uint32_t n_groups) {
    StampScope stamp_(b.stamp, b.epoch, UVHTTP_WS_STAMP_BUILD_SCAN2);
    constexpr int kPer = 4;
    uint64_t v[kPer], run = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t g = threadIdx.x * kPer + k;
        v[k] = g < n_groups ? b.grp[g] : 0;
        run += v[k];
    }
    uint64_t total;
    uint64_t pre = block_exclusive_sum_u64(run, &total);
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t g = threadIdx.x * kPer + k;
        if (g < n_groups) b.grp[g] = pre;
        pre += v[k];
    }
    if (threadIdx.x == 0) b.grp[n_groups] = total;
}

// header image of a built frame (<= 14 bytes: byte 0, byte 1, extended length, key)
__device__ inline u32x4 build_header(const uvhttp_ws_build_desc_t& d, uint32_t* hsz) {
    const uint64_t p = d.payload_len;
    const uint32_t hs = p < 126 ? 2 : p < 65536 ? 4 : 10;
    uint32_t w[4] = {0, 0, 0, 0};
    auto put = [&](uint32_t k, uint32_t byte) { w[k >> 2] |= (byte & 0xFF) << (8 * (k & 3)); };
    put(0, (d.fin ? 0x80 : 0) | (d.opcode & 0x0F));
    const uint32_t mb = d.mask ? 0x80 : 0;
    if (hs == 2) {
        put(1, mb | (uint32_t)p);
    } else if (hs == 4) {
        put(1, mb | 126);
        put(2, (uint32_t)(p >> 8));
        put(3, (uint32_t)p);
    } else {
        put(1, mb | 127);
#pragma unroll
        for (int k = 0; k < 8; ++k) put(2 + k, (uint32_t)(p >> (56 - 8 * k)));
    }
    if (d.mask) {
#pragma unroll
        for (int k = 0; k < 4; ++k) put(hs + k, d.masking_key >> (8 * k));
    }
    *hsz = hs + (d.mask ? 4u : 0u);
    return u32x4{w[0], w[1], w[2], w[3]};
}

__global__ __launch_bounds__(kBlock) void kb_offsets(BuildArgs b, uint32_t n_groups) {
    resolve_epoch(b);
    StampScope stamp_(b.stamp, b.epoch, UVHTTP_WS_STAMP_BUILD_OFFSETS);
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint64_t sz = i < b.n ? build_size(b.frames[i]) : 0;
    uint64_t total;
    const uint64_t local = block_exclusive_sum_u64(sz, &total);
    if (i >= b.n) return;
    const uint64_t off = b.grp[blockIdx.x / kBlock] + b.blk[blockIdx.x] + local;
    b.out_off[i] = off;
    if (i + 1 == b.n) b.out_off[b.n] = b.grp[n_groups];
    if (b.grp[n_groups] > b.out_cap) return;  // nothing will be written (no record is tagged)
    const uvhttp_ws_build_desc_t d = b.frames[i];
    BuildRec r;
    uint32_t hm;
    r.img = build_header(d, &hm);
    r.st = off;
    r.ps = off + hm;
    r.fe = r.ps + d.payload_len;
    r.src = d.payload_off;
    r.key = d.mask ? d.masking_key : 0u;
    r.frame = i;
    r.tag = b.epoch;
    r.pad = 0;
    const uint64_t g = 1ull << b.map_shift;
    for (uint64_t t = (off + g - 1) >> b.map_shift; (t << b.map_shift) < off + sz && t < b.n_map; ++t)
        b.mrec[t] = r;
}

// bytes of output vector [oa, oa + 16) that belong to frame (header image img over
// [fs, ps), payload src[sp ...] over [ps, fe), key for client frames)
__device__ inline void build_vector(const BuildArgs& b, uint64_t oa, uint64_t fs, uint64_t ps,
                                    uint64_t fe, uint64_t sp, uint32_t key, const u32x4& img,
                                    u32x4& out) {
    if (ps > oa && fs < oa + 16) {
        // the header image moved to the vector's byte phase: output byte q = image byte
        // q - (fs - oa), one 128-bit shift instead of a byte loop
        const int64_t d = (int64_t)fs - (int64_t)oa;  // -13 .. 15
        unsigned __int128 v = ((unsigned __int128)(((uint64_t)img.w << 32) | img.z) << 64) |
                              (((uint64_t)img.y << 32) | img.x);
        v = d >= 0 ? v << (8 * d) : v >> (-8 * d);
        const int lo_b = d > 0 ? (int)d : 0;
        const int hi_b = ps < oa + 16 ? (int)(ps - oa) : 16;
        const u32x4 sel{lane_bytes(lo_b, hi_b, 0), lane_bytes(lo_b, hi_b, 1),
                        lane_bytes(lo_b, hi_b, 2), lane_bytes(lo_b, hi_b, 3)};
        const uint64_t lo = (uint64_t)v, hi = (uint64_t)(v >> 64);
        out |= u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)} & sel;
    }
    if (fe > ps && ps < oa + 16 && fe > oa) {
        const int lo_b = ps > oa ? (int)(ps - oa) : 0;
        const int hi_b = fe < oa + 16 ? (int)(fe - oa) : 16;
        const int64_t wstart = (int64_t)sp + ((int64_t)oa - (int64_t)ps);
        const u32x4 w = load16_any(b.src, wstart, b.src_len);
        const uint32_t rk = rotr32(key, 8u * (uint32_t)((oa - ps) & 3u));
        const u32x4 sel{lane_bytes(lo_b, hi_b, 0), lane_bytes(lo_b, hi_b, 1),
                        lane_bytes(lo_b, hi_b, 2), lane_bytes(lo_b, hi_b, 3)};
        out |= (w ^ u32x4{rk, rk, rk, rk}) & sel;
    }
}

template <int BLOCK, int VPT>
__global__ __launch_bounds__(BLOCK) void kb_emit(BuildArgs b, uint64_t tile_base) {
    resolve_epoch(b);
    StampScope stamp_(b.stamp, b.epoch, UVHTTP_WS_STAMP_PAYLOAD, false, tile_base);
    constexpr uint64_t kT = (uint64_t)BLOCK * VPT * 16;
    __shared__ uint64_t s_start[BLOCK];  // frame start in out
    __shared__ uint64_t s_pstart[BLOCK]; // payload start in out
    __shared__ uint64_t s_end[BLOCK];
    __shared__ uint64_t s_src[BLOCK];
    __shared__ uint32_t s_key[BLOCK];    // 0 for server frames (XOR no-op)
    __shared__ u32x4 s_hdr[BLOCK];       // header image (<= 14 bytes)

    const uint64_t t0 = (tile_base + stamp_.anchor_s(blockIdx.x)) * kT;
    // map tiles are a power of two >= kT (host), so the tile lies inside map tile c0
    const uint64_t c0 = t0 >> b.map_shift, c1 = c0 + 1;
    if (c0 >= b.n_map) return;
    // both records in one round trip (the map has a spare entry past n_map, never tagged);
    // the empty asm makes the compiler issue every field's load before the tag test
    const BuildRec r0 = b.mrec[c0];
    const BuildRec r1 = b.mrec[c0 + 1];
    asm volatile("" ::"s"(r0.st), "s"(r0.ps), "s"(r0.fe), "s"(r0.src), "s"(r0.key),
                 "s"(r1.st), "s"(r1.ps), "s"(r1.fe), "s"(r1.src), "s"(r1.key), "s"(r1.frame),
                 "s"(r1.tag));
    if (r0.tag != b.epoch) return;  // tile past the end of the output (or over capacity)
    const bool v1 = c1 < b.n_map && r1.tag == b.epoch;

    uint64_t oa[VPT];
    u32x4 out[VPT];
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        oa[v] = t0 + ((uint64_t)v * BLOCK + threadIdx.x) * 16u;
        out[v] = u32x4{0, 0, 0, 0};
    }
    if (v1 && r1.frame - r0.frame < 2) {
        // fast path (frames of ~4 KiB and up): the frame covering the tile start and the one
        // covering the next map tile's start cover every byte of the tile, and both records
        // arrived with the lookup — every vector is whole, no bound check
#pragma unroll
        for (int v = 0; v < VPT; ++v)
            if (r0.fe > oa[v])
                build_vector(b, oa[v], r0.st, r0.ps, r0.fe, r0.src, r0.key, r0.img, out[v]);
        if (r1.frame != r0.frame) {
#pragma unroll
            for (int v = 0; v < VPT; ++v)
                if (r1.st < oa[v] + 16)
                    build_vector(b, oa[v], r1.st, r1.ps, r1.fe, r1.src, r1.key, r1.img, out[v]);
        }
#pragma unroll
        for (int v = 0; v < VPT; ++v)
            __builtin_nontemporal_store(out[v], reinterpret_cast<u32x4*>(b.out + oa[v]));
        return;
    }
    const uint64_t total = b.out_off[b.n];
    const uint32_t last = b.n - 1;
    const uint32_t f0 = r0.frame;
    uint32_t f1 = v1 ? r1.frame : last;
    if (f1 > last || f1 < f0) f1 = last;
    for (uint32_t base = f0; base <= f1; base += BLOCK) {
        const uint32_t cnt = (f1 - base + 1) < (uint32_t)BLOCK ? (f1 - base + 1) : BLOCK;
        __syncthreads();
        if (threadIdx.x < cnt) {
            const uint32_t f = base + threadIdx.x;
            const uvhttp_ws_build_desc_t d = b.frames[f];
            uint32_t hm;
            const u32x4 img = build_header(d, &hm);
            const uint64_t st = b.out_off[f];
            s_start[threadIdx.x] = st;
            s_pstart[threadIdx.x] = st + hm;
            s_end[threadIdx.x] = st + hm + d.payload_len;
            s_src[threadIdx.x] = d.payload_off;
            s_key[threadIdx.x] = d.mask ? d.masking_key : 0u;
            s_hdr[threadIdx.x] = img;
        }
        __syncthreads();
        if (s_start[0] >= t0 + kT) break;
#pragma unroll
        for (int v = 0; v < VPT; ++v) {
            int lo = 0, hi = (int)cnt - 1, j = -1;
            while (lo <= hi) {
                const int mid = (lo + hi) >> 1;
                if (s_start[mid] < oa[v] + 16) {
                    j = mid;
                    lo = mid + 1;
                } else {
                    hi = mid - 1;
                }
            }
            for (; j >= 0; --j) {
                if (s_end[j] <= oa[v]) break;
                build_vector(b, oa[v], s_start[j], s_pstart[j], s_end[j], s_src[j], s_key[j],
                             s_hdr[j], out[v]);
            }
        }
    }
#pragma unroll
    for (int v = 0; v < VPT; ++v) {
        if (oa[v] >= total) continue;
        if (oa[v] + 16 <= total) {
            __builtin_nontemporal_store(out[v], reinterpret_cast<u32x4*>(b.out + oa[v]));
        } else {
            const uint32_t ow[4] = {out[v].x, out[v].y, out[v].z, out[v].w};
            for (uint64_t bq = 0; oa[v] + bq < total; ++bq)
                b.out[oa[v] + bq] = (uint8_t)(ow[bq >> 2] >> (8 * (bq & 3)));
        }
    }
}

// Small-frame emit: one workgroup per kEmitF consecutive frames.  Their output [A, B) is
// contiguous; it is assembled in an LDS window (zeroed; header bytes and the edge vectors of
// each payload OR-ed in, interior payload vectors written whole) and then stored as aligned
// 16-byte vectors, so every global store is a full coalesced vector except the two partial
// vectors at the range's ends (their other bytes belong to the neighbouring workgroups).
// Work items are (frame, aligned output vector of its payload) pairs, flattened by a prefix
// over the workgroup's frames; a window takes the contiguous item range whose vectors fall
// inside it.  Per frame: one descriptor load and one offset load; per payload vector: one
// unaligned 16-byte source load — no per-tile map records and no per-vector frame search
// over the whole tile.
constexpr uint32_t kEmitF = 256;         // frames per workgroup at most (one per thread; FMAX)
#ifndef UVWS_EMIT_WIN
#define UVWS_EMIT_WIN 20480
#endif
constexpr uint32_t kEmitWin = UVWS_EMIT_WIN;  // LDS window bytes (64 frames of <= 300 bytes: one window)
constexpr uint32_t kEmitItems = 1280;    // item -> frame table entries (one-window workgroups; 5 per thread)

template <int BLOCK, int FMAX>
__global__ __launch_bounds__(BLOCK)
#ifdef UVWS_EMIT_WPE
__attribute__((amdgpu_waves_per_eu(UVWS_EMIT_WPE)))
#endif
void kb_emit_frames(BuildArgs b) {
    __shared__ u32x4 s_win[kEmitWin / 16];
    __shared__ uint64_t s_ps[FMAX], s_fe[FMAX], s_sp[FMAX], s_st[FMAX];
    __shared__ uint32_t s_key[FMAX];
    __shared__ u32x4 s_img[FMAX];
    __shared__ uint32_t s_cp[FMAX + 1];  // items of frames [0, j)
    __shared__ uint32_t s_q[2];
    __shared__ __attribute__((aligned(4))) uint8_t s_fof[kEmitItems];  // frame of item q (a workgroup with one window)
    __shared__ uint32_t s_wsum[BLOCK / 64];

    StampScope stamp_(b.stamp, b.epoch, UVHTTP_WS_STAMP_PAYLOAD, false);
    // the offsets: kb_size left each frame's within its 256-frame block, the scans the blocks'
    // (grp + blk); this kernel writes the final ones (the API's out_off) — also when the output
    // does not fit, where nothing else is written (as kb_emit)
    const uint64_t total = b.grp[b.n_groups];
    const uint32_t f0 = stamp_.anchor_s(blockIdx.x) * b.group;
    if (f0 >= b.n) return;
    const uint32_t nf = b.n - f0 < b.group ? b.n - f0 : b.group;
    if (total > b.out_cap) {
        if (threadIdx.x < nf) {
            const uint32_t f = f0 + threadIdx.x;
            b.out_off[f] += b.grp[f / (kBlock * kBlock)] + b.blk[f / kBlock];
            if (f + 1 == b.n) b.out_off[b.n] = total;
        }
        return;
    }
    static_assert(BLOCK >= FMAX && FMAX <= 256, "one thread per frame; frame ids fit a byte");
    {
        const uint32_t j = threadIdx.x, lane = j & 63, wave = j >> 6;
        uint32_t nv = 0;
        if (j < nf) {
            const uint32_t f = f0 + j;
            const uvhttp_ws_build_desc_t d = b.frames[f];
            const uint64_t st = b.out_off[f] + b.grp[f / (kBlock * kBlock)] + b.blk[f / kBlock];
            b.out_off[f] = st;
            if (f + 1 == b.n) b.out_off[b.n] = total;
            uint32_t hm;
            s_img[j] = build_header(d, &hm);
            s_st[j] = st;
            s_ps[j] = st + hm;
            s_fe[j] = st + hm + d.payload_len;
            s_sp[j] = d.payload_off;
            s_key[j] = d.mask ? d.masking_key : 0u;
            if (d.payload_len) nv = (uint32_t)(((st + hm + d.payload_len - 1) >> 4) - ((st + hm) >> 4) + 1);
        }
        uint32_t inc = nv;  // block-inclusive scan of the item counts
#pragma unroll
        for (int dd = 1; dd < 64; dd <<= 1) {
            const uint32_t o = __shfl_up(inc, dd, 64);
            if ((int)lane >= dd) inc += o;
        }
        if (lane == 63) s_wsum[wave] = inc;
        __syncthreads();
        for (uint32_t w = 0; w < wave; ++w) inc += s_wsum[w];
        if (j < FMAX) s_cp[j + 1] = inc;
        if (j == 0) s_cp[0] = 0;
    }
    __syncthreads();
    const uint64_t A = s_st[0], B = s_fe[nf - 1];
    const uint32_t nitems = s_cp[nf];
    // the common case: the whole range in one window and an item table that fits — each
    // frame's lane fills its items' entries, so an item finds its frame in one LDS read
    const bool one = B - (A & ~15ull) <= kEmitWin && nitems <= kEmitItems;
    if (one && threadIdx.x < nf) {
        // (the frame's item range: bytes up to a word boundary, whole words, then bytes — a
        // 256-byte frame's 17 entries in about 7 LDS stores instead of 17)
        const uint32_t c0 = s_cp[threadIdx.x], c1 = s_cp[threadIdx.x + 1];
        const uint32_t jb = threadIdx.x & 0xFFu, jw = jb * 0x01010101u;
        uint32_t q = c0;
        for (; q < c1 && (q & 3u); ++q) s_fof[q] = (uint8_t)jb;
        for (; q + 4 <= c1; q += 4) *reinterpret_cast<uint32_t*>(&s_fof[q]) = jw;
        for (; q < c1; ++q) s_fof[q] = (uint8_t)jb;
    }
    // frame of item q: the last j with s_cp[j] <= q
    auto frame_of = [&](uint32_t q) {
        uint32_t lo = 0, hi = nf - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (s_cp[mid] <= q) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    };
    auto item_oa = [&](uint32_t q, uint32_t j) { return ((s_ps[j] >> 4) + (q - s_cp[j])) << 4; };
    uint32_t* win32 = reinterpret_cast<uint32_t*>(s_win);
    for (uint64_t wlo = A & ~15ull; wlo < B; wlo += kEmitWin) {
        const uint64_t whi = wlo + kEmitWin;
// (zeroing only the vectors that are OR-ed into — a frame's header and payload-edge vectors —
        // measured even with zeroing the whole window: C4 build 97.8 vs 98.4 us, masked 103.0 vs
        // 102.9, profiles/r06q_emit_zero_edges_ab_*.txt)
        for (uint32_t v = threadIdx.x; v < kEmitWin / 16; v += BLOCK) s_win[v] = u32x4{0, 0, 0, 0};
        if (one) {
            if (threadIdx.x == 0) s_q[0] = 0, s_q[1] = nitems;
        } else if (threadIdx.x == 0) {  // items whose vectors lie in the window: [first oa >= wlo, first oa >= whi)
            uint32_t q0 = 0, q1 = nitems;
            for (int k = 0; k < 2; ++k) {
                const uint64_t bound = k ? whi : wlo;
                uint32_t lo = 0, hi = nitems;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (item_oa(mid, frame_of(mid)) < bound) lo = mid + 1;
                    else hi = mid;
                }
                (k ? q1 : q0) = lo;
            }
            s_q[0] = q0;
            s_q[1] = q1;
        }
        __syncthreads();
        // a payload item's source window and its LDS update (interior vectors whole, edges OR-ed)
        auto item_src = [&](uint32_t q, uint32_t j, uint64_t* oa) {
            *oa = item_oa(q, j);
            return (int64_t)s_sp[j] + ((int64_t)*oa - (int64_t)s_ps[j]);
        };
        auto put_item = [&](uint32_t j, uint64_t oa, u32x4 w) {
            const uint64_t ps = s_ps[j], fe = s_fe[j];
            const int lo_b = ps > oa ? (int)(ps - oa) : 0;
            const int hi_b = fe < oa + 16 ? (int)(fe - oa) : 16;
            const uint32_t rk = rotr32(s_key[j], 8u * (uint32_t)((oa - ps) & 3u));
            w = w ^ u32x4{rk, rk, rk, rk};
            const uint32_t wv = (uint32_t)((oa - wlo) >> 4);
            if (lo_b == 0 && hi_b == 16) {
                s_win[wv] = w;
            } else {
                const u32x4 sel{lane_bytes(lo_b, hi_b, 0), lane_bytes(lo_b, hi_b, 1),
                                lane_bytes(lo_b, hi_b, 2), lane_bytes(lo_b, hi_b, 3)};
                const u32x4 m = w & sel;
                if (m.x) atomicOr(&win32[4 * wv + 0], m.x);
                if (m.y) atomicOr(&win32[4 * wv + 1], m.y);
                if (m.z) atomicOr(&win32[4 * wv + 2], m.z);
                if (m.w) atomicOr(&win32[4 * wv + 3], m.w);
            }
        };
        auto put_headers = [&]() {  // header bytes (one lane per frame), a word per LDS atomic
            if (threadIdx.x >= nf) return;
            const uint32_t j = threadIdx.x;
            const uint64_t st = s_st[j], ps = s_ps[j];
            const u32x4 img = s_img[j];
            const uint32_t iw[4] = {img.x, img.y, img.z, img.w};
            const uint64_t a0 = st > wlo ? st : wlo, a1 = ps < whi ? ps : whi;
            // (an 8-byte masked header: 2-3 word atomics instead of 8 byte atomics; the window
            // is 16-byte aligned, so output words are window words)
            for (uint64_t d = a0 & ~3ull; d < a1; d += 4) {
                uint32_t val = 0;
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint64_t k = d + q;
                    if (k >= a0 && k < a1) {
                        const uint32_t ib = (uint32_t)(k - st);
                        val |= ((iw[ib >> 2] >> (8 * (ib & 3))) & 0xFFu) << (8 * q);
                    }
                }
                atomicOr(&win32[(d - wlo) >> 2], val);
            }
        };
        if (one && b.src_len >= 16) {
            // every item's 16-byte source load issued before any LDS work (an out-of-range
            // window loads from offset 0 and is redone bytewise below)
            // (only the loaded vectors stay in registers across the loads' flight; the item's
            // addresses are recomputed from LDS afterwards: 96 -> fewer VGPRs)
            constexpr int kIpt = kEmitItems / BLOCK;
            u32x4 w[kIpt];
#pragma unroll
            for (int k = 0; k < kIpt; ++k) {
                const uint32_t q = threadIdx.x + k * BLOCK;
                const uint32_t j = q < nitems ? s_fof[q] : 0;
                uint64_t oa;
                const int64_t ws = item_src(q < nitems ? q : s_cp[0], j, &oa);
                const bool ok = ws >= 0 && (uint64_t)ws + 16 <= b.src_len;
                __builtin_memcpy(&w[k], b.src + (ok ? ws : 0), 16);
            }
            __builtin_amdgcn_sched_barrier(0);
            put_headers();
#pragma unroll
            for (int k = 0; k < kIpt; ++k) {
                const uint32_t q = threadIdx.x + k * BLOCK;
                if (q >= nitems) continue;
                const uint32_t j = s_fof[q];
                uint64_t oa;
                const int64_t ws = item_src(q, j, &oa);
                if (!(ws >= 0 && (uint64_t)ws + 16 <= b.src_len)) w[k] = load16_any(b.src, ws, b.src_len);
                put_item(j, oa, w[k]);
            }
        } else {
            put_headers();
            const uint32_t q0 = s_q[0], q1 = s_q[1];
            for (uint32_t q = q0 + threadIdx.x; q < q1; q += BLOCK) {
                const uint32_t j = one ? s_fof[q] : frame_of(q);
                uint64_t oa;
                const int64_t wsrc = item_src(q, j, &oa);
                put_item(j, oa, load16_any(b.src, wsrc, b.src_len));
            }
        }
        __syncthreads();
        // store the window's part of [A, B)
        const uint64_t lo = A > wlo ? A : wlo, hi = B < whi ? B : whi;
        for (uint64_t oa = (lo & ~15ull) + 16ull * threadIdx.x; oa < hi; oa += 16ull * BLOCK) {
            const u32x4 v = s_win[(oa - wlo) >> 4];
            if (oa >= lo && oa + 16 <= hi) {
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(b.out + oa));
            } else {
                const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
                for (uint32_t k = 0; k < 16; ++k)
                    if (oa + k >= lo && oa + k < hi) b.out[oa + k] = (uint8_t)(vw[k >> 2] >> (8 * (k & 3)));
            }
        }
        __syncthreads();
    }
}

// plain unmask of one buffer with one key (uvhttp_ws_apply_mask over device memory).  The
// payload kernel's streaming shape: a 64-lane workgroup per 1 KiB tile of 16-byte vectors,
// one non-temporal load per lane, one sc1|nt buffer store (DESIGN.md §4 "Why 1 KiB
// workgroups"); bench.py also times it over the whole wire as the same-run copy ceiling.
constexpr int kMaskBlock = 64;
__global__ __launch_bounds__(kMaskBlock) void k_apply_mask(uint8_t* data, uint64_t len, uint32_t key,
                                                           uint64_t head, uint64_t tile_base) {
    // bytes [0, head) are the unaligned head; vectors start at data + head
    const uint64_t tile = tile_base + blockIdx.x;
    const uint64_t body = len > head ? len - head : 0;
    const uint64_t nvec = body / 16;
    const uint64_t v = tile * kMaskBlock + threadIdx.x;
    if (v < nvec) {
        const uint32_t rk = rotr32(key, 8u * (uint32_t)(head & 3u));
        uint8_t* base = data + head + tile * kMaskBlock * 16;
        const uint64_t room = (nvec - tile * kMaskBlock) * 16;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            base, 0, (int)(room < kMaskBlock * 16 ? room : kMaskBlock * 16), 0x00020000);
        const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base) + threadIdx.x) ^
                        u32x4{rk, rk, rk, rk};
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, x), rs,
            threadIdx.x * 16u, 0, 18);
    }
    if (tile == 0 && threadIdx.x < head && threadIdx.x < len)
        data[threadIdx.x] ^= (uint8_t)(key >> (8 * (threadIdx.x & 3)));
    const uint64_t tail0 = head + nvec * 16;
    if (tile == 0 && tail0 < len && threadIdx.x < len - tail0) {
        const uint64_t b = tail0 + threadIdx.x;
        data[b] ^= (uint8_t)(key >> (8 * (b & 3)));
    }
}

// ------------------------------------------------------------------------------------
// synthetic frames (definition shared with oracle_gen_frames)
// ------------------------------------------------------------------------------------
__device__ __host__ inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __host__ inline uint64_t gen_header_size(uint64_t p) {
    return p < 126 ? 2 : p < 65536 ? 4 : 10;
}

__global__ __launch_bounds__(kBlock) void k_gen_frames(uint8_t* wire, uint32_t first, uint32_t n,
                                                       uint32_t n_total, uint64_t plen,
                                                       uint64_t seed, int opcode0, int fragmented,
                                                       int force_keys, uint64_t words_per_frame) {
    const uint64_t gid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    const uint64_t total = (uint64_t)n * words_per_frame;
    const uint64_t hs = gen_header_size(plen);
    const uint64_t stride = hs + 4 + plen;
    for (uint64_t g = gid; g < total; g += (uint64_t)gridDim.x * kBlock) {
        const uint32_t li = (uint32_t)(g / words_per_frame);  // frame in this range
        const uint32_t i = first + li;                        // frame in the whole batch
        const uint64_t wi = g - (uint64_t)li * words_per_frame;
        uint8_t* w = wire + (uint64_t)li * stride;
        uint32_t key = (uint32_t)splitmix64(seed ^ (uint64_t)i);
        if (force_keys && i == 0) key = 0u;
        if (force_keys && i == 1) key = 0xFFFFFFFFu;
        if (wi == 0) {
            const int fin = !fragmented || i + 1 == n_total;
            const int op = (i == 0 || !fragmented) ? opcode0 : 0;
            w[0] = (uint8_t)((fin ? 0x80 : 0) | (op & 0x0F));
            if (hs == 2) {
                w[1] = (uint8_t)(0x80 | plen);
            } else if (hs == 4) {
                w[1] = 0x80 | 126;
                w[2] = (uint8_t)(plen >> 8);
                w[3] = (uint8_t)plen;
            } else {
                w[1] = 0x80 | 127;
                for (int k = 0; k < 8; ++k) w[2 + k] = (uint8_t)(plen >> (56 - 8 * k));
            }
            for (int k = 0; k < 4; ++k) w[hs + k] = (uint8_t)(key >> (8 * k));
        }
        const uint64_t b = wi * 8;
        if (b < plen) {
            const uint64_t r = splitmix64(seed + ((uint64_t)i << 32) + wi);
            uint8_t* pl = w + hs + 4;
            for (int k = 0; k < 8 && b + k < plen; ++k)
                pl[b + k] = (uint8_t)(r >> (8 * k)) ^ (uint8_t)(key >> (8 * ((b + k) & 3)));
        }
    }
}

// k_epoch: first kernel of a captured call.  Every block reads the current device epoch,
// then the last block to finish stores the next one (all reads happen before the store,
// which waits for every block's done-increment).  When the device half of the epoch space is
// used up the workspace and the send-side map are cleared first (grid-stride), so no stale
// tag can match after the wrap.
__global__ __launch_bounds__(kBlock) void k_epoch(uint32_t* ctl, uint64_t* ws_words,
                                                  uint64_t n_ws, uint64_t* bs_words,
                                                  uint64_t n_bs) {
    const uint32_t e = *reinterpret_cast<volatile uint32_t*>(ctl + kCtlEpoch);
    const bool wrap = e >= kMaxEpoch || e <= kMaxHostEpoch;  // also the first captured call
    if (wrap) {
        const uint64_t stride = (uint64_t)gridDim.x * kBlock;
        for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < n_ws; k += stride)
            ws_words[k] = 0;
        for (uint64_t k = (uint64_t)blockIdx.x * kBlock + threadIdx.x; k < n_bs; k += stride)
            bs_words[k] = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        const uint32_t t =
            __hip_atomic_fetch_add(&ctl[kCtlDone], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (t + 1 == gridDim.x) {
            __hip_atomic_store(&ctl[kCtlDone], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ctl[kCtlEpoch], wrap ? kMaxHostEpoch + 1 : e + 1, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace

// ======================================================================================
// engine + C ABI
// ======================================================================================
struct uvhttp_ws_gpu_engine {
    int device;
    void* ws_mem;
    size_t ws_bytes;
    uint32_t cap_frames;
    uint64_t cap_tiles, cap_arena_tiles;
    Workspace ws;
    int timing;                // 0: off; k >= 1: HIP events around every k-th call's payload kernel
    uint64_t timing_calls;     // calls seen while timing (the sampling counter)
    int tile_block, tile_vpt;  // payload kernel shape, 0 = automatic
    int store_aux;             // payload store cache policy (0 = nt global store, 18 = sc1|nt)
    uint32_t epoch;            // tag of the latest decode call, 1 .. kMaxEpoch
    int plan_fpt;              // k_plan frames per lane, 0 = automatic
    int fused_off;             // UVHTTP_WS_FUSED=0: stride batches take the k_plan-first path
    uint64_t fused_max_avg;    // fused only up to this many wire bytes per frame (UVHTTP_WS_FUSED_MAX)
    int rec_lookback;          // fused path: records scanned by k_plan (1) or reduce-then-scan (0)
    int plan_wide;             // records: k_plan with 1024-thread blocks (UVHTTP_WS_PLAN_WIDE=1; A/B)
    uint32_t plan_no_ticket;   // UVHTTP_WS_PLAN_TICKET=0: blockIdx order instead of tickets
    int walk_mode;             // stream frame discovery: 0 automatic, 1 lane, 2 wave
    void* ss_mem;              // stream-decode scratch
    uint32_t ss_frames, ss_reads;
    StreamScratch ss;
    void* wt_mem;              // single-pass walk scratch (frame starts per connection slice)
    uint64_t wt_cap;
    void* wr_mem;              // the wave walk's frame records (parallel to wt_mem)
    uint64_t wr_cap;
    int wr_rec_on;             // UVHTTP_WS_WALK_REC=0: k_stream_desc gathers every header (A/B)
    int walk_single_off;       // UVHTTP_WS_WALK_SINGLE=0: always walk twice (tests, A/B)
    int walk_fuse;             // UVHTTP_WS_WALK_FUSE=1: k_swalk_fused for the single-pass wave walk
    int stream_nt;             // UVHTTP_WS_STREAM_NT=1: streaming stores in the walk and k_stream_desc (A/B)
    int desc_scan_off;         // UVHTTP_WS_DESC_SCAN=0: k_swalk_scan before k_stream_desc always (A/B)
    int walk_nt_load;          // UVHTTP_WS_WALK_NT_LOAD=1: non-temporal header loads in the wave walk (A/B)
    int stream_spec;           // stream calls try the speculative decode first (k_sspec_*;
                               // UVHTTP_WS_STREAM_SPEC=0: the walk always)
    void* sp_mem;              // its scratch: SpecConn per connection, block counts, tile claims
    uint32_t sp_streams;
    uint64_t sp_tiles;
    int fused_block, fused_vpt;  // UVHTTP_WS_FUSED_TILE=BxV: the fused payload pass's tile (A/B)
    uint32_t fixup_blocks;     // k_fixup grid cap (UVHTTP_WS_FIXUP_BLOCKS, A/B)
    int fused_aux;             // fused payload stores' cache-policy bits (UVHTTP_WS_FUSED_AUX, A/B)
    int compact_recs;          // compact stride batches: records pass + k_plan on records
    int spec_on;               // compact stride batches: the speculative pass (UVHTTP_WS_SPEC=0: off)
    uint64_t spec_max_avg;     // ... up to this many wire bytes per frame (UVHTTP_WS_SPEC_MAX)
    int time_chain;            // UVHTTP_WS_TIME_CHAIN=1: stream decode timing brackets the whole
                               // kernel chain (walk .. payload), not only the payload kernel
    void* bs_mem;              // send-side output-map records (BuildRec per map tile)
    uint64_t bs_tiles;
    int build_small;           // emit shape for frames < 4 KiB (UVHTTP_WS_BUILD_SMALL, tuning)
    uint64_t build_frames_max; // frame-grouped LDS emit below this average frame (UVHTTP_WS_BUILD_FRAMES; 0 = off)
    int compact_mode;          // 0 automatic, 1 arena-driven gather, 2 wire-driven scatter
    int sum_fast;              // summary-only stride decode in one payload pass (UVHTTP_WS_SUMMARY_FAST=0: off)
    uvhttp_ws_frame_desc_t* dscr;  // descriptor scratch for d_desc == NULL calls
    uint64_t dscr_cap;
    uint32_t* ctl;             // device control words (kCtl*), own allocation
    uint32_t faults_seen;      // ctl[kCtlFaults] at the last engine_sync
    uint32_t max_polls;        // look-back wait bound (UVHTTP_WS_MAX_POLLS: tests)
    uint64_t* stamp_mem;       // device-side kernel stamps (kStampWords), null until enabled
    int stamp_on;
    int capturing;             // the current call is being captured into a graph
    int captured_ever;         // a call of this engine was captured (its replays leave later epochs)
    hipStream_t last_stream;   // stream of the previous call (calls are serialised on it)
    int have_last;
    int pool_ok;               // the device has the stream-ordered allocator (scratch_grow)
    int desc_emit;             // stride batches with descriptors: k_desc_emit (not k_plan on records)
    hipEvent_t order_ev;       // orders a call on a new stream after the previous stream's work
    hipEvent_t ev[2 * 1024];
    int ev_created;
    int ev_used;       // event pairs recorded and not yet harvested
    double time_ms;
    uint64_t launches;
    char err[256];
};

static void scratch_free(uvhttp_ws_gpu_engine_t* e, void* p);
static int set_err(uvhttp_ws_gpu_engine_t* e, int code, const char* what, hipError_t h) {
    if (e) snprintf(e->err, sizeof(e->err), "%s: %s", what, h == hipSuccess ? "" : hipGetErrorString(h));
    return code;
}

template <int BLOCK, int VPT>
static void launch_emit(const BuildArgs& b, uint32_t n_frames, uint64_t out_cap, hipStream_t s) {
    const uint64_t tile_bytes = (uint64_t)BLOCK * VPT * 16;
    const uint64_t n_ptiles = (out_cap + tile_bytes - 1) / tile_bytes;
    const uint64_t max_tiles = (1ull << 24);
    for (uint64_t tb = 0; n_frames && tb < n_ptiles; tb += max_tiles) {
        const uint32_t grid_p = (uint32_t)((n_ptiles - tb) < max_tiles ? (n_ptiles - tb) : max_tiles);
        hipLaunchKernelGGL((kb_emit<BLOCK, VPT>), dim3(grid_p), dim3(BLOCK), 0, s, b, tb);
    }
}

extern "C" {

const char* uvhttp_ws_amd_version(void) { return "uvhttp_ws_amd 0.1.0 gfx950"; }

uint64_t uvhttp_ws_gen_frame_stride(uint64_t payload_len) {
    return gen_header_size(payload_len) + 4 + payload_len;
}

#ifdef UVWS_EXPERIMENTS
// Experiment / test builds only (libuvhttp_ws_amd_testhooks.so, -DUVWS_EXPERIMENTS): the A/B
// switches the measurements in DESIGN.md and profiles/ were taken with, and the test hooks
// (look-back give-up, epoch wrap).  The product library reads no environment: two of these
// (UVHTTP_WS_PLAN_TICKET=0, UVHTTP_WS_WALK_FUSE=1) order workgroups by blockIdx and rely on
// in-order dispatch, which the product must not.  Every
// variant reachable here gives the product's results (tests/ run them against the oracle).
static void experiment_knobs(uvhttp_ws_gpu_engine_t* e) {
    if (const char* mp = getenv("UVHTTP_WS_MAX_POLLS")) e->max_polls = (uint32_t)strtoul(mp, nullptr, 0);
    if (const char* po = getenv("UVHTTP_WS_SCRATCH_POOL")) e->pool_ok &= atoi(po) != 0;
    if (const char* sp = getenv("UVHTTP_WS_STORE_POLICY")) e->store_aux = atoi(sp) == 18 ? 18 : 0;
    if (const char* fp = getenv("UVHTTP_WS_PLAN_FPT")) e->plan_fpt = atoi(fp);
    if (const char* pt = getenv("UVHTTP_WS_PLAN_TICKET")) e->plan_no_ticket = atoi(pt) == 0;
    // start near the end of the epoch space to exercise the wrap-around clear
    if (const char* ep = getenv("UVHTTP_WS_EPOCH_START")) {
        const unsigned long v = strtoul(ep, nullptr, 0);
        e->epoch = v < kMaxHostEpoch ? (uint32_t)v : 0;
    }
    if (const char* bs = getenv("UVHTTP_WS_BUILD_SMALL")) e->build_small = atoi(bs);
    if (const char* fu = getenv("UVHTTP_WS_FUSED")) e->fused_off = atoi(fu) == 0;
    if (const char* fm = getenv("UVHTTP_WS_FUSED_MAX")) e->fused_max_avg = strtoull(fm, nullptr, 10);
    if (const char* pw = getenv("UVHTTP_WS_PLAN_WIDE")) e->plan_wide = atoi(pw);
    if (const char* rs = getenv("UVHTTP_WS_REC_SCAN")) e->rec_lookback = strcmp(rs, "3pass") != 0;
    if (const char* bf = getenv("UVHTTP_WS_BUILD_FRAMES")) e->build_frames_max = strtoull(bf, nullptr, 10);
    if (const char* cm = getenv("UVHTTP_WS_COMPACT"))
        e->compact_mode = strcmp(cm, "gather") == 0 ? 1 : strcmp(cm, "scatter") == 0 ? 2 : 0;
    if (const char* ws = getenv("UVHTTP_WS_WALK_SINGLE")) e->walk_single_off = atoi(ws) == 0;
    if (const char* wf = getenv("UVHTTP_WS_WALK_FUSE")) e->walk_fuse = atoi(wf) != 0;
    if (const char* sn = getenv("UVHTTP_WS_STREAM_NT")) e->stream_nt = atoi(sn) != 0;
    if (const char* ds = getenv("UVHTTP_WS_DESC_SCAN")) e->desc_scan_off = atoi(ds) == 0;
    if (const char* wn = getenv("UVHTTP_WS_WALK_NT_LOAD")) e->walk_nt_load = atoi(wn) != 0;
    if (const char* sq = getenv("UVHTTP_WS_STREAM_SPEC")) e->stream_spec = atoi(sq) != 0;
    if (const char* wr = getenv("UVHTTP_WS_WALK_REC")) e->wr_rec_on = atoi(wr) != 0;
    if (const char* wm = getenv("UVHTTP_WS_WALK"))
        e->walk_mode = strcmp(wm, "lane") == 0 ? 1 : strcmp(wm, "wave") == 0 ? 2 : 0;
    if (const char* tc = getenv("UVHTTP_WS_TIME_CHAIN")) e->time_chain = atoi(tc) != 0;
    if (const char* cr = getenv("UVHTTP_WS_COMPACT_RECS")) e->compact_recs = atoi(cr) != 0;
    if (const char* sp2 = getenv("UVHTTP_WS_SPEC")) e->spec_on = atoi(sp2) != 0;
    if (const char* sm = getenv("UVHTTP_WS_SPEC_MAX")) e->spec_max_avg = strtoull(sm, nullptr, 10);
    if (const char* fa = getenv("UVHTTP_WS_FUSED_AUX")) e->fused_aux = atoi(fa);
    if (const char* sf = getenv("UVHTTP_WS_SUMMARY_FAST")) e->sum_fast = atoi(sf) != 0;
    if (const char* de = getenv("UVHTTP_WS_DESC_EMIT")) e->desc_emit = atoi(de);
    if (const char* tl = getenv("UVHTTP_WS_TILE")) {  // payload tile shape "BxV" (0x0 = auto)
        int tb = 0, tv = 0;
        if (sscanf(tl, "%dx%d", &tb, &tv) == 2) (void)uvhttp_ws_gpu_engine_set_tile(e, tb, tv);  // (validated)
    }
    if (const char* fx = getenv("UVHTTP_WS_FIXUP_BLOCKS")) e->fixup_blocks = (uint32_t)strtoul(fx, nullptr, 10);
    if (e->fixup_blocks == 0) e->fixup_blocks = 1;
    if (const char* ft = getenv("UVHTTP_WS_FUSED_TILE")) {
        int fb = 0, fv = 0;
        if (sscanf(ft, "%dx%d", &fb, &fv) == 2) {
            e->fused_block = fb;
            e->fused_vpt = fv;
        }
    }
}
#endif

int uvhttp_ws_gpu_engine_create(int device, uvhttp_ws_gpu_engine_t** out) {
    if (!out) return UVHTTP_WS_GPU_EINVAL;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || device < 0 || device >= count)
        return UVHTTP_WS_GPU_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return UVHTTP_WS_GPU_ENODEV;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return UVHTTP_WS_GPU_ENODEV;
    uvhttp_ws_gpu_engine_t* e = (uvhttp_ws_gpu_engine_t*)calloc(1, sizeof(*e));
    if (!e) return UVHTTP_WS_GPU_ENOMEM;
    e->device = device;
    // the product configuration (each choice measured: DESIGN.md §4-5)
    e->store_aux = 18;
    e->max_polls = kMaxPolls;
    e->fused_max_avg = kFusedMaxAvg;
    // the fused path scans its records with k_plan's look-back (C4: 133-136 us per step against
    // 144-145 for reduce-then-scan, profiles/r03p6_*)
    e->rec_lookback = 1;
    e->plan_wide = 0;  // 1024-thread blocks measured slower on C4 (1690 vs 1785 GiB/s, r03p7)
    e->build_frames_max = 4096;
    e->wr_rec_on = 1;
    e->compact_recs = 0;
    e->spec_on = 1;
    e->spec_max_avg = kFusedMaxAvg;
    e->fused_aux = 18;
    e->fixup_blocks = 1024;
    e->sum_fast = 1;
    // 3: in place the scan and k_desc_emit rebuild the info bytes from the records (C4 step 114.0
    // vs 115.9 us with them left by the payload pass, profiles/r06h_desc_emit_ab_*.txt); compact
    // the speculative pass leaves them (123.9 vs 126.9 us, profiles/r06j_desc_emit_compact_ab.txt)
    e->desc_emit = 3;
    e->stream_spec = 1;
    {
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(device);
        hipError_t h = hipMalloc(&e->ctl, kCtlWords * sizeof(uint32_t));
        if (h == hipSuccess) h = hipMemset(e->ctl, 0, kCtlWords * sizeof(uint32_t));
        if (h == hipSuccess) h = hipDeviceSynchronize();
        (void)hipSetDevice(prev);
        if (h != hipSuccess) {
            if (e->ctl) (void)hipFree(e->ctl);
            free(e);
            return UVHTTP_WS_GPU_ENOMEM;
        }
    }
    {
        int pools = 0;
        if (hipDeviceGetAttribute(&pools, hipDeviceAttributeMemoryPoolsSupported, device) != hipSuccess)
            pools = 0;
        e->pool_ok = pools ? 1 : 0;
    }
#ifdef UVWS_EXPERIMENTS
    experiment_knobs(e);
#endif
    *out = e;
    return UVHTTP_WS_GPU_OK;
}

void uvhttp_ws_gpu_engine_free(uvhttp_ws_gpu_engine_t* e) {
    if (!e) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(e->device);
    (void)hipDeviceSynchronize();
    scratch_free(e, e->ws_mem);
    scratch_free(e, e->ss_mem);
    scratch_free(e, e->bs_mem);
    scratch_free(e, e->wt_mem);
    scratch_free(e, e->wr_mem);
    scratch_free(e, e->dscr);
    scratch_free(e, e->sp_mem);
    if (e->pool_ok) (void)hipStreamSynchronize(nullptr);
    if (e->ctl) (void)hipFree(e->ctl);
    if (e->stamp_mem) (void)hipFree(e->stamp_mem);
    if (e->order_ev) (void)hipEventDestroy(e->order_ev);
    for (int k = 0; k < e->ev_created; ++k) (void)hipEventDestroy(e->ev[k]);
    (void)hipSetDevice(prev);
    free(e);
}

const char* uvhttp_ws_gpu_engine_last_error(const uvhttp_ws_gpu_engine_t* e) {
    return e ? e->err : "no engine";
}

int uvhttp_ws_gpu_engine_sync(uvhttp_ws_gpu_engine_t* e, void* stream) {
    if (!e) return UVHTTP_WS_GPU_EINVAL;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != e->device) (void)hipSetDevice(e->device);
    hipError_t h = hipStreamSynchronize((hipStream_t)stream);
    uint32_t faults = e->faults_seen;
    if (h == hipSuccess)
        h = hipMemcpy(&faults, e->ctl + kCtlFaults, sizeof(faults), hipMemcpyDeviceToHost);
    if (prev != e->device) (void)hipSetDevice(prev);
    if (h != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "sync", h);
    if (faults != e->faults_seen) {
        const uint32_t n = faults - e->faults_seen;
        e->faults_seen = faults;
        snprintf(e->err, sizeof(e->err),
                 "%u call(s) gave up waiting in the single-pass scan: nothing of them was decoded", n);
        return UVHTTP_WS_GPU_ELAUNCH;
    }
    return UVHTTP_WS_GPU_OK;
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Scratch growth without a device-wide wait.  Inside a call (s = the call's
// stream) the old block is released and the new one allocated and zeroed ON that stream with
// the stream-ordered allocator: call_begin already ordered every earlier call of this engine
// before s's next work, so those calls finish with the old block first, the call's own kernels
// see the zeroed block, and no other stream of the process waits (hipDeviceSynchronize here made
// a batcher's first large flush stall its upload stream and every other engine's work).  A later
// call on another stream is ordered behind s by call_begin too.  From the host outside any call
// (s = null: engine_reserve before a capture, a call's first use) the device is drained before the
// old block goes and after the new one is zeroed, as the API promises a reserve that is complete
// when it returns.  Devices without memory pools keep hipMalloc / hipFree and the device syncs.
static hipError_t scratch_grow(uvhttp_ws_gpu_engine_t* e, void** p, size_t bytes, bool zero,
                               hipStream_t s, bool in_call) {
    hipError_t h = hipSuccess;
    if (!in_call || !e->pool_ok) h = hipDeviceSynchronize();
    if (*p) (void)(e->pool_ok ? hipFreeAsync(*p, in_call ? s : nullptr) : hipFree(*p));
    *p = nullptr;
    if (h != hipSuccess) return h;
    if (e->pool_ok) {
        const hipStream_t st = in_call ? s : nullptr;
        h = hipMallocAsync(p, bytes, st);
        if (h == hipSuccess && zero) h = hipMemsetAsync(*p, 0, bytes, st);
        if (h == hipSuccess && !in_call) h = hipStreamSynchronize(nullptr);
        if (h != hipSuccess && *p) {
            (void)hipFreeAsync(*p, st);
            *p = nullptr;
        }
        return h;
    }
    h = hipMalloc(p, bytes);
    if (h == hipSuccess && zero) h = hipMemset(*p, 0, bytes);
    if (h == hipSuccess) h = hipDeviceSynchronize();
    if (h != hipSuccess && *p) {
        (void)hipFree(*p);
        *p = nullptr;
    }
    return h;
}
// an engine-owned scratch block at engine_free (the device is drained first)
static void scratch_free(uvhttp_ws_gpu_engine_t* e, void* p) {
    if (!p) return;
    if (e->pool_ok) (void)hipFreeAsync(p, nullptr);
    else (void)hipFree(p);
}

// the workspace for max_frames / wire / arena; in_call: grown on the call's stream s
static int reserve_ws(uvhttp_ws_gpu_engine_t* e, uint32_t max_frames, uint64_t max_wire_bytes,
                      uint64_t max_arena_bytes, hipStream_t s, bool in_call) {
    if (!e) return UVHTTP_WS_GPU_EINVAL;
    if (max_frames > kMaxFrames) return set_err(e, UVHTTP_WS_GPU_EINVAL, "too many frames", hipSuccess);
    const uint64_t tiles = (max_wire_bytes + kMapTile - 1) / kMapTile + 1;
    const uint64_t atiles = (max_arena_bytes + kMapTile - 1) / kMapTile + 1;
    if (e->ws_mem && max_frames <= e->cap_frames && tiles <= e->cap_tiles &&
        atiles <= e->cap_arena_tiles)
        return UVHTTP_WS_GPU_OK;
    if (e->capturing)
        return set_err(e, UVHTTP_WS_GPU_EINVAL, "workspace too small for a captured call: reserve first",
                       hipSuccess);
    const uint32_t fr = max_frames > e->cap_frames ? max_frames : e->cap_frames;
    const uint64_t tl = tiles > e->cap_tiles ? tiles : e->cap_tiles;
    const uint64_t at = atiles > e->cap_arena_tiles ? atiles : e->cap_arena_tiles;
    const uint64_t nblk = (fr + kBlock - 1) / kBlock + 2;
    const uint64_t ngrp = nblk / kBlock + 2;
    size_t off_agg = 0;
    size_t off_grp = align_up(off_agg + nblk * sizeof(ScanElem), 256);
    size_t off_incl = align_up(off_grp + ngrp * sizeof(ScanElem), 256);
    size_t off_excl = align_up(off_incl + nblk * sizeof(ScanElem), 256);
    size_t off_reca = align_up(off_excl + nblk * sizeof(ScanElem), 256);
    size_t off_recp = align_up(off_reca + nblk * sizeof(LbRec), 256);
    size_t off_cnt = align_up(off_recp + nblk * sizeof(LbRec), 256);
    size_t off_tiles = align_up(off_cnt + 16, 256);
    size_t off_bad = align_up(off_tiles + tl * sizeof(uint64_t), 256);
    size_t off_arena = align_up(off_bad + 16, 256);
    size_t off_recs = align_up(off_arena + at * sizeof(uint64_t), 256);
    size_t off_parts = align_up(off_recs + (size_t)fr * sizeof(FrameRec8), 256);
    size_t off_info = align_up(off_parts + ((size_t)fr / (kBlock * kScanFpt) + 2) * sizeof(TilePart), 256);
    size_t bytes = align_up(off_info + (size_t)fr + 64, 256);
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(e->device);
    // zero: ticket counters start at 0 and no flag / tag matches a live epoch (epochs >= 1)
    hipError_t h = scratch_grow(e, &e->ws_mem, bytes, true, s, in_call);
    (void)hipSetDevice(prev);
    if (h != hipSuccess) {
        e->ws_mem = nullptr;
        e->cap_frames = 0;
        e->cap_tiles = e->cap_arena_tiles = 0;
        return set_err(e, UVHTTP_WS_GPU_ENOMEM, "hipMalloc workspace", h);
    }
    char* b = (char*)e->ws_mem;
    e->ws.block_agg = (ScanElem*)(b + off_agg);
    e->ws.group_agg = (ScanElem*)(b + off_grp);
    e->ws.block_incl = (ScanElem*)(b + off_incl);
    e->ws.block_excl = (ScanElem*)(b + off_excl);
    e->ws.rec_a = (LbRec*)(b + off_reca);
    e->ws.rec_p = (LbRec*)(b + off_recp);
    e->ws.counters = (uint32_t*)(b + off_cnt);
    e->ws.tile_first = (uint64_t*)(b + off_tiles);
    e->ws.first_bad = (uint64_t*)(b + off_bad);
    e->ws.spec_bad = e->ws.first_bad + 1;  // (off_bad reserves 16 bytes)
    e->ws.arena_first = (uint64_t*)(b + off_arena);
    e->ws.recs = b + off_recs;
    e->ws.parts = b + off_parts;
    e->ws.info = (uint8_t*)(b + off_info);
    e->ws.ctl = e->ctl;
    e->ws_bytes = bytes;
    e->cap_frames = fr;
    e->cap_tiles = tl;
    e->cap_arena_tiles = at;
    return UVHTTP_WS_GPU_OK;
}

int uvhttp_ws_gpu_engine_reserve(uvhttp_ws_gpu_engine_t* e, uint32_t max_frames,
                                 uint64_t max_wire_bytes, uint64_t max_arena_bytes) {
    return reserve_ws(e, max_frames, max_wire_bytes, max_arena_bytes, nullptr, false);
}

int uvhttp_ws_gpu_engine_set_tile(uvhttp_ws_gpu_engine_t* e, int block, int vectors_per_lane) {
    if (!e) return UVHTTP_WS_GPU_EINVAL;
    static const int ok[][2] = {{0, 0}, {64, 1}, {64, 2}, {64, 4}, {128, 1},
                                {128, 2}, {256, 1}, {256, 2}, {256, 4}};
    for (const auto& c : ok) {
        if (c[0] == block && c[1] == vectors_per_lane) {
            e->tile_block = block;
            e->tile_vpt = vectors_per_lane;
            return UVHTTP_WS_GPU_OK;
        }
    }
    return set_err(e, UVHTTP_WS_GPU_EINVAL, "unsupported tile shape", hipSuccess);
}

int uvhttp_ws_gpu_engine_set_timing(uvhttp_ws_gpu_engine_t* e, int enable) {
    if (!e) return UVHTTP_WS_GPU_EINVAL;
    e->timing = enable > 0 ? enable : 0;
    e->timing_calls = 0;
    return UVHTTP_WS_GPU_OK;
}

static void harvest(uvhttp_ws_gpu_engine_t* e) {
    if (!e->ev_used) return;
    (void)hipEventSynchronize(e->ev[2 * e->ev_used - 1]);
    for (int k = 0; k < e->ev_used; ++k) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e->ev[2 * k], e->ev[2 * k + 1]) == hipSuccess) {
            e->time_ms += ms;
            e->launches++;
        }
    }
    e->ev_used = 0;
}

int uvhttp_ws_gpu_engine_kernel_time(uvhttp_ws_gpu_engine_t* e, double* ms, uint64_t* launches) {
    if (!e) return UVHTTP_WS_GPU_EINVAL;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(e->device);
    harvest(e);
    (void)hipSetDevice(prev);
    if (ms) *ms = e->time_ms;
    if (launches) *launches = e->launches;
    e->time_ms = 0;
    e->launches = 0;
    return UVHTTP_WS_GPU_OK;
}

int uvhttp_ws_gpu_engine_set_stamps(uvhttp_ws_gpu_engine_t* e, int enable) {
    if (!e) return UVHTTP_WS_GPU_EINVAL;
    if (enable && !e->stamp_mem) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(e->device);
        hipError_t h = hipMalloc(&e->stamp_mem, kStampAlloc * 8);
        if (h == hipSuccess) h = hipMemset(e->stamp_mem, 0, kStampAlloc * 8);
        if (h == hipSuccess) h = hipDeviceSynchronize();
        (void)hipSetDevice(prev);
        if (h != hipSuccess) {
            if (e->stamp_mem) (void)hipFree(e->stamp_mem);
            e->stamp_mem = nullptr;
            return set_err(e, UVHTTP_WS_GPU_ENOMEM, "hipMalloc stamps", h);
        }
    }
    e->stamp_on = enable ? 1 : 0;
    return UVHTTP_WS_GPU_OK;
}

int uvhttp_ws_gpu_engine_read_stamps(uvhttp_ws_gpu_engine_t* e, uvhttp_ws_gpu_stamp_t* out,
                                     uint32_t cap, uint32_t* n_out) {
    if (!e || (!out && cap) || !n_out) return UVHTTP_WS_GPU_EINVAL;
    *n_out = 0;
    if (!e->stamp_mem) return UVHTTP_WS_GPU_OK;
    uint64_t* host = (uint64_t*)malloc(kStampWords * 8);
    if (!host) return UVHTTP_WS_GPU_ENOMEM;
    int prev = 0, khz = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(e->device);
    hipError_t h = hipDeviceSynchronize();
    if (h == hipSuccess) h = hipMemcpy(host, e->stamp_mem, kStampWords * 8, hipMemcpyDeviceToHost);
    if (h == hipSuccess) h = hipMemset(e->stamp_mem, 0, kStampWords * 8);
    if (h == hipSuccess) h = hipDeviceSynchronize();
    if (h == hipSuccess && hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, e->device) != hipSuccess)
        khz = 0;
    (void)hipSetDevice(prev);
    if (h != hipSuccess) {
        free(host);
        return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "read stamps", h);
    }
    if (khz <= 0) khz = 100000;  // gfx9 wall clock: 100 MHz
    const int rc = uvhttp_ws_gpu_stamps_reduce(host, e->epoch, (uint32_t)khz, out, cap, n_out);
    free(host);
    return rc;
}

uint64_t uvhttp_ws_gpu_stamp_ring_words(void) { return kStampWords; }

// the ring -> one record per (call, kernel): the newest call's words of each slot, earliest
// begin and latest end (host only; read_stamps runs it on the copied ring, tests on a ring
// written by uvhttp_ws_gpu_stamp_simulate)
int uvhttp_ws_gpu_stamps_reduce(const uint64_t* host, uint32_t epoch, uint32_t khz,
                                uvhttp_ws_gpu_stamp_t* out, uint32_t cap, uint32_t* n_out) {
    if (!host || (!out && cap) || !n_out || !khz) return UVHTTP_WS_GPU_EINVAL;
    *n_out = 0;
    // a call's age: how many calls ago it ran, from the latest call's tag (tags wrap after
    // 2^24 - 1 calls, so neither "largest tag" nor the tag order is the call order)
    const uint32_t cur = stamp_tag(epoch);
    auto age = [&](uint64_t t) -> uint32_t {
        return (uint32_t)((cur + (uint64_t)kStampTagPeriod - t) % kStampTagPeriod);
    };
    uint32_t n = 0;
    std::vector<uint32_t> ages;
    for (uint32_t r = 0; r < kStampRing; ++r) {
        for (uint32_t k = 0; k < kStampKinds; ++k) {
            const uint64_t* sl = host + ((uint64_t)r * kStampKinds + k) * kStampPer;
            uint64_t tag = 0;  // the newest call that stamped this slot
            for (uint64_t j = 0; j < kStampPer; ++j) {
                const uint64_t t = sl[j] >> 40;
                if (t && (!tag || age(t) < age(tag))) tag = t;
            }
            if (!tag) continue;
            uint64_t b = ~0ull, en = 0;
            for (uint64_t j = 0; j < kStampPer; ++j) {
                if ((sl[j] >> 40) != tag) continue;
                const uint64_t t = sl[j] & kStampLow;
                if (j < kStampBegin) b = t < b ? t : b;
                else en = t > en ? t : en;
            }
            if (b == ~0ull || !en) continue;
            if (n < cap) {
                out[n].call = (uint32_t)tag;
                out[n].kernel = k;
                out[n].begin_ns = b * 1000000ull / (uint64_t)khz;
                out[n].end_ns = en * 1000000ull / (uint64_t)khz;
                ages.push_back(age(tag));
            }
            ++n;
        }
    }
    if (n > cap) n = cap;
    // call order (oldest first), then start order within a call
    for (uint32_t i = 1; i < n; ++i) {
        const uvhttp_ws_gpu_stamp_t x = out[i];
        const uint32_t xa = ages[i];
        uint32_t j = i;
        while (j > 0 && (ages[j - 1] < xa || (ages[j - 1] == xa && out[j - 1].begin_ns > x.begin_ns))) {
            out[j] = out[j - 1];
            ages[j] = ages[j - 1];
            --j;
        }
        out[j] = x;
        ages[j] = xa;
    }
    *n_out = n;
    return UVHTTP_WS_GPU_OK;
}

// What one launch piece of `blocks` workgroups (indices base .. base + blocks - 1 in the whole
// pass, `waves` waves each) stores into the ring, as ~StampScope does: workgroup i of the piece
// starts at t_begin + i * (t_end - t_begin) / blocks and its waves end `dur` ticks later.
int uvhttp_ws_gpu_stamp_simulate(uint64_t* ring, uint32_t epoch, uint32_t kind, uint64_t base,
                                 uint32_t blocks, uint32_t waves, uint64_t t_begin, uint64_t t_end,
                                 uint64_t dur) {
    if (!ring || kind >= kStampKinds || !blocks || !waves || t_end < t_begin) return UVHTTP_WS_GPU_EINVAL;
    uint64_t* sl = ring + ((uint64_t)(epoch % kStampRing) * kStampKinds + kind) * kStampPer;
    const uint64_t tag = (uint64_t)stamp_tag(epoch) << 40;
    for (uint32_t i = 0; i < blocks; ++i) {
        const uint64_t g = base + i;
        const bool sample = stamp_sampled(g);
        if (g >= kStampBegin && !sample) continue;
        const uint64_t t0 = t_begin + (t_end - t_begin) * i / blocks;
        if (g < kStampBegin) sl[g] = tag | (t0 & kStampLow);
        if (!sample) continue;
        for (uint32_t w = 0; w < waves; ++w) sl[kStampBegin + stamp_end_word(g, w)] = tag | ((t0 + dur) & kStampLow);
    }
    return UVHTTP_WS_GPU_OK;
}

#ifdef UVWS_PLAN_PHASES
// experiment builds only: copy k_plan's per-block phase words (8 per block) and clear them
extern "C" int uvhttp_ws_gpu_engine_debug_phases(uvhttp_ws_gpu_engine_t* e, uint64_t* out, uint32_t blocks) {
    if (!e || !e->stamp_mem || blocks > 8192) return UVHTTP_WS_GPU_EINVAL;
    (void)hipDeviceSynchronize();
    hipError_t h = hipMemcpy(out, e->stamp_mem + kStampWords, 64ull * blocks, hipMemcpyDeviceToHost);
    if (h == hipSuccess) h = hipMemset(e->stamp_mem + kStampWords, 0, 8 * kPhaseWords);
    if (h == hipSuccess) h = hipDeviceSynchronize();
    return h == hipSuccess ? 0 : UVHTTP_WS_GPU_ELAUNCH;
}
#endif

static int timing_begin(uvhttp_ws_gpu_engine_t* e, hipStream_t s) {
    if (!e->timing || e->capturing) return -1;
    // a timed marker between two kernels idles the device for a few us (the CP drains the
    // first kernel and writes the timestamp): sampled timing keeps that off most calls
    if (e->timing_calls++ % (uint64_t)e->timing != 0) return -1;
    if (e->ev_used * 2 + 2 > (int)(sizeof(e->ev) / sizeof(e->ev[0]))) harvest(e);
    const int k = e->ev_used;
    while (e->ev_created < 2 * k + 2) {
        // timing-only events: no system-scope fence (a fenced marker between two kernels
        // idled the device ~5.8 us per event, profiles/r03p1 kernel trace); the caller's own
        // synchronisation still orders the results.  UVHTTP_WS_TIMING_FENCE=1: fenced (A/B)
#ifdef UVWS_EXPERIMENTS
        static const unsigned flags = getenv("UVHTTP_WS_TIMING_FENCE") && atoi(getenv("UVHTTP_WS_TIMING_FENCE"))
                                          ? hipEventDefault : hipEventDisableSystemFence;
#else
        const unsigned flags = hipEventDisableSystemFence;
#endif
        if (hipEventCreateWithFlags(&e->ev[e->ev_created], flags) != hipSuccess) return -1;
        e->ev_created++;
    }
    (void)hipEventRecord(e->ev[2 * k], s);
    return k;
}

static void timing_end(uvhttp_ws_gpu_engine_t* e, int k, hipStream_t s) {
    if (k < 0) return;
    (void)hipEventRecord(e->ev[2 * k + 1], s);
    e->ev_used = k + 1;
}

// Record tags hold the epoch in 30 bits.  When the epoch space is used up the workspace is
// cleared on the call's stream (once per 2^30 - 1 calls), so no entry left by an earlier call
// can carry a live tag.

static uint32_t next_epoch(uvhttp_ws_gpu_engine_t* e, hipStream_t s) {
    if (e->capturing) {  // the replay's k_epoch issues it; kernels read ctl[kCtlEpoch]
        hipLaunchKernelGGL(k_epoch, dim3(64), dim3(kBlock), 0, s, e->ctl, (uint64_t*)e->ws_mem,
                           (uint64_t)(e->ws_mem ? e->ws_bytes / 8 : 0), (uint64_t*)e->bs_mem,
                           (uint64_t)(e->bs_mem ? e->bs_tiles * sizeof(BuildRec) / 8 : 0));
        return 0;
    }
    if (e->epoch >= kMaxHostEpoch) {
        (void)hipMemsetAsync(e->ws_mem, 0, e->ws_bytes, s);
        if (e->bs_mem) (void)hipMemsetAsync(e->bs_mem, 0, e->bs_tiles * sizeof(BuildRec), s);
        e->epoch = 0;
    }
    return ++e->epoch;
}

// scope of one API call: call_begin decides capture mode; leaving the call clears it
struct CallScope {
    uvhttp_ws_gpu_engine_t* e;
    ~CallScope() { e->capturing = 0; }
};

// Start of every call: is the stream being captured, and does the call switch streams?  The
// engine's workspace serves one call at a time, so a call on a new stream first waits for
// what the previous call's stream has queued.
static void call_begin(uvhttp_ws_gpu_engine_t* e, hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
    e->capturing = cs == hipStreamCaptureStatusActive;
    if (e->capturing) e->captured_ever = 1;
    if (!e->capturing && e->have_last && e->last_stream != s) {
        if (!e->order_ev) (void)hipEventCreateWithFlags(&e->order_ev, hipEventDisableTiming);
        if (e->order_ev && hipEventRecord(e->order_ev, e->last_stream) == hipSuccess)
            (void)hipStreamWaitEvent(s, e->order_ev, 0);
    }
    e->last_stream = s;
    e->have_last = 1;
}

// k_plan launch: frames per lane chosen so the grid stays within ~512 blocks — every block
// costs a ticket atomic and a look-back round on device-coherent records, so the call's time
// grows with the block count (C4, 1 048 576 frames: 4096 blocks 148 us, 2048 96, 1024 82,
// 512 64, 256 68 for k_plan + k_finalize); UVHTTP_WS_PLAN_FPT pins it for tuning
static void launch_plan(uvhttp_ws_gpu_engine_t* e, BatchArgs& a, uint32_t n_cap,
                        uvhttp_ws_frame_desc_t* d_desc, uvhttp_ws_message_desc_t* d_msgs,
                        hipStream_t s) {
    int fpt = e->plan_fpt;
    if (fpt != 1 && fpt != 2 && fpt != 4 && fpt != 8 && fpt != 16) {
        // records (fused stride path): contiguous 16-byte loads, no header gather to hide, so
        // fewer blocks (C4 fused: 512 blocks 143.8 us per step, 256 blocks 136.4, r03p4)
        const uint64_t max_blocks = a.recs ? 256 : 512;
        fpt = 1;
        while (fpt < 16 && ((uint64_t)n_cap + kBlock * fpt - 1) / (kBlock * fpt) > max_blocks) fpt *= 2;
    }
    a.no_ticket = e->plan_no_ticket;
    if (a.recs && e->plan_wide >= 2) {
        // records, A/B (UVHTTP_WS_PLAN_WIDE=2 / 3): 512-thread blocks, 8 or 16 frames per lane
        const int f5 = e->plan_wide == 3 ? 16 : 8;
        const uint32_t per5 = 512u * (uint32_t)f5;
        a.plan_frames = per5;
        const uint32_t g5 = n_cap ? (n_cap + per5 - 1) / per5 : 1;
        if (f5 == 8) hipLaunchKernelGGL((k_plan<8, 512>), dim3(g5), dim3(512), 0, s, a, d_desc, d_msgs, e->ws);
        else hipLaunchKernelGGL((k_plan<16, 512>), dim3(g5), dim3(512), 0, s, a, d_desc, d_msgs, e->ws);
        return;
    }
    if (a.recs && e->plan_wide) {
        // records: 1024-thread blocks, so the per-lane state-machine chain is 4x shorter at
        // the same block count (occupancy 4 waves / SIMD instead of 1)
        int wf = 1;
        while (wf < 4 && ((uint64_t)n_cap + 1024 * wf - 1) / (1024 * wf) > 256) wf *= 2;
        const uint32_t wper = 1024 * wf;
        a.plan_frames = wper;
        const uint32_t wgrid = n_cap ? (n_cap + wper - 1) / wper : 1;
        if (wf == 1) hipLaunchKernelGGL((k_plan<1, 1024>), dim3(wgrid), dim3(1024), 0, s, a, d_desc, d_msgs, e->ws);
        else if (wf == 2) hipLaunchKernelGGL((k_plan<2, 1024>), dim3(wgrid), dim3(1024), 0, s, a, d_desc, d_msgs, e->ws);
        else hipLaunchKernelGGL((k_plan<4, 1024>), dim3(wgrid), dim3(1024), 0, s, a, d_desc, d_msgs, e->ws);
        return;
    }
    const uint32_t per = kBlock * fpt;
    a.plan_frames = per;
    const uint32_t grid = n_cap ? (n_cap + per - 1) / per : 1;
    if (a.recs) {  // the records-only instantiation (its registers sized for records alone)
        switch (fpt) {
            case 1: hipLaunchKernelGGL((k_plan<1, kBlock, true>), dim3(grid), dim3(kBlock), 0, s, a, d_desc, d_msgs, e->ws); break;
            case 2: hipLaunchKernelGGL((k_plan<2, kBlock, true>), dim3(grid), dim3(kBlock), 0, s, a, d_desc, d_msgs, e->ws); break;
            case 4: hipLaunchKernelGGL((k_plan<4, kBlock, true>), dim3(grid), dim3(kBlock), 0, s, a, d_desc, d_msgs, e->ws); break;
            case 8: hipLaunchKernelGGL((k_plan<8, kBlock, true>), dim3(grid), dim3(kBlock), 0, s, a, d_desc, d_msgs, e->ws); break;
            default: hipLaunchKernelGGL((k_plan<16, kBlock, true>), dim3(grid), dim3(kBlock), 0, s, a, d_desc, d_msgs, e->ws); break;
        }
        return;
    }
    switch (fpt) {
        case 1: hipLaunchKernelGGL(k_plan<1>, dim3(grid), dim3(kBlock), 0, s, a, d_desc, d_msgs, e->ws); break;
        case 2: hipLaunchKernelGGL(k_plan<2>, dim3(grid), dim3(kBlock), 0, s, a, d_desc, d_msgs, e->ws); break;
        case 4: hipLaunchKernelGGL(k_plan<4>, dim3(grid), dim3(kBlock), 0, s, a, d_desc, d_msgs, e->ws); break;
        case 8: hipLaunchKernelGGL(k_plan<8>, dim3(grid), dim3(kBlock), 0, s, a, d_desc, d_msgs, e->ws); break;
        default: hipLaunchKernelGGL(k_plan<16>, dim3(grid), dim3(kBlock), 0, s, a, d_desc, d_msgs, e->ws); break;
    }
}

// The uniform payload length of a stride batch: P with header(P) + 4 + P == stride, header(P)
// the minimal encoding (2 / 4 / 10 bytes) — what a masked frame filling its slot carries; 0 when
// no such P exists (strides 132 and 133, or below 6)
static uint64_t spec_payload(uint64_t stride) {
    static const uint64_t hs[3] = {2, 4, 10};
    for (uint64_t h : hs) {
        if (stride < h + 4) continue;
        const uint64_t p = stride - h - 4;
        if ((p < 126 ? 2u : p < 65536 ? 4u : 10u) == h) return p;
    }
    return 0;
}

// Largest payload a delivered frame of `slot` wire bytes can declare: the shortest header
// that encodes it (7-bit up to 125, 16-bit up to 65535 — non-minimal forms are legal,
// src/uvhttp_websocket.c:133-185), plus the key a server requires
static uint64_t max_payload_in(uint64_t slot, int32_t is_server) {
    const uint64_t m = is_server ? 4u : 0u;
    uint64_t best = 0;
    if (slot >= 2 + m) best = slot - 2 - m < 125 ? slot - 2 - m : 125;
    if (slot >= 4 + m) {
        const uint64_t p = slot - 4 - m < 65535 ? slot - 4 - m : 65535;
        best = p > best ? p : best;
    }
    if (slot >= 10 + m && slot - 10 - m > best) best = slot - 10 - m;
    return best;
}

// the engine's descriptor scratch for calls that pass d_desc == NULL on a path that needs
// descriptors internally (grown on demand; a captured call must not grow it)
static uvhttp_ws_frame_desc_t* desc_scratch(uvhttp_ws_gpu_engine_t* e, uint32_t n, hipStream_t s) {
    const uint64_t want = n ? n : 1;
    if (e->dscr && e->dscr_cap >= want) return e->dscr;
    if (e->capturing) return nullptr;
    e->dscr_cap = 0;
    if (scratch_grow(e, reinterpret_cast<void**>(&e->dscr), want * sizeof(uvhttp_ws_frame_desc_t),
                     false, s, true) != hipSuccess) {
        e->dscr = nullptr;
        return nullptr;
    }
    e->dscr_cap = want;
    return e->dscr;
}

// The summary-only kernels' fragment state machine is exact for a stride batch when every slot
// but the last is too long for a control frame (stride >= kSumMinStride) and no message can
// reach max_message_size even if every frame joined it
static bool sum_ok(const uvhttp_ws_gpu_engine_t* e, const uvhttp_ws_batch_t* b) {
    if (!e->sum_fast || b->frame_off || b->n_frames == 0 || b->frame_stride < kSumMinStride) return false;
    const uint64_t n = b->n_frames;
    if ((n - 1) > (b->wire_len - 1) / b->frame_stride) return false;
    const uint64_t lim = (uint64_t)(int64_t)b->max_message_size;
    const uint64_t last_slot = b->wire_len - (n - 1) * b->frame_stride;
    const uint64_t msg_bound = (n - 1) * max_payload_in(b->frame_stride, b->is_server) +
                               max_payload_in(last_slot, b->is_server);
    return lim == 0 || msg_bound <= lim;
}

static int check_batch(uvhttp_ws_gpu_engine_t* e, const uvhttp_ws_batch_t* b,
                       const void* d_summary) {
    if (!e || !b || !d_summary) return UVHTTP_WS_GPU_EINVAL;
    if (b->n_frames && !b->wire) return set_err(e, UVHTTP_WS_GPU_EINVAL, "wire is NULL", hipSuccess);
    if (((uintptr_t)b->wire) & 15u)
        return set_err(e, UVHTTP_WS_GPU_EINVAL, "wire must be 16-byte aligned", hipSuccess);
    if (b->n_frames > kMaxFrames) return set_err(e, UVHTTP_WS_GPU_EINVAL, "too many frames", hipSuccess);
    if (!b->frame_off && b->n_frames > 1 && b->frame_stride == 0)
        return set_err(e, UVHTTP_WS_GPU_EINVAL, "stride 0", hipSuccess);
    return UVHTTP_WS_GPU_OK;
}

static int run_decode(uvhttp_ws_gpu_engine_t* e, const uvhttp_ws_batch_t* b, uint8_t* arena,
                      uint64_t arena_cap, uvhttp_ws_frame_desc_t* d_desc,
                      uvhttp_ws_message_desc_t* d_msgs, uvhttp_ws_batch_summary_t* d_summary,
                      void* stream) {
    int rc = check_batch(e, b, d_summary);
    if (rc) return rc;
    CallScope scope{e};
    call_begin(e, (hipStream_t)stream);
    const uint64_t n_tiles = (b->wire_len + kMapTile - 1) / kMapTile;
    // arena tiles: bounded by both the capacity and the data payload that can exist
    uint64_t arena_need = arena ? (arena_cap < b->wire_len ? arena_cap : b->wire_len) : 0;
    const uint64_t n_atiles = arena ? (arena_need + kMapTile - 1) / kMapTile : 0;
    rc = reserve_ws(e, b->n_frames, b->wire_len, arena_need, (hipStream_t)stream, true);
    if (rc) return rc;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != e->device) (void)hipSetDevice(e->device);
    hipStream_t s = (hipStream_t)stream;

    BatchArgs a;
    memset(&a, 0, sizeof(a));  // stream-mode fields stay null in batch mode
    a.wire = b->wire;
    a.wire_len = b->wire_len;
    a.frame_off = b->frame_off;
    a.frame_stride = b->frame_stride;
    a.n = b->n_frames;
    a.max_frame_size = b->max_frame_size;
    a.max_message_size = b->max_message_size;
    a.is_server = b->is_server;
    a.n_tiles = n_tiles;
    a.arena = arena;
    a.arena_cap = arena_cap;
    a.n_arena_tiles = n_atiles;
    a.summary = d_summary;
    a.msgs = arena ? d_msgs : nullptr;
    a.max_polls = e->max_polls;
    a.dev_epoch = e->capturing ? 1u : 0u;
    a.epoch = next_epoch(e, s);
    a.stamp = (e->stamp_on && !e->capturing) ? e->stamp_mem : nullptr;
    a.cas_claims = e->captured_ever ? 1u : 0u;

    // stride batches in place: the fused path (payload pass parses the headers, k_plan runs
    // on its records, k_fixup undoes what a failure must leave untouched)
    const bool fused = !arena && !b->frame_off && !e->fused_off && a.n > 0 &&
                       b->wire_len / a.n <= e->fused_max_avg &&
                       b->frame_stride >= kFusedMinStride && b->wire_len > 0 &&
                       b->wire_len < (1ull << 52) &&
                       (uint64_t)(a.n - 1) <= (b->wire_len - 1) / b->frame_stride;
    if (fused) {
        a.recs = reinterpret_cast<FrameRec8*>(e->ws.recs);
        a.stride_inv = 1.0 / (double)b->frame_stride;
        // 16 KiB tiles at every fused frame size: the tile's LDS staging, parse and barriers
        // are paid per tile, so the fused pass wants larger tiles than the plain payload
        // kernel (r03p34: 256x4 97.9 us on C4, 256x2 112.6, 64x1 182.7; r03p35: 32 KiB tiles
        // lose, 256x8 +16 %, 512x4 +5 %)
        int fb = e->tile_block, fv = e->tile_vpt;
        if (!fb) {
            fb = 256;
            fv = 4;
        }
        if (e->fused_block) {
            fb = e->fused_block;
            fv = e->fused_vpt;
        }
        const uint64_t ft = (uint64_t)fb * fv * 16;
        const uint64_t f_tiles = (b->wire_len + ft - 1) / ft;
        const uint64_t f_max = (1ull << 24);
        // Summary-only decode (d_desc == NULL): the payload pass also runs the fragment state
        // machine (the previous frame decides it when every frame before a delivered one is a
        // data frame — stride >= kSumMinStride — and no message can reach max_message_size: the
        // bound below) and leaves one TilePart per tile; k_sum_tail writes the summary and undoes
        // a failure.  No records, no k_plan, no descriptors.
        const bool sum_fast = !d_desc && fb == 256 && fv == 4 && e->fused_aux == 18 && sum_ok(e, b);
        // descriptors under the same bounds: records + info bytes, the info-byte scan, then the
        // parallel descriptor pass (k_desc_emit) instead of k_plan on the records + k_fixup
        const bool desc_emit = d_desc && e->desc_emit && fb == 256 && fv == 4 && e->fused_aux == 18 &&
                               sum_ok(e, b);
        if (desc_emit) {
            // (desc_emit >= 2: no info bytes — the scan and k_desc_emit rebuild them from the records)
            const bool from_rec = e->desc_emit >= 2;
            const int stk = timing_begin(e, s);
            for (uint64_t tb = 0; tb < f_tiles; tb += f_max) {
                const uint32_t grid_p = (uint32_t)((f_tiles - tb) < f_max ? (f_tiles - tb) : f_max);
                if (from_rec)
                    hipLaunchKernelGGL((k_unmask_stride<256, 4, 18, kLeaveRec>), dim3(grid_p), dim3(256), 0, s, a,
                                       e->ws, tb);
                else
                    hipLaunchKernelGGL((k_unmask_stride<256, 4, 18, kLeaveBoth>), dim3(grid_p), dim3(256), 0, s, a,
                                       e->ws, tb);
            }
            timing_end(e, stk, s);
            const uint32_t n_parts = (a.n + kBlock * kScanFpt - 1) / (kBlock * kScanFpt);
            if (from_rec) {
                hipLaunchKernelGGL((k_sum_scan<false, UVHTTP_WS_STAMP_SUM_SCAN, true>), dim3(n_parts), dim3(kBlock),
                                   0, s, a, e->ws);
                hipLaunchKernelGGL(k_desc_emit<true>, dim3(n_parts), dim3(kBlock), 0, s, a, e->ws, n_parts, d_desc);
            } else {
                BatchArgs ai = a;  // the scan reads the info bytes
                ai.recs = reinterpret_cast<FrameRec8*>(e->ws.info);
                hipLaunchKernelGGL((k_sum_scan<false, UVHTTP_WS_STAMP_SUM_SCAN>), dim3(n_parts), dim3(kBlock), 0,
                                   s, ai, e->ws);
                hipLaunchKernelGGL(k_desc_emit<false>, dim3(n_parts), dim3(kBlock), 0, s, a, e->ws, n_parts, d_desc);
            }
            hipError_t hs = hipGetLastError();
            if (prev != e->device) (void)hipSetDevice(prev);
            if (hs != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "launch", hs);
            return UVHTTP_WS_GPU_OK;
        }
        if (sum_fast) {
            a.recs = reinterpret_cast<FrameRec8*>(e->ws.recs);  // (the info bytes: 1 per frame)
            const int stk = timing_begin(e, s);
            for (uint64_t tb = 0; tb < f_tiles; tb += f_max) {
                const uint32_t grid_p = (uint32_t)((f_tiles - tb) < f_max ? (f_tiles - tb) : f_max);
                hipLaunchKernelGGL((k_unmask_stride<256, 4, 18, kLeaveInfo>), dim3(grid_p), dim3(256), 0, s, a,
                                   e->ws, tb);
            }
            timing_end(e, stk, s);
            const uint32_t n_parts = (a.n + kBlock * kScanFpt - 1) / (kBlock * kScanFpt);
            hipLaunchKernelGGL(k_sum_scan<false>, dim3(n_parts), dim3(kBlock), 0, s, a, e->ws);
            hipLaunchKernelGGL(k_sum_tail, dim3(kSumTailGrid), dim3(kBlock), 0, s, a, e->ws, n_parts);
            hipError_t hs = hipGetLastError();
            if (prev != e->device) (void)hipSetDevice(prev);
            if (hs != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "launch", hs);
            return UVHTTP_WS_GPU_OK;
        }
        if (!d_desc && !(d_desc = desc_scratch(e, a.n, s))) {
            if (prev != e->device) (void)hipSetDevice(prev);
            return set_err(e, UVHTTP_WS_GPU_ENOMEM, "descriptor scratch (reserve before capturing)", hipSuccess);
        }
        const int ftk = timing_begin(e, s);
        for (uint64_t tb = 0; tb < f_tiles; tb += f_max) {
            const uint32_t grid_p = (uint32_t)((f_tiles - tb) < f_max ? (f_tiles - tb) : f_max);
#define UVWS_FUSED(B, V)                                                                         \
    if (fb == B && fv == V) {                                                                    \
        if (B == 256 && V == 4 && e->fused_aux == 2)                                             \
            hipLaunchKernelGGL((k_unmask_stride<256, 4, 2>), dim3(grid_p), dim3(B), 0, s, a, e->ws, tb);  \
        else if (B == 256 && V == 4 && e->fused_aux == 0)                                        \
            hipLaunchKernelGGL((k_unmask_stride<256, 4, 0>), dim3(grid_p), dim3(B), 0, s, a, e->ws, tb);  \
        else if (B == 256 && V == 4 && e->fused_aux == 16)                                       \
            hipLaunchKernelGGL((k_unmask_stride<256, 4, 16>), dim3(grid_p), dim3(B), 0, s, a, e->ws, tb); \
        else                                                                                     \
            hipLaunchKernelGGL((k_unmask_stride<B, V>), dim3(grid_p), dim3(B), 0, s, a, e->ws, tb); \
    } else
            UVWS_FUSED(64, 1) UVWS_FUSED(64, 2) UVWS_FUSED(64, 4) UVWS_FUSED(128, 1)
            UVWS_FUSED(128, 2) UVWS_FUSED(256, 1) UVWS_FUSED(256, 2) UVWS_FUSED(256, 4)
            UVWS_FUSED(256, 8) UVWS_FUSED(512, 4) UVWS_FUSED(512, 8) {
                if (prev != e->device) (void)hipSetDevice(prev);
                return set_err(e, UVHTTP_WS_GPU_EINVAL, "unsupported fused tile shape", hipSuccess);
            }
#undef UVWS_FUSED
        }
        timing_end(e, ftk, s);
        if (e->rec_lookback) {
            launch_plan(e, a, a.n, d_desc, d_msgs, s);
        } else {
            constexpr int kRecFpt = 4;
            a.plan_frames = kBlock * kRecFpt;
            const uint32_t nblk = (a.n + a.plan_frames - 1) / a.plan_frames;
            hipLaunchKernelGGL(k_rec_reduce<kRecFpt>, dim3(nblk), dim3(kBlock), 0, s, a, e->ws);
            hipLaunchKernelGGL(k_rec_scan, dim3(1), dim3(kScanBlock), 0, s, e->ws, nblk);
            hipLaunchKernelGGL(k_rec_resolve<kRecFpt>, dim3(nblk), dim3(kBlock), 0, s, a, d_desc,
                               d_msgs, e->ws);
        }
        const uint32_t fx = (a.n + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(k_fixup, dim3(fx < e->fixup_blocks ? fx : e->fixup_blocks), dim3(kBlock), 0, s,
                           a, d_desc, e->ws);
        hipError_t hf = hipGetLastError();
        if (prev != e->device) (void)hipSetDevice(prev);
        if (hf != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "launch", hf);
        return UVHTTP_WS_GPU_OK;
    }
    // every other path keeps per-frame descriptors internally: a caller without them gets the
    // engine's scratch
    const bool no_desc = !d_desc;
    if (!d_desc && !(d_desc = desc_scratch(e, a.n, s))) {
        if (prev != e->device) (void)hipSetDevice(prev);
        return set_err(e, UVHTTP_WS_GPU_ENOMEM, "descriptor scratch (reserve before capturing)", hipSuccess);
    }
    // compact stride batches of small frames, speculatively: the payload pass
    // parses the headers (records) and writes every uniform frame's payload to f * P right
    // away; k_plan on the records checks that every delivered frame is where it went, and
    // k_spec_fix redoes the batch with the full scatter when one is not
    const uint64_t spec_p = spec_payload(b->frame_stride);
    const bool spec = arena && !b->frame_off && e->spec_on && a.n > 0 && spec_p &&
                      b->wire_len / a.n <= e->spec_max_avg && e->compact_mode != 1 &&
                      b->frame_stride >= kFusedMinStride && b->wire_len > 0 &&
                      b->wire_len < (1ull << 52) && arena_cap < (1ull << 52) &&
                      (uint64_t)(a.n - 1) <= (b->wire_len - 1) / b->frame_stride;
    if (spec) {
        a.recs = reinterpret_cast<FrameRec8*>(e->ws.recs);
        a.stride_inv = 1.0 / (double)b->frame_stride;
        a.spec_P = spec_p;
        constexpr uint64_t kSt = 256ull * 4 * 16;
        const uint64_t s_tiles = (b->wire_len + kSt - 1) / kSt;
        // summary-only (d_desc == NULL): the pass leaves info bytes instead of records;
        // k_sum_scan / k_sum_tail / k_sum_msgs run the state machine, check the speculation and
        // write the summary and the message table; a batch that broke the speculation (a control
        // frame, another length, ...) is decoded again by k_plan + k_spec_fix, which otherwise
        // return at once (ctl[kCtlGate])
        const bool sum_c = no_desc && sum_ok(e, b) && arena_cap / spec_p >= a.n;
        // with descriptors under the same bounds: the records pass, the scan and k_sum_msgs
        // rebuilding the info bytes from the records, k_sum_msgs also writing the descriptors
        const bool desc_c = !no_desc && e->desc_emit && sum_ok(e, b) && arena_cap / spec_p >= a.n;
        if (sum_c) a.recs = reinterpret_cast<FrameRec8*>(e->ws.recs);  // (the info bytes)
        const int stk = timing_begin(e, s);
        const bool both = desc_c && e->desc_emit != 2;  // (records + info bytes from the pass)
        for (uint64_t tb = 0; tb < s_tiles; tb += (1ull << 24)) {
            const uint32_t grid_s = (uint32_t)((s_tiles - tb) < (1ull << 24) ? (s_tiles - tb) : (1ull << 24));
            if (both)
                hipLaunchKernelGGL((k_unmask_stride<256, 4, kSpecCompact, kLeaveBoth>), dim3(grid_s), dim3(256), 0,
                                   s, a, e->ws, tb);
            else if (sum_c)
                hipLaunchKernelGGL((k_unmask_stride<256, 4, kSpecCompact, kLeaveInfo>), dim3(grid_s), dim3(256), 0, s, a,
                                   e->ws, tb);
            else
                hipLaunchKernelGGL((k_unmask_stride<256, 4, kSpecCompact>), dim3(grid_s), dim3(256), 0, s, a, e->ws, tb);
        }
        timing_end(e, stk, s);
        if (sum_c) {
            const uint32_t n_parts = (a.n + kBlock * kScanFpt - 1) / (kBlock * kScanFpt);
            hipLaunchKernelGGL(k_sum_scan<true>, dim3(n_parts), dim3(kBlock), 0, s, a, e->ws);
            hipLaunchKernelGGL(k_sum_msgs<>, dim3(n_parts), dim3(kBlock), 0, s, a, e->ws, n_parts, d_msgs,
                               nullptr);
            a.recs = nullptr;  // the fallback's k_plan gathers the headers
            a.gate = 1;
        } else if (desc_c) {
            const uint32_t n_parts = (a.n + kBlock * kScanFpt - 1) / (kBlock * kScanFpt);
            if (both) {
                BatchArgs ai = a;  // the scan reads the info bytes
                ai.recs = reinterpret_cast<FrameRec8*>(e->ws.info);
                hipLaunchKernelGGL((k_sum_scan<true, UVHTTP_WS_STAMP_SUM_SCAN>), dim3(n_parts), dim3(kBlock), 0, s,
                                   ai, e->ws);
                hipLaunchKernelGGL((k_sum_msgs<false, true>), dim3(n_parts), dim3(kBlock), 0, s, a, e->ws, n_parts,
                                   d_msgs, d_desc);
            } else {
                hipLaunchKernelGGL((k_sum_scan<true, UVHTTP_WS_STAMP_SUM_SCAN, true>), dim3(n_parts), dim3(kBlock),
                                   0, s, a, e->ws);
                hipLaunchKernelGGL((k_sum_msgs<true, true>), dim3(n_parts), dim3(kBlock), 0, s, a, e->ws, n_parts,
                                   d_msgs, d_desc);
            }
            a.gate = 1;  // (the fall-back's k_plan reads the same records)
        }
        launch_plan(e, a, a.n, d_desc, d_msgs, s);
        // (gated — it returns at once unless the speculation failed — a smaller grid: the
        // no-op launch costs less, the rare fall-back strides over more frames per block)
        const uint32_t nblk = (a.n + kBlock - 1) / kBlock;
        const uint32_t fix_max = a.gate ? 256u : 1024u;
        hipLaunchKernelGGL(k_spec_fix, dim3(nblk < fix_max ? nblk : fix_max), dim3(kBlock), 0, s, a, d_desc,
                           e->ws, s_tiles);
        const hipError_t hs = hipGetLastError();
        if (prev != e->device) (void)hipSetDevice(prev);
        if (hs != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "launch", hs);
        return UVHTTP_WS_GPU_OK;
    }
    // compact stride batches of small frames: a records-only pass over the wire (linear reads;
    // k_plan's scattered header gather costs as much as reading everything),
    // then k_plan on the records (UVHTTP_WS_COMPACT_RECS=1; off by default)
    const uint64_t cavg = a.n ? b->wire_len / a.n : 0;
    const bool rec_compact = arena && e->compact_recs && !b->frame_off && a.n > 0 &&
                             cavg <= e->fused_max_avg && cavg < kScatterAvg && e->compact_mode != 1 &&
                             b->frame_stride >= kFusedMinStride && b->wire_len > 0 &&
                             b->wire_len < (1ull << 52) &&
                             (uint64_t)(a.n - 1) <= (b->wire_len - 1) / b->frame_stride;
    if (rec_compact) {
        a.recs = reinterpret_cast<FrameRec8*>(e->ws.recs);
        a.stride_inv = 1.0 / (double)b->frame_stride;
        constexpr uint64_t kRt = 256ull * 4 * 16;
        const uint64_t r_tiles = (b->wire_len + kRt - 1) / kRt;
        for (uint64_t tb = 0; tb < r_tiles; tb += (1ull << 24)) {
            const uint32_t grid_r = (uint32_t)((r_tiles - tb) < (1ull << 24) ? (r_tiles - tb) : (1ull << 24));
            hipLaunchKernelGGL((k_unmask_stride<256, 4, -1>), dim3(grid_r), dim3(256), 0, s, a, e->ws, tb);
        }
    }
    launch_plan(e, a, a.n, d_desc, d_msgs, s);
    // payload kernel tile shape: explicit (set_tile) or by average wire bytes per frame
    // (auto shapes from tools/tile_sweep.py on MI355X, profiles/r01_tile_sweep.txt)
    int blk = e->tile_block, vpt = e->tile_vpt;
    const uint64_t avg = a.n ? b->wire_len / a.n : 0;
    // compact decode: frames below kScatterAvg wire bytes on average take the wire-driven
    // scatter kernel, larger ones the arena-driven gather (UVHTTP_WS_COMPACT=gather|scatter)
    const bool scatter = arena && (e->compact_mode ? e->compact_mode == 2 : avg < kScatterAvg);
    if (!blk) {
        if (!arena) {
            inplace_tile_shape(avg, blk, vpt);
        } else if (scatter) {
            blk = avg >= 32768 ? 64 : 256;
            vpt = avg >= 32768 ? 1 : avg >= 2048 ? 2 : 4;
            // the scatter kernel wants 16 KiB tiles at 2-16 KiB frames too (C2 compact 86.2 ->
            // 84.3 us, profiles/r04_tile_ab.txt)
            if (avg >= 2048 && avg < 16384) vpt = 4;
        } else {
            blk = avg >= 2048 ? 64 : 256;
            vpt = 2;
        }
    }
    const uint64_t span = arena && !scatter ? n_atiles * kMapTile : b->wire_len;
    const uint64_t tile_bytes = (uint64_t)blk * vpt * 16;
    uint64_t n_ptiles = (span + tile_bytes - 1) / tile_bytes;
    // in place and wire-driven compact: the payload kernel's first ceil(n / blk) blocks also
    // finalize (no k_finalize launch; not over an empty wire: its tile loads would have no
    // buffer to read)
    const bool fold_fin = b->wire_len != 0 && (!arena || scatter);
    const uint64_t n_fin = (a.n + blk - 1) / blk;
    if (fold_fin && n_ptiles < n_fin) n_ptiles = n_fin;
    // the dispatch packet counts work-items in 32 bits: split very large passes
    const uint64_t max_tiles = (1ull << 24);
    const int tk = timing_begin(e, s);
    for (uint64_t tb = 0; a.n && tb < n_ptiles; tb += max_tiles) {
        const uint32_t grid_p = (uint32_t)((n_ptiles - tb) < max_tiles ? (n_ptiles - tb) : max_tiles);
#define UVWS_LAUNCH(B, V)                                                                        \
    if (blk == B && vpt == V) {                                                                  \
        if (!arena && e->store_aux == 18)                                                        \
            hipLaunchKernelGGL((k_unmask_inplace<B, V, 18>), dim3(grid_p), dim3(B), 0, s, a,     \
                               d_desc, e->ws, tb);                                               \
        else if (!arena)                                                                         \
            hipLaunchKernelGGL((k_unmask_inplace<B, V>), dim3(grid_p), dim3(B), 0, s, a, d_desc, \
                               e->ws, tb);                                                       \
        else if (scatter)                                                                        \
            hipLaunchKernelGGL((k_scatter_compact<B, V>), dim3(grid_p), dim3(B), 0, s, a,        \
                               d_desc, e->ws, arena_cap, tb);                                    \
        else                                                                                     \
            hipLaunchKernelGGL((k_gather_compact<B, V>), dim3(grid_p), dim3(B), 0, s, a, d_desc, \
                               e->ws, arena_cap, tb);                                            \
    } else
        UVWS_LAUNCH(64, 1) UVWS_LAUNCH(64, 2) UVWS_LAUNCH(64, 4) UVWS_LAUNCH(128, 1)
        UVWS_LAUNCH(128, 2) UVWS_LAUNCH(256, 1) UVWS_LAUNCH(256, 2) UVWS_LAUNCH(256, 4) {}
#undef UVWS_LAUNCH
    }
    timing_end(e, tk, s);
    if (!fold_fin || !a.n) {
        const uint32_t grid_fin = a.n ? (a.n + kBlock - 1) / kBlock : 1;
        hipLaunchKernelGGL(k_finalize, dim3(grid_fin), dim3(kBlock), 0, s, a, d_desc, e->ws);
    }
    hipError_t h = hipGetLastError();
    if (prev != e->device) (void)hipSetDevice(prev);
    if (h != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "launch", h);
    return UVHTTP_WS_GPU_OK;
}

int uvhttp_ws_gpu_decode_inplace(uvhttp_ws_gpu_engine_t* e, const uvhttp_ws_batch_t* b,
                                 uvhttp_ws_frame_desc_t* d_desc,
                                 uvhttp_ws_batch_summary_t* d_summary, void* stream) {
    return run_decode(e, b, nullptr, 0, d_desc, nullptr, d_summary, stream);
}

int uvhttp_ws_gpu_decode_compact(uvhttp_ws_gpu_engine_t* e, const uvhttp_ws_batch_t* b,
                                 uint8_t* d_arena, uint64_t arena_cap,
                                 uvhttp_ws_frame_desc_t* d_desc, uvhttp_ws_message_desc_t* d_msgs,
                                 uvhttp_ws_batch_summary_t* d_summary, void* stream) {
    if (!d_arena || !d_msgs) return set_err(e, UVHTTP_WS_GPU_EINVAL, "arena/msgs NULL", hipSuccess);
    if (((uintptr_t)d_arena) & 15u)
        return set_err(e, UVHTTP_WS_GPU_EINVAL, "arena must be 16-byte aligned", hipSuccess);
    return run_decode(e, b, d_arena, arena_cap, d_desc, d_msgs, d_summary, stream);
}

static int reserve_streams(uvhttp_ws_gpu_engine_t* e, uint32_t frames, uint32_t streams,
                           uint32_t reads, hipStream_t s) {
    if (reads == 0) reads = 1;
    // (the look-back records are sized for the most blocks k_swalk_fused runs, 16 384 / 4, so
    // the connection count of a call never reallocates: a caller such as the batcher issues a
    // call while its previous one still runs on the stream)
    (void)streams;
    if (e->ss_mem && frames <= e->ss_frames && reads <= e->ss_reads) return UVHTTP_WS_GPU_OK;
    if (e->capturing)
        return set_err(e, UVHTTP_WS_GPU_EINVAL, "stream scratch too small for a captured call",
                       hipSuccess);
    const uint32_t fr = frames > e->ss_frames ? frames : e->ss_frames;
    const uint32_t rd = reads > e->ss_reads ? reads : e->ss_reads;
    size_t o_off = 0;
    size_t o_tot = align_up(o_off + (size_t)fr * 8, 256);
    size_t o_rsize = align_up(o_tot + 16, 256);
    size_t o_agg = align_up(o_rsize + (size_t)rd * 8, 256);
    size_t o_ctr = align_up(o_agg + ((size_t)kMaxFrames / kBlock + 2) * 4, 256);
    size_t o_srec = align_up(o_ctr + 16, 256);
    size_t bytes = align_up(o_srec + (size_t)kSwalkFusedMaxBlocks * 32, 256);
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(e->device);
    // (zero: the counters start at 0 and no record tag matches a live epoch.  On the call's
    // stream: a call of this engine may still run there with the old block — the batcher issues
    // a call while its previous one runs — and releases it first; scratch_grow)
    hipError_t h = scratch_grow(e, &e->ss_mem, bytes, true, s, true);
    (void)hipSetDevice(prev);
    if (h != hipSuccess) {
        e->ss_mem = nullptr;
        e->ss_frames = e->ss_reads = 0;
        return set_err(e, UVHTTP_WS_GPU_ENOMEM, "hipMalloc stream scratch", h);
    }
    char* b = (char*)e->ss_mem;
    e->ss.frame_off = (uint64_t*)(b + o_off);
    e->ss.n_total = (uint32_t*)(b + o_tot);
    e->ss.read_size = (uint64_t*)(b + o_rsize);
    e->ss.agg = (uint32_t*)(b + o_agg);
    e->ss.ctr = (uint32_t*)(b + o_ctr);
    e->ss.srec = (void*)(b + o_srec);
    e->ss_frames = fr;
    e->ss_reads = rd;
    return UVHTTP_WS_GPU_OK;
}

// the speculative stream decode's scratch (zeroed: no tile claim matches a live epoch)
static int reserve_spec(uvhttp_ws_gpu_engine_t* e, uint32_t streams, uint64_t tiles, hipStream_t s) {
    if (e->sp_mem && streams <= e->sp_streams && tiles <= e->sp_tiles) return UVHTTP_WS_GPU_OK;
    if (e->capturing)
        return set_err(e, UVHTTP_WS_GPU_EINVAL, "stream scratch too small for a captured call", hipSuccess);
    const uint32_t ns = streams > e->sp_streams ? streams : e->sp_streams;
    const uint64_t nt = tiles > e->sp_tiles ? tiles : e->sp_tiles;
    const size_t o_blk = align_up((size_t)ns * sizeof(SpecConn), 256);
    const size_t o_tile = align_up(o_blk + ((size_t)ns / kBlock + 2) * 8, 256);  // (counts, prefixes)
    const size_t o_trec = align_up(o_tile + (size_t)(nt + 1) * 8, 256);
    const size_t bytes = align_up(o_trec + (size_t)(nt + 1) * sizeof(SpecTile), 256);
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(e->device);
    const hipError_t h = scratch_grow(e, &e->sp_mem, bytes, true, s, true);
    (void)hipSetDevice(prev);
    if (h != hipSuccess) {
        e->sp_mem = nullptr;
        e->sp_streams = 0;
        e->sp_tiles = 0;
        return set_err(e, UVHTTP_WS_GPU_ENOMEM, "hipMalloc speculative stream scratch", h);
    }
    e->sp_streams = ns;
    e->sp_tiles = nt;
    return UVHTTP_WS_GPU_OK;
}

int uvhttp_ws_gpu_decode_streams(uvhttp_ws_gpu_engine_t* e, uint8_t* d_wire, uint64_t wire_len,
                                 const uvhttp_ws_stream_t* d_streams, uint32_t n_streams,
                                 uint32_t max_frames, uvhttp_ws_frame_desc_t* d_desc,
                                 uvhttp_ws_stream_result_t* d_results, void* stream) {
    return uvhttp_ws_gpu_decode_reads(e, d_wire, wire_len, d_streams, n_streams, nullptr, 0,
                                      max_frames, d_desc, d_results, stream);
}

// The stream decode: walk (per connection: calls, frames, state machine, result) -> first
// frames -> descriptors -> tile claims -> the in-place payload kernel.  Frame starts go to
// per-connection slices (single pass) when the slice scratch fits; otherwise the walk runs
// twice (count, then write the starts).
int uvhttp_ws_gpu_decode_reads(uvhttp_ws_gpu_engine_t* e, uint8_t* d_wire, uint64_t wire_len,
                               const uvhttp_ws_stream_t* d_streams, uint32_t n_streams,
                               const uint64_t* d_read_end, uint32_t n_reads_total,
                               uint32_t max_frames, uvhttp_ws_frame_desc_t* d_desc,
                               uvhttp_ws_stream_result_t* d_results, void* stream) {
    if (!e || (!d_wire && wire_len) || (!d_streams && n_streams) || !d_results ||
        (!d_desc && max_frames) || (!d_read_end && n_reads_total))
        return UVHTTP_WS_GPU_EINVAL;
    if (((uintptr_t)d_wire) & 15u)
        return set_err(e, UVHTTP_WS_GPU_EINVAL, "wire must be 16-byte aligned", hipSuccess);
    if (max_frames > kMaxFrames || n_streams > kMaxFrames)
        return set_err(e, UVHTTP_WS_GPU_EINVAL, "too many frames/streams", hipSuccess);
    if (!n_streams) return UVHTTP_WS_GPU_OK;
    CallScope scope{e};
    call_begin(e, (hipStream_t)stream);
    const uint32_t cap = max_frames ? max_frames : 1;
    int rc = reserve_ws(e, cap, wire_len, 0, (hipStream_t)stream, true);
    if (!rc) rc = reserve_streams(e, cap, n_streams, n_reads_total, (hipStream_t)stream);
    if (rc) return rc;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != e->device) (void)hipSetDevice(e->device);
    hipStream_t s = (hipStream_t)stream;

    // a wave per connection when the waves fill the chip in about one round, else a lane
    // (UVHTTP_WS_WALK=lane|wave pins it).  (Behind a speculative attempt, below, the walk path is
    // the fall-back, launched whether it runs or not; the lane walk's 64 times smaller grids
    // return at once a few us sooner, but as the fall-back of long connections it took C4 streams
    // 848 us per step instead of 139: the same rule as without the attempt.)
    const bool spec_try = e->stream_spec && wire_len > 0 && (uint64_t)max_frames >= 8ull * n_streams &&
                          (n_streams + kBlock - 1) / kBlock <= kSpecMaxBlk;
    const bool wave_walk = e->walk_mode ? e->walk_mode == 2 : n_streams <= 16384;
    // single pass (starts written into per-connection slices) unless UVHTTP_WS_WALK_SINGLE=0.
    // (The idle between calls of some C2 stream runs, DESIGN.md §5, is not the slices: with
    // the lane walk in two passes and no slice scratch, 2 of 10 runs idled all the same, r03p51.)
    const bool single_ok = e->walk_single_off == 0;
    // slices: connection s's starts at walk_tmp[begin / 2 + s ...] (4-byte entries)
    // (up to 16 GiB of slices — twice the wire, on a 288 GB device: C3's 4.3 GB streams call
    // walks in one pass; above 8 GiB it walked twice, the second walk + scan ~1 % of its step)
    const uint64_t want = wire_len / 2 + n_streams + 1;
    if (single_ok && !e->capturing && want * 4 <= (16ull << 30) && want > e->wt_cap) {
        // (an earlier call may still use the slices: released behind it on the stream)
        e->wt_cap = 0;
        if (scratch_grow(e, &e->wt_mem, want * 4, false, s, true) == hipSuccess) e->wt_cap = want;
    }
    // the wave walk's frame records (8 bytes per slice entry) while slices and records stay
    // within 8 GiB together; larger calls gather every header again in k_stream_desc
    // (only the wave walk writes and reads them: none for the lane walk — 1 GB less for C2)
    if (single_ok && wave_walk && !e->capturing && want * 12 <= (8ull << 30) && want > e->wr_cap) {
        e->wr_cap = 0;
        if (scratch_grow(e, &e->wr_mem, want * 8, false, s, true) == hipSuccess) e->wr_cap = want;
    }
    WalkArgs w;
    w.wire = d_wire;
    w.wire_len = wire_len;
    w.streams = d_streams;
    w.n_streams = n_streams;
    w.max_frames = max_frames;
    w.read_end = d_read_end;
    w.n_reads_total = n_reads_total;
    w.single = (single_ok && e->wt_cap >= want) ? 1u : 0u;
    w.results = d_results;
    w.desc = d_desc;
    w.tile_first = e->ws.tile_first;
    w.n_tiles = (wire_len + kMapTile - 1) / kMapTile;
    w.ctl = e->ctl;
    w.dev_epoch = e->capturing ? 1u : 0u;
    w.epoch = next_epoch(e, s);
    w.sc = e->ss;
    w.sc.walk_tmp = (uint32_t*)e->wt_mem;
    w.sc.walk_rec = (w.single && e->wr_cap >= want && e->wr_rec_on) ? (uint2*)e->wr_mem : nullptr;
    w.agg = e->ss.agg;
    w.stamp = (e->stamp_on && !e->capturing) ? e->stamp_mem : nullptr;
    w.cas_claims = e->captured_ever ? 1u : 0u;
    w.max_polls = e->max_polls;
    w.no_ticket = e->plan_no_ticket;
    w.nt_stores = e->stream_nt ? 1u : 0u;
    w.desc_scan = 0;
    w.nt_loads = e->walk_nt_load ? 1u : 0u;
    w.first_bad = e->ws.first_bad;
    const uint32_t nsb = (n_streams + kBlock - 1) / kBlock;
    const uint32_t nwb = (n_streams + kBlock / 64 - 1) / (kBlock / 64);
    const int tk_chain = e->time_chain ? timing_begin(e, s) : -1;
    // calls whose connections carry several frames each (by the caller's frame
    // capacity): the speculative decode first, the walk path behind it (gated)
    const uint64_t sp_tiles = (wire_len + kSpecT - 1) / kSpecT;
    const bool spec = spec_try && reserve_spec(e, n_streams, sp_tiles, s) == UVHTTP_WS_GPU_OK;
    int tk_spec = -1;
    SpecArgs sa_keep;
    memset(&sa_keep, 0, sizeof(sa_keep));
    if (spec) {
        SpecArgs& sa = sa_keep;
        sa.wire = d_wire;
        sa.wire_len = wire_len;
        sa.streams = d_streams;
        sa.n_streams = n_streams;
        sa.max_frames = max_frames;
        sa.read_end = d_read_end;
        sa.n_reads_total = n_reads_total;
        char* sb = (char*)e->sp_mem;
        sa.conns = (SpecConn*)sb;
        sa.blk = (uint32_t*)(sb + align_up((size_t)e->sp_streams * sizeof(SpecConn), 256));
        sa.blk_pre = sa.blk + ((size_t)e->sp_streams / kBlock + 2);
        sa.n_blk = nsb;
        sa.conn_tile = (uint64_t*)(sb + align_up(align_up((size_t)e->sp_streams * sizeof(SpecConn), 256) +
                                                     ((size_t)e->sp_streams / kBlock + 2) * 4, 256));
        sa.tiles = (SpecTile*)(sb + align_up(align_up(align_up((size_t)e->sp_streams * sizeof(SpecConn), 256) +
                                                            ((size_t)e->sp_streams / kBlock + 2) * 8, 256) +
                                                   (size_t)(e->sp_tiles + 1) * 8, 256));
        sa.n_tiles = sp_tiles;
        sa.recs = reinterpret_cast<FrameRec8*>(e->ws.recs);
        sa.desc = d_desc;
        sa.results = d_results;
        sa.ctl = e->ctl;
        sa.epoch = w.epoch;
        sa.dev_epoch = w.dev_epoch;
        sa.cas_claims = w.cas_claims;
        sa.stamp = w.stamp;
        hipLaunchKernelGGL(k_sspec_plan, dim3(nsb), dim3(kBlock), 0, s, sa);
        hipLaunchKernelGGL(k_sspec_tiles, dim3((uint32_t)((sp_tiles + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, sa);
        tk_spec = timing_begin(e, s);
        for (uint64_t tb = 0; tb < sp_tiles; tb += (1ull << 24)) {
            const uint32_t g = (uint32_t)((sp_tiles - tb) < (1ull << 24) ? (sp_tiles - tb) : (1ull << 24));
            hipLaunchKernelGGL(k_sspec_pass, dim3(g), dim3(kBlock), 0, s, sa, tb);
        }
        timing_end(e, tk_spec, s);
        hipLaunchKernelGGL(k_sspec_emit, dim3(nwb), dim3(kBlock), 0, s, sa);
        w.spec = 1;
    } else {
        w.spec = 0;
    }
    // UVHTTP_WS_WALK_FUSE=1: walk, scan and descriptors in one launch (k_swalk_fused; its
    // results are finished by the payload kernel's first workgroup, so not for an empty wire).
    // Not the default: it measured even with the three launches (C4 142.8 vs 142.6 us per
    // step, profiles/r05fy_*) and only without the block tickets (with them 155 us).
    const bool fused = !spec && wave_walk && w.single && e->walk_fuse && wire_len > 0 &&
                       n_streams <= kSwalkFusedMaxBlocks * (kBlock / 64);  // (its records)
    if (fused) {
        hipLaunchKernelGGL(k_swalk_fused, dim3(nwb), dim3(kBlock), 0, s, w);
    } else {
        // (behind the speculative decode, gated: the wave walk's kernels with kGatedGrid
        // workgroups striding over the blocks)
        const uint32_t ggrid = nwb < kGatedGrid ? nwb : kGatedGrid;
        if (wave_walk && spec) {
            if (w.single) hipLaunchKernelGGL(k_swalk_wave_gated<2>, dim3(ggrid), dim3(kBlock), 0, s, w, nwb);
            else hipLaunchKernelGGL(k_swalk_wave_gated<0>, dim3(ggrid), dim3(kBlock), 0, s, w, nwb);
        } else if (wave_walk) {
            if (w.single) hipLaunchKernelGGL(k_swalk_wave<2>, dim3(nwb), dim3(kBlock), 0, s, w);
            else hipLaunchKernelGGL(k_swalk_wave<0>, dim3(nwb), dim3(kBlock), 0, s, w);
        } else {
            if (w.single) hipLaunchKernelGGL(k_swalk_lane<2>, dim3(nsb), dim3(kBlock), 0, s, w);
            else hipLaunchKernelGGL(k_swalk_lane<0>, dim3(nsb), dim3(kBlock), 0, s, w);
        }
        // (single pass over at most kDescScanMax / kDescScanLaneMax connections: k_stream_desc /
        // k_stream_desc_lane scan)
        w.desc_scan = (w.single && n_streams <= (wave_walk ? kDescScanMax : kDescScanLaneMax) &&
                       !e->desc_scan_off) ? 1u : 0u;
        if (!w.desc_scan) hipLaunchKernelGGL(k_swalk_scan, dim3(1), dim3(kBlock), 0, s, w, wave_walk ? 0u : 1u);
        if (!w.single) {
            if (wave_walk && spec) hipLaunchKernelGGL(k_swalk_wave_gated<1>, dim3(ggrid), dim3(kBlock), 0, s, w, nwb);
            else if (wave_walk) hipLaunchKernelGGL(k_swalk_wave<1>, dim3(nwb), dim3(kBlock), 0, s, w);
            else hipLaunchKernelGGL(k_swalk_lane<1>, dim3(nsb), dim3(kBlock), 0, s, w);
        }
        if (wave_walk && spec) hipLaunchKernelGGL(k_stream_desc_gated, dim3(ggrid), dim3(kBlock), 0, s, w, nwb);
        else if (wave_walk) hipLaunchKernelGGL(k_stream_desc, dim3(nwb), dim3(kBlock), 0, s, w);
        else hipLaunchKernelGGL(k_stream_desc_lane, dim3(nsb), dim3(kBlock), 0, s, w);
    }

    BatchArgs a;
    memset(&a, 0, sizeof(a));
    a.wire = d_wire;
    a.wire_len = wire_len;
    a.n = cap;
    a.n_tiles = (wire_len + kMapTile - 1) / kMapTile;
    a.streams = d_streams;
    a.n_dev = e->ss.n_total;
    if (fused) {  // (the payload kernel's first workgroup: stream_fix)
        a.s_results = d_results;
        a.s_over = e->ss.ctr + 2;
        a.n_streams = n_streams;
    }
    a.max_polls = e->max_polls;
    a.dev_epoch = w.dev_epoch;
    a.epoch = w.epoch;
    a.stamp = w.stamp;
    a.cas_claims = w.cas_claims;
    // (k_stream_desc / k_stream_desc_lane claimed the tile map)
    if (spec) {  // the walk path's payload pass (after undoing the speculative one), gated
        const uint32_t g = sp_tiles < kSpecUndoGrid ? (uint32_t)sp_tiles : kSpecUndoGrid;
        hipLaunchKernelGGL(k_sspec_fallback, dim3(g), dim3(kBlock), 0, s, sa_keep, a, d_desc, e->ws, sp_tiles);
        timing_end(e, tk_chain, s);
        const hipError_t hs = hipGetLastError();
        if (prev != e->device) (void)hipSetDevice(prev);
        if (hs != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "launch", hs);
        return UVHTTP_WS_GPU_OK;
    }
    // payload tile shape: the frame count is only known on the device, so the caller's frame
    // capacity stands in for it (wire bytes per frame slot; the same rule as the batch decode)
    int blk = e->tile_block, vpt = e->tile_vpt;
    if (!blk) {
        const uint64_t avg = max_frames ? wire_len / max_frames : wire_len;
        inplace_tile_shape(avg, blk, vpt);
    }
    const uint64_t tile_bytes = (uint64_t)blk * vpt * 16;
    const uint64_t n_ptiles = (wire_len + tile_bytes - 1) / tile_bytes;
    const uint64_t max_tiles = (1ull << 24);
    const int tk = e->time_chain ? -1 : timing_begin(e, s);
    for (uint64_t tb = 0; tb < n_ptiles; tb += max_tiles) {
        const uint32_t grid_p = (uint32_t)((n_ptiles - tb) < max_tiles ? (n_ptiles - tb) : max_tiles);
#define UVWS_LAUNCH(B, V)                                                                        \
    if (blk == B && vpt == V) {                                                                  \
        if (e->store_aux == 18)                                                                  \
            hipLaunchKernelGGL((k_unmask_inplace<B, V, 18>), dim3(grid_p), dim3(B), 0, s, a,     \
                               d_desc, e->ws, tb);                                               \
        else                                                                                     \
            hipLaunchKernelGGL((k_unmask_inplace<B, V>), dim3(grid_p), dim3(B), 0, s, a, d_desc, \
                               e->ws, tb);                                                       \
    } else
        UVWS_LAUNCH(64, 1) UVWS_LAUNCH(64, 2) UVWS_LAUNCH(64, 4) UVWS_LAUNCH(128, 1)
        UVWS_LAUNCH(128, 2) UVWS_LAUNCH(256, 1) UVWS_LAUNCH(256, 2) UVWS_LAUNCH(256, 4) {}
#undef UVWS_LAUNCH
    }
    timing_end(e, tk, s);
    timing_end(e, tk_chain, s);
    const hipError_t h = hipGetLastError();
    if (prev != e->device) (void)hipSetDevice(prev);
    if (h != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "launch", h);
    return UVHTTP_WS_GPU_OK;
}

int uvhttp_ws_gpu_build_frames(uvhttp_ws_gpu_engine_t* e, const uint8_t* d_src, uint64_t src_len,
                               const uvhttp_ws_build_desc_t* d_frames, uint32_t n_frames,
                               uint8_t* d_out, uint64_t out_cap, uint64_t* d_out_off,
                               void* stream) {
    if (!e || (!d_frames && n_frames) || !d_out_off || (!d_out && out_cap) ||
        (!d_src && src_len))
        return UVHTTP_WS_GPU_EINVAL;
    if (((uintptr_t)d_out) & 15u)
        return set_err(e, UVHTTP_WS_GPU_EINVAL, "out must be 16-byte aligned", hipSuccess);
    if (n_frames > kMaxFrames) return set_err(e, UVHTTP_WS_GPU_EINVAL, "too many frames", hipSuccess);
    CallScope scope{e};
    call_begin(e, (hipStream_t)stream);
    // scratch: reuse the engine workspace (block/group aggregates as u64, arena map)
    int rc = reserve_ws(e, n_frames ? n_frames : 1, 0, 0, (hipStream_t)stream, true);
    if (rc) return rc;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != e->device) (void)hipSetDevice(e->device);
    hipStream_t s = (hipStream_t)stream;
    BuildArgs b;
    b.group = kEmitF;
    b.src = d_src;
    b.src_len = src_len;
    b.frames = d_frames;
    b.n = n_frames;
    b.out = d_out;
    b.out_cap = out_cap;
    b.out_off = d_out_off;
    b.blk = reinterpret_cast<uint64_t*>(e->ws.block_agg);
    b.grp = reinterpret_cast<uint64_t*>(e->ws.group_agg);
    // emit shape and map granularity from the average frame (the caller's capacity per frame):
    // frames >= 4 KiB take 2 KiB tiles whose two map records (the frame covering the tile's map
    // tile and the next one's) usually cover the whole tile; smaller frames take 16 KiB tiles
    // that stage their frames in LDS.  Map tile = largest power of two <= the average frame,
    // clamped to [tile, 64 KiB], so consecutive map records are at most one frame apart.
    const uint64_t avg = n_frames ? out_cap / n_frames : out_cap;
    const bool small = avg < 4096;
    // below build_frames_max the frame-grouped kernel (kb_emit_frames) replaces the tiles
    const bool grouped = n_frames && avg < e->build_frames_max;
    // small-frame tile: 0 = 64 x 2 (2 KiB, default), 1 = 64 x 4, 2 = 128 x 2, 3 = 256 x 4
    const int sh = small ? e->build_small : 0;
    const uint32_t tile_shift = sh == 3 ? 14 : (sh == 1 || sh == 2) ? 12 : 11;
    uint32_t shift = small ? 14 : 11;
    if (shift < tile_shift) shift = tile_shift;
    while (shift < 16 && (2ull << shift) <= avg) ++shift;
    b.map_shift = shift;
    b.n_map = grouped ? 0 : (out_cap + (1ull << shift) - 1) >> shift;  // grouped: no map records
    if (!grouped && b.n_map + 1 > e->bs_tiles) {
        if (e->capturing) {
            if (prev != e->device) (void)hipSetDevice(prev);
            return set_err(e, UVHTTP_WS_GPU_EINVAL, "build map too small for a captured call",
                           hipSuccess);
        }
        e->bs_tiles = 0;
        // + 1: kb_emit reads the record after its tile's; that spare entry is never tagged.
        // zero: tag 0 never matches a live epoch (epochs >= 1)
        hipError_t h = scratch_grow(e, &e->bs_mem, (b.n_map + 1) * sizeof(BuildRec), true, s, true);
        if (h != hipSuccess) {
            e->bs_mem = nullptr;
            if (prev != e->device) (void)hipSetDevice(prev);
            return set_err(e, UVHTTP_WS_GPU_ENOMEM, "hipMalloc build map", h);
        }
        e->bs_tiles = b.n_map + 1;
    }
    b.mrec = reinterpret_cast<BuildRec*>(e->bs_mem);
    b.ctl = e->ctl;
    b.dev_epoch = e->capturing ? 1u : 0u;
    b.epoch = next_epoch(e, s);
    b.stamp = (e->stamp_on && !e->capturing) ? e->stamp_mem : nullptr;
    const uint32_t grid_f = n_frames ? (n_frames + kBlock - 1) / kBlock : 1;
    const uint32_t n_groups = (grid_f + kBlock - 1) / kBlock;
    b.n_groups = n_groups;
    // sizes -> offsets: kb_size (within 256-frame blocks) and the scan of the block totals (one
    // workgroup up to 1 M frames); the grouped emit finishes the offsets itself, the tile emit
    // needs kb_offsets' map records (C4 send side: kb_scan_groups + kb_scan_top + kb_offsets were
    // 4.8 + 4.6 + 8.6 us of a 130 us step, profiles/r05pmc_c4_build_kernel_stats.csv)
    hipLaunchKernelGGL(kb_size, dim3(grid_f), dim3(kBlock), 0, s, b);
    if (grid_f <= kScanOne) {
        hipLaunchKernelGGL(kb_scan_one, dim3(1), dim3(kBlock), 0, s, b, grid_f);
    } else {
        hipLaunchKernelGGL(kb_scan_groups, dim3(n_groups), dim3(kBlock), 0, s, b, grid_f);
        hipLaunchKernelGGL(kb_scan_top, dim3(1), dim3(kBlock), 0, s, b, n_groups);
    }
    const uint64_t avg0 = n_frames ? out_cap / n_frames : out_cap;
    if (!(n_frames && avg0 < e->build_frames_max))
        hipLaunchKernelGGL(kb_offsets, dim3(grid_f), dim3(kBlock), 0, s, b, n_groups);
    if (!n_frames) {
        // d_out_off[0] = 0 (total) for an empty batch
        (void)hipMemsetAsync(d_out_off, 0, 8, s);
    }
    const int tk = timing_begin(e, s);
    if (grouped) {
        // frames per workgroup: as many as keep an average group inside one LDS window and
        // the item table (payload vectors ~ avg / 16 + 1 per frame)
        uint64_t g = kEmitItems / (avg / 16 + 2);
        if (g > kEmitWin / (avg + 16)) g = kEmitWin / (avg + 16);
        if (g > kEmitF) g = kEmitF;
        if (g < 1) g = 1;
        // up to 64 frames the smaller LDS footprint keeps 6 workgroups per CU (256-byte frames:
        // 100 us with 64 per group vs 116 with 71 in the large footprint); tiny frames (room for
        // >= 128 per group) take up to 256 (64-byte frames: 287 -> 149 us)
        const bool wide = g >= 128;
        if (!wide && g > 64) g = 64;
        b.group = (uint32_t)g;
        const dim3 grid((n_frames + b.group - 1) / b.group);
        if (wide) hipLaunchKernelGGL((kb_emit_frames<256, 256>), grid, dim3(256), 0, s, b);
        else hipLaunchKernelGGL((kb_emit_frames<256, 64>), grid, dim3(256), 0, s, b);
    }
    else if (sh == 3) launch_emit<256, 4>(b, n_frames, out_cap, s);
    else if (sh == 2) launch_emit<128, 2>(b, n_frames, out_cap, s);
    else if (sh == 1) launch_emit<64, 4>(b, n_frames, out_cap, s);
    else launch_emit<64, 2>(b, n_frames, out_cap, s);
    timing_end(e, tk, s);
    const hipError_t h = hipGetLastError();
    if (prev != e->device) (void)hipSetDevice(prev);
    if (h != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "launch", h);
    return UVHTTP_WS_GPU_OK;
}

int uvhttp_ws_gpu_apply_mask(uvhttp_ws_gpu_engine_t* e, uint8_t* d_data, uint64_t len,
                             const uint8_t key[4], void* stream) {
    if (!e || (!d_data && len) || !key) return UVHTTP_WS_GPU_EINVAL;
    if (!len) return UVHTTP_WS_GPU_OK;
    const uint32_t k = (uint32_t)key[0] | ((uint32_t)key[1] << 8) | ((uint32_t)key[2] << 16) |
                       ((uint32_t)key[3] << 24);
    uint64_t head = (16u - ((uintptr_t)d_data & 15u)) & 15u;
    if (head > len) head = len;
    const uint64_t nvec = (len - head) / 16;
    uint64_t tiles = (nvec + kMaskBlock - 1) / kMaskBlock;
    if (tiles < 1) tiles = 1;  // tile 0 also does the head and tail bytes
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != e->device) (void)hipSetDevice(e->device);
    hipStream_t s = (hipStream_t)stream;
    CallScope scope{e};
    call_begin(e, s);
    const int tk = timing_begin(e, s);
    const uint64_t max_tiles = (1ull << 24);
    for (uint64_t tb = 0; tb < tiles; tb += max_tiles) {
        const uint32_t grid = (uint32_t)((tiles - tb) < max_tiles ? (tiles - tb) : max_tiles);
        hipLaunchKernelGGL(k_apply_mask, dim3(grid), dim3(kMaskBlock), 0, s, d_data, len, k, head, tb);
    }
    timing_end(e, tk, s);
    hipError_t h = hipGetLastError();
    if (prev != e->device) (void)hipSetDevice(prev);
    if (h != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "launch", h);
    return UVHTTP_WS_GPU_OK;
}

int uvhttp_ws_gpu_gen_frames(uvhttp_ws_gpu_engine_t* e, uint8_t* d_wire, uint32_t n_frames,
                             uint64_t payload_len, uint64_t seed, int opcode0, int fragmented,
                             int force_keys, void* stream) {
    return uvhttp_ws_gpu_gen_frames_range(e, d_wire, 0, n_frames, n_frames, payload_len, seed,
                                          opcode0, fragmented, force_keys, stream);
}

int uvhttp_ws_gpu_gen_frames_range(uvhttp_ws_gpu_engine_t* e, uint8_t* d_wire, uint32_t first,
                                   uint32_t count, uint32_t n_frames, uint64_t payload_len,
                                   uint64_t seed, int opcode0, int fragmented, int force_keys,
                                   void* stream) {
    if (!e || (!d_wire && count)) return UVHTTP_WS_GPU_EINVAL;
    if ((uint64_t)first + count > n_frames) return set_err(e, UVHTTP_WS_GPU_EINVAL, "range past n_frames", hipSuccess);
    if (!count) return UVHTTP_WS_GPU_OK;
    const uint64_t wpf = payload_len ? (payload_len + 7) / 8 : 1;
    uint64_t total = (uint64_t)count * wpf;
    uint64_t grid = (total + kBlock - 1) / kBlock;
    if (grid > 65536) grid = 65536;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != e->device) (void)hipSetDevice(e->device);
    hipLaunchKernelGGL(k_gen_frames, dim3((uint32_t)grid), dim3(kBlock), 0, (hipStream_t)stream,
                       d_wire, first, count, n_frames, payload_len, seed, opcode0, fragmented,
                       force_keys, wpf);
    hipError_t h = hipGetLastError();
    if (prev != e->device) (void)hipSetDevice(prev);
    if (h != hipSuccess) return set_err(e, UVHTTP_WS_GPU_ELAUNCH, "launch", h);
    return UVHTTP_WS_GPU_OK;
}

// ---- host-memory pipeline ----------------------------------------------------------------

// Host-memory pipeline.  Two streams, as the batcher (ws_batcher.hip): every slot's H2D goes
// on the upload stream and its decode + D2H on the compute stream behind an event, so one
// slot's upload overlaps the previous slot's download on the two copy queues (round 3 gave
// each slot its own stream and engine: 25.2 GiB/s end to end against the batcher's 38.5 on
// the same box — the per-slot streams shared hardware queues and serialised the directions).
struct PipeSlot {
    uint8_t* h_wire;   // pinned
    uint64_t* h_off;   // pinned
    uvhttp_ws_frame_desc_t* h_desc;  // pinned
    uvhttp_ws_batch_summary_t* h_sum;  // pinned
    uint8_t* d_wire;
    uint64_t* d_off;
    uvhttp_ws_frame_desc_t* d_desc;
    uvhttp_ws_batch_summary_t* d_sum;
    hipEvent_t up_ev, done_ev;
    int busy;
    // compact submissions (allocated at a slot's first one): the message arena and table
    uint8_t* h_arena;  // pinned
    uvhttp_ws_message_desc_t* h_msgs;  // pinned
    uint8_t* d_arena;
    uvhttp_ws_message_desc_t* d_msgs;
    int compact;       // the slot's last submission was compact
    int with_desc;     //   ... and decoded into descriptors (not summary-only)
};

struct uvhttp_ws_gpu_pipeline {
    int device, depth;
    uint64_t slot_bytes;
    uint32_t slot_frames;
    uvhttp_ws_gpu_engine_t* eng;  // one workspace: the decodes run in order on `cs`
    hipStream_t up, cs;
    PipeSlot* slots;
    int in_flight;    // submit first waits (host) until fewer earlier submissions are in flight
    int recent[16];   // slots of the latest submissions (ring)
    uint64_t n_sub;   // submissions so far
};

// Submissions a pipeline lets run ahead of the host.  With more than three queued, H2D / decode /
// D2H chains of 16-256 MiB slots ran at 24-27 GiB/s (depth 4) and 16-26 (depth 8) against 43-44
// at depth 3, at every slot size; holding the device back instead (each upload waiting on the
// done event of the submission three earlier) did not help, bounding what the host has queued
// does: depth 4 43.9, depth 8 43.4 GiB/s (tools/r05_pipe5.sh, profiles/r05v_pipeline_in_flight.jsonl).
// With HSA_ENABLE_SDMA=0 depth 3 is as slow as depth 4, so the deeper queues most likely move
// the runtime's copies off the SDMA engines; UVHTTP_WS_PIPE_IN_FLIGHT overrides (0: no bound).
constexpr int kPipeInFlight = 3;

void uvhttp_ws_gpu_pipeline_free(uvhttp_ws_gpu_pipeline_t* p) {
    if (!p) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(p->device);
    if (p->up) (void)hipStreamSynchronize(p->up);
    if (p->cs) (void)hipStreamSynchronize(p->cs);
    for (int k = 0; k < p->depth && p->slots; ++k) {
        PipeSlot& s = p->slots[k];
        if (s.h_wire) (void)hipHostFree(s.h_wire);
        if (s.h_off) (void)hipHostFree(s.h_off);
        if (s.h_desc) (void)hipHostFree(s.h_desc);
        if (s.h_sum) (void)hipHostFree(s.h_sum);
        if (s.d_wire) (void)hipFree(s.d_wire);
        if (s.d_off) (void)hipFree(s.d_off);
        if (s.d_desc) (void)hipFree(s.d_desc);
        if (s.d_sum) (void)hipFree(s.d_sum);
        if (s.h_arena) (void)hipHostFree(s.h_arena);
        if (s.h_msgs) (void)hipHostFree(s.h_msgs);
        if (s.d_arena) (void)hipFree(s.d_arena);
        if (s.d_msgs) (void)hipFree(s.d_msgs);
        if (s.up_ev) (void)hipEventDestroy(s.up_ev);
        if (s.done_ev) (void)hipEventDestroy(s.done_ev);
    }
    if (p->up) (void)hipStreamDestroy(p->up);
    if (p->cs) (void)hipStreamDestroy(p->cs);
    uvhttp_ws_gpu_engine_free(p->eng);
    free(p->slots);
    (void)hipSetDevice(prev);
    free(p);
}

int uvhttp_ws_gpu_pipeline_create(int device, int depth, uint64_t slot_bytes,
                                  uint32_t slot_frames, uvhttp_ws_gpu_pipeline_t** out) {
    if (!out || depth < 1 || depth > 16 || !slot_bytes || !slot_frames) return UVHTTP_WS_GPU_EINVAL;
    *out = nullptr;
    uvhttp_ws_gpu_pipeline_t* p = (uvhttp_ws_gpu_pipeline_t*)calloc(1, sizeof(*p));
    if (!p) return UVHTTP_WS_GPU_ENOMEM;
    p->device = device;
    p->depth = depth;
    p->slot_bytes = slot_bytes;
    p->slot_frames = slot_frames;
    p->in_flight = kPipeInFlight;
#ifdef UVWS_EXPERIMENTS
    if (const char* pf = getenv("UVHTTP_WS_PIPE_IN_FLIGHT")) p->in_flight = atoi(pf);
#endif
    p->slots = (PipeSlot*)calloc((size_t)depth, sizeof(PipeSlot));
    if (!p->slots) {
        free(p);
        return UVHTTP_WS_GPU_ENOMEM;
    }
    int rc = uvhttp_ws_gpu_engine_create(device, &p->eng);
    if (!rc) rc = uvhttp_ws_gpu_engine_reserve(p->eng, slot_frames, slot_bytes, 0);
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    if (!rc && (hipStreamCreateWithFlags(&p->up, hipStreamNonBlocking) != hipSuccess ||
                hipStreamCreateWithFlags(&p->cs, hipStreamNonBlocking) != hipSuccess))
        rc = UVHTTP_WS_GPU_ENOMEM;
    for (int k = 0; k < depth && rc == UVHTTP_WS_GPU_OK; ++k) {
        PipeSlot& s = p->slots[k];
        const size_t pad = 64;
        if (hipHostMalloc((void**)&s.h_wire, slot_bytes + pad, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&s.h_off, (size_t)slot_frames * 8, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&s.h_desc, (size_t)slot_frames * sizeof(uvhttp_ws_frame_desc_t),
                          hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&s.h_sum, sizeof(uvhttp_ws_batch_summary_t), hipHostMallocDefault) !=
                hipSuccess ||
            hipMalloc((void**)&s.d_wire, slot_bytes + pad) != hipSuccess ||
            hipMalloc((void**)&s.d_off, (size_t)slot_frames * 8) != hipSuccess ||
            hipMalloc((void**)&s.d_desc, (size_t)slot_frames * sizeof(uvhttp_ws_frame_desc_t)) !=
                hipSuccess ||
            hipMalloc((void**)&s.d_sum, sizeof(uvhttp_ws_batch_summary_t)) != hipSuccess ||
            hipEventCreateWithFlags(&s.up_ev, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s.done_ev, hipEventDisableTiming) != hipSuccess)
            rc = UVHTTP_WS_GPU_ENOMEM;
    }
    (void)hipSetDevice(prev);
    if (rc) {
        uvhttp_ws_gpu_pipeline_free(p);
        return rc;
    }
    *out = p;
    return UVHTTP_WS_GPU_OK;
}

uint8_t* uvhttp_ws_gpu_pipeline_slot_buffer(uvhttp_ws_gpu_pipeline_t* p, int slot) {
    return (p && slot >= 0 && slot < p->depth) ? p->slots[slot].h_wire : nullptr;
}

uint64_t* uvhttp_ws_gpu_pipeline_slot_offsets(uvhttp_ws_gpu_pipeline_t* p, int slot) {
    return (p && slot >= 0 && slot < p->depth) ? p->slots[slot].h_off : nullptr;
}

int uvhttp_ws_gpu_pipeline_submit(uvhttp_ws_gpu_pipeline_t* p, int slot, uint64_t wire_len,
                                  int use_offsets, uint64_t stride, uint32_t n_frames,
                                  int32_t max_frame_size, int32_t max_message_size,
                                  int32_t is_server) {
    if (!p || slot < 0 || slot >= p->depth) return UVHTTP_WS_GPU_EINVAL;
    PipeSlot& s = p->slots[slot];
    if (s.busy || wire_len > p->slot_bytes || n_frames > p->slot_frames) return UVHTTP_WS_GPU_EINVAL;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(p->device);
    // upload stream: the slot's bytes (its previous round was waited for, so d_wire is free)
    hipError_t h = hipSuccess;
    // at most in_flight submissions queued: wait for the one in_flight submissions back (its
    // slot's latest done event; a slot cycled faster than that only waits longer)
    if (p->in_flight > 0 && p->in_flight < 16 && p->n_sub >= (uint64_t)p->in_flight)
        h = hipEventSynchronize(p->slots[p->recent[(p->n_sub - p->in_flight) % 16]].done_ev);
    if (h == hipSuccess && wire_len) h = hipMemcpyAsync(s.d_wire, s.h_wire, wire_len, hipMemcpyHostToDevice, p->up);
    if (h == hipSuccess && use_offsets && n_frames)
        h = hipMemcpyAsync(s.d_off, s.h_off, (size_t)n_frames * 8, hipMemcpyHostToDevice, p->up);
    if (h == hipSuccess) h = hipEventRecord(s.up_ev, p->up);
    // compute stream: decode once the upload landed, then the results come back
    if (h == hipSuccess) h = hipStreamWaitEvent(p->cs, s.up_ev, 0);
    int rc = h == hipSuccess ? UVHTTP_WS_GPU_OK : UVHTTP_WS_GPU_ELAUNCH;
    if (!rc) {
        uvhttp_ws_batch_t b;
        b.wire = s.d_wire;
        b.wire_len = wire_len;
        b.frame_off = use_offsets ? s.d_off : nullptr;
        b.frame_stride = stride;
        b.n_frames = n_frames;
        b.max_frame_size = max_frame_size;
        b.max_message_size = max_message_size;
        b.is_server = is_server;
        rc = uvhttp_ws_gpu_decode_inplace(p->eng, &b, s.d_desc, s.d_sum, p->cs);
    }
    if (!rc && wire_len) h = hipMemcpyAsync(s.h_wire, s.d_wire, wire_len, hipMemcpyDeviceToHost, p->cs);
    if (!rc && h == hipSuccess && n_frames)
        h = hipMemcpyAsync(s.h_desc, s.d_desc, (size_t)n_frames * sizeof(uvhttp_ws_frame_desc_t),
                           hipMemcpyDeviceToHost, p->cs);
    if (!rc && h == hipSuccess)
        h = hipMemcpyAsync(s.h_sum, s.d_sum, sizeof(uvhttp_ws_batch_summary_t), hipMemcpyDeviceToHost,
                           p->cs);
    if (!rc && h == hipSuccess) h = hipEventRecord(s.done_ev, p->cs);
    if (!rc && h != hipSuccess) rc = UVHTTP_WS_GPU_ELAUNCH;
    if (!rc) {
        s.busy = 1;
        s.compact = 0;
        p->recent[p->n_sub % 16] = slot;
        p->n_sub++;
    }
    (void)hipSetDevice(prev);
    return rc;
}

// Compact submission (include/uvhttp_ws_amd.h): H2D -> decode_compact -> D2H of the arena, the
// message table and the summary.  A stride batch of >= 140-byte frames decodes summary-only (the
// fast path: no descriptors) and only its last frame's slot comes back into the slot buffer
// (deliver_messages reads a control frame there); any other batch decodes into descriptors, and
// they and the wire (control payloads, unmasked in place) come back too.
int uvhttp_ws_gpu_pipeline_submit_compact(uvhttp_ws_gpu_pipeline_t* p, int slot, uint64_t wire_len,
                                          int use_offsets, uint64_t stride, uint32_t n_frames,
                                          int32_t max_frame_size, int32_t max_message_size,
                                          int32_t is_server) {
    if (!p || slot < 0 || slot >= p->depth) return UVHTTP_WS_GPU_EINVAL;
    PipeSlot& s = p->slots[slot];
    if (s.busy || wire_len > p->slot_bytes || n_frames > p->slot_frames) return UVHTTP_WS_GPU_EINVAL;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(p->device);
    hipError_t h = hipSuccess;
    const size_t arena_cap = (size_t)p->slot_bytes + 64;
    const size_t msg_bytes = (size_t)p->slot_frames * sizeof(uvhttp_ws_message_desc_t);
    if (!s.d_arena) {
        if (hipHostMalloc((void**)&s.h_arena, arena_cap, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&s.h_msgs, msg_bytes, hipHostMallocDefault) != hipSuccess ||
            hipMalloc((void**)&s.d_msgs, msg_bytes) != hipSuccess ||
            hipMalloc((void**)&s.d_arena, arena_cap) != hipSuccess) {
            if (s.h_arena) (void)hipHostFree(s.h_arena);
            if (s.h_msgs) (void)hipHostFree(s.h_msgs);
            if (s.d_msgs) (void)hipFree(s.d_msgs);
            s.h_arena = nullptr;
            s.h_msgs = nullptr;
            s.d_msgs = nullptr;
            s.d_arena = nullptr;
            (void)hipSetDevice(prev);
            return UVHTTP_WS_GPU_ENOMEM;
        }
    }
    if (p->in_flight > 0 && p->in_flight < 16 && p->n_sub >= (uint64_t)p->in_flight)
        h = hipEventSynchronize(p->slots[p->recent[(p->n_sub - p->in_flight) % 16]].done_ev);
    if (h == hipSuccess && wire_len) h = hipMemcpyAsync(s.d_wire, s.h_wire, wire_len, hipMemcpyHostToDevice, p->up);
    if (h == hipSuccess && use_offsets && n_frames)
        h = hipMemcpyAsync(s.d_off, s.h_off, (size_t)n_frames * 8, hipMemcpyHostToDevice, p->up);
    if (h == hipSuccess) h = hipEventRecord(s.up_ev, p->up);
    if (h == hipSuccess) h = hipStreamWaitEvent(p->cs, s.up_ev, 0);
    int rc = h == hipSuccess ? UVHTTP_WS_GPU_OK : UVHTTP_WS_GPU_ELAUNCH;
    const bool sum_only = !use_offsets && stride >= 140;
    if (!rc) {
        uvhttp_ws_batch_t b;
        b.wire = s.d_wire;
        b.wire_len = wire_len;
        b.frame_off = use_offsets ? s.d_off : nullptr;
        b.frame_stride = stride;
        b.n_frames = n_frames;
        b.max_frame_size = max_frame_size;
        b.max_message_size = max_message_size;
        b.is_server = is_server;
        rc = uvhttp_ws_gpu_decode_compact(p->eng, &b, s.d_arena, arena_cap, sum_only ? nullptr : s.d_desc,
                                          s.d_msgs, s.d_sum, p->cs);
    }
    // the arena holds at most the wire's bytes; the table n_frames entries (the open one included)
    if (!rc && wire_len) h = hipMemcpyAsync(s.h_arena, s.d_arena, wire_len, hipMemcpyDeviceToHost, p->cs);
    if (!rc && h == hipSuccess && n_frames)
        h = hipMemcpyAsync(s.h_msgs, s.d_msgs, (size_t)n_frames * sizeof(uvhttp_ws_message_desc_t),
                           hipMemcpyDeviceToHost, p->cs);
    if (!rc && h == hipSuccess && n_frames) {
        if (sum_only) {  // the last frame's slot (a control frame there is read from it)
            const uint64_t at = (uint64_t)(n_frames - 1) * stride;
            if (at < wire_len)
                h = hipMemcpyAsync(s.h_wire + at, s.d_wire + at, wire_len - at, hipMemcpyDeviceToHost, p->cs);
        } else {
            h = hipMemcpyAsync(s.h_desc, s.d_desc, (size_t)n_frames * sizeof(uvhttp_ws_frame_desc_t),
                               hipMemcpyDeviceToHost, p->cs);
            if (h == hipSuccess && wire_len)
                h = hipMemcpyAsync(s.h_wire, s.d_wire, wire_len, hipMemcpyDeviceToHost, p->cs);
        }
    }
    if (!rc && h == hipSuccess)
        h = hipMemcpyAsync(s.h_sum, s.d_sum, sizeof(uvhttp_ws_batch_summary_t), hipMemcpyDeviceToHost, p->cs);
    if (!rc && h == hipSuccess) h = hipEventRecord(s.done_ev, p->cs);
    if (!rc && h != hipSuccess) rc = UVHTTP_WS_GPU_ELAUNCH;
    if (!rc) {
        s.busy = 1;
        s.compact = 1;
        s.with_desc = sum_only ? 0 : 1;
        p->recent[p->n_sub % 16] = slot;
        p->n_sub++;
    }
    (void)hipSetDevice(prev);
    return rc;
}

int uvhttp_ws_gpu_pipeline_wait_compact(uvhttp_ws_gpu_pipeline_t* p, int slot, const uint8_t** arena,
                                        const uvhttp_ws_message_desc_t** msgs,
                                        const uvhttp_ws_frame_desc_t** desc,
                                        const uvhttp_ws_batch_summary_t** summary) {
    if (!p || slot < 0 || slot >= p->depth) return UVHTTP_WS_GPU_EINVAL;
    PipeSlot& s = p->slots[slot];
    if (!s.busy || !s.compact) return UVHTTP_WS_GPU_EINVAL;
    const hipError_t h = hipEventSynchronize(s.done_ev);
    s.busy = 0;
    if (arena) *arena = s.h_arena;
    if (msgs) *msgs = s.h_msgs;
    if (desc) *desc = s.with_desc ? s.h_desc : nullptr;
    if (summary) *summary = s.h_sum;
    return h == hipSuccess ? UVHTTP_WS_GPU_OK : UVHTTP_WS_GPU_ELAUNCH;
}

int uvhttp_ws_gpu_pipeline_wait(uvhttp_ws_gpu_pipeline_t* p, int slot,
                                const uvhttp_ws_frame_desc_t** desc,
                                const uvhttp_ws_batch_summary_t** summary) {
    if (!p || slot < 0 || slot >= p->depth) return UVHTTP_WS_GPU_EINVAL;
    PipeSlot& s = p->slots[slot];
    if (!s.busy || s.compact) return UVHTTP_WS_GPU_EINVAL;
    const hipError_t h = hipEventSynchronize(s.done_ev);
    s.busy = 0;
    if (desc) *desc = s.h_desc;
    if (summary) *summary = s.h_sum;
    return h == hipSuccess ? UVHTTP_WS_GPU_OK : UVHTTP_WS_GPU_ELAUNCH;
}

}  // extern "C"
