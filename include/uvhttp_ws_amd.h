/*
 * uvhttp_ws_amd.h — C ABI of the MI355X-native WebSocket frame-decode / unmask path.
 *
 * Two surfaces live here:
 *
 *  1. The DROP-IN decode surface of the reference header include/uvhttp_websocket.h
 *     (adam-ikari/uvhttp v2.7.0).  Same symbol names, same argument meaning, same
 *     struct layouts (x86-64: uvhttp_ws_frame_header_t 16 B, uvhttp_ws_frame_t 48 B,
 *     uvhttp_ws_connection_t 248 B), same error convention (UVHTTP_OK = 0, every decode
 *     failure UVHTTP_ERROR_INVALID_PARAM = -1).  When the reference header has already
 *     been included (UVHTTP_WEBSOCKET_H defined) its own type definitions are used and
 *     only the function prototypes below are re-stated.
 *
 *  2. The BATCHED DEVICE surface (new): many masked frames resident in MI355X HBM are
 *     header-parsed, validated, fragment-checked and unmasked by hand-written gfx950
 *     kernels.  Plain pointers and sizes only; the stream is an opaque hipStream_t.
 *     These entry points never compute on the CPU: with no usable GPU they return
 *     UVHTTP_WS_GPU_ENODEV.
 *
 * Batch semantics (the parity contract, checked against the oracle in tests/):
 *   a batch of n frames laid out back to back is decoded exactly as the reference's
 *   uvhttp_ws_process_data (src/uvhttp_websocket.c:825-1097) decodes the same bytes when
 *   it is called once per frame with exactly that frame's wire bytes on a fresh server
 *   connection with the given limits: frames before the first failing frame are
 *   delivered (unmasked), the first failing frame and everything after it are left
 *   untouched, and the failure reason is reported per frame.
 */
#ifndef UVHTTP_WS_AMD_H
#define UVHTTP_WS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------ */
/* 1. Drop-in types (ABI-identical to the reference; only when its header is absent)    */
/* ------------------------------------------------------------------------------------ */
#ifndef UVHTTP_WEBSOCKET_H

#ifndef UVHTTP_ERROR_H
/* include/uvhttp_error.h:16-20 — only the two codes the decode path returns. */
typedef int uvhttp_error_t;
#define UVHTTP_OK 0
#define UVHTTP_ERROR_INVALID_PARAM (-1)
#endif

#ifndef UVHTTP_CONFIG_H
/* include/uvhttp_config.h — full layout kept so uvhttp_ws_connection_create can read
 * websocket_* at the reference offsets (64..79). */
typedef struct {
    int max_connections;
    int read_buffer_size;
    int backlog;
    int keepalive_timeout;
    int request_timeout;
    int connection_timeout;
    size_t max_body_size;
    size_t max_header_size;
    size_t max_url_size;
    size_t max_file_size;
    int max_requests_per_connection;
    int rate_limit_window;
    int websocket_max_frame_size;
    int websocket_max_message_size;
    int websocket_ping_interval;
    int websocket_ping_timeout;
    int tcp_keepalive_timeout;
    int sendfile_timeout_ms;
    int sendfile_max_retry;
    int cache_default_max_entries;
    int cache_default_ttl;
    int lru_cache_batch_eviction_size;
    int rate_limit_max_requests;
    int rate_limit_max_window_seconds;
    int rate_limit_min_timeout_seconds;
} uvhttp_config_t;
#endif

/* mbedtls is never touched on the decode path; the pointer is carried opaquely. */
typedef struct mbedtls_ssl_context mbedtls_ssl_context;

/* include/uvhttp_websocket.h:24-31 */
typedef enum {
    UVHTTP_WS_OPCODE_CONTINUATION = 0x0,
    UVHTTP_WS_OPCODE_TEXT = 0x1,
    UVHTTP_WS_OPCODE_BINARY = 0x2,
    UVHTTP_WS_OPCODE_CLOSE = 0x8,
    UVHTTP_WS_OPCODE_PING = 0x9,
    UVHTTP_WS_OPCODE_PONG = 0xA
} uvhttp_ws_opcode_t;

/* include/uvhttp_websocket.h:34-39 */
typedef enum {
    UVHTTP_WS_STATE_CONNECTING = 0,
    UVHTTP_WS_STATE_OPEN = 1,
    UVHTTP_WS_STATE_CLOSING = 2,
    UVHTTP_WS_STATE_CLOSED = 3
} uvhttp_ws_state_t;

/* include/uvhttp_websocket.h:42-51 — 16 bytes, payload_length at offset 8. */
typedef struct {
    uint8_t fin : 1;
    uint8_t rsv1 : 1;
    uint8_t rsv2 : 1;
    uint8_t rsv3 : 1;
    uint8_t opcode : 4;
    uint8_t mask : 1;
    uint8_t payload_len : 7;  /* raw 7-bit length code (0..127) */
    uint64_t payload_length;  /* decoded length */
} uvhttp_ws_frame_header_t;

/* include/uvhttp_websocket.h:54-60 — 48 bytes. */
typedef struct {
    uvhttp_ws_frame_header_t header;
    uint64_t payload_length;
    uint8_t masking_key[4];
    uint8_t* payload;
    size_t payload_size;
} uvhttp_ws_frame_t;

/* include/uvhttp_websocket.h:63-69 */
typedef struct {
    int max_frame_size;
    int max_message_size;
    int ping_interval;
    int ping_timeout;
    int enable_compression;
} uvhttp_ws_config_t;

struct uvhttp_ws_connection;

/* include/uvhttp_websocket.h:75-82 */
typedef int (*uvhttp_ws_on_message_callback)(struct uvhttp_ws_connection* conn,
                                             const char* data, size_t len, int opcode);
typedef int (*uvhttp_ws_on_close_callback)(struct uvhttp_ws_connection* conn, int code,
                                           const char* reason);
typedef int (*uvhttp_ws_on_error_callback)(struct uvhttp_ws_connection* conn,
                                           int error_code, const char* error_msg);

/* include/uvhttp_websocket.h:85-121 — 248 bytes. */
typedef struct uvhttp_ws_connection {
    int fd;
    uvhttp_ws_state_t state;
    uvhttp_ws_config_t config;
    mbedtls_ssl_context* ssl;
    int is_server;
    char client_key[64];
    uint8_t* recv_buffer;
    size_t recv_buffer_size;
    size_t recv_buffer_pos;
    uint8_t* send_buffer;
    size_t send_buffer_size;
    uint8_t* fragmented_message;
    size_t fragmented_size;
    size_t fragmented_capacity;
    uvhttp_ws_opcode_t fragmented_opcode;
    uvhttp_ws_on_message_callback on_message;
    uvhttp_ws_on_close_callback on_close;
    uvhttp_ws_on_error_callback on_error;
    void* user_data;
    uint64_t bytes_sent;
    uint64_t bytes_received;
    uint64_t frames_sent;
    uint64_t frames_received;
} uvhttp_ws_connection_t;

#endif /* !UVHTTP_WEBSOCKET_H */

/* Reference defaults (include/uvhttp_defaults.h:171-207). */
#define UVHTTP_WS_AMD_DEFAULT_MAX_FRAME_SIZE (16 * 1024 * 1024)
#define UVHTTP_WS_AMD_DEFAULT_MAX_MESSAGE_SIZE (64 * 1024 * 1024)
#define UVHTTP_WS_AMD_DEFAULT_RECV_BUFFER_SIZE (64 * 1024)
#define UVHTTP_WS_AMD_DEFAULT_PING_INTERVAL 30
#define UVHTTP_WS_AMD_DEFAULT_PING_TIMEOUT 10

/* ------------------------------------------------------------------------------------ */
/* 1b. Drop-in decode functions (replace the reference symbols of the same name)        */
/* ------------------------------------------------------------------------------------ */

/* replaces src/uvhttp_websocket.c:71-109 (decl include/uvhttp_websocket.h:128-130) */
struct uvhttp_ws_connection* uvhttp_ws_connection_create(int fd, mbedtls_ssl_context* ssl,
                                                         int is_server,
                                                         const uvhttp_config_t* config);
/* replaces src/uvhttp_websocket.c:112-130 (decl include/uvhttp_websocket.h:135) */
void uvhttp_ws_connection_free(struct uvhttp_ws_connection* conn);
/* replaces src/uvhttp_websocket.c:1100-1111 (decl include/uvhttp_websocket.h:217-220) */
void uvhttp_ws_set_callbacks(struct uvhttp_ws_connection* conn,
                             uvhttp_ws_on_message_callback on_message,
                             uvhttp_ws_on_close_callback on_close,
                             uvhttp_ws_on_error_callback on_error);
/* replaces src/uvhttp_websocket.c:133-185 (decl include/uvhttp_websocket.h:228-230) */
uvhttp_error_t uvhttp_ws_parse_frame_header(const uint8_t* data, size_t len,
                                            uvhttp_ws_frame_header_t* header,
                                            size_t* header_size);
/* replaces src/uvhttp_websocket.c:188-197 (decl include/uvhttp_websocket.h:250-251) */
void uvhttp_ws_apply_mask(uint8_t* data, size_t len, const uint8_t* masking_key);
/* replaces src/uvhttp_websocket.c:825-1097 (decl include/uvhttp_websocket.h:212-213) */
uvhttp_error_t uvhttp_ws_process_data(struct uvhttp_ws_connection* conn, const uint8_t* data,
                                      size_t len);

/* Control-frame hooks (new).  The reference answers PING with uvhttp_ws_send_pong and
 * echoes CLOSE with uvhttp_ws_send_frame through the server context reached from the
 * wrapper in conn->user_data (src/uvhttp_websocket.c:1028-1084); for CLOSE it captures that
 * context BEFORE calling on_close (which frees the wrapper) and sends AFTER.  The send side
 * lives outside this library, so the integration layer registers:
 *   resolver(conn) -> the server context (wrapper->conn->server->context) or NULL; called
 *                     only when conn->user_data != NULL, at the point the reference reads it;
 *   sink(ctx, conn, opcode, payload, len) -> send; called only with a non-NULL ctx.
 * opcode is UVHTTP_WS_OPCODE_PONG (payload = the ping payload) or UVHTTP_WS_OPCODE_CLOSE
 * (payload = code + reason truncated to 125 B, empty when the close had < 2 bytes). */
typedef void* (*uvhttp_ws_amd_context_resolver)(struct uvhttp_ws_connection* conn);
typedef void (*uvhttp_ws_amd_control_sink)(void* ctx, struct uvhttp_ws_connection* conn,
                                           int opcode, const uint8_t* payload, size_t len);
void uvhttp_ws_amd_set_control_hooks(uvhttp_ws_amd_context_resolver resolver,
                                     uvhttp_ws_amd_control_sink sink);

/* ------------------------------------------------------------------------------------ */
/* 2. Batched device surface (MI355X / gfx950)                                          */
/* ------------------------------------------------------------------------------------ */

/* Return codes of the device surface (0 = OK; negative = failure, nothing launched). */
#define UVHTTP_WS_GPU_OK 0
#define UVHTTP_WS_GPU_EINVAL (-1)  /* bad argument (NULL, misaligned, sizes) */
#define UVHTTP_WS_GPU_ENODEV (-2)  /* no usable MI355X / HIP runtime error at setup */
#define UVHTTP_WS_GPU_ENOMEM (-3)  /* device workspace allocation failed */
#define UVHTTP_WS_GPU_ELAUNCH (-4) /* kernel launch / HIP call failed */

/* Per-frame status (uvhttp_ws_frame_desc_t.status).  Negative values are the reasons
 * uvhttp_ws_process_data returns UVHTTP_ERROR_INVALID_PARAM, with the reference check
 * that raises each one. */
#define UVHTTP_WS_FRAME_OK 0
#define UVHTTP_WS_FRAME_INCOMPLETE 1        /* last frame not fully present (need more data, :925-932) */
#define UVHTTP_WS_FRAME_SKIPPED 2           /* after the first failing frame: not processed */
#define UVHTTP_WS_FRAME_ERR_PARSE (-1)      /* 64-bit length with MSB set (:178-180) */
#define UVHTTP_WS_FRAME_ERR_RSV (-2)        /* RSV1-3 set (:895-897) */
#define UVHTTP_WS_FRAME_ERR_CONTROL (-3)    /* control frame > 125 B or FIN=0 (:902-906) */
#define UVHTTP_WS_FRAME_ERR_UNMASKED (-4)   /* server got an unmasked frame (:910-912) */
#define UVHTTP_WS_FRAME_ERR_TOO_BIG (-5)    /* payload > max_frame_size (:919-921) */
#define UVHTTP_WS_FRAME_ERR_BUFFER (-6)     /* wire bytes exceed recv-buffer cap (:851-857) */
#define UVHTTP_WS_FRAME_ERR_FRAGMENT (-7)   /* CONT with no start / data inside fragment (:964-996) */
#define UVHTTP_WS_FRAME_ERR_MESSAGE (-8)    /* fragments exceed max_message_size (:786-791) */
#define UVHTTP_WS_FRAME_ERR_LAYOUT (-9)     /* offset table disagrees with the frame lengths */
#define UVHTTP_WS_FRAME_ERR_CAPACITY (-10)  /* stream decode: more frames than the desc array holds */
#define UVHTTP_WS_FRAME_ERR_DEVICE (-11)    /* the device could not complete the call (a bounded
                                               wait in the single-pass scan gave up): nothing was
                                               decoded; uvhttp_ws_gpu_engine_sync reports ELAUNCH */

/* Frame flags (uvhttp_ws_frame_desc_t.flags). */
#define UVHTTP_WS_FLAG_FIN 0x01u
#define UVHTTP_WS_FLAG_MASK 0x02u
#define UVHTTP_WS_FLAG_RSV1 0x04u
#define UVHTTP_WS_FLAG_RSV2 0x08u
#define UVHTTP_WS_FLAG_RSV3 0x10u
#define UVHTTP_WS_FLAG_MSG_END 0x20u  /* this frame completes a data message (on_message fires) */

/* One decoded frame (device-written, 32 bytes). */
typedef struct {
    uint64_t payload_off;  /* byte offset of the unmasked payload: in the wire buffer
                              (in-place decode, and control frames of a compact decode)
                              or in the message arena (data frames of a compact decode) */
    uint64_t payload_len;  /* header.payload_length */
    uint32_t masking_key;  /* key bytes k0..k3 as a little-endian word (k0 = low byte) */
    uint32_t message;      /* index of the message this data frame belongs to (compact) */
    uint8_t opcode;        /* header.opcode */
    uint8_t flags;         /* UVHTTP_WS_FLAG_* */
    uint8_t header_size;   /* 2 / 4 / 10 (mask key excluded, as parse_frame_header) */
    int8_t status;         /* UVHTTP_WS_FRAME_* */
    uint32_t wire_len;     /* header + key + payload bytes (saturated at 2^32-1) */
} uvhttp_ws_frame_desc_t;

/* One complete data message (compact decode only, 32 bytes).  The payload handed to
 * on_message is arena[arena_off, arena_off + len); the opcode is the first frame's.  When the
 * summary reports pending_bytes != 0, entry [n_messages] describes the message still open
 * after the last delivered frame (its bytes so far, last_frame = the latest fragment) and
 * `reserved` holds its first fragment's payload length; otherwise reserved is 0. */
typedef struct {
    uint64_t arena_off;
    uint64_t len;
    uint32_t first_frame;
    uint32_t last_frame;
    int32_t opcode;
    uint32_t reserved;
} uvhttp_ws_message_desc_t;

/* Batch summary (device-written; copy back after the stream completes). */
typedef struct {
    uint32_t n_frames;        /* frames in the batch */
    uint32_t n_delivered;     /* frames processed before the first failing frame */
    int32_t status;           /* UVHTTP_OK, or UVHTTP_ERROR_INVALID_PARAM on a failing frame */
    int32_t first_status;     /* status of frame n_delivered (0 if all delivered) */
    uint64_t consumed_bytes;  /* wire bytes of the delivered frames (recv-buffer drain) */
    uint64_t payload_bytes;   /* sum of delivered payload bytes */
    uint32_t n_messages;      /* complete data messages among the delivered frames */
    uint32_t state_closed;    /* 1 if a delivered CLOSE frame set state = CLOSED */
    uint64_t arena_bytes;     /* compact: arena bytes written */
    uint64_t pending_bytes;   /* bytes of a fragmented message still open at the end */
} uvhttp_ws_batch_summary_t;

/* A batch of frames resident in device memory. */
typedef struct {
    uint8_t* wire;             /* device pointer, 16-byte aligned; frames back to back */
    uint64_t wire_len;         /* bytes readable at wire */
    const uint64_t* frame_off; /* device pointer: n_frames start offsets, or NULL */
    uint64_t frame_stride;     /* when frame_off == NULL: frame i starts at i*stride */
    uint32_t n_frames;
    int32_t max_frame_size;    /* uvhttp_ws_config_t.max_frame_size */
    int32_t max_message_size;  /* uvhttp_ws_config_t.max_message_size */
    int32_t is_server;         /* 1: unmasked frames are rejected (reference server) */
} uvhttp_ws_batch_t;

typedef struct uvhttp_ws_gpu_engine uvhttp_ws_gpu_engine_t;

/* Create an engine bound to HIP device `device` (owns the scratch workspace). */
int uvhttp_ws_gpu_engine_create(int device, uvhttp_ws_gpu_engine_t** out);
void uvhttp_ws_gpu_engine_free(uvhttp_ws_gpu_engine_t* eng);
/* Pre-size the workspace so later decode calls never allocate (hipGraph capture). */
int uvhttp_ws_gpu_engine_reserve(uvhttp_ws_gpu_engine_t* eng, uint32_t max_frames,
                                 uint64_t max_wire_bytes, uint64_t max_arena_bytes);
/* Payload-kernel workgroup shape: `block` threads x `vectors_per_lane` 16-byte vectors per
 * workgroup tile; (0, 0) = automatic (by average frame size).  Supported: 64x1, 64x2, 64x4,
 * 128x1, 128x2, 256x1, 256x2, 256x4.  A tuning knob only: results are identical. */
int uvhttp_ws_gpu_engine_set_tile(uvhttp_ws_gpu_engine_t* eng, int block, int vectors_per_lane);
/* Kernel timing: with enable = k >= 1, HIP events bracket the dominant (payload) kernel of
 * every k-th call (k = 1: every call) on its stream — each timed marker idles the device a few
 * microseconds, so sampling keeps that cost off most calls; 0 disables.  kernel_time returns
 * the summed milliseconds and the number of bracketed launches completed so far
 * (synchronises on the last event). */
int uvhttp_ws_gpu_engine_set_timing(uvhttp_ws_gpu_engine_t* eng, int enable);
int uvhttp_ws_gpu_engine_kernel_time(uvhttp_ws_gpu_engine_t* eng, double* ms,
                                     uint64_t* launches);
const char* uvhttp_ws_gpu_engine_last_error(const uvhttp_ws_gpu_engine_t* eng);
/* Wait for `stream` and report device-side failures of the calls made since the previous
 * sync: UVHTTP_WS_GPU_ELAUNCH if any of them flagged UVHTTP_WS_FRAME_ERR_DEVICE (their
 * summaries / results say so too, and nothing of them was unmasked), else OK. */
int uvhttp_ws_gpu_engine_sync(uvhttp_ws_gpu_engine_t* eng, void* stream);

/* Device-side kernel stamps (diagnostics).  With stamps on, every kernel of a decode call
 * records on the GPU's constant wall clock when its first workgroups started and when its
 * last wave ended, so the time between the kernels of a call — and between one call's last
 * kernel and the next call's first — is read off the device timeline rather than inferred
 * from host events.  The engine keeps the last 128 calls (71 MB of device memory, allocated
 * when stamps are first turned on); read_stamps returns one record per (call, kernel) it holds,
 * in call then start order, and clears them.  While on, each kernel's first 256 workgroups and
 * a sample of its waves store a word each (plain stores; C3 0.2 %, C4 1 % slower); off (the
 * default) it costs one untaken branch per kernel.  Calls made while their stream is captured
 * are not stamped.  The payload kernel of a compact decode of large frames (k_gather_compact)
 * is not stamped. */
#define UVHTTP_WS_STAMP_WALK 0        /* k_swalk_lane / k_swalk_wave (frame discovery) */
#define UVHTTP_WS_STAMP_WALK_SCAN 1   /* k_swalk_scan (first frame per connection) */
#define UVHTTP_WS_STAMP_WALK2 2       /* second walk (two-pass mode) */
#define UVHTTP_WS_STAMP_STREAM_DESC 3 /* k_stream_desc / k_stream_desc_lane */
#define UVHTTP_WS_STAMP_CLAIMS 4      /* (k_stream_claims until round 5: unused) */
#define UVHTTP_WS_STAMP_PAYLOAD 5     /* the payload kernel (unmask / scatter / gather) */
#define UVHTTP_WS_STAMP_PLAN 6        /* k_plan */
#define UVHTTP_WS_STAMP_FIXUP 7       /* k_fixup (fused stride path) */
#define UVHTTP_WS_STAMP_FINALIZE 8    /* k_finalize; summary-only compact: k_sum_msgs */
#define UVHTTP_WS_STAMP_BUILD_SIZE 9  /* send side: kb_size (the emit kernels stamp as PAYLOAD) */
#define UVHTTP_WS_STAMP_BUILD_SCAN 10 /* kb_scan_one / kb_scan_groups */
#define UVHTTP_WS_STAMP_BUILD_SCAN2 11 /* kb_scan_top */
#define UVHTTP_WS_STAMP_BUILD_OFFSETS 12 /* kb_offsets (tile emit only) */
#define UVHTTP_WS_STAMP_DESC_EMIT 13  /* k_desc_emit (stride batches with descriptors) */
#define UVHTTP_WS_STAMP_SUM_SCAN 14   /* k_sum_scan ahead of k_desc_emit (the summary-only
                                         decodes' k_sum_scan stamps as PLAN) */
#define UVHTTP_WS_STAMP_SPEC_PLAN 15  /* k_sspec_plan (speculative stream decode; its pass
                                         stamps as PAYLOAD, k_sspec_emit as STREAM_DESC) */
typedef struct {
    uint32_t call;      /* the call's tag: 1 .. 2^24 - 1, one more per decode call (after
                           2^24 - 1 wraps to 1); records come oldest call first */
    uint32_t kernel;    /* UVHTTP_WS_STAMP_* */
    uint64_t begin_ns;  /* device wall clock, ns: earliest sampled workgroup start */
    uint64_t end_ns;    /* latest wave end */
} uvhttp_ws_gpu_stamp_t;
int uvhttp_ws_gpu_engine_set_stamps(uvhttp_ws_gpu_engine_t* eng, int enable);
/* Waits for the device; *n_out = records written (at most cap).  A pass launched as several
 * dispatch pieces (over 2^24 workgroups, e.g. a C5 pass) reads as one record spanning all of
 * them: begin = the first piece's start, end = the latest wave end of any piece. */
int uvhttp_ws_gpu_engine_read_stamps(uvhttp_ws_gpu_engine_t* eng, uvhttp_ws_gpu_stamp_t* out,
                                     uint32_t cap, uint32_t* n_out);
/* Host-only pieces of the stamp ring (no device needed; tests drive them):
 * ring_words = the ring's size in 64-bit words; stamps_reduce = read_stamps's reduction of a
 * ring copy (epoch = the engine's latest call, khz = wall-clock rate); stamp_simulate writes
 * what one launch piece of `blocks` workgroups starting at pass index `base` stores, with the
 * kernels' own slot mapping (workgroup i starts at t_begin + i (t_end - t_begin) / blocks and
 * ends dur ticks later). */
uint64_t uvhttp_ws_gpu_stamp_ring_words(void);
int uvhttp_ws_gpu_stamps_reduce(const uint64_t* ring, uint32_t epoch, uint32_t khz,
                                uvhttp_ws_gpu_stamp_t* out, uint32_t cap, uint32_t* n_out);
int uvhttp_ws_gpu_stamp_simulate(uint64_t* ring, uint32_t epoch, uint32_t kind, uint64_t base,
                                 uint32_t blocks, uint32_t waves, uint64_t t_begin, uint64_t t_end,
                                 uint64_t dur);

/* Streams and graphs.  An engine owns one workspace, so its calls must execute one after
 * another: when a call names a different stream than the previous call, the engine makes the
 * new stream wait for the work already queued on the old one (an event), so calls from
 * several streams serialise on the device instead of corrupting each other.  For concurrency
 * use one engine per stream (the pipelines do).
 * A call made while its stream is being captured (hipStreamBeginCapture) is graph-safe: its
 * kernels take their epoch tag from device memory, bumped by a small kernel at the start of
 * every replay, so replays of the same graph over changing frame bytes never accept tags a
 * previous replay left behind.  Reserve the workspace before capturing (engine_reserve;
 * stream decode: one uncaptured call of the same or larger shape) — a captured call that
 * would allocate fails with EINVAL.  Kernel timing is not recorded inside a capture. */

/* In-place decode: parse + validate every frame, run the fragment state machine, then
 * unmask the payload of every delivered frame in place in batch->wire (the reference
 * unmasks inside recv_buffer, src/uvhttp_websocket.c:937-947).  d_desc (n_frames
 * entries) and d_summary are device pointers.  Asynchronous on `stream`.
 * d_desc may be NULL (summary-only decode): the wire and d_summary come out exactly as with
 * descriptors, and no per-frame output is written.  A fixed-stride batch of small frames
 * (stride >= 140 bytes, every frame able to fit the message limit) then runs as one payload
 * pass writing an info byte per frame plus two short kernels (fragment state machine and
 * summary; after a failure the frames from it on are masked again); any other batch is decoded
 * into descriptors in engine scratch (grown on demand, so reserve or run one uncaptured call
 * of the shape before capturing a graph).  For a caller that only needs "every frame delivered"
 * or the first failure, e.g. a server that re-walks delivered frames on the host. */
int uvhttp_ws_gpu_decode_inplace(uvhttp_ws_gpu_engine_t* eng, const uvhttp_ws_batch_t* batch,
                                 uvhttp_ws_frame_desc_t* d_desc,
                                 uvhttp_ws_batch_summary_t* d_summary, void* stream);

/* Compact decode: as above, but data-frame payloads are unmasked out of place into
 * d_arena at the exclusive prefix sum of data payload lengths, so every message —
 * including a fragmented one (uvhttp_ws_fragment_append, :781-822) — is one contiguous
 * arena range described by d_msgs.  Control-frame payloads are unmasked in place in the
 * wire.  d_msgs needs room for n_frames entries; arena_cap must cover the data payload.
 * Arena bytes past summary->arena_bytes (up to arena_cap) are scratch: a fixed-stride batch is
 * decoded speculatively, and when it fails part-way the payloads of frames after the failure
 * may have been written there.  d_desc may be NULL (descriptors then go to engine scratch;
 * the arena, d_msgs and d_summary are the same). */
int uvhttp_ws_gpu_decode_compact(uvhttp_ws_gpu_engine_t* eng, const uvhttp_ws_batch_t* batch,
                                 uint8_t* d_arena, uint64_t arena_cap,
                                 uvhttp_ws_frame_desc_t* d_desc,
                                 uvhttp_ws_message_desc_t* d_msgs,
                                 uvhttp_ws_batch_summary_t* d_summary, void* stream);

/* Unmask only (no framing): data[i] ^= key[i % 4] for a device buffer — the batched form
 * of uvhttp_ws_apply_mask for callers that parsed headers themselves. */
int uvhttp_ws_gpu_apply_mask(uvhttp_ws_gpu_engine_t* eng, uint8_t* d_data, uint64_t len,
                             const uint8_t masking_key[4], void* stream);

/* Synthetic masked-frame generator (bench / parity inputs; not on the decode path).
 * Writes n_frames frames of payload_len bytes back to back at d_wire (stride =
 * header + 4 + payload_len).  Frame i: opcode = (i == 0 || !fragmented) ? opcode0 :
 * CONTINUATION; FIN = !fragmented || i == n_frames - 1; key = splitmix64(seed ^ i)
 * low 32 bits (frames 0 and 1 forced to 0x00000000 / 0xFFFFFFFF when force_keys);
 * plaintext byte b = byte (b & 7) of splitmix64(seed + ((uint64)i << 32) + (b >> 3)).
 * Same definition as oracle/ws_oracle.c:oracle_gen_frames. */
uint64_t uvhttp_ws_gen_frame_stride(uint64_t payload_len);
int uvhttp_ws_gpu_gen_frames(uvhttp_ws_gpu_engine_t* eng, uint8_t* d_wire, uint32_t n_frames,
                             uint64_t payload_len, uint64_t seed, int opcode0, int fragmented,
                             int force_keys, void* stream);
/* Frames [first, first + count) of that n_frames batch, written from d_wire on (the bench's
 * ranks: rank r's shard is frames [first, ...) of the whole configuration, as
 * oracle_gen_frames(first, count, n_frames) writes them). */
int uvhttp_ws_gpu_gen_frames_range(uvhttp_ws_gpu_engine_t* eng, uint8_t* d_wire, uint32_t first,
                                   uint32_t count, uint32_t n_frames, uint64_t payload_len,
                                   uint64_t seed, int opcode0, int fragmented, int force_keys,
                                   void* stream);

/* ---- batched stateful stream decode (many connections per launch) --------------------- */
/* One entry per connection: the bytes uvhttp_ws_process_data would hold after appending the
 * new reads (recv_buffer[0, recv_buffer_pos) followed by the reads), placed at wire[begin,
 * begin + len), plus the connection state the decoder reads.  Streams must be ordered by
 * `begin` and must not overlap.  Frame boundaries are found on the device (one lane or wave
 * walks each connection's headers), so no offset table is needed.
 *
 * Reads.  n_reads == 0: the bytes are ONE process_data call.  n_reads > 0: they are n_reads
 * consecutive calls, read k ending at stream offset read_end[first_read + k] (relative to
 * begin; non-decreasing; the last equals len; the buffered prefix belongs to call 0).  The
 * device applies process_data's per-call rules exactly as the reference meets them when
 * on_websocket_read feeds one libuv read or one mbedtls_ssl_read chunk per call
 * (src/uvhttp_connection.c:1128-1164): the recv-buffer growth and its max_frame_size cap at
 * the start of every call (src/uvhttp_websocket.c:832-857), a frame is delivered by the call
 * that completes it, a frame whose header fails a check fails the call in which its header
 * bytes arrive, and the calls after a failing call never run (the caller closes). */
typedef struct {
    uint64_t begin;             /* offset of the connection's bytes in the batch wire */
    uint64_t len;               /* recv_buffer_pos + new bytes */
    uint64_t recv_buffer_size;  /* conn->recv_buffer_size before the first call */
    uint64_t pending_bytes;     /* conn->fragmented_size if conn->fragmented_message, else 0 */
    int32_t pending_opcode;     /* conn->fragmented_opcode */
    int32_t max_frame_size;     /* conn->config.max_frame_size */
    int32_t max_message_size;   /* conn->config.max_message_size */
    int32_t is_server;          /* conn->is_server */
    uint32_t first_read;        /* this connection's reads: read_end[first_read, +n_reads) */
    uint32_t n_reads;           /* 0 = one call with all len bytes */
    uint64_t reserved;
} uvhttp_ws_stream_t;           /* 64 bytes */

/* Per-connection outcome: exactly what the process_data calls return and leave behind
 * (src/uvhttp_websocket.c:825-1097). */
typedef struct {
    uint32_t first_frame;        /* this connection's frames start at desc[first_frame] */
    uint32_t n_frames;           /* frames found: delivered + (if it failed) the failing one */
    uint32_t n_delivered;
    int32_t status;              /* the last call's return: UVHTTP_OK or ..._INVALID_PARAM */
    int32_t first_status;        /* UVHTTP_WS_FRAME_* of the failure (0 if none) */
    uint32_t calls;              /* process_data calls that ran (a failing call included) */
    uint64_t consumed_bytes;     /* complete frames drained from the front of the stream */
    uint64_t recv_buffer_size;   /* after the last call that ran (the buffer may have grown) */
    uint64_t pending_bytes;      /* open fragmented message after the calls (0 = none) */
    uint64_t buffered_end;       /* stream bytes [consumed_bytes, buffered_end) are what
                                    recv_buffer holds afterwards (0 when the first call failed
                                    its growth check: recv_buffer is then untouched) */
    uint64_t reserved;
} uvhttp_ws_stream_result_t;     /* 64 bytes */

/* Decode every connection's frames in one set of launches, in place (delivered payloads
 * unmasked inside wire).  d_desc has room for max_frames; if the streams hold more frames
 * every result reports UVHTTP_WS_FRAME_ERR_CAPACITY and nothing is unmasked. */
int uvhttp_ws_gpu_decode_streams(uvhttp_ws_gpu_engine_t* eng, uint8_t* d_wire, uint64_t wire_len,
                                 const uvhttp_ws_stream_t* d_streams, uint32_t n_streams,
                                 uint32_t max_frames, uvhttp_ws_frame_desc_t* d_desc,
                                 uvhttp_ws_stream_result_t* d_results, void* stream);
/* As decode_streams, with several process_data calls per connection: d_read_end (device,
 * n_reads_total entries) holds the read boundaries the streams' first_read / n_reads index.
 * A connection whose read table is malformed (out of range, decreasing, last != len) reports
 * UVHTTP_WS_FRAME_ERR_LAYOUT and is not decoded.  decode_streams == decode_reads with no
 * read table (every stream must then have n_reads == 0). */
int uvhttp_ws_gpu_decode_reads(uvhttp_ws_gpu_engine_t* eng, uint8_t* d_wire, uint64_t wire_len,
                               const uvhttp_ws_stream_t* d_streams, uint32_t n_streams,
                               const uint64_t* d_read_end, uint32_t n_reads_total,
                               uint32_t max_frames, uvhttp_ws_frame_desc_t* d_desc,
                               uvhttp_ws_stream_result_t* d_results, void* stream);

/* Host side of the stream decode.  stream_init fills a descriptor from a live connection
 * (the caller copies recv_buffer[0, recv_buffer_pos) and the new reads to wire[begin, ...);
 * n_reads = 0, set first_read / n_reads for several calls); deliver_stream then applies a
 * decoded result to the connection exactly as the process_data calls would have: recv buffer
 * growth, on_message / on_close / control hooks for the delivered frames (fragments
 * reassembled in conn->fragmented_message), the bytes left in recv_buffer — including a
 * failing data frame the reference had already unmasked before its fragment check rejected
 * it (src/uvhttp_websocket.c:944 before :964-1000) — and the fragment state that check left.
 * `wire` and `desc` are host copies of the decoded batch. */
void uvhttp_ws_stream_init(const struct uvhttp_ws_connection* conn, uint64_t begin,
                           uint64_t len, uvhttp_ws_stream_t* out);
uvhttp_error_t uvhttp_ws_deliver_stream(struct uvhttp_ws_connection* conn, const uint8_t* wire,
                                        const uvhttp_ws_frame_desc_t* desc,
                                        const uvhttp_ws_stream_t* s,
                                        const uvhttp_ws_stream_result_t* r);

/* ---- batched send-side framing ---------------------------------------------------------- */
/* One frame to build: uvhttp_ws_build_frame(ctx, buf, size, payload, len, opcode, mask, fin)
 * (src/uvhttp_websocket.c:204-285).  The reference draws a client's masking key from the
 * context DRBG (:257-266, host-side mbedtls); here the caller supplies it. */
typedef struct {
    uint64_t payload_off;  /* payload = src[payload_off, payload_off + payload_len) */
    uint64_t payload_len;
    uint32_t masking_key;  /* used when mask != 0; key bytes k0..k3, k0 = low byte */
    uint8_t opcode;        /* written as opcode & 0x0F */
    uint8_t fin;
    uint8_t mask;          /* 0: server frame (no key, payload copied); 1: client frame */
    uint8_t reserved0;
    uint64_t reserved1;
} uvhttp_ws_build_desc_t;  /* 32 bytes */

/* Build n frames back to back into d_out: frame i at d_out_off[i] (exclusive prefix sum of
 * the frame sizes, header 2/4/10 by payload length, +4 key bytes when masked); d_out_off[n]
 * = total bytes.  If the total exceeds out_cap nothing is written to d_out (d_out_off still
 * is, so the caller can size the buffer), like build_frame's buffer_size check. */
int uvhttp_ws_gpu_build_frames(uvhttp_ws_gpu_engine_t* eng, const uint8_t* d_src,
                               uint64_t src_len, const uvhttp_ws_build_desc_t* d_frames,
                               uint32_t n_frames, uint8_t* d_out, uint64_t out_cap,
                               uint64_t* d_out_off, void* stream);

/* ---- host-memory pipeline (libuv read buffers in, decoded payloads out) ---------------- */
/* A pipeline owns `depth` slots.  Each slot = a pinned host staging buffer (the caller
 * writes masked frames there, e.g. hands it out from the libuv alloc callback) and a device
 * wire buffer.  Every slot's H2D copy runs on the pipeline's upload stream and its decode and
 * D2H copy on its compute stream (behind an event), so slot k's upload overlaps slot k-1's
 * kernels and download on the two copy queues.  submit() enqueues
 *   H2D(wire[0, wire_len)) -> decode_inplace -> D2H(wire, desc, summary)
 * and returns at once; wait() blocks until the slot's decoded bytes, descriptors and
 * summary are back in pinned host memory (the in-place contract: delivered payloads are
 * unmasked inside the slot buffer).  At most three submissions are in flight: submit() first
 * waits for the submission three back to finish, so depth 4 and up give the caller more slots
 * to fill while three are in flight (with more queued, the copies ran at 22-27 instead of 44
 * GiB/s on MI355X). */
typedef struct uvhttp_ws_gpu_pipeline uvhttp_ws_gpu_pipeline_t;
int uvhttp_ws_gpu_pipeline_create(int device, int depth, uint64_t slot_bytes,
                                  uint32_t slot_frames, uvhttp_ws_gpu_pipeline_t** out);
void uvhttp_ws_gpu_pipeline_free(uvhttp_ws_gpu_pipeline_t* p);
uint8_t* uvhttp_ws_gpu_pipeline_slot_buffer(uvhttp_ws_gpu_pipeline_t* p, int slot);
uint64_t* uvhttp_ws_gpu_pipeline_slot_offsets(uvhttp_ws_gpu_pipeline_t* p, int slot);
/* offsets: when use_offsets != 0 the first n entries of slot_offsets() are used, else
 * frame i starts at i * stride.  Limits as uvhttp_ws_batch_t. */
int uvhttp_ws_gpu_pipeline_submit(uvhttp_ws_gpu_pipeline_t* p, int slot, uint64_t wire_len,
                                  int use_offsets, uint64_t stride, uint32_t n_frames,
                                  int32_t max_frame_size, int32_t max_message_size,
                                  int32_t is_server);
int uvhttp_ws_gpu_pipeline_wait(uvhttp_ws_gpu_pipeline_t* p, int slot,
                                const uvhttp_ws_frame_desc_t** desc,
                                const uvhttp_ws_batch_summary_t** summary);
/* Compact submissions: H2D -> uvhttp_ws_gpu_decode_compact -> D2H of the message arena, the
 * message table and the summary, for uvhttp_ws_deliver_messages (messages reassembled on the
 * device: on_message reads the arena, no fragment copying on the host).  A fixed-stride batch
 * of >= 140-byte frames decodes summary-only (no descriptors) and only its last frame's slot
 * comes back into the slot buffer; any other batch decodes into descriptors, which come back
 * with the decoded wire.  wait_compact returns host pointers valid until the slot's next
 * submission; *desc is NULL for a summary-only batch.  Deliver with
 *   uvhttp_ws_deliver_messages(conn, arena, msgs, summary, slot_buffer(slot), desc, stride).
 * A slot's arena and table are allocated at its first compact submission (slot_bytes + 64 and
 * slot_frames entries). */
int uvhttp_ws_gpu_pipeline_submit_compact(uvhttp_ws_gpu_pipeline_t* p, int slot, uint64_t wire_len,
                                          int use_offsets, uint64_t stride, uint32_t n_frames,
                                          int32_t max_frame_size, int32_t max_message_size,
                                          int32_t is_server);
int uvhttp_ws_gpu_pipeline_wait_compact(uvhttp_ws_gpu_pipeline_t* p, int slot, const uint8_t** arena,
                                        const uvhttp_ws_message_desc_t** msgs,
                                        const uvhttp_ws_frame_desc_t** desc,
                                        const uvhttp_ws_batch_summary_t** summary);

/* Deliver a decoded in-place batch to a connection exactly as uvhttp_ws_process_data would
 * have (src/uvhttp_websocket.c:950-1084): on_message per complete message (fragments
 * reassembled in conn->fragmented_message with the reference growth rules), on_close +
 * state = CLOSED for CLOSE, control-sink echo / pong when conn->user_data != NULL.  `wire`
 * is the host copy of the decoded wire (slot buffer).  Frames [0, summary->n_delivered) are
 * delivered; returns UVHTTP_OK, or UVHTTP_ERROR_INVALID_PARAM if the batch failed (after
 * delivering the frames before the failure, like process_data). */
uvhttp_error_t uvhttp_ws_deliver_batch(struct uvhttp_ws_connection* conn, const uint8_t* wire,
                                       const uvhttp_ws_frame_desc_t* desc,
                                       const uvhttp_ws_batch_summary_t* summary);

/* Deliver a decoded COMPACT batch (uvhttp_ws_gpu_decode_compact, with or without descriptors)
 * to a connection as uvhttp_ws_process_data would have (src/uvhttp_websocket.c:950-1084, the
 * caller's dispatch src/uvhttp_connection.c:1234-1263): on_message(arena + msgs[m].arena_off,
 * msgs[m].len, msgs[m].opcode) per complete message, CLOSE (on_close, echo, state = CLOSED) and
 * PING (pong) through the same hooks as uvhttp_ws_deliver_batch, all in frame order; and a
 * message still open after the last delivered frame (summary->pending_bytes != 0, described by
 * msgs[summary->n_messages], which a compact decode writes then) is left in
 * conn->fragmented_message with the reference's size, capacity and opcode, so the connection's
 * next process_data call continues it.  Like uvhttp_ws_deliver_batch the batch's bytes never
 * passed through recv_buffer, which is not touched; the connection must have no message open
 * (the batch was decoded from a fresh connection's state), else UVHTTP_ERROR_INVALID_PARAM and
 * nothing is delivered.
 *   arena, msgs: host copies of arena[0, summary->arena_bytes) and msgs[0, n_messages + 1).
 *   Control frames keep their (unmasked) payloads in the wire.  With descriptors (desc != NULL,
 *   host copy of the n_delivered + 1 first entries) they are found there and read from `wire`
 *   (host copy of the decoded wire; only control payloads are read).  Summary-only (desc ==
 *   NULL) needs a fixed-stride batch with frame_stride >= 140 — a control frame (<= 131 wire
 *   bytes) then cannot fill a slot, so only the LAST delivered frame can be one; when that
 *   frame belongs to no message, `wire` must hold it at wire + (n_delivered - 1) *
 *   frame_stride (a caller may copy back just those frame_stride bytes into a buffer it
 *   offsets accordingly).  Reserved opcodes 3-7 / 11-15 are delivered without a callback, as
 *   the reference ignores them.  Returns UVHTTP_OK, or UVHTTP_ERROR_INVALID_PARAM if the batch
 *   failed (after delivering the frames before the failure, like process_data) or the
 *   arguments cannot describe the batch. */
uvhttp_error_t uvhttp_ws_deliver_messages(struct uvhttp_ws_connection* conn, const uint8_t* arena,
                                          const uvhttp_ws_message_desc_t* msgs,
                                          const uvhttp_ws_batch_summary_t* summary,
                                          const uint8_t* wire, const uvhttp_ws_frame_desc_t* desc,
                                          uint64_t frame_stride);

/* ---- batcher: live libuv reads -> one device decode per flush -------------------------- */
/* The caller side of the reference, on_websocket_read (src/uvhttp_connection.c:1098-1175),
 * calls uvhttp_ws_process_data once per libuv read.  The batcher takes those reads instead
 * (submit_read copies them, as process_data copies into recv_buffer) and decodes everything
 * queued at flush(): per connection, exactly the sequence of process_data calls the reads
 * would have made — same return codes, callbacks, recv-buffer and fragment state (tests/
 * test_c1_echo.py, tests/test_gpu_batcher.py check it against the oracle).  Callbacks fire
 * from flush(), connection by connection in first-read order; within a connection in read
 * order.  A flush whose queued bytes are below min_device_bytes runs the host decoder (one
 * libuv-sized read does not pay for a device round trip); a larger one goes
 * through the device: buffered bytes + reads in a pinned arena -> H2D -> gather ->
 * uvhttp_ws_gpu_decode_reads -> D2H -> uvhttp_ws_deliver_stream per connection.
 *
 * Asynchronous flushes.  The batcher holds two queues.  flush_async() hands the queue being
 * filled to the device and returns at once; submit_read() keeps queueing into the other one
 * (whose arena already streams to HBM while it fills, once it holds min_device_bytes).  The
 * decoded queue is delivered — callbacks fire — by poll() once its results are back in host
 * memory (or by flush()); a queue is staged for the device only after the queue before it
 * was delivered (a connection's later reads see the state its earlier ones left, so every
 * connection still sees exactly the process_data sequence).  With the host decoder (device -1, or a small queue) every
 * flush delivers before it returns.  Integration: flush_async() in the loop's uv_check
 * callback, poll() from a uv_async_t that on_ready signals.
 * Not thread-safe (the loop thread owns it, like the reference); only on_ready runs on
 * another thread. */
typedef struct uvhttp_ws_amd_batcher uvhttp_ws_amd_batcher_t;
/* a connection's queued reads failed: process_data returned rc (the reference then sends
 * close 1002 and closes, :1166-1174); the batcher drops the connection's later reads until
 * uvhttp_ws_amd_batcher_forget */
typedef void (*uvhttp_ws_amd_failure_cb)(void* ctx, struct uvhttp_ws_connection* conn, int rc);
/* an asynchronous flush's results are in host memory (called from a HIP runtime thread:
 * only signal the loop, e.g. uv_async_send; then call poll() on the loop thread) */
typedef void (*uvhttp_ws_amd_ready_cb)(void* ctx);
/* A TLS connection's record stream reached something that is not authenticated application
 * data the device may open: an alert or handshake record (first_status
 * UVHTTP_TLS_REC_CONTROL: close_notify, KeyUpdate, NewSessionTicket ...).  The records before it
 * were decrypted and decoded; `ciphertext` (len bytes, valid during the call) is everything
 * from that record on, including reads queued since, and next_seq is the read sequence number
 * of its first record.  The batcher forgets the connection's TLS state: the caller hands the
 * bytes to mbedtls (mbedtls_ssl_read, as src/uvhttp_connection.c:1128-1144 does) and may
 * register the connection again with uvhttp_ws_amd_batcher_set_tls (e.g. after a KeyUpdate). */
/* first_status of a handback that is not about a record: the device could not open this
 * connection's queued records (a device or launch error, or a queue that did not fit the device
 * layout).  Nothing of them was delivered; `ciphertext` is all of it from next_seq on. */
#define UVHTTP_WS_BATCHER_HANDBACK_DEVICE (-100)
typedef void (*uvhttp_ws_amd_tls_handback_cb)(void* ctx, struct uvhttp_ws_connection* conn,
                                              const uint8_t* ciphertext, size_t len,
                                              uint64_t next_seq, int first_status);
typedef struct {
    int device;                /* HIP device for large flushes; -1 = host decoder only */
    uint64_t min_device_bytes; /* flushes with fewer queued bytes run on the host */
    uint64_t max_bytes;        /* staging capacity (buffered bytes + reads) per flush; with a
                                  device, max_bytes / 6 + max_connections must stay < 2^26 */
    uint32_t max_connections;  /* connections per flush */
    uint32_t max_reads;        /* reads per flush */
    uvhttp_ws_amd_failure_cb on_failure;
    void* ctx;
    uvhttp_ws_amd_ready_cb on_ready; /* optional */
    void* ready_ctx;
    uvhttp_ws_amd_tls_handback_cb on_tls_handback; /* TLS connections (called with ctx) */
} uvhttp_ws_amd_batcher_config_t;
typedef struct {
    uint64_t flushes, device_flushes, host_flushes;
    uint64_t host_reads, device_reads;    /* reads decoded by each path */
    uint64_t device_frames, device_bytes; /* frames / staged bytes decoded on the device */
    uint64_t failures;                    /* connections reported through on_failure */
    uint64_t capacity_flushes;            /* device flushes re-run on the host (frame capacity) */
    double device_ms;                     /* wall time of device flushes (stage -> deliver) */
    uint64_t async_flushes;               /* queues handed to the device */
    uint64_t fallback_flushes;            /* queues that did not fit the device layout: host */
    uint64_t device_errors;               /* device failures; those queues ran on the host */
    uint64_t direct_reads;                /* reads larger than a flush, decoded in submit_read */
    double blocked_ms;                    /* loop-thread time inside batcher calls that flush,
                                             poll or wait: staging, delivering, waiting */
    double max_blocked_ms;                /* the longest single such call */
    double wait_ms;                       /* of blocked_ms: waiting for a device decode */
    double copy_ms;                       /* submit_read: copying reads into the pinned arena */
    double upload_ms;                     /* submit_read: enqueueing early H2D pieces */
    double stage_ms;                      /* staging a queue (prefixes, tables) + enqueueing */
    double deliver_ms;                    /* delivering device results (callbacks included) */
    uint64_t tls_records;                 /* TLS records opened and delivered on the device */
    uint64_t tls_bytes;                   /* their ciphertext bytes */
    uint64_t tls_handbacks;               /* connections handed back (on_tls_handback) */
    uint64_t desc_refetches;              /* flushes whose descriptors outgrew the copy-back
                                             high-water mark (rest fetched on completion) */
    uint64_t blocked_calls;               /* batcher calls counted in blocked_ms */
    double blocked_p50_ms, blocked_p99_ms;  /* their distribution (the last 65 536 calls) */
    double max_blocked_wait_ms;           /* the longest call's split: waiting for the device */
    double max_blocked_stage_ms;          /*   staging + enqueueing */
    double max_blocked_deliver_ms;        /*   delivering (callbacks included) */
    uint64_t zero_copy_reads;             /* reads queued through alloc_read / commit_read */
} uvhttp_ws_amd_batcher_stats_t;
void uvhttp_ws_amd_batcher_config_init(uvhttp_ws_amd_batcher_config_t* cfg);
/* UVHTTP_WS_GPU_ENODEV if cfg->device >= 0 names no usable MI355X (no silent host mode) */
int uvhttp_ws_amd_batcher_create(const uvhttp_ws_amd_batcher_config_t* cfg,
                                 uvhttp_ws_amd_batcher_t** out);
void uvhttp_ws_amd_batcher_free(uvhttp_ws_amd_batcher_t* b);
/* Queue one read of `conn` (the bytes are copied).  When the read would not fit the staging
 * capacity the queue is handed over first (flush_async); a read larger than a whole flush is
 * decoded right here, after the connection's earlier reads were delivered.  Returns
 * UVHTTP_OK, or UVHTTP_ERROR_INVALID_PARAM for a NULL argument, a connection whose earlier
 * reads already failed, or — only from inside a batcher callback, where no flush can start —
 * a read that does not fit the queue. */
uvhttp_error_t uvhttp_ws_amd_batcher_submit_read(uvhttp_ws_amd_batcher_t* b,
                                                 struct uvhttp_ws_connection* conn,
                                                 const uint8_t* data, size_t len);
/* Zero-copy reads: the loop's uv_alloc_cb / uv_read_cb pair (src/uvhttp_connection.c:128-158,
 * 1098-1175).  alloc_read returns space for conn's next read inside the queue's own (pinned)
 * staging arena — *buf, *len bytes, len <= suggested (less when the read would not fit a whole
 * flush); libuv reads the socket straight into it; commit_read then queues the nread bytes
 * exactly as submit_read(conn, buf, nread) would, without copying them.  nread = 0 (EAGAIN, EOF,
 * an error) gives the space back.  One allocation is outstanding at a time: libuv calls the
 * read callback right after the alloc callback for the same stream; any other batcher call in
 * between (a flush may hand the queue over) makes commit_read refuse with
 * UVHTTP_ERROR_INVALID_PARAM, as does a commit for another connection or nread > *len.
 * alloc_read may hand a full queue over first, like submit_read.  TLS connections: the space
 * takes ciphertext (as submit_tls_read). */
uvhttp_error_t uvhttp_ws_amd_batcher_alloc_read(uvhttp_ws_amd_batcher_t* b,
                                                struct uvhttp_ws_connection* conn, size_t suggested,
                                                uint8_t** buf, size_t* len);
uvhttp_error_t uvhttp_ws_amd_batcher_commit_read(uvhttp_ws_amd_batcher_t* b,
                                                 struct uvhttp_ws_connection* conn, size_t nread);
/* Hand everything queued to the decoder and return (see "Asynchronous flushes").  Never waits
 * for the device: when a queue is still in flight the request is remembered and poll() starts
 * this queue right after delivering that one (until then reads keep joining it; a read that
 * no longer fits makes submit_read wait).  0, or the UVHTTP_WS_GPU_* error of a device decode
 * that failed (its queue was decoded by the host decoder instead, so nothing is lost; stats
 * count it).  From inside a batcher callback: does nothing. */
int uvhttp_ws_amd_batcher_flush_async(uvhttp_ws_amd_batcher_t* b);
/* Deliver the queue in flight if its results are back (never waits), then start the queue a
 * flush_async asked for meanwhile: 1 delivered, 0 nothing to deliver yet, or a
 * UVHTTP_WS_GPU_* error as flush_async. */
int uvhttp_ws_amd_batcher_poll(uvhttp_ws_amd_batcher_t* b);
/* 1 while a queue is in flight (the loop must poll or flush before it can idle) */
int uvhttp_ws_amd_batcher_in_flight(const uvhttp_ws_amd_batcher_t* b);
/* Decode everything queued — the queue in flight, then the one being filled — and deliver it
 * before returning (callbacks fire here); returns as flush_async. */
int uvhttp_ws_amd_batcher_flush(uvhttp_ws_amd_batcher_t* b);
/* Drop a connection's queued reads (in both queues), failure mark and TLS state (call before
 * freeing the connection; safe from inside callbacks of a flush). */
void uvhttp_ws_amd_batcher_forget(uvhttp_ws_amd_batcher_t* b, struct uvhttp_ws_connection* conn);

/* TLS connections (the on_websocket_read TLS branch, src/uvhttp_connection.c:1122-1159:
 * mbedtls_ssl_read until WANT_READ, process_data on every decrypted chunk).  set_tls registers
 * the connection's read key (include/uvhttp_tls_amd.h: AES-128/256-GCM or ChaCha20-Poly1305,
 * TLS 1.3 or 1.2, from mbedtls's key export) and the sequence number of its next record;
 * submit_tls_read then queues ciphertext as libuv delivers it.  A flush opens the records of
 * every TLS connection on the device (uvhttp_tls_gpu_open_records), hands each delivered
 * record's content to the WebSocket decoder as one process_data call
 * (uvhttp_tls_gpu_ws_streams -> uvhttp_ws_gpu_decode_reads) and delivers as for plain
 * connections; an incomplete trailing record is kept for the next flush.  A record that is
 * not application data ends the batcher's TLS handling of the connection
 * (on_tls_handback); a record that fails (bad MAC, overflow, bad type or version) reports the
 * connection through on_failure with UVHTTP_ERROR_INVALID_PARAM, as the reference closes it
 * (:1139-1144).  TLS queues always decode on the device (the host decoder has no AEAD):
 * set_tls returns UVHTTP_WS_GPU_ENODEV for a host-only batcher.  A connection is either
 * plain or TLS: submit_read on a TLS connection (and submit_tls_read on a plain one) is
 * UVHTTP_ERROR_INVALID_PARAM.  set_tls flushes the connection's queued plain reads first; from
 * inside a batcher callback, where no flush can run, it returns UVHTTP_WS_GPU_EINVAL while such
 * reads are queued (call it again after the flush). */
int uvhttp_ws_amd_batcher_set_tls(uvhttp_ws_amd_batcher_t* b, struct uvhttp_ws_connection* conn,
                                  const void* tls_key /* uvhttp_tls_key_t */, uint64_t read_seq);
uvhttp_error_t uvhttp_ws_amd_batcher_submit_tls_read(uvhttp_ws_amd_batcher_t* b,
                                                     struct uvhttp_ws_connection* conn,
                                                     const uint8_t* ciphertext, size_t len);
/* Zero the counters (e.g. after a warm-up), so stats() describes what follows. */
void uvhttp_ws_amd_batcher_reset_stats(uvhttp_ws_amd_batcher_t* b);
int uvhttp_ws_amd_batcher_stats(const uvhttp_ws_amd_batcher_t* b,
                                uvhttp_ws_amd_batcher_stats_t* out);
/* NUMA node of the batcher's GPU (its PCI device's sysfs numa_node), or -1 (host-only batcher,
 * or not known).  Run the loop thread that calls submit_read on this node: submit_read copies
 * each read into pinned memory that HIP places next to the GPU, and on the MI355X box that copy
 * ran at 91 GB/s from the GPU's node against 48 GB/s from the other socket — the live shape end
 * to end 38 vs 22 GiB/s (profiles/r03p44_numa_copy_e2e.txt). */
int uvhttp_ws_amd_batcher_numa_node(const uvhttp_ws_amd_batcher_t* b);

/* ---- batcher group: the live path over several GPUs ------------------------------------ */
/* One batcher per device (the same config, cfg->device replaced by devices[k]; a device may be
 * listed twice, -1 = a host-decoder member).  Each connection is pinned to one member on its
 * first call — the member with the fewest live connections — until group_forget, so its reads
 * keep their process_data order (the member guarantees it) while different connections flush
 * over different PCIe links.  flush_async / poll / flush fan out to every member (flush: every
 * member's queue is handed over before any is waited for); poll returns the queues delivered
 * (summed) or the first error.  Callbacks are the members' (cfg's).  Not thread-safe, like the
 * batcher: one loop thread owns the group.  A loop thread copies reads at full rate only into
 * members on its own NUMA node (uvhttp_ws_amd_batcher_numa_node): on a two-socket node run one
 * loop per socket, each with a group of that socket's GPUs. */
typedef struct uvhttp_ws_amd_batcher_group uvhttp_ws_amd_batcher_group_t;
int uvhttp_ws_amd_batcher_group_create(const uvhttp_ws_amd_batcher_config_t* cfg, const int* devices,
                                       int n_devices, uvhttp_ws_amd_batcher_group_t** out);
void uvhttp_ws_amd_batcher_group_free(uvhttp_ws_amd_batcher_group_t* g);
int uvhttp_ws_amd_batcher_group_size(const uvhttp_ws_amd_batcher_group_t* g);
/* member i (its stats, NUMA node), or NULL */
uvhttp_ws_amd_batcher_t* uvhttp_ws_amd_batcher_group_batcher(uvhttp_ws_amd_batcher_group_t* g, int i);
/* the member a connection is pinned to, or -1 if it is not pinned (a query: never pins) */
int uvhttp_ws_amd_batcher_group_member(uvhttp_ws_amd_batcher_group_t* g, struct uvhttp_ws_connection* conn);
uvhttp_error_t uvhttp_ws_amd_batcher_group_submit_read(uvhttp_ws_amd_batcher_group_t* g,
                                                       struct uvhttp_ws_connection* conn,
                                                       const uint8_t* data, size_t len);
/* TLS records open only on device members: a new connection is pinned among them, and one
 * pinned to a host-decoder member moves to a device member when the host member holds nothing
 * of it (reads queued, a failure mark); otherwise, or with no device member, UVHTTP_WS_GPU_ENODEV */
int uvhttp_ws_amd_batcher_group_set_tls(uvhttp_ws_amd_batcher_group_t* g, struct uvhttp_ws_connection* conn,
                                        const void* tls_key, uint64_t read_seq);
/* zero-copy reads through the connection's member (pinned on its first alloc_read) */
uvhttp_error_t uvhttp_ws_amd_batcher_group_alloc_read(uvhttp_ws_amd_batcher_group_t* g,
                                                      struct uvhttp_ws_connection* conn, size_t suggested,
                                                      uint8_t** buf, size_t* len);
uvhttp_error_t uvhttp_ws_amd_batcher_group_commit_read(uvhttp_ws_amd_batcher_group_t* g,
                                                       struct uvhttp_ws_connection* conn, size_t nread);
uvhttp_error_t uvhttp_ws_amd_batcher_group_submit_tls_read(uvhttp_ws_amd_batcher_group_t* g,
                                                           struct uvhttp_ws_connection* conn,
                                                           const uint8_t* ciphertext, size_t len);
int uvhttp_ws_amd_batcher_group_flush_async(uvhttp_ws_amd_batcher_group_t* g);
int uvhttp_ws_amd_batcher_group_poll(uvhttp_ws_amd_batcher_group_t* g);
int uvhttp_ws_amd_batcher_group_flush(uvhttp_ws_amd_batcher_group_t* g);
int uvhttp_ws_amd_batcher_group_in_flight(const uvhttp_ws_amd_batcher_group_t* g);
void uvhttp_ws_amd_batcher_group_forget(uvhttp_ws_amd_batcher_group_t* g, struct uvhttp_ws_connection* conn);
/* counters summed over the members; max_blocked / percentiles: the worst member's */
int uvhttp_ws_amd_batcher_group_stats(const uvhttp_ws_amd_batcher_group_t* g,
                                      uvhttp_ws_amd_batcher_stats_t* out);
void uvhttp_ws_amd_batcher_group_reset_stats(uvhttp_ws_amd_batcher_group_t* g);

/* Library identity, for the loader checks in tests/. */
const char* uvhttp_ws_amd_version(void);

#ifdef __cplusplus
}
#endif

#endif /* UVHTTP_WS_AMD_H */
