/*
 * uvhttp_tls_amd.h — batched TLS record open (AES-GCM, ChaCha20-Poly1305) on MI355X, ahead of
 * the WebSocket decoder.
 *
 * What it replaces.  For a TLS connection the reference's WebSocket read callback decrypts
 * with mbedtls before framing: on_websocket_read (src/uvhttp_connection.c:1122-1159) calls
 * mbedtls_ssl_read into read_buffer until WANT_READ, hands every decrypted chunk to
 * uvhttp_ws_process_data (:1152-1153), closes the WebSocket on PEER_CLOSE_NOTIFY (:1136-1138)
 * and on any other negative return (:1139-1144).  mbedtls (an un-vendored submodule,
 * .gitmodules; absent here) opens each record with the negotiated AEAD — for the TLS 1.2/1.3
 * AEAD suites, AES-128/256-GCM (NIST SP 800-38D, RFC 5288) and ChaCha20-Poly1305 (RFC 8439,
 * RFC 7905), TLS 1.3 (RFC 8446 §5.2-5.3) and TLS 1.2.  This surface
 * opens the application-data records of many connections in one device call and leaves each
 * connection's plaintext contiguous in device memory, where uvhttp_ws_gpu_decode_streams
 * (include/uvhttp_ws_amd.h) takes it as its wire stream.
 *
 * Division of labour with mbedtls.  The handshake, alerts, post-handshake handshake messages
 * (KeyUpdate, NewSessionTicket) and renegotiation stay in mbedtls on the host.  The device
 * opens records while they are authenticated application data and stops a connection at the
 * first record that is not (status UVHTTP_TLS_REC_CONTROL, or an error): the host advances
 * mbedtls's read sequence number by n_delivered and feeds it the remaining ciphertext from
 * consumed_bytes on.  Keys come from the host (mbedtls's key-export callback:
 * TLS 1.3 traffic secret -> HKDF-Expand-Label key/iv, TLS 1.2 key block), one slot per
 * connection direction.
 *
 * Batch contract (the parity contract, restated by oracle/tls_oracle.c).  Connection s owns
 * the ciphertext bytes wire[begin, begin + len).  Records are walked from begin (5-byte header:
 * type, version, big-endian length).  The walk stops
 *   - with fewer than 5 bytes left, or fewer than 5 + length (incomplete: not an error, the
 *     bytes wait for the next read, like MBEDTLS_ERR_SSL_WANT_READ);
 *   - at a record whose header fails a check, in this order (the record is counted, with its
 *     status): version != 0x0303 (ERR_VERSION); type not application_data (TLS 1.3) / not
 *     alert, handshake or application_data (TLS 1.2) (ERR_BAD_TYPE); length over the limit
 *     (ERR_OVERFLOW: 2^14 content bytes (+ 1 inner type byte for TLS 1.3) + the AEAD
 *     overhead); length below the AEAD overhead (ERR_BAD_MAC).  The overhead is the 16-byte
 *     tag, plus the 8-byte explicit nonce of TLS 1.2 AES-GCM.
 * Counted record k of connection s is opened with sequence number seq + k.  Nonce: iv XOR
 * (0^32 || be64(seq)) for TLS 1.3 and for TLS 1.2 ChaCha20-Poly1305 (RFC 7905); iv[0..3] ||
 * the 8 explicit-nonce bytes after the header for TLS 1.2 AES-GCM (RFC 5288).  AAD: the 5
 * header bytes (TLS 1.3); be64(seq) || type || 0x03 0x03 || be16(plaintext length) (TLS 1.2).
 * TLS 1.3 inner plaintext = content || type || zero padding (type = last non-zero byte; none
 * = ERR_EMPTY).  A record is delivered if it authenticates (else
 * ERR_BAD_MAC) and its (inner) type is application_data (23), else it is CONTROL.  The first
 * record not delivered stops the connection; the records after it are SKIPPED.
 *
 * Output.  Connection s's delivered content is contiguous at out[out_off, out_off + plain_len)
 * in record order.  out_off is the connection's base in a layout where every counted record
 * reserves its largest possible content (length - overhead, - 1 more for TLS 1.3, never
 * below 0), connections in index order from 0; out_cap >= the total wire bytes of the
 * connections always suffices.  Bytes of out outside the delivered ranges are unspecified
 * and MAY HOLD UNAUTHENTICATED PLAINTEXT: records are decrypted in parallel, so a record whose
 * tag fails, and records after a connection's first undelivered record, may have had their
 * plaintext written to their reservation before the verdict.  Read only
 * [out_off, out_off + plain_len) of a connection (and the records' [out_off, + content_len)).
 * The ciphertext in wire is not modified.
 *
 * A connection's reservation is ws_prefix bytes followed by its records' reservations; its
 * plaintext starts at out_off = reservation start + ws_prefix.
 */
#ifndef UVHTTP_TLS_AMD_H
#define UVHTTP_TLS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UVHTTP_TLS_VERSION_12 0x0303u
#define UVHTTP_TLS_VERSION_13 0x0304u
#define UVHTTP_TLS_CONTENT_ALERT 21u
#define UVHTTP_TLS_CONTENT_HANDSHAKE 22u
#define UVHTTP_TLS_CONTENT_APPLICATION_DATA 23u

/* Return codes (same values as the WebSocket device surface). */
#define UVHTTP_TLS_GPU_OK 0
#define UVHTTP_TLS_GPU_EINVAL (-1)
#define UVHTTP_TLS_GPU_ENODEV (-2)
#define UVHTTP_TLS_GPU_ENOMEM (-3)
#define UVHTTP_TLS_GPU_ELAUNCH (-4)

/* Per-record status. */
#define UVHTTP_TLS_REC_OK 0               /* authenticated application data, delivered */
#define UVHTTP_TLS_REC_SKIPPED 2          /* after the connection's first undelivered record */
#define UVHTTP_TLS_REC_CONTROL 3          /* authenticated alert / handshake: host (mbedtls) */
#define UVHTTP_TLS_REC_ERR_OVERFLOW (-1)  /* record_overflow (RFC 8446 §5.2, RFC 5246 §6.2.3) */
#define UVHTTP_TLS_REC_ERR_BAD_MAC (-2)   /* tag mismatch, or too short for nonce + tag */
#define UVHTTP_TLS_REC_ERR_BAD_TYPE (-3)  /* outer content type not allowed */
#define UVHTTP_TLS_REC_ERR_VERSION (-4)   /* legacy_record_version != 0x0303 */
#define UVHTTP_TLS_REC_ERR_EMPTY (-5)     /* TLS 1.3 inner plaintext has no content type */
#define UVHTTP_TLS_REC_ERR_CAPACITY (-6)  /* records / layout exceed records[] or out_cap */
#define UVHTTP_TLS_REC_ERR_KEY (-7)       /* key slot out of range, or key_len / version / cipher invalid
                                             (connection result only; no record counted) */

/* AEAD of a key slot (uvhttp_tls_key_t.cipher). */
#define UVHTTP_TLS_CIPHER_AES_GCM 0u            /* AES-128/256-GCM (key_len 16 / 32) */
#define UVHTTP_TLS_CIPHER_CHACHA20_POLY1305 1u  /* RFC 8439 (key_len 32) */

/* Keys of one connection direction (64 bytes). */
typedef struct {
    uint8_t key[32];   /* key_len bytes used */
    uint8_t iv[12];    /* TLS 1.3 and TLS 1.2 ChaCha20-Poly1305: the write iv (nonce = iv XOR
                          seq); TLS 1.2 AES-GCM: salt = iv[0..3], rest ignored */
    uint32_t key_len;  /* 16 or 32 (AES-GCM), 32 (ChaCha20-Poly1305) */
    uint32_t version;  /* UVHTTP_TLS_VERSION_12 or UVHTTP_TLS_VERSION_13 */
    uint32_t cipher;   /* UVHTTP_TLS_CIPHER_* (0 = AES-GCM) */
    uint32_t reserved[2];
} uvhttp_tls_key_t;

/* One connection's buffered ciphertext (32 bytes). */
typedef struct {
    uint64_t begin;     /* offset in wire */
    uint64_t len;       /* bytes */
    uint64_t seq;       /* read sequence number of the first record */
    uint32_t key;       /* key slot */
    uint32_t ws_prefix; /* bytes reserved in out directly before the plaintext (out_off -
                           ws_prefix ...): room for what the connection's WebSocket decoder
                           already buffers (recv_buffer[0, recv_buffer_pos)), so the decoded
                           stream is contiguous; 0 = none */
} uvhttp_tls_stream_t;

/* One counted record (device-written, 32 bytes). */
typedef struct {
    uint64_t rec_off;      /* record start (header) in wire */
    uint64_t out_off;      /* delivered content start in out (0 if not delivered) */
    uint32_t content_len;  /* content bytes (0 unless opened) */
    uint32_t stream;       /* connection index */
    uint8_t type;          /* inner (TLS 1.3) / outer (TLS 1.2) content type once opened */
    int8_t status;         /* UVHTTP_TLS_REC_* */
    uint16_t reserved;
    uint32_t reserved2;
} uvhttp_tls_record_t;

/* One connection's result (device-written, 64 bytes). */
typedef struct {
    uint32_t first_record;    /* index of its first record in records[] */
    uint32_t n_records;       /* counted records */
    uint32_t n_delivered;     /* records delivered before the first stop */
    int32_t status;           /* 0, or -1 if the stop is an error (the reference closes) */
    int32_t first_status;     /* status of record n_delivered (0 if all delivered) */
    uint32_t reserved;
    uint64_t consumed_bytes;  /* ciphertext bytes of the delivered records */
    uint64_t next_seq;        /* seq + n_delivered */
    uint64_t out_off;         /* base of the connection's plaintext in out */
    uint64_t plain_len;       /* delivered content bytes */
    uint64_t reserved3;
} uvhttp_tls_result_t;

/* One record to seal (32 bytes). */
typedef struct {
    uint64_t src_off;    /* plaintext content in src */
    uint64_t out_off;    /* record start in out */
    uint64_t seq;        /* write sequence number */
    uint32_t plain_len;  /* content bytes, <= 2^14 */
    uint16_t key;        /* key slot */
    uint8_t type;        /* content type */
    uint8_t reserved;
} uvhttp_tls_seal_t;

typedef struct uvhttp_tls_gpu_engine uvhttp_tls_gpu_engine_t;

/* UVHTTP_TLS_GPU_ENODEV without a gfx950 device (there is no CPU fallback). */
int uvhttp_tls_gpu_engine_create(int device, uvhttp_tls_gpu_engine_t** out);
void uvhttp_tls_gpu_engine_free(uvhttp_tls_gpu_engine_t* eng);
const char* uvhttp_tls_gpu_engine_last_error(const uvhttp_tls_gpu_engine_t* eng);
/* HIP-event time of the record-crypto kernel over the calls since the last read. */
int uvhttp_tls_gpu_engine_set_timing(uvhttp_tls_gpu_engine_t* eng, int enable);
int uvhttp_tls_gpu_engine_kernel_time(uvhttp_tls_gpu_engine_t* eng, double* ms,
                                      uint64_t* launches);

/* Open the records of n_streams connections.  Device pointers: wire[wire_len], keys[n_keys],
 * streams[n_streams], records[max_records], results[n_streams], out[out_cap].  Asynchronous
 * on `stream` (a hipStream_t; NULL = default stream).  If the records do not fit records[] or
 * the layout does not fit out, every connection reports UVHTTP_TLS_REC_ERR_CAPACITY and
 * nothing is delivered. */
int uvhttp_tls_gpu_open_records(uvhttp_tls_gpu_engine_t* eng, const uint8_t* wire,
                                uint64_t wire_len, const uvhttp_tls_key_t* keys, uint32_t n_keys,
                                const uvhttp_tls_stream_t* streams, uint32_t n_streams,
                                uvhttp_tls_record_t* records, uint32_t max_records,
                                uvhttp_tls_result_t* results, uint8_t* out, uint64_t out_cap,
                                void* stream);

/* Seal records (the send side, and the bench's input generator).  Record i: header (type 23
 * for TLS 1.3, `type` for TLS 1.2), TLS 1.2 AES-GCM explicit nonce = be64(seq), ciphertext, tag; the
 * TLS 1.3 inner plaintext is content || type with no padding.  Device pointers throughout;
 * records must not overlap src. */
/* The TLS -> WebSocket hand-off on the device.  For every connection s: the ws_prefix bytes
 * at prefix_src[prefix_off[s]] (its recv_buffer[0, recv_buffer_pos), staged by the caller;
 * prefix_src may be NULL when every ws_prefix is 0) are copied to out[out_off - ws_prefix,
 * out_off), and ws_streams[s] (the caller filled the connection state with
 * uvhttp_ws_stream_init) gets begin = out_off - ws_prefix, len = ws_prefix + plain_len and
 * one process_data call per delivered record:
 * first_read = first_record, n_reads = n_delivered, read_end[first_record + k] = ws_prefix +
 * the content of records 0..k — exactly the chunks on_websocket_read hands to process_data,
 * one per mbedtls_ssl_read (src/uvhttp_connection.c:1128-1159; a read returns one record's
 * content when read_buffer_size >= 16384, the reference default).  read_end has max_records
 * entries.  Connections whose result is ERR_CAPACITY or ERR_KEY must not be decoded. */
int uvhttp_tls_gpu_ws_streams(uvhttp_tls_gpu_engine_t* eng, const uvhttp_tls_result_t* results,
                              const uvhttp_tls_record_t* records, uint32_t n_streams,
                              const uvhttp_tls_stream_t* streams, const uint8_t* prefix_src,
                              const uint64_t* prefix_off, uint8_t* out, void* ws_streams,
                              uint64_t* read_end, void* stream);

int uvhttp_tls_gpu_seal_records(uvhttp_tls_gpu_engine_t* eng, const uint8_t* src,
                                uint64_t src_len, const uvhttp_tls_seal_t* recs,
                                uint32_t n_records, const uvhttp_tls_key_t* keys,
                                uint32_t n_keys, uint8_t* out, uint64_t out_cap, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* UVHTTP_TLS_AMD_H */
