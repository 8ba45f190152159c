// tls_gpu.hip — batched TLS record open / seal (AES-128/256-GCM, ChaCha20-Poly1305) for
// gfx950 (MI355X).
//
// the record decrypt that runs ahead of the WebSocket decoder in the
// reference (mbedtls_ssl_read in on_websocket_read, src/uvhttp_connection.c:1122-1159).  The
// contract is in include/uvhttp_tls_amd.h and is restated on the CPU by oracle/tls_oracle.c.
//
// One call = key schedules -> record walk (count, scan, write) -> record crypto -> finalize
// (stop rules, final content offsets) -> left-shift fix-up for connections whose TLS 1.3
// records carried padding.  All on one stream, no host synchronisation.
//
// Record crypto (k_tls_crypt): AES-GCM is integer/bitwise work with no matrix shape — no MFMA.
// One wavefront per record (<= 1028 GHASH blocks):
//   * block i of the record's GHASH sequence (AAD, ciphertext blocks, length block; left-padded
//     with zero blocks to a multiple of 64) goes to lane i % 64, so every load and store of the
//     wave is one contiguous 1 KiB run of ciphertext;
//   * AES-CTR with the T-table round (four lookups + XORs per column) from ONE 1 KiB table
//     replicated in LDS (copy = lane % copies, word = x * copies + copy): ds_read_b32 banks
//     are (addr / 4) % 32 per 32-lane half, so 32 copies are conflict-free and 16 copies cost
//     at most 2-way; 16 copies leave room for 3 workgroups per CU and measured faster; the
//     other three tables are byte rotations;
//   * GHASH: each lane runs Horner with multiplier H^64 over its strided blocks, then a
//     6-level shuffle tree (multipliers H, H^2 ... H^32) and a final x H combine the lanes.
//     Multiplies use Shoup's table method: 4-bit tables (256 B per multiplier P: 16 entries of
//     16 B fill one LDS bank row, so a 16-lane group's ds_read_b128 never conflicts) for
//     H^(2^k), k = 0..6, built once per key by k_tls_keys; the Horner multiplier H^64 also
//     gets an 8-bit table (4 KiB, built per wave from its 4-bit table when the key changes),
//     which halves the steps of the dominant multiply.
//   * the lane holding the AAD block computes E(K, J0) for the tag instead of a keystream
//     block; TLS 1.3's content type is the last non-zero inner byte, found by a wave max.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "uvhttp_tls_amd.h"
#include "uvhttp_ws_amd.h"

namespace {

constexpr int kBlock = 256;            // walk / finalize kernels: one lane per connection
constexpr int kCryptWG = 256;          // crypto kernel: 4 waves, one record per wave
constexpr int kCryptWaves = kCryptWG / 64;
// tuning switches (tools/build_variant.sh -D...; defaults = the shipped configuration)
// (A/B on MI355X, tools/tls_ab.sh, 65 536 x 4 x 16 KiB TLS 1.3 AES-128-GCM; kernel GB/s of
// plaintext: 4-bit Horner + 32 copies 310, 8-bit Horner + 32 copies 355, 8-bit + 16 copies 394,
// 8-bit + 8 copies 379; forcing 4 waves/SIMD spills and loses)
#ifndef TLS_TE_COPIES
#define TLS_TE_COPIES 16   // copies of Te0 in LDS for the packed kernel (16: more workgroups per CU)
#endif
#ifndef TLS_RED8
#define TLS_RED8 1         // GHASH byte-step reduction: 0 shifts, 1 a 256-word LDS table, 2 two
                           // 16-word tables (one per nibble: conflict-free ds_read_b32)
#endif
#ifndef TLS_TE_COPIES_REC
#define TLS_TE_COPIES_REC 64  // copies for the one-record-per-wave kernels: 32 or more make every
                              // ds_read_b32 conflict-free (lane l reads copy l % 32, one bank);
                              // 64 (one per lane) also let one v_perm_b32 form the address
                              // (round 3, 16 KiB records: 16 copies x 4 waves 483 GB/s, 32 x 8
                              // 529, 64 x 16 589; profiles/r03_tls_aes_ab.txt)
#endif
#ifndef TLS_GHASH8
#define TLS_GHASH8 2       // Horner multiplier H^64 one byte per step: 1 through an 8-bit table
                           // (4 KiB per wave), 2 through two 4-bit tables (H^64 and H^64 x^4;
                           // 475.8 vs 469.7 GB/s, 15 KiB less LDS per workgroup, round 2)
#endif
#ifndef TLS_WPE
#define TLS_WPE 0          // >0: amdgpu_waves_per_eu hint for the crypto kernels
#endif
#if TLS_WPE > 0
#define CRYPT_ATTR __launch_bounds__(kCryptWG) __attribute__((amdgpu_waves_per_eu(TLS_WPE)))
#else
#define CRYPT_ATTR __launch_bounds__(kCryptWG)
#endif
#ifndef TLS_PACK_WPE
#define TLS_PACK_WPE 2     // amdgpu_waves_per_eu of the packed ChaCha20-Poly1305 kernel
#endif
#ifndef TLS_POLY_SGPR
#define TLS_POLY_SGPR 1    // 1: the Poly1305 key powers r^(2^t) in scalar registers
#endif
#ifndef TLS_CHACHA_WPE
#define TLS_CHACHA_WPE 4   // >0: amdgpu_waves_per_eu hint for the ChaCha20-Poly1305 kernels (4: 975 vs 960 GB/s at 3)
#endif
#if TLS_CHACHA_WPE > 0
#define CHACHA_ATTR __launch_bounds__(kCryptWG) __attribute__((amdgpu_waves_per_eu(TLS_CHACHA_WPE)))
#else
#define CHACHA_ATTR __launch_bounds__(kCryptWG)
#endif
#ifndef TLS_OPEN_WAVES
#define TLS_OPEN_WAVES 16  // waves per workgroup of the one-record-per-wave AES-GCM kernels
                           // (k_tls_open / k_tls_seal): they share one T-table copy set
#endif
#ifndef TLS_OPEN_WPE
#define TLS_OPEN_WPE TLS_WPE  // >0: amdgpu_waves_per_eu hint for those two kernels
#endif
constexpr int kOpenWaves = TLS_OPEN_WAVES;
constexpr int kOpenWG = 64 * kOpenWaves;
#if TLS_OPEN_WPE > 0
#define OPEN_ATTR __launch_bounds__(kOpenWG) __attribute__((amdgpu_waves_per_eu(TLS_OPEN_WPE)))
#else
#define OPEN_ATTR __launch_bounds__(kOpenWG)
#endif
[[maybe_unused]] constexpr uint32_t kTeShift = TLS_TE_COPIES == 64 ? 6 : TLS_TE_COPIES == 32 ? 5 : TLS_TE_COPIES == 16 ? 4 : 3;
[[maybe_unused]] constexpr uint32_t kTeShiftRec = TLS_TE_COPIES_REC == 64 ? 6 : TLS_TE_COPIES_REC == 32 ? 5 : TLS_TE_COPIES_REC == 16 ? 4 : 3;

struct U128 {  // a GCM block as a big-endian 128-bit value (bit 0 of the spec = MSB of hi)
    uint64_t hi, lo;
};

// Per key slot, built by k_tls_keys (2 KiB).
struct __attribute__((aligned(64))) KeySched {
    U128 tab[7][16];   // AES-GCM: 4-bit Shoup tables of H^(2^k), k = 0..6
    U128 tab3[16];     // AES-GCM: the table of H^3 (the packed kernel's lane combine)
    uint32_t rk[60];   // AES: FIPS-197 round-key words, big-endian; ChaCha20: key words [0..7], LE
    uint32_t nr;       // 10 / 14 (AES), 20 (ChaCha20); 0 = invalid key
    uint32_t version;  // UVHTTP_TLS_VERSION_12 / _13
    uint32_t iv[3];    // AES-GCM: iv as big-endian words; ChaCha20: little-endian words
    uint32_t cipher;   // UVHTTP_TLS_CIPHER_*
    uint32_t pad[10];
    uvhttp_tls_key_t src;  // the key this slot was built from (key_len 0: none): a call that
                           // passes the same key again skips the expansion
};
static_assert(sizeof(KeySched) == 2432, "key schedule layout");

// One counted record (walk -> crypto -> finalize).
struct RecWork {
    uint64_t rec_off;     // header offset in wire
    uint64_t spec_off;    // content position in out if every earlier record fills its reservation
    uint64_t seq;         // sequence number
    uint32_t len;         // TLSCiphertext.length
    uint32_t stream;
    uint32_t key;
    int32_t status;       // header status from the walk, then the open result
    uint32_t content_len;
    uint16_t type;
    int16_t walk_status;  // header status from the walk, never rewritten: kernels that split
                          // the records between them decide from it (and from len / cipher)
};
static_assert(sizeof(RecWork) == 48, "record work layout");

struct StreamWork {       // walk pass 1 -> pass 2
    uint32_t n_rec;
    uint32_t key_bad;
    uint64_t cap;
};

struct TlsArgs {
    const uint8_t* wire;
    uint64_t wire_len;
    const uvhttp_tls_key_t* keys;
    uint32_t n_keys;
    const uvhttp_tls_stream_t* streams;
    uint32_t n_streams;
    uvhttp_tls_record_t* records;
    uint32_t max_records;
    uvhttp_tls_result_t* results;
    uint8_t* out;
    uint64_t out_cap;
    const KeySched* sched;
    RecWork* work;
    StreamWork* sw;
    uint64_t* blk;        // per-256-stream block: [2b] records, [2b+1] reserved bytes
    uint32_t* n_total;    // [0] records to open (0 on capacity failure), [1] capacity failed,
                          // [2] bit c set: some record under cipher c (UVHTTP_TLS_CIPHER_*)
    uint32_t* fix;        // per connection: 1 = content must move left (padding)
    const uint32_t* te0;  // AES T-table (1 KiB), built once per engine
};

// ---- GF(2^128) ------------------------------------------------------------------------

__device__ inline U128 gf_xor(U128 a, U128 b) { return U128{a.hi ^ b.hi, a.lo ^ b.lo}; }

// multiply by x (SP 800-38D: right shift, reduce with R = 0xE1 || 0^120)
__device__ inline U128 gf_mulx(U128 v) {
    const uint64_t lsb = v.lo & 1;
    v.lo = (v.lo >> 1) | (v.hi << 63);
    v.hi = (v.hi >> 1) ^ (lsb ? 0xE100000000000000ull : 0ull);
    return v;
}

// generic bit-serial multiply (SP 800-38D Algorithm 1): key setup only
__device__ U128 gf_mul_slow(U128 x, U128 y) {
    U128 z{0, 0};
    for (int i = 0; i < 128; ++i) {
        const uint64_t bit = i < 64 ? (x.hi >> (63 - i)) & 1 : (x.lo >> (127 - i)) & 1;
        if (bit) z = gf_xor(z, y);
        y = gf_mulx(y);
    }
    return z;
}

// Shoup 4-bit table of P: T[8] = P, T[4] = P.x, T[2] = P.x^2, T[1] = P.x^3, T[a ^ b] = T[a] ^ T[b]
__device__ void gf_table(U128 p, U128* t) {
    U128 b[4];
    b[3] = p;  // index 8
    for (int k = 2; k >= 0; --k) b[k] = gf_mulx(b[k + 1]);  // b[2] = idx 4, b[1] = 2, b[0] = 1
    for (int v = 0; v < 16; ++v) {
        U128 r{0, 0};
        for (int k = 0; k < 4; ++k)
            if (v & (1 << k)) r = gf_xor(r, b[k]);
        t[v] = r;
    }
}

// reduction of the four bits shifted out by a multiply by x^4 (bits 112..127 of hi): bit p of
// r (p = 0 is b_127) becomes x^(128 + 3 - p) -> R >> (3 - p), i.e. carry-less r * 0x1C20
__device__ inline uint64_t gf_last4(uint32_t r) {
    return (uint64_t)((r << 5) ^ (r << 10) ^ (r << 11) ^ (r << 12)) << 48;
}

// the same for the eight bits shifted out by x^8: carry-less r * 0x1C2 (0x1C2 = 0xE100 >> 7)
__device__ inline uint64_t gf_last8(uint32_t r) {
    return (uint64_t)((r << 1) ^ (r << 6) ^ (r << 7) ^ (r << 8)) << 48;
}

// X . P with P's 4-bit table T (in LDS): Horner in x^4 from the last nibble of X
#ifndef TLS_MUL_CHUNK
#define TLS_MUL_CHUNK 16   // >0: the packed kernel's gf_mul_tab loads its table entries CHUNK
                           // Horner steps at a time (bounds the entries loaded ahead: 214 -> 108
                           // VGPRs, 2 -> 4 waves per SIMD)
#endif
template <int CHUNK = 0>
__device__ inline U128 gf_mul_tab(U128 x, const U128* __restrict__ t) {
    U128 z = t[x.lo & 0xF];
#pragma unroll
    for (int k = 30; k >= 0; --k) {
        if (CHUNK > 0 && k % (CHUNK > 0 ? CHUNK : 1) == 0 && k < 30) {
            // the remaining nibbles of x pass through an empty asm that also reads z: their
            // table loads cannot be hoisted above this step (the compiler would otherwise load
            // all 32 entries up front: 128 VGPRs)
            asm volatile("" : "+v"(x.lo), "+v"(x.hi) : "v"(z.lo));
        }
        const uint32_t n = k >= 16 ? (uint32_t)(x.lo >> ((31 - k) * 4)) & 0xF
                                   : (uint32_t)(x.hi >> ((15 - k) * 4)) & 0xF;
        const uint32_t r = (uint32_t)z.lo & 0xF;
        z.lo = (z.lo >> 4) | (z.hi << 60);
        z.hi = (z.hi >> 4) ^ gf_last4(r);
        const U128 e = t[n];
        z.hi ^= e.hi;
        z.lo ^= e.lo;
    }
    return z;
}

// X . P with P's 8-bit table T8 (256 entries of P * (byte polynomials)): Horner in x^8.  The
// reduction of the byte shifted out each step comes from red8 (gf_last8 >> 32, 256 words in
// LDS: one lookup instead of four shifts and three XORs)
[[maybe_unused]] __device__ inline U128 gf_mul_tab8(U128 x, const U128* __restrict__ t,
                                                    const uint32_t* __restrict__ red8) {
    U128 z = t[x.lo & 0xFF];
#pragma unroll
    for (int k = 14; k >= 0; --k) {
        const uint32_t n = k >= 8 ? (uint32_t)(x.lo >> ((15 - k) * 8)) & 0xFF
                                  : (uint32_t)(x.hi >> ((7 - k) * 8)) & 0xFF;
        const uint32_t r = (uint32_t)z.lo & 0xFF;
        z.lo = (z.lo >> 8) | (z.hi << 56);
#if TLS_RED8 == 2
        z.hi = (z.hi >> 8) ^ ((uint64_t)(red8[r >> 4] ^ red8[16 + (r & 15)]) << 32);
#elif TLS_RED8
        z.hi = (z.hi >> 8) ^ ((uint64_t)red8[r] << 32);
#else
        (void)red8;
        z.hi = (z.hi >> 8) ^ gf_last8(r);
#endif
        const U128 e = t[n];
        z.hi ^= e.hi;
        z.lo ^= e.lo;
    }
    return z;
}

// red8[r] = gf_last8(r) >> 32 (TLS_RED8 2: red8[v] = that of v << 4, red8[16 + v] of v)
__device__ inline void fill_red8(uint32_t* red8) {
#if TLS_RED8 == 2
    for (uint32_t r = threadIdx.x; r < 32; r += blockDim.x)
        red8[r] = (uint32_t)(gf_last8(r < 16 ? r << 4 : r - 16) >> 32);
#else
    for (uint32_t r = threadIdx.x; r < 256; r += blockDim.x) red8[r] = (uint32_t)(gf_last8(r) >> 32);
#endif
}

// X . P one byte per step from two conflict-free 4-bit tables: T8[v] = T4[v >> 4] ^ T4x4[v & 15]
// (T4x4 = the table of P . x^4), so a step reads two 256-byte tables (16 entries of 16 B: a
// 16-lane ds_read_b128 group never conflicts) instead of one 4 KiB table whose rows share
// banks every 256 B.  The reduction byte as TLS_RED8 says.
[[maybe_unused]] __device__ inline U128 gf_mul_tab8n(U128 x, const U128* __restrict__ t4,
                                                     const U128* __restrict__ t4x4,
                                                     const uint32_t* __restrict__ red8) {
    auto e8 = [&](uint32_t v) { return gf_xor(t4[v >> 4], t4x4[v & 15]); };
    U128 z = e8((uint32_t)x.lo & 0xFF);
#pragma unroll
    for (int k = 14; k >= 0; --k) {
        const uint32_t n = k >= 8 ? (uint32_t)(x.lo >> ((15 - k) * 8)) & 0xFF
                                  : (uint32_t)(x.hi >> ((7 - k) * 8)) & 0xFF;
        const uint32_t r = (uint32_t)z.lo & 0xFF;
        z.lo = (z.lo >> 8) | (z.hi << 56);
#if TLS_RED8 == 2
        z.hi = (z.hi >> 8) ^ ((uint64_t)(red8[r >> 4] ^ red8[16 + (r & 15)]) << 32);
#elif TLS_RED8
        z.hi = (z.hi >> 8) ^ ((uint64_t)red8[r] << 32);
#else
        (void)red8;
        z.hi = (z.hi >> 8) ^ gf_last8(r);
#endif
        const U128 a = t4[n >> 4], b = t4x4[n & 15];
        z.hi ^= a.hi ^ b.hi;
        z.lo ^= a.lo ^ b.lo;
    }
    return z;
}

// T4x4[v] = T4[v] . x^4 (16 lanes of one wave)
[[maybe_unused]] __device__ inline void gf_table_x4(const U128* t4, U128* t4x4) {
    const uint32_t lane = threadIdx.x & 63;
    if (lane < 16) {
        U128 v = t4[lane];
        const uint32_t r = (uint32_t)v.lo & 0xF;
        v.lo = (v.lo >> 4) | (v.hi << 60);
        v.hi = (v.hi >> 4) ^ gf_last4(r);
        t4x4[lane] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 8-bit table from the 4-bit one: byte v = (high nibble: x^0..x^3)(low nibble: x^4..x^7), so
// T8[v] = T4[v >> 4] ^ T4[v & 15] . x^4; one wave fills the 256 entries
[[maybe_unused]] __device__ inline void gf_table8(const U128* t4, U128* t8) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t v = lane; v < 256; v += 64) {
        U128 lo = t4[v & 15];
        const uint32_t r = (uint32_t)lo.lo & 0xF;
        lo.lo = (lo.lo >> 4) | (lo.hi << 60);
        lo.hi = (lo.hi >> 4) ^ gf_last4(r);
        t8[v] = gf_xor(t4[v >> 4], lo);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- AES ----------------------------------------------------------------------------------

__device__ inline uint32_t ror32(uint32_t x, int s) { return (x >> s) | (x << (32 - s)); }
__device__ inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// AES rounds R0 .. NR of one block with the T-table accessor te(s, k) (Te0[byte k of s], byte 0
// = least significant; k is always a constant); rk = big-endian
// round keys; s0..s3 = the state entering round R0; the ciphertext goes to out.  NR is a
// template argument so every round-key index is a constant (the keys stay in scalar registers
// when rk is wave-uniform).
// a ^ b ^ c in one instruction (v_bitop3_b32, truth table 0x96): the compiler splits a three-way
// XOR into two v_xor_b32 on gfx950; and (a | b) ^ c (0x56) for the last round's byte merge
__device__ inline uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ inline uint32_t or_xor(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x56);
}

template <int NR, int R0, typename TE>
__device__ inline void aes_rounds(const uint32_t* __restrict__ rk, uint32_t s0, uint32_t s1, uint32_t s2,
                                  uint32_t s3, uint32_t out[4], TE te) {
    constexpr uint32_t nr = NR;
#pragma unroll
    for (uint32_t r = R0; r < nr; ++r) {
        const uint32_t t0 = xor3(xor3(te(s0, 3), ror32(te(s1, 2), 8), ror32(te(s2, 1), 16)),
                                 ror32(te(s3, 0), 24), rk[4 * r]);
        const uint32_t t1 = xor3(xor3(te(s1, 3), ror32(te(s2, 2), 8), ror32(te(s3, 1), 16)),
                                 ror32(te(s0, 0), 24), rk[4 * r + 1]);
        const uint32_t t2 = xor3(xor3(te(s2, 3), ror32(te(s3, 2), 8), ror32(te(s0, 1), 16)),
                                 ror32(te(s1, 0), 24), rk[4 * r + 2]);
        const uint32_t t3 = xor3(xor3(te(s3, 3), ror32(te(s0, 2), 8), ror32(te(s1, 1), 16)),
                                 ror32(te(s2, 0), 24), rk[4 * r + 3]);
        s0 = t0, s1 = t1, s2 = t2, s3 = t3;
    }
    // last round: the S-box byte is byte 2 of Te0[x]; v_perm_b32 moves two of them into place
    // (selector bytes 4-7 pick from the first operand, 0-3 from the second, 0x0C gives zero)
    const uint32_t* k = rk + 4 * nr;
    auto word = [&](uint32_t ta, uint32_t tb, uint32_t tc, uint32_t td, uint32_t key) {
        const uint32_t hi = __builtin_amdgcn_perm(ta, tb, 0x06020C0Cu);
        const uint32_t lo = __builtin_amdgcn_perm(tc, td, 0x0C0C0602u);
        return or_xor(hi, lo, key);
    };
    out[0] = word(te(s0, 3), te(s1, 2), te(s2, 1), te(s3, 0), k[0]);
    out[1] = word(te(s1, 3), te(s2, 2), te(s3, 1), te(s0, 0), k[1]);
    out[2] = word(te(s2, 3), te(s3, 2), te(s0, 1), te(s1, 0), k[2]);
    out[3] = word(te(s3, 3), te(s0, 2), te(s1, 1), te(s2, 0), k[3]);
}

template <int NR, typename TE>
__device__ inline void aes_enc(const uint32_t* __restrict__ rk, uint32_t in[4], TE te) {
    aes_rounds<NR, 1>(rk, in[0] ^ rk[0], in[1] ^ rk[1], in[2] ^ rk[2], in[3] ^ rk[3], in, te);
}

template <typename TE>
__device__ inline void aes_encrypt(const uint32_t* __restrict__ rk, uint32_t nr, uint32_t in[4], TE te) {
    if (nr == 10)
        aes_enc<10>(rk, in, te);
    else
        aes_enc<14>(rk, in, te);
}

// AES-CTR with a counter below 2^16 (every GCM counter of a TLS record: J0 + 1 + block index,
// at most 1043): of the counter block only bytes 14 and 15 change, so round 1 depends on two
// varying bytes (columns 0 and 1 of its output) and round 2 reads eight varying bytes; the
// other 22 of those rounds' 32 table lookups are the same for every block of the record and
// are folded into six words once per record (the counter-mode caching of Bernstein-Schwabe).
struct CtrCache {
    uint32_t c0, c1;          // round-1 output columns 0 / 1 without their varying lookup
    uint32_t d0, d1, d2, d3;  // round-2 output without the lookups of round-1 columns 0 / 1
};

template <typename TE>
__device__ inline CtrCache ctr_cache(const uint32_t* __restrict__ rk, const uint32_t nonce[3], TE te) {
    const uint32_t s0 = nonce[0] ^ rk[0], s1 = nonce[1] ^ rk[1], s2 = nonce[2] ^ rk[2];
    const uint32_t s3 = rk[3];  // bytes 12, 13 of the counter are zero; 14, 15 vary
    CtrCache c;
    c.c0 = te(s0, 3) ^ ror32(te(s1, 2), 8) ^ ror32(te(s2, 1), 16) ^ rk[4];
    c.c1 = te(s1, 3) ^ ror32(te(s2, 2), 8) ^ ror32(te(s0, 0), 24) ^ rk[5];
    const uint32_t t2 = te(s2, 3) ^ ror32(te(s3, 2), 8) ^ ror32(te(s0, 1), 16) ^
                        ror32(te(s1, 0), 24) ^ rk[6];
    const uint32_t t3 = te(s3, 3) ^ ror32(te(s0, 2), 8) ^ ror32(te(s1, 1), 16) ^
                        ror32(te(s2, 0), 24) ^ rk[7];
    c.d0 = ror32(te(t2, 1), 16) ^ ror32(te(t3, 0), 24) ^ rk[8];
    c.d1 = ror32(te(t2, 2), 8) ^ ror32(te(t3, 1), 16) ^ rk[9];
    c.d2 = te(t2, 3) ^ ror32(te(t3, 2), 8) ^ rk[10];
    c.d3 = te(t3, 3) ^ ror32(te(t2, 0), 24) ^ rk[11];
    return c;
}

// E(K, nonce || ctr) for ctr < 2^16 from the record's cache (out = the 4 big-endian words)
template <int NR, typename TE>
__device__ inline void aes_ctr_cached(const uint32_t* __restrict__ rk, const CtrCache& c, uint32_t ctr,
                                      uint32_t out[4], TE te) {
    const uint32_t s3 = rk[3] ^ ctr;
    const uint32_t t0 = c.c0 ^ ror32(te(s3, 0), 24);
    const uint32_t t1 = c.c1 ^ ror32(te(s3, 1), 16);
    const uint32_t u0 = xor3(te(t0, 3), ror32(te(t1, 2), 8), c.d0);
    const uint32_t u1 = xor3(te(t1, 3), ror32(te(t0, 0), 24), c.d1);
    const uint32_t u2 = xor3(ror32(te(t0, 1), 16), ror32(te(t1, 0), 24), c.d2);
    const uint32_t u3 = xor3(ror32(te(t0, 2), 8), ror32(te(t1, 1), 16), c.d3);
    aes_rounds<NR, 3>(rk, u0, u1, u2, u3, out, te);
}

// S-box (FIPS-197 §5.1.1: inverse in GF(2^8), then the affine map) and Te0, one thread
__global__ void k_tls_te0(uint32_t* te0) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint8_t sbox[256];
    uint8_t p = 1, q = 1;
    do {
        p = (uint8_t)(p ^ (uint8_t)(p << 1) ^ ((p & 0x80) ? 0x1B : 0));
        q ^= (uint8_t)(q << 1);
        q ^= (uint8_t)(q << 2);
        q ^= (uint8_t)(q << 4);
        if (q & 0x80) q ^= 0x09;
        const uint8_t x = (uint8_t)(q ^ (uint8_t)((q << 1) | (q >> 7)) ^ (uint8_t)((q << 2) | (q >> 6)) ^
                                    (uint8_t)((q << 3) | (q >> 5)) ^ (uint8_t)((q << 4) | (q >> 4)));
        sbox[p] = (uint8_t)(x ^ 0x63);
    } while (p != 1);
    sbox[0] = 0x63;
    for (int x = 0; x < 256; ++x) {
        const uint32_t s = sbox[x];
        const uint32_t s2 = ((s << 1) ^ ((s & 0x80) ? 0x1B : 0)) & 0xFF;
        te0[x] = (s2 << 24) | (s << 16) | (s << 8) | (s2 ^ s);
    }
}

__device__ inline bool key_valid(const uvhttp_tls_key_t& k) {
    if (k.version != UVHTTP_TLS_VERSION_12 && k.version != UVHTTP_TLS_VERSION_13) return false;
    if (k.cipher == UVHTTP_TLS_CIPHER_AES_GCM) return k.key_len == 16 || k.key_len == 32;
    return k.cipher == UVHTTP_TLS_CIPHER_CHACHA20_POLY1305 && k.key_len == 32;
}

// explicit nonce bytes after the header: TLS 1.2 AES-GCM only (RFC 5288; RFC 7905 has none)
__device__ inline uint32_t explicit_len(uint32_t version, uint32_t cipher) {
    return version == UVHTTP_TLS_VERSION_12 && cipher == UVHTTP_TLS_CIPHER_AES_GCM ? 8u : 0u;
}

// key slot -> AES round keys, H = E(K, 0^128), tables of H^(2^k) (AES-GCM), or the ChaCha20
// key / iv words; one lane per slot
__global__ __launch_bounds__(kBlock) void k_tls_keys(const uvhttp_tls_key_t* keys, uint32_t n,
                                                     const uint32_t* te0, KeySched* ks) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uvhttp_tls_key_t k = keys[i];
    KeySched* o = ks + i;
    if (!key_valid(k)) {
        o->src.key_len = 0;
        o->nr = 0;
        o->version = 0;
        return;
    }
    {  // the slot already holds this key (the workspace is zeroed when allocated)
        const uvhttp_tls_key_t& c = o->src;
        bool same = c.key_len == k.key_len && c.version == k.version && c.cipher == k.cipher;
        for (int j = 0; j < 32 && same; ++j) same = c.key[j] == k.key[j];
        for (int j = 0; j < 12 && same; ++j) same = c.iv[j] == k.iv[j];
        if (same) return;
    }
    o->src.key_len = 0;  // (rebuilding)
    o->cipher = k.cipher;
    o->version = k.version;
    if (k.cipher == UVHTTP_TLS_CIPHER_CHACHA20_POLY1305) {  // RFC 8439: little-endian words
        for (int j = 0; j < 8; ++j)
            o->rk[j] = (uint32_t)k.key[4 * j] | ((uint32_t)k.key[4 * j + 1] << 8) |
                       ((uint32_t)k.key[4 * j + 2] << 16) | ((uint32_t)k.key[4 * j + 3] << 24);
        for (int j = 0; j < 3; ++j)
            o->iv[j] = (uint32_t)k.iv[4 * j] | ((uint32_t)k.iv[4 * j + 1] << 8) |
                       ((uint32_t)k.iv[4 * j + 2] << 16) | ((uint32_t)k.iv[4 * j + 3] << 24);
        o->nr = 20;
        o->src = k;
        return;
    }
    auto sb = [&](uint32_t x) { return (te0[x] >> 16) & 0xFF; };
    const uint32_t nk = k.key_len / 4, nr = nk + 6, total = 4 * (nr + 1);
    uint32_t w[60];
    for (uint32_t j = 0; j < nk; ++j)
        w[j] = ((uint32_t)k.key[4 * j] << 24) | ((uint32_t)k.key[4 * j + 1] << 16) |
               ((uint32_t)k.key[4 * j + 2] << 8) | k.key[4 * j + 3];
    uint32_t rcon = 1;
    for (uint32_t j = nk; j < total; ++j) {
        uint32_t t = w[j - 1];
        if (j % nk == 0) {
            t = (sb((t >> 16) & 0xFF) << 24) | (sb((t >> 8) & 0xFF) << 16) | (sb(t & 0xFF) << 8) |
                sb(t >> 24);
            t ^= rcon << 24;
            rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1B : 0)) & 0xFF;
        } else if (nk > 6 && j % nk == 4) {
            t = (sb(t >> 24) << 24) | (sb((t >> 16) & 0xFF) << 16) | (sb((t >> 8) & 0xFF) << 8) |
                sb(t & 0xFF);
        }
        w[j] = w[j - nk] ^ t;
    }
    for (uint32_t j = 0; j < total; ++j) o->rk[j] = w[j];
    o->nr = nr;
    for (int j = 0; j < 3; ++j)
        o->iv[j] = ((uint32_t)k.iv[4 * j] << 24) | ((uint32_t)k.iv[4 * j + 1] << 16) |
                   ((uint32_t)k.iv[4 * j + 2] << 8) | k.iv[4 * j + 3];
    uint32_t z[4] = {0, 0, 0, 0};
    aes_encrypt(w, nr, z, [&](uint32_t v, int k) { return te0[(v >> (8 * k)) & 0xFF]; });
    U128 p{((uint64_t)z[0] << 32) | z[1], ((uint64_t)z[2] << 32) | z[3]};
    const U128 h = p;
    U128 t[16];
    for (int l = 0; l < 7; ++l) {
        gf_table(p, t);
        for (int v = 0; v < 16; ++v) o->tab[l][v] = t[v];
        if (l == 1) {  // p = H^2
            gf_table(gf_mul_slow(p, h), t);
            for (int v = 0; v < 16; ++v) o->tab3[v] = t[v];
        }
        p = gf_mul_slow(p, p);
    }
    o->src = k;
}

// ---- record walk ------------------------------------------------------------------------

__device__ inline uint32_t be16(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }

// header checks in contract order; 0 or the record status.  AEAD overhead = 16-byte tag +
// explicit nonce; the limit is 2^14 content bytes (+ the TLS 1.3 inner type byte) + overhead
__device__ inline int32_t header_status(uint32_t version, uint32_t cipher, uint32_t type,
                                        uint32_t ver, uint32_t len) {
    const uint32_t over = 16 + explicit_len(version, cipher);
    if (ver != 0x0303) return UVHTTP_TLS_REC_ERR_VERSION;
    if (version == UVHTTP_TLS_VERSION_13 ? type != 23 : (type < 21 || type > 23))
        return UVHTTP_TLS_REC_ERR_BAD_TYPE;
    if (len > 16384u + (version == UVHTTP_TLS_VERSION_13 ? 1u : 0u) + over)
        return UVHTTP_TLS_REC_ERR_OVERFLOW;
    if (len < over) return UVHTTP_TLS_REC_ERR_BAD_MAC;
    return 0;
}

__device__ inline uint64_t record_cap(uint32_t version, uint32_t cipher, uint32_t len) {
    const uint32_t over = 16 + explicit_len(version, cipher) + (version == UVHTTP_TLS_VERSION_13 ? 1u : 0u);
    return len > over ? len - over : 0;
}

// walk one connection's records; WRITE fills RecWork from index `first` (spec offsets from base)
// ChaCha20-Poly1305 records up to this TLSCiphertext.length (8 KiB of content + the TLS 1.3 type
// byte) are opened kPack to a wave (k_tls_open_chacha_packed), longer ones one per wave
// (measured, TLS 1.3 GiB/s per-record -> packed: 256 B 34 -> 122, 1 KiB 128 -> 323, 2 KiB
// 249 -> 466, 4 KiB 463 -> 599, 8 KiB 698 -> 726; 16 KiB 913 -> 812, so 16 KiB stays per record)
constexpr uint32_t kPackMaxLen = 8192 + 1 + 16;
// AES-GCM records up to this length (4 KiB of content with either version's overhead) are
// opened kPack to a wave (k_tls_open_aes_packed); measured TLS 1.3 GiB/s per-record -> packed:
// 256 B 32 -> 79, 1 KiB 93 -> 163, 4 KiB 233 -> 264, 8 KiB 311 -> 297 (so 8 KiB stays per record)
constexpr uint32_t kPackMaxLenAes = 4096 + 1 + 24;

template <bool WRITE>
__device__ inline uint32_t walk(const TlsArgs& a, uint32_t s, uint64_t* cap_out, uint32_t first,
                                uint64_t base, uint32_t* size_bits = nullptr) {
    const uvhttp_tls_stream_t st = a.streams[s];
    *cap_out = st.ws_prefix;  // the connection's reservation starts with its WebSocket prefix
    if (st.key >= a.n_keys) return 0;
    const uvhttp_tls_key_t k = a.keys[st.key];
    if (!key_valid(k)) return 0;
    // bounds test that cannot wrap (a begin near 2^64 fails it)
    const uint64_t L = st.len <= a.wire_len && st.begin <= a.wire_len - st.len ? st.len : 0;
    const uint8_t* p = a.wire + st.begin;
    uint32_t n = 0;
    uint64_t pos = 0, cap = st.ws_prefix;
    // one record: false = the walk ends here (header failure: counted; incomplete: not)
    auto step = [&](uint32_t type, uint32_t ver, uint32_t len) {
        const int32_t hs = header_status(k.version, k.cipher, type, ver, len);
        if (!hs && L - pos - 5 < len) return false;  // incomplete: waits for more bytes
        if (size_bits && !hs)
            *size_bits |= len <= (k.cipher == UVHTTP_TLS_CIPHER_AES_GCM ? kPackMaxLenAes : kPackMaxLen) ? 1u : 2u;
        if (WRITE) {
            RecWork w;
            w.rec_off = st.begin + pos;
            w.spec_off = base + cap;
            w.seq = st.seq + n;
            w.len = len;
            w.stream = s;
            w.key = st.key;
            w.status = hs;
            w.walk_status = (int16_t)hs;
            w.content_len = 0;
            w.type = 0;
            a.work[first + n] = w;
        }
        ++n;
        if (hs) return false;
        cap += record_cap(k.version, k.cipher, len);
        pos += 5 + (uint64_t)len;
        return true;
    };
    // The walk is a chain of dependent header loads (one memory round trip per record).  With
    // the header at pos known, the headers kSpec records ahead are loaded at once on the guess
    // that the records have the same length (a connection's full-size records); each guess is
    // used while it holds, so a run of equal records costs one round trip per kSpec + 1.
    constexpr int kSpec = 3;
    while (L - pos >= 5) {
        const uint32_t type = p[pos], ver = be16(p + pos + 1), len = be16(p + pos + 3);
        const uint64_t stride = 5 + (uint64_t)len;
        uint32_t gt[kSpec], gv[kSpec], gl[kSpec];
        bool have[kSpec];
#pragma unroll
        for (int j = 0; j < kSpec; ++j) {
            const uint64_t q = pos + (j + 1) * stride;
            have[j] = q <= L && L - q >= 5;
            if (have[j]) gt[j] = p[q], gv[j] = be16(p + q + 1), gl[j] = be16(p + q + 3);
        }
        if (!step(type, ver, len)) break;
        bool go = true;
#pragma unroll
        for (int j = 0; j < kSpec; ++j) {
            // pos advanced by stride per record of length len: the guess is the next header
            // while every earlier guessed record had length len
            if (!go || !have[j]) break;
            if (!step(gt[j], gv[j], gl[j])) {
                go = false;
                break;
            }
            if (gl[j] != len) break;
        }
        if (!go) break;
    }
    *cap_out = cap;
    return n;
}

template <typename T>
__device__ inline T block_exclusive_sum(T v, T* total) {
    __shared__ T wsum[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    T inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T o = __shfl_up(inc, d, 64);
        if (lane >= d) inc += o;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    T pre = 0, all = 0;
    for (int k = 0; k < kBlock / 64; ++k) {
        if (k < wave) pre += wsum[k];
        all += wsum[k];
    }
    __syncthreads();
    *total = all;
    return pre + inc - v;
}

__global__ __launch_bounds__(kBlock) void k_tls_walk_count(TlsArgs a) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    uint64_t cap = 0;
    uint32_t n = 0, cipher = 0, sizes = 0;
    if (s < a.n_streams) {
        n = walk<false>(a, s, &cap, 0, 0, &sizes);
        a.sw[s] = StreamWork{n, 0u, cap};
        if (n) cipher = a.keys[a.streams[s].key].cipher;  // walk counted records: key valid
    }
    uint64_t tn, tc;
    (void)block_exclusive_sum<uint64_t>(n, &tn);
    (void)block_exclusive_sum<uint64_t>(cap, &tc);
    // which AEADs the block's records use, in the top byte of its record count: the crypto
    // kernel of an AEAD no record uses returns at once
    // (bit 0 AES-GCM, bit 1 ChaCha20-Poly1305, bits 2 / 3: ChaCha records short / long enough
    // for the packed / per-record kernel, bits 4 / 5: the same for AES-GCM)
    const bool cc = n && cipher == UVHTTP_TLS_CIPHER_CHACHA20_POLY1305;
    const bool ag = n && cipher == UVHTTP_TLS_CIPHER_AES_GCM;
    const uint64_t m = (__syncthreads_or(ag) ? 1u : 0u) |
                       (__syncthreads_or(cc) ? 2u : 0u) | (__syncthreads_or(cc && (sizes & 1)) ? 4u : 0u) |
                       (__syncthreads_or(cc && (sizes & 2)) ? 8u : 0u) |
                       (__syncthreads_or(ag && (sizes & 1)) ? 16u : 0u) |
                       (__syncthreads_or(ag && (sizes & 2)) ? 32u : 0u);
    if (threadIdx.x == 0) {
        a.blk[2 * blockIdx.x] = tn | (m << 56);
        a.blk[2 * blockIdx.x + 1] = tc;
    }
}

// exclusive prefix of the per-block (records, bytes) pairs; capacity decision
__global__ __launch_bounds__(kBlock) void k_tls_walk_scan(TlsArgs a, uint32_t n_blocks) {
    const uint32_t per = (n_blocks + kBlock - 1) / kBlock;
    const uint32_t beg = threadIdx.x * per;
    const uint32_t fin = beg + per < n_blocks ? beg + per : n_blocks;
    constexpr uint64_t kCount = (1ull << 56) - 1;
    uint64_t rn = 0, rc = 0;
    uint32_t m = 0;
    for (uint32_t b = beg; b < fin; ++b) {
        rn += a.blk[2 * b] & kCount, rc += a.blk[2 * b + 1];
        m |= (uint32_t)(a.blk[2 * b] >> 56);
    }
    uint64_t tn, tc;
    uint64_t pn = block_exclusive_sum<uint64_t>(rn, &tn);
    uint64_t pc = block_exclusive_sum<uint64_t>(rc, &tc);
    uint32_t mask = 0;
#pragma unroll
    for (int bit = 0; bit < 6; ++bit) mask |= __syncthreads_or(m & (1u << bit)) ? 1u << bit : 0u;
    for (uint32_t b = beg; b < fin; ++b) {
        const uint64_t vn = a.blk[2 * b] & kCount, vc = a.blk[2 * b + 1];
        a.blk[2 * b] = pn;
        a.blk[2 * b + 1] = pc;
        pn += vn;
        pc += vc;
    }
    if (threadIdx.x == 0) {
        const bool fail = tn > a.max_records || tc > a.out_cap;
        a.n_total[0] = fail ? 0u : (uint32_t)tn;
        a.n_total[1] = fail ? 1u : 0u;
        a.n_total[2] = mask;
    }
}

__global__ __launch_bounds__(kBlock) void k_tls_walk_write(TlsArgs a) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    const StreamWork sw = s < a.n_streams ? a.sw[s] : StreamWork{0, 0, 0};
    uint64_t tn, tc;
    const uint64_t first = a.blk[2 * blockIdx.x] + block_exclusive_sum<uint64_t>(sw.n_rec, &tn);
    const uint64_t base = a.blk[2 * blockIdx.x + 1] + block_exclusive_sum<uint64_t>(sw.cap, &tc);
    if (s >= a.n_streams || a.n_total[1]) return;
    uint64_t cap;
    (void)walk<true>(a, s, &cap, (uint32_t)first, base);
    a.sw[s].key_bad = (uint32_t)first;  // reused: first record index for finalize
    a.sw[s].cap = base;                 // reused: the connection's base in out
}

// ---- record crypto ---------------------------------------------------------------------------

// 16 bytes at p + [lo, hi) of a 16-byte window (others zero); little-endian words
__device__ inline void load_part(const uint8_t* p, int lo, int hi, uint32_t w[4]) {
    if (lo == 0 && hi == 16) {
        __builtin_memcpy(w, p, 16);
        return;
    }
    w[0] = w[1] = w[2] = w[3] = 0;
    for (int b = lo; b < hi; ++b) w[b >> 2] |= (uint32_t)p[b] << (8 * (b & 3));
}

__device__ inline void store_part(uint8_t* p, int n, const uint32_t w[4]) {
    if (n == 16) {
        __builtin_memcpy(p, w, 16);
        return;
    }
    for (int b = 0; b < n; ++b) p[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
}

__device__ inline U128 le_to_block(const uint32_t w[4]) {
    return U128{((uint64_t)bswap32(w[0]) << 32) | bswap32(w[1]),
                ((uint64_t)bswap32(w[2]) << 32) | bswap32(w[3])};
}

__device__ inline U128 shfl_down128(U128 v, int d) {
    const uint32_t a = __shfl_down((uint32_t)v.hi, d, 64), b = __shfl_down((uint32_t)(v.hi >> 32), d, 64);
    const uint32_t c = __shfl_down((uint32_t)v.lo, d, 64), e = __shfl_down((uint32_t)(v.lo >> 32), d, 64);
    return U128{((uint64_t)b << 32) | a, ((uint64_t)e << 32) | c};
}

struct SealArgs {
    const uint8_t* src;
    uint64_t src_len;
    const uvhttp_tls_seal_t* recs;
    uint32_t n;
    uint8_t* out;
    uint64_t out_cap;
    const KeySched* sched;
    uint32_t n_keys;
    const uint32_t* te0;
};

// One record's GCM on one wave, in two parts around the lane combine.  OPEN: ciphertext at
// ct[0, clen) -> plaintext content to dst[0, wlen) (wlen = bytes to keep), then tag match +
// (TLS 1.3) the last non-zero byte.  SEAL: plaintext from the (content, type) generator ->
// ciphertext at ct, tag after it.
struct CryptOut {
    bool tag_ok;
    uint32_t last_nz;  // (index + 1) << 8 | byte of the last non-zero inner byte, 0 if none
};

// TLS 1.3 content type: each lane keeps the last (highest-offset) non-zero 16-byte block of
// inner plaintext it saw (blocks arrive in increasing order per lane) and resolves the byte
// once at the end: (index + 1) << 8 | byte, 0 if none — the wave max is the last non-zero byte
struct LastNz {
    uint32_t off1;  // block offset + 1, 0 = none
    uint32_t w[4];
    __device__ inline void see(uint32_t off, const uint32_t pt[4]) {
        if (pt[0] | pt[1] | pt[2] | pt[3]) {
            off1 = off + 1;
            w[0] = pt[0], w[1] = pt[1], w[2] = pt[2], w[3] = pt[3];
        }
    }
    __device__ inline uint32_t resolve() const {
        if (!off1) return 0;
        for (int b = 3; b >= 0; --b) {
            if (w[b]) {
                const uint32_t byte_i = 4 * b + (31 - __builtin_clz(w[b])) / 8;
                return ((off1 + byte_i) << 8) | ((w[b] >> (8 * (byte_i & 3))) & 0xFF);
            }
        }
        return 0;
    }
};

struct Lanes {          // per-lane state after the Horner pass
    U128 acc;           // the lane's Horner sum (multiplier H^64)
    uint32_t ej0[4];    // E(K, J0) in the lane that held the AAD block
    uint32_t last_nz;
    uint32_t src_lane;  // that lane
};

template <bool SEAL>
__device__ Lanes gcm_lanes(const KeySched* __restrict__ ks, const uint32_t* te, uint32_t lane32,
                           const U128 (*tabs)[16], const U128* t8, const uint32_t* red8,
                           const uint32_t nonce[3], U128 aad,
                           uint32_t alen, const uint8_t* ct_in, uint8_t* ct_out, uint32_t clen,
                           uint8_t* dst, uint32_t wlen, const uint8_t* src, uint32_t src_n,
                           uint32_t inner_type, bool is13) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nr = ks->nr;
    const uint32_t nblk = (clen + 15) / 16;
    const uint32_t m = nblk + 2;             // AAD, ciphertext blocks, length block
    const uint32_t J = (m + 63) / 64;
    const uint32_t pad = 64 * J - m;
#if TLS_TE_COPIES_REC == 64
    // entry x of lane l's copy at byte 256 x + 4 l: one v_perm_b32 builds the address from the
    // state byte and the lane offset (no extract + shift-or)
    const uint32_t lane4 = lane32 << 2;
    const uint8_t* te8 = reinterpret_cast<const uint8_t*>(te);
    auto te_lds = [&](uint32_t v, int k) {
        return *reinterpret_cast<const uint32_t*>(te8 + __builtin_amdgcn_perm(v, lane4, 0x0C0C0000u | ((4u + k) << 8)));
    };
#else
    auto te_lds = [&](uint32_t v, int k) { return te[(((v >> (8 * k)) & 0xFF) << kTeShiftRec) | lane32]; };
#endif
    const uint32_t* __restrict__ rk = ks->rk;
    U128 acc{0, 0};
    uint32_t ej0[4] = {0, 0, 0, 0};
    LastNz nz{0, {0, 0, 0, 0}};
    // every counter of the record below 2^16 (always, for TLS record sizes): rounds 1-2 cached
    const bool cached = m + 1 < 65536u;
    CtrCache cc{0, 0, 0, 0, 0, 0};
    if (cached) cc = ctr_cache(rk, nonce, te_lds);
    for (uint32_t j = 0; j < J; ++j) {
        const int32_t q = (int32_t)(64 * j + lane) - (int32_t)pad;  // position in the sequence
        U128 x{0, 0};
        // counter block: J0 for the AAD lane (tag mask), J0 + 1 + k for ciphertext block k
        uint32_t cb[4] = {nonce[0], nonce[1], nonce[2], q <= 0 ? 1u : (uint32_t)q + 1u};
        // (loading the ciphertext block ahead of the rounds, pinned by a sched_barrier, measured
        // neutral here — 410 GB/s either way — unlike ChaCha20-Poly1305, where it gained 20%)
        if (!cached)
            aes_encrypt(rk, nr, cb, te_lds);
        else if (nr == 10)
            aes_ctr_cached<10>(rk, cc, cb[3], cb, te_lds);
        else
            aes_ctr_cached<14>(rk, cc, cb[3], cb, te_lds);
        if (q == 0) {
            x = aad;
            ej0[0] = cb[0], ej0[1] = cb[1], ej0[2] = cb[2], ej0[3] = cb[3];
        } else if (q > 0 && (uint32_t)q <= nblk) {
            const uint32_t k = (uint32_t)q - 1;
            const uint32_t off = 16 * k;
            const int n = clen - off < 16 ? (int)(clen - off) : 16;
            uint32_t d[4];
            const uint32_t ks4[4] = {bswap32(cb[0]), bswap32(cb[1]), bswap32(cb[2]), bswap32(cb[3])};
            if (!SEAL) {
                load_part(ct_in + off, 0, n, d);
                x = le_to_block(d);
                uint32_t pt[4];
                for (int b = 0; b < 4; ++b) pt[b] = d[b] ^ ks4[b];
                if (n < 16) {  // keep zero beyond the record
                    for (int b = 0; b < 4; ++b) {
                        const int lo = 4 * b;
                        const uint32_t msk = n >= lo + 4 ? 0xFFFFFFFFu : n <= lo ? 0u : ((1u << (8 * (n - lo))) - 1u);
                        pt[b] &= msk;
                    }
                }
                if (is13) nz.see(off, pt);
                if (off < wlen) store_part(dst + off, wlen - off < 16 ? (int)(wlen - off) : 16, pt);
            } else {
                // inner plaintext byte b of the record = content b (< src_n), type (== src_n), 0
                const int cn = src_n > off ? (src_n - off < 16 ? (int)(src_n - off) : 16) : 0;
                load_part(src + off, 0, cn, d);
                if (is13 && src_n >= off && src_n < off + 16) {
                    const uint32_t bq = src_n - off;
                    d[bq >> 2] |= inner_type << (8 * (bq & 3));
                }
                for (int b = 0; b < 4; ++b) d[b] ^= ks4[b];
                if (n < 16) {
                    for (int b = 0; b < 4; ++b) {
                        const int lo = 4 * b;
                        const uint32_t msk = n >= lo + 4 ? 0xFFFFFFFFu : n <= lo ? 0u : ((1u << (8 * (n - lo))) - 1u);
                        d[b] &= msk;
                    }
                }
                store_part(ct_out + off, n, d);
                x = le_to_block(d);
            }
        } else if ((uint32_t)q == m - 1) {
            x = U128{(uint64_t)alen * 8, (uint64_t)clen * 8};
        }
#if TLS_GHASH8 == 2
        acc = j == 0 ? x : gf_xor(gf_mul_tab8n(acc, tabs[6], t8, red8), x);  // Horner, H^64
#elif TLS_GHASH8
        acc = j == 0 ? x : gf_xor(gf_mul_tab8(acc, t8, red8), x);  // Horner, multiplier H^64
#else
        acc = j == 0 ? x : gf_xor(gf_mul_tab(acc, tabs[6]), x);  // Horner, multiplier H^64
#endif
    }
    // E(K, J0) lives in the lane that held the AAD block: lane pad % 64 of iteration pad / 64
    return Lanes{acc, {ej0[0], ej0[1], ej0[2], ej0[3]}, nz.resolve(), pad & 63};
}

// combine one wave's lanes: level t joins groups of 2^t lanes with multiplier H^(2^t); lane 0
// ends with the GHASH
[[maybe_unused]] __device__ inline U128 wave_tree(U128 acc, const U128 (*tabs)[16]) {
#pragma unroll
    for (int t = 0; t < 6; ++t) {
        const U128 right = shfl_down128(acc, 1 << t);
        acc = gf_xor(gf_mul_tab(acc, tabs[t]), right);
    }
    return gf_mul_tab(acc, tabs[0]);
}

// the same combine for the workgroup's four records at once, through LDS: at level t the
// 4 x 32 / 2^t pairs are spread over the workgroup's threads, so the four trees cost about two
// wave-wide multiplies per record instead of seven (s_acc[w][l] = record w, lane l)
template <int W>
[[maybe_unused]] __device__ inline void wg_tree(U128 (*s_acc)[64], const U128 (*tabs)[7][16]) {
#pragma unroll
    for (int t = 0; t < 6; ++t) {
        const uint32_t per = 32u >> t;  // pairs per record at this level
        if (threadIdx.x < W * per) {
            const uint32_t w = threadIdx.x / per, p = threadIdx.x % per;
            const uint32_t l = p << (t + 1), r = l + (1u << t);
            s_acc[w][l] = gf_xor(gf_mul_tab(s_acc[w][l], tabs[w][t]), s_acc[w][r]);
        }
        __syncthreads();
    }
    if (threadIdx.x < W) s_acc[threadIdx.x][0] = gf_mul_tab(s_acc[threadIdx.x][0], tabs[threadIdx.x][0]);
    __syncthreads();
}

// tag from the GHASH (valid in lane 0): SEAL stores it after the ciphertext, OPEN compares
template <bool SEAL>
__device__ CryptOut gcm_finish(const Lanes& L, U128 acc, const uint8_t* ct_in, uint8_t* ct_out,
                               uint32_t clen) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t last_nz = L.last_nz;
    uint32_t e[4];
    for (int b = 0; b < 4; ++b) e[b] = __shfl(L.ej0[b], L.src_lane, 64);
    const U128 tag{acc.hi ^ (((uint64_t)e[0] << 32) | e[1]), acc.lo ^ (((uint64_t)e[2] << 32) | e[3])};
    CryptOut r{false, 0};
    if (SEAL) {
        if (lane == 0) {
            const uint32_t w[4] = {bswap32((uint32_t)(tag.hi >> 32)), bswap32((uint32_t)tag.hi),
                                   bswap32((uint32_t)(tag.lo >> 32)), bswap32((uint32_t)tag.lo)};
            store_part(ct_out + clen, 16, w);
        }
        return r;
    }
    uint32_t t4[4];
    load_part(ct_in + clen, 0, 16, t4);
    const U128 want = le_to_block(t4);
    r.tag_ok = want.hi == tag.hi && want.lo == tag.lo;  // lane 0's tag is the valid one
    // wave max of last_nz
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(last_nz, d, 64);
        if (o > last_nz) last_nz = o;
    }
    r.last_nz = last_nz;
    return r;
}

// ---- ChaCha20-Poly1305 (RFC 8439) -------------------------------------------------------
//
// One wavefront per record, like AES-GCM.  ChaCha20: lane l of round j produces the 64-byte
// keystream block of ciphertext chunk 64 j + l (counter chunk + 1): twenty ARX rounds in
// registers, no tables.  The chunk's ciphertext (read, or produced when sealing) goes to a
// 4 KiB LDS window per wave, from which Poly1305 reads it with a 16-byte-block-per-lane
// mapping: ciphertext block k -> lane k % 64.  Poly1305 in radix 2^26 (five limbs, 25
// 32x32->64 multiplies per block): each lane runs Horner with multiplier r^64 over its blocks,
// the AAD block is folded into lane 0's first step (multiplier r), and the lanes combine in a
// shuffle tree after a rotation that orders them by exponent; the length block ends it.

struct P130 {  // a Poly1305 field element, radix 2^26 (limbs may exceed 26 bits between carries)
    uint32_t h[5];
};

__device__ inline P130 p_from_le16(const uint32_t w[4], uint32_t hibit) {
    P130 r;
    r.h[0] = w[0] & 0x3ffffff;
    r.h[1] = ((w[0] >> 26) | (w[1] << 6)) & 0x3ffffff;
    r.h[2] = ((w[1] >> 20) | (w[2] << 12)) & 0x3ffffff;
    r.h[3] = ((w[2] >> 14) | (w[3] << 18)) & 0x3ffffff;
    r.h[4] = (w[3] >> 8) | hibit;
    return r;
}

__device__ inline P130 p_add(P130 a, const P130& b) {
#pragma unroll
    for (int i = 0; i < 5; ++i) a.h[i] += b.h[i];
    return a;
}

// a * b mod 2^130 - 5, result limbs carried (h1 may carry one extra bit)
__device__ inline P130 p_mul(const P130& a, const P130& b) {
    const uint32_t b1s = b.h[1] * 5, b2s = b.h[2] * 5, b3s = b.h[3] * 5, b4s = b.h[4] * 5;
    auto m = [](uint32_t x, uint32_t y) { return (uint64_t)x * y; };
    uint64_t d0 = m(a.h[0], b.h[0]) + m(a.h[1], b4s) + m(a.h[2], b3s) + m(a.h[3], b2s) + m(a.h[4], b1s);
    uint64_t d1 = m(a.h[0], b.h[1]) + m(a.h[1], b.h[0]) + m(a.h[2], b4s) + m(a.h[3], b3s) + m(a.h[4], b2s);
    uint64_t d2 = m(a.h[0], b.h[2]) + m(a.h[1], b.h[1]) + m(a.h[2], b.h[0]) + m(a.h[3], b4s) + m(a.h[4], b3s);
    uint64_t d3 = m(a.h[0], b.h[3]) + m(a.h[1], b.h[2]) + m(a.h[2], b.h[1]) + m(a.h[3], b.h[0]) + m(a.h[4], b4s);
    uint64_t d4 = m(a.h[0], b.h[4]) + m(a.h[1], b.h[3]) + m(a.h[2], b.h[2]) + m(a.h[3], b.h[1]) + m(a.h[4], b.h[0]);
    P130 r;
    uint64_t c = d0 >> 26;
    r.h[0] = (uint32_t)d0 & 0x3ffffff;
    d1 += c, c = d1 >> 26, r.h[1] = (uint32_t)d1 & 0x3ffffff;
    d2 += c, c = d2 >> 26, r.h[2] = (uint32_t)d2 & 0x3ffffff;
    d3 += c, c = d3 >> 26, r.h[3] = (uint32_t)d3 & 0x3ffffff;
    d4 += c, c = d4 >> 26, r.h[4] = (uint32_t)d4 & 0x3ffffff;
    const uint64_t t = (uint64_t)r.h[0] + c * 5;
    r.h[0] = (uint32_t)t & 0x3ffffff;
    r.h[1] += (uint32_t)(t >> 26);
    return r;
}

// (h mod 2^130 - 5) + s mod 2^128, as four little-endian words (RFC 8439 §2.5.1 final step)
__device__ inline void p_tag(P130 h, const uint32_t s[4], uint32_t out[4]) {
    uint32_t c;
    for (int pass = 0; pass < 2; ++pass) {  // two full carry passes: every limb < 2^26
        c = h.h[0] >> 26, h.h[0] &= 0x3ffffff, h.h[1] += c;
        c = h.h[1] >> 26, h.h[1] &= 0x3ffffff, h.h[2] += c;
        c = h.h[2] >> 26, h.h[2] &= 0x3ffffff, h.h[3] += c;
        c = h.h[3] >> 26, h.h[3] &= 0x3ffffff, h.h[4] += c;
        c = h.h[4] >> 26, h.h[4] &= 0x3ffffff, h.h[0] += c * 5;
    }
    c = h.h[0] >> 26, h.h[0] &= 0x3ffffff, h.h[1] += c;
    // g = h + 5 - 2^130; take g when it does not borrow (h >= p)
    uint32_t g[5];
    c = h.h[0] + 5, g[0] = c & 0x3ffffff, c >>= 26;
    c += h.h[1], g[1] = c & 0x3ffffff, c >>= 26;
    c += h.h[2], g[2] = c & 0x3ffffff, c >>= 26;
    c += h.h[3], g[3] = c & 0x3ffffff, c >>= 26;
    g[4] = h.h[4] + c - (1u << 26);
    const uint32_t keep_g = (g[4] >> 31) - 1u;  // all ones if g did not borrow
    for (int i = 0; i < 5; ++i) h.h[i] = (h.h[i] & ~keep_g) | (g[i] & keep_g);
    const uint32_t w0 = h.h[0] | (h.h[1] << 26), w1 = (h.h[1] >> 6) | (h.h[2] << 20);
    const uint32_t w2 = (h.h[2] >> 12) | (h.h[3] << 14), w3 = (h.h[3] >> 18) | (h.h[4] << 8);
    uint64_t f = (uint64_t)w0 + s[0];
    out[0] = (uint32_t)f;
    f = (uint64_t)w1 + s[1] + (f >> 32), out[1] = (uint32_t)f;
    f = (uint64_t)w2 + s[2] + (f >> 32), out[2] = (uint32_t)f;
    f = (uint64_t)w3 + s[3] + (f >> 32), out[3] = (uint32_t)f;
}

__device__ inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// RFC 8439 §2.3 block function: x[16] = keystream words (little-endian byte order)
__device__ inline void chacha_block(const uint32_t* __restrict__ key, uint32_t counter,
                                    const uint32_t nonce[3], uint32_t x[16]) {
    uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                       key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                       counter, nonce[0], nonce[1], nonce[2]};
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = st[i];
#define CQR(a, b, c, d)                                                                       \
    x[a] += x[b], x[d] = rotl(x[d] ^ x[a], 16), x[c] += x[d], x[b] = rotl(x[b] ^ x[c], 12),  \
    x[a] += x[b], x[d] = rotl(x[d] ^ x[a], 8), x[c] += x[d], x[b] = rotl(x[b] ^ x[c], 7)
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        CQR(0, 4, 8, 12); CQR(1, 5, 9, 13); CQR(2, 6, 10, 14); CQR(3, 7, 11, 15);
        CQR(0, 5, 10, 15); CQR(1, 6, 11, 12); CQR(2, 7, 8, 13); CQR(3, 4, 9, 14);
    }
#undef CQR
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] += st[i];
}

__device__ inline P130 shfl_p(const P130& v, int src) {
    P130 r;
#pragma unroll
    for (int i = 0; i < 5; ++i) r.h[i] = __shfl(v.h[i], src, 64);
    return r;
}

// One record on one wave.  OPEN: ct[0, clen) -> content dst[0, wlen), tag compared with
// ct[clen, +16); SEAL: plaintext from (src, src_n, inner_type) -> ciphertext at ct_out, tag
// stored after it.  aad16: the AAD block (<= 13 bytes) as four little-endian words.

template <bool SEAL>
__device__ CryptOut chacha_record(const KeySched* __restrict__ ks, const uint32_t nonce[3],
                                  const uint32_t aad16[4], uint32_t alen, const uint8_t* ct_in,
                                  uint8_t* ct_out, uint32_t clen, uint8_t* dst, uint32_t wlen,
                                  const uint8_t* src, uint32_t src_n, uint32_t inner_type,
                                  bool is13, uint8_t* win) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t* __restrict__ key = ks->rk;
    // one-time Poly1305 key: block 0 (every lane computes it: one uniform extra block)
    uint32_t x[16];
    chacha_block(key, 0, nonce, x);
    // wave-uniform: held in scalar registers (readfirstlane), freeing vector registers
    const uint32_t rw[4] = {x[0] & 0x0fffffffu, x[1] & 0x0ffffffcu, x[2] & 0x0ffffffcu, x[3] & 0x0ffffffcu};
    uint32_t sw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) sw[i] = __builtin_amdgcn_readfirstlane(x[4 + i]);
    P130 pr[7];  // r^(2^t), t = 0..6
    pr[0] = p_from_le16(rw, 0);
#pragma unroll
    for (int t = 1; t < 7; ++t) pr[t] = p_mul(pr[t - 1], pr[t - 1]);
#if TLS_POLY_SGPR
#pragma unroll
    for (int t = 0; t < 7; ++t)
#pragma unroll
        for (int i = 0; i < 5; ++i) pr[t].h[i] = __builtin_amdgcn_readfirstlane(pr[t].h[i]);
#endif
    const uint32_t nct = (clen + 15) / 16;       // ciphertext Poly blocks
    const uint32_t nchunk = (clen + 63) / 64;    // ChaCha blocks (counter 1 ..)
    const uint32_t J = (nchunk + 63) / 64;       // rounds of 64 chunks = 4 KiB of ciphertext
    P130 acc{{0, 0, 0, 0, 0}};
    LastNz nz{0, {0, 0, 0, 0}};
    for (uint32_t j = 0; j < J; ++j) {
        const uint32_t chunk = 64 * j + lane;
        const uint32_t off = 64 * chunk;
        // ChaCha20 over the lane's 64-byte chunk.  Full chunks (all but a record's last) load
        // their 64 bytes unconditionally before the block function, so the loads' latency runs
        // under the twenty rounds; the byte-exact path below handles the last chunk.  (A variant
        // that loaded the next round's chunk a round ahead measured 22% slower.)
        uint32_t d[16];
        if (chunk < nchunk && off + 64 <= (SEAL ? src_n : clen)) {
            uint32_t in[16];
            const uint8_t* ip = (SEAL ? src : ct_in) + off;
#pragma unroll
            for (int v = 0; v < 4; ++v) __builtin_memcpy(in + 4 * v, ip + 16 * v, 16);
            __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of the rounds
            chacha_block(key, chunk + 1, nonce, x);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint32_t o = off + 16 * v;
                uint32_t w[4];
#pragma unroll
                for (int b = 0; b < 4; ++b) w[b] = in[4 * v + b] ^ x[4 * v + b];
                if (!SEAL) {  // w = plaintext; Poly1305 reads the ciphertext
                    if (is13) nz.see(o, w);
                    if (o + 16 <= wlen) __builtin_memcpy(dst + o, w, 16);
                    else if (o < wlen) store_part(dst + o, (int)(wlen - o), w);
#pragma unroll
                    for (int b = 0; b < 4; ++b) d[4 * v + b] = in[4 * v + b];
                } else {      // w = ciphertext
                    __builtin_memcpy(ct_out + o, w, 16);
#pragma unroll
                    for (int b = 0; b < 4; ++b) d[4 * v + b] = w[b];
                }
            }
        } else if (chunk < nchunk) {
            chacha_block(key, chunk + 1, nonce, x);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint32_t o = off + 16 * v;
                const int n = o >= clen ? 0 : (clen - o < 16 ? (int)(clen - o) : 16);
                uint32_t w[4] = {0, 0, 0, 0};
                if (!SEAL) {
                    if (n) load_part(ct_in + o, 0, n, w);
                    uint32_t pt[4];
                    for (int b = 0; b < 4; ++b) pt[b] = w[b] ^ x[4 * v + b];
                    if (n < 16) {
                        for (int b = 0; b < 4; ++b) {
                            const int lo = 4 * b;
                            pt[b] &= n >= lo + 4 ? 0xFFFFFFFFu : n <= lo ? 0u : ((1u << (8 * (n - lo))) - 1u);
                        }
                    }
                    if (is13) nz.see(o, pt);
                    if (n && o < wlen) store_part(dst + o, wlen - o < 16 ? (int)(wlen - o) : 16, pt);
                } else {
                    const int cn = src_n > o ? (src_n - o < 16 ? (int)(src_n - o) : 16) : 0;
                    if (cn) load_part(src + o, 0, cn, w);
                    if (is13 && src_n >= o && src_n < o + 16) {
                        const uint32_t bq = src_n - o;
                        w[bq >> 2] |= inner_type << (8 * (bq & 3));
                    }
                    for (int b = 0; b < 4; ++b) w[b] ^= x[4 * v + b];
                    if (n < 16) {
                        for (int b = 0; b < 4; ++b) {
                            const int lo = 4 * b;
                            w[b] &= n >= lo + 4 ? 0xFFFFFFFFu : n <= lo ? 0u : ((1u << (8 * (n - lo))) - 1u);
                        }
                    }
                    if (n) store_part(ct_out + o, n, w);
                }
                d[4 * v] = w[0], d[4 * v + 1] = w[1], d[4 * v + 2] = w[2], d[4 * v + 3] = w[3];
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) d[i] = 0;
        }
        // the round's 4 KiB of ciphertext through LDS: chunk order in, block-per-lane out
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int v = 0; v < 4; ++v)
            *reinterpret_cast<uint4*>(win + 64 * lane + 16 * v) = uint4{d[4 * v], d[4 * v + 1], d[4 * v + 2], d[4 * v + 3]};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t k = 256 * j + 64 * q + lane;  // ciphertext block
            if (k < nct) {
                const uint4 c4 = *reinterpret_cast<const uint4*>(win + 16 * (64 * q + lane));
                const uint32_t cw[4] = {c4.x, c4.y, c4.z, c4.w};
                P130 c = p_from_le16(cw, 1u << 24);
                if (k == 0) {  // lane 0's first block: the AAD block comes first (multiplier r)
                    const P130 a = p_from_le16(aad16, 1u << 24);
                    c = p_add(p_mul(a, pr[0]), c);
                }
                acc = (k < 64) ? c : p_add(p_mul(acc, pr[6]), c);
            }
        }
    }
    // Tag = (T r + c_LEN) r with T = c_AAD r^nct + sum_k c_k r^(nct-1-k).  Lane l's Horner sum
    // A_l ends at its last block K_l, so T = sum_l A_l r^(nct-1-K_l); with R = nct - 64 (Jb-1)
    // blocks in the last round that exponent is (R - 1 - l) mod 64: every value 0..63 once.
    // Rank i = 63 - exponent is lane (i + R) mod 64, and a 6-level tree over ranks with
    // multipliers r^(2^t) leaves T in lane 0.
    P130 total;
    if (nct == 0) {
        total = p_mul(p_from_le16(aad16, 1u << 24), pr[0]);  // T = c_AAD
    } else {
        const uint32_t R = nct - 64 * ((nct - 1) / 64);
        P130 b = shfl_p(acc, (int)((lane + R) & 63));
#pragma unroll
        for (int t = 0; t < 6; ++t) {
            P130 right;
#pragma unroll
            for (int i = 0; i < 5; ++i) right.h[i] = __shfl_down(b.h[i], 1 << t, 64);
            b = p_add(p_mul(b, pr[t]), right);
        }
        total = p_mul(b, pr[0]);  // T r
    }
    const uint32_t lens[4] = {alen, 0, clen, 0};
    total = p_mul(p_add(total, p_from_le16(lens, 1u << 24)), pr[0]);
    uint32_t tag[4];
    p_tag(total, sw, tag);
    CryptOut r{false, 0};
    if (SEAL) {
        if (lane == 0) store_part(ct_out + clen, 16, tag);
        return r;
    }
    uint32_t t4[4];
    load_part(ct_in + clen, 0, 16, t4);
    r.tag_ok = t4[0] == tag[0] && t4[1] == tag[1] && t4[2] == tag[2] && t4[3] == tag[3];
    uint32_t last_nz = nz.resolve();
#pragma unroll
    for (int dd = 32; dd >= 1; dd >>= 1) {
        const uint32_t o = __shfl_xor(last_nz, dd, 64);
        if (o > last_nz) last_nz = o;
    }
    r.last_nz = last_nz;
    return r;
}

__device__ inline void load_tables(const KeySched* ks, U128 (*tabs)[16]) {
    const uint32_t lane = threadIdx.x & 63;
    const uint4* s = reinterpret_cast<const uint4*>(ks->tab);
    uint4* d = reinterpret_cast<uint4*>(tabs);
    for (uint32_t i = lane; i < 7 * 16; i += 64) d[i] = s[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <uint32_t COPIES = TLS_TE_COPIES>
__device__ inline void fill_te(const uint32_t* te0, uint32_t* te) {
    constexpr uint32_t sh = COPIES == 64 ? 6 : COPIES == 32 ? 5 : COPIES == 16 ? 4 : 3;
    for (uint32_t i = threadIdx.x; i < 256 * COPIES; i += blockDim.x) te[i] = te0[i >> sh];
    __syncthreads();
}

#ifndef TLS_WG_TREE
#define TLS_WG_TREE 1      // 1: the lane combine of the workgroup's 4 records shared through LDS
#endif

// Packed ChaCha20-Poly1305 open for records up to 8 KiB: 64 / SEG consecutive work items
// share one wave, SEG lanes per record (segment k = lanes [k SEG, (k+1) SEG)), so a
// small record no longer costs a whole wave round of the block function plus its own one-time
// key, key powers and lane combine.  Same structure as chacha_record within each segment: lane
// u of round j takes chunk SEG j + u, the round's ciphertext goes through the wave's LDS window,
// Poly1305 block b of the record is Horner-accumulated by lane b % SEG (multiplier r^SEG),
// and the segment's lanes combine after the rotation by R = nct mod SEG in log2(SEG) shuffle
// levels confined to the segment.  Record parameters live in vector registers (they differ
// between segments).
// kPack: the record groups both AEADs route by (a group holding a long record goes to the
// one-record-per-wave kernel); TLS_CC_SEG: lanes per record in the packed ChaCha20-Poly1305
// kernel (16 records per wave at 4: a 256-byte record has four 64-byte chunks, so 16-lane
// segments left 12 lanes idle in the block function)
constexpr int kPack = 4;
#ifndef TLS_CC_SEG
#define TLS_CC_SEG 4
#endif
constexpr int kCcSeg = TLS_CC_SEG;
constexpr int kCcSegLog = kCcSeg == 16 ? 4 : kCcSeg == 8 ? 3 : 2;
constexpr int kCcPackW = 64 / kCcSeg;  // records per wave
static_assert((1 << kCcSegLog) == kCcSeg && kCcPackW % kPack == 0, "ChaCha segment size");

template <int SEG>
__device__ inline P130 shfl_seg(const P130& v, int src) {
    P130 r;
#pragma unroll
    for (int i = 0; i < 5; ++i) r.h[i] = __shfl(v.h[i], src, SEG);
    return r;
}

// record status (lane u == 0 of each segment; open_status's rules)
__device__ inline void open_status_at(const TlsArgs& a, uint32_t r, const CryptOut& co, bool is13,
                                      uint32_t clen, uint32_t outer_type) {
    int32_t st;
    uint32_t type = 0, cl = 0;
    if (!co.tag_ok) {
        st = UVHTTP_TLS_REC_ERR_BAD_MAC;
    } else if (is13) {
        if (co.last_nz == 0) {
            st = UVHTTP_TLS_REC_ERR_EMPTY;
        } else {
            type = co.last_nz & 0xFF;
            cl = (co.last_nz >> 8) - 1;
            st = type == 23 ? UVHTTP_TLS_REC_OK : UVHTTP_TLS_REC_CONTROL;
        }
    } else {
        type = outer_type;
        cl = clen;
        st = type == 23 ? UVHTTP_TLS_REC_OK : UVHTTP_TLS_REC_CONTROL;
    }
    a.work[r].status = st;
    a.work[r].type = type;
    a.work[r].content_len = cl;
}

// does group g (work items [g kPack, g kPack + kPack)) hold a record of `cipher` too long to
// pack?  (wave-uniform; the per-record and the packed kernel of a cipher decide the same way:
// only fields no kernel rewrites are read — the walk's header status, the length, the key —
// so a record the first kernel already opened, whatever its outcome, cannot move its group)
__device__ inline bool group_has_long(const TlsArgs& a, uint32_t g, uint32_t n,
                                      uint32_t cipher = UVHTTP_TLS_CIPHER_CHACHA20_POLY1305) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lim = cipher == UVHTTP_TLS_CIPHER_AES_GCM ? kPackMaxLenAes : kPackMaxLen;
    bool big = false;
    if (lane < kPack && g * kPack + lane < n) {
        const RecWork w = a.work[g * kPack + lane];
        big = w.walk_status == 0 && w.len > lim && a.sched[w.key].cipher == cipher;
    }
    return __builtin_amdgcn_readfirstlane(__ballot(big) != 0 ? 1u : 0u) != 0;
}

// records r0 .. r0 + 64/SEG - 1, each skipped when its group of kPack holds a long ChaCha
// record (that group goes to k_tls_open_chacha)
template <int SEG, int LOG>
__device__ void chacha_open_packed(const TlsArgs& a, uint32_t r0, uint8_t* win) {
    const uint32_t lane = threadIdx.x & 63, k = lane / SEG, u = lane % SEG;
    const uint32_t r = r0 + k;
    const uint32_t n = a.n_total[0];
    bool big = false;
    if (lane < 64u / SEG && r0 + lane < n) {
        const RecWork wb = a.work[r0 + lane];
        big = wb.walk_status == 0 && wb.len > kPackMaxLen &&
              a.sched[wb.key].cipher == UVHTTP_TLS_CIPHER_CHACHA20_POLY1305;
    }
    const uint64_t bigm = __ballot(big);
    const uint32_t gfirst = (r0 / kPack) * kPack;  // (r0 is a multiple of kPack)
    const bool grp_long = ((bigm >> ((r - gfirst) / kPack * kPack)) & ((1ull << kPack) - 1)) != 0;
    bool act = r < n && !grp_long;
    RecWork w;
    if (act) {
        w = a.work[r];
        act = w.status == 0 && a.sched[w.key].cipher == UVHTTP_TLS_CIPHER_CHACHA20_POLY1305;
    }
    uint32_t key[8], nonce[3] = {0, 0, 0}, aad16[4] = {0, 0, 0, 0};
    uint32_t clen = 0, wlen = 0, alen = 0, otype = 0;
    bool is13 = false;
    const uint8_t* rec = a.wire;
    uint8_t* dst = a.out;
#pragma unroll
    for (int i = 0; i < 8; ++i) key[i] = 0;
    if (act) {
        const KeySched* ks = a.sched + w.key;
#pragma unroll
        for (int i = 0; i < 8; ++i) key[i] = ks->rk[i];
        is13 = ks->version == UVHTTP_TLS_VERSION_13;
        nonce[0] = ks->iv[0];
        nonce[1] = ks->iv[1] ^ bswap32((uint32_t)(w.seq >> 32));
        nonce[2] = ks->iv[2] ^ bswap32((uint32_t)w.seq);
        rec = a.wire + w.rec_off;
        dst = a.out + w.spec_off;
        clen = w.len - 16;
        otype = rec[0];
        if (is13) {
            load_part(rec, 0, 5, aad16);
        } else {
            aad16[0] = bswap32((uint32_t)(w.seq >> 32));
            aad16[1] = bswap32((uint32_t)w.seq);
            aad16[2] = otype | 0x030300u | ((clen >> 8) << 24);
            aad16[3] = clen & 0xFF;
        }
        wlen = is13 ? (clen > 0 ? clen - 1 : 0) : clen;
        alen = is13 ? 5u : 13u;
    }
    const uint8_t* ct_in = rec + 5;
    uint32_t x[16];
    chacha_block(key, 0, nonce, x);  // the segment's one-time key
    const uint32_t rw[4] = {x[0] & 0x0fffffffu, x[1] & 0x0ffffffcu, x[2] & 0x0ffffffcu, x[3] & 0x0ffffffcu};
    const uint32_t sw[4] = {x[4], x[5], x[6], x[7]};
    P130 pr[LOG + 1];  // r^(2^t), t = 0..log2(SEG)
    pr[0] = p_from_le16(rw, 0);
#pragma unroll
    for (int t = 1; t <= LOG; ++t) pr[t] = p_mul(pr[t - 1], pr[t - 1]);
    const uint32_t nct = (clen + 15) / 16;
    const uint32_t nchunk = (clen + 63) / 64;
    uint32_t J = (nchunk + SEG - 1) / SEG;  // rounds this segment needs; the wave runs the max
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(J, d, 64);
        if (o > J) J = o;
    }
    J = __builtin_amdgcn_readfirstlane(J);
    P130 acc{{0, 0, 0, 0, 0}};
    LastNz nz{0, {0, 0, 0, 0}};
    for (uint32_t j = 0; j < J; ++j) {
        const uint32_t chunk = SEG * j + u;
        const uint32_t off = 64 * chunk;
        uint32_t d[16];
        if (chunk < nchunk) {
            const bool full = off + 64 <= clen;
            uint32_t in[16];
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint32_t o = off + 16 * v;
                const int nb = o >= clen ? 0 : (clen - o < 16 ? (int)(clen - o) : 16);
                if (full) __builtin_memcpy(in + 4 * v, ct_in + o, 16);
                else load_part(ct_in + o, 0, nb, in + 4 * v);
            }
            chacha_block(key, chunk + 1, nonce, x);
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const uint32_t o = off + 16 * v;
                const int nb = o >= clen ? 0 : (clen - o < 16 ? (int)(clen - o) : 16);
                uint32_t pt[4];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int lo = 4 * b;
                    pt[b] = (in[4 * v + b] ^ x[4 * v + b]) &
                            (nb >= lo + 4 ? 0xFFFFFFFFu : nb <= lo ? 0u : ((1u << (8 * (nb - lo))) - 1u));
                    d[4 * v + b] = in[4 * v + b];
                }
                if (is13) nz.see(o, pt);
                if (o + 16 <= wlen) __builtin_memcpy(dst + o, pt, 16);
                else if (nb && o < wlen) store_part(dst + o, (int)(wlen - o), pt);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) d[i] = 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int v = 0; v < 4; ++v)
            *reinterpret_cast<uint4*>(win + 64 * lane + 16 * v) = uint4{d[4 * v], d[4 * v + 1], d[4 * v + 2], d[4 * v + 3]};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t blk = 4 * SEG * j + SEG * q + u;  // the record's Poly1305 block
            if (blk < nct) {
                const uint4 c4 = *reinterpret_cast<const uint4*>(win + 64 * SEG * k + 16 * (SEG * q + u));
                const uint32_t cw[4] = {c4.x, c4.y, c4.z, c4.w};
                P130 c = p_from_le16(cw, 1u << 24);
                if (blk == 0) c = p_add(p_mul(p_from_le16(aad16, 1u << 24), pr[0]), c);
                acc = blk < SEG ? c : p_add(p_mul(acc, pr[LOG]), c);
            }
        }
    }
    // T = sum over the segment's lanes of A_u r^((R - 1 - u) mod SEG); rank i = lane (i + R)
    const uint32_t R = nct ? nct - SEG * ((nct - 1) / SEG) : 0;
    P130 b = shfl_seg<SEG>(acc, (int)((u + R) & (SEG - 1)));
#pragma unroll
    for (int t = 0; t < LOG; ++t) {
        P130 right;
#pragma unroll
        for (int i = 0; i < 5; ++i) right.h[i] = __shfl_down(b.h[i], 1 << t, SEG);
        b = p_add(p_mul(b, pr[t]), right);
    }
    P130 total = nct ? p_mul(b, pr[0]) : p_mul(p_from_le16(aad16, 1u << 24), pr[0]);
    const uint32_t lens[4] = {alen, 0, clen, 0};
    total = p_mul(p_add(total, p_from_le16(lens, 1u << 24)), pr[0]);
    uint32_t tag[4];
    p_tag(total, sw, tag);
    uint32_t last_nz = nz.resolve();
#pragma unroll
    for (int d = SEG / 2; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(last_nz, d, SEG);
        if (o > last_nz) last_nz = o;
    }
    if (act && u == 0) {
        uint32_t t4[4];
        load_part(ct_in + clen, 0, 16, t4);
        CryptOut co{t4[0] == tag[0] && t4[1] == tag[1] && t4[2] == tag[2] && t4[3] == tag[3], last_nz};
        open_status_at(a, r, co, is13, clen, otype);
    }
}

// Packed AES-GCM: the records of a group of short records share one wave, SEG lanes per
// record (segment k = lanes [k SEG, (k+1) SEG)).  Segment k stages its key's round keys and the
// 4-bit GHASH tables of H, H^2 ... H^SEG in LDS (the record's key differs per segment); lane u of
// round j takes GHASH position SEG j + u of the record's left-padded sequence (AAD, ciphertext
// blocks, length block), runs AES-CTR for it from the shared T-table and Horner with multiplier
// H^SEG; the segment's lanes combine in log2(SEG) shuffle levels (H, H^2, ...) and a final x H.
// SEG = 4 (sixteen records per wave): per record the 4-bit-table multiplies of the lane tree
// and the idle AES lanes of the last round cost less than with 16 lanes, so every packed size
// gets cheaper (modelled per 256-byte record: ~25 k lane operations at SEG 4 vs ~69 k at 16).
template <int SEG>
__device__ inline U128 shfl_down128_w(U128 v, int d) {
    const uint32_t a = __shfl_down((uint32_t)v.hi, d, SEG), b = __shfl_down((uint32_t)(v.hi >> 32), d, SEG);
    const uint32_t c = __shfl_down((uint32_t)v.lo, d, SEG), e = __shfl_down((uint32_t)(v.lo >> 32), d, SEG);
    return U128{((uint64_t)b << 32) | a, ((uint64_t)e << 32) | c};
}

#ifndef TLS_AES_SEG
#define TLS_AES_SEG 4
#endif
constexpr int kAesSeg = TLS_AES_SEG;         // lanes per record in k_tls_open_aes_packed
constexpr int kAesSegLog = kAesSeg == 16 ? 4 : kAesSeg == 8 ? 3 : kAesSeg == 4 ? 2 : 1;
constexpr int kAesPackW = 64 / kAesSeg;      // records per wave
#ifndef TLS_RK_STRIDE
#define TLS_RK_STRIDE 60   // words per record of staged round keys (60 = AES-256's schedule):
                           // record k starts 4 k banks lower, so the records of a ds_read_b128
                           // lane group hit different banks (64: 4-way conflicts)
#endif
constexpr int kRkStride = TLS_RK_STRIDE;
#ifndef TLS_PACK_GTREE
#define TLS_PACK_GTREE 1   // 1: the lane combine of k_tls_open_aes_packed reads H^(2^t) from the
                           // key schedule in global memory; only H^SEG (Horner) is staged in LDS
#endif
constexpr int kPackTabs = TLS_PACK_GTREE ? 1 : kAesSegLog + 1;  // staged tables per record
#ifndef TLS_PACK_AES_WAVES
#define TLS_PACK_AES_WAVES 16  // waves per workgroup of k_tls_open_aes_packed (they share the T-table)
#endif
constexpr int kPackAesWaves = TLS_PACK_AES_WAVES;
constexpr int kPackAesWG = 64 * kPackAesWaves;
static_assert((1 << kAesSegLog) == kAesSeg && kAesPackW % kPack == 0, "AES segment size");

// records r0 .. r0 + 64/SEG - 1, each skipped when its group of kPack holds a long AES record
// (that group goes to k_tls_open)
template <int SEG, int LOG>
__device__ void aes_open_packed(const TlsArgs& a, uint32_t r0, const uint32_t* te, uint32_t (*s_rk)[kRkStride],
                                U128 (*s_tab)[kPackTabs][16]) {
    const uint32_t lane = threadIdx.x & 63, k = lane / SEG, u = lane % SEG;
    const uint32_t r = r0 + k;
    const uint32_t n = a.n_total[0];
    // long-record groups among the wave's records: lane l < 64/SEG looks at record r0 + l
    bool big = false;
    if (lane < 64u / SEG && r0 + lane < n) {
        const RecWork wb = a.work[r0 + lane];
        big = wb.walk_status == 0 && wb.len > kPackMaxLenAes && a.sched[wb.key].cipher == UVHTTP_TLS_CIPHER_AES_GCM;
    }
    const uint64_t bigm = __ballot(big);
    const uint32_t gfirst = (r0 / kPack) * kPack;  // (r0 is a multiple of kPack)
    const bool grp_long = ((bigm >> ((r - gfirst) / kPack * kPack)) & ((1ull << kPack) - 1)) != 0;
    bool act = r < n && !grp_long;
    RecWork w;
    if (act) {
        w = a.work[r];
        act = w.status == 0 && a.sched[w.key].cipher == UVHTTP_TLS_CIPHER_AES_GCM;
    }
    const KeySched* ks = a.sched + (act ? w.key : 0);
    if (act) {  // the segment's round keys and H^(2^t) tables, t = 0..LOG
        for (uint32_t i = u; i < 60; i += SEG) s_rk[k][i] = ks->rk[i];
#pragma unroll
        for (int i = 0; i < kPackTabs; ++i)
            for (uint32_t e = u; e < 16; e += SEG) s_tab[k][i][e] = ks->tab[TLS_PACK_GTREE ? LOG : i][e];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t nonce[3] = {0, 0, 0}, clen = 0, wlen = 0, alen = 0, nr = 10, otype = 0;
    U128 aad{0, 0};
    bool is13 = false;
    const uint8_t* rec = a.wire;
    const uint8_t* ct = a.wire;
    uint8_t* dst = a.out;
    if (act) {
        is13 = ks->version == UVHTTP_TLS_VERSION_13;
        nr = ks->nr;
        rec = a.wire + w.rec_off;
        dst = a.out + w.spec_off;
        otype = rec[0];
        if (is13) {
            nonce[0] = ks->iv[0];
            nonce[1] = ks->iv[1] ^ (uint32_t)(w.seq >> 32);
            nonce[2] = ks->iv[2] ^ (uint32_t)w.seq;
            uint32_t h[4];
            load_part(rec, 0, 5, h);
            aad = le_to_block(h);
            alen = 5;
            clen = w.len - 16;
            ct = rec + 5;
        } else {
            uint32_t ex[4];
            load_part(rec + 5, 0, 8, ex);
            nonce[0] = ks->iv[0];
            nonce[1] = bswap32(ex[0]);
            nonce[2] = bswap32(ex[1]);
            clen = w.len - 24;
            aad = U128{w.seq, ((uint64_t)otype << 56) | (0x0303ull << 40) | ((uint64_t)clen << 24)};
            alen = 13;
            ct = rec + 13;
        }
        wlen = is13 ? (clen > 0 ? clen - 1 : 0) : clen;
    }
    const uint32_t nblk = (clen + 15) / 16;
    const uint32_t m = act ? nblk + 2 : 0;             // AAD, ciphertext blocks, length block
    const uint32_t Jr = (m + SEG - 1) / SEG;            // this segment's rounds
    const uint32_t pad = SEG * Jr - m;                  // left padding (< SEG)
    uint32_t J = Jr;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(J, d, 64);
        if (o > J) J = o;
    }
    J = __builtin_amdgcn_readfirstlane(J);
#if TLS_TE_COPIES == 64
    const uint32_t lane4 = lane << 2;  // (layout as in gcm_lanes)
    const uint8_t* te8 = reinterpret_cast<const uint8_t*>(te);
    auto te_lds = [&](uint32_t v, int k) {
        return *reinterpret_cast<const uint32_t*>(te8 + __builtin_amdgcn_perm(v, lane4, 0x0C0C0000u | ((4u + k) << 8)));
    };
#else
    const uint32_t lane_te = lane & (TLS_TE_COPIES - 1);
    auto te_lds = [&](uint32_t v, int k) { return te[(((v >> (8 * k)) & 0xFF) << kTeShift) | lane_te]; };
#endif
    U128 acc{0, 0};
    uint32_t ej0[4] = {0, 0, 0, 0};
    LastNz nz{0, {0, 0, 0, 0}};
    // rounds 1-2 of the record's counter blocks cached (packed records are far below 2^16 blocks)
    const CtrCache cc = ctr_cache(s_rk[k], nonce, te_lds);
    for (uint32_t j = 0; j < J; ++j) {
        const int32_t q = (int32_t)(SEG * j + u) - (int32_t)pad;
        uint32_t cb[4] = {nonce[0], nonce[1], nonce[2], q <= 0 ? 1u : (uint32_t)q + 1u};
        if (j < Jr) {  // (segments with fewer rounds idle)
            if (nr == 10)
                aes_ctr_cached<10>(s_rk[k], cc, cb[3], cb, te_lds);
            else
                aes_ctr_cached<14>(s_rk[k], cc, cb[3], cb, te_lds);
        }
        if (j >= Jr) continue;
        U128 x{0, 0};
        if (q == 0) {
            x = aad;
            ej0[0] = cb[0], ej0[1] = cb[1], ej0[2] = cb[2], ej0[3] = cb[3];
        } else if (q > 0 && (uint32_t)q <= nblk) {
            const uint32_t off = 16 * ((uint32_t)q - 1);
            const int nb = clen - off < 16 ? (int)(clen - off) : 16;
            uint32_t d[4];
            load_part(ct + off, 0, nb, d);
            x = le_to_block(d);
            uint32_t pt[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int lo = 4 * b;
                pt[b] = (d[b] ^ bswap32(cb[b])) &
                        (nb >= lo + 4 ? 0xFFFFFFFFu : nb <= lo ? 0u : ((1u << (8 * (nb - lo))) - 1u));
            }
            if (is13) nz.see(off, pt);
            if (off < wlen) store_part(dst + off, wlen - off < 16 ? (int)(wlen - off) : 16, pt);
        } else if ((uint32_t)q == m - 1) {
            x = U128{(uint64_t)alen * 8, (uint64_t)clen * 8};
        }
        acc = j == 0 ? x : gf_xor(gf_mul_tab<TLS_MUL_CHUNK>(acc, s_tab[k][kPackTabs - 1]), x);  // Horner, H^SEG
    }
    if constexpr (SEG == 4 && TLS_PACK_GTREE) {
        // lane u's sum takes H^(4 - u) (the tree below, unrolled: a0 H^4 + a1 H^3 + a2 H^2 +
        // a3 H): one multiply per lane instead of three, then two shuffle-XORs into lane 0
        const U128* tp = u == 0 ? ks->tab[2] : u == 1 ? ks->tab3 : u == 2 ? ks->tab[1] : ks->tab[0];
        acc = gf_mul_tab<TLS_MUL_CHUNK>(acc, tp);
        acc = gf_xor(acc, shfl_down128_w<SEG>(acc, 1));
        acc = gf_xor(acc, shfl_down128_w<SEG>(acc, 2));
    } else {
#pragma unroll
        for (int t = 0; t < LOG; ++t)
            acc = gf_xor(gf_mul_tab<TLS_MUL_CHUNK>(acc, TLS_PACK_GTREE ? ks->tab[t] : s_tab[k][t]), shfl_down128_w<SEG>(acc, 1 << t));
        acc = gf_mul_tab<TLS_MUL_CHUNK>(acc, TLS_PACK_GTREE ? ks->tab[0] : s_tab[k][0]);
    }
    uint32_t e[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) e[b] = __shfl(ej0[b], (int)pad, SEG);  // E(K, J0): round 0, lane pad
    const U128 tag{acc.hi ^ (((uint64_t)e[0] << 32) | e[1]), acc.lo ^ (((uint64_t)e[2] << 32) | e[3])};
    uint32_t last_nz = nz.resolve();
#pragma unroll
    for (int d = SEG / 2; d >= 1; d >>= 1) {
        const uint32_t o = __shfl_xor(last_nz, d, SEG);
        if (o > last_nz) last_nz = o;
    }
    if (act && u == 0) {
        uint32_t t4[4];
        load_part(ct + clen, 0, 16, t4);
        const U128 want = le_to_block(t4);
        const CryptOut co{want.hi == tag.hi && want.lo == tag.lo, last_nz};
        open_status_at(a, r, co, is13, clen, otype);
    }
}

// record status from the AEAD result (lane 0): TLS 1.3 type = last non-zero inner byte
__device__ inline void open_status(const TlsArgs& a, uint32_t r, const CryptOut& co, bool is13,
                                   uint32_t clen, uint32_t outer_type) {
    if ((threadIdx.x & 63) != 0) return;
    int32_t st;
    uint32_t type = 0, cl = 0;
    if (!co.tag_ok) {
        st = UVHTTP_TLS_REC_ERR_BAD_MAC;
    } else if (is13) {
        if (co.last_nz == 0) {
            st = UVHTTP_TLS_REC_ERR_EMPTY;
        } else {
            type = co.last_nz & 0xFF;
            cl = (co.last_nz >> 8) - 1;
            st = type == 23 ? UVHTTP_TLS_REC_OK : UVHTTP_TLS_REC_CONTROL;
        }
    } else {
        type = outer_type;
        cl = clen;
        st = type == 23 ? UVHTTP_TLS_REC_OK : UVHTTP_TLS_REC_CONTROL;
    }
    a.work[r].status = st;
    a.work[r].type = type;
    a.work[r].content_len = cl;
}

__global__ OPEN_ATTR void k_tls_open(TlsArgs a) {
    __shared__ uint32_t te[256 * TLS_TE_COPIES_REC];
    __shared__ U128 tabs[kOpenWaves][7][16];
#if TLS_GHASH8
    __shared__ U128 t8s[kOpenWaves][TLS_GHASH8 == 2 ? 16 : 256];
    U128* t8 = t8s[threadIdx.x >> 6];
#else
    U128* t8 = nullptr;
#endif
#if TLS_WG_TREE
    __shared__ U128 s_acc[kOpenWaves][64];
#endif
    __shared__ uint32_t red8[TLS_RED8 == 2 ? 32 : 256];
    if (!(a.n_total[2] & 32u)) return;  // no AES-GCM record too long to pack
    fill_red8(red8);
    fill_te<TLS_TE_COPIES_REC>(a.te0, te);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t n = a.n_total[0];
    uint32_t cur = 0xFFFFFFFFu, cur8 = 0xFFFFFFFFu;  // key slots of the wave's 4-bit / 8-bit tables
    // a wave takes a group of kPack records holding a long AES-GCM record (the others go to
    // k_tls_open_aes_packed) and opens them one per round; rounds are workgroup-uniform (the
    // shared combine has barriers); r is wave-uniform: readfirstlane makes the record and
    // key-schedule loads scalar
    for (uint32_t gb = blockIdx.x * kOpenWaves; gb * kPack < n; gb += gridDim.x * kOpenWaves) {
    const uint32_t g = __builtin_amdgcn_readfirstlane(gb + wave);
    const bool grp = g * kPack < n && group_has_long(a, g, n, UVHTTP_TLS_CIPHER_AES_GCM);
    for (uint32_t i = 0; i < kPack; ++i) {
        const uint32_t r = g * kPack + i;
        RecWork w;
        bool active = grp && r < n;
        if (active) {
            w = a.work[r];
            active = w.status == 0;  // header failure: nothing to open
        }
        Lanes L{U128{0, 0}, {0, 0, 0, 0}, 0, 0};
        const KeySched* ks = a.sched + (active ? w.key : 0);
        const uint8_t* rec = a.wire + (active ? w.rec_off : 0);
        bool is13 = false;
        uint32_t clen = 0;
        const uint8_t* ct = rec;
        if (active) active = ks->cipher == UVHTTP_TLS_CIPHER_AES_GCM;  // else k_tls_open_chacha
        if (active) {
            if (w.key != cur) {
                load_tables(ks, tabs[wave]);
                cur = w.key;
            }
            // the 8-bit table serves only the Horner steps of records over 62 blocks: a run of
            // small records under changing keys skips building it
            const uint32_t cl = w.len - (ks->version == UVHTTP_TLS_VERSION_13 ? 16u : 24u);
            if (TLS_GHASH8 && (cl + 15) / 16 + 2 > 64 && cur8 != w.key) {
                if (TLS_GHASH8 == 2) gf_table_x4(tabs[wave][6], t8);
                else gf_table8(tabs[wave][6], t8);
                cur8 = w.key;
            }
            is13 = ks->version == UVHTTP_TLS_VERSION_13;
            uint32_t nonce[3];
            U128 aad;
            uint32_t alen;
            if (is13) {
                nonce[0] = ks->iv[0];
                nonce[1] = ks->iv[1] ^ (uint32_t)(w.seq >> 32);
                nonce[2] = ks->iv[2] ^ (uint32_t)w.seq;
                uint32_t h[4];
                load_part(rec, 0, 5, h);
                aad = le_to_block(h);
                alen = 5;
                clen = w.len - 16;
                ct = rec + 5;
            } else {
                uint32_t ex[4];
                load_part(rec + 5, 0, 8, ex);
                nonce[0] = ks->iv[0];
                nonce[1] = bswap32(ex[0]);
                nonce[2] = bswap32(ex[1]);
                clen = w.len - 24;
                aad = U128{w.seq, ((uint64_t)rec[0] << 56) | (0x0303ull << 40) | ((uint64_t)clen << 24)};
                alen = 13;
                ct = rec + 13;
            }
            const uint32_t wlen = is13 ? (clen > 0 ? clen - 1 : 0) : clen;
            L = gcm_lanes<false>(ks, te, lane & (TLS_TE_COPIES_REC - 1), tabs[wave], t8, red8, nonce, aad,
                                 alen, ct, nullptr, clen, a.out + w.spec_off, wlen, nullptr, 0, 0,
                                 is13);
        }
#if TLS_WG_TREE
        // a round with no AES-GCM record in the workgroup (ChaCha20-Poly1305 records, header
        // failures) skips the combine: its serial multiplies are pure latency
        U128 ghash{0, 0};
        if (__syncthreads_or(active)) {
            s_acc[wave][lane] = L.acc;
            __syncthreads();
            wg_tree<kOpenWaves>(s_acc, tabs);
            ghash = s_acc[wave][0];
        }
#else
        const U128 ghash = active ? wave_tree(L.acc, tabs[wave]) : U128{0, 0};
#endif
        if (!active) continue;
        open_status(a, r, gcm_finish<false>(L, ghash, ct, nullptr, clen), is13, clen, rec[0]);
    }
    }
}

#ifndef TLS_PACK_AES_WPE
#define TLS_PACK_AES_WPE 4  // >0: amdgpu_waves_per_eu hint for k_tls_open_aes_packed
#endif
#if TLS_PACK_AES_WPE > 0
#define PACK_AES_ATTR __launch_bounds__(kPackAesWG) __attribute__((amdgpu_waves_per_eu(TLS_PACK_AES_WPE)))
#else
#define PACK_AES_ATTR __launch_bounds__(kPackAesWG)
#endif
__global__ PACK_AES_ATTR void k_tls_open_aes_packed(TlsArgs a) {
    __shared__ uint32_t te[256 * TLS_TE_COPIES];
    __shared__ uint32_t s_rk[kPackAesWaves][kAesPackW][kRkStride];
    __shared__ U128 s_tab[kPackAesWaves][kAesPackW][kPackTabs][16];
    if (!(a.n_total[2] & 16u)) return;  // no short AES-GCM record
    fill_te(a.te0, te);
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t n = a.n_total[0];
    for (uint32_t g = blockIdx.x * kPackAesWaves + wave; g * kAesPackW < n; g += gridDim.x * kPackAesWaves)
        aes_open_packed<kAesSeg, kAesSegLog>(a, g * kAesPackW, te, s_rk[wave], s_tab[wave]);
}

// ChaCha20-Poly1305 records (the AES-GCM kernel skips them): one wave per record, no shared
// tables and no workgroup barriers, so waves take records independently
__global__ CHACHA_ATTR void k_tls_open_chacha(TlsArgs a) {
    __shared__ uint4 wins[kCryptWaves][256];
    uint8_t* win = reinterpret_cast<uint8_t*>(wins[threadIdx.x >> 6]);
    if (!(a.n_total[2] & 8u)) return;  // no long ChaCha20-Poly1305 record
    const uint32_t n = a.n_total[0];
    // the record index is wave-uniform by construction (readfirstlane of the wave id): a
    // per-lane loop bound would make every branch of the record code divergent
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // groups of kPack consecutive records: a group holding a long ChaCha record is opened here
    // one record per wave, the others by k_tls_open_chacha_packed
    for (uint32_t g = blockIdx.x * kCryptWaves + wave; g * kPack < n; g += gridDim.x * kCryptWaves) {
        if (!group_has_long(a, g, n)) continue;
        for (uint32_t r = g * kPack; r < g * kPack + kPack && r < n; ++r) {
        const RecWork w = a.work[r];
        if (w.status != 0) continue;
        const KeySched* ks = a.sched + w.key;
        if (ks->cipher != UVHTTP_TLS_CIPHER_CHACHA20_POLY1305) continue;
        // RFC 8439 AEAD; nonce = iv XOR be64(seq) for TLS 1.3 and TLS 1.2 (RFC 7905)
        const uint8_t* rec = a.wire + w.rec_off;
        const bool is13 = ks->version == UVHTTP_TLS_VERSION_13;
        const uint32_t nonce[3] = {ks->iv[0], ks->iv[1] ^ bswap32((uint32_t)(w.seq >> 32)),
                                   ks->iv[2] ^ bswap32((uint32_t)w.seq)};
        const uint32_t clen = w.len - 16;
        uint32_t aad16[4];
        if (is13) {
            load_part(rec, 0, 5, aad16);
        } else {
            aad16[0] = bswap32((uint32_t)(w.seq >> 32));
            aad16[1] = bswap32((uint32_t)w.seq);
            aad16[2] = (uint32_t)rec[0] | 0x030300u | ((clen >> 8) << 24);
            aad16[3] = clen & 0xFF;
        }
        const uint32_t wlen = is13 ? (clen > 0 ? clen - 1 : 0) : clen;
        const CryptOut co = chacha_record<false>(ks, nonce, aad16, is13 ? 5u : 13u, rec + 5, nullptr,
                                                 clen, a.out + w.spec_off, wlen, nullptr, 0, 0, is13, win);
        open_status(a, r, co, is13, clen, rec[0]);
    }
    }
}

__global__ __launch_bounds__(kCryptWG) __attribute__((amdgpu_waves_per_eu(TLS_PACK_WPE))) void
k_tls_open_chacha_packed(TlsArgs a) {
    __shared__ uint4 wins[kCryptWaves][256];
    uint8_t* win = reinterpret_cast<uint8_t*>(wins[threadIdx.x >> 6]);
    if (!(a.n_total[2] & 4u)) return;  // no short ChaCha20-Poly1305 record
    const uint32_t n = a.n_total[0];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t g = blockIdx.x * kCryptWaves + wave; g * kCcPackW < n; g += gridDim.x * kCryptWaves)
        chacha_open_packed<kCcSeg, kCcSegLog>(a, g * kCcPackW, win);
}

// seal descriptor r checked against the contract (key slot, key, content size, buffers) and
// the AEAD a kernel handles; record sizes out
__device__ inline bool seal_prep(const SealArgs& a, uint32_t r, uint32_t cipher, uvhttp_tls_seal_t* sr,
                                 const KeySched** ks, bool* is13, uint32_t* clen, uint32_t* rlen) {
    *sr = a.recs[r];
    if (sr->key >= a.n_keys) return false;
    const KeySched* k = a.sched + sr->key;
    if (k->nr == 0 || k->cipher != cipher || sr->plain_len > 16384) return false;
    *ks = k;
    *is13 = k->version == UVHTTP_TLS_VERSION_13;
    *clen = sr->plain_len + (*is13 ? 1u : 0u);
    *rlen = *clen + 16 + explicit_len(k->version, cipher);
    return sr->out_off + 5 + *rlen <= a.out_cap && sr->src_off + sr->plain_len <= a.src_len;
}

__global__ OPEN_ATTR void k_tls_seal(SealArgs a) {
    __shared__ uint32_t te[256 * TLS_TE_COPIES_REC];
    __shared__ U128 tabs[kOpenWaves][7][16];
#if TLS_GHASH8
    __shared__ U128 t8s[kOpenWaves][TLS_GHASH8 == 2 ? 16 : 256];
    U128* t8 = t8s[threadIdx.x >> 6];
#else
    U128* t8 = nullptr;
#endif
#if TLS_WG_TREE
    __shared__ U128 s_acc[kOpenWaves][64];
#endif
    __shared__ uint32_t red8[TLS_RED8 == 2 ? 32 : 256];
    fill_red8(red8);
    fill_te<TLS_TE_COPIES_REC>(a.te0, te);
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t cur = 0xFFFFFFFFu, cur8 = 0xFFFFFFFFu;  // key slots of the wave's 4-bit / 8-bit tables
    for (uint32_t rb = blockIdx.x * kOpenWaves; rb < a.n; rb += gridDim.x * kOpenWaves) {
        const uint32_t r = __builtin_amdgcn_readfirstlane(rb + wave);
        uvhttp_tls_seal_t sr;
        const KeySched* ks = a.sched;
        bool is13 = false;
        uint32_t clen = 0, rlen = 0;
        bool active = r < a.n && seal_prep(a, r, UVHTTP_TLS_CIPHER_AES_GCM, &sr, &ks, &is13, &clen, &rlen);
        Lanes L{U128{0, 0}, {0, 0, 0, 0}, 0, 0};
        uint8_t* ct = a.out;
        if (active) {
            if (sr.key != cur) {
                load_tables(ks, tabs[wave]);
                cur = sr.key;
            }
            if (TLS_GHASH8 && (clen + 15) / 16 + 2 > 64 && cur8 != sr.key) {
                if (TLS_GHASH8 == 2) gf_table_x4(tabs[wave][6], t8);
                else gf_table8(tabs[wave][6], t8);
                cur8 = sr.key;
            }
            uint8_t* rec = a.out + sr.out_off;
            const uint32_t otype = is13 ? 23u : sr.type;
            uint32_t nonce[3];
            U128 aad;
            uint32_t alen;
            if (is13) {
                nonce[0] = ks->iv[0];
                nonce[1] = ks->iv[1] ^ (uint32_t)(sr.seq >> 32);
                nonce[2] = ks->iv[2] ^ (uint32_t)sr.seq;
                aad = U128{((uint64_t)otype << 56) | (0x0303ull << 40) | ((uint64_t)rlen << 24), 0};
                alen = 5;
                ct = rec + 5;
            } else {
                nonce[0] = ks->iv[0];
                nonce[1] = (uint32_t)(sr.seq >> 32);
                nonce[2] = (uint32_t)sr.seq;
                aad = U128{sr.seq, ((uint64_t)otype << 56) | (0x0303ull << 40) | ((uint64_t)clen << 24)};
                alen = 13;
                ct = rec + 13;
            }
            if (lane < 5) {
                const uint32_t hb[5] = {otype, 3, 3, rlen >> 8, rlen & 0xFF};
                rec[lane] = (uint8_t)hb[lane];
            } else if (!is13 && lane < 13) {
                rec[lane] = (uint8_t)(sr.seq >> (8 * (12 - lane)));
            }
            L = gcm_lanes<true>(ks, te, lane & (TLS_TE_COPIES_REC - 1), tabs[wave], t8, red8, nonce, aad,
                                alen, nullptr, ct, clen, nullptr, 0, a.src + sr.src_off,
                                sr.plain_len, sr.type, is13);
        }
#if TLS_WG_TREE
        // a round with no AES-GCM record in the workgroup (ChaCha20-Poly1305 records, header
        // failures) skips the combine: its serial multiplies are pure latency
        U128 ghash{0, 0};
        if (__syncthreads_or(active)) {
            s_acc[wave][lane] = L.acc;
            __syncthreads();
            wg_tree<kOpenWaves>(s_acc, tabs);
            ghash = s_acc[wave][0];
        }
#else
        const U128 ghash = active ? wave_tree(L.acc, tabs[wave]) : U128{0, 0};
#endif
        if (active) (void)gcm_finish<true>(L, ghash, nullptr, ct, clen);
    }
}

__global__ CHACHA_ATTR void k_tls_seal_chacha(SealArgs a) {
    __shared__ uint4 wins[kCryptWaves][256];
    uint8_t* win = reinterpret_cast<uint8_t*>(wins[threadIdx.x >> 6]);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t r = blockIdx.x * kCryptWaves + wave; r < a.n; r += gridDim.x * kCryptWaves) {
        uvhttp_tls_seal_t sr;
        const KeySched* ks;
        bool is13;
        uint32_t clen, rlen;
        if (!seal_prep(a, r, UVHTTP_TLS_CIPHER_CHACHA20_POLY1305, &sr, &ks, &is13, &clen, &rlen)) continue;
        uint8_t* rec = a.out + sr.out_off;
        const uint32_t otype = is13 ? 23u : sr.type;
        const uint32_t nonce[3] = {ks->iv[0], ks->iv[1] ^ bswap32((uint32_t)(sr.seq >> 32)),
                                   ks->iv[2] ^ bswap32((uint32_t)sr.seq)};
        uint32_t aad16[4];
        if (is13) {
            aad16[0] = otype | 0x030300u | ((rlen >> 8) << 24);
            aad16[1] = rlen & 0xFF;
            aad16[2] = aad16[3] = 0;
        } else {
            aad16[0] = bswap32((uint32_t)(sr.seq >> 32));
            aad16[1] = bswap32((uint32_t)sr.seq);
            aad16[2] = otype | 0x030300u | ((clen >> 8) << 24);
            aad16[3] = clen & 0xFF;
        }
        if (lane < 5) {
            const uint32_t hb[5] = {otype, 3, 3, rlen >> 8, rlen & 0xFF};
            rec[lane] = (uint8_t)hb[lane];
        }
        (void)chacha_record<true>(ks, nonce, aad16, is13 ? 5u : 13u, nullptr, rec + 5, clen, nullptr,
                                  0, a.src + sr.src_off, sr.plain_len, sr.type, is13, win);
    }
}

// ---- finalize / fix-up ---------------------------------------------------------------------

__global__ __launch_bounds__(kBlock) void k_tls_finalize(TlsArgs a) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= a.n_streams) return;
    const uvhttp_tls_stream_t st = a.streams[s];
    uvhttp_tls_result_t r;
    memset(&r, 0, sizeof(r));
    r.next_seq = st.seq;
    a.fix[s] = 0;
    if (a.n_total[1]) {  // capacity: nothing delivered anywhere
        r.status = -1;
        r.first_status = UVHTTP_TLS_REC_ERR_CAPACITY;
        a.results[s] = r;
        return;
    }
    const StreamWork sw = a.sw[s];
    r.first_record = sw.key_bad;
    r.n_records = sw.n_rec;
    r.out_off = sw.cap + st.ws_prefix;
    const bool kbad = st.key >= a.n_keys || !key_valid(a.keys[st.key]);
    if (kbad) {
        r.status = -1;
        r.first_status = UVHTTP_TLS_REC_ERR_KEY;
        a.results[s] = r;
        return;
    }
    uint64_t plain = 0;
    bool stopped = false, moved = false;
    // the lane's records four at a time: the four loads are issued before the stores (the
    // stores could alias them as far as the compiler knows, which serialised one load per record)
    constexpr uint32_t kAhead = 4;
    for (uint32_t j0 = 0; j0 < sw.n_rec; j0 += kAhead) {
        RecWork wb[kAhead];
#pragma unroll
        for (uint32_t i = 0; i < kAhead; ++i)
            if (j0 + i < sw.n_rec) wb[i] = a.work[r.first_record + j0 + i];
#pragma unroll
        for (uint32_t i = 0; i < kAhead; ++i) {
            if (j0 + i >= sw.n_rec) break;
            const RecWork& w = wb[i];
            uvhttp_tls_record_t o;
            o.rec_off = w.rec_off;
            o.out_off = 0;
            o.content_len = 0;
            o.stream = s;
            o.type = 0;
            o.reserved = 0;
            o.reserved2 = 0;
            if (stopped) {
                o.status = UVHTTP_TLS_REC_SKIPPED;
            } else {
                o.status = (int8_t)w.status;
                o.type = (uint8_t)w.type;
                o.content_len = w.content_len;
                if (w.status == UVHTTP_TLS_REC_OK) {
                    o.out_off = r.out_off + plain;
                    if (o.out_off != w.spec_off) moved = true;
                    plain += w.content_len;
                    r.n_delivered++;
                    r.consumed_bytes = w.rec_off - st.begin + 5 + w.len;
                } else {
                    stopped = true;
                    r.first_status = w.status;
                    r.status = w.status < 0 ? -1 : 0;
                }
            }
            a.records[r.first_record + j0 + i] = o;
        }
    }
    r.next_seq = st.seq + r.n_delivered;
    r.plain_len = plain;
    a.results[s] = r;
    a.fix[s] = moved ? 1u : 0u;
}

// Move the delivered contents of a connection with padded TLS 1.3 records to their final
// (lower) offsets: records in order, each copied in WG-sized chunks read fully before written.
__global__ __launch_bounds__(kBlock) void k_tls_fixup(TlsArgs a) {
    const uint32_t s = blockIdx.x;
    if (s >= a.n_streams || !a.fix[s]) return;
    const uvhttp_tls_result_t r = a.results[s];
    for (uint32_t j = 0; j < r.n_delivered; ++j) {
        const RecWork w = a.work[r.first_record + j];
        const uint64_t dst = a.records[r.first_record + j].out_off, src = w.spec_off;
        if (dst == src) continue;
        for (uint64_t c = 0; c < w.content_len; c += kBlock * 16) {
            const uint64_t o = c + threadIdx.x * 16;
            uint32_t v[4] = {0, 0, 0, 0};
            const int n = o < w.content_len ? (w.content_len - o < 16 ? (int)(w.content_len - o) : 16) : 0;
            if (n) load_part(a.out + src + o, 0, n, v);
            __syncthreads();
            if (n) store_part(a.out + dst + o, n, v);
            __syncthreads();
        }
    }
}

// k_tls_ws_streams: one lane per connection — the WebSocket stream descriptor over its
// plaintext, one process_data call per delivered record (uvhttp_tls_gpu_ws_streams)
__global__ __launch_bounds__(kBlock) void k_tls_ws_streams(const uvhttp_tls_result_t* results,
                                                           const uvhttp_tls_record_t* records,
                                                           uint32_t n_streams,
                                                           const uvhttp_tls_stream_t* streams,
                                                           uvhttp_ws_stream_t* ws,
                                                           uint64_t* read_end) {
    const uint32_t s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= n_streams) return;
    const uvhttp_tls_result_t r = results[s];
    const uint64_t prefix = streams[s].ws_prefix;
    uvhttp_ws_stream_t w = ws[s];
    w.begin = r.out_off - prefix;
    w.len = prefix + r.plain_len;
    w.first_read = r.first_record;
    w.n_reads = r.n_delivered;
    uint64_t end = prefix;
    for (uint32_t k = 0; k < r.n_delivered; ++k) {
        end += records[r.first_record + k].content_len;
        read_end[r.first_record + k] = end;
    }
    ws[s] = w;
}

// k_tls_ws_prefix: one workgroup per connection copies its buffered WebSocket bytes in front
// of its plaintext
__global__ __launch_bounds__(kBlock) void k_tls_ws_prefix(const uvhttp_tls_result_t* results,
                                                          const uvhttp_tls_stream_t* streams,
                                                          const uint8_t* src,
                                                          const uint64_t* src_off, uint8_t* out) {
    const uint32_t s = blockIdx.x;
    const uint64_t n = streams[s].ws_prefix;
    if (!n || results[s].first_status == UVHTTP_TLS_REC_ERR_CAPACITY) return;
    const uint8_t* p = src + src_off[s];
    uint8_t* q = out + results[s].out_off - n;
    for (uint64_t o = threadIdx.x; o < n; o += kBlock) q[o] = p[o];
}

}  // namespace

// ---- engine ---------------------------------------------------------------------------------

struct uvhttp_tls_gpu_engine {
    int device;
    uint32_t* te0;
    void* ws;
    size_t ws_bytes;
    uint32_t cap_keys, cap_streams, cap_records;
    KeySched* sched;
    RecWork* work;
    StreamWork* sw;
    uint64_t* blk;
    uint32_t* n_total;
    uint32_t* fix;
    int timing;
    hipEvent_t ev[2 * 256];
    int ev_created, ev_used;
    double time_ms;
    uint64_t launches;
    int crypt_grid;
    hipStream_t last_stream;  // calls share one workspace: a call on a new stream waits for
    int have_last;            // the previous stream's queued work (order_ev)
    hipEvent_t order_ev;
    char err[256];
};

static void tls_call_begin(uvhttp_tls_gpu_engine_t* e, hipStream_t s) {
    if (e->have_last && e->last_stream != s) {
        if (!e->order_ev) (void)hipEventCreateWithFlags(&e->order_ev, hipEventDisableTiming);
        if (e->order_ev && hipEventRecord(e->order_ev, e->last_stream) == hipSuccess)
            (void)hipStreamWaitEvent(s, e->order_ev, 0);
    }
    e->last_stream = s;
    e->have_last = 1;
}

static int tls_err(uvhttp_tls_gpu_engine_t* e, int code, const char* what, hipError_t h) {
    if (e) snprintf(e->err, sizeof(e->err), "%s: %s", what, h == hipSuccess ? "" : hipGetErrorString(h));
    return code;
}

static size_t al(size_t x) { return (x + 255) / 256 * 256; }

static int tls_reserve(uvhttp_tls_gpu_engine_t* e, uint32_t keys, uint32_t streams, uint32_t records) {
    if (e->ws && keys <= e->cap_keys && streams <= e->cap_streams && records <= e->cap_records)
        return UVHTTP_TLS_GPU_OK;
    keys = keys > e->cap_keys ? keys : e->cap_keys;
    streams = streams > e->cap_streams ? streams : e->cap_streams;
    records = records > e->cap_records ? records : e->cap_records;
    const size_t nblk = (streams + kBlock - 1) / kBlock + 1;
    const size_t o_sched = 0;
    const size_t o_work = al(o_sched + (size_t)(keys ? keys : 1) * sizeof(KeySched));
    const size_t o_sw = al(o_work + (size_t)(records ? records : 1) * sizeof(RecWork));
    const size_t o_blk = al(o_sw + (size_t)(streams ? streams : 1) * sizeof(StreamWork));
    const size_t o_tot = al(o_blk + 2 * nblk * sizeof(uint64_t));
    const size_t o_fix = al(o_tot + 16);
    const size_t bytes = al(o_fix + (size_t)(streams ? streams : 1) * sizeof(uint32_t));
    if (e->ws) (void)hipFree(e->ws);
    e->ws = nullptr;
    const hipError_t h = hipMalloc(&e->ws, bytes);
    if (h != hipSuccess) {
        e->cap_keys = e->cap_streams = e->cap_records = 0;
        return tls_err(e, UVHTTP_TLS_GPU_ENOMEM, "hipMalloc tls workspace", h);
    }
    char* b = (char*)e->ws;
    e->sched = (KeySched*)(b + o_sched);
    // no slot holds a key yet (KeySched.src.key_len 0)
    const hipError_t hz = hipMemset(e->ws, 0, o_work);
    if (hz != hipSuccess) {
        (void)hipFree(e->ws);
        e->ws = nullptr;
        e->cap_keys = e->cap_streams = e->cap_records = 0;
        return tls_err(e, UVHTTP_TLS_GPU_ENOMEM, "hipMemset tls key slots", hz);
    }
    e->work = (RecWork*)(b + o_work);
    e->sw = (StreamWork*)(b + o_sw);
    e->blk = (uint64_t*)(b + o_blk);
    e->n_total = (uint32_t*)(b + o_tot);
    e->fix = (uint32_t*)(b + o_fix);
    e->ws_bytes = bytes;
    e->cap_keys = keys;
    e->cap_streams = streams;
    e->cap_records = records;
    return UVHTTP_TLS_GPU_OK;
}

static void tls_harvest(uvhttp_tls_gpu_engine_t* e) {
    for (int k = 0; k < e->ev_used; ++k) {
        float ms = 0;
        if (hipEventSynchronize(e->ev[2 * k + 1]) == hipSuccess &&
            hipEventElapsedTime(&ms, e->ev[2 * k], e->ev[2 * k + 1]) == hipSuccess) {
            e->time_ms += ms;
            e->launches++;
        }
    }
    e->ev_used = 0;
}

static int tls_timing_begin(uvhttp_tls_gpu_engine_t* e, hipStream_t s) {
    if (!e->timing) return -1;
    if (e->ev_used * 2 + 2 > (int)(sizeof(e->ev) / sizeof(e->ev[0]))) tls_harvest(e);
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

static void tls_timing_end(uvhttp_tls_gpu_engine_t* e, int k, hipStream_t s) {
    if (k < 0) return;
    (void)hipEventRecord(e->ev[2 * k + 1], s);
    e->ev_used = k + 1;
}

extern "C" {

int uvhttp_tls_gpu_engine_create(int device, uvhttp_tls_gpu_engine_t** out) {
    if (!out) return UVHTTP_TLS_GPU_EINVAL;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0 || device < 0 || device >= count)
        return UVHTTP_TLS_GPU_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return UVHTTP_TLS_GPU_ENODEV;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return UVHTTP_TLS_GPU_ENODEV;
    uvhttp_tls_gpu_engine_t* e = (uvhttp_tls_gpu_engine_t*)calloc(1, sizeof(*e));
    if (!e) return UVHTTP_TLS_GPU_ENOMEM;
    e->device = device;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    hipError_t h = hipMalloc(&e->te0, 256 * sizeof(uint32_t));
    if (h == hipSuccess) {
        hipLaunchKernelGGL(k_tls_te0, dim3(1), dim3(64), 0, 0, e->te0);
        h = hipDeviceSynchronize();
    }
    // crypto grid: enough 4-wave workgroups for every CU several times over
    e->crypt_grid = prop.multiProcessorCount * 8;
#ifdef UVWS_EXPERIMENTS  // (A/B builds only: the product library reads no environment)
    if (const char* g = getenv("UVHTTP_TLS_CRYPT_GRID")) e->crypt_grid = atoi(g) > 0 ? atoi(g) : e->crypt_grid;
#endif
    (void)hipSetDevice(prev);
    if (h != hipSuccess) {
        if (e->te0) (void)hipFree(e->te0);
        free(e);
        return UVHTTP_TLS_GPU_ENODEV;
    }
    *out = e;
    return UVHTTP_TLS_GPU_OK;
}

void uvhttp_tls_gpu_engine_free(uvhttp_tls_gpu_engine_t* e) {
    if (!e) return;
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(e->device);
    if (e->ws) (void)hipFree(e->ws);
    if (e->te0) (void)hipFree(e->te0);
    if (e->order_ev) (void)hipEventDestroy(e->order_ev);
    for (int k = 0; k < e->ev_created; ++k) (void)hipEventDestroy(e->ev[k]);
    (void)hipSetDevice(prev);
    free(e);
}

const char* uvhttp_tls_gpu_engine_last_error(const uvhttp_tls_gpu_engine_t* e) {
    return e ? e->err : "no engine";
}

int uvhttp_tls_gpu_engine_set_timing(uvhttp_tls_gpu_engine_t* e, int enable) {
    if (!e) return UVHTTP_TLS_GPU_EINVAL;
    e->timing = enable ? 1 : 0;
    return UVHTTP_TLS_GPU_OK;
}

int uvhttp_tls_gpu_engine_kernel_time(uvhttp_tls_gpu_engine_t* e, double* ms, uint64_t* launches) {
    if (!e || !ms || !launches) return UVHTTP_TLS_GPU_EINVAL;
    tls_harvest(e);
    *ms = e->time_ms;
    *launches = e->launches;
    e->time_ms = 0;
    e->launches = 0;
    return UVHTTP_TLS_GPU_OK;
}

int uvhttp_tls_gpu_open_records(uvhttp_tls_gpu_engine_t* e, const uint8_t* wire, uint64_t wire_len,
                                const uvhttp_tls_key_t* keys, uint32_t n_keys,
                                const uvhttp_tls_stream_t* streams, uint32_t n_streams,
                                uvhttp_tls_record_t* records, uint32_t max_records,
                                uvhttp_tls_result_t* results, uint8_t* out, uint64_t out_cap,
                                void* stream) {
    if (!e || (!wire && wire_len) || (!keys && n_keys) || (!streams && n_streams) ||
        (!records && max_records) || (!results && n_streams) || (!out && out_cap))
        return UVHTTP_TLS_GPU_EINVAL;
    if (n_streams > (1u << 26) || max_records > (1u << 28))
        return tls_err(e, UVHTTP_TLS_GPU_EINVAL, "too many streams / records", hipSuccess);
    if (!n_streams) return UVHTTP_TLS_GPU_OK;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != e->device) (void)hipSetDevice(e->device);
    int rc = tls_reserve(e, n_keys, n_streams, max_records);
    if (rc) {
        if (prev != e->device) (void)hipSetDevice(prev);
        return rc;
    }
    hipStream_t s = (hipStream_t)stream;
    tls_call_begin(e, s);
    TlsArgs a;
    a.wire = wire;
    a.wire_len = wire_len;
    a.keys = keys;
    a.n_keys = n_keys;
    a.streams = streams;
    a.n_streams = n_streams;
    a.records = records;
    a.max_records = max_records;
    a.results = results;
    a.out = out;
    a.out_cap = out_cap;
    a.sched = e->sched;
    a.work = e->work;
    a.sw = e->sw;
    a.blk = e->blk;
    a.n_total = e->n_total;
    a.fix = e->fix;
    a.te0 = e->te0;
    const uint32_t nb = (n_streams + kBlock - 1) / kBlock;
    if (n_keys)
        hipLaunchKernelGGL(k_tls_keys, dim3((n_keys + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                           keys, n_keys, (const uint32_t*)e->te0, e->sched);
    hipLaunchKernelGGL(k_tls_walk_count, dim3(nb), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(k_tls_walk_scan, dim3(1), dim3(kBlock), 0, s, a, nb);
    hipLaunchKernelGGL(k_tls_walk_write, dim3(nb), dim3(kBlock), 0, s, a);
    const uint32_t need = (max_records + kCryptWaves - 1) / kCryptWaves;
    const uint32_t grid = need < (uint32_t)e->crypt_grid ? (need ? need : 1) : (uint32_t)e->crypt_grid;
    const int tk = tls_timing_begin(e, s);
    // k_tls_open: a wave per group of kPack records, kOpenWaves waves per workgroup
    const uint32_t need_o = (max_records + kPack * kOpenWaves - 1) / (kPack * kOpenWaves);
    const uint32_t cap_o = (uint32_t)e->crypt_grid * kCryptWaves / kOpenWaves;
    const uint32_t grid_o = need_o < cap_o ? (need_o ? need_o : 1) : cap_o;
    hipLaunchKernelGGL(k_tls_open, dim3(grid_o), dim3(kOpenWG), 0, s, a);
    // k_tls_open_aes_packed: kAesPackW records per wave, kPackAesWaves waves per workgroup
    const uint32_t need_p = (max_records + kAesPackW * kPackAesWaves - 1) / (kAesPackW * kPackAesWaves);
    const uint32_t cap_p = (uint32_t)e->crypt_grid * kCryptWaves / kPackAesWaves;
    const uint32_t grid_p = need_p < cap_p ? (need_p ? need_p : 1) : cap_p;
    hipLaunchKernelGGL(k_tls_open_aes_packed, dim3(grid_p), dim3(kPackAesWG), 0, s, a);
    hipLaunchKernelGGL(k_tls_open_chacha, dim3(grid), dim3(kCryptWG), 0, s, a);
    hipLaunchKernelGGL(k_tls_open_chacha_packed, dim3(grid), dim3(kCryptWG), 0, s, a);
    tls_timing_end(e, tk, s);
    hipLaunchKernelGGL(k_tls_finalize, dim3(nb), dim3(kBlock), 0, s, a);
    hipLaunchKernelGGL(k_tls_fixup, dim3(n_streams), dim3(kBlock), 0, s, a);
    const hipError_t h = hipGetLastError();
    if (prev != e->device) (void)hipSetDevice(prev);
    if (h != hipSuccess) return tls_err(e, UVHTTP_TLS_GPU_ELAUNCH, "launch", h);
    return UVHTTP_TLS_GPU_OK;
}

int uvhttp_tls_gpu_seal_records(uvhttp_tls_gpu_engine_t* e, const uint8_t* src, uint64_t src_len,
                                const uvhttp_tls_seal_t* recs, uint32_t n_records,
                                const uvhttp_tls_key_t* keys, uint32_t n_keys, uint8_t* out,
                                uint64_t out_cap, void* stream) {
    if (!e || (!src && src_len) || (!recs && n_records) || (!keys && n_keys) || (!out && out_cap))
        return UVHTTP_TLS_GPU_EINVAL;
    if (!n_records) return UVHTTP_TLS_GPU_OK;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != e->device) (void)hipSetDevice(e->device);
    int rc = tls_reserve(e, n_keys, 1, 1);
    if (rc) {
        if (prev != e->device) (void)hipSetDevice(prev);
        return rc;
    }
    hipStream_t s = (hipStream_t)stream;
    tls_call_begin(e, s);
    if (n_keys)
        hipLaunchKernelGGL(k_tls_keys, dim3((n_keys + kBlock - 1) / kBlock), dim3(kBlock), 0, s,
                           keys, n_keys, (const uint32_t*)e->te0, e->sched);
    SealArgs a{src, src_len, recs, n_records, out, out_cap, e->sched, n_keys, e->te0};
    const uint32_t need = (n_records + kCryptWaves - 1) / kCryptWaves;
    const uint32_t grid = need < (uint32_t)e->crypt_grid ? need : (uint32_t)e->crypt_grid;
    const int tk = tls_timing_begin(e, s);
    const uint32_t need_s = (n_records + kOpenWaves - 1) / kOpenWaves;
    const uint32_t cap_s = (uint32_t)e->crypt_grid * kCryptWaves / kOpenWaves;
    hipLaunchKernelGGL(k_tls_seal, dim3(need_s < cap_s ? need_s : cap_s), dim3(kOpenWG), 0, s, a);
    hipLaunchKernelGGL(k_tls_seal_chacha, dim3(grid), dim3(kCryptWG), 0, s, a);
    tls_timing_end(e, tk, s);
    const hipError_t h = hipGetLastError();
    if (prev != e->device) (void)hipSetDevice(prev);
    if (h != hipSuccess) return tls_err(e, UVHTTP_TLS_GPU_ELAUNCH, "launch", h);
    return UVHTTP_TLS_GPU_OK;
}

int uvhttp_tls_gpu_ws_streams(uvhttp_tls_gpu_engine_t* e, const uvhttp_tls_result_t* results,
                              const uvhttp_tls_record_t* records, uint32_t n_streams,
                              const uvhttp_tls_stream_t* streams, const uint8_t* prefix_src,
                              const uint64_t* prefix_off, uint8_t* out, void* ws_streams,
                              uint64_t* read_end, void* stream) {
    if (!e || (n_streams && (!results || !streams || !ws_streams || !out)) ||
        (prefix_src && !prefix_off))
        return UVHTTP_TLS_GPU_EINVAL;
    if (!n_streams) return UVHTTP_TLS_GPU_OK;
    int prev = 0;
    (void)hipGetDevice(&prev);
    if (prev != e->device) (void)hipSetDevice(e->device);
    hipStream_t s = (hipStream_t)stream;
    tls_call_begin(e, s);
    if (prefix_src)
        hipLaunchKernelGGL(k_tls_ws_prefix, dim3(n_streams), dim3(kBlock), 0, s, results, streams,
                           prefix_src, prefix_off, out);
    hipLaunchKernelGGL(k_tls_ws_streams, dim3((n_streams + kBlock - 1) / kBlock), dim3(kBlock), 0,
                       s, results, records, n_streams, streams, (uvhttp_ws_stream_t*)ws_streams,
                       read_end);
    const hipError_t h = hipGetLastError();
    if (prev != e->device) (void)hipSetDevice(prev);
    if (h != hipSuccess) return tls_err(e, UVHTTP_TLS_GPU_ELAUNCH, "launch", h);
    return UVHTTP_TLS_GPU_OK;
}

}  // extern "C"
