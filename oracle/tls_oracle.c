/*
 * oracle/tls_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the TLS record layer that sits ahead of the WebSocket decoder in the
 * reference: on_websocket_read (src/uvhttp_connection.c:1122-1159)
 * decrypts every record with mbedtls_ssl_read before uvhttp_ws_process_data sees the bytes.
 * mbedtls itself is an un-vendored submodule (.gitmodules, deps/mbedtls: empty here), so the
 * AEADs it runs (AES-GCM, ChaCha20-Poly1305) are restated from the published standards:
 *   aes_*         FIPS-197 (key expansion §5.2, cipher §5.1), byte-oriented, S-box generated
 *   gf_mult       NIST SP 800-38D §6.3 Algorithm 1 (bit-serial multiply in GF(2^128))
 *   gcm_crypt     NIST SP 800-38D §7.1/7.2 with a 96-bit IV (J0 = IV || 0^31 || 1)
 *   chacha20_*    RFC 8439 §2.3 (block function)
 *   poly_*        RFC 8439 §2.5 (Poly1305, plain 130-bit arithmetic)
 *   chachapoly_*  RFC 8439 §2.8 (AEAD_CHACHA20_POLY1305)
 *   TLS records   RFC 8446 §5.2 (TLSInnerPlaintext, AAD = record header) and §5.3 (nonce);
 *                 RFC 5288 §3 (TLS 1.2 AES-GCM: salt || explicit nonce, AAD = seq || type ||
 *                 version || len); RFC 7905 §2 (TLS 1.2 ChaCha20-Poly1305: iv XOR seq)
 *   oracle_tls_open_batch  the batch contract of include/uvhttp_tls_amd.h (walk, open,
 *                 stop at the first record that is not delivered application data, layout)
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it; the product
 * library never links or calls anything here.
 *
 * Pinning: FIPS-197 Appendix C.1/C.3, the GCM specification's test cases and RFC 8439's
 * ChaCha20 / Poly1305 / AEAD test vectors (tests/golden/tls_known_answers.json), and records
 * written by a real TLS stack — OpenSSL 3.0.2's libssl in this container, TLS 1.3 and TLS 1.2
 * sessions with AES-GCM and ChaCha20-Poly1305 over memory BIOs, keys recovered from the key
 * log (tests/golden/make_tls_vectors.py -> tests/golden/tls_openssl_records.json).
 * tests/test_tls_oracle.py checks both.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- AES (FIPS-197) ------------------------------------------------------------------ */

static uint8_t SBOX[256];
static int sbox_ready;

static uint8_t rotl8(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }
static uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1B : 0)); }

/* S-box from the multiplicative inverse and the affine map (FIPS-197 §5.1.1): p walks the
 * powers of 3 and q the powers of 3^-1, so q = p^-1 at every step. */
static void sbox_init(void) {
    if (sbox_ready) return;
    uint8_t p = 1, q = 1;
    do {
        p = (uint8_t)(p ^ (uint8_t)(p << 1) ^ ((p & 0x80) ? 0x1B : 0));
        q ^= (uint8_t)(q << 1);
        q ^= (uint8_t)(q << 2);
        q ^= (uint8_t)(q << 4);
        if (q & 0x80) q ^= 0x09;
        SBOX[p] = (uint8_t)(q ^ rotl8(q, 1) ^ rotl8(q, 2) ^ rotl8(q, 3) ^ rotl8(q, 4) ^ 0x63);
    } while (p != 1);
    SBOX[0] = 0x63;
    sbox_ready = 1;
}

uint8_t oracle_aes_sbox(uint8_t x) {
    sbox_init();
    return SBOX[x];
}

typedef struct {
    int nr;
    uint8_t rk[240];
} orc_aes_t;

/* §5.2 KeyExpansion, Nk = 4 or 8 */
static int aes_setkey(orc_aes_t* a, const uint8_t* key, int klen) {
    sbox_init();
    if (klen != 16 && klen != 32) return -1;
    const int nk = klen / 4;
    a->nr = nk + 6;
    const int total = 4 * (a->nr + 1);
    uint8_t* w = a->rk;
    memcpy(w, key, (size_t)klen);
    uint8_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint8_t t[4];
        memcpy(t, w + 4 * (i - 1), 4);
        if (i % nk == 0) {
            const uint8_t u = t[0];
            t[0] = (uint8_t)(SBOX[t[1]] ^ rcon);
            t[1] = SBOX[t[2]];
            t[2] = SBOX[t[3]];
            t[3] = SBOX[u];
            rcon = xtime(rcon);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; k++) t[k] = SBOX[t[k]];
        }
        for (int k = 0; k < 4; k++) w[4 * i + k] = (uint8_t)(w[4 * (i - nk) + k] ^ t[k]);
    }
    return 0;
}

/* §5.1 Cipher; state byte (row r, column c) = s[r + 4c] */
static void aes_encrypt(const orc_aes_t* a, const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; i++) s[i] = (uint8_t)(in[i] ^ a->rk[i]);
    for (int r = 1; r <= a->nr; r++) {
        for (int c = 0; c < 4; c++)
            for (int row = 0; row < 4; row++)
                t[row + 4 * c] = SBOX[s[row + 4 * ((c + row) & 3)]];  /* SubBytes, ShiftRows */
        if (r != a->nr) {
            for (int c = 0; c < 4; c++) {  /* MixColumns */
                const uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c + 0] = (uint8_t)(xtime(a0) ^ xtime(a1) ^ a1 ^ a2 ^ a3);
                s[4 * c + 1] = (uint8_t)(a0 ^ xtime(a1) ^ xtime(a2) ^ a2 ^ a3);
                s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ xtime(a2) ^ xtime(a3) ^ a3);
                s[4 * c + 3] = (uint8_t)(xtime(a0) ^ a0 ^ a1 ^ a2 ^ xtime(a3));
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; i++) s[i] ^= a->rk[16 * r + i];  /* AddRoundKey */
    }
    memcpy(out, s, 16);
}

int oracle_aes_encrypt_block(const uint8_t* key, int klen, const uint8_t in[16], uint8_t out[16]) {
    orc_aes_t a;
    if (aes_setkey(&a, key, klen)) return -1;
    aes_encrypt(&a, in, out);
    return 0;
}

/* ---- GCM (NIST SP 800-38D) ----------------------------------------------------------- */

/* Algorithm 1: Z = X . Y; bit 0 is the most significant bit of byte 0 */
static void gf_mult(const uint8_t X[16], const uint8_t Y[16], uint8_t Z[16]) {
    uint8_t V[16], acc[16];
    memcpy(V, Y, 16);
    memset(acc, 0, 16);
    for (int i = 0; i < 128; i++) {
        if (X[i >> 3] & (0x80 >> (i & 7)))
            for (int k = 0; k < 16; k++) acc[k] ^= V[k];
        const int lsb = V[15] & 1;
        for (int k = 15; k > 0; k--) V[k] = (uint8_t)((V[k] >> 1) | (V[k - 1] << 7));
        V[0] >>= 1;
        if (lsb) V[0] ^= 0xE1;
    }
    memcpy(Z, acc, 16);
}

void oracle_gf_mult(const uint8_t X[16], const uint8_t Y[16], uint8_t Z[16]) { gf_mult(X, Y, Z); }

/* GHASH_H over data zero-padded to whole blocks, folded into Y */
static void ghash_update(const uint8_t H[16], uint8_t Y[16], const uint8_t* d, size_t n) {
    for (size_t off = 0; off < n; off += 16) {
        const size_t m = n - off < 16 ? n - off : 16;
        for (size_t k = 0; k < m; k++) Y[k] ^= d[off + k];
        gf_mult(Y, H, Y);
    }
}

static void put_be64(uint8_t* p, uint64_t v) {
    for (int k = 0; k < 8; k++) p[k] = (uint8_t)(v >> (56 - 8 * k));
}

/* §7.1 (encrypt) / §7.2 (decrypt, tag computed over the input ciphertext) with a 96-bit IV.
 * out may alias in.  tag receives the computed tag. */
static void gcm_crypt(const orc_aes_t* a, const uint8_t iv[12], const uint8_t* aad, size_t alen,
                      const uint8_t* in, size_t n, uint8_t* out, uint8_t tag[16], int decrypt) {
    uint8_t H[16] = {0}, Y[16] = {0}, J[16], ks[16], lens[16];
    aes_encrypt(a, H, H);
    ghash_update(H, Y, aad, alen);
    if (decrypt) ghash_update(H, Y, in, n);
    memcpy(J, iv, 12);
    for (size_t off = 0, blk = 0; off < n; off += 16, blk++) {
        const uint32_t ctr = (uint32_t)(2 + blk);  /* inc32 from J0 + 1 */
        J[12] = (uint8_t)(ctr >> 24), J[13] = (uint8_t)(ctr >> 16);
        J[14] = (uint8_t)(ctr >> 8), J[15] = (uint8_t)ctr;
        aes_encrypt(a, J, ks);
        const size_t m = n - off < 16 ? n - off : 16;
        for (size_t k = 0; k < m; k++) out[off + k] = (uint8_t)(in[off + k] ^ ks[k]);
    }
    if (!decrypt) ghash_update(H, Y, out, n);
    put_be64(lens, (uint64_t)alen * 8);
    put_be64(lens + 8, (uint64_t)n * 8);
    ghash_update(H, Y, lens, 16);
    J[12] = J[13] = J[14] = 0, J[15] = 1;
    aes_encrypt(a, J, ks);
    for (int k = 0; k < 16; k++) tag[k] = (uint8_t)(Y[k] ^ ks[k]);
}

/* raw AES-GCM for the known-answer tests: returns 0, or (decrypt) -2 on a tag mismatch */
int oracle_gcm(const uint8_t* key, int klen, const uint8_t iv[12], const uint8_t* aad,
               size_t alen, const uint8_t* in, size_t n, uint8_t* out, uint8_t tag[16],
               int decrypt) {
    orc_aes_t a;
    if (aes_setkey(&a, key, klen)) return -1;
    uint8_t t[16];
    gcm_crypt(&a, iv, aad, alen, in, n, out, t, decrypt);
    if (decrypt) return memcmp(t, tag, 16) ? -2 : 0;
    memcpy(tag, t, 16);
    return 0;
}

/* ---- ChaCha20 and Poly1305 (RFC 8439) ------------------------------------------------ */

static uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static uint32_t le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* §2.3: the 64-byte block for (key, counter, nonce) */
static void chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                           uint8_t out[64]) {
    uint32_t st[16], x[16];
    st[0] = 0x61707865, st[1] = 0x3320646e, st[2] = 0x79622d32, st[3] = 0x6b206574;
    for (int i = 0; i < 8; i++) st[4 + i] = le32(key + 4 * i);
    st[12] = counter;
    for (int i = 0; i < 3; i++) st[13 + i] = le32(nonce + 4 * i);
    memcpy(x, st, sizeof(x));
#define QR(a, b, c, d)                                                                          \
    x[a] += x[b], x[d] ^= x[a], x[d] = rotl32(x[d], 16), x[c] += x[d], x[b] ^= x[c],            \
        x[b] = rotl32(x[b], 12), x[a] += x[b], x[d] ^= x[a], x[d] = rotl32(x[d], 8),           \
        x[c] += x[d], x[b] ^= x[c], x[b] = rotl32(x[b], 7)
    for (int r = 0; r < 10; r++) {
        QR(0, 4, 8, 12), QR(1, 5, 9, 13), QR(2, 6, 10, 14), QR(3, 7, 11, 15);
        QR(0, 5, 10, 15), QR(1, 6, 11, 12), QR(2, 7, 8, 13), QR(3, 4, 9, 14);
    }
#undef QR
    for (int i = 0; i < 16; i++) {
        const uint32_t v = x[i] + st[i];
        out[4 * i] = (uint8_t)v, out[4 * i + 1] = (uint8_t)(v >> 8);
        out[4 * i + 2] = (uint8_t)(v >> 16), out[4 * i + 3] = (uint8_t)(v >> 24);
    }
}

void oracle_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12],
                           uint8_t out[64]) {
    chacha20_block(key, counter, nonce, out);
}

/* §2.5: Poly1305 with plain 130-bit arithmetic (three 64-bit limbs, 128-bit products) */
typedef struct {
    uint64_t r0, r1, s0, s1;
    uint64_t h0, h1, h2;
} orc_poly_t;

static void poly_init(orc_poly_t* p, const uint8_t k[32]) {
    uint64_t r0 = 0, r1 = 0, s0 = 0, s1 = 0;
    for (int i = 7; i >= 0; i--) {
        r0 = (r0 << 8) | k[i];
        r1 = (r1 << 8) | k[8 + i];
        s0 = (s0 << 8) | k[16 + i];
        s1 = (s1 << 8) | k[24 + i];
    }
    p->r0 = r0 & 0x0ffffffc0fffffffull;  /* clamp: r &= 0x0ffffffc0ffffffc0ffffffc0fffffff */
    p->r1 = r1 & 0x0ffffffc0ffffffcull;
    p->s0 = s0, p->s1 = s1;
    p->h0 = p->h1 = p->h2 = 0;
}

/* h = (h + n) * r mod 2^130 - 5, n = 16 bytes of m (+ 2^(8 len) : the appended 0x01) */
static void poly_block(orc_poly_t* p, const uint8_t* m, size_t len) {
    uint8_t b[17] = {0};
    memcpy(b, m, len);
    b[len] = 1;
    uint64_t n0 = 0, n1 = 0;
    for (int i = 7; i >= 0; i--) n0 = (n0 << 8) | b[i], n1 = (n1 << 8) | b[8 + i];
    unsigned __int128 t = (unsigned __int128)p->h0 + n0;
    uint64_t a0 = (uint64_t)t;
    t = (t >> 64) + p->h1 + n1;
    uint64_t a1 = (uint64_t)t;
    uint64_t a2 = (uint64_t)(t >> 64) + p->h2 + b[16];
    /* (a2:a1:a0) * (r1:r0): a2 < 8, r < 2^124 */
    unsigned __int128 m00 = (unsigned __int128)a0 * p->r0;
    unsigned __int128 m01 = (unsigned __int128)a0 * p->r1;
    unsigned __int128 m10 = (unsigned __int128)a1 * p->r0;
    unsigned __int128 m11 = (unsigned __int128)a1 * p->r1;
    unsigned __int128 m20 = (unsigned __int128)a2 * p->r0;
    unsigned __int128 m21 = (unsigned __int128)a2 * p->r1;
    uint64_t d0 = (uint64_t)m00;
    unsigned __int128 c = (m00 >> 64) + (uint64_t)m01 + (uint64_t)m10;
    uint64_t d1 = (uint64_t)c;
    c = (c >> 64) + (m01 >> 64) + (m10 >> 64) + (uint64_t)m11 + (uint64_t)m20;
    uint64_t d2 = (uint64_t)c;
    c = (c >> 64) + (m11 >> 64) + (m20 >> 64) + (uint64_t)m21;
    uint64_t d3 = (uint64_t)c;  /* product < 2^255: fits d3:d2:d1:d0 with (m21 >> 64) == 0 */
    /* fold: x = lo130 + hi * 2^130 == lo130 + 5 * hi (mod p) */
    uint64_t l0 = d0, l1 = d1, l2 = d2 & 3;
    uint64_t h0 = (d2 >> 2) | (d3 << 62), h1 = d3 >> 2;  /* hi = x >> 130 */
    unsigned __int128 u = (unsigned __int128)l0 + (unsigned __int128)h0 * 5;
    l0 = (uint64_t)u;
    u = (u >> 64) + l1 + (unsigned __int128)h1 * 5;
    l1 = (uint64_t)u;
    l2 += (uint64_t)(u >> 64);
    /* once more for the bits above 2^130 (l2 < 2^64 small) */
    const uint64_t top = l2 >> 2;
    l2 &= 3;
    u = (unsigned __int128)l0 + top * 5;
    l0 = (uint64_t)u;
    u = (u >> 64) + l1;
    l1 = (uint64_t)u;
    l2 += (uint64_t)(u >> 64);
    p->h0 = l0, p->h1 = l1, p->h2 = l2;
}

static void poly_finish(orc_poly_t* p, uint8_t tag[16]) {
    /* full reduction mod p = 2^130 - 5: h < 2^131 here, subtract p while h >= p */
    for (int k = 0; k < 2; k++) {
        /* g = h + 5; if g >= 2^130 then h - p = g - 2^130 */
        unsigned __int128 g = (unsigned __int128)p->h0 + 5;
        const uint64_t g0 = (uint64_t)g;
        g = (g >> 64) + p->h1;
        const uint64_t g1 = (uint64_t)g;
        const uint64_t g2 = p->h2 + (uint64_t)(g >> 64);
        if (g2 >= 4) p->h0 = g0, p->h1 = g1, p->h2 = g2 - 4;
    }
    unsigned __int128 t = (unsigned __int128)p->h0 + p->s0;
    const uint64_t t0 = (uint64_t)t;
    const uint64_t t1 = (uint64_t)((t >> 64) + p->h1 + p->s1);
    for (int i = 0; i < 8; i++) tag[i] = (uint8_t)(t0 >> (8 * i)), tag[8 + i] = (uint8_t)(t1 >> (8 * i));
}

void oracle_poly1305(const uint8_t key[32], const uint8_t* m, size_t n, uint8_t tag[16]) {
    orc_poly_t p;
    poly_init(&p, key);
    for (size_t off = 0; off < n; off += 16) poly_block(&p, m + off, n - off < 16 ? n - off : 16);
    poly_finish(&p, tag);
}

/* §2.8 AEAD_CHACHA20_POLY1305: encrypt/decrypt in place-safe, tag over AAD || pad || CT || pad
 * || le64(aad len) || le64(ct len) */
static void chachapoly_crypt(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad,
                             size_t alen, const uint8_t* in, size_t n, uint8_t* out,
                             uint8_t tag[16], int decrypt) {
    uint8_t blk[64], otk[64], lens[16];
    chacha20_block(key, 0, nonce, otk);
    orc_poly_t p;
    poly_init(&p, otk);
    for (size_t off = 0; off < alen; off += 16) {
        uint8_t b[16] = {0};
        memcpy(b, aad + off, alen - off < 16 ? alen - off : 16);
        poly_block(&p, b, 16);
    }
    if (decrypt)
        for (size_t off = 0; off < n; off += 16) {
            uint8_t b[16] = {0};
            memcpy(b, in + off, n - off < 16 ? n - off : 16);
            poly_block(&p, b, 16);
        }
    for (size_t off = 0, c = 1; off < n; off += 64, c++) {
        chacha20_block(key, (uint32_t)c, nonce, blk);
        const size_t m = n - off < 64 ? n - off : 64;
        for (size_t k = 0; k < m; k++) out[off + k] = (uint8_t)(in[off + k] ^ blk[k]);
    }
    if (!decrypt)
        for (size_t off = 0; off < n; off += 16) {
            uint8_t b[16] = {0};
            memcpy(b, out + off, n - off < 16 ? n - off : 16);
            poly_block(&p, b, 16);
        }
    for (int i = 0; i < 8; i++) lens[i] = (uint8_t)((uint64_t)alen >> (8 * i)), lens[8 + i] = (uint8_t)((uint64_t)n >> (8 * i));
    poly_block(&p, lens, 16);
    poly_finish(&p, tag);
}

int oracle_chachapoly(const uint8_t key[32], const uint8_t nonce[12], const uint8_t* aad, size_t alen,
                      const uint8_t* in, size_t n, uint8_t* out, uint8_t tag[16], int decrypt) {
    uint8_t t[16];
    chachapoly_crypt(key, nonce, aad, alen, in, n, out, t, decrypt);
    if (decrypt) return memcmp(t, tag, 16) ? -2 : 0;
    memcpy(tag, t, 16);
    return 0;
}

/* ---- TLS records (RFC 8446 §5.2-5.3, RFC 5288 §3, RFC 7905 §2) ------------------------ */

/* layouts identical to include/uvhttp_tls_amd.h (kept separate: the oracle does not depend
 * on the product's headers) */
typedef struct {
    uint8_t key[32];
    uint8_t iv[12];
    uint32_t key_len, version, cipher, reserved[2];
} orc_tls_key_t;
typedef struct {
    uint64_t begin, len, seq;
    uint32_t key, ws_prefix;
} orc_tls_stream_t;
typedef struct {
    uint64_t rec_off, out_off;
    uint32_t content_len, stream;
    uint8_t type;
    int8_t status;
    uint16_t reserved;
    uint32_t reserved2;
} orc_tls_record_t;
typedef struct {
    uint32_t first_record, n_records, n_delivered;
    int32_t status, first_status;
    uint32_t reserved;
    uint64_t consumed_bytes, next_seq, out_off, plain_len, reserved3;
} orc_tls_result_t;

enum {
    T_OK = 0, T_SKIPPED = 2, T_CONTROL = 3,
    T_OVERFLOW = -1, T_BAD_MAC = -2, T_BAD_TYPE = -3, T_VERSION = -4, T_EMPTY = -5,
    T_CAPACITY = -6, T_KEY = -7,
};
#define V12 0x0303u
#define V13 0x0304u
#define C_AESGCM 0u
#define C_CHACHA 1u

static int key_ok(const orc_tls_key_t* k) {
    if (k->version != V12 && k->version != V13) return 0;
    if (k->cipher == C_AESGCM) return k->key_len == 16 || k->key_len == 32;
    return k->cipher == C_CHACHA && k->key_len == 32;
}

/* bytes of explicit nonce after the header: TLS 1.2 AES-GCM only (RFC 5288); the TLS 1.2
 * ChaCha20-Poly1305 nonce is implicit (RFC 7905) */
static uint32_t explicit_len(const orc_tls_key_t* k) {
    return k->version == V12 && k->cipher == C_AESGCM ? 8u : 0u;
}

typedef struct {
    orc_aes_t aes;
    const orc_tls_key_t* k;
} orc_aead_t;

static int aead_init(orc_aead_t* a, const orc_tls_key_t* k) {
    a->k = k;
    if (!key_ok(k)) return -1;
    return k->cipher == C_AESGCM ? aes_setkey(&a->aes, k->key, (int)k->key_len) : 0;
}

static void aead_crypt(const orc_aead_t* a, const uint8_t nonce[12], const uint8_t* aad,
                       size_t alen, const uint8_t* in, size_t n, uint8_t* out, uint8_t tag[16],
                       int decrypt) {
    if (a->k->cipher == C_AESGCM) gcm_crypt(&a->aes, nonce, aad, alen, in, n, out, tag, decrypt);
    else chachapoly_crypt(a->k->key, nonce, aad, alen, in, n, out, tag, decrypt);
}

/* nonce of record `seq`: iv XOR (0^32 || be64(seq)) (TLS 1.3, RFC 8446 §5.3; TLS 1.2
 * ChaCha20-Poly1305, RFC 7905 §2), or salt || explicit nonce (TLS 1.2 AES-GCM) */
static void tls_nonce(const orc_tls_key_t* k, uint64_t seq, const uint8_t* explicit8,
                      uint8_t nonce[12]) {
    if (explicit_len(k)) {
        memcpy(nonce, k->iv, 4);
        memcpy(nonce + 4, explicit8, 8);
    } else {
        memcpy(nonce, k->iv, 12);
        for (int b = 0; b < 8; b++) nonce[4 + b] ^= (uint8_t)(seq >> (56 - 8 * b));
    }
}

/* header checks of the walk, in contract order; returns 0 or the record's status */
static int header_status(const orc_tls_key_t* k, const uint8_t* h) {
    const uint32_t type = h[0], ver = ((uint32_t)h[1] << 8) | h[2];
    const uint32_t len = ((uint32_t)h[3] << 8) | h[4];
    const uint32_t over = explicit_len(k) + 16;
    if (ver != 0x0303) return T_VERSION;
    if (k->version == V13 ? type != 23 : (type < 21 || type > 23)) return T_BAD_TYPE;
    if (len > 16384u + (k->version == V13 ? 1u : 0u) + over) return T_OVERFLOW;
    if (len < over) return T_BAD_MAC;
    return 0;
}

/* reserved content bytes of a counted record (largest content it can deliver) */
static uint64_t record_cap(const orc_tls_key_t* k, uint32_t len) {
    const uint32_t over = explicit_len(k) + 16 + (k->version == V13 ? 1u : 0u);
    return len > over ? len - over : 0;
}

/* open one complete record whose header passed; writes its content to out (content_len
 * bytes), returns the status, sets *type and *content_len */
static int open_record(const orc_aead_t* a, uint64_t seq, const uint8_t* rec, uint8_t* out,
                       uint8_t* type, uint32_t* content_len) {
    const orc_tls_key_t* k = a->k;
    const uint32_t len = ((uint32_t)rec[3] << 8) | rec[4];
    const uint32_t ex = explicit_len(k);
    const uint32_t clen = len - ex - 16;
    const uint8_t* ct = rec + 5 + ex;
    uint8_t nonce[12], tag[16], aad[13];
    size_t alen;
    *type = 0;
    *content_len = 0;
    tls_nonce(k, seq, rec + 5, nonce);
    if (k->version == V13) {
        memcpy(aad, rec, 5);
        alen = 5;
    } else {
        put_be64(aad, seq);
        aad[8] = rec[0], aad[9] = 3, aad[10] = 3;
        aad[11] = (uint8_t)(clen >> 8), aad[12] = (uint8_t)clen;
        alen = 13;
    }
    uint8_t* plain = (uint8_t*)malloc(clen ? clen : 1);
    aead_crypt(a, nonce, aad, alen, ct, clen, plain, tag, 1);
    if (memcmp(tag, ct + clen, 16)) {
        free(plain);
        return T_BAD_MAC;
    }
    if (k->version == V13) {
        uint32_t i = clen;
        while (i > 0 && plain[i - 1] == 0) i--;
        if (i == 0) {
            free(plain);
            return T_EMPTY;
        }
        *type = plain[i - 1];
        *content_len = i - 1;
    } else {
        *type = rec[0];
        *content_len = clen;
    }
    memcpy(out, plain, *content_len);
    free(plain);
    return *type == 23 ? T_OK : T_CONTROL;
}

/* one stream's walk: counted records and their reserved bytes */
static void walk_stream(const uint8_t* wire, uint64_t wire_len, const orc_tls_stream_t* st,
                        const orc_tls_key_t* keys, uint32_t n_keys, uint32_t* n_rec,
                        uint64_t* cap, int* key_bad) {
    *n_rec = 0;
    *cap = st->ws_prefix; /* the connection's reservation starts with the WebSocket prefix */
    *key_bad = st->key >= n_keys || !key_ok(&keys[st->key]);
    if (*key_bad) return;
    const orc_tls_key_t* k = &keys[st->key];
    const uint64_t L = st->len <= wire_len && st->begin <= wire_len - st->len ? st->len : 0;
    const uint8_t* p = wire + st->begin;
    uint64_t pos = 0;
    while (L - pos >= 5) {
        const int hs = header_status(k, p + pos);
        const uint32_t len = ((uint32_t)p[pos + 3] << 8) | p[pos + 4];
        if (!hs && L - pos - 5 < len) break;  /* incomplete: waits for more bytes */
        ++*n_rec;
        if (hs) break;
        *cap += record_cap(k, len);
        pos += 5 + (uint64_t)len;
    }
}

/* The batch contract of include/uvhttp_tls_amd.h.  Returns the number of counted records
 * (0 with every result at ERR_CAPACITY when they do not fit). */
uint64_t oracle_tls_open_batch(const uint8_t* wire, uint64_t wire_len, const orc_tls_key_t* keys,
                               uint32_t n_keys, const orc_tls_stream_t* streams,
                               uint32_t n_streams, orc_tls_record_t* records,
                               uint32_t max_records, orc_tls_result_t* results, uint8_t* out,
                               uint64_t out_cap) {
    uint64_t total_rec = 0, total_cap = 0;
    for (uint32_t s = 0; s < n_streams; s++) {
        uint32_t n;
        uint64_t cap;
        int kb;
        walk_stream(wire, wire_len, &streams[s], keys, n_keys, &n, &cap, &kb);
        total_rec += n;
        total_cap += cap;
    }
    if (total_rec > max_records || total_cap > out_cap) {
        for (uint32_t s = 0; s < n_streams; s++) {
            orc_tls_result_t* r = &results[s];
            memset(r, 0, sizeof(*r));
            r->status = -1;
            r->first_status = T_CAPACITY;
            r->next_seq = streams[s].seq;
        }
        return 0;
    }
    uint64_t rec_base = 0, out_base = 0;
    for (uint32_t s = 0; s < n_streams; s++) {
        const orc_tls_stream_t* st = &streams[s];
        orc_tls_result_t* r = &results[s];
        uint32_t n;
        uint64_t cap;
        int kb;
        walk_stream(wire, wire_len, st, keys, n_keys, &n, &cap, &kb);
        memset(r, 0, sizeof(*r));
        r->first_record = (uint32_t)rec_base;
        r->n_records = n;
        r->out_off = out_base + st->ws_prefix;
        r->next_seq = st->seq;
        if (kb) {
            r->status = -1;
            r->first_status = T_KEY;
            continue;
        }
        const orc_tls_key_t* k = &keys[st->key];
        orc_aead_t a;
        aead_init(&a, k);
        const uint8_t* p = wire + st->begin;
        uint64_t pos = 0, plain = 0;
        int stopped = 0;
        for (uint32_t j = 0; j < n; j++) {
            orc_tls_record_t* rec = &records[rec_base + j];
            const uint32_t len = ((uint32_t)p[pos + 3] << 8) | p[pos + 4];
            memset(rec, 0, sizeof(*rec));
            rec->rec_off = st->begin + pos;
            rec->stream = s;
            if (stopped) {
                rec->status = T_SKIPPED;
            } else {
                int status = header_status(k, p + pos);
                if (!status) {
                    uint8_t type;
                    uint32_t clen;
                    status = open_record(&a, st->seq + j, p + pos, out + r->out_off + plain,
                                         &type, &clen);
                    rec->type = type;
                    rec->content_len = clen;
                }
                rec->status = (int8_t)status;
                if (status == T_OK) {
                    rec->out_off = r->out_off + plain;
                    plain += rec->content_len;
                    r->n_delivered++;
                    r->consumed_bytes = pos + 5 + len;
                } else {
                    stopped = 1;
                    r->first_status = status;
                    r->status = status < 0 ? -1 : 0;
                }
            }
            pos += 5 + (uint64_t)len;
        }
        r->next_seq = st->seq + r->n_delivered;
        r->plain_len = plain;
        rec_base += n;
        out_base += cap;
    }
    return rec_base;
}

/* Seal one record (send side / test-data generator): returns its length, or 0 on bad input.
 * TLS 1.3: outer type 23, inner = content || type + `pad` zero bytes; TLS 1.2: outer type =
 * type, AES-GCM explicit nonce = be64(seq). */
uint64_t oracle_tls_seal_record(const orc_tls_key_t* k, uint64_t seq, uint8_t type,
                                const uint8_t* content, uint32_t n, uint32_t pad, uint8_t* rec) {
    orc_aead_t a;
    if (aead_init(&a, k)) return 0;
    const uint32_t ex = explicit_len(k);
    const uint32_t clen = k->version == V13 ? n + 1 + pad : n;
    const uint32_t len = ex + clen + 16;
    if (len > 0xFFFF) return 0;
    uint8_t nonce[12], aad[13];
    rec[0] = k->version == V13 ? 23 : type, rec[1] = 3, rec[2] = 3;
    rec[3] = (uint8_t)(len >> 8), rec[4] = (uint8_t)len;
    if (ex) put_be64(rec + 5, seq);
    uint8_t* ct = rec + 5 + ex;
    memmove(ct, content, n);
    if (k->version == V13) {
        ct[n] = type;
        memset(ct + n + 1, 0, pad);
        memcpy(aad, rec, 5);
    } else {
        put_be64(aad, seq);
        aad[8] = type, aad[9] = 3, aad[10] = 3, aad[11] = (uint8_t)(n >> 8), aad[12] = (uint8_t)n;
    }
    tls_nonce(k, seq, rec + 5, nonce);
    aead_crypt(&a, nonce, aad, k->version == V13 ? 5 : 13, ct, clen, ct, ct + clen, 0);
    return 5 + (uint64_t)len;
}

/* CPU baseline: open `n` complete TLS records laid out back to back (one connection, one
 * key, sequence numbers from seq); returns the content bytes delivered */
uint64_t oracle_tls_open_stream_bytes(const orc_tls_key_t* k, uint64_t seq, const uint8_t* wire,
                                      uint64_t len, uint8_t* out) {
    orc_aead_t a;
    if (aead_init(&a, k)) return 0;
    uint64_t pos = 0, plain = 0;
    while (len - pos >= 5) {
        const uint32_t rl = ((uint32_t)wire[pos + 3] << 8) | wire[pos + 4];
        if (header_status(k, wire + pos) || len - pos - 5 < rl) break;
        uint8_t type;
        uint32_t clen;
        if (open_record(&a, seq++, wire + pos, out + plain, &type, &clen) != T_OK) break;
        plain += clen;
        pos += 5 + (uint64_t)rl;
    }
    return plain;
}
