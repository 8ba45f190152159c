/*
 * copy_check.c — the batcher's read copy (uvhttp_ws_amd_copy_stream + uvhttp_ws_amd_copy_fence,
 * ws_host.c) against memcpy: every length 0..2100 and 16 KiB +- 40 at every source and
 * destination alignment 0..63, bytes outside the destination range untouched.  Built under
 * ASan/UBSan; UVHTTP_WS_COPY_SSE2=1 runs the SSE2 path instead of AVX2 (tests/test_c1_echo.py).
 * Prints "ok <path>" or the first mismatch; exit status 0 / 1.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void uvhttp_ws_amd_copy_stream(void* dst, const void* src, size_t len);
void uvhttp_ws_amd_copy_fence(void);

static int check(uint8_t* dbuf, const uint8_t* sbuf, size_t cap, size_t len, size_t da, size_t sa) {
    memset(dbuf, 0xA5, cap);
    uvhttp_ws_amd_copy_stream(dbuf + 64 + da, sbuf + sa, len);
    uvhttp_ws_amd_copy_fence();
    for (size_t i = 0; i < cap; ++i) {
        const int inside = i >= 64 + da && i < 64 + da + len;
        const uint8_t want = inside ? sbuf[sa + (i - 64 - da)] : 0xA5;
        if (dbuf[i] != want) {
            printf("mismatch len %zu dst+%zu src+%zu at %zu\n", len, da, sa, i);
            return 1;
        }
    }
    return 0;
}

int main(void) {
    const size_t cap = 16384 + 256;
    uint8_t* sbuf = (uint8_t*)malloc(cap);
    uint8_t* dbuf = (uint8_t*)malloc(cap);
    for (size_t i = 0; i < cap; ++i) sbuf[i] = (uint8_t)(i * 131u + 7u);
    for (size_t da = 0; da < 64; ++da)
        for (size_t sa = 0; sa < 64; sa += 5) {
            for (size_t len = 0; len <= 2100; len += (len < 300 ? 1 : 37))
                if (check(dbuf, sbuf, cap, len, da, sa)) return 1;
            for (size_t len = 16384 - 40; len <= 16384 + 40 && len + da + 128 <= cap; ++len)
                if (check(dbuf, sbuf, cap, len, da, sa)) return 1;
        }
    const char* f = getenv("UVHTTP_WS_COPY_SSE2");
    printf("ok %s\n", f && f[0] == '1' ? "sse2" : "default");
    free(sbuf);
    free(dbuf);
    return 0;
}
