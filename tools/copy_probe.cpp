// copy_probe.cpp — the batcher's submit_read copy (uvhttp_ws_amd_copy_stream, ws_host.c) against
// other ways of moving 16 KiB reads into pinned host memory, alone and while a 256 MiB H2D and
// D2H run (the async flush's situation).  One JSON line per variant.   copy_probe [reps=3]
#include <hip/hip_runtime_api.h>
#include <immintrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

extern "C" void uvhttp_ws_amd_copy_stream(void* dst, const void* src, size_t len);  // product

#define CK(x)                                                          \
    do {                                                               \
        hipError_t e_ = (x);                                           \
        if (e_ != hipSuccess) {                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));   \
            exit(1);                                                   \
        }                                                              \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__attribute__((target("avx2"))) static void copy_avx2_nt(void* dst, const void* src, size_t n) {
    char* d = (char*)dst;
    const char* s = (const char*)src;
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        __m256i a = _mm256_loadu_si256((const __m256i*)(s + i));
        __m256i b = _mm256_loadu_si256((const __m256i*)(s + i + 32));
        __m256i c = _mm256_loadu_si256((const __m256i*)(s + i + 64));
        __m256i e = _mm256_loadu_si256((const __m256i*)(s + i + 96));
        _mm256_stream_si256((__m256i*)(d + i), a);
        _mm256_stream_si256((__m256i*)(d + i + 32), b);
        _mm256_stream_si256((__m256i*)(d + i + 64), c);
        _mm256_stream_si256((__m256i*)(d + i + 96), e);
    }
    memcpy(d + i, s + i, n - i);
}

__attribute__((target("avx512f"))) static void copy_avx512_nt(void* dst, const void* src, size_t n) {
    char* d = (char*)dst;
    const char* s = (const char*)src;
    size_t i = 0;
    for (; i + 256 <= n; i += 256) {
        __m512i a = _mm512_loadu_si512((const void*)(s + i));
        __m512i b = _mm512_loadu_si512((const void*)(s + i + 64));
        __m512i c = _mm512_loadu_si512((const void*)(s + i + 128));
        __m512i e = _mm512_loadu_si512((const void*)(s + i + 192));
        _mm512_stream_si512((__m512i*)(d + i), a);
        _mm512_stream_si512((__m512i*)(d + i + 64), b);
        _mm512_stream_si512((__m512i*)(d + i + 128), c);
        _mm512_stream_si512((__m512i*)(d + i + 192), e);
    }
    memcpy(d + i, s + i, n - i);
}

static void copy_memcpy(void* dst, const void* src, size_t n) { memcpy(dst, src, n); }

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    const size_t n = 256u << 20, chunk = 16384, src_len = 4 * 65550;
    uint8_t *h_arena, *h_up, *h_down, *d_up, *d_down;
    CK(hipHostMalloc((void**)&h_arena, n, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&h_up, n, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&h_down, n, hipHostMallocDefault));
    CK(hipMalloc((void**)&d_up, n));
    CK(hipMalloc((void**)&d_down, n));
    memset(h_arena, 1, n);
    memset(h_up, 2, n);
    memset(h_down, 3, n);
    uint8_t* src = (uint8_t*)malloc(src_len);  // one connection's stream, as in batcher_e2e
    memset(src, 4, src_len);
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    struct V {
        const char* name;
        void (*fn)(void*, const void*, size_t);
    } vs[] = {{"copy_stream (product)", uvhttp_ws_amd_copy_stream},
              {"avx2_nt", copy_avx2_nt},
              {"avx512_nt", copy_avx512_nt},
              {"memcpy", copy_memcpy}};
    for (int r = 0; r < reps; ++r) {
        for (const V& v : vs) {
            double t_alone = 0, t_dma = 0;
            for (int dma = 0; dma < 2; ++dma) {
                if (dma) {
                    CK(hipMemcpyAsync(d_up, h_up, n, hipMemcpyHostToDevice, a));
                    CK(hipMemcpyAsync(h_down, d_down, n, hipMemcpyDeviceToHost, b));
                }
                const double t = now();
                size_t so = 0;
                for (size_t o = 0; o < n; o += chunk) {
                    v.fn(h_arena + o, src + so, chunk);
                    so = so + chunk + chunk <= src_len ? so + chunk : 0;
                }
                (dma ? t_dma : t_alone) = now() - t;
                CK(hipStreamSynchronize(a));
                CK(hipStreamSynchronize(b));
            }
            printf("{\"variant\": \"%s\", \"alone_GBs\": %.1f, \"during_dma_GBs\": %.1f, \"alone_ms\": %.2f, "
                   "\"during_dma_ms\": %.2f}\n",
                   v.name, n / t_alone / 1e9, n / t_dma / 1e9, t_alone * 1e3, t_dma * 1e3);
        }
    }
    return 0;
}
