// pcie_probe.hip — PCIe copy ceilings for the batcher's live-shape flush: pinned
// host <-> HBM, 256 MiB, H2D alone, D2H alone, both at once on two streams, a host memcpy (nt
// stores) into pinned memory alongside the two copies, and the batcher's own shape (reads
// copied into pinned memory and sent up in 8 MiB pieces while the previous round comes down).
// One JSON line per repetition.  Built by `make` (tools/bin/pcie_probe); bench.py --e2e runs it
// beside the live-shape batcher so each e2e rate comes with the PCIe ceiling of that box.
//   pcie_probe [MiB=256] [reps=5]
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            exit(1);                                                        \
        }                                                                   \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void nt_copy(void* dst, const void* src, size_t n) {
    char* d = (char*)dst;
    const char* s = (const char*)src;
    for (size_t i = 0; i + 64 <= n; i += 64) {
        __m128i a = _mm_loadu_si128((const __m128i*)(s + i)), b = _mm_loadu_si128((const __m128i*)(s + i + 16));
        __m128i c = _mm_loadu_si128((const __m128i*)(s + i + 32)), e = _mm_loadu_si128((const __m128i*)(s + i + 48));
        _mm_stream_si128((__m128i*)(d + i), a);
        _mm_stream_si128((__m128i*)(d + i + 16), b);
        _mm_stream_si128((__m128i*)(d + i + 32), c);
        _mm_stream_si128((__m128i*)(d + i + 48), e);
    }
    _mm_sfence();
}

int main(int argc, char** argv) {
    const size_t n = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 256) << 20;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    uint8_t *h_up, *h_down, *h_copy, *d_up, *d_down;
    CK(hipHostMalloc((void**)&h_up, n, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&h_down, n, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&h_copy, n, hipHostMallocDefault));
    CK(hipMalloc((void**)&d_up, n));
    CK(hipMalloc((void**)&d_down, n));
    memset(h_up, 1, n);
    memset(h_down, 2, n);
    memset(h_copy, 3, n);
    uint8_t* src = (uint8_t*)malloc(1 << 18);  // the reads' source: cache-resident, as in batcher_e2e
    memset(src, 4, 1 << 18);
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    auto h2d = [&] { CK(hipMemcpyAsync(d_up, h_up, n, hipMemcpyHostToDevice, a)); };
    auto d2h = [&] { CK(hipMemcpyAsync(h_down, d_down, n, hipMemcpyDeviceToHost, b)); };
    auto cpu = [&] {
        for (size_t o = 0; o < n; o += 1 << 18) nt_copy(h_copy + o, src, 1 << 18);
    };
    h2d();
    d2h();
    CK(hipDeviceSynchronize());
    const double gb = n / 1e9;
    for (int r = 0; r < reps; ++r) {
        double t = now();
        h2d();
        CK(hipStreamSynchronize(a));
        const double t_h2d = now() - t;
        t = now();
        d2h();
        CK(hipStreamSynchronize(b));
        const double t_d2h = now() - t;
        t = now();
        h2d();
        d2h();
        CK(hipStreamSynchronize(a));
        CK(hipStreamSynchronize(b));
        const double t_both = now() - t;
        t = now();
        cpu();
        const double t_cpu = now() - t;
        t = now();
        h2d();
        d2h();
        cpu();
        const double t_cpu_in = now() - t;
        CK(hipStreamSynchronize(a));
        CK(hipStreamSynchronize(b));
        const double t_all = now() - t;
        // the batcher's shape: the next round's reads copied into pinned memory and sent up in
        // 8 MiB pieces as they fill, while the previous round's wire comes down (whole, or in
        // 8 MiB pieces)
        const size_t piece = 8u << 20;
        double t_pieces[2];
        for (int split = 0; split < 2; ++split) {
            t = now();
            if (!split) d2h();
            for (size_t o = 0; o < n; o += piece) {
                if (split) CK(hipMemcpyAsync(h_down + o, d_down + o, piece, hipMemcpyDeviceToHost, b));
                for (size_t q = o; q < o + piece; q += 1 << 18) nt_copy(h_copy + q, src, 1 << 18);
                CK(hipMemcpyAsync(d_up + o, h_copy + o, piece, hipMemcpyHostToDevice, a));
            }
            CK(hipStreamSynchronize(a));
            CK(hipStreamSynchronize(b));
            t_pieces[split] = now() - t;
        }
        printf("{\"batcher_shape_ms\": %.2f, \"batcher_shape_d2h_pieces_ms\": %.2f, ", t_pieces[0] * 1e3,
               t_pieces[1] * 1e3);
        printf("\"bytes\": %zu, \"h2d_GBs\": %.1f, \"d2h_GBs\": %.1f, \"both_GBs_each\": %.1f, "
               "\"both_ms\": %.2f, \"cpu_nt_copy_GBs\": %.1f, \"all_three_ms\": %.2f, "
               "\"cpu_copy_during_dma_ms\": %.2f}\n",
               n, gb / t_h2d, gb / t_d2h, gb / t_both, t_both * 1e3, gb / t_cpu, t_all * 1e3,
               t_cpu_in * 1e3);
    }
    return 0;
}
