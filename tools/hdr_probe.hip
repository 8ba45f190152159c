// hdr_probe.hip — how fast can a kernel read one frame header per 264-byte slot (C4's
// 1 048 576 x 256-byte frames)?  The floor of k_plan's pass 1.
//   g1   : a lane per frame, one aligned 16-byte load
//   g2   : a lane per frame, two aligned 16-byte loads (load16_at's window)
//   g8   : 8 consecutive frames per lane, 512 blocks (k_plan<8>'s mapping), two loads each
//   gb   : a lane per frame, one unaligned 16-byte buffer load (hardware unaligned access)
//   lin  : the whole wire read linearly, 16 bytes per lane (the streaming alternative)
// Each is timed cold (a 1 GiB buffer written in between, so the wire is out of the 256 MB
// Infinity Cache) and warm (run again at once).   hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void g1(const uint8_t* w, uint64_t stride, uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t x = 0;
    if (i < n) {
        const uint64_t o = (uint64_t)i * stride;
        const u32x4 v = *reinterpret_cast<const u32x4*>(w + (o & ~15ull));
        x = v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) out[i] = x;
}

__global__ __launch_bounds__(256) void g2(const uint8_t* w, uint64_t stride, uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    uint32_t x = 0;
    if (i < n) {
        const uint64_t o = (uint64_t)i * stride;
        const u32x4 v = *reinterpret_cast<const u32x4*>(w + (o & ~15ull));
        const u32x4 u = *reinterpret_cast<const u32x4*>(w + (o & ~15ull) + 16);
        x = v.x ^ v.y ^ v.z ^ v.w ^ u.x ^ u.w;
    }
    if (x == 0x12345678u) out[i] = x;
}

__global__ __launch_bounds__(256) void g8(const uint8_t* w, uint64_t stride, uint32_t n, uint32_t* out) {
    const uint32_t i0 = (blockIdx.x * 256 + threadIdx.x) * 8;
    u32x4 v[8], u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t i = i0 + k < n ? i0 + k : n - 1;
        const uint64_t o = ((uint64_t)i * stride) & ~15ull;
        v[k] = *reinterpret_cast<const u32x4*>(w + o);
        u[k] = *reinterpret_cast<const u32x4*>(w + o + 16);
    }
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) x ^= v[k].x ^ v[k].w ^ u[k].y;
    if (x == 0x12345678u) out[i0] = x;
}

__global__ __launch_bounds__(256) void gb(const uint8_t* w, uint64_t stride, uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(w), 0, 0x7FFFFFFF, 0x00020000);
    uint32_t x = 0;
    if (i < n) {
        const uint64_t o = (uint64_t)i * stride;  // < 2^31 here
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)o, 0, 0);
        x = v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (x == 0x12345678u) out[i] = x;
}

__global__ __launch_bounds__(256) void lin(const uint8_t* w, uint64_t len, uint32_t* out) {
    const uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 16;
    uint32_t x = 0;
    if (i + 16 <= len) {
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(w + i));
        x = v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x12345678u) out[i / 16] = x;
}

__global__ void fill(uint32_t* p, uint64_t n, uint32_t v) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v ^ (uint32_t)i;
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1048576;
    const uint64_t stride = argc > 2 ? strtoull(argv[2], nullptr, 10) : 264;
    const uint64_t len = (uint64_t)n * stride;
    uint8_t* w;
    uint32_t *out, *junk;
    const uint64_t junk_words = 1ull << 28;  // 1 GiB
    CK(hipMalloc(&w, len + 64));
    CK(hipMalloc(&out, (size_t)n * 4 + 64));
    CK(hipMalloc(&junk, junk_words * 4));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)w, len / 4, 7u);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[] = {"g1", "g2", "g8", "gb", "lin"};
    for (int rep = 0; rep < 3; ++rep) {
        for (int k = 0; k < 5; ++k) {
            for (int warm = 0; warm < 2; ++warm) {
                if (!warm) hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, junk, junk_words, (uint32_t)rep);
                CK(hipEventRecord(e0, 0));
                const dim3 b(256);
                if (k == 0) hipLaunchKernelGGL(g1, dim3((n + 255) / 256), b, 0, 0, w, stride, n, out);
                if (k == 1) hipLaunchKernelGGL(g2, dim3((n + 255) / 256), b, 0, 0, w, stride, n, out);
                if (k == 2) hipLaunchKernelGGL(g8, dim3((n + 2047) / 2048), b, 0, 0, w, stride, n, out);
                if (k == 3) hipLaunchKernelGGL(gb, dim3((n + 255) / 256), b, 0, 0, w, stride, n, out);
                if (k == 4) hipLaunchKernelGGL(lin, dim3((uint32_t)((len / 16 + 255) / 256)), b, 0, 0, w, len, out);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep) printf("%-4s %-4s %8.2f us  (%.1f ns/frame)\n", names[k], warm ? "warm" : "cold", ms * 1e3, ms * 1e6 / n);
            }
        }
    }
    return 0;
}
