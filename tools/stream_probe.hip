// tools/stream_probe.hip — HBM streaming ceilings on MI355X for the unmask pass.
//
// Measures, interleaved in one process (methodology: cdna_hip_programming.md §5.4 rule 24),
// the practical ceiling of the payload kernel's access pattern: a plain 16-byte copy, and
// in-place 16-byte read-XOR-write with different vectors per lane, cache policies, block
// sizes and grid shapes.  Bytes counted = read + write.
//   hipcc --offload-arch=gfx950 -O3 -o stream_probe tools/stream_probe.hip && ./stream_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

template <int BLOCK, int VPT, bool NT_LD, bool NT_ST>
__global__ __launch_bounds__(BLOCK) void k_copy(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                uint64_t nvec) {
    const uint64_t base = (uint64_t)blockIdx.x * BLOCK * VPT + threadIdx.x;
    u32x4 v[VPT];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const uint64_t i = base + (uint64_t)k * BLOCK;
        if (i < nvec) v[k] = NT_LD ? __builtin_nontemporal_load(src + i) : src[i];
    }
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const uint64_t i = base + (uint64_t)k * BLOCK;
        if (i < nvec) {
            if (NT_ST) __builtin_nontemporal_store(v[k], dst + i);
            else dst[i] = v[k];
        }
    }
}

template <int BLOCK, int VPT, bool NT_LD, bool NT_ST>
__global__ __launch_bounds__(BLOCK) void k_xor(u32x4* __restrict__ buf, uint64_t nvec, uint32_t key) {
    const uint64_t base = (uint64_t)blockIdx.x * BLOCK * VPT + threadIdx.x;
    u32x4 v[VPT];
    const u32x4 km{key, key, key, key};
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const uint64_t i = base + (uint64_t)k * BLOCK;
        const uint64_t j = i < nvec ? i : nvec - 1;
        v[k] = NT_LD ? __builtin_nontemporal_load(buf + j) : buf[j];
    }
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const uint64_t i = base + (uint64_t)k * BLOCK;
        if (i < nvec) {
            if (NT_ST) __builtin_nontemporal_store(v[k] ^ km, buf + i);
            else buf[i] = v[k] ^ km;
        }
    }
}

// persistent: grid-stride over tiles, next tile's loads issued before this tile's stores
template <int BLOCK, int VPT, bool NT>
__global__ __launch_bounds__(BLOCK) void k_xor_persist(u32x4* __restrict__ buf, uint64_t nvec,
                                                       uint32_t key) {
    const uint64_t tile_vec = (uint64_t)BLOCK * VPT;
    const uint64_t ntiles = (nvec + tile_vec - 1) / tile_vec;
    const u32x4 km{key, key, key, key};
    uint64_t t = blockIdx.x;
    if (t >= ntiles) return;
    u32x4 cur[VPT];
    auto load = [&](uint64_t tt, u32x4* v) {
#pragma unroll
        for (int k = 0; k < VPT; ++k) {
            uint64_t i = tt * tile_vec + (uint64_t)k * BLOCK + threadIdx.x;
            i = i < nvec ? i : nvec - 1;
            v[k] = NT ? __builtin_nontemporal_load(buf + i) : buf[i];
        }
    };
    load(t, cur);
    for (; t < ntiles; t += gridDim.x) {
        u32x4 nxt[VPT];
        const uint64_t tn = t + gridDim.x;
        if (tn < ntiles) load(tn, nxt);
#pragma unroll
        for (int k = 0; k < VPT; ++k) {
            const uint64_t i = t * tile_vec + (uint64_t)k * BLOCK + threadIdx.x;
            if (i < nvec) {
                if (NT) __builtin_nontemporal_store(cur[k] ^ km, buf + i);
                else buf[i] = cur[k] ^ km;
            }
        }
#pragma unroll
        for (int k = 0; k < VPT; ++k) cur[k] = nxt[k];
    }
}


// wave-contiguous: wave w of the block owns a contiguous VPT KiB span
template <int BLOCK, int VPT>
__global__ __launch_bounds__(BLOCK) void k_xor_wavecontig(u32x4* __restrict__ buf, uint64_t nvec,
                                                          uint32_t key) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * BLOCK * VPT + (uint64_t)wave * 64 * VPT + lane;
    const u32x4 km{key, key, key, key};
    u32x4 v[VPT];
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        uint64_t i = base + (uint64_t)k * 64;
        i = i < nvec ? i : nvec - 1;
        v[k] = __builtin_nontemporal_load(buf + i);
    }
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
        const uint64_t i = base + (uint64_t)k * 64;
        if (i < nvec) __builtin_nontemporal_store(v[k] ^ km, buf + i);
    }
}

// raw buffer ops with explicit cache-policy aux bits (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
template <int BLOCK, int VPT, int AUXL, int AUXS>
__global__ __launch_bounds__(BLOCK) void k_xor_buf(u32x4* buf, uint64_t nvec, uint32_t key) {
    // one descriptor per 2 GiB window (32-bit voffset)
    const uint64_t tile0 = (uint64_t)blockIdx.x * BLOCK * VPT;
    const uint64_t win = tile0 & ~((1ull << 27) - 1);  // in vectors: 2 GiB windows
    char* wbase = (char*)(buf + win);
    const uint64_t left = (nvec - win) * 16;
    const uint32_t nbytes = left > 0x80000000ull ? 0x80000000u : (uint32_t)left;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(wbase, 0, nbytes, 0x00020000);
    const u32x4 km{key, key, key, key};
    u32x4 v[VPT];
    const uint32_t off0 = (uint32_t)((tile0 - win) * 16) + threadIdx.x * 16;
#pragma unroll
    for (int k = 0; k < VPT; ++k)
        v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off0 + k * BLOCK * 16, 0, AUXL));
#pragma unroll
    for (int k = 0; k < VPT; ++k)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v[k] ^ km), r, off0 + k * BLOCK * 16, 0, AUXS);
}


// v1 tile + the production kernel's per-tile lookups (first_bad, tile map, descriptor)
struct Desc { uint64_t ps, pl; uint32_t key, msg; uint32_t misc, wl; };
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_xor_lookup(u32x4* __restrict__ buf, uint64_t nvec,
                                                      const uint32_t* __restrict__ first_bad,
                                                      const uint32_t* __restrict__ tmap,
                                                      const Desc* __restrict__ desc) {
    const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t j = i < nvec ? i : nvec - 1;
    u32x4 v = __builtin_nontemporal_load(buf + j);
    const uint32_t nb = *first_bad;
    if (nb == 0) return;
    const uint32_t f = tmap[blockIdx.x];
    const uint32_t key = desc[f].key;
    const uint64_t ps = desc[f].ps, pe = ps + desc[f].pl;
    const uint64_t a = i * 16;
    if (a >= ps && a + 16 <= pe && i < nvec) {
        const u32x4 km{key, key, key, key};
        __builtin_nontemporal_store(v ^ km, buf + i);
    }
}

struct Variant {
    std::string name;
    std::function<void(hipStream_t)> run;
    std::vector<float> ms;
};

int main(int argc, char** argv) {
    uint64_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 0) : 0;
    if (!bytes) bytes = 65536ull * 65552ull;
    const int rounds = argc > 2 ? atoi(argv[2]) : 10;
    const uint64_t nvec = bytes / 16;
    u32x4 *a, *b;
    CK(hipMalloc(&a, nvec * 16));
    CK(hipMalloc(&b, nvec * 16));
    CK(hipMemset(a, 0x5a, nvec * 16));
    CK(hipMemset(b, 0, nvec * 16));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));

    std::vector<Variant> V;
#define GRID(B, VPT) dim3((unsigned)((nvec + (uint64_t)(B) * (VPT) - 1) / ((uint64_t)(B) * (VPT))))
#define ADD_COPY(B, VPT, NL, NS)                                                                     \
    V.push_back({"copy b" #B " v" #VPT " ntld" #NL " ntst" #NS,                                      \
                 [=](hipStream_t st) { hipLaunchKernelGGL((k_copy<B, VPT, NL, NS>), GRID(B, VPT), dim3(B), 0, st, a, b, nvec); }, {}})
#define ADD_XOR(B, VPT, NL, NS)                                                                      \
    V.push_back({"xor  b" #B " v" #VPT " ntld" #NL " ntst" #NS,                                      \
                 [=](hipStream_t st) { hipLaunchKernelGGL((k_xor<B, VPT, NL, NS>), GRID(B, VPT), dim3(B), 0, st, a, nvec, 0x12345678u); }, {}})
#define ADD_PERSIST(B, VPT, NT, WPC)                                                                 \
    V.push_back({"pers b" #B " v" #VPT " nt" #NT " wg/cu" #WPC,                                      \
                 [=](hipStream_t st) { hipLaunchKernelGGL((k_xor_persist<B, VPT, NT>), dim3(ncu * WPC), dim3(B), 0, st, a, nvec, 0x9u); }, {}})
    ADD_COPY(64, 1, true, true);
    ADD_XOR(64, 1, true, true);
    ADD_XOR(64, 1, false, false);
    ADD_XOR(64, 1, true, false);
    ADD_XOR(64, 1, false, true);
    ADD_XOR(128, 1, true, true);
    ADD_XOR(256, 1, true, true);
    V.push_back({"buf b64 aux nt/nt", [=](hipStream_t st) { hipLaunchKernelGGL((k_xor_buf<64, 1, 2, 2>), GRID(64, 1), dim3(64), 0, st, a, nvec, 5u); }, {}});
    V.push_back({"buf b64 aux sc1|nt/nt", [=](hipStream_t st) { hipLaunchKernelGGL((k_xor_buf<64, 1, 18, 2>), GRID(64, 1), dim3(64), 0, st, a, nvec, 5u); }, {}});
    V.push_back({"buf b64 aux nt/sc1|nt", [=](hipStream_t st) { hipLaunchKernelGGL((k_xor_buf<64, 1, 2, 18>), GRID(64, 1), dim3(64), 0, st, a, nvec, 5u); }, {}});
    V.push_back({"buf b64 aux sc0|nt/sc0|nt", [=](hipStream_t st) { hipLaunchKernelGGL((k_xor_buf<64, 1, 3, 3>), GRID(64, 1), dim3(64), 0, st, a, nvec, 5u); }, {}});
    {
        const uint64_t ntile = (nvec + 255) / 256;
        uint32_t *fb, *tm;
        Desc* dd;
        CK(hipMalloc(&fb, 4));
        CK(hipMalloc(&tm, ntile * 4));
        CK(hipMalloc(&dd, 65536 * sizeof(Desc)));
        std::vector<uint32_t> h(ntile);
        for (uint64_t t = 0; t < ntile; ++t) h[t] = (uint32_t)std::min<uint64_t>((t * 4096) / 65550, 65535);
        CK(hipMemcpy(tm, h.data(), ntile * 4, hipMemcpyHostToDevice));
        uint32_t nbv = 65536;
        CK(hipMemcpy(fb, &nbv, 4, hipMemcpyHostToDevice));
        std::vector<Desc> hd(65536);
        for (int f = 0; f < 65536; ++f) hd[f] = Desc{(uint64_t)f * 65550 + 14, 65536, 0x11223344u, 0, 0, 0};
        CK(hipMemcpy(dd, hd.data(), 65536 * sizeof(Desc), hipMemcpyHostToDevice));
        V.push_back({"lookup b256 v1", [=](hipStream_t st) { hipLaunchKernelGGL((k_xor_lookup<256>), dim3((unsigned)ntile), dim3(256), 0, st, a, nvec, fb, tm, dd); }, {}});
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v : V) v.run(s);  // warm
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < rounds; ++r) {
        for (auto& v : V) {
            CK(hipEventRecord(e0, s));
            v.run(s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms);
        }
    }
    printf("buffer %.3f GB, %d rounds, %d CUs; GB/s = (read+write bytes)/time\n", nvec * 16 / 1e9,
           rounds, ncu);
    for (auto& v : V) {
        std::sort(v.ms.begin(), v.ms.end());
        const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
        printf("%-34s median %8.3f ms  %7.1f GB/s   best %7.1f GB/s\n", v.name.c_str(), med,
               2.0 * nvec * 16 / (med * 1e-3) / 1e9, 2.0 * nvec * 16 / (best * 1e-3) / 1e9);
    }
    return 0;
}
