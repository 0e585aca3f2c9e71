// sol.hip — speed-of-light micro-benchmarks for the receive path's traffic mix
// on MI355X: how fast can a kernel that does NO parsing move the same bytes?
//   read      : stream 1 GiB with coalesced dwordx4 loads, fold into one word/wave
//   read+cols : the same reads + 26 B/frame of SoA column stores (64-B frames)
//   copy      : float4 copy 1 GiB -> 1 GiB (the guide's 6.29 TB/s reference point)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/sol/sol tools/sol/sol.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void read_kernel(const uint4* __restrict__ in, size_t n16, uint32_t* out) {
    uint32_t acc = 0;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < n16; i += UNROLL * stride) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if (NT) { u32x4_t t = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(in + i + u * stride)); v[u] = make_uint4(t.x, t.y, t.z, t.w); }
            else v[u] = in[i + u * stride];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) { uint4 t = in[i]; acc += t.x ^ t.y ^ t.z ^ t.w; }
    if (acc == 0x12345678u) out[0] = acc;   // keep the loads alive
}

// 64-B frames: wave loads 4 KiB (64 frames) coalesced, writes 26 B/frame of columns
__global__ __launch_bounds__(256) void read_cols_kernel(const uint4* __restrict__ in, size_t nframes, uint16_t* c16,
                                                        uint32_t* c32, uint8_t* c8) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t run = wave; run * 64 < nframes; run += nwaves) {
        const uint4* p = in + run * 256;
        uint4 v0 = p[lane], v1 = p[64 + lane], v2 = p[128 + lane], v3 = p[192 + lane];
        uint32_t x = v0.x ^ v1.y ^ v2.z ^ v3.w;
        const size_t f = run * 64 + lane;
        // 8 x u16 columns + 2 x u32 + 2 x u8 = 26 B
#pragma unroll
        for (int k = 0; k < 8; ++k) c16[(size_t)k * nframes + f] = (uint16_t)(x + k);
        c32[f] = x;
        c32[nframes + f] = x ^ 1;
        c8[f] = (uint8_t)x;
        c8[nframes + f] = (uint8_t)(x >> 8);
    }
}

// 128 frames (8 KiB) per wave iteration, 2 frames per lane: every column store
// is a full-line wave instruction (u8 pairs 128 B, u16 pairs 256 B, u32 pairs 512 B)
__global__ __launch_bounds__(256) void read_cols2_kernel(const uint4* __restrict__ in, size_t nframes, uint16_t* c16,
                                                         uint32_t* c32, uint8_t* c8) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t run = wave; run * 128 < nframes; run += nwaves) {
        const uint4* p = in + run * 512;
        uint4 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = p[64 * i + lane];
        uint32_t x = v[0].x ^ v[1].y ^ v[2].z ^ v[3].w, y = v[4].x ^ v[5].y ^ v[6].z ^ v[7].w;
        const size_t f = run * 128 + 2 * lane;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            *reinterpret_cast<uint32_t*>(c16 + (size_t)k * nframes + f) = (x + k) & 0xFFFFu | ((y + k) << 16);
        *reinterpret_cast<uint2*>(c32 + f) = make_uint2(x, y);
        *reinterpret_cast<uint2*>(c32 + nframes + f) = make_uint2(x ^ 1, y ^ 1);
        *reinterpret_cast<uint16_t*>(c8 + f) = (uint16_t)((x & 0xFF) | ((y & 0xFF) << 8));
        *reinterpret_cast<uint16_t*>(c8 + nframes + f) = (uint16_t)(((x >> 8) & 0xFF) | (y & 0xFF00));
    }
}

// same reads as read_cols, stores non-temporal (the receive kernels' policy)
__global__ __launch_bounds__(256) void read_cols_nt_kernel(const uint4* __restrict__ in, size_t nframes, uint16_t* c16,
                                                           uint32_t* c32, uint8_t* c8) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t run = wave; run * 64 < nframes; run += nwaves) {
        const uint4* p = in + run * 256;
        uint4 v0 = p[lane], v1 = p[64 + lane], v2 = p[128 + lane], v3 = p[192 + lane];
        uint32_t x = v0.x ^ v1.y ^ v2.z ^ v3.w;
        const size_t f = run * 64 + lane;
#pragma unroll
        for (int k = 0; k < 8; ++k) __builtin_nontemporal_store((uint16_t)(x + k), c16 + (size_t)k * nframes + f);
        __builtin_nontemporal_store(x, c32 + f);
        __builtin_nontemporal_store(x ^ 1, c32 + nframes + f);
        __builtin_nontemporal_store((uint8_t)x, c8 + f);
        __builtin_nontemporal_store((uint8_t)(x >> 8), c8 + nframes + f);
    }
}

// same reads; the run's 26 B/frame of columns staged in LDS and written as
// 16-B-per-lane stores (2 wave instructions instead of 12 narrow ones)
__global__ __launch_bounds__(256) void read_cols_lds_kernel(const uint4* __restrict__ in, size_t nframes,
                                                            uint16_t* c16, uint32_t* c32, uint8_t* c8) {
    __shared__ __attribute__((aligned(16))) uint8_t stage[4][1664];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint8_t* st = stage[wv];
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t run = wave; run * 64 < nframes; run += nwaves) {
        const uint4* p = in + run * 256;
        uint4 v0 = p[lane], v1 = p[64 + lane], v2 = p[128 + lane], v3 = p[192 + lane];
        uint32_t x = v0.x ^ v1.y ^ v2.z ^ v3.w;
        // staging layout: 8 u16 columns (128 B each), 2 u32 (256 B each), 2 u8 (64 B each)
#pragma unroll
        for (int k = 0; k < 8; ++k) reinterpret_cast<uint16_t*>(st + 128 * k)[lane] = (uint16_t)(x + k);
        reinterpret_cast<uint32_t*>(st + 1024)[lane] = x;
        reinterpret_cast<uint32_t*>(st + 1280)[lane] = x ^ 1;
        st[1536 + lane] = (uint8_t)x;
        st[1600 + lane] = (uint8_t)(x >> 8);
        __builtin_amdgcn_wave_barrier();
        const size_t f0 = run * 64;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = h * 64 + lane;       // 16-B piece index, 104 pieces
            if (q < 104) {
                const uint4 val = *reinterpret_cast<const uint4*>(st + 16 * q);
                uint8_t* dst;
                if (q < 64) dst = reinterpret_cast<uint8_t*>(c16 + (size_t)(q >> 3) * nframes + f0) + 16 * (q & 7);
                else if (q < 96) dst = reinterpret_cast<uint8_t*>(c32 + (size_t)((q - 64) >> 4) * nframes + f0) + 16 * ((q - 64) & 15);
                else dst = c8 + (size_t)((q - 96) >> 2) * nframes + f0 + 16 * ((q - 96) & 3);
                __builtin_nontemporal_store(*reinterpret_cast<const u32x4_t*>(&val), reinterpret_cast<u32x4_t*>(dst));
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// same reads, one packed 32-B record per frame (two dwordx4 stores per lane)
__global__ __launch_bounds__(256) void read_rec_kernel(const uint4* __restrict__ in, size_t nframes, uint4* rec) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t run = wave; run * 64 < nframes; run += nwaves) {
        const uint4* p = in + run * 256;
        uint4 v0 = p[lane], v1 = p[64 + lane], v2 = p[128 + lane], v3 = p[192 + lane];
        uint32_t x = v0.x ^ v1.y ^ v2.z ^ v3.w;
        const size_t f = run * 64 + lane;
        rec[2 * f] = make_uint4(x, x + 1, x + 2, x + 3);
        rec[2 * f + 1] = make_uint4(x + 4, x + 5, x + 6, x + 7);
    }
}

// each wave streams whole contiguous chunks of U*R KiB: R rounds of U 1-KiB
// wave loads (U in flight); chunks handed out round-robin over the waves
template <int U, int R>
__global__ __launch_bounds__(256) void read_chunk_kernel(const uint4* __restrict__ in, size_t n16, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    constexpr size_t kChunk = (size_t)U * R * 64;   // uint4 per chunk
    uint32_t acc = 0;
    for (size_t ch = wave; (ch + 1) * kChunk <= n16; ch += nwaves) {
        const uint4* p = in + ch * kChunk + lane;
#pragma unroll 1
        for (int r = 0; r < R; ++r) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = p[(r * U + u) * 64];
#pragma unroll
            for (int u = 0; u < U; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) out[i] = in[i];
}

template <class F>
float time_it(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    f(); f();
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(a); f(); hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const size_t bytes = 1ull << 30, n16 = bytes / 16, nframes = bytes / 64;
    uint4 *in, *out; uint32_t* o; uint16_t* c16; uint32_t* c32; uint8_t* c8;
    CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes)); CK(hipMalloc(&o, 64));
    CK(hipMalloc(&c16, nframes * 16)); CK(hipMalloc(&c32, nframes * 8)); CK(hipMalloc(&c8, nframes * 2));
    CK(hipMemset(in, 1, bytes));
    int cus = 256;
    for (int bpc : {4, 8, 16}) {
        const int grid = cus * bpc;
        float ms = time_it([&] { read_kernel<4, false><<<grid, 256>>>(in, n16, o); }, 20);
        printf("read    plain U4 grid=%5d: %7.1f us  %6.0f GB/s\n", grid, ms * 1e3, bytes / ms / 1e6);
        ms = time_it([&] { read_kernel<4, true><<<grid, 256>>>(in, n16, o); }, 20);
        printf("read    nt    U4 grid=%5d: %7.1f us  %6.0f GB/s\n", grid, ms * 1e3, bytes / ms / 1e6);
        ms = time_it([&] { read_kernel<8, false><<<grid, 256>>>(in, n16, o); }, 20);
        printf("read    plain U8 grid=%5d: %7.1f us  %6.0f GB/s\n", grid, ms * 1e3, bytes / ms / 1e6);
#define CHUNK(U, R)                                                                                   \
        ms = time_it([&] { read_chunk_kernel<U, R><<<grid, 256>>>(in, n16, o); }, 20);                    \
        printf("read    chunk U%-2d R%d (%3d KiB) grid=%5d: %7.1f us  %6.0f GB/s\n", U, R, U * R, grid, ms * 1e3, \
               bytes / ms / 1e6);
        CHUNK(4, 1) CHUNK(12, 1)
        ms = time_it([&] { read_cols_kernel<<<grid, 256>>>(in, nframes, c16, c32, c8); }, 20);
        printf("read+26B cols  grid=%5d: %7.1f us  %6.0f GB/s (alg %zu B)\n", grid, ms * 1e3,
               (bytes + nframes * 26) / ms / 1e6, bytes + nframes * 26);
        ms = time_it([&] { read_cols_nt_kernel<<<grid, 256>>>(in, nframes, c16, c32, c8); }, 20);
        printf("read+26B cols nt grid=%5d: %7.1f us  %6.0f GB/s\n", grid, ms * 1e3, (bytes + nframes * 26) / ms / 1e6);
        ms = time_it([&] { read_cols_lds_kernel<<<grid, 256>>>(in, nframes, c16, c32, c8); }, 20);
        printf("read+26B cols lds16 grid=%5d: %7.1f us  %6.0f GB/s\n", grid, ms * 1e3, (bytes + nframes * 26) / ms / 1e6);
        ms = time_it([&] { read_cols2_kernel<<<grid, 256>>>(in, nframes, c16, c32, c8); }, 20);
        printf("read+26B cols x2 grid=%5d: %7.1f us  %6.0f GB/s\n", grid, ms * 1e3, (bytes + nframes * 26) / ms / 1e6);
        ms = time_it([&] { read_rec_kernel<<<grid, 256>>>(in, nframes, out); }, 20);
        printf("read+32B rec   grid=%5d: %7.1f us  %6.0f GB/s (alg %zu B)\n", grid, ms * 1e3,
               (bytes + nframes * 32) / ms / 1e6, bytes + nframes * 32);
        ms = time_it([&] { copy_kernel<<<grid, 256>>>(in, out, n16); }, 20);
        printf("copy           grid=%5d: %7.1f us  %6.0f GB/s (r+w)\n", grid, ms * 1e3, 2.0 * bytes / ms / 1e6);
    }
    return 0;
}
