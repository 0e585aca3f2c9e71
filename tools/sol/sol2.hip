// sol2.hip — speed-of-light micro-benchmarks for an LDS-DMA (global_load_lds)
// receive pipeline on MI355X, beside the register-staged loads the kernels use today.
//   glds  <S>      : each wave streams 4-KiB runs (64 frames x 64 B) straight into an
//                    S-stage LDS ring with global_load_lds_dwordx4 (no VGPR destination),
//                    counted vmcnt, lane l reads frame l back (source-swizzled, conflict-free)
//   glds+cols <S>  : the same + 26 B/frame of non-temporal SoA column stores
//   reg+cols       : register-staged 4 KiB per run, one run prefetched (today's shape)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/sol/sol2 tools/sol/sol2.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) const void* gptr_t;

// LDS-DMA issued from inline asm: hipcc does not track it, so it does not put a
// vmcnt(0) before every ds_read of the ring (it does for the builtin, whose LDS
// write it must assume aliases every LDS read); completion is counted by hand.
template <int AUX>
__device__ __forceinline__ void glds16(const void* gsrc, const void* lds) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)lds);
    uint32_t keep;
    if (AUX == 2)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(m) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(m) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

struct Cols { uint16_t* c16; uint32_t* c32; uint8_t* c8; };

// FPL frames per lane: lane l owns frames [FPL*l, FPL*l + FPL) of the wave's
// 64*FPL-frame step, so one store instruction writes FPL elements per lane
// (u16: 128/256/512 B per wave instruction, u32: 256/512/1024 B, u8: 64/128/256 B).
template <int FPL> struct Vec;
template <> struct Vec<1> { typedef uint16_t h; typedef uint32_t w; typedef uint8_t b; };
template <> struct Vec<2> { typedef uint32_t h; typedef uint2 w; typedef uint16_t b; };
template <> struct Vec<4> { typedef uint2 h; typedef uint4 w; typedef uint32_t b; };
template <class T> __device__ __forceinline__ T splat(uint32_t x) {
    if constexpr (sizeof(T) == 16) return T{x, x + 1, x + 2, x + 3};
    else if constexpr (sizeof(T) == 8) return T{x, x + 1};
    else return (T)x;
}
template <class T, bool NT> __device__ __forceinline__ void st(T* p, T v) {
    if constexpr (NT) {
        if constexpr (sizeof(T) == 16) {
            typedef unsigned int v4 __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(v4{v.x, v.y, v.z, v.w}, reinterpret_cast<v4*>(p));
        } else if constexpr (sizeof(T) == 8) {
            typedef unsigned int v2 __attribute__((ext_vector_type(2)));
            __builtin_nontemporal_store(v2{v.x, v.y}, reinterpret_cast<v2*>(p));
        } else {
            __builtin_nontemporal_store(v, p);
        }
    } else {
        *p = v;
    }
}
// 12 store instructions: 8 u16 columns, 2 u32, 2 u8 (26 B/frame); g = FPL-group index
template <int FPL, bool NT>
__device__ __forceinline__ void store_cols(const Cols& c, size_t nframes, size_t g, uint32_t x) {
    typedef typename Vec<FPL>::h H; typedef typename Vec<FPL>::w W; typedef typename Vec<FPL>::b B;
    const size_t ng = nframes / FPL;
#pragma unroll
    for (int k = 0; k < 8; ++k) st<H, NT>(reinterpret_cast<H*>(c.c16) + (size_t)k * ng + g, splat<H>(x + k));
    st<W, NT>(reinterpret_cast<W*>(c.c32) + g, splat<W>(x));
    st<W, NT>(reinterpret_cast<W*>(c.c32) + ng + g, splat<W>(x ^ 1));
    st<B, NT>(reinterpret_cast<B*>(c.c8) + g, splat<B>(x));
    st<B, NT>(reinterpret_cast<B*>(c.c8) + ng + g, splat<B>(x >> 8));
}
constexpr int kNst = 12;   // store instructions per step above

// S-stage ring per wave, each stage FPL runs of 4 KiB (64*FPL frames); WPB waves per block.
template <int S, int WPB, int FPL, int AUX, int COLS>   // COLS 0: none, 1: nt stores, 2: plain stores
__global__ __launch_bounds__(64 * WPB) void glds_kernel(const uint8_t* __restrict__ in, size_t nframes, Cols c,
                                                        uint32_t* o) {
    constexpr int kStage = 4096 * FPL;
    __shared__ __attribute__((aligned(16))) uint8_t ring[WPB][S][kStage];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t nsteps = nframes / (64 * FPL);
    const size_t w = (size_t)blockIdx.x * WPB + wv, nw = (size_t)gridDim.x * WPB;
    // LDS granule p = 64i + L holds chunk ((L&3) - (L>>4)) & 3 of frame 16i + L/4
    const uint32_t lane_off = (uint32_t)(lane >> 2) * 64u + ((uint32_t)((lane & 3) - (lane >> 4)) & 3u) * 16u;
    auto issue = [&](size_t step, int stg) {
        const uint8_t* src = in + step * kStage + lane_off;
#pragma unroll
        for (int i = 0; i < 4 * FPL; ++i) glds16<AUX>(src + i * 1024, &ring[wv][stg][i * 1024]);
    };
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
        if (w + s * nw < nsteps) issue(w + s * nw, s);
    uint32_t acc = 0;
    int stg = 0;
    for (size_t step = w; step < nsteps; step += nw) {
        const size_t ahead = step + (size_t)(S - 1) * nw;
        const bool full = ahead < nsteps;
        if (full) issue(ahead, (stg + S - 1) % S);
        if (full) wait_vm<(S - 1) * (4 * FPL + (COLS ? kNst : 0))>();
        else wait_vm<0>();
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < FPL; ++j) {
            const uint8_t* fr = &ring[wv][stg][j * 4096 + lane * 64];
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                const int cp = (cc + (lane >> 2)) & 3;
                const uint4 v = *reinterpret_cast<const uint4*>(fr + 16 * cp);
                x += v.x ^ (v.y + cc) ^ v.z ^ v.w;
            }
        }
        if (COLS) store_cols<FPL, COLS == 1>(c, nframes, step * 64 + lane, x);
        else acc += x;
        stg = (stg + 1) % S;
    }
    if (acc == 0x12345678u) o[0] = acc;
}

// write-only: the 26 B/frame column stores alone
template <int FPL, bool NT>
__global__ __launch_bounds__(256) void write_kernel(size_t nframes, Cols c) {
    const size_t ng = nframes / FPL;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t g = (size_t)blockIdx.x * blockDim.x + threadIdx.x; g < ng; g += stride)
        store_cols<FPL, NT>(c, nframes, g, (uint32_t)g);
}

// register-staged, one run prefetched (the rx_small_kernel load shape)
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void reg_cols_kernel(const uint4* __restrict__ in, size_t nframes, Cols c) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t nruns = nframes / 64;
    const size_t w = (size_t)blockIdx.x * WPB + wv, nw = (size_t)gridDim.x * WPB;
    typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
    auto ld = [&](size_t run, uint4* v) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            u32x4_t t = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(in + run * 256 + 64 * i + lane));
            v[i] = make_uint4(t.x, t.y, t.z, t.w);
        }
    };
    uint4 cur[4], nxt[4];
    if (w < nruns) ld(w, cur);
    for (size_t run = w; run < nruns; run += nw) {
        if (run + nw < nruns) ld(run + nw, nxt);
        uint32_t x = cur[0].x ^ cur[1].y ^ cur[2].z ^ cur[3].w;
        store_cols<1, true>(c, nframes, run * 64 + lane, x);
#pragma unroll
        for (int i = 0; i < 4; ++i) cur[i] = nxt[i];
    }
}

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n16) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) out[i] = in[i];
}

template <class F>
float time_it(F f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    f(); f();
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
        (void)hipEventRecord(a); f(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms; (void)hipEventElapsedTime(&ms, a, b); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    const size_t bytes = 1ull << 30, nframes = bytes / 64;
    uint8_t* in; uint8_t* out; uint32_t* o; Cols c;
    CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, bytes)); CK(hipMalloc(&o, 64));
    CK(hipMalloc(&c.c16, nframes * 16)); CK(hipMalloc(&c.c32, nframes * 8)); CK(hipMalloc(&c.c8, nframes * 2));
    CK(hipMemset(in, 1, bytes));
    const int cus = 256;
    const double rd = (double)bytes, rw = (double)bytes + nframes * 26.0;
    auto run_k = [&](const char* label, int wpb, int bpc, double total, auto kern, auto... args) {
        const int grid = cus * bpc;
        float ms = time_it([&] { kern<<<grid, 64 * wpb>>>(args...); }, 20);
        printf("%-34s wpb=%d blk/CU=%2d waves/CU=%2d: %7.1f us %6.0f GB/s\n", label, wpb, bpc, wpb * bpc, ms * 1e3,
               total / ms / 1e6);
    };
#define RUN(label, kern, args, wpb, bpc, total) run_k(label, wpb, bpc, total, kern, UNPAREN args);
#define UNPAREN(...) __VA_ARGS__
    const double wr = nframes * 26.0;
    RUN("copy (reference point)", (copy_kernel), ((const uint4*)in, (uint4*)out, bytes / 16), 4, 8, 2.0 * bytes)
    // read-only streams (S stages x FPL runs per wave)
    RUN("glds S4 F1 nt read", (glds_kernel<4, 4, 1, 2, 0>), (in, nframes, c, o), 4, 2, rd)
    RUN("glds S3 F1 nt read", (glds_kernel<3, 4, 1, 2, 0>), (in, nframes, c, o), 4, 3, rd)
    RUN("glds S4 F1 nt read", (glds_kernel<4, 1, 1, 2, 0>), (in, nframes, c, o), 1, 8, rd)
    RUN("glds S3 F2 nt read", (glds_kernel<3, 2, 2, 2, 0>), (in, nframes, c, o), 2, 3, rd)
    RUN("glds S2 F2 nt read", (glds_kernel<2, 4, 2, 2, 0>), (in, nframes, c, o), 4, 2, rd)
    RUN("glds S6 F1 nt read", (glds_kernel<6, 2, 1, 2, 0>), (in, nframes, c, o), 2, 3, rd)
    RUN("glds S4 F1 def read", (glds_kernel<4, 4, 1, 0, 0>), (in, nframes, c, o), 4, 2, rd)
    // write-only
    RUN("write F1 nt", (write_kernel<1, true>), (nframes, c), 4, 8, wr)
    RUN("write F2 nt", (write_kernel<2, true>), (nframes, c), 4, 8, wr)
    RUN("write F4 nt", (write_kernel<4, true>), (nframes, c), 4, 8, wr)
    RUN("write F1 plain", (write_kernel<1, false>), (nframes, c), 4, 8, wr)
    RUN("write F4 plain", (write_kernel<4, false>), (nframes, c), 4, 8, wr)
    // read + 26 B/frame of columns
    RUN("reg +cols (today's shape)", (reg_cols_kernel<4>), ((const uint4*)in, nframes, c), 4, 3, rw)
    RUN("glds S3 F1 +cols nt", (glds_kernel<3, 4, 1, 2, 1>), (in, nframes, c, o), 4, 3, rw)
    RUN("glds S4 F1 +cols nt", (glds_kernel<4, 4, 1, 2, 1>), (in, nframes, c, o), 4, 2, rw)
    RUN("glds S4 F1 +cols nt", (glds_kernel<4, 1, 1, 2, 1>), (in, nframes, c, o), 1, 8, rw)
    RUN("glds S3 F1 +cols plain", (glds_kernel<3, 4, 1, 2, 2>), (in, nframes, c, o), 4, 3, rw)
    RUN("glds S4 F1 +cols plain", (glds_kernel<4, 4, 1, 2, 2>), (in, nframes, c, o), 4, 2, rw)
    RUN("glds S2 F2 +cols nt", (glds_kernel<2, 4, 2, 2, 1>), (in, nframes, c, o), 4, 2, rw)
    RUN("glds S3 F2 +cols nt", (glds_kernel<3, 2, 2, 2, 1>), (in, nframes, c, o), 2, 3, rw)
    RUN("glds S3 F2 +cols nt", (glds_kernel<3, 1, 2, 2, 1>), (in, nframes, c, o), 1, 6, rw)
    RUN("glds S4 F2 +cols nt", (glds_kernel<4, 1, 2, 2, 1>), (in, nframes, c, o), 1, 4, rw)
    RUN("glds S3 F2 +cols plain", (glds_kernel<3, 2, 2, 2, 2>), (in, nframes, c, o), 2, 3, rw)
    RUN("glds S2 F4 +cols nt", (glds_kernel<2, 1, 4, 2, 1>), (in, nframes, c, o), 1, 4, rw)
    RUN("glds S3 F4 +cols nt", (glds_kernel<3, 1, 4, 2, 1>), (in, nframes, c, o), 1, 3, rw)
    RUN("glds S2 F4 +cols plain", (glds_kernel<2, 1, 4, 2, 2>), (in, nframes, c, o), 1, 4, rw)
    return 0;
}
