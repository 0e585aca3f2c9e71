// sol3.hip — load shapes for MTU-size frames (1500-B stride, 2^20 frames = 1.5 GiB) on MI355X:
//   contig   : glds of the byte stream, 1 KiB contiguous per wave instruction (the reference point)
//   grp8     : 8 lanes per frame, 8 frames x 128 B per wave instruction (the MTU kernel's shape),
//              loaded by glds into an S-deep ring of 1-KiB slots, or into registers (U in flight)
// Every lane reads back only the granule it loaded (sum of words), so LDS is conflict-free.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/sol/sol3 tools/sol/sol3.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void glds16(const void* gsrc, const void* lds) {
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_ptr_t)lds);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(m) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ uint32_t sad(uint32_t d, uint32_t acc) { return __builtin_amdgcn_sad_u16(d, 0u, acc); }
__device__ __forceinline__ uint32_t sum16(uint4 v, uint32_t a) { return sad(v.w, sad(v.z, sad(v.y, sad(v.x, a)))); }

constexpr uint32_t kStride = 1500;

// contiguous stream, S-deep ring of 1-KiB slots per wave
template <int S, int WPB>
__global__ __launch_bounds__(64 * WPB) void contig_kernel(const uint8_t* __restrict__ in, size_t bytes, uint32_t* o) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[WPB][S][1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t w = (size_t)blockIdx.x * WPB + wv, nw = (size_t)gridDim.x * WPB;
    constexpr size_t kChunk = 16384;   // a wave streams 16 KiB contiguous, then jumps
    const size_t nchunks = bytes / kChunk;
    uint32_t acc = 0;
    for (size_t ch = w; ch < nchunks; ch += nw) {
        const uint8_t* src = in + ch * kChunk + 16 * lane;
#pragma unroll
        for (int s = 0; s < S - 1; ++s) glds16(src + s * 1024, &ring[wv][s][0]);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (i + S - 1 < 16) { glds16(src + (i + S - 1) * 1024, &ring[wv][(i + S - 1) % S][0]); wait_vm<S - 1>(); }
            else wait_vm<0>();
            acc = sum16(*reinterpret_cast<const uint4*>(&ring[wv][i % S][16 * lane]), acc);
        }
    }
    if (acc == 0x12345678u) o[0] = acc;
}

// 8 lanes per frame: lane (q = lane/8, r = lane%8) loads granule 8k + r of frame q of the wave's
// current 8-frame round; a wave owns 64 consecutive frames = 8 rounds. 1500 B = 11.7 x 128 B,
// so 12 instructions per round (the last one partly masked).
template <int S, int WPB>
__global__ __launch_bounds__(64 * WPB) void grp8_glds_kernel(const uint8_t* __restrict__ in, size_t nframes, uint32_t* o) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[WPB][S][1024];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t w = (size_t)blockIdx.x * WPB + wv, nw = (size_t)gridDim.x * WPB;
    const size_t nruns = nframes / 64;
    uint32_t acc = 0;
    const int q = lane >> 3, r = lane & 7;
    constexpr int kIns = (kStride + 127) / 128;   // 12
    for (size_t run = w; run < nruns; run += nw) {
        for (int rd = 0; rd < 8; ++rd) {
            const uint8_t* fr = in + (run * 64 + rd * 8 + q) * kStride;
            const uint8_t* src = fr + 16 * r;
            // masked granules past the frame end re-load granule 0 (same lines, harmless)
            auto addr = [&](int k) { const int off = 128 * k + 16 * r; return off + 16 <= (int)kStride ? fr + off : src; };
#pragma unroll
            for (int s = 0; s < S - 1; ++s) glds16(addr(s), &ring[wv][s][0]);
#pragma unroll
            for (int k = 0; k < kIns; ++k) {
                if (k + S - 1 < kIns) { glds16(addr(k + S - 1), &ring[wv][(k + S - 1) % S][0]); wait_vm<S - 1>(); }
                else wait_vm<0>();
                acc = sum16(*reinterpret_cast<const uint4*>(&ring[wv][k % S][16 * lane]), acc);
            }
        }
    }
    if (acc == 0x12345678u) o[0] = acc;
}

template <int U, int WPB>
__global__ __launch_bounds__(64 * WPB) void grp8_reg_kernel(const uint8_t* __restrict__ in, size_t nframes, uint32_t* o) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const size_t w = (size_t)blockIdx.x * WPB + wv, nw = (size_t)gridDim.x * WPB;
    const size_t nruns = nframes / 64;
    uint32_t acc = 0;
    const int q = lane >> 3, r = lane & 7;
    constexpr int kIns = (kStride + 127) / 128;
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    for (size_t run = w; run < nruns; run += nw) {
        for (int rd = 0; rd < 8; ++rd) {
            const uint8_t* fr = in + (run * 64 + rd * 8 + q) * kStride;
            for (int k0 = 0; k0 < kIns; k0 += U) {
                uint4 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int off = 128 * (k0 + u) + 16 * r;
                    v[u] = make_uint4(0, 0, 0, 0);
                    if (k0 + u < kIns && off + 16 <= (int)kStride) {
                        v4 t = __builtin_nontemporal_load(reinterpret_cast<const v4*>(fr + off));
                        v[u] = make_uint4(t.x, t.y, t.z, t.w);
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) acc = sum16(v[u], acc);
            }
        }
    }
    if (acc == 0x12345678u) o[0] = acc;
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
    const size_t nframes = 1u << 20, bytes = nframes * kStride;
    uint8_t* in; uint32_t* o;
    CK(hipMalloc(&in, bytes + 4096)); CK(hipMalloc(&o, 64));
    CK(hipMemset(in, 1, bytes + 4096));
    const int cus = 256;
    auto run_k = [&](const char* label, int wpb, int bpc, auto kern, auto... args) {
        const int grid = cus * bpc;
        float ms = time_it([&] { kern<<<grid, 64 * wpb>>>(args...); }, 20);
        printf("%-28s wpb=%d blk/CU=%2d waves/CU=%2d: %7.1f us %6.0f GB/s\n", label, wpb, bpc, wpb * bpc, ms * 1e3,
               bytes / ms / 1e6);
    };
    const size_t cbytes = bytes / 16384 * 16384;
    run_k("contig glds S8", 4, 2, contig_kernel<8, 4>, in, cbytes, o);
    run_k("contig glds S8", 4, 4, contig_kernel<8, 4>, in, cbytes, o);
    run_k("contig glds S16", 4, 2, contig_kernel<16, 4>, in, cbytes, o);
    run_k("contig glds S16", 4, 4, contig_kernel<16, 4>, in, cbytes, o);
    run_k("grp8 glds S4", 4, 4, grp8_glds_kernel<4, 4>, in, nframes, o);
    run_k("grp8 glds S8", 4, 2, grp8_glds_kernel<8, 4>, in, nframes, o);
    run_k("grp8 glds S8", 4, 4, grp8_glds_kernel<8, 4>, in, nframes, o);
    run_k("grp8 glds S12", 4, 4, grp8_glds_kernel<12, 4>, in, nframes, o);
    run_k("grp8 glds S12", 4, 8, grp8_glds_kernel<12, 4>, in, nframes, o);
    run_k("grp8 reg U4", 4, 4, grp8_reg_kernel<4, 4>, in, nframes, o);
    run_k("grp8 reg U4", 4, 8, grp8_reg_kernel<4, 4>, in, nframes, o);
    run_k("grp8 reg U6", 4, 4, grp8_reg_kernel<6, 4>, in, nframes, o);
    run_k("grp8 reg U12", 4, 2, grp8_reg_kernel<12, 4>, in, nframes, o);
    run_k("grp8 reg U12", 4, 4, grp8_reg_kernel<12, 4>, in, nframes, o);
    return 0;
}
