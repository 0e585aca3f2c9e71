// sol5.hip — write shapes on MI355X: how fast can a kernel write 416 MiB
// (the 64-B workload's 26 B/frame of result columns), alone and beside a
// 1-GiB read stream, as a function of the bytes one wave store instruction covers.
//   wN   : pure writes, each lane stores N bytes (one instruction = 64 N bytes)
//   r+wN : glds read stream (4-KiB steps, 3-step ring) + the same writes, per step
//          64 N bytes x K instructions so that writes / reads = 26 / 64
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/sol/sol5 tools/sol/sol5.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void glds16_nt_s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_addr) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// dword store with explicit gfx950 cache-policy bits (POL: 0 none, 1 nt, 2 sc0 sc1, 3 sc0 sc1 nt, 4 sc1, 5 sc0)
template <int POL>
__device__ __forceinline__ void st_pol(uint8_t* p, uint32_t x) {
    if constexpr (POL == 0) asm volatile("global_store_dword %0, %1, off" ::"v"(p), "v"(x) : "memory");
    else if constexpr (POL == 1) asm volatile("global_store_dword %0, %1, off nt" ::"v"(p), "v"(x) : "memory");
    else if constexpr (POL == 2) asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(x) : "memory");
    else if constexpr (POL == 3) asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(x) : "memory");
    else if constexpr (POL == 4) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
    else asm volatile("global_store_dword %0, %1, off sc0" ::"v"(p), "v"(x) : "memory");
}
template <int NB, bool NT>
__device__ __forceinline__ void st(uint8_t* p, uint32_t x) {
    if constexpr (NB == 16) {
        v4u v = {x, x + 1, x + 2, x + 3};
        if (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p)); else *reinterpret_cast<v4u*>(p) = v;
    } else if constexpr (NB == 8) {
        v2u v = {x, x + 1};
        if (NT) __builtin_nontemporal_store(v, reinterpret_cast<v2u*>(p)); else *reinterpret_cast<v2u*>(p) = v;
    } else if constexpr (NB == 4) {
        if (NT) __builtin_nontemporal_store(x, reinterpret_cast<uint32_t*>(p)); else *reinterpret_cast<uint32_t*>(p) = x;
    } else if constexpr (NB == 2) {
        if (NT) __builtin_nontemporal_store((uint16_t)x, reinterpret_cast<uint16_t*>(p)); else *reinterpret_cast<uint16_t*>(p) = (uint16_t)x;
    } else {
        if (NT) __builtin_nontemporal_store((uint8_t)x, p); else *p = (uint8_t)x;
    }
}

// pure writes: grid-stride over 64*NB-byte wave pieces
template <int NB, bool NT>
__global__ __launch_bounds__(256) void write_kernel(uint8_t* out, size_t bytes) {
    const size_t n = bytes / NB;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) st<NB, NT>(out + i * NB, (uint32_t)i);
}

// read stream + writes: per 4-KiB step, K store instructions of 64*NB bytes into
// a separate contiguous output region of the wave (wbytes per step)
template <int NB, int K, bool NT, int EVERY = 1, bool SAME = false, int MODE = 0>
__global__ __launch_bounds__(64) void rw_kernel(const uint8_t* __restrict__ in, size_t bytes, uint8_t* out, uint32_t* o) {
    constexpr int S = 3, kStep = 4096;
    __shared__ __attribute__((aligned(16))) uint8_t ring[S * kStep + 10240];
    const int lane = threadIdx.x;
    const size_t nsteps = bytes / kStep;
    const size_t nw = gridDim.x, w = blockIdx.x;
    const size_t q = nsteps / nw, rem = nsteps % nw;
    const size_t sbeg = q * w + min(w, rem), send = sbeg + q + (w < rem ? 1 : 0);
    const uint32_t src_off = (uint32_t)(lane & ~3) * 16u + ((uint32_t)((lane & 3) - (lane >> 4)) & 3u) * 16u;
    const uint32_t ring0 = (uint32_t)(uintptr_t)(lds_ptr_t)&ring[0];
    size_t is = sbeg;
    uint32_t islot = 0;
    auto issue = [&]() {
        if (is >= send) return;
        const uint8_t* sp = in + is * kStep;
#pragma unroll
        for (int i = 0; i < 4; ++i) glds16_nt_s(sp, src_off + 1024u * i, ring0 + islot * kStep + 1024u * i);
        islot = islot == S - 1 ? 0 : islot + 1;
        ++is;
    };
    issue(); issue();
    uint32_t acc = 0, cslot = 0;
    constexpr size_t kW = (size_t)64 * NB * K;   // written bytes per step
    for (size_t s = sbeg; s < send; ++s) {
        // MODE 1: this step's stores go out before the next step's loads are issued
        const bool sthis = K > 0 && (EVERY == 1 || s % EVERY == 0);
        if (MODE != 1 || !sthis) issue();
        if (s + S - 1 < send) wait_vm<(4 * (S - 1) + K * (S - 1) > 63 ? 63 : 4 * (S - 1) + K * (S - 1))>();
        else wait_vm<0>();
        const uint4 v = *reinterpret_cast<const uint4*>(&ring[cslot * kStep + 64 * lane]);
        const uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
        acc += x;
        if (sthis && MODE != 3) {
            if (MODE == 2) wait_vm<0>();   // drain every load before the stores
#pragma unroll
            for (int k = 0; k < K; ++k)
                st<NB, NT>(out + (SAME ? w : s / EVERY) * kW + (size_t)k * 64 * NB + (size_t)lane * NB, x + k);
            if (MODE == 1) issue();
        }
        cslot = cslot == S - 1 ? 0 : cslot + 1;
    }
    if (MODE == 3) {   // every deferred store of the range at the end
        for (size_t s = sbeg; s < send; ++s) {
            if (EVERY == 1 || s % EVERY == 0) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    st<NB, NT>(out + (s / EVERY) * kW + (size_t)k * 64 * NB + (size_t)lane * NB, acc + k);
            }
        }
    }
    if (acc == 0x12345678u) o[0] = acc;
}

// register-staged read stream (2 steps of 4 KiB in flight per wave) + the same sparse writes
template <int NB, int K, int EVERY, int WPB>
__global__ __launch_bounds__(64 * WPB) void rw_reg_kernel(const uint8_t* __restrict__ in, size_t bytes, uint8_t* out,
                                                          uint32_t* o) {
    const int lane = threadIdx.x & 63;
    const size_t nsteps = bytes / 4096;
    const size_t nw = (size_t)gridDim.x * WPB, w = (size_t)blockIdx.x * WPB + (threadIdx.x >> 6);
    const size_t q = nsteps / nw, rem = nsteps % nw;
    const size_t sbeg = q * w + min(w, rem), send = sbeg + q + (w < rem ? 1 : 0);
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    auto ld = [&](size_t st, uint4* v) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v4 t = __builtin_nontemporal_load(reinterpret_cast<const v4*>(in + st * 4096 + 1024 * i + 16 * lane));
            v[i] = make_uint4(t.x, t.y, t.z, t.w);
        }
    };
    uint4 a[4], b[4];
    if (sbeg < send) ld(sbeg, a);
    if (sbeg + 1 < send) ld(sbeg + 1, b);
    uint32_t acc = 0;
    constexpr size_t kW = (size_t)64 * NB * K;
    for (size_t s = sbeg; s < send; ++s) {
        uint32_t x = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) x += a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
        acc += x;
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = b[i];
        if (s + 2 < send) ld(s + 2, b);
        if (K > 0 && s % EVERY == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) st<NB, true>(out + (s / EVERY) * kW + (size_t)k * 64 * NB + (size_t)lane * NB, x + k);
        }
    }
    if (acc == 0x12345678u) o[0] = acc;
}

// LDS-DMA read stream + K dword stores (256 B per instruction) every EVERY steps, policy POL
template <int K, int EVERY, int POL>
__global__ __launch_bounds__(64) void rw_pol_kernel(const uint8_t* __restrict__ in, size_t bytes, uint8_t* out, uint32_t* o) {
    constexpr int S = 3, kStep = 4096;
    __shared__ __attribute__((aligned(16))) uint8_t ring[S * kStep + 10240];
    const int lane = threadIdx.x;
    const size_t nsteps = bytes / kStep;
    const size_t nw = gridDim.x, w = blockIdx.x;
    const size_t q = nsteps / nw, rem = nsteps % nw;
    const size_t sbeg = q * w + min(w, rem), send = sbeg + q + (w < rem ? 1 : 0);
    const uint32_t src_off = (uint32_t)(lane & ~3) * 16u + ((uint32_t)((lane & 3) - (lane >> 4)) & 3u) * 16u;
    const uint32_t ring0 = (uint32_t)(uintptr_t)(lds_ptr_t)&ring[0];
    size_t is = sbeg;
    uint32_t islot = 0;
    auto issue = [&]() {
        if (is >= send) return;
        const uint8_t* sp = in + is * kStep;
#pragma unroll
        for (int i = 0; i < 4; ++i) glds16_nt_s(sp, src_off + 1024u * i, ring0 + islot * kStep + 1024u * i);
        islot = islot == S - 1 ? 0 : islot + 1;
        ++is;
    };
    issue(); issue();
    uint32_t acc = 0, cslot = 0;
    constexpr size_t kW = (size_t)256 * K;
    for (size_t s = sbeg; s < send; ++s) {
        issue();
        if (s + S - 1 < send) wait_vm<(4 * (S - 1) + K * (S - 1) > 63 ? 63 : 4 * (S - 1) + K * (S - 1))>();
        else wait_vm<0>();
        const uint4 v = *reinterpret_cast<const uint4*>(&ring[cslot * kStep + 64 * lane]);
        const uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
        acc += x;
        if (K > 0 && s % EVERY == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) st_pol<POL>(out + (s / EVERY) * kW + (size_t)k * 256 + (size_t)lane * 4, x + k);
        }
        cslot = cslot == S - 1 ? 0 : cslot + 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

int main(int argc, char** argv) {
    const size_t rbytes = 1ull << 30, wbytes = 416ull << 20;
    uint8_t *in, *out; uint32_t* o;
    CK(hipMalloc(&in, rbytes)); CK(hipMalloc(&out, 1ull << 30)); CK(hipMalloc(&o, 64));
    CK(hipMemset(in, 1, rbytes));
    auto wr = [&](const char* label, auto kern, int bpc) {
        const int grid = 256 * bpc;
        kern<<<grid, 256>>>(out, wbytes);
        CK(hipDeviceSynchronize());
        float ms = time_it([&] { kern<<<grid, 256>>>(out, wbytes); }, 20);
        printf("%-28s grid=%5d: %7.1f us %6.0f GB/s\n", label, grid, ms * 1e3, wbytes / ms / 1e6);
        return 0;
    };
    wr("write 2 B/lane nt", write_kernel<2, true>, 8);
    // read 1 GiB + write 416 MiB (26/64 of the reads): per 4-KiB step 1664 B
    auto rw = [&](const char* label, auto kern, size_t wstep) {
        int nb = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 64, 0);
        const int grid = 256 * nb;
        kern<<<grid, 64>>>(in, rbytes, out, o);
        CK(hipDeviceSynchronize());
        float ms = time_it([&] { kern<<<grid, 64>>>(in, rbytes, out, o); }, 20);
        const double wb = (double)(rbytes / 4096) * wstep;
        printf("%-28s blk/CU=%2d: %7.1f us %6.0f GB/s (r %0.0f MB + w %0.0f MB)\n", label, nb, ms * 1e3,
               (rbytes + wb) / ms / 1e6, rbytes / 1e6, wb / 1e6);
        return 0;
    };
    rw("read only", rw_kernel<16, 0, true>, 0);
    // the MTU shape: 16 narrow stores (2 B/lane) once per 24 steps (64 frames of 1.5 KB)
    rw("r + 16x 128B nt every 24", rw_kernel<2, 16, true, 24>, 2048 / 24);
    rw("r + 16x 128B nt every 24 (wait all)", rw_kernel<2, 16, true, 24>, 2048 / 24);
    rw("r + 16x 128B plain every 24", rw_kernel<2, 16, false, 24>, 2048 / 24);
    rw("r + 1x 128B nt every 24", rw_kernel<2, 1, true, 24>, 128 / 24);
    rw("r + 2x 1KiB nt every 24", rw_kernel<16, 2, true, 24>, 2048 / 24);
    rw("r + 2x 1KiB nt every 24, same addr", rw_kernel<16, 2, true, 24, true>, 2048 / 24);
    auto rwr = [&](const char* label, auto kern, int wpb, size_t wstep) {
        int nb = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 64 * wpb, 0);
        const int grid = 256 * nb;
        kern<<<grid, 64 * wpb>>>(in, rbytes, out, o);
        CK(hipDeviceSynchronize());
        float ms = time_it([&] { kern<<<grid, 64 * wpb>>>(in, rbytes, out, o); }, 20);
        const double wb = (double)(rbytes / 4096) * wstep;
        printf("%-40s waves/CU=%2d: %7.1f us %6.0f GB/s (w %0.0f MB)\n", label, nb * wpb, ms * 1e3,
               (rbytes + wb) / ms / 1e6, wb / 1e6);
        return 0;
    };
    if (argc > 1 && argv[1][0] == 'r') {   // the 64-B verify-only record (R = 6) against the full one (R = 26)
        for (int k = 0; k < 3; ++k) {
            rw("read only", rw_kernel<2, 0, true, 1>, 0);
            rw("r + 3x 128B nt every step (R=6)", rw_kernel<2, 3, true, 1, false, 0>, 384);
            rw("r + 13x 128B nt every step (R=26)", rw_kernel<2, 13, true, 1, false, 0>, 1664);
            rwr("reg read only", rw_reg_kernel<2, 0, 1, 4>, 4, 0);
            rwr("reg r + 3x 128B nt every step (R=6)", rw_reg_kernel<2, 3, 1, 4>, 4, 384);
            rwr("reg r + 13x 128B nt every step (R=26)", rw_reg_kernel<2, 13, 1, 4>, 4, 1664);
        }
        return 0;
    }
    if (argc > 1) {   // dense writes (the 64-B workload's 26 B/frame) in bursts of M steps
        rw("read only", rw_kernel<2, 0, true, 1>, 0);
        rw("r + 13x 128B nt every step", rw_kernel<2, 13, true, 1, false, 0>, 1664);
        rw("r + 13x 128B nt every step, at end", rw_kernel<2, 13, true, 1, false, 3>, 1664);
        rw("r + 104x 128B nt every 8", rw_kernel<2, 104, true, 8, false, 0>, 1664);
        rw("r + 13x 1KiB nt every 8", rw_kernel<16, 13, true, 8, false, 0>, 1664);
        rw("r + 13x 1KiB plain every 8", rw_kernel<16, 13, false, 8, false, 0>, 1664);
        rw("r + 52x 1KiB nt every 32", rw_kernel<16, 52, true, 32, false, 0>, 1664);
        rw("r + 13x 1KiB nt every 8, drain first", rw_kernel<16, 13, true, 8, false, 2>, 1664);
        rw("r + 13x 1KiB nt every 8, st before ld", rw_kernel<16, 13, true, 8, false, 1>, 1664);
        rw("r + 13x 128B nt every step", rw_kernel<2, 13, true, 1, false, 0>, 1664);
        return 0;
    }
    rw("pol none  8x256B every 24", rw_pol_kernel<8, 24, 0>, 2048 / 24);
    rw("pol nt    8x256B every 24", rw_pol_kernel<8, 24, 1>, 2048 / 24);
    rw("pol sc0sc1 8x256B every 24", rw_pol_kernel<8, 24, 2>, 2048 / 24);
    rw("pol sc0sc1nt 8x256B every 24", rw_pol_kernel<8, 24, 3>, 2048 / 24);
    rw("pol sc1   8x256B every 24", rw_pol_kernel<8, 24, 4>, 2048 / 24);
    rw("pol sc0   8x256B every 24", rw_pol_kernel<8, 24, 5>, 2048 / 24);
    rw("pol none  7x256B every step", rw_pol_kernel<7, 1, 0>, 1792);
    rw("pol nt    7x256B every step", rw_pol_kernel<7, 1, 1>, 1792);
    rw("pol sc0sc1 7x256B every step", rw_pol_kernel<7, 1, 2>, 1792);
    rw("pol sc0sc1nt 7x256B every step", rw_pol_kernel<7, 1, 3>, 1792);
    rwr("reg read only", rw_reg_kernel<2, 0, 24, 4>, 4, 0);
    rwr("reg r + 16x 128B nt every 24", rw_reg_kernel<2, 16, 24, 4>, 4, 2048 / 24);
    rwr("reg r + 2x 1KiB nt every 24", rw_reg_kernel<16, 2, 24, 4>, 4, 2048 / 24);
    rw("r + 16x 128B nt every 24, at end", rw_kernel<2, 16, true, 24, false, 3>, 2048 / 24);
    rw("r + 2x 1KiB nt every 24, at end", rw_kernel<16, 2, true, 24, false, 3>, 2048 / 24);
    rw("r + 13x 128B nt every step, at end", rw_kernel<2, 13, true, 1, false, 3>, 1664);
    rw("r + 13x 128B nt every step", rw_kernel<2, 13, true, 1, false, 0>, 1664);
    rw("r + 8x 1KiB nt every 96", rw_kernel<16, 8, true, 96>, 8192 / 96);
    rw("r + 32x 1KiB nt every 384", rw_kernel<16, 32, true, 384>, 32768 / 384);
    rw("r + 8x 1KiB plain every 96", rw_kernel<16, 8, false, 96>, 8192 / 96);
    rw("r + 2x 1KiB nt every 24, st before ld", rw_kernel<16, 2, true, 24, false, 1>, 2048 / 24);
    rw("r + 2x 1KiB nt every 24, drain first", rw_kernel<16, 2, true, 24, false, 2>, 2048 / 24);
    rw("r + 16x 128B nt every 24, drain first", rw_kernel<2, 16, true, 24, false, 2>, 2048 / 24);
    rw("r + 2x 1KiB plain every 24, same addr", rw_kernel<16, 2, false, 24, true>, 2048 / 24);
    rw("r + 16x 128B plain every 24, same", rw_kernel<2, 16, false, 24, true>, 2048 / 24);
    rw("r + 4x 512B nt every 24", rw_kernel<8, 4, true, 24>, 2048 / 24);
    rw("r + 8x 256B nt every 24", rw_kernel<4, 8, true, 24>, 2048 / 24);
    rw("r + 4x 128B nt every 24", rw_kernel<2, 4, true, 24>, 512 / 24);
    rw("r + 32x 64B nt every 24", rw_kernel<1, 32, true, 24>, 2048 / 24);
    return 0;
}
