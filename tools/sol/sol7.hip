// sol7.hip — the IMIX shape of sol6 read through an LDS-DMA ring instead of
// register loads: each wave (one-wave blocks) owns a contiguous block of runs
// and streams its byte range in 4-KiB steps (4 x global_load_lds_dwordx4 of
// 1 KiB), S-step ring, S-1 steps in flight; per step each lane reads its 64
// stream bytes back (4 ds_read_b128), sums them, and (SCAN) does the prefix
// bookkeeping a real kernel needs (lane-local prefix of its 4 granules, one wave
// scan, the 64 prefixes written to an LDS table); a run's 12 record columns
// (26 B/frame, nt stores) go out when the stream passes the run's last byte.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/sol/sol7 tools/sol/sol7.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ void glds16_nt_s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_addr) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ uint32_t sad(uint32_t d, uint32_t acc) { return __builtin_amdgcn_sad_u16(d, 0u, acc); }
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return v;
}

struct Cols {
    uint16_t *st, *ipc, *l4c, *et, *l4o, *l4l, *sp, *dp;
    uint8_t *proto, *ttl;
    uint32_t *s4, *d4;
};
template <class T>
__device__ __forceinline__ void put(T* c, uint64_t i, T v) { __builtin_nontemporal_store(v, c + i); }

constexpr int kStep = 4096;

template <int S, bool COLS, bool SCAN, int PV = 0, bool WIN = false>
__global__ __launch_bounds__(64) void glds_persist(const uint8_t* data, const uint32_t* offs, const uint16_t* lens,
                                                   uint64_t n, Cols C, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[S * kStep];
    __shared__ __attribute__((aligned(16))) uint32_t ptab[256];
    // WIN: 64 padded 132-B window slots (the mixed kernel's), filled from the ring
    __shared__ __attribute__((aligned(16))) uint32_t slots[WIN ? 64 * 33 : 1];
    const int lane = threadIdx.x;
    const uint64_t nruns = (n + 63) / 64;
    const uint64_t nw = gridDim.x, w = blockIdx.x;
    const uint64_t r0 = nruns * w / nw, r1 = nruns * (w + 1) / nw;
    if (r0 >= r1) return;
    const uint64_t fa = r0 * 64, fb = min(n, r1 * 64);
    const uint32_t lo = offs[fa] & ~15u;
    const uint32_t hi = offs[fb - 1] + lens[fb - 1];
    const uint32_t nsteps = (hi - lo + kStep - 1) / kStep;
    // lane l reads stream bytes [64 l, 64 l + 64) of a step back with four
    // conflict-free ds_read_b128: source addresses permuted inside each 64-B piece
    const uint32_t src_off = (uint32_t)(lane & ~3) * 16u + ((uint32_t)((lane & 3) - (lane >> 4)) & 3u) * 16u;
    const uint32_t ring0 = (uint32_t)(uintptr_t)(lds_ptr_t)&ring[0];
    uint32_t is = 0, islot = 0;
    auto issue = [&]() {
        if (is >= nsteps) return;
        const uint8_t* sp = data + lo + (uint64_t)is * kStep;
#pragma unroll
        for (int i = 0; i < 4; ++i) glds16_nt_s(sp, src_off + 1024u * i, ring0 + islot * kStep + 1024u * i);
        islot = islot == S - 1 ? 0 : islot + 1;
        ++is;
    };
    uint64_t run = r0;
    auto run_end = [&](uint64_t r) -> uint32_t {
        const uint64_t last = min(n, r * 64 + 64) - 1;
        return offs[last] + lens[last] - lo;
    };
    uint32_t rend = run_end(run);
#pragma unroll
    for (int k = 0; k < S - 1; ++k) issue();
    uint32_t acc = 0, cslot = 0, base = 0;
    for (uint32_t s = 0; s < nsteps; ++s) {
        issue();
        if (s + S - 1 < nsteps) wait_vm<4 * (S - 1)>();
        else wait_vm<0>();
        const uint8_t* slot = ring + cslot * kStep;
        uint32_t g[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            // piece i of the lane's 64 B, rotated so that 16 lanes of one LDS pass hit distinct banks
            const uint4 v = *reinterpret_cast<const uint4*>(slot + 64 * lane + 16 * ((i + (lane >> 2)) & 3));
            g[i] = sad(v.w, sad(v.z, sad(v.y, sad(v.x, 0u))));
        }
        if (SCAN) {
            const uint32_t t01 = g[0] + g[1], t012 = t01 + g[2], tot = t012 + g[3];
            const uint32_t ex = wave_incl_scan(tot) - tot + base;
            *reinterpret_cast<uint4*>(&ptab[4 * lane]) = make_uint4(ex, ex + g[0], ex + t01, ex + t012);
            base += (uint32_t)__builtin_amdgcn_readlane((int)(ex + tot - base), 63);
            acc += ptab[(lane * 37) & 255];
        } else {
            acc += g[0] + g[1] + g[2] + g[3];
        }
        if (WIN) {
            // every lane copies 8 ring granules into a slot (an upper bound on the
            // per-step window capture: ~10 frames start per 4 KiB of IMIX)
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint4 v = *reinterpret_cast<const uint4*>(slot + 16 * ((lane * 7 + c * 13) & 255));
                uint32_t* dst = slots + ((lane * 5 + c) & 63) * 33 + 4 * c;
                dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
            }
        }
        cslot = cslot == S - 1 ? 0 : cslot + 1;
        const uint32_t done_b = (s + 1) * kStep;
        while (run < r1 && rend <= done_b) {   // wave-uniform
            const uint64_t f = run * 64 + lane;
            uint32_t e0 = acc, e1 = acc ^ 1u, e2 = acc ^ 2u, e3 = acc ^ 3u;
            if (PV) {
                // the per-run parse emulated: PV VALU ops in four independent chains
                // reading the slots (WIN) so they cannot be hoisted
                const uint32_t sv = WIN ? slots[lane * 33] : 0u;
#pragma unroll 1
                for (int k = 0; k < PV / 4; ++k) {
                    e0 = sad(e0 ^ sv, e0); e1 = sad(e1 + sv, e1); e2 = sad(e2 ^ (uint32_t)k, e2); e3 = sad(e3 + (uint32_t)k, e3);
                }
            }
            if (f < n) {
                const uint32_t r = acc + (uint32_t)f + (e0 ^ e1 ^ e2 ^ e3);
                if (COLS) {
                    put<uint16_t>(C.st, f, (uint16_t)r);
                    put<uint16_t>(C.ipc, f, (uint16_t)(r >> 1));
                    put<uint16_t>(C.l4c, f, (uint16_t)(r >> 2));
                    put<uint16_t>(C.et, f, (uint16_t)(r >> 3));
                    put<uint8_t>(C.proto, f, (uint8_t)r);
                    put<uint8_t>(C.ttl, f, (uint8_t)(r >> 5));
                    put<uint16_t>(C.l4o, f, (uint16_t)(r >> 4));
                    put<uint16_t>(C.l4l, f, (uint16_t)(r >> 6));
                    put<uint16_t>(C.sp, f, (uint16_t)(r >> 7));
                    put<uint16_t>(C.dp, f, (uint16_t)(r >> 8));
                    put<uint32_t>(C.s4, f, r ^ 1);
                    put<uint32_t>(C.d4, f, r ^ 2);
                } else {
                    put<uint32_t>(out, f, r);
                }
            }
            ++run;
            if (run < r1) rend = run_end(run);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int S, bool COLS, bool SCAN, int PV = 0, bool WIN = false>
static float timeit(const uint8_t* d, const uint32_t* o, const uint16_t* l, uint64_t n, Cols c, uint32_t* out,
                    int blocks, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((glds_persist<S, COLS, SCAN, PV, WIN>), dim3(blocks), dim3(64), 0, 0, d, o, l, n, c, out);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((glds_persist<S, COLS, SCAN, PV, WIN>), dim3(blocks), dim3(64), 0, 0, d, o, l, n, c, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main(int argc, char** argv) {
    (void)argv;
    const uint64_t n = 1ull << 22;
    std::mt19937_64 rng(7);
    std::vector<uint32_t> offs(n);
    std::vector<uint16_t> lens(n);
    uint64_t pos = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t r = rng() % 12;
        lens[i] = r < 7 ? 64 : (r < 11 ? 576 : 1500);
        offs[i] = (uint32_t)pos;
        pos += lens[i];
    }
    const uint64_t bytes = pos;
    uint8_t* d;
    uint32_t *o, *out;
    uint16_t* l;
    CK(hipMalloc(&d, bytes + 8192));
    CK(hipMemset(d, 0x5A, bytes + 8192));
    CK(hipMalloc(&o, 4 * n));
    CK(hipMalloc(&l, 2 * n));
    CK(hipMalloc(&out, 4 * n));
    CK(hipMemcpy(o, offs.data(), 4 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(l, lens.data(), 2 * n, hipMemcpyHostToDevice));
    Cols c;
    uint8_t* cb;
    CK(hipMalloc(&cb, 26 * n + 4096));
    uint8_t* p = cb;
    auto take = [&](size_t b) { uint8_t* r = p; p += (b * n + 255) / 256 * 256; return r; };
    c.st = (uint16_t*)take(2); c.ipc = (uint16_t*)take(2); c.l4c = (uint16_t*)take(2); c.et = (uint16_t*)take(2);
    c.proto = take(1); c.ttl = take(1); c.l4o = (uint16_t*)take(2); c.l4l = (uint16_t*)take(2);
    c.sp = (uint16_t*)take(2); c.dp = (uint16_t*)take(2); c.s4 = (uint32_t*)take(4); c.d4 = (uint32_t*)take(4);
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const double alg_cols = (double)bytes + 32.0 * n, alg_read = (double)bytes + 10.0 * n;
    printf("IMIX-shaped batch: %llu frames, %.3f GB\n", (unsigned long long)n, bytes / 1e9);
    for (int round = 0; round < 3; ++round) {
        for (int wpc : (argc > 1 ? std::vector<int>{7, 8} : std::vector<int>{8, 12, 16})) {
            const int blocks = prop.multiProcessorCount * wpc;
            float t;
#define RUN(S, COLS, SCAN, ALG)                                                                                  \
    t = timeit<S, COLS, SCAN>(d, o, l, n, c, out, blocks, 20);                                                   \
    printf("waves/CU %2d S=%d %-9s %-5s %8.1f us  %6.0f GB/s (%.1f%% of 8 TB/s)\n", wpc, S, COLS ? "read+cols" : "read", \
           SCAN ? "+scan" : "", t * 1e3, (ALG) / (t * 1e-3) / 1e9, (ALG) / (t * 1e-3) / 1e9 / 80.0);
            if (argc > 1) {   // the per-run parse and window capture emulated (wpc 7/8: LDS allows 7)
#define RUNP(PV, WIN)                                                                                          \
    t = timeit<3, true, true, PV, WIN>(d, o, l, n, c, out, blocks, 20);                                        \
    printf("waves/CU %2d cols+scan PV=%4d WIN=%d %8.1f us  %6.0f GB/s (%.1f%% of 8 TB/s)\n", wpc, PV, (int)WIN, t * 1e3, \
           alg_cols / (t * 1e-3) / 1e9, alg_cols / (t * 1e-3) / 1e9 / 80.0);
                RUNP(0, false)
                RUNP(0, true)
                RUNP(400, true)
                RUNP(800, true)
                RUNP(1600, true)
                continue;
            }
            RUN(3, false, false, alg_read)
            RUN(3, true, false, alg_cols)
            RUN(3, true, true, alg_cols)
            if (wpc <= 8) {
                RUN(4, true, true, alg_cols)
            }
        }
    }
    return 0;
}
