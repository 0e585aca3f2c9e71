// sol6.hip — speed of light for a run-contiguous IMIX kernel on MI355X.
// The bench's IMIX shape (2^22 frames of 64/576/1500 B at 7:4:1, packed back to
// back, compact u32/u16 descriptors, 26 B of result columns per frame) read as
// ONE contiguous byte range per run of 64 frames: each wave instruction loads
// 1 KiB (lane l: 16 B at 16 l), U instructions in flight per lane, per-lane sums.
//   read      runs streamed, one 4-B result per frame (the sums must be used)
//   read+cols runs streamed + the 12 record columns (26 B/frame, nt stores)
//   +scan     each 1-KiB chunk also does the per-chunk prefix bookkeeping a real
//             kernel needs (wave scan of the granule sums + 2 ds_bpermute reads)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/sol/sol6 tools/sol/sol6.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

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

template <int U, bool COLS, bool SCAN>
__global__ __launch_bounds__(256, 4) void run_stream(const uint8_t* data, const uint32_t* offs, const uint16_t* lens,
                                                     uint64_t n, Cols C, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const uint64_t nruns = (n + 63) / 64;
    const uint64_t wstride = (uint64_t)gridDim.x * 4;
    for (uint64_t run = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64; run < nruns; run += wstride) {
        const uint64_t f = run * 64 + lane;
        const bool in = f < n;
        const uint32_t off = in ? offs[f] : 0u, len = in ? lens[f] : 0u;
        const uint64_t last = min(n, run * 64 + 64) - 1 - run * 64;
        const uint32_t lo = __shfl((int)off, 0) & ~15u;
        const uint32_t hi = (uint32_t)__shfl((int)(off + len), (int)last);
        const uint32_t ng = (hi - lo + 15) >> 4;
        // frame lane: two granule indices whose prefix it needs (tail start / end)
        const uint32_t gs = ((off - lo) >> 4) + 7, ge = ((off + len - lo) >> 4);
        uint32_t acc = 0, pa = 0, pb = 0, base = 0;
        for (uint32_t g0 = 0; g0 < ng; g0 += 64 * U) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t g = g0 + 64 * u + lane;
                v[u] = g < ng ? *reinterpret_cast<const uint4*>(data + lo + 16u * g) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t s = sad(v[u].w, sad(v[u].z, sad(v[u].y, sad(v[u].x, 0u))));
                if (SCAN) {
                    const uint32_t p = wave_incl_scan(s);
                    const uint32_t cb = g0 + 64 * u;
                    const uint32_t ta = __builtin_amdgcn_ds_bpermute((int)((gs - cb) & 63) * 4, (int)p);
                    const uint32_t tb = __builtin_amdgcn_ds_bpermute((int)((ge - cb) & 63) * 4, (int)p);
                    if (gs - cb < 64u) pa = base + ta;
                    if (ge - cb < 64u) pb = base + tb;
                    base += (uint32_t)__builtin_amdgcn_readlane((int)p, 63);
                } else {
                    acc += s;
                }
            }
        }
        const uint32_t r = SCAN ? pb - pa : acc;
        if (!in) continue;
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
}

template <int U, bool COLS, bool SCAN>
static float timeit(const uint8_t* d, const uint32_t* o, const uint16_t* l, uint64_t n, Cols c, uint32_t* out,
                    int blocks, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((run_stream<U, COLS, SCAN>), dim3(blocks), dim3(256), 0, 0, d, o, l, n, c, out);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((run_stream<U, COLS, SCAN>), dim3(blocks), dim3(256), 0, 0, d, o, l, n, c, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

// persistent variant: each wave owns a contiguous block of runs and streams its
// whole byte range with U chunks always in flight (loads are never drained at
// a run boundary); a run's 12 column stores go out when the stream passes the
// run's last granule
template <int U, bool COLS>
__global__ __launch_bounds__(256, 4) void run_persist(const uint8_t* data, const uint32_t* offs, const uint16_t* lens,
                                                      uint64_t n, Cols C, uint32_t* out) {
    const int lane = threadIdx.x & 63;
    const uint64_t nruns = (n + 63) / 64;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + threadIdx.x / 64;
    const uint64_t r0 = nruns * w / nw, r1 = nruns * (w + 1) / nw;
    if (r0 >= r1) return;
    const uint64_t fa = r0 * 64, fb = min(n, r1 * 64);
    const uint32_t lo = offs[fa] & ~15u;
    const uint32_t hi = offs[fb - 1] + lens[fb - 1];
    const uint32_t ng = (hi - lo + 15) >> 4;
    uint64_t run = r0;
    // granule (relative to lo) at which the current run ends
    auto run_end = [&](uint64_t r) -> uint32_t {
        const uint64_t last = min(n, r * 64 + 64) - 1;
        return (offs[last] + lens[last] - lo + 15) >> 4;
    };
    uint32_t rend = run_end(run);
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t g = 64 * u + lane;
        v[u] = g < ng ? *reinterpret_cast<const uint4*>(data + lo + 16u * g) : make_uint4(0, 0, 0, 0);
    }
    uint32_t acc = 0;
    for (uint32_t c0 = 0; c0 < ng; c0 += 64 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc = sad(v[u].w, sad(v[u].z, sad(v[u].y, sad(v[u].x, acc))));
            const uint32_t gn = c0 + 64 * (u + U) + lane;
            v[u] = gn < ng ? *reinterpret_cast<const uint4*>(data + lo + 16u * gn) : make_uint4(0, 0, 0, 0);
            const uint32_t done_g = c0 + 64 * (u + 1);
            while (run < r1 && rend <= done_g) {          // wave-uniform
                const uint64_t f = run * 64 + lane;
                if (f < n) {
                    const uint32_t r = acc + (uint32_t)f;
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
    }
}

template <int U, bool COLS>
static float timeit_p(const uint8_t* d, const uint32_t* o, const uint16_t* l, uint64_t n, Cols c, uint32_t* out,
                      int blocks, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((run_persist<U, COLS>), dim3(blocks), dim3(256), 0, 0, d, o, l, n, c, out);
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((run_persist<U, COLS>), dim3(blocks), dim3(256), 0, 0, d, o, l, n, c, out);
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
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
    CK(hipMalloc(&d, bytes + 64));
    CK(hipMemset(d, 0x5A, bytes + 64));
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
        for (int bpc : {4, 8}) {
            const int blocks = prop.multiProcessorCount * bpc;
            float t;
#define RUN(U, COLS, SCAN, ALG)                                                                                   \
    t = timeit<U, COLS, SCAN>(d, o, l, n, c, out, blocks, 20);                                                    \
    printf("blocks/CU %d U=%2d %-9s %-5s %8.1f us  %6.0f GB/s (%.1f%% of 8 TB/s)\n", bpc, U, COLS ? "read+cols" : "read", \
           SCAN ? "+scan" : "", t * 1e3, (ALG) / (t * 1e-3) / 1e9, (ALG) / (t * 1e-3) / 1e9 / 80.0);
            RUN(4, false, false, alg_read)
            RUN(8, false, false, alg_read)
            RUN(8, true, false, alg_cols)
            RUN(4, true, true, alg_cols)
            RUN(8, true, true, alg_cols)
#define RUNP(U, COLS, ALG)                                                                                        \
    t = timeit_p<U, COLS>(d, o, l, n, c, out, blocks, 20);                                                        \
    printf("blocks/CU %d U=%2d %-9s persist %8.1f us  %6.0f GB/s (%.1f%% of 8 TB/s)\n", bpc, U,                  \
           COLS ? "read+cols" : "read", t * 1e3, (ALG) / (t * 1e-3) / 1e9, (ALG) / (t * 1e-3) / 1e9 / 80.0);
            RUNP(4, false, alg_read)
            RUNP(8, false, alg_read)
            RUNP(4, true, alg_cols)
            RUNP(8, true, alg_cols)
            RUNP(12, true, alg_cols)
        }
    }
    return 0;
}
