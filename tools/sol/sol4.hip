// sol4.hip — the stream kernel's load skeleton on MI355X without the receive work:
// one-wave blocks, an S-step LDS ring of 4-KiB steps filled by global_load_lds
// (saddr form, per-lane source offsets permuted inside 64-B pieces), per-wave
// contiguous ranges, LDS padded to the stream kernel's footprint; the consumer
// reads its 64-B piece and sums it, plus W dependent VALU ops of fake work per step.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/sol/sol4 tools/sol/sol4.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
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

template <int S, int PAD, int W, int WPB, int STEPK>
__global__ __launch_bounds__(64 * WPB) void stream_kernel(const uint8_t* __restrict__ in, size_t bytes, uint32_t* o) {
    constexpr int kStep = 4096 * STEPK;
    __shared__ __attribute__((aligned(16))) uint8_t ring[WPB][S * kStep + PAD];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const size_t nsteps = bytes / kStep;
    const size_t nw = (size_t)gridDim.x * WPB, w = (size_t)blockIdx.x * WPB + wv;
    const size_t q = nsteps / nw, rem = nsteps % nw;
    const size_t sbeg = q * w + min(w, rem), send = sbeg + q + (w < rem ? 1 : 0);
    const uint32_t src_off = (uint32_t)(lane & ~3) * 16u + ((uint32_t)((lane & 3) - (lane >> 4)) & 3u) * 16u;
    const uint32_t ring0 = (uint32_t)(uintptr_t)(lds_ptr_t)&ring[wv][0];
    size_t is = sbeg;
    uint32_t islot = 0;
    auto issue = [&]() {
        if (is >= send) return;
        const uint8_t* sp = in + is * kStep;
#pragma unroll
        for (int i = 0; i < 4 * STEPK; ++i) glds16_nt_s(sp, src_off + 1024u * i, ring0 + islot * kStep + 1024u * i);
        islot = islot == S - 1 ? 0 : islot + 1;
        ++is;
    };
#pragma unroll
    for (int s = 0; s < S - 1; ++s) issue();
    uint32_t acc = 0, cslot = 0;
    for (size_t st = sbeg; st < send; ++st) {
        issue();
        if (st + S - 1 < send) wait_vm<4 * STEPK * (S - 1)>();
        else wait_vm<0>();
        uint32_t t = 0;
#pragma unroll
        for (int j = 0; j < STEPK; ++j) {
            const uint8_t* pc = &ring[wv][cslot * kStep + j * 4096 + 64 * lane];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const uint4 v = *reinterpret_cast<const uint4*>(pc + 16 * ((c + (lane >> 2)) & 3));
                t = sad(v.w, sad(v.z, sad(v.y, sad(v.x, t))));
            }
        }
        // fake per-step work: W dependent VALU ops
#pragma unroll
        for (int i = 0; i < W; ++i) t = t * 3u + (uint32_t)i;
        acc += t;
        cslot = cslot == S - 1 ? 0 : cslot + 1;
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
    const size_t bytes = 1536ull << 20;
    uint8_t* in; uint32_t* o;
    CK(hipMalloc(&in, bytes)); CK(hipMalloc(&o, 64));
    CK(hipMemset(in, 1, bytes));
    auto run = [&](const char* label, auto kern, int wpb) {
        int nb = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 64 * wpb, 0);
        hipFuncAttributes fa;
        (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(kern));
        printf("  occ rc=%d lds=%zu regs=%d\n", (int)e, fa.sharedSizeBytes, fa.numRegs);
        const int grid = 256 * nb;
        kern<<<grid, 64 * wpb>>>(in, bytes, o);
        e = hipDeviceSynchronize();
        if (e != hipSuccess) { printf("  launch: %s\n", hipGetErrorString(e)); exit(1); }
        float ms = time_it([&] { kern<<<grid, 64 * wpb>>>(in, bytes, o); }, 20);
        printf("%-40s blk/CU=%2d waves/CU=%2d: %7.1f us %6.0f GB/s\n", label, nb, nb * wpb, ms * 1e3, bytes / ms / 1e6);
    };
    // the stream kernel's footprint: S x 4 KiB ring + ~10 KiB of slots and records
    run("S3 pad10K W0", stream_kernel<3, 10240, 0, 1, 1>, 1);
    run("S3 pad10K W100", stream_kernel<3, 10240, 100, 1, 1>, 1);
    run("S3 pad10K W200", stream_kernel<3, 10240, 200, 1, 1>, 1);
    run("S4 pad10K W0", stream_kernel<4, 10240, 0, 1, 1>, 1);
    run("S4 pad10K W100", stream_kernel<4, 10240, 100, 1, 1>, 1);
    run("S3 pad0 W0", stream_kernel<3, 0, 0, 1, 1>, 1);
    run("S3 pad0 W100", stream_kernel<3, 0, 100, 1, 1>, 1);
    run("S4 pad0 W100", stream_kernel<4, 0, 100, 1, 1>, 1);
    run("S2 pad0 W100", stream_kernel<2, 0, 100, 1, 1>, 1);
    run("S3 pad10K W100 2-wave blocks", stream_kernel<3, 10240, 100, 2, 1>, 2);
    run("S2 8KiB-steps pad10K W100", stream_kernel<2, 10240, 100, 1, 2>, 1);
    run("S3 8KiB-steps pad10K W100", stream_kernel<3, 10240, 100, 1, 2>, 1);
    return 0;
}
