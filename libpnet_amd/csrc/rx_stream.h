// rx_stream.h — rx_stream_kernel, the opt-in LDS-DMA stream kernel for fixed strides >= 1 KiB
// Part of the receive-path kernels; included once, by rx_kernel.hip (one
// translation unit, so every kernel still sees the shared device helpers inline).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pnetgpu.h"
#include "rx_internal.h"
#include "rx_common.h"

namespace pnetgpu {
namespace {

// ============================================================================
// rx_stream_kernel: fixed stride >= 1 KiB (MTU and jumbo frames), LDS-DMA stream.
// ============================================================================
// A wave owns a run of 64 frames and streams the run's whole byte span
// [base of frame 0, end of frame 63) in 4-KiB steps straight into an S-step
// LDS ring with global_load_lds_dwordx4: four fully contiguous 1-KiB wave
// instructions per step, no VGPR destination, S-1 steps in flight, crossing
// from one run into the next. The source addresses are permuted inside each
// 64-B piece so that lane l finds stream bytes [64 l, 64 l + 64) of the step
// at conflict-free LDS addresses (four ds_read_b128).
// Per step, lane l sums its 64-B piece (16 v_sad_u16, keeping the prefix after
// each 16-B granule) and one wave scan turns the piece sums into P(x), the
// weighted byte sum of the run's stream before any granule-aligned position x.
// A frame's tail (slot bytes [128, end), rx_kernel's speculative tail) is then
// P(TE) - P(TS) plus its last granule's bytes, with TS = slot base + 128 and
// TE = (end - 1) rounded down to 16: both granule-aligned, at most one of them per
// 64-B piece, recorded by the lane whose piece holds it. That lane also copies
// window granules (slot bytes [0, 128)) and the end granule into LDS. After the
// run's last step the parse, window sums and column stores are rx_kernel's.
// Why: a wave instruction reading 1 KiB contiguous streams at ~6.8 TB/s, the
// 8 x 128-B pieces of the group-per-frame shape at ~5.9 TB/s (tools/sol3.hip,
// same box); LDS-DMA keeps loads in flight without VGPRs, and one scan per
// 4 KiB keeps the instruction count per byte below the register kernel's.
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// global_load_lds_dwordx4, non-temporal: lane l's 16 B land at lds + 16 l.
// Issued from inline asm so hipcc neither tracks it (its vmcnt bookkeeping
// would put a vmcnt(0) before every LDS read of the ring) nor reorders memory
// operations across it; completion is counted by hand (wait_steps). M0 is
// written and restored inside the statement.
__device__ __forceinline__ void glds16_nt(const void* gsrc, uint32_t lds_addr) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
}
// The same with a wave-uniform 64-bit base (SGPRs) and a per-lane 32-bit offset:
// no per-lane address arithmetic at all.
__device__ __forceinline__ void glds16_nt_s(const void* sbase, uint32_t voff, uint32_t lds_addr) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds_addr)
                 : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(4 * min(n, N)) for a wave-uniform n (the immediate is static).
// vmcnt retires in issue order, so VMEM ops issued after the step (column
// stores) only make this wait longer, never too short.
template <int N>
__device__ __forceinline__ void wait_steps(int n) {
    if constexpr (N == 0) {
        wait_vm<0>();
    } else {
        if (n >= N) wait_vm<4 * N>();
        else wait_steps<N - 1>(n);
    }
}
// s_waitcnt vmcnt(n) for a wave-uniform n in [LO, HI]: a binary search of
// static immediates.
template <int LO, int HI>
__device__ __forceinline__ void wait_vm_dyn(int n) {
    if constexpr (LO == HI) {
        wait_vm<LO>();
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (n <= MID) wait_vm_dyn<LO, MID>(n);
        else wait_vm_dyn<MID + 1, HI>(n);
    }
}
// Store instructions store_columns issues for a column set (one per non-null column).
__device__ __forceinline__ int column_stores(const pnetgpu_rx_columns& C) {
    return (C.status != nullptr) + (C.ip_csum != nullptr) + (C.l4_csum != nullptr) + (C.ethertype != nullptr) +
           (C.ip_proto != nullptr) + (C.ttl != nullptr) + (C.l4_offset != nullptr) + (C.l4_length != nullptr) +
           (C.src_port != nullptr) + (C.dst_port != nullptr) + (C.src_ipv4 != nullptr) + (C.dst_ipv4 != nullptr) +
           (C.vlan_tci != nullptr) + (C.l3_offset != nullptr) + (C.src_ipv6 != nullptr) + (C.dst_ipv6 != nullptr);
}

constexpr int kStreamStep = 4096;   // bytes per step: 64 lanes x 64 B

template <int S>
struct StreamLds {
    uint8_t ring[S][kStreamStep];
    uint8_t win[kWave * WaveLds<8>::kSlot];
    uint4 endg[kWave];        // each frame's last granule (slot bytes [TE, TE + 16))
    uint32_t pts[kWave];      // P(TS) per frame
    uint32_t pte[kWave];      // P(TE) per frame
};

// Byte span of the run of frames [f0, f0 + nf): aligned start, step count, first frame offset.
struct RunSpan {
    uint64_t a0, off0;
    uint32_t nsteps;
};
__device__ __forceinline__ RunSpan run_span(const RxArgs& a, uint64_t f0, uint32_t nf) {
    RunSpan s;
    s.off0 = a.first + a.delta + f0 * a.stride;
    s.a0 = s.off0 & ~15ull;
    const uint64_t a1 = s.off0 + (uint64_t)(nf - 1) * a.stride + a.frame_len;
    s.nsteps = (uint32_t)((a1 - s.a0 + kStreamStep - 1) / kStreamStep);
    return s;
}

// One wave per block (the LDS ring and slots bound residency, not registers).
// Wave w owns the contiguous frames [n w / W, n (w + 1) / W) of the batch (W
// waves), processed as runs of up to 64: balanced to one frame, which a
// grid-stride over whole runs is not (2^17 jumbo frames = 2048 runs on ~1800
// resident waves would leave most of them one run short of the slowest).
template <int S, bool EXT>
__global__ __launch_bounds__(kWave) void rx_stream_kernel(RxArgs a) {
    constexpr int kSlot = WaveLds<8>::kSlot;
    constexpr int kWin = 128;
    __shared__ StreamLds<S> L;
    const int lane = threadIdx.x;
    uint8_t* slot = L.win + lane * kSlot;
    Counters K;
    const uint32_t stride = a.stride, flen = a.frame_len;
    const float inv_stride = 1.0f / (float)stride;
    const uint64_t lim16 = ((a.limit + 15) & ~15ull) - 16;   // last readable granule
    // source permutation inside each 64-B piece (ring byte 1024 i + 16 L holds
    // stream granule 64 i + 4 (L/4) + ((L - L/16) & 3)); lane l reads granule c
    // of its piece at ring granule 4 l + ((c + l/4) & 3)
    const uint32_t src_off = (uint32_t)(lane & ~3) * 16u + ((uint32_t)((lane & 3) - (lane >> 4)) & 3u) * 16u;
    const uint32_t ring0 = (uint32_t)(uintptr_t)(lds_ptr_t)&L.ring[0][0];

    const uint64_t nw = gridDim.x, w = blockIdx.x;
    const uint64_t q = a.n / nw, rem = a.n % nw;
    const uint64_t fbeg = q * w + min(w, rem), fstop = fbeg + q + (w < rem ? 1u : 0u);

    // issuer: the next step to put in flight (up to S-1 steps ahead of the
    // consumer, into this wave's next run when the current one ends)
    uint64_t ifr = fbeg;
    uint32_t ik = 0, icount = 0;
    RunSpan is = ifr < fstop ? run_span(a, ifr, (uint32_t)min((uint64_t)kWave, fstop - ifr)) : RunSpan{};
    uint32_t islot = 0;   // ring slot of the next issue
    auto issue_next = [&]() {
        if (ifr >= fstop) return;
        const uint64_t sa = is.a0 + (uint64_t)kStreamStep * ik;
        const uint32_t dst = ring0 + islot * kStreamStep;
        if (sa + kStreamStep <= lim16 + 16) {
            const uint8_t* sp = a.data + sa;
#pragma unroll
            for (int i = 0; i < 4; ++i) glds16_nt_s(sp, src_off + 1024u * i, dst + 1024u * i);
        } else {   // the batch's last step: granules past the buffer re-read its last one
            const uint64_t sb = sa + src_off;
#pragma unroll
            for (int i = 0; i < 4; ++i) glds16_nt(a.data + min(sb + 1024u * i, lim16), dst + 1024u * i);
        }
        islot = islot == S - 1 ? 0u : islot + 1u;
        ++icount;
        if (++ik == is.nsteps) {
            ik = 0;
            ifr += kWave;
            if (ifr < fstop) is = run_span(a, ifr, (uint32_t)min((uint64_t)kWave, fstop - ifr));
        }
    };
#pragma unroll
    for (int s = 0; s < S - 1; ++s) issue_next();
    uint32_t ccount = 0, cslot = 0;
    // steps issued before the latest column stores, and how many store instructions those were
    uint32_t st_mark = 0;
    const int n_st = column_stores(a.cols);

    for (uint64_t f0 = fbeg; f0 < fstop; f0 += kWave) {
        const uint32_t nf = (uint32_t)min((uint64_t)kWave, fstop - f0);
        const RunSpan rs = run_span(a, f0, nf);
        // frame geometry relative to the run's aligned start (32 bits: 64 frames x stride <= 1 MiB)
        const uint32_t s0 = (uint32_t)(rs.off0 - rs.a0);           // sh of frame 0
        const uint32_t fmax = nf - 1;
        uint32_t base = 0;                                         // P at the current step start
        for (uint32_t k = 0; k < rs.nsteps; ++k) {
            issue_next();
            if (ccount < st_mark) {
                // this step was issued before the last run's column stores, which
                // retire after it (vmcnt is in order): count them in exactly
                wait_vm_dyn<0, 63>(4 * (int)min(icount - ccount - 1, (uint32_t)(S - 1)) + n_st);
            } else {
                wait_steps<S - 1>((int)(icount - ccount - 1));
            }
            const uint8_t* ring = &L.ring[cslot][0];
            ++ccount;
            cslot = cslot == S - 1 ? 0u : cslot + 1u;
            // the lane's 64-B piece, granule c at ring granule 4 l + ((c + l/4) & 3)
            uint4 g[4];
#pragma unroll
            for (int c = 0; c < 4; ++c)
                g[c] = *reinterpret_cast<const uint4*>(ring + 64 * lane + 16 * ((c + (lane >> 2)) & 3));
            uint32_t pre[4];                                       // pre[c]: sum of granules < c
            uint32_t t = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                pre[c] = t;
                t = sad(g[c].w, sad(g[c].z, sad(g[c].y, sad(g[c].x, t))));
            }
            const uint32_t incl = wave_incl_scan(t);
            const uint32_t excl = base + incl - t;                 // P at the piece start
            base += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);

            // the frame whose stride slot holds the piece start (frame 0 before it)
            const uint32_t x = kStreamStep * k + 64u * (uint32_t)lane;
            const uint32_t r = x - s0;
            int fi = (int)((float)(int)r * inv_stride);            // r < 0 (x < s0): fi <= 0
            fi -= (int)((uint32_t)fi * stride > r && fi > 0);
            fi += (int)((uint32_t)(fi + 1) * stride <= r && x >= s0);
            const uint32_t f = x < s0 ? 0u : min((uint32_t)fi, fmax);
            const uint32_t sf = s0 + f * stride, bf = sf & ~15u;
            const uint32_t ts = bf + kWin, te = (sf + flen - 1u) & ~15u;   // te: the granule holding the last byte
            // P at TS or TE when it lies in this piece (never both: they are >= 880 B apart)
            const uint32_t dts = ts - x, dte = te - x;
            if (dts < 64u || dte < 64u) {
                const uint32_t cut = dts < 64u ? dts : dte;
                uint32_t pc = cut >= 16u ? pre[1] : 0u;
                pc = cut >= 32u ? pre[2] : pc;
                pc = cut >= 48u ? pre[3] : pc;
                uint32_t* rec = dts < 64u ? L.pts : L.pte;
                rec[f] = excl + pc;
            }
            // window granules (at most one frame's window meets a 64-B piece: frame
            // f's, or frame f + 1's when it starts inside the piece) and frame f's
            // last granule
            const uint32_t bg = f < fmax ? ((sf + stride) & ~15u) : 0xFFFFFFF0u;
            const bool wn = x + 64u > bg;
            const int wo0 = (int)x - (int)(wn ? bg : bf);
            uint8_t* wslot = L.win + (f + (wn ? 1u : 0u)) * kSlot + wo0;
            const uint32_t ce = dte < 64u ? (dte >> 4) : 4u;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if ((uint32_t)(wo0 + 16 * c) < (uint32_t)kWin) {
                    uint32_t* dst = reinterpret_cast<uint32_t*>(wslot + 16 * c);
                    dst[0] = g[c].x; dst[1] = g[c].y; dst[2] = g[c].z; dst[3] = g[c].w;
                }
                if (ce == (uint32_t)c) L.endg[f] = g[c];
            }
        }
        wave_sync();

        // ---- parse + window sums + stores (as rx_kernel steps 4-5) ---------
        const bool in_batch = (uint32_t)lane < nf;
        const uint64_t off = rs.off0 + (uint64_t)lane * stride;
        const uint32_t len = in_batch ? flen : 0u;
        const int sh = (int)(off & 15);
        const uint64_t base_g = off - (uint64_t)sh;
        const uint32_t fend = (uint32_t)sh + len;
        Parsed P{};
        if (in_batch) P = parse_frame(FrameBytes{slot + sh, a.data + off, kWin - sh}, len, EXT ? a.flags : 0u);
        const int p0 = P.a_lo + sh, p1 = P.a_hi + sh, p2 = P.b_lo + sh, p3 = P.b_hi + sh;
        uint32_t tA = 0, tB = 0;
        window_sums(slot, p0, p1, min(p2, kWin), min(p3, kWin), tA, tB);
        if (P.l4do && p3 > kWin) {
            // slot bytes [128, fend) = P(TE) - P(TS) + the end granule's bytes below fend
            const int e = (int)((fend - 1u) & 15u) + 1;
            const uint4 eg = L.endg[lane];
            uint32_t tail = L.pte[lane] - L.pts[lane];
            tail = sad(eg.x & first_bytes(clamp04(e)), tail);
            tail = sad(eg.y & first_bytes(clamp04(e - 4)), tail);
            tail = sad(eg.z & first_bytes(clamp04(e - 8)), tail);
            tail = sad(eg.w & first_bytes(clamp04(e - 12)), tail);
            tB += tail;
            const uint8_t* fbp = a.data + base_g;
            if (p2 > kWin) tB -= lane_range_sum(fbp, kWin, p2);
            if ((uint32_t)p3 < fend) tB -= lane_range_sum(fbp, p3, (int)fend);
        }
        uint32_t ipc = 0, l4c = 0;
        finalize(P, tA, tB, (off & 1) != 0, ipc, l4c);
        st_mark = icount;
        store_columns(a.cols, f0, lane, in_batch, P, ipc, l4c, slot, sh);
        if (a.cols.counters) K.add(in_batch, len, P.st);
        wave_sync();   // slots and records are rewritten by the next run
    }
    wait_vm<0>();
    if (a.cols.counters) K.flush_wave(a.cols.counters, lane);
}

}  // namespace
}  // namespace pnetgpu
