// rx_flat.h — rx_flat_kernel: compact-descriptor batches (IMIX and ring batches), any frame sizes, any order
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
// rx_flat_kernel: one wave per run of 64 frames, every granule of the run in
// ONE flat list streamed by the whole wave.
// ============================================================================
// rx_kernel (mixed shape) spends a run in dependent phases: the window loads,
// then 2-3 rounds of the tail groups (G lanes per frame, rounding waste per
// frame). Here the run's frames are numbered out as a flat list of granules:
// frame k (of those with bytes) owns list entries [cum_k, cum_k + n_k), n_k its
// aligned 16-B granules, cum_k the exclusive wave scan of n. Round r loads
// entries [64 U r, 64 U (r + 1)) with U coalesced-per-frame wave loads per lane,
// so a run of IMIX frames (~1,450 granules) takes 3 rounds of 512 instead of
// window + 3 tail rounds, and no slot is wasted on a frame's rounding.
//   Entry -> frame: per 64-entry block a 64-bit mask of the entries where a
//   frame starts (one LDS OR per frame, by the frame's lane), so a lane's frame
//   is (frames starting before the block: one ballot) + mbcnt(mask) - 1. Every
//   read the loads depend on (the round's masks, then the entries' frame info)
//   is issued as one batch, and the loads themselves are branch-free (entries
//   past the run's end reload its last entry), so the U loads leave together.
//   Window entries (j < NW) also go to the frame's LDS slot for the parse.
//   Every entry's 16 B are summed (v_sad_u16) and one wave scan per
//   instruction gives the running prefix P; a frame's tail (slot bytes
//   [NW*16, end), rx_kernel's speculative tail) is P(last entry) - P(entry
//   NW-1) minus the bytes of its last granule past the frame end, taken from
//   that granule loaded by the frame's own lane at the start of the run.
template <int NW, int U>
struct FlatLds {
    static constexpr int kSlot = NW * 16 + 4;   // +4 B pad: conflict-free parse reads
    uint8_t win[kWave * kSlot];
    uint4 info[kWave];         // compact frame index -> {amin lo, amin hi, cum, granules | lane << 24}
    uint32_t pwin[kWave];      // by lane: P at the frame's last window entry
    uint32_t pend[kWave];      // by lane: P at the frame's last entry
    uint64_t mask[U];          // this round's blocks: entries where a frame starts
};

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int U, bool EXT, bool TX>
__global__ __launch_bounds__(kBlock, 4) void rx_flat_kernel(RxArgs a) {
    constexpr int NW = 8;
    constexpr int kSlot = FlatLds<NW, U>::kSlot;
    constexpr int kWin = NW * 16;
    constexpr uint32_t kRound = 64u * U;

    __shared__ FlatLds<NW, U> lds_all[kWavesPerBlock];
    __shared__ uint64_t blk_ctr[kWavesPerBlock][PNETGPU_NCOUNTERS];

    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    FlatLds<NW, U>& L = lds_all[wv];
    uint8_t* slot = L.win + lane * kSlot;
    Counters K;

    const uint64_t wave_stride = (uint64_t)gridDim.x * kWavesPerBlock;
    uint32_t d_off = 0, d_len = 0;   // compact descriptor of this lane's frame, one run ahead
    auto fetch_desc = [&](uint64_t r) {
        const uint64_t fr = r * kWave + lane;
        if (r < a.nruns && fr < a.n) {
            d_off = reinterpret_cast<const uint32_t*>(a.offsets)[fr];
            d_len = reinterpret_cast<const uint16_t*>(a.lengths)[fr];
        }
    };
    fetch_desc((uint64_t)blockIdx.x * kWavesPerBlock + wv);
    for (uint64_t run = (uint64_t)blockIdx.x * kWavesPerBlock + wv; run < a.nruns; run += wave_stride) {
        // ---- 1. descriptor, granule count, flat numbering ----------------------
        const uint64_t f0 = run * kWave;
        const bool in_batch = f0 + lane < a.n;
        uint64_t off = 0;
        uint32_t len = 0;
        if (in_batch) {
            off = (uint64_t)d_off + a.delta;
            len = d_len;
        }
        const bool desc_bad = in_batch && (off > a.limit || (uint64_t)len > a.limit - off);
        if (!in_batch || desc_bad) {   // nothing is loaded for it
            len = 0;
            off = 0;
        }
        fetch_desc(run + wave_stride);
        const int sh = (int)(off & 15);
        const uint64_t base = off - (uint64_t)sh;
        const uint32_t fend = (uint32_t)sh + len;            // slot-relative end of the frame
        const uint32_t n = len ? (fend + 15u) >> 4 : 0u;     // granules
        const uint32_t incl = wave_incl_scan(n);
        const uint32_t cum = incl - n;
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
        const uint64_t nz = __ballot(n > 0u);
        // the frame's last granule, in flight during the rounds (its bytes past
        // the frame end are taken off the tail)
        uint4 endg = make_uint4(0, 0, 0, 0);
        if (n > (uint32_t)NW) endg = load16(a.data + base + 16u * (n - 1u));
        if (n) {
            const uint32_t k = mbcnt64(nz);
            const uint64_t amin = base - 16ull * cum;        // entry q of this frame is at amin + 16 q
            L.info[k] = make_uint4((uint32_t)amin, (uint32_t)(amin >> 32), cum, n | ((uint32_t)lane << 24));
        }

        // ---- 2. the flat rounds: window entries -> slots, every entry summed ---
        // Lane l takes U consecutive entries of the round, [q0 + U l, q0 + U l + U):
        // its frame lookups are one mask word per round, its sums a running
        // prefix in registers, and one wave scan per round (not per entry) turns
        // the lanes' totals into P. The U loads of an instruction are 16 B per
        // lane at a 16 U-byte stride; the U instructions together cover the
        // round's entries whole.
        const uint32_t e0 = (uint32_t)(U * lane);                     // round-relative first entry
        const uint32_t blk = e0 >> 6;
        // issue round q0: its masks, its entries' frames, their U loads
        auto issue = [&](uint32_t q0, uint4 (&v)[U], uint2 (&zw)[U]) {
            if (lane < U) L.mask[lane] = 0;
            wave_sync();
            if (n && cum >= q0 && cum < q0 + kRound)
                atomicOr(reinterpret_cast<unsigned long long*>(&L.mask[(cum - q0) >> 6]), 1ull << (cum & 63u));
            wave_sync();
            uint32_t pre = 0;                                          // frames starting before my block
#pragma unroll
            for (int bb = 0; bb < U; ++bb) {
                const uint32_t c = (uint32_t)__popcll(__ballot(n && cum < q0 + 64u * bb));
                pre = blk == (uint32_t)bb ? c : pre;
            }
            const uint64_t m = L.mask[blk];
            // my first entry's frame from the mask, the next ones by the start bits
            // (a lane's U entries are consecutive, so they sit in one mask word)
            const uint32_t pos0 = e0 & 63u;
            const uint32_t bits = (uint32_t)(m >> pos0);             // start bits of my U entries
            uint32_t k = pre + (uint32_t)__popcll(pos0 ? (m & ((1ull << pos0) - 1ull)) : 0ull);
            uint4 in[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                k += (bits >> u) & 1u;
                in[u] = L.info[k ? min(k - 1u, (uint32_t)kWave - 1u) : 0u];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t q = min(q0 + e0 + u, total - 1u);      // past the end: reload
                const uint64_t amin = ((uint64_t)in[u].y << 32) | in[u].x;
                v[u] = load16(a.data + amin + 16ull * q);
                zw[u] = make_uint2(in[u].z, in[u].w);
            }
        };
        uint4 v[U], vn[U];
        uint2 zw[U], zwn[U];
        uint32_t carry = 0;
        // sum round q0 (granules v, frame info zw) into the prefix and record
        // the frames' P at their last window entry and their last entry
        auto process = [&](uint32_t q0, const uint4 (&v)[U], const uint2 (&zw)[U]) {
            uint32_t run_sum[U];
            uint32_t acc = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t q = q0 + e0 + u;
                const bool valid = q < total;
                const uint32_t j = q - zw[u].x;
                const int fl = (int)(zw[u].y >> 24);
                if (valid && j < (uint32_t)NW) {                 // window granule -> the frame's slot
                    uint32_t* dst = reinterpret_cast<uint32_t*>(L.win + fl * kSlot + 16 * j);
                    dst[0] = v[u].x; dst[1] = v[u].y; dst[2] = v[u].z; dst[3] = v[u].w;
                }
                acc += valid ? sad(v[u].w, sad(v[u].z, sad(v[u].y, sad(v[u].x, 0u)))) : 0u;
                run_sum[u] = acc;
            }
            const uint32_t incl = wave_incl_scan(acc);
            const uint32_t base_p = carry + incl - acc;               // P before my first entry
            carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t q = q0 + e0 + u;
                const uint32_t j = q - zw[u].x;
                const uint32_t nk = zw[u].y & 0xFFFFFFu;
                const int fl = (int)(zw[u].y >> 24);
                if (q < total && nk > (uint32_t)NW) {
                    if (j == (uint32_t)NW - 1u) L.pwin[fl] = base_p + run_sum[u];
                    if (j == nk - 1u) L.pend[fl] = base_p + run_sum[u];
                }
            }
        };
        // Two register sets used in turn (a copy of in-flight load registers
        // would wait for them), and every path that sums a round either issued
        // the next round first or issues none, so the compiler's wait counts
        // let the sums start while the next round's loads are in flight.
        if (total) {
            issue(0u, v, zw);
            uint32_t q0 = 0;
            while (true) {
                if (q0 + kRound >= total) { process(q0, v, zw); break; }
                issue(q0 + kRound, vn, zwn);                           // in flight while this round is summed
                process(q0, v, zw);
                q0 += kRound;
                if (q0 + kRound >= total) { process(q0, vn, zwn); break; }
                issue(q0 + kRound, v, zw);
                process(q0, vn, zwn);
                q0 += kRound;
            }
        }
        wave_sync();
        uint32_t tail = 0;
        if (n > (uint32_t)NW) {
            // entries NW..n-1 summed whole: drop the last granule's bytes at slot offsets >= fend
            const int hi = (int)fend - 16 * (int)(n - 1u);      // 1..16 bytes of the frame in it
            uint32_t ex = sad(endg.x & ~first_bytes(clamp04(hi)), 0u);
            ex = sad(endg.y & ~first_bytes(clamp04(hi - 4)), ex);
            ex = sad(endg.z & ~first_bytes(clamp04(hi - 8)), ex);
            ex = sad(endg.w & ~first_bytes(clamp04(hi - 12)), ex);
            tail = L.pend[lane] - L.pwin[lane] - ex;
        }

        // ---- 3. parse + window sums (lane l <-> frame l), as rx_kernel -------
        Parsed P{};
        if (desc_bad) P.st = PNET_ST_DESC_INVALID;
        else if (in_batch)
            P = parse_frame(FrameBytes{slot + sh, a.data + off, kWin - sh}, len, EXT ? a.flags : 0u);
        const int p0 = P.a_lo + sh, p1 = P.a_hi + sh, p2 = P.b_lo + sh, p3 = P.b_hi + sh;
        uint32_t tA = 0, tB = 0;
        window_sums(slot, p0, p1, min(p2, kWin), min(p3, kWin), tA, tB);
        if (P.l4do && p3 > kWin) {
            // B past the window = the tail minus [kWin, p2) and [p3, fend)
            tB += tail;
            const uint8_t* fb = a.data + base;
            if (p2 > kWin) tB -= lane_range_sum(fb, kWin, p2);
            if ((uint32_t)p3 < fend) tB -= lane_range_sum(fb, p3, (int)fend);
        }

        // ---- 4. finalize + stores ------------------------------------------
        uint32_t ipc = 0, l4c = 0;
        finalize(P, tA, tB, (off & 1) != 0, ipc, l4c);
        if (TX && in_batch && !desc_bad) tx_write(const_cast<uint8_t*>(a.data) + off, P, ipc, l4c);
        store_columns(a.cols, f0, lane, in_batch, P, ipc, l4c, slot, sh);
#ifndef PNET_NO_FIELD_COLUMNS
        if (EXT && a.field_cols && in_batch)
            store_field_columns(a.cols, f0 + lane, P, FrameBytes{slot + sh, a.data + off, kWin - sh}, a.l3mode);
#endif
        if (a.cols.counters) K.add(in_batch && !desc_bad, len, P.st);
        wave_sync();   // slots, info and prefix slots are rewritten by the next run
    }
    if (a.cols.counters) K.flush(a.cols.counters, blk_ctr, wv, lane);
}

}  // namespace
}  // namespace pnetgpu
