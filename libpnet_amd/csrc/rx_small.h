// rx_small.h — rx_small_kernel (fixed stride, frames 16-B aligned, at most 64 B: the 64-B configs)
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
// rx_small_kernel: fixed stride, frames 16-B aligned, span <= 64 B.
// ============================================================================
// 64-B slots with granule c of frame f at slot granule (c + f/4) & 3: the
// transpose's ds_write_b128 (4 frames x 4 granules per 16-lane pass) and its
// ds_read_b128 (16 frames, one granule each) both hit 16 distinct 4-bank groups
// (the 80-B linear slots had 2-way conflicts on every write pass:
// SQ_LDS_BANK_CONFLICT 2.9e7 per launch, profiles/r03/pmc_lds). Paths that read
// the slot as frame bytes (slow parse, TX, header fields, IPv6 addresses)
// first rewrite it linearly from the lane's registers. Same box, four
// interleaved rounds (profiles/r03/small_swz): udp64 275-280 vs 277-280 us,
// the verify-only record 221-225 vs 222-232 us; bit-exact.
constexpr int kSmallSlot = 64;
__device__ __forceinline__ int small_gpos(int f, int c) { return f * kSmallSlot + 16 * ((c + (f >> 2)) & 3); }

struct SmallRun {
    uint4 g[4];
};

// Coalesced: instruction i, lane L loads granule L%4 of frame 16i + L/4 (for
// stride 64 that is one contiguous 1-KiB wave load); transposed through LDS.
__device__ __forceinline__ SmallRun small_load(const RxArgs& a, uint64_t run, int lane) {
    SmallRun r;
    const uint32_t span = (a.frame_len + 15u) >> 4;
    const uint32_t c = (uint32_t)(lane & 3);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint64_t f = run * kWave + 16 * i + (lane >> 2);
        r.g[i] = make_uint4(0, 0, 0, 0);
        if (f < a.n && c < span)
            r.g[i] = load16_nt(a.data + (a.first + a.delta) + f * a.stride + 16u * c);
    }
    return r;
}

// The small kernel's register fast path (frame bytes [0, 64) of a 16-B-aligned
// frame in w[0..15]): IPv4 with IHL 5, and every frame the dispatch classifies
// without reading past the Ethernet header, with every field at a compile-time
// position. Returns true for the frames that need parse_frame (IPv6, IPv4
// options or an IHL below 5); P, ipc and l4c are complete otherwise.
// packetdump.rs:155-217, ipv4.rs:165-178, udp/tcp/icmp layouts and sizes.
__device__ __forceinline__ bool small_fast(const uint32_t (&w)[16], uint32_t len, Parsed& P, uint32_t& ipc,
                                           uint32_t& l4c) {
    [[maybe_unused]] const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    const uint32_t w3 = w[3];
    const uint32_t w4 = w[4], w5 = w[5], w6 = w[6], w7 = w[7];
    const uint32_t w8 = w[8], w9 = w[9], w10 = w[10], w11 = w[11];
    const uint32_t w12 = w[12], w13 = w[13], w14 = w[14], w15 = w[15];
    bool slow = false;
    if (len < 14) {
        P.st = PNET_ST_ETH_MALFORMED;
    } else {
        P.et = bswap16(w3 & 0xFFFFu);
        P.l3 = 14;
        if (P.et == 0x0800u) {
            if (len < 34) {
                P.st = PNET_ST_L3_IPV4 | PNET_ST_L3_MALFORMED;
            } else if (((w3 >> 16) & 0xFu) != 5u) {
                slow = true;                       // IPv4 options / IHL clamp: generic path
            } else {
                // ---- fast path: IPv4, IHL 5; every position below is static ----
                P.st = PNET_ST_L3_IPV4;
                P.is_v4 = true;
                const uint32_t eplen = len - 14;
                const uint32_t tl = bswap16(w4 & 0xFFFFu);
                P.ttl = (w5 >> 16) & 0xFFu;
                P.proto = w5 >> 24;
                P.ipstored = bswap16(w6 & 0xFFFFu);
                P.s4 = (bswap16(w6 >> 16) << 16) | bswap16(w7 & 0xFFFFu);   // bytes 26..29
                P.d4 = (bswap16(w7 >> 16) << 16) | bswap16(w8 & 0xFFFFu);   // bytes 30..33
                // header sum [14,34) without the checksum word (bytes 24,25)
                uint32_t tA = sad(w3 & 0xFFFF0000u, 0u);
                tA = sad(w4, tA);
                tA = sad(w5, tA);
                tA = sad(w6 & 0xFFFF0000u, tA);
                tA = sad(w7, tA);
                tA = sad(w8 & 0x0000FFFFu, tA);
                ipc = (~bswap16(fold16(tA))) & 0xFFFFu;
                if (ipc == P.ipstored) P.st |= PNET_ST_IP_CSUM_OK;
                const uint32_t plen = tl > 20u ? tl - 20u : 0u;
                if (eplen > 20u) {
                    P.l4off = 34;
                    P.l4len = min(20u + plen, eplen) - 20u;
                }
                uint32_t kind = 0, minlen = 0;
                switch (P.proto) {
                    case 17: kind = PNET_ST_L4_UDP; minlen = 8; break;
                    case 6: kind = PNET_ST_L4_TCP; minlen = 20; break;
                    case 1: kind = PNET_ST_L4_ICMP; minlen = 4; break;
                    case 58: kind = PNET_ST_L4_ICMPV6; minlen = 4; break;
                    default: break;
                }
                if (!kind) {
                    P.st |= PNET_ST_UNKNOWN_PROTO;
                } else {
                    P.st |= kind;
                    if (P.l4len < minlen) {
                        P.st |= PNET_ST_L4_MALFORMED;
                    } else {
                        P.sp = bswap16(w8 >> 16);                            // bytes 34,35
                        uint32_t stored_le;
                        if (P.proto == 17) {
                            P.dp = bswap16(w9 & 0xFFFFu);
                            stored_le = w10 & 0xFFFFu;                       // bytes 40,41
                        } else if (P.proto == 6) {
                            P.dp = bswap16(w9 & 0xFFFFu);
                            stored_le = w12 >> 16;                           // bytes 50,51
                        } else {
                            P.dp = P.l4len >= 8 ? bswap16(w9 >> 16) : 0u;    // bytes 38,39
                            stored_le = w9 & 0xFFFFu;                        // bytes 36,37
                        }
                        P.l4stored = bswap16(stored_le);
                        P.l4csum_at = P.proto == 17 ? 40 : (P.proto == 6 ? 50 : 36);
                        if (P.proto != 58) {       // ICMPv6 over IPv4: no checksum defined
                            const int e = 34 + (int)P.l4len;
                            uint32_t tB = sad(w8 & 0xFFFF0000u, 0u);
                            tB = sad(w9 & first_bytes(clamp04(e - 36)), tB);
                            tB = sad(w10 & first_bytes(clamp04(e - 40)), tB);
                            tB = sad(w11 & first_bytes(clamp04(e - 44)), tB);
                            tB = sad(w12 & first_bytes(clamp04(e - 48)), tB);
                            tB = sad(w13 & first_bytes(clamp04(e - 52)), tB);
                            tB = sad(w14 & first_bytes(clamp04(e - 56)), tB);
                            tB = sad(w15 & first_bytes(clamp04(e - 60)), tB);
                            tB -= stored_le;
                            uint32_t pseudo = 0;
                            if (P.proto != 1)
                                pseudo = (P.s4 >> 16) + (P.s4 & 0xFFFFu) + (P.d4 >> 16) + (P.d4 & 0xFFFFu) +
                                         P.proto + P.l4len;
                            l4c = (~fold16(bswap16(fold16(tB)) + pseudo)) & 0xFFFFu;
                            P.st |= PNET_ST_L4_CSUM_DONE;
                            if (l4c == P.l4stored) P.st |= PNET_ST_L4_CSUM_OK;
                        }
                    }
                }
            }
        } else if (P.et == 0x86DDu) {
            slow = true;
        } else {
            P.st = PNET_ST_UNKNOWN_ETHERTYPE;
        }
    }
    return slow;
}

// FIELDS: the header-field columns may be requested (a separate instantiation:
// their code in the loop cost the plain record 3-10 % on MI355X)
template <bool TX, bool FIELDS>
__global__ __launch_bounds__(kBlock, PNET_SMALL_WAVES) void rx_small_kernel(RxArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_slots[kWavesPerBlock][kWave * kSmallSlot + 16];
    __shared__ uint64_t blk_ctr[kWavesPerBlock][PNETGPU_NCOUNTERS];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    uint8_t* slot = lds_slots[wv] + lane * kSmallSlot;
    Counters K;

    const uint64_t wave_stride = (uint64_t)gridDim.x * kWavesPerBlock;
    PNET_WT_BEGIN;
    RunQueue q(a.sched, a.nruns, (uint64_t)blockIdx.x * kWavesPerBlock + wv, wave_stride);
    uint64_t run = q.take();
    SmallRun cur = run < a.nruns ? small_load(a, run, lane) : SmallRun{};
    while (run < a.nruns) {
        PNET_WT_RUN;
        // software pipelining: the next run's loads are in flight while this one is processed
        // (two runs ahead measured no faster: the wave is not short of loads in flight)
        const uint64_t nrun = q.take();
        SmallRun nxt = nrun < a.nruns ? small_load(a, nrun, lane) : SmallRun{};

        const uint64_t f0 = run * kWave;
        const bool in_batch = f0 + lane < a.n;
        const uint32_t len = in_batch ? a.frame_len : 0u;
        {
            // granule (frame 16i + lane/4, chunk lane%4) -> that frame's slot; read back own frame
#pragma unroll
            for (int i = 0; i < 4; ++i)
                *reinterpret_cast<uint4*>(lds_slots[wv] + small_gpos(16 * i + (lane >> 2), lane & 3)) = cur.g[i];
            wave_sync();
#pragma unroll
            for (int c = 0; c < 4; ++c)
                cur.g[c] = *reinterpret_cast<const uint4*>(lds_slots[wv] + small_gpos(lane, c));
        }

        Parsed P{};
        uint32_t ipc = 0, l4c = 0;
        const uint32_t wv16[16] = {cur.g[0].x, cur.g[0].y, cur.g[0].z, cur.g[0].w, cur.g[1].x, cur.g[1].y,
                                   cur.g[1].z, cur.g[1].w, cur.g[2].x, cur.g[2].y, cur.g[2].z, cur.g[2].w,
                                   cur.g[3].x, cur.g[3].y, cur.g[3].z, cur.g[3].w};
        PNET_PH(0);   // probe: next run's loads issued, this run's transpose (waits for its loads)
        const bool slow = in_batch && small_fast(wv16, len, P, ipc, l4c);
        // ---- generic path through LDS for the lanes the fast path did not take ----
        const bool need_v6 = a.cols.src_ipv6 || a.cols.dst_ipv6;
        // the slot as frame bytes (wave-uniform): each lane rewrites its own slot
        // linearly from its registers (no other lane reads it before the next sync)
        if (TX || (FIELDS && a.field_cols) || need_v6 || __ballot(slow)) {
#pragma unroll
            for (int c = 0; c < 4; ++c) *reinterpret_cast<uint4*>(slot + 16 * c) = cur.g[c];
        }
        if (__ballot(slow) || need_v6) {
            if (slow) {
                // flags are 0 here and the frame (<= 64 B) is entirely in its slot
                P = parse_frame(FrameBytes{slot, slot, 64}, len, 0u);
                uint32_t tA = 0, tB = 0;
                window_sums(slot, P.a_lo, P.a_hi, P.b_lo, P.b_hi, tA, tB);
                finalize(P, tA, tB, false, ipc, l4c);
            }
        }
        if (TX) {
            // patch the frame's LDS copy, then write the run's granules back the
            // way they were loaded (four coalesced 1-KiB wave stores): whole
            // lines instead of four scattered byte stores per frame, which left
            // every line of the batch partially dirty (0.63 ms -> see DESIGN.md)
            if (in_batch) tx_write(slot, P, ipc, l4c);
            wave_sync();
            const uint32_t span = (a.frame_len + 15u) >> 4;
            const uint32_t c = (uint32_t)(lane & 3);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint64_t f = f0 + 16 * i + (lane >> 2);
                if (f < a.n && c < span) {
                    const uint4 v = *reinterpret_cast<const uint4*>(lds_slots[wv] + (16 * i + (lane >> 2)) * kSmallSlot +
                                                                    16 * c);
                    __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w},
                                                reinterpret_cast<u32x4_t*>(const_cast<uint8_t*>(a.data) +
                                                                           (a.first + a.delta) + f * a.stride + 16u * c));
                }
            }
        }
        PNET_PH(2);   // probe: fast path / parse
        store_columns(a.cols, f0, lane, in_batch, P, ipc, l4c, slot, 0);
        if (FIELDS && a.field_cols && in_batch)
            store_field_columns(a.cols, f0 + lane, P, FrameBytes{slot, slot, 64}, false);
        if (a.cols.counters) K.add(in_batch, len, P.st);
        wave_sync();
        PNET_PH(3);   // probe: stores, counters
        cur = nxt;
        run = nrun;
    }
    if (a.cols.counters) K.flush(a.cols.counters, blk_ctr, wv, lane);
    PNET_WT_END((uint64_t)blockIdx.x * kWavesPerBlock + wv);
}

}  // namespace
}  // namespace pnetgpu
