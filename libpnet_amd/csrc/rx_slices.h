// rx_slices.h — slice_kernel, the batched util::checksum / ipv4_checksum / ipv6_checksum (and *_adv) entry points
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

// ---------------------------------------------------------------------------
// Batched util::checksum / ipv4_checksum / ipv6_checksum over slices.
// One group of 16 lanes per slice (4 slices per wave per step): coalesced
// 16-B granules, masked sums, shuffle reduce, lane 0 of the group finalizes.

#ifndef PNET_SLICE_U
#define PNET_SLICE_U 4   // loads in flight per lane in the slice kernels
#endif
// Weighted byte sum of [off, off+len) (absolute offsets into a.data) by one
// 16-lane group: coalesced aligned granules, U loads in flight per lane (the
// 16 lanes cover 256 B per load round), byte masks only on the slice's first
// and last granule, shuffle-reduced so every lane of the group returns the total.
__device__ __forceinline__ uint32_t group_range_sum(const uint8_t* data, uint64_t off, uint32_t len, int j) {
    constexpr int G = 16, U = PNET_SLICE_U;
    const int sh = (int)(off & 15);
    const uint8_t* fb = data + (off - (uint64_t)sh);
    const int e = sh + (int)len;
    const uint32_t nneed = len ? (uint32_t)((e + 15) >> 4) : 0u;
    uint32_t acc = 0;
#pragma unroll 1
    for (uint32_t c0 = j; c0 < nneed; c0 += G * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * G;
            v[u] = c < nneed ? *reinterpret_cast<const uint4*>(fb + 16u * c) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = c0 + u * G;
            const uint32_t dw[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            if (c == 0 || c + 1 == nneed) {          // edge granule (zero when c >= nneed)
                const int p = (int)(16u * c);
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint32_t mk = first_bytes(clamp04(e - p - 4 * t)) & ~first_bytes(clamp04(sh - p - 4 * t));
                    acc = sad(dw[t] & mk, acc);
                }
            } else {
                acc = sad(dw[3], sad(dw[2], sad(dw[1], sad(dw[0], acc))));
            }
        }
    }
#pragma unroll
    for (int o = G / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
    return acc;
}

// PSEUDO: 0 = util::checksum, 4 = util::ipv4_checksum, 16 = util::ipv6_checksum.
// EXTRA: the *_checksum_adv form with an extra_data slice (util.rs:109-114).
template <int PSEUDO, bool EXTRA>
__global__ __launch_bounds__(kBlock) void slice_kernel(SliceArgs a) {
    constexpr int G = 16;
    const int lane = threadIdx.x & (kWave - 1);
    const int j = lane % G;
    const uint64_t gid = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / G;
    const uint64_t ngroups = (uint64_t)gridDim.x * kBlock / G;
    // groups are 16-lane aligned, so every shuffle stays inside one group, whose
    // lanes share i (and therefore control flow)
    for (uint64_t i = gid; i < a.n; i += ngroups) {
        uint64_t off;
        uint32_t len, skip;
        if (a.strided) {            // wave-uniform branches: strided, compact or full descriptors
            off = a.first + i * a.stride;
            len = a.slice_len;
            skip = a.skipword;
        } else if (a.compact) {
            const uint2 dsc = reinterpret_cast<const uint2*>(a.offsets)[i];
            off = dsc.x;
            len = dsc.y & 0xFFFFu;
            skip = dsc.y >> 16;
        } else {
            off = a.offsets[i];
            len = a.lengths[i];
            skip = a.skipwords[i];
        }
        off += a.delta;
        if (off > a.limit || (uint64_t)len > a.limit - off) len = 0;
        uint32_t acc = group_range_sum(a.data, off, len, j);
        uint32_t pe = 0, elen = 0;
        if (EXTRA) {
            // sum_be_words(extra, extra.len() / 2): every whole word, never the odd
            // trailing byte (util.rs:114; the quirk documented at udp.rs:42-44); the
            // extra slice starts its own word alignment
            const uint64_t eoff = a.extra_offsets[i] + a.delta;
            elen = a.extra_lengths[i];
            if (eoff > a.limit || (uint64_t)elen > a.limit - eoff) elen = 0;
            const uint32_t te = group_range_sum(a.data, eoff, elen & ~1u, j);
            pe = fold16(te);
            if (!(eoff & 1)) pe = bswap16(pe);
        }
        if (j == 0) {
            // skipped word: bytes [2*skip, 2*skip+2) of the slice that exist (util.rs:166-178)
            const uint8_t* sb = a.data + off;
            if ((uint64_t)skip * 2 < len) {
                const uint64_t q = 2ull * skip;
                const uint32_t b0 = sb[q];
                acc -= ((off + q) & 1) ? (b0 << 8) : b0;
                if (q + 1 < len) {
                    const uint32_t b1 = sb[q + 1];
                    acc -= ((off + q + 1) & 1) ? (b1 << 8) : b1;
                }
            }
            uint32_t p = fold16(acc);
            if (!(off & 1)) p = bswap16(p);
            uint32_t r;
            if (PSEUDO == 0) {
                r = len ? ((~p) & 0xFFFFu) : 0u;            // util.rs:77-79
            } else {
                const uint8_t* ad = a.addrs + i * (2 * PSEUDO);
                uint32_t s = 0;
#pragma unroll
                for (int k = 0; k < 2 * PSEUDO; k += 2) s += ((uint32_t)ad[k] << 8) | ad[k + 1];
                s += a.protos[i] + len + elen + p + pe;     // util.rs:103-114
                r = (~fold16(s)) & 0xFFFFu;
            }
            a.out[i] = (uint16_t)r;
        }
    }
}

// slice_run_kernel: the same results without the extra slice (util::checksum,
// ipv4_checksum, ipv6_checksum), for batches of any slice sizes but built for
// small ones (the reference's own bench shape is a 20-B slice,
// checksum_benchmarks.rs:8-12). One wave per run of 64 slices, lane l <-> slice
// l: coalesced descriptor loads, a slice of at most kSmall granules summed by
// its own lane (all its loads issued at once, with the two skipped-word bytes),
// longer slices listed and summed by 16-lane groups as in slice_kernel, and one
// coalesced 2-B store per lane. slice_kernel gave 16 lanes to every slice: a
// 20-B slice left 14 of them idle and the results went out as 2-B stores
// scattered 32 B apart.
template <int PSEUDO>
__global__ __launch_bounds__(kBlock) void slice_run_kernel(SliceArgs a) {
    constexpr int kSmall = 4;    // granules summed by the slice's own lane
    constexpr int G = 16;
    __shared__ uint32_t gsum[kWavesPerBlock][kWave];
    __shared__ uint8_t glist[kWavesPerBlock][kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    const uint64_t nruns = (a.n + kWave - 1) / kWave;
    const uint64_t wave_stride = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t run = (uint64_t)blockIdx.x * kWavesPerBlock + wv; run < nruns; run += wave_stride) {
        const uint64_t i = run * kWave + lane;
        const bool in = i < a.n;
        uint64_t off = 0;
        uint32_t len = 0, skip = 0;
        if (in) {
            if (a.strided) {        // wave-uniform branches: strided, compact (one 8-B load) or full descriptors
                off = a.first + i * a.stride;
                len = a.slice_len;
                skip = a.skipword;
            } else if (a.compact) {
                const uint2 dsc = reinterpret_cast<const uint2*>(a.offsets)[i];
                off = dsc.x;
                len = dsc.y & 0xFFFFu;
                skip = dsc.y >> 16;
            } else {
                off = a.offsets[i];
                len = a.lengths[i];
                skip = a.skipwords[i];
            }
            off += a.delta;
            if (off > a.limit || (uint64_t)len > a.limit - off) {
                len = 0;
                off = 0;
            }
        }
        const int sh = (int)(off & 15);
        const uint8_t* fb = a.data + (off - (uint64_t)sh);
        const int e = sh + (int)len;
        const uint32_t nneed = len ? (uint32_t)((e + 15) >> 4) : 0u;
        const bool small = nneed <= (uint32_t)kSmall;
        // skipped word: its bytes [2 skip, 2 skip + 2) that lie in the slice (util.rs:166-178)
        const uint64_t q = 2ull * skip;
        const bool s0 = q < len, s1 = q + 1 < len;
        uint32_t b0 = 0, b1 = 0;                 // in flight across the group phase
        if (s0) b0 = a.data[off + q];
        if (s1) b1 = a.data[off + q + 1];
        // slices past kSmall granules: 16-lane groups over the wave's list of them
        // (before the small slices' loads: no granule registers held across it)
        const uint64_t bmask = __ballot(in && !small);
        if (bmask) {
            if (in && !small) glist[wv][__popcll(bmask & ((1ull << lane) - 1ull))] = (uint8_t)lane;
            wave_sync();
            const int nb = __popcll(bmask);
            const int j = lane % G;
            for (int k0 = 0; k0 < nb; k0 += kWave / G) {   // wave-uniform; a group's lanes share k
                const int k = k0 + lane / G;
                const int sl = k < nb ? glist[wv][k] : 0;
                // both shuffles unconditional: a shuffle under `k < nb` would read
                // its source lane with that lane masked off
                const uint64_t soff = (uint64_t)__shfl((unsigned long long)off, sl);
                const uint32_t sl_len = (uint32_t)__shfl((int)len, sl);
                const uint32_t slen = k < nb ? sl_len : 0u;
                const uint32_t t = group_range_sum(a.data, soff, slen, j);
                if (k < nb && j == 0) gsum[wv][sl] = t;
            }
            wave_sync();
        }
        uint4 v[kSmall];
#pragma unroll
        for (int c = 0; c < kSmall; ++c)
            v[c] = small && (uint32_t)c < nneed ? load16(fb + 16 * c) : make_uint4(0, 0, 0, 0);
        uint32_t acc = 0;
        if (small) {
            // every loaded granule summed whole (the others are zero), then the
            // bytes before the slice in granule 0 and after it in the last one
            // subtracted: ~50 VALU instead of a mask pair per dword (~190; a
            // wave64 VALU op takes 4 cycles, and VALU bound this shape)
#pragma unroll
            for (int c = 0; c < kSmall; ++c) acc = sad(v[c].w, sad(v[c].z, sad(v[c].y, sad(v[c].x, acc))));
            if (nneed) {
                // head: bytes [0, sh) of granule 0
                const uint32_t q = (uint32_t)sh >> 2, r = (uint32_t)sh & 3u;
                const uint32_t s1 = sad(v[0].x, 0u), s2 = sad(v[0].y, s1), s3 = sad(v[0].z, s2);
                uint32_t hw = v[0].x, hs = 0u;
                hw = q == 1u ? v[0].y : hw; hs = q == 1u ? s1 : hs;
                hw = q == 2u ? v[0].z : hw; hs = q == 2u ? s2 : hs;
                hw = q == 3u ? v[0].w : hw; hs = q == 3u ? s3 : hs;
                acc -= sad(hw & (r ? 0xFFFFFFFFu >> (32u - 8u * r) : 0u), hs);
                // tail: bytes [e - 16 c, 16) of every granule c, clamped: nothing
                // below the last granule, zero data above it (no dynamic
                // indexing of v: a select of whole granules became a scratch
                // array and ran 3.5x slower)
#pragma unroll
                for (int c = 0; c < kSmall; ++c) {
                    const int ebi = e - 16 * c;
                    const uint32_t eb = (uint32_t)min(max(ebi, 0), 16);
                    const uint32_t tq = eb >> 2, tr = eb & 3u;
                    const uint32_t u3 = sad(v[c].w, 0u), u2 = sad(v[c].z, u3), u1 = sad(v[c].y, u2);
                    uint32_t tw = v[c].x, ts = u1;
                    tw = tq == 1u ? v[c].y : tw; ts = tq == 1u ? u2 : ts;
                    tw = tq == 2u ? v[c].z : tw; ts = tq == 2u ? u3 : ts;
                    tw = tq >= 3u ? v[c].w : tw; ts = tq >= 3u ? 0u : ts;
                    const uint32_t keep = tr ? 0xFFFFFFFFu >> (32u - 8u * tr) : 0u;
                    acc -= tq >= 4u ? 0u : sad(tw & ~keep, ts);
                }
            }
        } else {
            acc = gsum[wv][lane];
        }
        acc -= s0 ? (((off + q) & 1) ? (b0 << 8) : b0) : 0u;
        acc -= s1 ? (((off + q + 1) & 1) ? (b1 << 8) : b1) : 0u;
        uint32_t p = fold16(acc);
        if (!(off & 1)) p = bswap16(p);
        uint32_t r;
        if (PSEUDO == 0) {
            r = len ? ((~p) & 0xFFFFu) : 0u;                    // util.rs:77-79
        } else {
            uint32_t s = 0;
            if (in) {
                const uint8_t* ad = a.addrs + i * (2 * PSEUDO);
                if (!(reinterpret_cast<uintptr_t>(a.addrs) & 3u)) {   // wave-uniform
#pragma unroll
                    for (int k = 0; k < 2 * PSEUDO; k += 4) {
                        const uint32_t w = *reinterpret_cast<const uint32_t*>(ad + k);   // 4 octets, LE load
                        s += bswap16(w & 0xFFFFu) + bswap16(w >> 16);
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 2 * PSEUDO; k += 2) s += ((uint32_t)ad[k] << 8) | ad[k + 1];
                }
                s += a.protos[i];
            }
            s += len + p;                                        // util.rs:103-113
            r = (~fold16(s)) & 0xFFFFu;
        }
        if (in) a.out[i] = (uint16_t)r;
        wave_sync();   // glist / gsum are rewritten by the next run
    }
}

// slice_strided_kernel: util::checksum over uniform slices, slice i = [first +
// i * stride, +slice_len) with stride and slice_len at most 64 B (the
// reference's own bench shape: 20-B slices, checksum_benchmarks.rs:8-12, here
// back to back). No descriptors. One wave per "block" of R runs of 64 slices,
// R = the most runs whose span fits 4 KiB (3 for 20-B slices, 16 for <= 4-B
// strides): the block's span arrives as (at most) five coalesced 1-KiB wave
// loads, the NEXT block's loads are issued before this one is summed (two
// register sets), and the span goes through an LDS stage that keeps memory's
// dword alignment (so the byte weights are the absolute ones) with one pad
// dword after every 64 B: lane l reads slice 64 r + l as ND dwords (all issued
// at once, masks past its ends), and lanes 16, 32 or 64 B apart hit distinct
// banks (17 l instead of 16 l). Then the skipped word is removed and each run's
// 64 results go out as one coalesced 2-B store per lane.
// ND = dwords read per slice (>= ceil((slice_len + 3) / 4)); EXACT: ND equals it
// (the 20-B and 64-B shapes), which allows the cheaper sum.
constexpr int kStageDwords = 1152;   // padded (4175 + 4 * 17) / 4 * 17 / 16, rounded up
// PAD: one pad dword per 16 (strides that are multiples of 8 B would put lanes
// on the same banks); without it the ND reads are one address + immediate offsets
template <bool PAD>
__device__ __forceinline__ int stage_index(int d) { return PAD ? d + (d >> 4) : d; }

template <int ND, bool EXACT, bool PAD>
__global__ __launch_bounds__(kBlock) void slice_strided_kernel(SliceArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[kWavesPerBlock][kStageDwords];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    uint32_t* st = stage[wv];
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(st);
    const uint32_t s = a.stride, L = a.slice_len;
    // runs per block: span (R * 64 - 1) * s + L + 15 <= 4096 + 64 + 15
    const uint32_t R = s ? max(1u, min(16u, 4096u / (64u * s))) : 16u;
    const uint64_t per = (uint64_t)kWave * R;
    const uint64_t nblk = (a.n + per - 1) / per;
    const uint64_t wave_stride = (uint64_t)gridDim.x * kWavesPerBlock;
    struct Blk {
        uint64_t i0, g0;
        uint32_t nsl, ng;
    };
    auto locate = [&](uint64_t b) {
        Blk k{};
        if (b < nblk) {
            k.i0 = b * per;
            k.nsl = (uint32_t)min(per, a.n - k.i0);
            const uint64_t b0 = a.first + a.delta + k.i0 * s;   // a.data is 16-B aligned
            k.g0 = b0 & ~15ull;
            k.ng = (uint32_t)((b0 + (uint64_t)(k.nsl - 1) * s + L - k.g0 + 15) >> 4);
        }
        return k;
    };
    auto load = [&](const Blk& k, uint4 (&v)[5]) {
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            const uint32_t g = 64u * c + lane;
            v[c] = g < k.ng ? load16_nt(a.data + k.g0 + 16u * g) : make_uint4(0, 0, 0, 0);
        }
    };
    uint64_t b = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
    Blk cur = locate(b);
    uint4 v[5], w[5];
    load(cur, v);
    for (; b < nblk; b += wave_stride) {
        const Blk nxt = locate(b + wave_stride);
        load(nxt, w);                                 // in flight while this block is summed
#pragma unroll
        for (int c = 0; c < 5; ++c) {
            const int g = 64 * c + lane;
            if ((uint32_t)g < cur.ng) {
                if (PAD) {
                    uint32_t* dst = st + stage_index<PAD>(4 * g);   // a granule never straddles a pad
                    dst[0] = v[c].x; dst[1] = v[c].y; dst[2] = v[c].z; dst[3] = v[c].w;
                } else {
                    *reinterpret_cast<uint4*>(st + 4 * g) = v[c];
                }
            }
        }
        wave_sync();
        const int pb = (int)(a.first + a.delta + cur.i0 * s - cur.g0);   // stage byte of the block's slice 0
#ifdef PNET_STRIDED_NOCOMP   // A/B: one result per block from the stage, no slice sums
        if (lane == 0 && st[lane * 17] == 0x12345u) a.out[cur.i0] = 1;
        if (false)
#endif
#pragma unroll 1
        for (uint32_t r = 0; r < R; ++r) {
            const uint32_t k = 64u * r + lane;
            uint32_t res = 0;
            if (k < cur.nsl && L) {
                const int p = pb + (int)(k * s), q = p + (int)L;   // unpadded stage bytes [p, q)
                const int d0 = p >> 2;
                uint32_t x[ND];
#pragma unroll
                for (int t = 0; t < ND; ++t) x[t] = st[stage_index<PAD>(d0 + t)];
                // every dword read summed whole, then the excess removed: the
                // bytes before p in dword 0 and the bytes from q on (dword tq,
                // ND-2 or ND-1, in part; the dwords after it whole). VALU is the
                // limit of this shape (a wave64 op takes 4 cycles), so no
                // per-dword masks (round 3: 20-B slices 85 -> see DESIGN §3)
                uint32_t acc = 0;
                if constexpr (EXACT) {
                    // ND = (slice_len + 6) / 4 exactly: every dword read summed
                    // whole, then the excess removed — the bytes before p in
                    // dword 0 and the 0..6 bytes from q on (dword tq = ND - 2 or
                    // ND - 1 in part and the dword after it; none when q ends
                    // dword ND - 1). VALU is this shape's limit (a wave64 op
                    // takes 4 cycles), so no per-dword masks.
#pragma unroll
                    for (int t = 0; t < ND; ++t) acc = sad(x[t], acc);
                    const uint32_t ph = (uint32_t)p & 3u, qt = (uint32_t)q & 3u;
                    const uint32_t hmask = ph ? 0xFFFFFFFFu >> (32u - 8u * ph) : 0u;   // bytes [4 d0, p)
                    const uint32_t tkeep = qt ? 0xFFFFFFFFu >> (32u - 8u * qt) : 0u;   // bytes [4 (q>>2), q)
                    acc -= sad(x[0] & hmask, 0u);
                    const int tq = (q >> 2) - d0;
                    const uint32_t ex1 = sad(x[ND - 1] & ~tkeep, 0u);
                    uint32_t ex = tq == ND - 1 ? ex1 : 0u;
                    if constexpr (ND >= 2) ex = tq == ND - 2 ? sad(x[ND - 2] & ~tkeep, sad(x[ND - 1], 0u)) : ex;
                    acc -= ex;
                } else {
#pragma unroll
                    for (int t = 0; t < ND; ++t) {
                        const int pos = 4 * (d0 + t);
                        acc = sad(x[t] & first_bytes(clamp04(q - pos)) & ~first_bytes(clamp04(p - pos)), acc);
                    }
                }
                // skipped word: its bytes [2 skip, 2 skip + 2) that lie in the slice (util.rs:166-178)
                const uint64_t qq = 2ull * a.skipword;
                if (qq < L) {
                    const int y = p + (int)qq;
                    const uint32_t b0 = sb[4 * stage_index<PAD>(y >> 2) + (y & 3)];
                    acc -= (y & 1) ? (b0 << 8) : b0;
                    if (qq + 1 < L) {
                        const int z = y + 1;
                        const uint32_t b1 = sb[4 * stage_index<PAD>(z >> 2) + (z & 3)];
                        acc -= (z & 1) ? (b1 << 8) : b1;
                    }
                }
                uint32_t f = fold16(acc);
                if (!(p & 1)) f = bswap16(f);
                res = (~f) & 0xFFFFu;                           // util.rs:76-82 (non-empty)
            }
#ifdef PNET_STRIDED_NOSTORE   // A/B: results stored only if they hit a magic value
            if (k < cur.nsl && res == 0x12345u) a.out[cur.i0 + k] = (uint16_t)res;
#else
            if (k < cur.nsl) a.out[cur.i0 + k] = (uint16_t)res;
#endif
        }
        wave_sync();   // the stage is rewritten by the next block
        cur = nxt;
#pragma unroll
        for (int c = 0; c < 5; ++c) v[c] = w[c];
    }
}

}  // namespace
}  // namespace pnetgpu
