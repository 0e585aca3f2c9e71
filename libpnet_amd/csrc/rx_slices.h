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
        const uint64_t off = (a.strided ? a.first + i * a.stride : a.offsets[i]) + a.delta;   // wave-uniform branch
        uint32_t len = a.strided ? a.slice_len : a.lengths[i];
        const uint32_t skip = a.strided ? a.skipword : a.skipwords[i];
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
            off = (a.strided ? a.first + i * a.stride : a.offsets[i]) + a.delta;   // wave-uniform branch
            len = a.strided ? a.slice_len : a.lengths[i];
            skip = a.strided ? a.skipword : a.skipwords[i];
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
#pragma unroll
            for (int c = 0; c < kSmall; ++c) {
                const uint32_t dw[4] = {v[c].x, v[c].y, v[c].z, v[c].w};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int p = 16 * c + 4 * t;
                    acc = sad(dw[t] & first_bytes(clamp04(e - p)) & ~first_bytes(clamp04(sh - p)), acc);
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
// back to back). No descriptors: one wave per run of 64 slices, the run's span
// (<= 4 KiB + 15 B) arrives as coalesced 1-KiB wave loads into an LDS stage
// (aligned like memory, so the byte weights are the absolute ones), lane l sums
// slice l's dwords from the stage with masks on the first and last, removes the
// skipped word, and the 64 results go out as one coalesced 2-B store per lane.
constexpr int kStageGranules = 264;   // >= ceil((63 * 64 + 64 + 15) / 16) + 1

__global__ __launch_bounds__(kBlock) void slice_strided_kernel(SliceArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[kWavesPerBlock][kStageGranules * 4];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    uint32_t* st = stage[wv];
    const uint8_t* sb = reinterpret_cast<const uint8_t*>(st);
    const uint64_t nruns = (a.n + kWave - 1) / kWave;
    const uint64_t wave_stride = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint32_t s = a.stride, L = a.slice_len;
    for (uint64_t run = (uint64_t)blockIdx.x * kWavesPerBlock + wv; run < nruns; run += wave_stride) {
        const uint64_t i0 = run * kWave;
        const uint32_t nr = (uint32_t)min((uint64_t)kWave, a.n - i0);
        const uint64_t b0 = a.first + a.delta + i0 * s;         // first slice of the run (a.data is 16-B aligned)
        const uint64_t g0 = b0 & ~15ull;
        const uint32_t ng = (uint32_t)((b0 + (uint64_t)(nr - 1) * s + L - g0 + 15) >> 4);   // <= 258
        uint4 v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t g = 64u * k + lane;
            v[k] = g < ng ? load16_nt(a.data + g0 + 16u * g) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t g = 64u * k + lane;
            if (g < ng) *reinterpret_cast<uint4*>(st + 4 * g) = v[k];
        }
        wave_sync();
        uint32_t r = 0;
        if ((uint32_t)lane < nr && L) {
            const int p = (int)(b0 - g0) + lane * (int)s, q = p + (int)L;   // stage bytes [p, q)
            uint32_t acc = 0;
#pragma unroll 1
            for (int k = p >> 2; 4 * k < q; ++k)
                acc = sad(st[k] & first_bytes(clamp04(q - 4 * k)) & ~first_bytes(clamp04(p - 4 * k)), acc);
            // skipped word: its bytes [2 skip, 2 skip + 2) that lie in the slice (util.rs:166-178)
            const uint64_t qq = 2ull * a.skipword;
            if (qq < L) {
                const int x = p + (int)qq;
                acc -= (x & 1) ? ((uint32_t)sb[x] << 8) : (uint32_t)sb[x];
                if (qq + 1 < L) acc -= ((x + 1) & 1) ? ((uint32_t)sb[x + 1] << 8) : (uint32_t)sb[x + 1];
            }
            uint32_t f = fold16(acc);
            if (!(p & 1)) f = bswap16(f);
            r = (~f) & 0xFFFFu;                                     // util.rs:76-82 (non-empty)
        }
        if ((uint32_t)lane < nr) a.out[i0 + lane] = (uint16_t)r;
        wave_sync();   // the stage is rewritten by the next run
    }
}

}  // namespace
}  // namespace pnetgpu
