// rx_split.h — rx_split_kernel: a streaming wave and a parsing wave per block (descriptor or stride batches, receive only)
// Part of the receive-path kernels; included once, by rx_kernel.hip (one
// translation unit, so every kernel still sees the shared device helpers inline).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pnetgpu.h"
#include "rx_internal.h"
#include "rx_common.h"
#include "rx_generic.h"
#include "rx_stream.h"

// stream-wave instruction priority (0-3; 0, 1 and 3 measured alike, profiles/r02/split/)
#ifndef PNET_SPLIT_PRIO
#define PNET_SPLIT_PRIO 3
#endif

namespace pnetgpu {
namespace {

// ============================================================================
// rx_split_kernel: two-wave blocks. Wave 0 streams, wave 1 parses.
// ============================================================================
// The register kernels read frames as group-per-frame pieces (8 frames x 128 B,
// or 16 x 64 B, per wave instruction), a shape the memory system serves at
// ~5.3-5.9 TB/s, against ~6.8 TB/s for 1-KiB-contiguous wave instructions
// through an LDS-DMA ring (profiles/r01/sol/). rx_stream_kernel reads that way
// but parses and stores in the same wave, which stalls its stream once per run.
// Here the stream never waits for a parse:
//   Streaming wave (lane f <-> frame f of the run): the run's byte range
//   [lo, hi) (granule-aligned bases of its frames; runs whose frames are not
//   packed within 9/8 of their bytes plus 8 KiB take a per-lane path instead)
//   flows through an S-step LDS ring in 4-KiB steps by global_load_lds_dwordx4,
//   S-1 steps in flight, crossing into the next run. Per step, lane l sums its
//   64-B piece (16 v_sad_u16), one wave scan gives P(x) (the weighted byte sum
//   of [lo, x)) at each of the step's 256 granule starts, kept in an LDS table;
//   each frame's lane then takes P at its tail start TS = base + 128 and at its
//   last granule TE when they fall in the step. At the run's end tail = P(TE) -
//   P(TS) + the end granule's bytes below the frame end (rx_kernel's
//   speculative tail), for the parsing wave.
//   Parsing wave: loads the descriptors three runs ahead into LDS (so the
//   streaming wave issues no VMEM op but the ring's) and each frame's window
//   (its first 8 granules) one run ahead into registers — lines the streaming
//   wave fetches at the same time, so on-chip hits — then per run parses every
//   frame from its slot, trims the tail to the L4 range and stores the columns
//   exactly as rx_kernel does; its stores never sit in the stream's vmcnt.
//   (Copying the windows out of the ring in the streaming wave instead cost
//   ~1,000 cycles per 4-KiB step: 0.51 ms vs 0.24 ms for IMIX without it.)
//   The waves meet at one s_barrier per run: tails are double-buffered, the
//   descriptors triple-buffered.
template <int S>
struct SplitLds {
    static constexpr int kSlot = 8 * 16 + 4;   // 132 B: conflict-free parse reads
    uint8_t ring[S][kStreamStep];
    uint8_t win[2][kWave * kSlot];   // each parsing wave's window slots
    uint4 ptab[kWave];               // P at the step's granule starts, 4 per piece
    uint32_t tail[4][kWave];         // run k: tail[k % 4]
    uint64_t doff[6][kWave];         // run k: [k % 6]; delta applied, 0 for an invalid or out-of-batch frame
    uint32_t dlen[6][kWave];
    uint8_t dst[6][kWave];           // bit 0 in batch, bit 1 invalid descriptor
};

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int o) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// The byte range a run streams: aligned start, step count, and whether the
// frames are packed enough to stream at all.
struct SplitSpan {
    uint64_t lo;
    uint32_t nsteps;
    bool dense;
};

template <int S>
__device__ __forceinline__ SplitSpan split_span(const SplitLds<S>& L, int db, int lane) {
    const uint64_t off = L.doff[db][lane];
    const uint32_t len = L.dlen[db][lane];
    const uint64_t base = off & ~15ull;
    const uint64_t span_b = len ? ((off + len + 15ull) & ~15ull) - base : 0ull;   // granule bytes
    uint64_t lo = len ? base : ~0ull, hi = len ? base + span_b : 0ull, tot = span_b;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const uint64_t l2 = shfl_xor_u64(lo, o), h2 = shfl_xor_u64(hi, o), t2 = shfl_xor_u64(tot, o);
        lo = l2 < lo ? l2 : lo;
        hi = h2 > hi ? h2 : hi;
        tot += t2;
    }
    lo = uniform_u64(lo);
    hi = uniform_u64(hi);
    tot = uniform_u64(tot);
    SplitSpan s;
    s.lo = lo;
    const bool any = hi > 0;
    s.dense = any && hi - lo <= tot + tot / 8 + 8192;
    s.nsteps = s.dense ? (uint32_t)((hi - lo + kStreamStep - 1) / kStreamStep) : 0u;
    return s;
}

template <int S, bool EXT>
__global__ __launch_bounds__(3 * kWave) void rx_split_kernel(RxArgs a) {
    constexpr int kSlot = SplitLds<S>::kSlot;
    constexpr int kWin = 128;
    __shared__ SplitLds<S> L;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);   // 0 streams, 1-2 parse
    const uint64_t nb = gridDim.x, b0 = blockIdx.x;
    const uint64_t K = a.nruns > b0 ? (a.nruns - b0 + nb - 1) / nb : 0;   // runs of this block: b0 + k nb
    const uint64_t NP = (K + 1) / 2;                                       // pairs of runs

    // Schedule, in periods p = 0..NP separated by block barriers: the streaming
    // wave streams the runs of pair p (2p, 2p+1); parsing wave j parses run
    // 2(p-1)+j, so each parse has two runs' streaming time; the parsing waves
    // commit the descriptors of pair p+2 (pairs 0 and 1 before period 0).
    if (wave != 0) {
        // ================= parsing wave j =================
        const uint64_t j = (uint64_t)(wave - 1);
        Counters C;
        // descriptors of run k: raw loads first (fetch), validated and written to
        // LDS later (commit), so the loads' latency hides under a parse and the
        // wait for them never includes this wave's column stores
        uint64_t r_off = 0;
        uint32_t r_len = 0;
        auto fetch = [&](uint64_t k) {
            const uint64_t f = (b0 + k * nb) * kWave + lane;
            r_off = 0;
            r_len = 0;
            if (f < a.n) {
                if (a.stride) {
                    r_off = a.first + f * a.stride;
                    r_len = a.frame_len;
                } else if (a.desc_compact) {
                    r_off = reinterpret_cast<const uint32_t*>(a.offsets)[f];
                    r_len = reinterpret_cast<const uint16_t*>(a.lengths)[f];
                } else {
                    r_off = a.offsets[f];
                    r_len = a.lengths[f];
                }
            }
        };
        auto commit = [&](uint64_t k) {
            const uint64_t f = (b0 + k * nb) * kWave + lane;
            const bool in_batch = f < a.n;
            const uint64_t off = r_off + a.delta;
            const bool bad = in_batch && (off > a.limit || (uint64_t)r_len > a.limit - off);
            const int db = (int)(k % 6);
            L.doff[db][lane] = in_batch && !bad ? off : 0ull;
            L.dlen[db][lane] = in_batch && !bad ? r_len : 0u;
            L.dst[db][lane] = (uint8_t)((in_batch ? 1 : 0) | (bad ? 2 : 0));
        };
        for (uint64_t k = j; k < 4 && k < K; k += 2) {   // pairs 0 and 1
            fetch(k);
            commit(k);
        }
        // the window (first 8 granules) of this lane's frame of the next run to
        // parse, loaded a period ahead into registers: the streaming wave
        // fetches these lines in the same period, so they are on-chip hits
        uint4 wv[8];
        auto load_window = [&](uint64_t k) {
            const int db = (int)(k % 6);
            const uint64_t o = L.doff[db][lane];
            const uint32_t n = L.dlen[db][lane];
            const uint32_t span = n ? ((uint32_t)(o & 15) + n + 15u) >> 4 : 0u;
            const uint8_t* fb = a.data + (o & ~15ull);
#pragma unroll
            for (int c = 0; c < 8; ++c) wv[c] = (uint32_t)c < span ? load16(fb + 16 * c) : make_uint4(0, 0, 0, 0);
        };
        if (j < K) load_window(j);
        __syncthreads();   // #0
        uint8_t* slot = L.win[j] + lane * kSlot;
        for (uint64_t p = 0; p <= NP; ++p) {
            const uint64_t r = 2 * p + j - 2;    // the run to parse (p >= 1)
            const uint64_t rc = 2 * p + 4 + j;   // the run whose descriptors to commit
            if (p == 0) {
                if (rc < K) {
                    fetch(rc);
                    commit(rc);
                }
            } else if (r < K) {
                const int db = (int)(r % 6);
                const uint64_t off = L.doff[db][lane];
                const uint32_t len = L.dlen[db][lane];
                const uint32_t stb = L.dst[db][lane];
#pragma unroll
                for (int c = 0; c < 8; ++c) {   // 132-B slots: dword stores
                    uint32_t* d = reinterpret_cast<uint32_t*>(slot + 16 * c);
                    d[0] = wv[c].x; d[1] = wv[c].y; d[2] = wv[c].z; d[3] = wv[c].w;
                }
                if (r + 2 < K) load_window(r + 2);
                if (rc < K) fetch(rc);
                const bool in_batch = (stb & 1u) != 0, desc_bad = (stb & 2u) != 0;
                const int sh = (int)(off & 15);
                const uint64_t base = off - (uint64_t)sh;
                const uint32_t fend = (uint32_t)sh + len;
#ifndef PNET_SPLIT_NOPARSE   // A/B: the parsing waves only keep pace
                Parsed P{};
                if (desc_bad) P.st = PNET_ST_DESC_INVALID;
                else if (in_batch)
                    P = parse_frame(FrameBytes{slot + sh, a.data + off, kWin - sh}, len, EXT ? a.flags : 0u);
                const int p0 = P.a_lo + sh, p1 = P.a_hi + sh, p2 = P.b_lo + sh, p3 = P.b_hi + sh;
                uint32_t tA = 0, tB = 0;
                window_sums(slot, p0, p1, min(p2, kWin), min(p3, kWin), tA, tB);
                if (P.l4do && p3 > kWin) {
                    // B past the window = the tail minus [kWin, p2) and [p3, fend)
                    tB += L.tail[r % 4][lane];
                    const uint8_t* fb = a.data + base;
                    if (p2 > kWin) tB -= lane_range_sum(fb, kWin, p2);
                    if ((uint32_t)p3 < fend) tB -= lane_range_sum(fb, p3, (int)fend);
                }
                uint32_t ipc = 0, l4c = 0;
                finalize(P, tA, tB, (off & 1) != 0, ipc, l4c);
#endif
                if (rc < K) commit(rc);   // into run r's descriptor buffer, read above
#ifndef PNET_SPLIT_NOPARSE
                const uint64_t f0 = (b0 + r * nb) * kWave;
                store_columns(a.cols, f0, lane, in_batch, P, ipc, l4c, slot, sh);
#ifndef PNET_NO_FIELD_COLUMNS
                if (EXT && a.field_cols && in_batch)
                    store_field_columns(a.cols, f0 + lane, P, FrameBytes{slot + sh, a.data + off, kWin - sh},
                                        a.l3mode);
#endif
                if (a.cols.counters) C.add(in_batch && !desc_bad, len, P.st);
#else
                (void)in_batch; (void)desc_bad; (void)base; (void)fend;
#endif
            }
            __syncthreads();   // #p+1
        }
        if (a.cols.counters) C.flush_wave(a.cols.counters, lane);
        return;
    }

    // ================= streaming wave (lane f <-> frame f of the run) =================
    __builtin_amdgcn_s_setprio(PNET_SPLIT_PRIO);   // its DMA issue comes before the parses' VALU work
    const uint64_t lim16 = a.limit >= 16 ? ((a.limit + 15) & ~15ull) - 16 : 0;   // last readable granule
    const uint32_t src_off = (uint32_t)(lane & ~3) * 16u + ((uint32_t)((lane & 3) - (lane >> 4)) & 3u) * 16u;
    const uint32_t ring0 = (uint32_t)(uintptr_t)(lds_ptr_t)&L.ring[0][0];
    __syncthreads();   // #0
    if (K) {
        SplitSpan cur = split_span(L, 0, lane);
        SplitSpan nxt = K > 1 ? split_span(L, 1, lane) : SplitSpan{0, 0, false};
        uint64_t k = 0;           // consumed run
        uint64_t ir = 0;          // run the issuer is in (k or k + 1)
        uint32_t ik = 0;          // its next step
        uint32_t icount = 0, ccount = 0;
        auto issue_step = [&](uint64_t sa) {
            const uint32_t dst = ring0 + (icount % S) * kStreamStep;
            if (sa + kStreamStep <= lim16 + 16) {
                const uint8_t* sp = a.data + sa;
#pragma unroll
                for (int i = 0; i < 4; ++i) glds16_nt_s(sp, src_off + 1024u * i, dst + 1024u * i);
            } else {   // the buffer's last step: granules past it re-read its last one
                const uint64_t sb = sa + src_off;
#pragma unroll
                for (int i = 0; i < 4; ++i) glds16_nt(a.data + min(sb + 1024u * i, lim16), dst + 1024u * i);
            }
            ++icount;
        };
        // keep S-1 steps in flight, within the consumed run and the next one
        auto issue_next = [&]() {
            if (ir == k) {
                if (ik < cur.nsteps) {
                    issue_step(cur.lo + (uint64_t)kStreamStep * ik);
                    ++ik;
                    return;
                }
                ir = k + 1;
                ik = 0;
            }
            if (ir == k + 1 && k + 1 < K && ik < nxt.nsteps) {
                issue_step(nxt.lo + (uint64_t)kStreamStep * ik);
                ++ik;
            }
        };
#pragma unroll 1
        for (int s = 0; s < S - 1; ++s) issue_next();

        for (;; ) {
            const int db = (int)(k % 6);
            const uint64_t off = L.doff[db][lane];
            const uint32_t len = L.dlen[db][lane];
            const uint64_t base = off & ~15ull;
            const uint32_t fend = (uint32_t)(off & 15) + len;
            const uint32_t span = len ? (fend + 15u) >> 4 : 0u;
            const bool has_tail = fend > (uint32_t)kWin;
            uint32_t tail = 0;
            if (cur.dense) {
                const uint64_t ts = base + kWin, te = base + 16ull * (span - 1u);
                uint32_t pts = 0, pte = 0;
                uint4 endg = make_uint4(0, 0, 0, 0);
                uint32_t pbase = 0;
                for (uint32_t s = 0; s < cur.nsteps; ++s) {
                    issue_next();
                    wait_steps<S - 1>((int)(icount - ccount - 1));
                    const uint8_t* ring = &L.ring[ccount % S][0];
                    ++ccount;
                    uint4 g[4];
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        g[c] = *reinterpret_cast<const uint4*>(ring + 64 * lane + 16 * ((c + (lane >> 2)) & 3));
                    uint32_t pre[4];
                    uint32_t t = 0;
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        pre[c] = t;
                        t = sad(g[c].w, sad(g[c].z, sad(g[c].y, sad(g[c].x, t))));
                    }
                    const uint32_t incl = wave_incl_scan(t);
                    const uint32_t excl = pbase + incl - t;
                    pbase += (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
                    L.ptab[lane] = make_uint4(excl + pre[0], excl + pre[1], excl + pre[2], excl + pre[3]);
                    wave_sync();
                    const uint64_t x0 = cur.lo + (uint64_t)kStreamStep * s;
                    const uint32_t* ptab = reinterpret_cast<const uint32_t*>(L.ptab);
                    // this frame's tail marks in the step (skipped wave-wide when
                    // no frame has one)
                    const uint64_t dts = ts - x0, dte = te - x0;
                    const bool cts = has_tail && dts < (uint64_t)kStreamStep;
                    const bool cte = has_tail && dte < (uint64_t)kStreamStep;
                    if (__ballot(cts || cte)) {
                        if (cts) pts = ptab[dts >> 4];
                        if (cte) {
                            // ring position of step granule gi: piece gi/4, granule gi%4 of it
                            const uint32_t gi = (uint32_t)(dte >> 4), pc = gi >> 2;
                            pte = ptab[gi];
                            endg = *reinterpret_cast<const uint4*>(ring + 16u * (4u * pc + (((gi & 3u) + (pc >> 2)) & 3u)));
                        }
                    }
                    wave_sync();   // the ring slot and the P table are rewritten by later steps
                }
                if (has_tail) {
                    const int e = (int)((fend - 1u) & 15u) + 1;   // frame bytes in its last granule
                    tail = pte - pts;
                    tail = sad(endg.x & first_bytes(clamp04(e)), tail);
                    tail = sad(endg.y & first_bytes(clamp04(e - 4)), tail);
                    tail = sad(endg.z & first_bytes(clamp04(e - 8)), tail);
                    tail = sad(endg.w & first_bytes(clamp04(e - 12)), tail);
                }
            } else if (has_tail) {
                // frames spread out: each lane sums its own tail
                tail = lane_range_sum(a.data + base, kWin, (int)fend);
            }
            L.tail[k % 4][lane] = tail;
            if ((k & 1) || k + 1 == K) __syncthreads();   // #p+1: pair p to the parsing waves
            if (++k == K) break;
            cur = nxt;
            if (ir < k) {   // the issuer had not reached run k (it never skips a run's steps)
                ir = k;
                ik = 0;
            }
            nxt = k + 1 < K ? split_span(L, (int)((k + 1) % 6), lane) : SplitSpan{0, 0, false};
        }
        wait_vm<0>();
    }
    __syncthreads();   // #NP+1: the last pair's parse
}

}  // namespace
}  // namespace pnetgpu
