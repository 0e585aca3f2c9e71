// rx_generic.h — rx_kernel, the generic receive kernel (descriptor mode, any alignment, any length; mixed / MTU / jumbo shapes)
// Part of the receive-path kernels; included once, by rx_kernel.hip (one
// translation unit, so every kernel still sees the shared device helpers inline).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pnetgpu.h"
#include "rx_internal.h"
#include "rx_common.h"
#include "rx_small.h"   // small_fast (short runs)

namespace pnetgpu {
namespace {

// ============================================================================
// rx_kernel: generic (descriptor mode, any alignment, any length).
// ============================================================================
template <int NW>
struct WaveLds {
    static constexpr int kSlot = NW * 16 + 4;   // +4 B pad: conflict-free parse reads
    uint8_t win[kWave * kSlot];
    uint64_t base[kWave];     // aligned byte offset of granule 0 of each frame
    uint32_t end[kWave];      // window granules to load; then slot-relative frame end
    uint32_t tail[kWave];     // weighted sum of the frame's bytes past the window
    uint8_t list[kWave];      // frames with bytes past the window (longest class first)
    uint32_t qhead;           // next list entry for a group that runs out of work
};

// Weighted sum of slot bytes [lo, hi) of a frame whose granule 0 is at fb, read
// from memory by one lane (the rare correction when the L4 range does not run
// from the window to the end of the frame).
__device__ __forceinline__ uint32_t lane_range_sum(const uint8_t* fb, int lo, int hi) {
    uint32_t acc = 0;
#pragma unroll 1
    for (int c = lo >> 4; 16 * c < hi; ++c) {
        const uint4 v = load16(fb + 16 * c);
        const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int p = 16 * c + 4 * t;
            acc = sad(dw[t] & first_bytes(clamp04(hi - p)) & ~first_bytes(clamp04(lo - p)), acc);
        }
    }
    return acc;
}

// The speculative tail: every byte of every frame past its window,
// [kWin, end), summed before the parse by groups of G lanes that stream
// coalesced granules (U loads in flight per lane); a group takes the next frame
// of the wave's list as soon as it finishes one. Sums land in L.tail.
// UNI (unified): the group streams the whole frame from granule 0 and writes
// granules 0..NW-1 into the frame's LDS slot itself (zeros past the frame's
// span) instead of a separate window phase: one pass per frame, so the line
// holding the window/tail boundary and the line shared with the next frame are
// fetched once, while they are still in L2 (the windows-first order read ~15 %
// more than the frame bytes on MTU frames: TCC_EA0_RDREQ, profiles/).
// DYN: a group that finishes a frame takes the next list entry from a shared
// LDS counter instead of a fixed stride of the list, and the list holds the
// frames needing more than one round first, so mixed sizes balance across the
// groups (the caller sets L.qhead = kWave / G).
// ALT (the unified MTU shape): odd frames are streamed from
// their last granule backward, so the line a frame's end shares with the next
// frame's start is read by both groups in the same round (even frame: its
// last round; odd frame: its last round, which then covers its start), instead
// of rounds apart (the second read then comes from L2, not HBM).
template <int NW, int G, int U, bool NT, bool UNI, bool DYN, bool ALT = false>
__device__ __forceinline__ void tail_sums(const uint8_t* data, WaveLds<NW>& L, int lane, int count
#ifdef PNET_WAVE_TIMES
                                          , uint64_t (&stat)[3]
#endif
) {
    constexpr int kGroups = kWave / G;
    constexpr int kSlot = WaveLds<NW>::kSlot;
    constexpr uint32_t c_first = UNI ? 0u : (uint32_t)NW;
    static_assert(!UNI || G * U >= NW, "the first round must cover the window");
    const int j = lane % G;
    int idx = lane / G;
    int fl = 0;
    uint32_t fe = 0, nneed = 0, c0 = 0, acc = 0;
    const uint8_t* fb = data;
    if (idx < count) {
        fl = L.list[idx];
        fe = L.end[fl];
        fb = data + L.base[fl];
        nneed = (fe + 15u) >> 4;
        c0 = c_first + j;
    }
#ifdef PNET_WAVE_TIMES
    uint32_t iters = 0, issued = 0;
#endif
    while (__ballot(idx < count)) {
#ifdef PNET_WAVE_TIMES
        ++iters;
        issued += (uint32_t)__popcll(__ballot(idx < count && j == 0));
#endif
        if (idx < count) {
            uint4 v[U];
            // ALT: odd frames' granule order reversed (UNI: c_first = 0)
            const bool rev = ALT && (fl & 1);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t cs = c0 + u * G;
                const uint32_t c = rev && cs < nneed ? nneed - 1u - cs : cs;
                v[u] = cs < nneed ? (NT ? load16_nt(fb + 16u * c) : load16(fb + 16u * c)) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t cs = c0 + u * G;
                // past the frame (cs >= nneed): the same zero granule either way
                const uint32_t c = rev && cs < nneed ? nneed - 1u - cs : cs;
                uint32_t x = v[u].x, y = v[u].y, z = v[u].z, w = v[u].w;
                if (UNI && c < (uint32_t)NW) {                   // window granule -> the frame's slot
                    uint32_t* dst = reinterpret_cast<uint32_t*>(L.win + fl * kSlot + 16 * c);
                    dst[0] = x; dst[1] = y; dst[2] = z; dst[3] = w;
                    continue;
                }
                const int hi = (int)fe - (int)(16u * c);
                if (hi < 16) {                                   // the frame's last granule
                    x &= first_bytes(clamp04(hi));
                    y &= first_bytes(clamp04(hi - 4));
                    z &= first_bytes(clamp04(hi - 8));
                    w &= first_bytes(clamp04(hi - 12));
                }
                acc = sad(x, acc);
                acc = sad(y, acc);
                acc = sad(z, acc);
                acc = sad(w, acc);
            }
            c0 += U * G;
            if (c0 - j >= (nneed > c_first ? nneed : c_first + 1u)) {   // group-uniform: frame done
#pragma unroll
                for (int o = G / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
                if (j == 0) L.tail[fl] = acc;
                acc = 0;
                if (DYN) {
                    uint32_t nidx = 0;
                    if (j == 0) nidx = atomicAdd(&L.qhead, 1u);
                    idx = __shfl((int)nidx, lane - j);
                } else {
                    idx += kGroups;
                }
                if (idx < count) {
                    fl = L.list[idx];
                    fe = L.end[fl];
                    fb = data + L.base[fl];
                    nneed = (fe + 15u) >> 4;
                    c0 = c_first + j;
                }
            }
        }
    }
#ifdef PNET_WAVE_TIMES
    stat[0] += issued;
    stat[1] += (uint64_t)iters * kGroups;
    stat[2] += (uint64_t)((issued + kGroups - 1) / kGroups) * kGroups;
#endif
}

// PASS: 0 = window phase for every frame, then the tails of the long ones;
// 1 = unified: every frame streamed once by the group loop (a hybrid - windows
// of short frames first, long frames unified - measured 5-15 % slower on IMIX).
// EXT: batch flags may be non-zero (VLAN / IPv6 extension dispatch) or
// header-field columns may be requested; the plain instantiation compiles the
// parse without those branches (half the code, SGPR spills 118 -> 14, IMIX -2 %).
constexpr uint32_t kUniMin = 768;     // every frame of such a run at least this long (PNETGPU_DESC_HINT_LARGE's bar)
constexpr uint32_t kJumboMin = 4096;  // and shorter than this; runs of frames all this long: the jumbo tail
template <int NW, int G, int U, bool NT, int PASS, bool DYN, bool EXT, bool TX>
__global__ __launch_bounds__(kBlock, NT ? kJumboWaves : (NW < 8 ? 5 : 4)) void rx_kernel(RxArgs a) {
    // the window must hold every field the parse reads near (Ethernet + 2 VLAN
    // tags + the fixed IPv4 header / IPv6 addresses: 82 B) after a 15-B shift
    static_assert(NW >= 7 || NW == 6, "window granules");
    static_assert(G == 2 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "tail group");
    constexpr int kSlot = WaveLds<NW>::kSlot;
    constexpr int kWin = NW * 16;
    // runs of short aligned frames take the small kernel's fast path (the
    // mixed shape's plain instantiation: no dispatch flags, header-field
    // columns or TX)
    constexpr bool kShortRuns = PASS == 0 && DYN && !EXT && !TX;
    // the short-run realignment reads slot dwords up to byte sh + 67 (sh <= 15)
    static_assert(!kShortRuns || kSlot >= 15 + 68, "short runs need a slot of at least 83 B");

    __shared__ WaveLds<NW> lds_all[kWavesPerBlock];
    __shared__ uint64_t blk_ctr[kWavesPerBlock][PNETGPU_NCOUNTERS];

    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    WaveLds<NW>& L = lds_all[wv];
    uint8_t* slot = L.win + lane * kSlot;
    Counters K;

    const uint64_t wave_stride = (uint64_t)gridDim.x * kWavesPerBlock;
    // descriptor-mode offset/length of this lane's frame, loaded one run ahead
    // so the descriptor round trip overlaps the previous run
    uint64_t d_off = 0;
    uint32_t d_len = 0;
    auto fetch_desc = [&](uint64_t r) {
        const uint64_t fr = r * kWave + lane;
        if (!a.stride && r < a.nruns && fr < a.n) {
            if (a.desc_compact) {   // wave-uniform
                d_off = reinterpret_cast<const uint32_t*>(a.offsets)[fr];
                d_len = reinterpret_cast<const uint16_t*>(a.lengths)[fr];
            } else {
                d_off = a.offsets[fr];
                d_len = a.lengths[fr];
            }
        }
    };
    PNET_WT_BEGIN;
    uint32_t run_count = 0;
    (void)run_count;
    // Deferred record stores (kDeferRuns): a small write stream inside a read
    // stream costs out of proportion to its bytes; the unified shape
    // keeps the last kDefer runs' records in registers (8 dwords per run) and
    // stores a run's record only when a newer one needs its place, or at the
    // wave's end - with the MTU shape's few runs per wave (4 at 2^20 frames),
    // the record stores of a launch then go out together at its end instead
    // of between reads. 1500-B batches -1.6 % at 3 runs (128 VGPRs, still 4
    // waves/SIMD); 1 or 2 runs measured even (profiles/r05/defer/).
    constexpr int kDefer = (PASS == 1 && !EXT && !TX) ? kDeferRuns : 0;
    constexpr int kDq = kDefer > 0 ? kDefer : 1;
    const bool defer = kDefer > 0 && !a.cols.src_ipv6 && !a.cols.dst_ipv6;
    Rec dq[kDq];
    uint64_t dqf[kDq];
    int dqn = 0;
    // TX (kTxDeferRuns): the in-place checksum writes of the last kTxDefer
    // runs held back the same way (frame offset, field positions, values: 4
    // dwords per run): 1500-B TX fill -1 % at 3 runs, same box, three
    // interleaved rounds (profiles/r05/defer/ab_tx_defer.txt)
    constexpr int kTxDefer = (PASS == 1 && TX) ? kTxDeferRuns : 0;
    constexpr int kTq = kTxDefer > 0 ? kTxDefer : 1;
    uint64_t tqo[kTq];
    uint32_t tqp[kTq], tqv[kTq];
    int tqn = 0;
    auto tx_flush = [&](uint64_t o, uint32_t pos, uint32_t v) {
        uint8_t* fr = const_cast<uint8_t*>(a.data) + o;
        const uint32_t ip = pos & 0xFFFFu, l4 = pos >> 16;
        if (ip != 0xFFFFu) {
            fr[ip] = (uint8_t)(v >> 8);
            fr[ip + 1] = (uint8_t)v;
        }
        if (l4 != 0xFFFFu) {
            fr[l4] = (uint8_t)(v >> 24);
            fr[l4 + 1] = (uint8_t)(v >> 16);
        }
    };
    RunQueue q(a.sched, a.nruns, (uint64_t)blockIdx.x * kWavesPerBlock + wv, wave_stride);
    uint64_t run = q.take();
    fetch_desc(run);
    while (run < a.nruns) {
        PNET_WT_RUN;
        // the MTU shape (4 runs per wave at 2^20 frames: too few to balance by
        // claims) rotates its issue priority per run: 1500-B batches -1.5 %,
        // same box, four interleaved rounds (profiles/r03/claims/ab_rotate.txt);
        // jumbo frames rotated per frame measured even, not done
        if (PASS == 1) rotate_prio(run_count++);
        const uint64_t nrun = q.take();   // the next run (its claim went out a run ago)
        // ---- 1. descriptor -------------------------------------------------
        const uint64_t f0 = run * kWave;
        const uint64_t f = f0 + lane;
        const bool in_batch = f < a.n;
        uint64_t off = 0;
        uint32_t len = 0;
        if (in_batch) {
            if (a.stride) {
                off = a.first + f * a.stride;
                len = a.frame_len;
            } else {
                off = d_off;
                len = d_len;
            }
            off += a.delta;
        }
        const bool desc_bad = in_batch && (off > a.limit || (uint64_t)len > a.limit - off);
        if (!in_batch || desc_bad) {   // nothing is loaded for it (a wild offset must not be dereferenced)
            len = 0;
            off = 0;
        }
        const int sh = (int)(off & 15);
        const uint64_t base = off - (uint64_t)sh;
        const uint32_t fend = (uint32_t)sh + len;            // slot-relative end of the frame
        const uint32_t span = (fend + 15u) >> 4;
        const bool long_frame = fend > (uint32_t)kWin;
        L.base[lane] = base;
        L.end[lane] = span < (uint32_t)NW ? span : (uint32_t)NW;   // granules to load into the window
        wave_sync();

        // short run (descriptor batches of minimum-size frames: the AF_PACKET /
        // ring hand-off of 64- or 60-B traffic): every frame at most 64 B, so no
        // tail phase; four granule loads per frame when none straddles a fifth
        // granule, and step 4 runs the small kernel's register fast path
        // (small_fast: compile-time field positions) on the frame's 64 bytes
        // realigned from its slot, parse_frame only for the frames it leaves
        // (IPv6, IPv4 options). Descriptor 64-B batches -16 %, IMIX even
        // (profiles/r03/short_runs/).
        const bool short_run = kShortRuns && __ballot(in_batch && !desc_bad && len > 64u) == 0ull;
        const bool four = short_run && __ballot(span > 4u) == 0ull;
        // a run of large frames in the mixed shape (a descriptor batch of
        // MTU-size traffic without PNETGPU_DESC_HINT_LARGE, or a burst of it
        // inside a mix): each frame streamed once in the MTU shape's unified
        // order instead of window first, then tail
        constexpr bool kUniRuns = PASS == 0 && DYN;
        const bool uni = kUniRuns && __ballot(in_batch && (desc_bad || len < kUniMin || len >= kJumboMin)) == 0ull;
        // and a run of jumbo frames (every frame >= 4 KiB): the jumbo shape's
        // tail, one frame per wave round
        const bool jrun = kUniRuns && !uni &&
                          __ballot(in_batch && (desc_bad || len < kJumboMin)) == 0ull;
        // such runs rotate their issue priority as the MTU shape does: no-hint
        // 1500-B batches -2.6 %, IMIX even (profiles/r05/uni_runs/ab_rotate.txt)
        if (kUniRuns && uni) rotate_prio(run_count++);

        // ---- 2. window: NW*64 granule loads, all in flight before any store --
        if (kShortRuns && four) {   // wave-uniform: 4 granules per frame
            uint4 g[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int q = i * kWave + lane;
                const int fl = q >> 2, c = q & 3;
                g[i] = make_uint4(0, 0, 0, 0);
                if ((uint32_t)c < L.end[fl])
                    g[i] = load16_nt(a.data + L.base[fl] + 16u * c);
            }
            fetch_desc(nrun);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int q = i * kWave + lane;
                uint32_t* dst = reinterpret_cast<uint32_t*>(L.win + (q >> 2) * kSlot + 16 * (q & 3));
                dst[0] = g[i].x; dst[1] = g[i].y; dst[2] = g[i].z; dst[3] = g[i].w;
            }
        } else if (PASS != 1 && !uni) {
            uint4 g[NW];
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int q = i * kWave + lane;
                const int fl = q / NW, c = q % NW;
                g[i] = make_uint4(0, 0, 0, 0);
                if ((uint32_t)c < L.end[fl])
                    g[i] = load16(a.data + L.base[fl] + 16u * c);
            }
            fetch_desc(nrun);
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int q = i * kWave + lane;
                const int fl = q / NW, c = q % NW;
                uint32_t* dst = reinterpret_cast<uint32_t*>(L.win + fl * kSlot + 16 * c);
                dst[0] = g[i].x; dst[1] = g[i].y; dst[2] = g[i].z; dst[3] = g[i].w;
            }
        } else {
            fetch_desc(nrun);
        }

        PNET_PH(0);   // probe: descriptors + window (its loads complete at the LDS stores)
        // ---- 3. speculative tail: all frame bytes past the window ----------
        // Summed before the parse (no parse state is live, so more loads fit in
        // flight); the parse then trims it to the L4 range B, which in every
        // well-formed frame already runs to the end of the frame. Unified pass:
        // the group loop also fills the window of every frame.
        const bool has_tail = (PASS == 1 || uni) ? in_batch : long_frame;
        const uint64_t tmask = __ballot(has_tail);
        if (tmask) {
            // DYN: frames needing more than one group round go first
            const bool big = DYN && has_tail && span > (uint32_t)(NW + G * U);
            const uint64_t bmask = __ballot(big);
            const uint64_t below = (1ull << lane) - 1ull;
            if (has_tail) {
                const int pos = big ? __popcll(bmask & below) : __popcll(bmask) + __popcll(tmask & ~bmask & below);
                L.list[pos] = (uint8_t)lane;
                L.end[lane] = fend;
            }
            if (DYN && lane == 0) L.qhead = kWave / G;
            wave_sync();
            if (kUniRuns && uni)   // the MTU shape's tail configuration (PNET_MTU_CFG)
                tail_sums<NW, 8, 4, false, true, false, true>(a.data, L, lane, __popcll(tmask) PNET_TAIL_STAT);
            else if (kUniRuns && jrun)   // the jumbo shape's (PNET_JUMBO_CFG)
                tail_sums<NW, 64, (TX && EXT ? 8 : kMixedJumboU), true, false, false>(
                    a.data, L, lane, __popcll(tmask) PNET_TAIL_STAT);
            else
                tail_sums<NW, G, U, NT, (PASS != 0), DYN, (PASS == 1 && !DYN)>(
                    a.data, L, lane, __popcll(tmask) PNET_TAIL_STAT);
        }
        wave_sync();

        PNET_PH(1);   // probe: tail phase
        // ---- 4. parse + window sums (lane l <-> frame l) -------------------
        Parsed P{};
        uint32_t ipc = 0, l4c = 0;
        bool fast_done = false;
        if (kShortRuns && short_run && in_batch && !desc_bad) {
            // the frame's bytes [0, 64) from slot byte sh on (sh + 68 <= kSlot)
            const uint32_t* s32 = reinterpret_cast<const uint32_t*>(slot) + (sh >> 2);
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) w[k] = __builtin_amdgcn_alignbyte(s32[k + 1], s32[k], (uint32_t)(sh & 3));
            fast_done = !small_fast(w, len, P, ipc, l4c);
        }
        if (!fast_done) {
            P = Parsed{};
            if (desc_bad) P.st = PNET_ST_DESC_INVALID;
            else if (in_batch)
                P = parse_frame(FrameBytes{slot + sh, a.data + off, kWin - sh}, len, EXT ? a.flags : 0u);
            // A (<= 97 B into the frame) lies in the window unless the window is
            // shorter than 8 granules (IPv4 options past it); B may run past it
            const int p0 = P.a_lo + sh, p1 = P.a_hi + sh, p2 = P.b_lo + sh, p3 = P.b_hi + sh;
            uint32_t tA = 0, tB = 0;
            window_sums(slot, p0, min(p1, kWin), min(p2, kWin), min(p3, kWin), tA, tB);
            if (NW < 8 && p1 > kWin) tA += lane_range_sum(a.data + base, kWin, p1);
            if (P.l4do && p3 > kWin) {
                // B past the window = the speculative tail minus [kWin, p2) and [p3, fend)
                tB += L.tail[lane];
                const uint8_t* fb = a.data + base;
                if (p2 > kWin) tB -= lane_range_sum(fb, kWin, p2);
                if ((uint32_t)p3 < fend) tB -= lane_range_sum(fb, p3, (int)fend);
            }

            // ---- 5. finalize + stores --------------------------------------
            ipc = 0;
            l4c = 0;
            finalize(P, tA, tB, (off & 1) != 0, ipc, l4c);
        }
        PNET_PH(2);   // probe: parse, window sums, tail trims, finalize
        if (kTxDefer > 0) {
            // field offsets fit 16 bits: they lie within the first ~8.4 KB of a frame
            // (two VLAN tags, four IPv6 extension headers of at most 2 KB)
            const bool v4 = TX && in_batch && !desc_bad && P.is_v4;
            const bool l4 = TX && in_batch && !desc_bad && (P.st & PNET_ST_L4_CSUM_DONE);
            const uint32_t pos = (v4 ? (P.l3 + 10u) & 0xFFFFu : 0xFFFFu) | ((l4 ? (uint32_t)P.l4csum_at : 0xFFFFu) << 16);
            const uint32_t val = (ipc & 0xFFFFu) | (l4c << 16);
            if (tqn == kTxDefer) tx_flush(tqo[kTq - 1], tqp[kTq - 1], tqv[kTq - 1]);
#pragma unroll
            for (int k = kTq - 1; k > 0; --k) {
                tqo[k] = tqo[k - 1];
                tqp[k] = tqp[k - 1];
                tqv[k] = tqv[k - 1];
            }
            tqo[0] = off;
            tqp[0] = pos;
            tqv[0] = val;
            tqn = tqn < kTxDefer ? tqn + 1 : kTxDefer;
        } else if (TX && in_batch && !desc_bad) {
            tx_write(const_cast<uint8_t*>(a.data) + off, P, ipc, l4c);
        }
        if (kDefer > 0 && defer) {
            const Rec cur = pack_rec(P, ipc, l4c);
            if (dqn == kDefer) store_rec(a.cols, dqf[kDq - 1], lane, dqf[kDq - 1] + lane < a.n, dq[kDq - 1]);
#pragma unroll
            for (int k = kDq - 1; k > 0; --k) {
                dq[k] = dq[k - 1];
                dqf[k] = dqf[k - 1];
            }
            dq[0] = cur;
            dqf[0] = f0;
            dqn = dqn < kDefer ? dqn + 1 : kDefer;
        } else {
            store_columns(a.cols, f0, lane, in_batch, P, ipc, l4c, slot, sh);
        }
        if (EXT && a.field_cols && in_batch)   // header-field columns: EXT instantiations only
            store_field_columns(a.cols, f0 + lane, P, FrameBytes{slot + sh, a.data + off, kWin - sh}, EXT && a.l3mode);
        if (a.cols.counters) K.add(in_batch && !desc_bad, len, P.st);
        wave_sync();   // slots and lists are rewritten by the next run
        PNET_PH(3);   // probe: stores, counters
        run = nrun;
    }
    if (kTxDefer > 0) {
#pragma unroll
        for (int k = 0; k < kTq; ++k)
            if (k < tqn) tx_flush(tqo[k], tqp[k], tqv[k]);
    }
    if (kDefer > 0) {
#pragma unroll
        for (int k = 0; k < kDq; ++k)
            if (k < dqn) store_rec(a.cols, dqf[k], lane, dqf[k] + lane < a.n, dq[k]);
    }
    if (a.cols.counters) K.flush(a.cols.counters, blk_ctr, wv, lane);
    PNET_WT_END((uint64_t)blockIdx.x * kWavesPerBlock + wv);
}

}  // namespace
}  // namespace pnetgpu
