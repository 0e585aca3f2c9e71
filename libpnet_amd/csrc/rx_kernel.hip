// rx_kernel.hip — MI355X (gfx950) receive-path kernels: Ethernet/IPv4/IPv6
// parse + ones-complement checksums (UDP/TCP/ICMP/ICMPv6) for a batch of frames.
//
// What it computes is libpnet's per-frame receive chain (examples/packetdump.rs:120-217
// over pnet_packet's views and checksums, pnet_packet/src/util.rs:76-181); see
// include/pnetgpu.h for the exact contract and DESIGN.md for the layout.
//
// Execution model (one wavefront = 64 lanes owns a run of 64 consecutive frames):
//   1. descriptor : lane l computes frame l's (offset, length).
//   2. window     : the wave loads the first NW aligned 16-B granules of each of
//                   its 64 frames (NW*64 coalesced global_load_dwordx4, all issued
//                   before any is consumed) into a wave-private LDS slot per frame.
//   3. parse      : lane l parses frame l out of its LDS slot (byte reads, padded
//                   slots => conflict-free) and derives the two checksum ranges.
//   4. window sum : lane l sums its frame's window bytes under byte masks into two
//                   u32 accumulators with v_sad_u16 (one op per dword).
//   5. tail       : frames longer than the window are summed by groups of G lanes
//                   streaming coalesced 16-B granules straight from HBM, reduced
//                   with cross-lane shuffles, handed back through LDS.
//   6. finalize   : fold, byte-order fix-up, pseudo-header, compare, coalesced SoA
//                   stores; per-wave ballot counters, one atomic set per block.
//
// Checksum arithmetic (why the sums are bit-exact without byte swapping loads):
//   The reference sums big-endian 16-bit words relative to the start of the slice
//   (util.rs:158-181) into an exact u32 and folds with end-around carry. The fold
//   depends only on the sum mod 0xFFFF and on whether it is zero. Summing the
//   little-endian halves of aligned dwords weights byte b at absolute address a by
//   256^(a&1); since 65536 == 1 (mod 0xFFFF) that equals the BE weight up to one
//   factor 256, i.e. a byte swap of the folded result when the slice starts at an
//   even absolute address (every range here starts at an even frame offset, so
//   parity = frame offset parity). All partial sums are exact non-negative
//   integers, so "zero iff every in-range byte is zero" is preserved too.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pnetgpu.h"
#include "rx_internal.h"

namespace pnetgpu {

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

__device__ __forceinline__ uint32_t fold16(uint32_t x) {
    x = (x & 0xFFFFu) + (x >> 16);
    x = (x & 0xFFFFu) + (x >> 16);
    return x;
}
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }
// mask of the first x bytes of a dword, x in [0, 4]
__device__ __forceinline__ uint32_t first_bytes(int x) {
    return (uint32_t)(0xFFFFFFFFull >> (32 - 8 * x));
}
__device__ __forceinline__ int clamp04(int v) { return min(max(v, 0), 4); }
// LE 16-bit halves of d added to acc (v_sad_u16 with a zero operand)
__device__ __forceinline__ uint32_t sad(uint32_t d, uint32_t acc) {
    return __builtin_amdgcn_sad_u16(d, 0u, acc);
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t ld8(const uint8_t* w, int p) { return w[p]; }
__device__ __forceinline__ uint32_t ld16be(const uint8_t* w, int p) { return (ld8(w, p) << 8) | ld8(w, p + 1); }
__device__ __forceinline__ uint32_t ld32be(const uint8_t* w, int p) { return (ld16be(w, p) << 16) | ld16be(w, p + 2); }

// 16 bytes of a frame-relative run [p, p+16) read from an LDS slot at any
// alignment, as 4 little-endian dwords (memory order).
__device__ __forceinline__ uint4 lds_read16_unaligned(const uint8_t* slot, int p) {
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(slot);
    int q = p >> 2, sh = (p & 3);
    uint32_t d0 = s32[q], d1 = s32[q + 1], d2 = s32[q + 2], d3 = s32[q + 3], d4 = s32[q + 4];
    uint4 r;
    r.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
    r.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
    r.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
    r.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
    return r;
}

// Per-wave LDS: 64 frame slots of NW granules (+4 B pad so lane l's byte p sits
// in bank (l*SLOT/4 + p/4) % 32: conflict-free for the parse reads), plus the
// per-frame hand-off words used by the tail phase.
template <int NW>
struct WaveLds {
    static constexpr int kSlot = NW * 16 + 4;
    uint8_t  win[kWave * kSlot];
    uint64_t base[kWave];     // aligned byte offset of granule 0 of each frame
    uint32_t end[kWave];      // slot-relative end of the summed range
    uint32_t tail[kWave];     // tail-phase partial sum per frame
};

template <int NW, int G>
__global__ __launch_bounds__(kBlock) void rx_kernel(RxArgs a) {
    static_assert(NW == 4 || NW == 8, "window granules");
    static_assert(G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "tail group");
    constexpr int kSlot = WaveLds<NW>::kSlot;
    constexpr int kWin = NW * 16;           // window bytes per frame
    constexpr int kFps = kWave / G;         // frames per tail set

    __shared__ WaveLds<NW> lds_all[kWavesPerBlock];
    __shared__ uint64_t blk_ctr[kWavesPerBlock][PNETGPU_NCOUNTERS];

    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    WaveLds<NW>& L = lds_all[wv];
    uint8_t* slot = L.win + lane * kSlot;

    uint32_t c_frames = 0, c_v4 = 0, c_v6 = 0, c_ipbad = 0, c_l4bad = 0, c_malf = 0, c_unk = 0;
    uint64_t c_bytes = 0;

    const uint64_t wave_stride = (uint64_t)gridDim.x * kWavesPerBlock;
    for (uint64_t run = (uint64_t)blockIdx.x * kWavesPerBlock + wv; run < a.nruns; run += wave_stride) {
        // ---- 1. descriptor -------------------------------------------------
        const uint64_t f = run * kWave + lane;
        const bool in_batch = f < a.n;
        uint64_t off = 0;
        uint32_t len = 0;
        if (in_batch) {
            if (a.stride) {
                off = a.first + f * a.stride;
                len = a.frame_len;
            } else {
                off = a.offsets[f];
                len = a.lengths[f];
            }
            off += a.delta;
        }
        const bool desc_bad = in_batch && (off > a.limit || (uint64_t)len > a.limit - off);
        if (!in_batch || desc_bad) len = 0;
        const int sh = (int)(off & 15);
        const uint64_t base = off - (uint64_t)sh;
        const uint32_t span = len ? (uint32_t)((sh + (uint64_t)len + 15) >> 4) : 0u;
        const uint32_t nwin = span < (uint32_t)NW ? span : (uint32_t)NW;
        L.base[lane] = base;
        L.end[lane] = nwin;   // temporarily: granules to load into the window
        wave_sync();

        // ---- 2. window: NW*64 granule loads, all in flight before any store --
        uint4 g[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int q = i * kWave + lane;
            const int fl = q / NW, c = q % NW;
            g[i] = make_uint4(0, 0, 0, 0);
            if ((uint32_t)c < L.end[fl]) {
                g[i] = *reinterpret_cast<const uint4*>(a.data + L.base[fl] + 16u * c);
            }
        }
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            const int q = i * kWave + lane;
            const int fl = q / NW, c = q % NW;
            uint32_t* dst = reinterpret_cast<uint32_t*>(L.win + fl * kSlot + 16 * c);
            dst[0] = g[i].x; dst[1] = g[i].y; dst[2] = g[i].z; dst[3] = g[i].w;
        }
        wave_sync();

        // ---- 3. parse (lane l <-> frame l) ---------------------------------
        const uint8_t* W = slot + sh;
        uint32_t st = 0, et = 0, proto = 0, ttl = 0, l4off = 0, l4len = 0, sp = 0, dp = 0;
        uint32_t s4 = 0, d4 = 0, ipstored = 0, l4stored = 0, pseudo = 0;
        int r0 = 0, m = 0, e = 0;      // frame-relative range bounds: A=[r0,m), B=[m,e)
        int l4skip_at = 0;
        bool is_v4 = false, l4do = false, v6pseudo = false;
        if (desc_bad) {
            st = PNET_ST_DESC_INVALID;
        } else if (in_batch) {
            if (len < 14) {
                st = PNET_ST_ETH_MALFORMED;               // EthernetPacket::new == None
            } else {
                et = ld16be(W, 12);
                const uint32_t eplen = len - 14;          // Ethernet payload: unbounded
                bool l3ok = false, has_l4 = false, v6 = false;
                uint32_t l4s = 0;
                if (et == 0x0800u) {
                    st |= PNET_ST_L3_IPV4;
                    if (eplen < 20) {
                        st |= PNET_ST_L3_MALFORMED;
                    } else {
                        l3ok = true;
                        is_v4 = true;
                        const uint32_t ihl4 = (ld8(W, 14) & 15u) * 4u;
                        // ipv4.rs:169-175 clamp to [20, packet().len()]
                        const uint32_t hl = min(max(ihl4, 20u), eplen);
                        const uint32_t tl = ld16be(W, 16);
                        ttl = ld8(W, 22);
                        proto = ld8(W, 23);
                        ipstored = ld16be(W, 24);
                        s4 = ld32be(W, 26);
                        d4 = ld32be(W, 30);
                        r0 = 14;
                        m = 14 + (int)hl;
                        // decorator.rs:728-753 with ipv4.rs:226-243
                        const uint32_t start = max(20u, ihl4);
                        const uint32_t plen = tl > ihl4 ? tl - ihl4 : 0u;
                        if (eplen > start) {
                            has_l4 = true;
                            l4s = 14 + start;
                            l4len = min(start + plen, eplen) - start;
                        }
                    }
                } else if (et == 0x86DDu) {
                    st |= PNET_ST_L3_IPV6;
                    if (eplen < 40) {
                        st |= PNET_ST_L3_MALFORMED;
                    } else {
                        l3ok = true;
                        v6 = true;
                        proto = ld8(W, 20);
                        ttl = ld8(W, 21);
                        const uint32_t pl = ld16be(W, 18);
                        if (eplen > 40) {                  // ipv6.rs:34-36 #[length = "payload_length"]
                            has_l4 = true;
                            l4s = 54;
                            l4len = min(40u + pl, eplen) - 40u;
                        }
                    }
                } else {
                    st |= PNET_ST_UNKNOWN_ETHERTYPE;
                }
                if (has_l4) l4off = l4s;
                if (l3ok) {
                    uint32_t kind = 0, minlen = 0;
                    int soff = 0;
                    switch (proto) {
                        case 17: kind = PNET_ST_L4_UDP; minlen = 8; soff = 6; break;
                        case 6: kind = PNET_ST_L4_TCP; minlen = 20; soff = 16; break;
                        case 1: kind = PNET_ST_L4_ICMP; minlen = 4; soff = 2; break;
                        case 58: kind = PNET_ST_L4_ICMPV6; minlen = 4; soff = 2; break;
                        default: break;
                    }
                    if (!kind) {
                        st |= PNET_ST_UNKNOWN_PROTO;
                    } else {
                        st |= kind;
                        if (l4len < minlen) {
                            st |= PNET_ST_L4_MALFORMED;
                        } else {
                            const int p = (int)l4s;
                            sp = ld16be(W, p);
                            if (proto == 17 || proto == 6) dp = ld16be(W, p + 2);
                            else dp = l4len >= 8 ? ld16be(W, p + 4) : 0u;
                            l4skip_at = p + soff;
                            l4stored = ld16be(W, l4skip_at);
                            if (proto == 1) {                       // icmp::checksum: no pseudo-header
                                l4do = true;
                                if (v6) { r0 = 54; m = 54; }
                            } else if (v6) {                        // util::ipv6_checksum
                                l4do = true;
                                v6pseudo = true;
                                r0 = 22; m = 54;                   // pseudo-header address bytes
                                pseudo = proto + l4len;
                            } else if (proto != 58) {               // util::ipv4_checksum
                                l4do = true;
                                pseudo = (s4 >> 16) + (s4 & 0xFFFFu) + (d4 >> 16) + (d4 & 0xFFFFu) +
                                         proto + l4len;
                            }
                            if (l4do) e = p + (int)l4len;           // B = [l4s, l4s+len), l4s == m
                        }
                    }
                }
                if (!is_v4 && !l4do) { r0 = 0; m = 0; e = 0; }
                if (is_v4 && !l4do) e = m;
            }
        }

        // ---- 4. window sums: A=[r0,m), B=[m,min(e,win)) in slot coordinates --
        const int rs = r0 ? r0 + sh : 0;
        const int ms = m ? m + sh : 0;
        const int es = e ? e + sh : ms;
        const int ew = min(es, kWin);
        uint32_t tA = 0, tB = 0;
        {
            const uint32_t* s32 = reinterpret_cast<const uint32_t*>(slot);
#pragma unroll
            for (int k = 0; k < NW * 4; ++k) {
                const uint32_t d = s32[k];
                const int t = 4 * k;
                const uint32_t f0 = first_bytes(clamp04(rs - t));
                const uint32_t f1 = first_bytes(clamp04(ms - t));
                const uint32_t f2 = first_bytes(clamp04(ew - t));
                tA = sad(d & f1 & ~f0, tA);
                tB = sad(d & f2 & ~f1, tB);
            }
        }

        // ---- 5. tail: granules [NW, ceil(es/16)) by groups of G lanes ------
        const uint64_t need_tail = __ballot(es > kWin);
        if (need_tail) {
            L.end[lane] = (uint32_t)es;
            wave_sync();
            const int j = lane % G;
#pragma unroll 1
            for (int s = 0; s < G; ++s) {
                const uint64_t setmask = (kFps == 64 ? ~0ull : ((1ull << kFps) - 1ull)) << (s * kFps);
                if (!(need_tail & setmask)) continue;      // wave-uniform
                const int fl = s * kFps + lane / G;
                const uint32_t fe = L.end[fl];
                const uint8_t* fb = a.data + L.base[fl];
                const uint32_t nneed = (fe + 15u) >> 4;
                uint32_t acc = 0;
                constexpr int U = 4;
#pragma unroll 1
                for (uint32_t c0 = NW + j; c0 < nneed; c0 += U * G) {
                    uint4 v[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t c = c0 + u * G;
                        v[u] = c < nneed ? *reinterpret_cast<const uint4*>(fb + 16u * c) : make_uint4(0, 0, 0, 0);
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int p = (int)(16u * (c0 + u * G));
                        const uint32_t dw[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
                        for (int t = 0; t < 4; ++t) acc = sad(dw[t] & first_bytes(clamp04((int)fe - p - 4 * t)), acc);
                    }
                }
#pragma unroll
                for (int o = G / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
                if (j == 0) L.tail[fl] = acc;
            }
            wave_sync();
            if (es > kWin) tB += L.tail[lane];
        }

        // ---- 6. finalize ---------------------------------------------------
        const bool odd = (off & 1) != 0;
        uint32_t ipc = 0, l4c = 0;
        if (is_v4) {
            tA -= odd ? ipstored : bswap16(ipstored);      // skipword 5 (ipv4.rs:177)
        }
        if (l4do) {
            tB -= odd ? l4stored : bswap16(l4stored);      // skipword 3 / 8 / 1
        }
        uint32_t pA = fold16(tA), pB = fold16(tB);
        if (!odd) { pA = bswap16(pA); pB = bswap16(pB); }
        if (is_v4) {
            ipc = (~pA) & 0xFFFFu;
            if (ipc == ipstored) st |= PNET_ST_IP_CSUM_OK;
        }
        if (l4do) {
            const uint32_t sum = pB + pseudo + (v6pseudo ? pA : 0u);
            l4c = (~fold16(sum)) & 0xFFFFu;
            st |= PNET_ST_L4_CSUM_DONE;
            if (l4c == l4stored) st |= PNET_ST_L4_CSUM_OK;
        }

        if (in_batch) {
            const pnetgpu_rx_columns& C = a.cols;
            if (C.status) C.status[f] = (uint16_t)st;
            if (C.ip_csum) C.ip_csum[f] = (uint16_t)ipc;
            if (C.l4_csum) C.l4_csum[f] = (uint16_t)l4c;
            if (C.ethertype) C.ethertype[f] = (uint16_t)et;
            if (C.ip_proto) C.ip_proto[f] = (uint8_t)proto;
            if (C.ttl) C.ttl[f] = (uint8_t)ttl;
            if (C.l4_offset) C.l4_offset[f] = (uint16_t)l4off;
            if (C.l4_length) C.l4_length[f] = (uint16_t)l4len;
            if (C.src_port) C.src_port[f] = (uint16_t)sp;
            if (C.dst_port) C.dst_port[f] = (uint16_t)dp;
            if (C.src_ipv4) C.src_ipv4[f] = s4;
            if (C.dst_ipv4) C.dst_ipv4[f] = d4;
            if (C.src_ipv6 || C.dst_ipv6) {
                const bool v6ok = (st & (PNET_ST_L3_MASK | PNET_ST_L3_MALFORMED)) == PNET_ST_L3_IPV6;
                uint4 sv = make_uint4(0, 0, 0, 0), dv = make_uint4(0, 0, 0, 0);
                if (v6ok) {
                    sv = lds_read16_unaligned(slot, sh + 22);
                    dv = lds_read16_unaligned(slot, sh + 38);
                }
                if (C.src_ipv6) reinterpret_cast<uint4*>(C.src_ipv6)[f] = sv;
                if (C.dst_ipv6) reinterpret_cast<uint4*>(C.dst_ipv6)[f] = dv;
            }
        }
        if (a.cols.counters) {
            c_frames += (uint32_t)__popcll(__ballot(in_batch && !desc_bad));
            c_bytes += len;
            c_v4 += (uint32_t)__popcll(__ballot((st & PNET_ST_L3_MASK) == PNET_ST_L3_IPV4));
            c_v6 += (uint32_t)__popcll(__ballot((st & PNET_ST_L3_MASK) == PNET_ST_L3_IPV6));
            c_ipbad += (uint32_t)__popcll(__ballot(is_v4 && !(st & PNET_ST_IP_CSUM_OK)));
            c_l4bad += (uint32_t)__popcll(__ballot(l4do && !(st & PNET_ST_L4_CSUM_OK)));
            c_malf += (uint32_t)__popcll(__ballot((st & (PNET_ST_ETH_MALFORMED | PNET_ST_L3_MALFORMED |
                                                         PNET_ST_L4_MALFORMED | PNET_ST_DESC_INVALID)) != 0));
            c_unk += (uint32_t)__popcll(__ballot((st & (PNET_ST_UNKNOWN_ETHERTYPE | PNET_ST_UNKNOWN_PROTO)) != 0));
        }
        wave_sync();   // slots are rewritten by the next run
    }

    if (a.cols.counters) {
        // bytes: per-lane u64 -> wave sum; the ballot counters are already wave-uniform
        for (int o = 32; o >= 1; o >>= 1) {
            uint32_t lo = (uint32_t)c_bytes, hi = (uint32_t)(c_bytes >> 32);
            lo = __shfl_xor(lo, o);
            hi = __shfl_xor(hi, o);
            c_bytes += ((uint64_t)hi << 32) | lo;
        }
        if (lane == 0) {
            blk_ctr[wv][PNETGPU_CTR_FRAMES] = c_frames;
            blk_ctr[wv][PNETGPU_CTR_BYTES] = c_bytes;
            blk_ctr[wv][PNETGPU_CTR_IPV4] = c_v4;
            blk_ctr[wv][PNETGPU_CTR_IPV6] = c_v6;
            blk_ctr[wv][PNETGPU_CTR_IP_CSUM_BAD] = c_ipbad;
            blk_ctr[wv][PNETGPU_CTR_L4_CSUM_BAD] = c_l4bad;
            blk_ctr[wv][PNETGPU_CTR_MALFORMED] = c_malf;
            blk_ctr[wv][PNETGPU_CTR_UNKNOWN] = c_unk;
        }
        __syncthreads();
        if (threadIdx.x < PNETGPU_NCOUNTERS) {
            uint64_t v = 0;
            for (int w = 0; w < kWavesPerBlock; ++w) v += blk_ctr[w][threadIdx.x];
            if (v) atomicAdd(reinterpret_cast<unsigned long long*>(a.cols.counters + threadIdx.x),
                             (unsigned long long)v);
        }
    }
}

// ---------------------------------------------------------------------------
// Batched util::checksum / ipv4_checksum / ipv6_checksum over slices.
// One group of 16 lanes per slice (4 slices per wave per step): coalesced
// 16-B granules, masked sums, shuffle reduce, lane 0 of the group finalizes.
// PSEUDO: 0 = util::checksum, 4 = ipv4_checksum, 16 = ipv6_checksum.
template <int PSEUDO>
__global__ __launch_bounds__(kBlock) void slice_kernel(SliceArgs a) {
    constexpr int G = 16;
    const int lane = threadIdx.x & (kWave - 1);
    const int j = lane % G;
    const uint64_t gid = ((uint64_t)blockIdx.x * kBlock + threadIdx.x) / G;
    const uint64_t ngroups = (uint64_t)gridDim.x * kBlock / G;
    // groups are 16-lane aligned, so every shuffle below stays inside one group,
    // whose lanes share i (and therefore control flow)
    for (uint64_t i = gid; i < a.n; i += ngroups) {
        const bool active = true;
        uint64_t off = 0;
        uint32_t len = 0, skip = 0xFFFFFFFFu;
        if (active) {
            off = a.offsets[i] + a.delta;
            len = a.lengths[i];
            skip = a.skipwords[i];
        }
        const bool bad = active && (off > a.limit || (uint64_t)len > a.limit - off);
        if (bad) len = 0;
        const int sh = (int)(off & 15);
        const uint8_t* fb = a.data + (off - (uint64_t)sh);
        const int e = sh + (int)len;
        const uint32_t nneed = len ? (uint32_t)((e + 15) >> 4) : 0u;
        uint32_t acc = 0;
#pragma unroll 1
        for (uint32_t c = j; c < nneed; c += G) {
            const uint4 v = *reinterpret_cast<const uint4*>(fb + 16u * c);
            const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
            const int p = (int)(16u * c);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const uint32_t mk = first_bytes(clamp04(e - p - 4 * t)) & ~first_bytes(clamp04(sh - p - 4 * t));
                acc = sad(dw[t] & mk, acc);
            }
        }
#pragma unroll
        for (int o = G / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        if (j == 0 && active) {
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
                s += a.protos[i] + len + p;
                r = (~fold16(s)) & 0xFFFFu;
            }
            a.out[i] = (uint16_t)r;
        }
    }
}

template <int NW, int G>
int launch_rx_t(const RxArgs& args, int blocks, hipStream_t stream) {
    hipLaunchKernelGGL((rx_kernel<NW, G>), dim3(blocks), dim3(kBlock), 0, stream, args);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

int rx_blocks_per_cu(int nw, int g) {
    int nb = 0;
    hipError_t err = hipSuccess;
#define PNET_OCC(NW_, G_)                                                                     \
    if (nw == NW_ && g == G_)                                                                 \
        err = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, rx_kernel<NW_, G_>, kBlock, 0);
    PNET_OCC(4, 16) PNET_OCC(8, 4) PNET_OCC(8, 16) PNET_OCC(8, 64)
#undef PNET_OCC
    return err == hipSuccess && nb > 0 ? nb : 1;
}

int launch_rx(const RxArgs& args, int nw, int g, int blocks, hipStream_t stream) {
    if (nw == 4) return launch_rx_t<4, 16>(args, blocks, stream);
    if (g == 4) return launch_rx_t<8, 4>(args, blocks, stream);
    if (g == 64) return launch_rx_t<8, 64>(args, blocks, stream);
    return launch_rx_t<8, 16>(args, blocks, stream);
}

int launch_slices(const SliceArgs& args, int pseudo, int blocks, hipStream_t stream) {
    if (pseudo == 0) hipLaunchKernelGGL(slice_kernel<0>, dim3(blocks), dim3(kBlock), 0, stream, args);
    else if (pseudo == 4) hipLaunchKernelGGL(slice_kernel<4>, dim3(blocks), dim3(kBlock), 0, stream, args);
    else hipLaunchKernelGGL(slice_kernel<16>, dim3(blocks), dim3(kBlock), 0, stream, args);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace pnetgpu
