// rx_kernel.hip — MI355X (gfx950) receive-path kernels: Ethernet/IPv4/IPv6
// parse + ones-complement checksums (UDP/TCP/ICMP/ICMPv6) for a batch of frames.
//
// What it computes is libpnet's per-frame receive chain (examples/packetdump.rs:120-217
// over pnet_packet's views and checksums, pnet_packet/src/util.rs:76-181); see
// include/pnetgpu.h for the contract and DESIGN.md for layouts and rooflines.
//
// Receive kernels: one wavefront (64 lanes) per run of 64 consecutive frames:
//
//  rx_small_kernel  fixed-stride batches whose frames sit 16-B aligned and span
//                   at most 64 B (the 64-B configs). The run's 4 KiB arrive as
//                   four coalesced 1-KiB dwordx4 wave loads, are transposed
//                   through 16-B-aligned LDS slots (conflict-free ds_read_b128),
//                   and lane l then holds frame l in 16 VGPRs. The next run's
//                   loads are issued before the current run is processed
//                   (software pipelining). IPv4 with IHL 5 (and every trivially
//                   classified frame) takes a register-only fast path with
//                   compile-time field positions (small_fast); anything else
//                   (IPv6, IPv4 options) takes the generic parse on its LDS
//                   slot. TX patches the LDS copy and writes the run back with
//                   the same four coalesced 1-KiB wave instructions.
//
//  rx_kernel        everything else (descriptor mode, any alignment, any size).
//                   Per run: descriptors (prefetched a run ahead); the window
//                   (first NW=8 aligned 16-B granules of each frame) into a
//                   padded LDS slot; then, before any parsing, the speculative
//                   tail: every frame byte past the window is summed by groups
//                   of G lanes streaming coalesced granules (U loads in flight
//                   per lane) from a per-wave frame list; then lane l parses
//                   frame l from its slot, sums the window part of its ranges
//                   and trims the tail sum to the L4 range. Shapes per kind
//                   (mixed / MTU / jumbo) and the unified pass, where the group
//                   loop also fills the window, are at the end of this file.
//
//  rx_stream_kernel opt-in (PNETGPU_RX_KIND=4) for fixed strides >= 1 KiB: each
//                   wave streams its contiguous frame range through an LDS-DMA
//                   ring (global_load_lds_dwordx4) and derives every frame's
//                   tail from prefix sums of the byte stream; bit-exact, 1.00x
//                   traffic, slower than rx_kernel here.
//
//  slice_kernel     the batched util::checksum / ipv4_checksum / ipv6_checksum
//                   (and *_adv) entry points: 16 lanes per slice.
//
// Checksum arithmetic (why the sums are bit-exact without byte-swapping loads):
//   The reference sums big-endian 16-bit words relative to the start of the slice
//   (util.rs:158-181) into an exact u32 and folds with end-around carry. The fold
//   depends only on the sum mod 0xFFFF and on whether it is zero. Summing the
//   little-endian halves of aligned dwords (v_sad_u16) weights byte b at absolute
//   address a by 256^(a&1); since 65536 == 1 (mod 0xFFFF) that equals the BE
//   weight up to one factor 256, i.e. a byte swap of the folded result when the
//   slice starts at an even absolute address (every range here starts at an even
//   frame offset, so parity = frame offset parity). All partial sums are exact
//   non-negative integers, so "zero iff every in-range byte is zero" holds too.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pnetgpu.h"
#include "rx_internal.h"


namespace pnetgpu {

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

// ---- arithmetic helpers ----------------------------------------------------
__device__ __forceinline__ uint32_t fold16(uint32_t x) {
    x = (x & 0xFFFFu) + (x >> 16);
    x = (x & 0xFFFFu) + (x >> 16);
    return x;
}
__device__ __forceinline__ uint32_t bswap16(uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); }
// mask of the first x bytes of a dword, x in [0, 4]
__device__ __forceinline__ uint32_t first_bytes(int x) { return (uint32_t)(0xFFFFFFFFull >> (32 - 8 * x)); }
__device__ __forceinline__ int clamp04(int v) { return min(max(v, 0), 4); }
// LE 16-bit halves of d added to acc (v_sad_u16 with a zero operand)
__device__ __forceinline__ uint32_t sad(uint32_t d, uint32_t acc) { return __builtin_amdgcn_sad_u16(d, 0u, acc); }
// 16-B streaming load (read once: non-temporal hint)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 load16_nt(const void* p) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
// 16-B load with the default cache policy (granules other lanes/instructions
// of the same wave touch again: windows, strided per-lane frames)
__device__ __forceinline__ uint4 load16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---- LDS access --------------------------------------------------------------

// 16 bytes of a run [p, p+16) of an LDS slot at any alignment, as 4 LE dwords.
__device__ __forceinline__ uint4 lds_read16_unaligned(const uint8_t* slot, int p) {
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(slot);
    const int q = p >> 2, sh = (p & 3);
    const uint32_t d0 = s32[q], d1 = s32[q + 1], d2 = s32[q + 2], d3 = s32[q + 3], d4 = s32[q + 4];
    uint4 r;
    r.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
    r.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
    r.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
    r.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
    return r;
}

// ---- the reference's receive dispatch, restated for one lane ---------------
// Fields of one frame plus the two summed ranges, frame-relative:
//   A = [a_lo, a_hi)  the IPv4 header, or the IPv6 pseudo-header address bytes
//   B = [b_lo, b_hi)  the L4 slice
// with a_lo <= a_hi <= b_lo <= b_hi (empty ranges collapse onto their neighbour).
struct Parsed {
    uint32_t st, et, proto, ttl, l4off, l4len, sp, dp, s4, d4, ipstored, l4stored, pseudo, vlan_tci, l3;
    int a_lo, a_hi, b_lo, b_hi;
    int l4csum_at;            // frame offset of the L4 checksum field (valid when l4do)
    bool is_v4, l4do, v6pseudo;
};

// Frame bytes for the parse: the LDS window W holds bytes [0, wlim); anything
// past it (long IPv6 extension chains, L4 headers behind them) is read from the
// frame in HBM through G. The IPv4 header and VLAN tags always fit the window.
struct FrameBytes {
    const uint8_t* W;
    const uint8_t* G;
    int wlim;
    __device__ __forceinline__ uint32_t near8(int p) const { return W[p]; }
    __device__ __forceinline__ uint32_t near16(int p) const { return (near8(p) << 8) | near8(p + 1); }
    __device__ __forceinline__ uint32_t near32(int p) const { return (near16(p) << 16) | near16(p + 2); }
    __device__ __forceinline__ uint32_t far8(int p) const {
        if (p < wlim) return W[p];
        return G[p];
    }
    __device__ __forceinline__ uint32_t far16(int p) const { return (far8(p) << 8) | far8(p + 1); }
};

__device__ __forceinline__ bool is_vlan_tpid(uint32_t et) { return et == 0x8100u || et == 0x88A8u || et == 0x9100u; }

// Generic parse of one frame of `len` bytes (FLAGS: PNET_RX_* extensions).
// packetdump.rs:155-217 + ipv4.rs:165-178,226-243 + ipv6.rs:21-137 + vlan.rs:62-72
// + udp/tcp/icmp layouts and minimum sizes (decorator.rs:593-600) + payload
// bounds (decorator.rs:713-769). Mirrors oracle_rx_frame_ex.
__device__ __forceinline__ Parsed parse_frame(const FrameBytes& F, uint32_t len, uint32_t flags) {
    Parsed P{};
    uint32_t et;
    int l3;
    if (flags & PNETGPU_RX_L3) {                       // IP header at byte 0: version nibble
        const uint32_t ver = len ? F.near8(0) >> 4 : 0u;
        et = ver == 4u ? 0x0800u : ver == 6u ? 0x86DDu : 0u;
        l3 = 0;
    } else {
        if (len < 14) {
            P.st = PNET_ST_ETH_MALFORMED;              // EthernetPacket::new == None
            return P;
        }
        et = F.near16(12);
        l3 = 14;
    }
    if ((flags & (PNETGPU_RX_VLAN | PNETGPU_RX_L3)) == PNETGPU_RX_VLAN) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (!is_vlan_tpid(et)) break;
            P.st |= PNET_ST_VLAN;
            if (len < (uint32_t)l3 + 4u) {               // VlanPacket::new == None
                P.et = et;
                P.st |= PNET_ST_L3_MALFORMED;
                return P;
            }
            if (k == 0) P.vlan_tci = F.near16(l3);
            et = F.near16(l3 + 2);
            l3 += 4;
        }
    }
    P.et = et;
    P.l3 = (uint32_t)l3;
    const uint32_t eplen = len - (uint32_t)l3;            // Ethernet payload: unbounded
    bool l3ok = false, v6 = false;
    uint32_t l4s = 0, l4n = 0;                            // L4 slice [l4s, l4s + l4n)
    bool has_l4 = false;
    if (et == 0x0800u) {
        P.st |= PNET_ST_L3_IPV4;
        if (eplen < 20) {
            P.st |= PNET_ST_L3_MALFORMED;
        } else {
            l3ok = true;
            P.is_v4 = true;
            const uint32_t ihl4 = (F.near8(l3) & 15u) * 4u;
            const uint32_t hl = min(max(ihl4, 20u), eplen);   // ipv4.rs:169-175
            const uint32_t tl = F.near16(l3 + 2);
            P.ttl = F.near8(l3 + 8);
            P.proto = F.near8(l3 + 9);
            P.ipstored = F.near16(l3 + 10);
            P.s4 = F.near32(l3 + 12);
            P.d4 = F.near32(l3 + 16);
            P.a_lo = l3;
            P.a_hi = l3 + (int)hl;
            const uint32_t start = max(20u, ihl4);             // 20 + ipv4_options_length
            const uint32_t plen = tl > ihl4 ? tl - ihl4 : 0u;  // ipv4_payload_length
            if (eplen > start) {
                has_l4 = true;
                l4s = (uint32_t)l3 + start;
                l4n = min(start + plen, eplen) - start;
            }
        }
    } else if (et == 0x86DDu) {
        P.st |= PNET_ST_L3_IPV6;
        if (eplen < 40) {
            P.st |= PNET_ST_L3_MALFORMED;
        } else {
            l3ok = true;
            v6 = true;
            P.proto = F.near8(l3 + 6);
            P.ttl = F.near8(l3 + 7);
            const uint32_t pl = F.near16(l3 + 4);
            uint32_t pln = 0;                                   // #[length = "payload_length"]
            if (eplen > 40) pln = min(40u + pl, eplen) - 40u;
            const int pbase = l3 + 40;
            uint32_t pos = 0;
            if (flags & PNETGPU_RX_IPV6_EXT) {                  // ipv6.rs:39-137
                uint32_t nh = P.proto;
                for (int k = 0; k < 4; ++k) {
                    if (nh == 0 || nh == 60 || nh == 43) {
                        const uint32_t minl = nh == 43 ? 4u : 2u;
                        if (pln - pos < minl) { P.proto = nh; P.st |= PNET_ST_L4_MALFORMED; return P; }
                        const uint32_t el = F.far8(pbase + (int)pos + 1) * 8u + 8u;
                        if (el > pln - pos) { P.proto = nh; P.st |= PNET_ST_L4_MALFORMED; return P; }
                        nh = F.far8(pbase + (int)pos);
                        pos += el;
                    } else if (nh == 44) {
                        if (pln - pos < 8u) { P.proto = nh; P.st |= PNET_ST_L4_MALFORMED; return P; }
                        const uint32_t fo = F.far16(pbase + (int)pos + 2);
                        nh = F.far8(pbase + (int)pos);
                        pos += 8;
                        if (fo & 0xFFFCu) {                     // not the first fragment
                            P.proto = nh;
                            P.st |= PNET_ST_FRAGMENT;
                            if (pln > pos) {
                                P.l4off = (uint32_t)pbase + pos;
                                P.l4len = pln - pos;
                            }
                            return P;
                        }
                    } else {
                        break;
                    }
                }
                P.proto = nh;
            }
            if (pln > pos) {
                has_l4 = true;
                l4s = (uint32_t)pbase + pos;
                l4n = pln - pos;
            }
        }
    } else {
        P.st |= PNET_ST_UNKNOWN_ETHERTYPE;
    }
    if (has_l4) {
        P.l4off = l4s;
        P.l4len = l4n;
    }
    if (l3ok) {
        uint32_t kind = 0, minlen = 0;
        int soff = 0;
        switch (P.proto) {
            case 17: kind = PNET_ST_L4_UDP; minlen = 8; soff = 6; break;
            case 6: kind = PNET_ST_L4_TCP; minlen = 20; soff = 16; break;
            case 1: kind = PNET_ST_L4_ICMP; minlen = 4; soff = 2; break;
            case 58: kind = PNET_ST_L4_ICMPV6; minlen = 4; soff = 2; break;
            default: break;
        }
        if (!kind) {
            P.st |= PNET_ST_UNKNOWN_PROTO;
        } else {
            P.st |= kind;
            if (l4n < minlen) {
                P.st |= PNET_ST_L4_MALFORMED;
            } else {
                const int p = (int)l4s;
                P.sp = F.far16(p);
                if (P.proto == 17 || P.proto == 6) P.dp = F.far16(p + 2);
                else P.dp = l4n >= 8 ? F.far16(p + 4) : 0u;
                P.l4stored = F.far16(p + soff);
                P.l4csum_at = p + soff;
                if (P.proto == 1) {                            // icmp::checksum: no pseudo-header
                    P.l4do = true;
                } else if (v6) {                               // util::ipv6_checksum
                    P.l4do = true;
                    P.v6pseudo = true;
                    P.a_lo = l3 + 8;                           // pseudo-header address bytes
                    P.a_hi = l3 + 40;
                    P.pseudo = P.proto + l4n;
                } else if (P.proto != 58) {                    // util::ipv4_checksum
                    P.l4do = true;
                    P.pseudo = (P.s4 >> 16) + (P.s4 & 0xFFFFu) + (P.d4 >> 16) + (P.d4 & 0xFFFFu) +
                               P.proto + l4n;
                }
                if (P.l4do) {
                    P.b_lo = p;
                    P.b_hi = p + (int)l4n;
                }
            }
        }
    }
    // canonical empty ranges: a_lo <= a_hi <= b_lo <= b_hi
    if (!P.l4do) { P.b_lo = P.b_hi = P.a_hi; }
    if (P.l4do && !P.is_v4 && !P.v6pseudo) { P.a_lo = P.a_hi = P.b_lo; }   // ICMP over IPv6
    return P;
}

// Window sums of one lane's LDS slot: tA over [p0,p1), tB over [p2,p3), slot
// coordinates, p0 <= p1 <= p2 <= p3 <= window bytes (the slot has a readable
// pad dword, so p3>>2 may equal the dword count). With P(x) = weighted sum of
// the slot bytes in [4*(p0>>2), x): tA = P(p1) - P(p0), tB = P(p3) - P(p2).
// One runtime loop over whole dwords (v_sad_u16 each) plus four masked partials.
__device__ __forceinline__ void window_sums(const uint8_t* slot, int p0, int p1, int p2, int p3, uint32_t& tA,
                                            uint32_t& tB) {
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(slot);
    const int k0 = p0 >> 2, k1 = p1 >> 2, k2 = p2 >> 2, k3 = p3 >> 2;
    uint32_t acc = 0, c1 = 0, c2 = 0;
#pragma unroll 1
    for (int k = k0; k < k3; ++k) {
        if (k == k1) c1 = acc;
        if (k == k2) c2 = acc;
        acc = sad(s32[k], acc);
    }
    if (k1 >= k3) c1 = acc;
    if (k2 >= k3) c2 = acc;
    const uint32_t P0 = sad(s32[k0] & first_bytes(p0 & 3), 0u);
    const uint32_t P1 = sad(s32[k1] & first_bytes(p1 & 3), c1);
    const uint32_t P2 = sad(s32[k2] & first_bytes(p2 & 3), c2);
    const uint32_t P3 = sad(s32[k3] & first_bytes(p3 & 3), acc);
    tA += P1 - P0;
    tB += P3 - P2;
}

// Skip-word removal, fold, byte-order fix-up, pseudo-header, compare.
// odd = frame offset parity. Returns ip and l4 checksums through P.
__device__ __forceinline__ void finalize(Parsed& P, uint32_t tA, uint32_t tB, bool odd, uint32_t& ipc,
                                         uint32_t& l4c) {
    ipc = 0;
    l4c = 0;
    if (P.is_v4) tA -= odd ? P.ipstored : bswap16(P.ipstored);    // skipword 5 (ipv4.rs:177)
    if (P.l4do) tB -= odd ? P.l4stored : bswap16(P.l4stored);     // skipword 3 / 8 / 1
    uint32_t pA = fold16(tA), pB = fold16(tB);
    if (!odd) { pA = bswap16(pA); pB = bswap16(pB); }
    if (P.is_v4) {
        ipc = (~pA) & 0xFFFFu;
        if (ipc == P.ipstored) P.st |= PNET_ST_IP_CSUM_OK;
    }
    if (P.l4do) {
        l4c = (~fold16(pB + P.pseudo + (P.v6pseudo ? pA : 0u))) & 0xFFFFu;
        P.st |= PNET_ST_L4_CSUM_DONE;
        if (l4c == P.l4stored) P.st |= PNET_ST_L4_CSUM_OK;
    }
}

// TX: write the computed checksums into the frame's stored fields (big-endian),
// i.e. MutableIpv4Packet::set_checksum(ipv4::checksum(..)) and the L4
// set_checksum(udp|tcp::ipv4_checksum(..) / icmp::checksum(..)) of
// benches/rs_sender.rs:38-39,70-71. Byte stores: the fields may sit at odd addresses.
__device__ __forceinline__ void tx_write(uint8_t* frame, const Parsed& P, uint32_t ipc, uint32_t l4c) {
    if (P.is_v4) {
        frame[P.l3 + 10] = (uint8_t)(ipc >> 8);
        frame[P.l3 + 11] = (uint8_t)ipc;
    }
    if (P.st & PNET_ST_L4_CSUM_DONE) {
        frame[P.l4csum_at] = (uint8_t)(l4c >> 8);
        frame[P.l4csum_at + 1] = (uint8_t)l4c;
    }
}

// Per-wave counters (ballots: wave-uniform) and coalesced column stores.
struct Counters {
    uint32_t frames = 0, v4 = 0, v6 = 0, ipbad = 0, l4bad = 0, malf = 0, unk = 0;
    uint64_t bytes = 0;
    __device__ __forceinline__ void add(bool valid, uint32_t len, uint32_t st) {
        frames += (uint32_t)__popcll(__ballot(valid));
        bytes += len;
        v4 += (uint32_t)__popcll(__ballot((st & PNET_ST_L3_MASK) == PNET_ST_L3_IPV4));
        v6 += (uint32_t)__popcll(__ballot((st & PNET_ST_L3_MASK) == PNET_ST_L3_IPV6));
        ipbad += (uint32_t)__popcll(__ballot((st & (PNET_ST_L3_MASK | PNET_ST_L3_MALFORMED | PNET_ST_IP_CSUM_OK)) ==
                                             PNET_ST_L3_IPV4));
        l4bad += (uint32_t)__popcll(__ballot((st & (PNET_ST_L4_CSUM_DONE | PNET_ST_L4_CSUM_OK)) ==
                                             PNET_ST_L4_CSUM_DONE));
        malf += (uint32_t)__popcll(__ballot((st & (PNET_ST_ETH_MALFORMED | PNET_ST_L3_MALFORMED |
                                                   PNET_ST_L4_MALFORMED | PNET_ST_DESC_INVALID)) != 0));
        unk += (uint32_t)__popcll(__ballot((st & (PNET_ST_UNKNOWN_ETHERTYPE | PNET_ST_UNKNOWN_PROTO)) != 0));
    }
    // one atomic set per wave (one-wave blocks)
    __device__ __forceinline__ void flush_wave(uint64_t* out, int lane) {
        for (int o = 32; o >= 1; o >>= 1) {
            uint32_t lo = (uint32_t)bytes, hi = (uint32_t)(bytes >> 32);
            lo = __shfl_xor(lo, o);
            hi = __shfl_xor(hi, o);
            bytes += ((uint64_t)hi << 32) | lo;
        }
        const uint64_t v[PNETGPU_NCOUNTERS] = {frames, bytes, v4, v6, ipbad, l4bad, malf, unk};
        if (lane < PNETGPU_NCOUNTERS) {
            uint64_t x = 0;
#pragma unroll
            for (int c = 0; c < PNETGPU_NCOUNTERS; ++c) x = lane == c ? v[c] : x;
            if (x) atomicAdd(reinterpret_cast<unsigned long long*>(out + lane), (unsigned long long)x);
        }
    }
    // one atomic set per block (all waves must call)
    __device__ __forceinline__ void flush(uint64_t* out, uint64_t (*blk)[PNETGPU_NCOUNTERS], int wv, int lane) {
        for (int o = 32; o >= 1; o >>= 1) {
            uint32_t lo = (uint32_t)bytes, hi = (uint32_t)(bytes >> 32);
            lo = __shfl_xor(lo, o);
            hi = __shfl_xor(hi, o);
            bytes += ((uint64_t)hi << 32) | lo;
        }
        if (lane == 0) {
            blk[wv][PNETGPU_CTR_FRAMES] = frames;
            blk[wv][PNETGPU_CTR_BYTES] = bytes;
            blk[wv][PNETGPU_CTR_IPV4] = v4;
            blk[wv][PNETGPU_CTR_IPV6] = v6;
            blk[wv][PNETGPU_CTR_IP_CSUM_BAD] = ipbad;
            blk[wv][PNETGPU_CTR_L4_CSUM_BAD] = l4bad;
            blk[wv][PNETGPU_CTR_MALFORMED] = malf;
            blk[wv][PNETGPU_CTR_UNKNOWN] = unk;
        }
        __syncthreads();
        if (threadIdx.x < PNETGPU_NCOUNTERS) {
            uint64_t v = 0;
            for (int w = 0; w < kWavesPerBlock; ++w) v += blk[w][threadIdx.x];
            if (v) atomicAdd(reinterpret_cast<unsigned long long*>(out + threadIdx.x), (unsigned long long)v);
        }
    }
};

// Column element store (streaming: written once, never re-read by the kernel)
template <class T>
__device__ __forceinline__ void put(T* col, uint64_t i, T v) {
#ifdef PNET_PLAIN_STORES
    col[i] = v;
#else
    __builtin_nontemporal_store(v, col + i);
#endif
}

// Column stores for the frames of one run: the base is wave-uniform (SGPR) and
// the lane adds its index, so each store is one coalesced wave instruction.
__device__ __forceinline__ void store_columns(const pnetgpu_rx_columns& C, uint64_t f0, int lane, bool in_batch,
                                              const Parsed& P, uint32_t ipc, uint32_t l4c, const uint8_t* slot,
                                              int sh) {
    if (!in_batch) return;
    if (C.status) put<uint16_t>(C.status, f0 + lane, (uint16_t)P.st);
    if (C.ip_csum) put<uint16_t>(C.ip_csum, f0 + lane, (uint16_t)ipc);
    if (C.l4_csum) put<uint16_t>(C.l4_csum, f0 + lane, (uint16_t)l4c);
    if (C.ethertype) put<uint16_t>(C.ethertype, f0 + lane, (uint16_t)P.et);
    if (C.ip_proto) put<uint8_t>(C.ip_proto, f0 + lane, (uint8_t)P.proto);
    if (C.ttl) put<uint8_t>(C.ttl, f0 + lane, (uint8_t)P.ttl);
    if (C.l4_offset) put<uint16_t>(C.l4_offset, f0 + lane, (uint16_t)P.l4off);
    if (C.l4_length) put<uint16_t>(C.l4_length, f0 + lane, (uint16_t)P.l4len);
    if (C.src_port) put<uint16_t>(C.src_port, f0 + lane, (uint16_t)P.sp);
    if (C.dst_port) put<uint16_t>(C.dst_port, f0 + lane, (uint16_t)P.dp);
    if (C.src_ipv4) put<uint32_t>(C.src_ipv4, f0 + lane, P.s4);
    if (C.dst_ipv4) put<uint32_t>(C.dst_ipv4, f0 + lane, P.d4);
    if (C.vlan_tci) put<uint16_t>(C.vlan_tci, f0 + lane, (uint16_t)P.vlan_tci);
    if (C.l3_offset) put<uint8_t>(C.l3_offset, f0 + lane, (uint8_t)P.l3);
    if (C.src_ipv6 || C.dst_ipv6) {
        const bool v6ok = (P.st & (PNET_ST_L3_MASK | PNET_ST_L3_MALFORMED)) == PNET_ST_L3_IPV6;
        uint4 sv = make_uint4(0, 0, 0, 0), dv = make_uint4(0, 0, 0, 0);
        if (v6ok) {
            sv = lds_read16_unaligned(slot, sh + (int)P.l3 + 8);
            dv = lds_read16_unaligned(slot, sh + (int)P.l3 + 24);
        }
        if (C.src_ipv6) reinterpret_cast<uint4*>(C.src_ipv6)[f0 + lane] = sv;
        if (C.dst_ipv6) reinterpret_cast<uint4*>(C.dst_ipv6)[f0 + lane] = dv;
    }
}

// ============================================================================
// rx_small_kernel: fixed stride, frames 16-B aligned, span <= 64 B.
// ============================================================================
constexpr int kSmallSlot = 80;   // 16-B aligned slots; ds_read_b128 conflict-free (20l mod 64 distinct per 16 lanes)

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

#ifndef PNET_SMALL_WAVES
#define PNET_SMALL_WAVES 4   // waves/SIMD the small kernel is register-bounded for
#endif
template <bool TX>
__global__ __launch_bounds__(kBlock, PNET_SMALL_WAVES) void rx_small_kernel(RxArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_slots[kWavesPerBlock][kWave * kSmallSlot];
    __shared__ uint64_t blk_ctr[kWavesPerBlock][PNETGPU_NCOUNTERS];
    const int lane = threadIdx.x & (kWave - 1);
    const int wv = threadIdx.x / kWave;
    uint8_t* slot = lds_slots[wv] + lane * kSmallSlot;
    Counters K;

    const uint64_t wave_stride = (uint64_t)gridDim.x * kWavesPerBlock;
    uint64_t run = (uint64_t)blockIdx.x * kWavesPerBlock + wv;
    SmallRun cur = run < a.nruns ? small_load(a, run, lane) : SmallRun{};
    for (; run < a.nruns; run += wave_stride) {
        // software pipelining: the next run's loads are in flight while this one is processed
        // (two runs ahead measured no faster: the wave is not short of loads in flight)
#ifndef PNET_SMALL_NOPF
        const uint64_t nrun = run + wave_stride;
        SmallRun nxt = nrun < a.nruns ? small_load(a, nrun, lane) : SmallRun{};
#endif

        const uint64_t f0 = run * kWave;
        const bool in_batch = f0 + lane < a.n;
        const uint32_t len = in_batch ? a.frame_len : 0u;
        {
            // granule (frame 16i + lane/4, chunk lane%4) -> that frame's slot; read back own frame
#pragma unroll
            for (int i = 0; i < 4; ++i)
                *reinterpret_cast<uint4*>(lds_slots[wv] + (16 * i + (lane >> 2)) * kSmallSlot + 16 * (lane & 3)) =
                    cur.g[i];
            wave_sync();
#pragma unroll
            for (int c = 0; c < 4; ++c) cur.g[c] = *reinterpret_cast<const uint4*>(slot + 16 * c);
        }

        Parsed P{};
        uint32_t ipc = 0, l4c = 0;
        const uint32_t wv16[16] = {cur.g[0].x, cur.g[0].y, cur.g[0].z, cur.g[0].w, cur.g[1].x, cur.g[1].y,
                                   cur.g[1].z, cur.g[1].w, cur.g[2].x, cur.g[2].y, cur.g[2].z, cur.g[2].w,
                                   cur.g[3].x, cur.g[3].y, cur.g[3].z, cur.g[3].w};
        const bool slow = in_batch && small_fast(wv16, len, P, ipc, l4c);
        // ---- generic path through LDS for the lanes the fast path did not take ----
        const bool need_v6 = a.cols.src_ipv6 || a.cols.dst_ipv6;
#ifdef PNET_SMALL_NOSLOW
        if (slow) P.st = 0xFFFFu;
        if (false) {
#else
        if (__ballot(slow) || need_v6) {
#endif
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
        store_columns(a.cols, f0, lane, in_batch, P, ipc, l4c, slot, 0);
        if (a.cols.counters) K.add(in_batch, len, P.st);
        wave_sync();
#ifndef PNET_SMALL_NOPF
        cur = nxt;
#else
        if (run + wave_stride < a.nruns) cur = small_load(a, run + wave_stride, lane);
#endif
    }
    if (a.cols.counters) K.flush(a.cols.counters, blk_ctr, wv, lane);
}

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
template <int NW, int G, int U, bool NT, bool UNI, bool DYN>
__device__ __forceinline__ void tail_sums(const uint8_t* data, WaveLds<NW>& L, int lane, int count) {
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
    while (__ballot(idx < count)) {
        if (idx < count) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = c0 + u * G;
                v[u] = c < nneed ? (NT ? load16_nt(fb + 16u * c) : load16(fb + 16u * c)) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = c0 + u * G;
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
}

// PASS: 0 = window phase for every frame, then the tails of the long ones;
// 1 = unified: every frame streamed once by the group loop (a hybrid - windows
// of short frames first, long frames unified - measured 5-15 % slower on IMIX).
// EXT: batch flags may be non-zero (VLAN / IPv6 extension dispatch); the
// flags-0 instantiation compiles the parse without those branches (half the
// code, SGPR spills 118 -> 14, IMIX -2 %).
template <int NW, int G, int U, bool NT, int PASS, bool DYN, bool EXT, bool TX>
__global__ __launch_bounds__(kBlock, 4) void rx_kernel(RxArgs a) {
    static_assert(NW == 8, "window granules");
    static_assert(G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "tail group");
    constexpr int kSlot = WaveLds<NW>::kSlot;
    constexpr int kWin = NW * 16;

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
            d_off = a.offsets[fr];
            d_len = a.lengths[fr];
        }
    };
    fetch_desc((uint64_t)blockIdx.x * kWavesPerBlock + wv);
    for (uint64_t run = (uint64_t)blockIdx.x * kWavesPerBlock + wv; run < a.nruns; run += wave_stride) {
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
        if (!in_batch || desc_bad) len = 0;
        const int sh = (int)(off & 15);
        const uint64_t base = off - (uint64_t)sh;
        const uint32_t fend = (uint32_t)sh + len;            // slot-relative end of the frame
        const uint32_t span = (fend + 15u) >> 4;
        const bool long_frame = fend > (uint32_t)kWin;
        L.base[lane] = base;
        L.end[lane] = span < (uint32_t)NW ? span : (uint32_t)NW;   // granules to load into the window
        wave_sync();

        // ---- 2. window: NW*64 granule loads, all in flight before any store --
        if (PASS != 1) {
            uint4 g[NW];
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int q = i * kWave + lane;
                const int fl = q / NW, c = q % NW;
                g[i] = make_uint4(0, 0, 0, 0);
                if ((uint32_t)c < L.end[fl])
                    g[i] = load16(a.data + L.base[fl] + 16u * c);
            }
            fetch_desc(run + wave_stride);
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int q = i * kWave + lane;
                const int fl = q / NW, c = q % NW;
                uint32_t* dst = reinterpret_cast<uint32_t*>(L.win + fl * kSlot + 16 * c);
                dst[0] = g[i].x; dst[1] = g[i].y; dst[2] = g[i].z; dst[3] = g[i].w;
            }
        } else {
            fetch_desc(run + wave_stride);
        }

        // ---- 3. speculative tail: all frame bytes past the window ----------
        // Summed before the parse (no parse state is live, so more loads fit in
        // flight); the parse then trims it to the L4 range B, which in every
        // well-formed frame already runs to the end of the frame. Unified pass:
        // the group loop also fills the window of every frame.
        const bool has_tail = PASS == 1 ? in_batch : long_frame;
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
            tail_sums<NW, G, U, NT, (PASS != 0), DYN>(a.data, L, lane, __popcll(tmask));
        }
        wave_sync();

        // ---- 4. parse + window sums (lane l <-> frame l) -------------------
        Parsed P{};
        if (desc_bad) P.st = PNET_ST_DESC_INVALID;
        else if (in_batch)
            P = parse_frame(FrameBytes{slot + sh, a.data + off, kWin - sh}, len, EXT ? a.flags : 0u);
        // A (<= 97 B into the frame) always lies in the window; B may run past it
        const int p0 = P.a_lo + sh, p1 = P.a_hi + sh, p2 = P.b_lo + sh, p3 = P.b_hi + sh;
        uint32_t tA = 0, tB = 0;
        window_sums(slot, p0, p1, min(p2, kWin), min(p3, kWin), tA, tB);
        if (P.l4do && p3 > kWin) {
            // B past the window = the speculative tail minus [kWin, p2) and [p3, fend)
            tB += L.tail[lane];
            const uint8_t* fb = a.data + base;
            if (p2 > kWin) tB -= lane_range_sum(fb, kWin, p2);
            if ((uint32_t)p3 < fend) tB -= lane_range_sum(fb, p3, (int)fend);
        }

        // ---- 5. finalize + stores ------------------------------------------
        uint32_t ipc = 0, l4c = 0;
        finalize(P, tA, tB, (off & 1) != 0, ipc, l4c);
        if (TX && in_batch && !desc_bad) tx_write(const_cast<uint8_t*>(a.data) + off, P, ipc, l4c);
        store_columns(a.cols, f0, lane, in_batch, P, ipc, l4c, slot, sh);
        if (a.cols.counters) K.add(in_batch && !desc_bad, len, P.st);
        wave_sync();   // slots and lists are rewritten by the next run
    }
    if (a.cols.counters) K.flush(a.cols.counters, blk_ctr, wv, lane);
}

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

// Inclusive scan over the wave: DPP row_shr 1/2/4/8 inside each 16-lane row,
// then row_bcast:15 and row_bcast:31 carry the row totals forward.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
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
        const uint64_t off = a.offsets[i] + a.delta;
        uint32_t len = a.lengths[i];
        const uint32_t skip = a.skipwords[i];
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

// Resident 256-thread blocks per CU for a kernel, from its register and LDS
// footprint (a 256-thread block places one wave on each of the 4 SIMDs).
static int resident_blocks(const void* fn, int block_threads) {
    if (block_threads != kBlock) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, block_threads, 0) != hipSuccess) return -1;
        return nb > 0 ? nb : 1;
    }
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, fn) != hipSuccess) return -1;
    const int vgpr = fa.numRegs > 0 ? ((fa.numRegs + 7) / 8) * 8 : 128;
    int by_vgpr = vgpr > 0 ? 512 / vgpr : 1;
    if (by_vgpr > 8) by_vgpr = 8;
    const int lds = (int)fa.sharedSizeBytes;
    const int by_lds = lds > 0 ? (160 * 1024) / lds : 8;
    const int nb = by_vgpr < by_lds ? by_vgpr : by_lds;
    return nb > 0 ? nb : 1;
}

// Tail shapes per kernel kind: <G lanes per frame, U loads in flight per lane,
// non-temporal loads, PASS (0 window/tail split, 1 unified), DYN queue>, from same-box A/B runs on
// MI355X (tools/abvar.sh): descriptor batches of mixed sizes want narrow groups
// and deep loads; MTU frames 8-lane groups streaming each whole frame once
// (unified: -6 % time); jumbo frames the whole wave on one frame, 9 KiB in
// flight per round (one round per 9000-B frame), non-temporal.
#ifndef PNET_MIXED_CFG
#define PNET_MIXED_CFG 4, 8, false, 0, true
#endif
#ifndef PNET_MTU_CFG
#define PNET_MTU_CFG 8, 4, false, 1, false
#endif
#ifndef PNET_JUMBO_CFG
#define PNET_JUMBO_CFG 64, 9, true, 0, false
#endif

// LDS ring steps (4 KiB each) per wave of the stream kernel
#ifndef PNET_STREAM_SLOTS
#define PNET_STREAM_SLOTS 3
#endif

template <bool EXT, bool TX>
const void* pick_fn(int kind) {
    switch (kind) {
    case kKindSmall: return reinterpret_cast<const void*>(rx_small_kernel<TX>);
    case kKindMtu: return reinterpret_cast<const void*>(rx_kernel<8, PNET_MTU_CFG, EXT, TX>);
    case kKindJumbo: return reinterpret_cast<const void*>(rx_kernel<8, PNET_JUMBO_CFG, EXT, TX>);
    case kKindStream: return reinterpret_cast<const void*>(rx_stream_kernel<PNET_STREAM_SLOTS, EXT>);
    default: return reinterpret_cast<const void*>(rx_kernel<8, PNET_MIXED_CFG, EXT, TX>);
    }
}

template <bool EXT, bool TX>
void launch_t(const RxArgs& args, int kind, int blocks, hipStream_t stream) {
    switch (kind) {
    case kKindSmall:
        hipLaunchKernelGGL(rx_small_kernel<TX>, dim3(blocks), dim3(kBlock), 0, stream, args);
        break;
    case kKindMtu:
        hipLaunchKernelGGL((rx_kernel<8, PNET_MTU_CFG, EXT, TX>), dim3(blocks), dim3(kBlock), 0, stream, args);
        break;
    case kKindJumbo:
        hipLaunchKernelGGL((rx_kernel<8, PNET_JUMBO_CFG, EXT, TX>), dim3(blocks), dim3(kBlock), 0, stream, args);
        break;
    case kKindStream:   // receive only: the host never picks it for TX
        if (!TX)
            hipLaunchKernelGGL((rx_stream_kernel<PNET_STREAM_SLOTS, EXT>), dim3(blocks), dim3(kWave), 0, stream, args);
        break;
    default:
        hipLaunchKernelGGL((rx_kernel<8, PNET_MIXED_CFG, EXT, TX>), dim3(blocks), dim3(kBlock), 0, stream, args);
    }
}

}  // namespace

int rx_blocks_per_cu(int kind, bool ext, int* numregs, int* lds) {
    const void* fn = ext ? pick_fn<true, false>(kind) : pick_fn<false, false>(kind);
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, fn) == hipSuccess) {
        if (numregs) *numregs = fa.numRegs;
        if (lds) *lds = (int)fa.sharedSizeBytes;
    }
    return resident_blocks(fn, kind == kKindStream ? kWave : kBlock);
}

int rx_waves_per_block(int kind) { return kind == kKindStream ? 1 : kWavesPerBlock; }

int launch_rx(const RxArgs& args, int kind, int blocks, bool tx, hipStream_t stream) {
    const bool ext = args.flags != 0;
    if (tx) ext ? launch_t<true, true>(args, kind, blocks, stream) : launch_t<false, true>(args, kind, blocks, stream);
    else ext ? launch_t<true, false>(args, kind, blocks, stream) : launch_t<false, false>(args, kind, blocks, stream);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_slices(const SliceArgs& args, int pseudo, int blocks, hipStream_t stream) {
    const bool extra = args.extra_offsets != nullptr;
    if (pseudo == 0) hipLaunchKernelGGL((slice_kernel<0, false>), dim3(blocks), dim3(kBlock), 0, stream, args);
    else if (pseudo == 4 && !extra) hipLaunchKernelGGL((slice_kernel<4, false>), dim3(blocks), dim3(kBlock), 0, stream, args);
    else if (pseudo == 4) hipLaunchKernelGGL((slice_kernel<4, true>), dim3(blocks), dim3(kBlock), 0, stream, args);
    else if (!extra) hipLaunchKernelGGL((slice_kernel<16, false>), dim3(blocks), dim3(kBlock), 0, stream, args);
    else hipLaunchKernelGGL((slice_kernel<16, true>), dim3(blocks), dim3(kBlock), 0, stream, args);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace pnetgpu
