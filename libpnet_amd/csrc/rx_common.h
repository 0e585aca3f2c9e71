// rx_common.h — shared device code: arithmetic helpers, the per-lane receive dispatch (parse_frame), window sums, finalize, TX write-back, counters and column stores
// Part of the receive-path kernels; included once, by rx_kernel.hip (one
// translation unit, so every kernel still sees the shared device helpers inline).
#pragma once

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

#ifdef PNET_WAVE_TIMES
// the wave-time probe (rx_internal.h): lane 0 writes its wave's record with
// ordinary vector stores; the hardware ids come from s_getreg (XCC_ID, HW_ID)
__device__ uint64_t pnet_wave_times[kWaveTimeSlots * kWaveTimeWords];
struct WaveTimer {
    uint64_t t0 = wall_clock64();
    uint64_t c0 = clock64(), last = c0;
    uint64_t ph[5] = {0, 0, 0, 0, 0};
    // tail-phase makespan (rx_kernel's tail_sums, per run summed): group-rounds
    // issued, group-round slots (loop iterations x groups) and the slots a
    // perfect split of the issued rounds would need (ceil(issued / groups))
    uint64_t tail[3] = {0, 0, 0};
    uint32_t runs = 0;
    __device__ void mark(int i) {
        const uint64_t c = clock64();
        ph[i] += c - last;
        last = c;
    }
    __device__ void end(uint64_t wid, int lane) {
        const uint64_t t1 = wall_clock64();
        const uint64_t c1 = clock64();
        uint32_t xcc, hwid;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        if (lane == 0 && wid < (uint64_t)kWaveTimeSlots) {
            uint64_t* p = pnet_wave_times + wid * kWaveTimeWords;
            p[0] = t0;
            p[1] = t1;
            p[2] = ((uint64_t)(xcc & 15u) << 32) | hwid;
            p[3] = runs;
            for (int i = 0; i < 5; ++i) p[4 + i] = ph[i];
            p[9] = c1 - c0;
            for (int i = 0; i < 3; ++i) p[10 + i] = tail[i];
        }
    }
};
#define PNET_WT_BEGIN WaveTimer pnet_wt_
#define PNET_WT_RUN ++pnet_wt_.runs
#define PNET_WT_END(wid) pnet_wt_.end((wid), lane)
#define PNET_PH(i) pnet_wt_.mark(i)
#define PNET_TAIL_STAT , pnet_wt_.tail
#else
#define PNET_TAIL_STAT
#define PNET_WT_BEGIN
#define PNET_WT_RUN
#define PNET_WT_END(wid)
#define PNET_PH(i)
#endif

// The wave's issue priority rotated by a step count, phased by its hardware
// wave slot, so no wave of a SIMD keeps the age-order lead the arbiter gives
// the oldest (tools/wave_times.py: with fixed priorities the 4th wave of a
// SIMD ran 11 % longer than the 1st on the same work). Used where a launch has
// too few runs per wave to balance by claims (RunSched): the MTU shape.
__device__ __forceinline__ void rotate_prio(uint32_t step) {
    uint32_t hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    switch ((step + hwid) & 3u) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3);
    }
}

// The runs one wave processes (RxArgs::sched): its grid-stride share of
// [0, nstatic), then runs claimed from one of the launch's nctr counters (the
// wave's home counter, (wave id / kClaimChunk) % nctr, owns an equal slice of
// [nstatic, nruns); kClaimChunk = 32 consecutive wave ids are 8 blocks, which
// the dispatcher spreads over the 8 XCDs: rx_internal.h),
// one claim kept in flight ahead of its use so the atomic's round trip
// overlaps a whole run: claim() issues the atomic, and its value is read
// (and waited for) only at the next take(). take() returns the next run;
// >= nruns ends the loop, and then the wave reports its finish (finish()):
// the counters are left zero for the block's next launch.
struct RunQueue {
    uint64_t next_static, stride, nstatic, nruns, lo, hi;
    unsigned long long* ctr;
    uint64_t pend;          // claimed ahead (dynamic phase), nruns when none is pending
    uint32_t kraw;          // lane 0: the in-flight claim's count
    uint32_t gwaves;        // waves whose home is this wave's counter
    bool inflight, finished;
    unsigned long long* groups_done;
    uint32_t* done_host;
    uint32_t seq, ngroups;

    __device__ RunQueue(const RunSched& s, uint64_t n_units, uint64_t wave_id, uint64_t wave_stride)
        : next_static(wave_id), stride(wave_stride), nstatic(s.ctr ? s.nstatic : n_units), nruns(n_units), lo(0),
          hi(0), ctr(s.ctr), pend(n_units), kraw(0), gwaves(0), inflight(false), finished(false),
          groups_done(s.groups_done), done_host(s.done_host), seq(s.seq), ngroups(0) {
        if (ctr) {
            const uint64_t h = (wave_id / kClaimChunk) % s.nctr, d = nruns - nstatic;
            lo = nstatic + d * h / s.nctr;
            hi = nstatic + d * (h + 1) / s.nctr;
            ctr += h * s.ctr_stride;
            // the group's size: kClaimChunk-wave chunks c < ceil(W / kClaimChunk)
            // with c % nctr == h, the last chunk holding W % kClaimChunk waves
            // when W is not a multiple of kClaimChunk
            constexpr uint64_t C = kClaimChunk;
            const uint64_t nch = (wave_stride + C - 1) / C, full = wave_stride / C, rem = wave_stride % C;
            uint64_t g = h < nch ? ((nch - 1 - h) / s.nctr + 1) * C : 0;
            if (rem && full % s.nctr == h) g -= C - rem;
            gwaves = (uint32_t)g;
            // groups that have waves (all nctr when the host sized nctr from this
            // grid, as plan_sched does): the last of them hands the block back
            ngroups = (uint32_t)(nch < s.nctr ? nch : s.nctr);
            if (next_static >= nstatic) claim();   // no static share: the first claim now
        }
    }
    __device__ void claim() {
        if (__lane_id() == 0) kraw = (uint32_t)atomicAdd(ctr, 1ull);
        inflight = true;
    }
    // the in-flight claim's run (waits for the atomic's return)
    __device__ void resolve() {
        if (!inflight) return;
        inflight = false;
        const uint64_t r = lo + (uint64_t)__builtin_amdgcn_readfirstlane(kraw);
        pend = r < hi ? r : nruns;
    }
    // The wave is done with the counters (no claim in flight: its last one came
    // back past its counter's slice). The group's last wave zeroes the counter;
    // the last group's zeroes groups_done and, after a system-scope fence, hands
    // the block back to the host.
    __device__ void finish() {
        if (!ctr || finished) return;
        finished = true;
        if (__lane_id() == 0) {
            const unsigned long long old = atomicAdd(ctr, 1ull << 32);
            if ((uint32_t)(old >> 32) + 1 == gwaves) {
                (void)atomicExch(ctr, 0ull);
                if (atomicAdd(groups_done, 1ull) + 1 == ngroups) {
                    (void)atomicExch(groups_done, 0ull);
                    __threadfence_system();
                    __hip_atomic_store(done_host, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
    __device__ uint64_t take() {
        if (next_static < nstatic) {
            const uint64_t r = next_static;
            next_static += stride;
            if (ctr && next_static >= nstatic) claim();   // last static run: the first claim goes out
            return r;
        }
        resolve();
        const uint64_t r = pend;
        if (r < nruns) claim();
        else finish();
        return r;
    }
};

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
    __builtin_nontemporal_store(v, col + i);
}

// Column stores for the frames of one run: the base is wave-uniform (SGPR) and
// the lane adds its index, so each store is one coalesced wave instruction.
// An opaque per-run copy of a frame index: without it the compiler hoists
// column + lane * size for every column out of the run loop, holding ~2 VGPRs
// per column for the whole kernel (16 columns: 32 VGPRs, spills in the flat
// kernel); with it each store recomputes its address (one VALU op).
__device__ __forceinline__ uint64_t opaque_index(uint64_t i) {
    asm volatile("" : "+v"(i));
    return i;
}

__device__ __forceinline__ void store_columns(const pnetgpu_rx_columns& C, uint64_t f0, int lane, bool in_batch,
                                              const Parsed& P, uint32_t ipc, uint32_t l4c, const uint8_t* slot,
                                              int sh) {
    if (!in_batch) return;
    const uint64_t i = opaque_index(f0 + (uint64_t)lane);
    if (C.status) put<uint16_t>(C.status, i, (uint16_t)P.st);
    if (C.ip_csum) put<uint16_t>(C.ip_csum, i, (uint16_t)ipc);
    if (C.l4_csum) put<uint16_t>(C.l4_csum, i, (uint16_t)l4c);
    if (C.ethertype) put<uint16_t>(C.ethertype, i, (uint16_t)P.et);
    if (C.ip_proto) put<uint8_t>(C.ip_proto, i, (uint8_t)P.proto);
    if (C.ttl) put<uint8_t>(C.ttl, i, (uint8_t)P.ttl);
    if (C.l4_offset) put<uint16_t>(C.l4_offset, i, (uint16_t)P.l4off);
    if (C.l4_length) put<uint16_t>(C.l4_length, i, (uint16_t)P.l4len);
    if (C.src_port) put<uint16_t>(C.src_port, i, (uint16_t)P.sp);
    if (C.dst_port) put<uint16_t>(C.dst_port, i, (uint16_t)P.dp);
    if (C.src_ipv4) put<uint32_t>(C.src_ipv4, i, P.s4);
    if (C.dst_ipv4) put<uint32_t>(C.dst_ipv4, i, P.d4);
    if (C.vlan_tci) put<uint16_t>(C.vlan_tci, i, (uint16_t)P.vlan_tci);
    if (C.l3_offset) put<uint8_t>(C.l3_offset, i, (uint8_t)P.l3);
    if (C.src_ipv6 || C.dst_ipv6) {
        const bool v6ok = (P.st & (PNET_ST_L3_MASK | PNET_ST_L3_MALFORMED)) == PNET_ST_L3_IPV6;
        uint4 sv = make_uint4(0, 0, 0, 0), dv = make_uint4(0, 0, 0, 0);
        if (v6ok) {
            sv = lds_read16_unaligned(slot, sh + (int)P.l3 + 8);
            dv = lds_read16_unaligned(slot, sh + (int)P.l3 + 24);
        }
        if (C.src_ipv6) reinterpret_cast<uint4*>(C.src_ipv6)[i] = sv;
        if (C.dst_ipv6) reinterpret_cast<uint4*>(C.dst_ipv6)[i] = dv;
    }
}

// A frame's record packed in 8 dwords, for stores deferred past later runs
// (rx_kernel, kDeferRuns): every column of store_columns except the IPv6
// address columns (read from the LDS slot at store time).
struct Rec {
    uint32_t w[8];
};
__device__ __forceinline__ Rec pack_rec(const Parsed& P, uint32_t ipc, uint32_t l4c) {
    Rec r;
    r.w[0] = (P.st & 0xFFFFu) | (ipc << 16);
    r.w[1] = (l4c & 0xFFFFu) | (P.et << 16);
    r.w[2] = (P.proto & 0xFFu) | ((P.ttl & 0xFFu) << 8) | (P.l4off << 16);
    r.w[3] = (P.l4len & 0xFFFFu) | (P.sp << 16);
    r.w[4] = (P.dp & 0xFFFFu) | (P.vlan_tci << 16);
    r.w[5] = P.s4;
    r.w[6] = P.d4;
    r.w[7] = P.l3;
    return r;
}
__device__ __forceinline__ void store_rec(const pnetgpu_rx_columns& C, uint64_t f0, int lane, bool in_batch,
                                          const Rec& r) {
    if (!in_batch) return;
    const uint64_t i = opaque_index(f0 + (uint64_t)lane);
    if (C.status) put<uint16_t>(C.status, i, (uint16_t)r.w[0]);
    if (C.ip_csum) put<uint16_t>(C.ip_csum, i, (uint16_t)(r.w[0] >> 16));
    if (C.l4_csum) put<uint16_t>(C.l4_csum, i, (uint16_t)r.w[1]);
    if (C.ethertype) put<uint16_t>(C.ethertype, i, (uint16_t)(r.w[1] >> 16));
    if (C.ip_proto) put<uint8_t>(C.ip_proto, i, (uint8_t)r.w[2]);
    if (C.ttl) put<uint8_t>(C.ttl, i, (uint8_t)(r.w[2] >> 8));
    if (C.l4_offset) put<uint16_t>(C.l4_offset, i, (uint16_t)(r.w[2] >> 16));
    if (C.l4_length) put<uint16_t>(C.l4_length, i, (uint16_t)r.w[3]);
    if (C.src_port) put<uint16_t>(C.src_port, i, (uint16_t)(r.w[3] >> 16));
    if (C.dst_port) put<uint16_t>(C.dst_port, i, (uint16_t)r.w[4]);
    if (C.src_ipv4) put<uint32_t>(C.src_ipv4, i, r.w[5]);
    if (C.dst_ipv4) put<uint32_t>(C.dst_ipv4, i, r.w[6]);
    if (C.vlan_tci) put<uint16_t>(C.vlan_tci, i, (uint16_t)(r.w[4] >> 16));
    if (C.l3_offset) put<uint8_t>(C.l3_offset, i, (uint8_t)r.w[7]);
}

// Header-field columns (ABI v3): the remaining generated getters of the views
// the dispatch constructed, read from the frame's bytes (LDS window, or HBM past
// it) only for the columns a caller requested; 0 for a view that was not
// reached. ethernet.rs:20-30, ipv4.rs:138-161, ipv6.rs:21-37, udp.rs:23-31,
// tcp.rs:55-71, icmp.rs:221-232,303-314 (getter bit extraction:
// pnet_macros/src/decorator.rs:1563-1670). Mirrors oracle_rx_frame_ex.
// `l3mode`: PNETGPU_RX_L3 batch (no Ethernet view).
__device__ __forceinline__ void store_field_columns(const pnetgpu_rx_columns& C, uint64_t fi, const Parsed& P,
                                                 const FrameBytes& F, bool l3mode) {
    const uint64_t i = opaque_index(fi);
    const uint32_t st = P.st;
    const bool eth = !l3mode && !(st & (PNET_ST_ETH_MALFORMED | PNET_ST_DESC_INVALID));
    const bool v4 = (st & (PNET_ST_L3_MASK | PNET_ST_L3_MALFORMED)) == PNET_ST_L3_IPV4;
    const bool v6 = (st & (PNET_ST_L3_MASK | PNET_ST_L3_MALFORMED)) == PNET_ST_L3_IPV6;
    const uint32_t l4kind = (st & (PNET_ST_L4_MALFORMED | PNET_ST_FRAGMENT)) ? 0u : (st & PNET_ST_L4_MASK);
    const bool udp = l4kind == PNET_ST_L4_UDP, tcp = l4kind == PNET_ST_L4_TCP;
    // echo views only for the echo types: ICMP 0/8 (packetdump.rs:52-75), ICMPv6
    // 128/129 (icmpv6.rs:135-137); P.sp holds type << 8 | code for ICMP(v6)
    const uint32_t itype = P.sp >> 8;
    const bool echo = P.l4len >= 8u && ((l4kind == PNET_ST_L4_ICMP && (itype == 0u || itype == 8u)) ||
                                        (l4kind == PNET_ST_L4_ICMPV6 && (itype == 128u || itype == 129u)));
    const int l3 = (int)P.l3, l4 = (int)P.l4off;
    const uint32_t b0 = (v4 || v6) ? F.near8(l3) : 0u, b1 = (v4 || v6) ? F.near8(l3 + 1) : 0u;
    if (C.eth_dst || C.eth_src) {
        uint64_t d = 0, s = 0;
        if (eth) {
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                d = (d << 8) | F.near8(k);
                s = (s << 8) | F.near8(6 + k);
            }
        }
        if (C.eth_dst) put<uint64_t>(C.eth_dst, i, d);
        if (C.eth_src) put<uint64_t>(C.eth_src, i, s);
    }
    if (C.ip_version) put<uint8_t>(C.ip_version, i, (uint8_t)(b0 >> 4));                       // u4
    if (C.ip_header_length) put<uint8_t>(C.ip_header_length, i, v4 ? (uint8_t)(b0 & 15u) : 0);  // u4
    if (C.ip_dscp) put<uint8_t>(C.ip_dscp, i, v4 ? (uint8_t)(b1 >> 2) : 0);                     // u6
    if (C.ip_ecn) put<uint8_t>(C.ip_ecn, i, v4 ? (uint8_t)(b1 & 3u) : 0);                       // u2
    if (C.ip_total_length) put<uint16_t>(C.ip_total_length, i, v4 ? (uint16_t)F.near16(l3 + 2) : 0);
    if (C.ip_identification) put<uint16_t>(C.ip_identification, i, v4 ? (uint16_t)F.near16(l3 + 4) : 0);
    if (C.ip_flags) put<uint8_t>(C.ip_flags, i, v4 ? (uint8_t)(F.near8(l3 + 6) >> 5) : 0);     // u3
    if (C.ip_fragment_offset)                                                                    // u13be
        put<uint16_t>(C.ip_fragment_offset, i, v4 ? (uint16_t)(F.near16(l3 + 6) & 0x1FFFu) : 0);
    if (C.ip6_traffic_class)                                                                     // u8 over the nibbles
        put<uint8_t>(C.ip6_traffic_class, i, v6 ? (uint8_t)(((b0 & 15u) << 4) | (b1 >> 4)) : 0);
    if (C.ip6_flow_label)                                                                        // u20be
        put<uint32_t>(C.ip6_flow_label, i, v6 ? ((b1 & 15u) << 16) | F.near16(l3 + 2) : 0u);
    if (C.ip6_payload_length) put<uint16_t>(C.ip6_payload_length, i, v6 ? (uint16_t)F.near16(l3 + 4) : 0);
    // L4 views: an IPv6 extension chain may put them past the LDS window (far reads)
    if (C.udp_length) put<uint16_t>(C.udp_length, i, udp ? (uint16_t)F.far16(l4 + 4) : 0);
    if (C.tcp_sequence)
        put<uint32_t>(C.tcp_sequence, i, tcp ? (F.far16(l4 + 4) << 16) | F.far16(l4 + 6) : 0u);
    if (C.tcp_acknowledgement)
        put<uint32_t>(C.tcp_acknowledgement, i, tcp ? (F.far16(l4 + 8) << 16) | F.far16(l4 + 10) : 0u);
    if (C.tcp_data_offset || C.tcp_reserved || C.tcp_flags) {
        const uint32_t x = tcp ? F.far16(l4 + 12) : 0u;                  // data_offset:4 reserved:4 flags:8
        if (C.tcp_data_offset) put<uint8_t>(C.tcp_data_offset, i, (uint8_t)(x >> 12));
        if (C.tcp_reserved) put<uint8_t>(C.tcp_reserved, i, (uint8_t)((x >> 8) & 15u));
        if (C.tcp_flags) put<uint8_t>(C.tcp_flags, i, (uint8_t)x);
    }
    if (C.tcp_window) put<uint16_t>(C.tcp_window, i, tcp ? (uint16_t)F.far16(l4 + 14) : 0);
    if (C.tcp_urgent_ptr) put<uint16_t>(C.tcp_urgent_ptr, i, tcp ? (uint16_t)F.far16(l4 + 18) : 0);
    if (C.icmp_sequence) put<uint16_t>(C.icmp_sequence, i, echo ? (uint16_t)F.far16(l4 + 6) : 0);
}

}  // namespace
}  // namespace pnetgpu
