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
//  (Three opt-in kernels built in rounds 1-2 — an LDS-DMA stream kernel, a
//  flat granule-list kernel and a stream+parse split kernel — were bit-exact
//  but slower than these on every batch shape and were removed in round 3;
//  their measurements stay in DESIGN.md §3/§8 and profiles/r02/.)
//
//  slice_kernel     the batched util::checksum / ipv4_checksum / ipv6_checksum
//                   (and *_adv) entry points: 16 lanes per slice.
//
// Files: rx_common.h (helpers, parse_frame, window sums, finalize, TX write,
// counters, column stores), rx_small.h, rx_generic.h, rx_slices.h
// (one kernel family each), and this file: the launch glue and kernel choice.
// All are one translation unit.
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
#include "rx_common.h"
#include "rx_small.h"
#include "rx_generic.h"
#include "rx_slices.h"

namespace pnetgpu {

namespace {

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
// (PNET_MIXED_CFG / _MTU_CFG / _JUMBO_CFG, rx_config.h).
// Window granules of the mixed shape: PNET_MIXED_NW (6: 96-B window, 5 blocks/CU by LDS).
#define PNET_MIXED_FN(EXT, TX) rx_kernel<PNET_MIXED_NW, PNET_MIXED_CFG, EXT, TX>
// window granules of the MTU shape's plain instantiations (the EXT ones, with
// the VLAN / extension-header / field-column code, keep 8: at 6 they spill): PNET_MTU_NW
#define PNET_MTU_FN(EXT, TX) rx_kernel<((EXT) ? 8 : PNET_MTU_NW), PNET_MTU_CFG, EXT, TX>
#define PNET_JUMBO_FN(EXT, TX) rx_kernel<8, PNET_JUMBO_CFG, EXT, TX>

template <bool EXT, bool TX>
const void* pick_fn(int kind) {
    switch (kind) {
    case kKindSmall: return reinterpret_cast<const void*>(rx_small_kernel<TX, EXT>);
    case kKindMtu: return reinterpret_cast<const void*>(PNET_MTU_FN(EXT, TX));
    case kKindJumbo: return reinterpret_cast<const void*>(PNET_JUMBO_FN(EXT, TX));
    default: return reinterpret_cast<const void*>(PNET_MIXED_FN(EXT, TX));
    }
}

template <bool EXT, bool TX>
void launch_t(const RxArgs& args, int kind, int blocks, hipStream_t stream) {
    switch (kind) {
    case kKindSmall:
        hipLaunchKernelGGL((rx_small_kernel<TX, EXT>), dim3(blocks), dim3(kBlock), 0, stream, args);
        break;
    case kKindMtu:
        hipLaunchKernelGGL((PNET_MTU_FN(EXT, TX)), dim3(blocks), dim3(kBlock), 0, stream, args);
        break;
    case kKindJumbo:
        hipLaunchKernelGGL((PNET_JUMBO_FN(EXT, TX)), dim3(blocks), dim3(kBlock), 0, stream, args);
        break;
    default:
        hipLaunchKernelGGL((PNET_MIXED_FN(EXT, TX)), dim3(blocks), dim3(kBlock), 0, stream, args);
    }
}

}  // namespace

// Resident blocks of the small kernel: 4 per CU (4 waves/SIMD) measured best
// from 3 to 8 in one process (udp64 274 us at 4 vs 285-303 us at 5-8; its 75
// VGPRs would allow 6), tools/kbench.py --env PNETGPU_BLOCKS_PER_CU: PNET_SMALL_BLOCKS.
// The jumbo shape: 2 per CU (2 waves/SIMD, 9 KiB in flight per wave). With
// more, a batch that fills them reads slower: 2^18 / 2^19 9000-B frames 0.81 /
// 0.85 of 8 TB/s at 2 against 0.80 / 0.81 at 4 (bench.py --frames-scale 2 / 4,
// same box, profiles/r05/jumbo_blocks/); the bench's 2^17 frames (2048 runs)
// fill 2 per CU either way: PNET_JUMBO_BLOCKS.

int rx_blocks_per_cu(int kind, bool ext, int* numregs, int* lds) {
    const void* fn = ext ? pick_fn<true, false>(kind) : pick_fn<false, false>(kind);
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, fn) == hipSuccess) {
        if (numregs) *numregs = fa.numRegs;
        if (lds) *lds = (int)fa.sharedSizeBytes;
    }
    const int nb = resident_blocks(fn, kBlock);
    if (kind == kKindSmall && nb > PNET_SMALL_BLOCKS) return PNET_SMALL_BLOCKS;
    if (kind == kKindJumbo && nb > PNET_JUMBO_BLOCKS) return PNET_JUMBO_BLOCKS;
    return nb;
}

// runs per block per pass (one per wave)
int rx_waves_per_block(int) { return kWavesPerBlock; }

#define PNET_STR2(...) #__VA_ARGS__
#define PNET_STR(...) PNET_STR2(__VA_ARGS__)
// The launched instantiation as rocprofv3 prints it (template arguments in
// declaration order: rx_small_kernel<TX, FIELDS>, rx_kernel<NW, G, U, NT, PASS,
// DYN, EXT, TX>), from the same macros the launches use.
const char* rx_kernel_name(int kind, bool ext, bool tx) {
#define PNET_NAMES(HEAD)                                                                       \
    {HEAD ", false, false>", HEAD ", false, true>", HEAD ", true, false>", HEAD ", true, true>"}
    static const char* const mixed[4] = PNET_NAMES("rx_kernel<" PNET_STR(PNET_MIXED_NW) ", " PNET_STR(PNET_MIXED_CFG));
    static const char* const mtu[4] = {"rx_kernel<" PNET_STR(PNET_MTU_NW) ", " PNET_STR(PNET_MTU_CFG) ", false, false>",
                                       "rx_kernel<" PNET_STR(PNET_MTU_NW) ", " PNET_STR(PNET_MTU_CFG) ", false, true>",
                                       "rx_kernel<8, " PNET_STR(PNET_MTU_CFG) ", true, false>",
                                       "rx_kernel<8, " PNET_STR(PNET_MTU_CFG) ", true, true>"};
    static const char* const jumbo[4] = PNET_NAMES("rx_kernel<8, " PNET_STR(PNET_JUMBO_CFG));
    static const char* const small[4] = {"rx_small_kernel<false, false>", "rx_small_kernel<true, false>",
                                         "rx_small_kernel<false, true>", "rx_small_kernel<true, true>"};
#undef PNET_NAMES
    const int i = (ext ? 2 : 0) + (tx ? 1 : 0);
    switch (kind) {
    case kKindSmall: return small[i];
    case kKindMtu: return mtu[i];
    case kKindJumbo: return jumbo[i];
    default: return mixed[i];
    }
}

int launch_rx(const RxArgs& args, int kind, int blocks, bool tx, hipStream_t stream) {
    // EXT instantiations: dispatch extensions (flags; never with the small kernel)
    // or header-field columns
    const bool ext = args.flags != 0 || args.field_cols != 0;
    (void)hipGetLastError();   // a stale error of an unrelated earlier call is not this launch's
    set_last_rx_kernel(rx_kernel_name(kind, ext, tx));
    if (tx) ext ? launch_t<true, true>(args, kind, blocks, stream) : launch_t<false, true>(args, kind, blocks, stream);
    else ext ? launch_t<true, false>(args, kind, blocks, stream) : launch_t<false, false>(args, kind, blocks, stream);
    return (int)hipGetLastError();
}

// The instantiation of slice_strided_kernel<ND, EXACT, PAD> for a batch: ND =
// dwords a slice may touch at any alignment, (len + 6) / 4 — exact (the cheaper
// sum) for 18..21-B (6) and 62..64-B (17) slices, else the next masked one of
// 2 / 6 / 10 / 17; PAD for strides that are multiples of 8 B (bank spread).
int strided_variant(uint32_t slice_len, uint32_t stride) {
    const uint32_t nd = (slice_len + 6) / 4;
    const bool pad = stride % 8 == 0;
    if (nd == 6) return pad ? 1 : 0;
    if (nd == 17) return pad ? 3 : 2;
    return nd <= 2 ? 4 : nd <= 6 ? 5 : nd <= 10 ? 6 : 7;
}

template <int ND, bool EXACT, bool PAD>
static const void* strided_fn() { return reinterpret_cast<const void*>(slice_strided_kernel<ND, EXACT, PAD>); }
static const void* strided_pick(int v) {
    switch (v) {
    case 0: return strided_fn<6, true, false>();
    case 1: return strided_fn<6, true, true>();
    case 2: return strided_fn<17, true, false>();
    case 3: return strided_fn<17, true, true>();
    case 4: return strided_fn<2, false, true>();
    case 5: return strided_fn<6, false, true>();
    case 6: return strided_fn<10, false, true>();
    default: return strided_fn<17, false, true>();
    }
}

// Resident 256-thread blocks per CU of a slice kernel (0 strided, 1 run, 2 group, 3 tiny),
// so that the persistent grid is exactly one resident wave of blocks (a grid
// larger than what fits runs its last blocks after the first ones finish).
int slice_blocks_per_cu(int which, int pseudo, bool extra) {
    // which 0 (strided): pseudo holds strided_variant() of the instantiation
    const void* fn = which == 0 ? strided_pick(pseudo)
                   : which == 3 ? (pseudo ? reinterpret_cast<const void*>(slice_tiny_kernel<true>)
                                          : reinterpret_cast<const void*>(slice_tiny_kernel<false>))
                   : which == 1 ? (pseudo == 0 ? reinterpret_cast<const void*>(slice_run_kernel<0, false>)
                                  : pseudo == 4 ? (extra ? reinterpret_cast<const void*>(slice_run_kernel<4, true>)
                                                         : reinterpret_cast<const void*>(slice_run_kernel<4, false>))
                                                : (extra ? reinterpret_cast<const void*>(slice_run_kernel<16, true>)
                                                         : reinterpret_cast<const void*>(slice_run_kernel<16, false>)))
                   : (pseudo == 0 ? reinterpret_cast<const void*>(slice_kernel<0, false>)
                      : pseudo == 4 ? (extra ? reinterpret_cast<const void*>(slice_kernel<4, true>)
                                             : reinterpret_cast<const void*>(slice_kernel<4, false>))
                                    : (extra ? reinterpret_cast<const void*>(slice_kernel<16, true>)
                                             : reinterpret_cast<const void*>(slice_kernel<16, false>)));
    return resident_blocks(fn, kBlock);
}

static const char* const kStridedNames[8] = {
    "slice_strided_kernel<6, true, false>", "slice_strided_kernel<6, true, true>",
    "slice_strided_kernel<17, true, false>", "slice_strided_kernel<17, true, true>",
    "slice_strided_kernel<2, false, true>", "slice_strided_kernel<6, false, true>",
    "slice_strided_kernel<10, false, true>", "slice_strided_kernel<17, false, true>"};

int launch_slices_strided_small(const SliceArgs& args, int blocks, hipStream_t stream) {
    (void)hipGetLastError();
    set_last_rx_kernel(kStridedNames[strided_variant(args.slice_len, args.stride)]);
    // one launch per instantiation (hipLaunchKernelGGL needs the template at compile time)
#define PNET_STRIDED(ND, EX, PAD) \
    hipLaunchKernelGGL((slice_strided_kernel<ND, EX, PAD>), dim3(blocks), dim3(kBlock), 0, stream, args)
    switch (strided_variant(args.slice_len, args.stride)) {
    case 0: PNET_STRIDED(6, true, false); break;
    case 1: PNET_STRIDED(6, true, true); break;
    case 2: PNET_STRIDED(17, true, false); break;
    case 3: PNET_STRIDED(17, true, true); break;
    case 4: PNET_STRIDED(2, false, true); break;
    case 5: PNET_STRIDED(6, false, true); break;
    case 6: PNET_STRIDED(10, false, true); break;
    default: PNET_STRIDED(17, false, true);
    }
#undef PNET_STRIDED
    return (int)hipGetLastError();
}

int launch_slices(const SliceArgs& args, int pseudo, int which, int blocks, hipStream_t stream) {
    const bool extra = args.extra_offsets != nullptr;
    (void)hipGetLastError();
    if (pseudo == 0 && extra) return -1;   // util::checksum has no extra slice
    if (which == 3) {
        if (pseudo || extra || args.strided) return -1;
        set_last_rx_kernel(args.compact ? "slice_tiny_kernel<true>" : "slice_tiny_kernel<false>");
        if (args.compact) hipLaunchKernelGGL((slice_tiny_kernel<true>), dim3(blocks), dim3(kBlock), 0, stream, args);
        else hipLaunchKernelGGL((slice_tiny_kernel<false>), dim3(blocks), dim3(kBlock), 0, stream, args);
        return (int)hipGetLastError();
    }
    const bool run = which == 1;
    // rocprofv3's names: [run / group][pseudo 0, 4, 16][extra]
    static const char* const kNames[2][3][2] = {
        {{"slice_run_kernel<0, false>", ""}, {"slice_run_kernel<4, false>", "slice_run_kernel<4, true>"},
         {"slice_run_kernel<16, false>", "slice_run_kernel<16, true>"}},
        {{"slice_kernel<0, false>", ""}, {"slice_kernel<4, false>", "slice_kernel<4, true>"},
         {"slice_kernel<16, false>", "slice_kernel<16, true>"}}};
    set_last_rx_kernel(kNames[run ? 0 : 1][pseudo == 0 ? 0 : pseudo == 4 ? 1 : 2][extra ? 1 : 0]);
#define PNET_RUN(P, X) hipLaunchKernelGGL((slice_run_kernel<P, X>), dim3(blocks), dim3(kBlock), 0, stream, args)
    if (run) {
        if (pseudo == 0) PNET_RUN(0, false);
        else if (pseudo == 4 && !extra) PNET_RUN(4, false);
        else if (pseudo == 4) PNET_RUN(4, true);
        else if (!extra) PNET_RUN(16, false);
        else PNET_RUN(16, true);
    } else if (pseudo == 0) {
        hipLaunchKernelGGL((slice_kernel<0, false>), dim3(blocks), dim3(kBlock), 0, stream, args);
    } else if (pseudo == 4 && !extra) {
        hipLaunchKernelGGL((slice_kernel<4, false>), dim3(blocks), dim3(kBlock), 0, stream, args);
    } else if (pseudo == 4) {
        hipLaunchKernelGGL((slice_kernel<4, true>), dim3(blocks), dim3(kBlock), 0, stream, args);
    } else if (!extra) {
        hipLaunchKernelGGL((slice_kernel<16, false>), dim3(blocks), dim3(kBlock), 0, stream, args);
    } else {
        hipLaunchKernelGGL((slice_kernel<16, true>), dim3(blocks), dim3(kBlock), 0, stream, args);
    }
#undef PNET_RUN
    return (int)hipGetLastError();
}

}  // namespace pnetgpu

#ifdef PNET_WAVE_TIMES
// The wave-time probe's host side (variant builds only, tools/wave_times.py):
// clear the records before a launch, copy them out after it.
extern "C" int pnetgpu_probe_wave_times(uint64_t* host, size_t words, int clear) {
    using pnetgpu::pnet_wave_times;
    const size_t cap = (size_t)pnetgpu::kWaveTimeSlots * pnetgpu::kWaveTimeWords;
    if (words > cap) words = cap;
    if (clear) {
        void* p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(pnet_wave_times)) != hipSuccess) return -1;
        return hipMemset(p, 0, cap * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(pnet_wave_times), words * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#endif
