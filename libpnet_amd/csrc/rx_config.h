// rx_config.h — every build-time parameter of the receive kernels, in one place.
//
// The PNET_* macros below are the only ones a build may override (-D, as
// `make variant` and tools/abvar.sh do for same-box A/B runs); each sets a
// shipped kernel shape, and the shipped library uses the defaults here. The
// reasons for each value sit beside its use (rx_kernel.hip, rx_common.h,
// abi.cpp). tests/test_knobs.py fails on any other overridable PNET_* macro in
// csrc/. Parameters that earlier A/B rounds settled are plain constants at the
// end of this file, not knobs.
#pragma once

#include <stdint.h>

// ---- receive kernel shapes (rx_kernel.hip) -----------------------------------
// tail shapes: <G lanes per frame, U loads in flight per lane, non-temporal
// loads, PASS (0 window/tail split, 1 unified), DYN queue>
#ifndef PNET_MIXED_CFG
#define PNET_MIXED_CFG 4, 8, false, 0, true
#endif
#ifndef PNET_MTU_CFG
#define PNET_MTU_CFG 8, 4, false, 1, false
#endif
#ifndef PNET_JUMBO_CFG
#define PNET_JUMBO_CFG 64, 9, true, 0, false
#endif
// window granules of the mixed shape and of the MTU shape's plain instantiations
#ifndef PNET_MIXED_NW
#define PNET_MIXED_NW 8
#endif
#ifndef PNET_MTU_NW
#define PNET_MTU_NW 8
#endif
// resident blocks per CU of the small (64-B) and the jumbo shapes, and the
// small kernel's register bound (waves per SIMD)
#ifndef PNET_SMALL_BLOCKS
#define PNET_SMALL_BLOCKS 4
#endif
#ifndef PNET_JUMBO_BLOCKS
#define PNET_JUMBO_BLOCKS 2
#endif
#ifndef PNET_SMALL_WAVES
#define PNET_SMALL_WAVES 4
#endif

// ---- run scheduling (rx_internal.h RunSched, abi.cpp plan_sched) ------------
// consecutive wave ids per claim counter, the share of runs assigned in
// grid-stride order (100: no claims) and the claim counters per launch (the
// last two are also PNETGPU_TUNE_STATIC_PCT / _CLAIM_COUNTERS at run time)
#ifndef PNET_CLAIM_CHUNK
#define PNET_CLAIM_CHUNK 32
#endif
#ifndef PNET_STATIC_PCT
#define PNET_STATIC_PCT 88
#endif
#ifndef PNET_CLAIM_COUNTERS
#define PNET_CLAIM_COUNTERS 64
#endif

// ---- diagnostics --------------------------------------------------------------
// PNET_WAVE_TIMES (undefined in the product): the per-wave timing probe build
// read by tools/wave_times.py (rx_common.h WaveTimer).

namespace pnetgpu {
constexpr int kSliceU = 4;          // loads in flight per lane in the slice kernels
constexpr int kJumboWaves = 4;      // the jumbo (non-temporal) shape's launch bound, waves per SIMD
constexpr int kMixedJumboU = 9;     // loads in flight per lane of jumbo runs inside the mixed shape
constexpr int kDeferRuns = 3;       // runs whose records the unified (MTU) shape holds back
constexpr int kTxDeferRuns = 3;     // runs whose in-place TX writes the unified shape holds back
}  // namespace pnetgpu
