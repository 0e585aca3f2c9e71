// rx_internal.h — launch arguments shared by the C-ABI layer and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pnetgpu.h"
#include "rx_config.h"

namespace pnetgpu {

// Run scheduling of a persistent-grid launch (RunQueue in rx_common.h): units
// (runs, or slice blocks) [0, nstatic) go to the waves in grid-stride order
// (nstatic is a multiple of the wave count); units [nstatic, n) are claimed one
// at a time from nctr counters, ctr_stride u64 apart from ctr, so waves whose
// share ran slow do not set the kernel's end. ctr == nullptr: all units static.
// The counters are one block of the context's pool (abi.cpp plan_sched), owned
// by this launch alone: zero when it starts (low 32 bits of a counter: claims;
// high 32 bits: the waves of its group that have finished). The last wave of
// each group zeroes its counter, the last group zeroes groups_done and writes
// `seq` to the pinned host word done_host, which frees the block for another
// launch (the host reuses a block only once its word shows the seq it issued).
// Waves per claim chunk: a counter's group is the chunks c with c % nctr == h.
// 32 waves = 8 consecutive blocks, one per XCD. The dispatcher places blocks in
// rounds of one block per CU (256 blocks = 32 chunks per round), and a round's
// waves are younger on their SIMDs and run slower (4.37 vs 3.76 us per 64-B
// run from round 3 to round 0), so with 64 counters, counters h < 32 hold
// rounds 0 + 2 and the others rounds 1 + 3: two group speeds (median ends
// 251-265 us). 16-wave chunks give every group one chunk per round (254-261
// us) but do not end the launch sooner - its last few blocks set the end
// either way - and measured even to 1 % slower over 8 interleaved rounds
// (profiles/r05/wave_ends/), so 32 stays.
constexpr uint32_t kClaimChunk = PNET_CLAIM_CHUNK;

struct RunSched {
    unsigned long long* ctr;
    unsigned long long* groups_done;
    uint32_t* done_host;
    uint64_t nstatic;
    uint32_t seq;
    uint32_t nctr;
    uint32_t ctr_stride;
};

// `data` is 16-B aligned; every descriptor offset is shifted by `delta` (the
// caller pointer's misalignment) and must satisfy off + len <= limit.
struct RxArgs {
    const uint8_t* data;
    uint64_t delta;
    uint64_t limit;
    uint64_t n;
    uint64_t first;
    uint32_t stride;
    uint32_t frame_len;
    const uint64_t* offsets;
    const uint32_t* lengths;
    uint64_t nruns;          // ceil(n / 64): one wave per run of 64 frames
    uint32_t flags;          // PNETGPU_RX_* (the small kernel requires 0)
    uint32_t desc_compact;   // offsets/lengths are uint32_t/uint16_t arrays (PNETGPU_DESC_COMPACT)
    uint32_t field_cols;     // any ABI-v3 header-field column requested (store_field_columns)
    uint32_t l3mode;         // PNETGPU_RX_L3: frames start at the IP header (no Ethernet view)
    RunSched sched;          // run scheduling (static share + claimed runs)
    pnetgpu_rx_columns cols;
};

struct SliceArgs {
    const uint8_t* data;
    uint64_t delta;
    uint64_t limit;
    uint64_t n;
    const uint64_t* offsets;
    const uint32_t* lengths;
    const uint32_t* skipwords;
    const uint8_t* addrs;
    const uint8_t* protos;
    const uint64_t* extra_offsets;   // *_adv: extra_data slices (nullptr otherwise)
    const uint32_t* extra_lengths;
    uint16_t* out;
    // strided form (pnetgpu_checksum_slices_strided): slice i = [first + i * stride,
    // +slice_len), one skipword for all; offsets/lengths/skipwords are unused
    uint32_t compact;    // offsets points to pnetgpu_slice_desc[n] (u32 offset, u16 length, u16 skipword)
    uint32_t strided;
    uint32_t stride;
    uint32_t slice_len;
    uint32_t skipword;
    uint64_t first;
    // slice_run_kernel: a run of small sorted slices is staged through LDS when
    // its span is at least this many bytes (dense_span())
    uint32_t dense_min;
    RunSched sched;      // slice_run_kernel / slice_strided_kernel run scheduling
};

// Kernel kinds: the register-resident small-frame kernel (fixed stride, frames
// 16-B aligned, span <= 64 B, every descriptor valid) or the generic one.
// kernel kinds: rx_small_kernel, or rx_kernel with the tail shape for
// descriptor batches (mixed sizes), MTU-size and jumbo fixed-stride frames
constexpr int kKindMixed = 0;
constexpr int kKindSmall = 1;
constexpr int kKindMtu = 2;
constexpr int kKindJumbo = 3;

// Tuning probe (tools/wave_times.py; built only as a variant library with
// -DPNET_WAVE_TIMES, never in the shipped one): every wave of a receive launch
// records its start and end wall clock (100 MHz), hardware ids and run count.
constexpr int kWaveTimeSlots = 16384;
// t_start, t_end, (xcc << 32) | HW_ID, runs, then the shader clocks (s_memtime)
// the wave spent in each phase of its runs (PNET_PH marks: rx_kernel's window,
// tail, parse, stores), the wave's whole s_memtime span, then the tail phase's
// group-rounds issued, slots used and ideal slots (WaveTimer::tail)
constexpr int kWaveTimeWords = 13;

// PNETGPU_DESC_HINT_* of a descriptor batch from its length statistics (n
// frames, their bytes, frames >= 768 B, bytes in frames >= 4096 B): the rule of
// pnetgpu_desc_size_hint, shared with the ring's per-batch counts
inline uint32_t desc_size_hint(uint64_t n, uint64_t bytes, uint64_t large, uint64_t jumbo_bytes) {
    if (n == 0) return 0;
    if (jumbo_bytes && jumbo_bytes * 5 >= bytes * 4) return PNETGPU_DESC_HINT_JUMBO;
    if (large * 16 >= n * 15) return PNETGPU_DESC_HINT_LARGE;
    return 0;
}
constexpr uint32_t kHintLargeMin = 768;     // bytes: a frame the MTU shape takes well
constexpr uint32_t kHintJumboMin = 4096;    // bytes: a frame of the jumbo shape

// device index a context is bound to (abi.cpp)
int ctx_device(const pnetgpu_ctx* ctx);
// the context's device scratch of at least `bytes` (grown on demand) and its
// own stream, for the host-memory entry points (util_host.cpp); sets the device
int ctx_util_scratch(pnetgpu_ctx* ctx, size_t bytes, uint8_t** d, hipStream_t* stream);

int rx_blocks_per_cu(int kind, bool ext, int* numregs, int* lds);
int rx_waves_per_block(int kind);
// both return the hipError_t of the launch (0 = hipSuccess); errors pending
// from earlier, unrelated HIP calls are cleared first
int launch_rx(const RxArgs& args, int kind, int blocks, bool tx, hipStream_t stream);
// buffers of at most this many bytes per slice take slice_tiny_kernel
// (util::checksum batches; rx_slices.h)
constexpr uint32_t kTinyBytesPerSlice = 32;
// which: 1 slice_run_kernel, 2 slice_kernel, 3 slice_tiny_kernel (util::checksum only, no extra)
int launch_slices(const SliceArgs& args, int pseudo, int which, int blocks, hipStream_t stream);
// resident blocks per CU of slice kernel `which` (0 strided: `pseudo` = its
// strided_variant(), 1 run, 2 group, 3 tiny: `pseudo` = 1 for compact descriptors)
int slice_blocks_per_cu(int which, int pseudo, bool extra);
int strided_variant(uint32_t slice_len, uint32_t stride);
// uniform slices of at most 64 B at a stride of at most 64 B (util::checksum)
int launch_slices_strided_small(const SliceArgs& args, int blocks, hipStream_t stream);
// the HIP error code behind the last PNETGPU_EHIP a launch returned on this thread
int last_hip_error();
void set_last_hip_error(int e);
// the instantiation name of a receive kernel kind, and the thread's last launch
const char* rx_kernel_name(int kind, bool ext, bool tx);
void set_last_rx_kernel(const char* name);
// records `e` as the thread's last HIP error and returns PNETGPU_EHIP: every
// EHIP return site reports its own hipError_t (entry points reset it to 0)
int hip_fail(hipError_t e);

}  // namespace pnetgpu
