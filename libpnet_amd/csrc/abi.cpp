// abi.cpp — C-ABI entry points of libpnetgpu.so (include/pnetgpu.h).
//
// Validates arguments, binds the context's device, sizes the persistent grid
// and launches the HIP kernels of rx_kernel.hip. No compute happens on the
// host: there is no CPU fallback path in this library.
#include <hip/hip_runtime.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <new>

#include "pnetgpu.h"
#include "pnetgpu_afpacket.h"
#include "pnetgpu_ring.h"
#include "rx_internal.h"

// run-claim counter blocks per context: each launch that claims runs takes a
// block no other unfinished launch holds (abi.cpp plan_sched); its last wave
// leaves the counters zero and marks the block free in pinned host memory
constexpr uint32_t kSchedBlocks = 64;
constexpr uint32_t kMaxCtrs = 128;                                   // counters per block
constexpr size_t kCtrStride = 256 / sizeof(unsigned long long);      // 256 B apart
// a block: kMaxCtrs counters, then the groups-done line
constexpr size_t kSchedStride = (kMaxCtrs + 1) * kCtrStride;
constexpr size_t kSchedBytes = kSchedBlocks * kSchedStride * sizeof(unsigned long long);

struct pnetgpu_ctx {
    int device;
    int cus;
    // resident blocks per CU of each receive kernel (kind x EXT), queried once
    int per_cu[8][2] = {};
    // of each slice kernel: [strided, run, group, tiny] x pseudo {0, 4, 16} x extra
    // (strided: its variant; tiny: compact descriptors or not)
    int slice_per_cu[4][8][2] = {};
    // run-claim counter blocks (RunSched): kSchedBlocks blocks of kSchedStride
    // u64. Block b is free when done_host[b] (pinned, written by the last wave
    // of the launch that held it) equals seq[b], the sequence number the host
    // gave that launch.
    unsigned long long* d_sched = nullptr;
    uint32_t* done_host = nullptr;
    uint32_t* done_dev = nullptr;      // the device alias of done_host (hipHostGetDevicePointer): what kernels write
    uint32_t seq[kSchedBlocks] = {};
    uint32_t next_seq = 0;
    uint32_t next_block = 0;
    uint64_t claimed_launches = 0;     // launches that took a block
    uint64_t static_fallbacks = 0;     // launches that would have claimed, ran static: every block busy
    uint64_t captured_static = 0;      // launches captured into a graph: static schedule
    // PNETGPU_TUNE_* (-1: default), from the environment at creation only
    int64_t tune[PNETGPU_NTUNE];
    // host-memory entry points (pnetgpu_util.h): device scratch they stage
    // through and the stream they run on, both created on first use
    uint8_t* util_scratch = nullptr;
    size_t util_cap = 0;
    hipStream_t util_stream = nullptr;
};

namespace pnetgpu {
int ctx_device(const pnetgpu_ctx* ctx) { return ctx->device; }

int ctx_util_scratch(pnetgpu_ctx* ctx, size_t bytes, uint8_t** d, hipStream_t* stream) {
    if (hipSetDevice(ctx->device) != hipSuccess) return hip_fail(hipGetLastError());
    if (!ctx->util_stream && hipStreamCreateWithFlags(&ctx->util_stream, hipStreamNonBlocking) != hipSuccess) {
        ctx->util_stream = nullptr;
        return hip_fail(hipGetLastError());
    }
    if (bytes > ctx->util_cap) {
        size_t cap = 1u << 16;
        while (cap < bytes) cap *= 2;
        uint8_t* p = nullptr;
        if (hipMalloc((void**)&p, cap) != hipSuccess) {
            (void)hipGetLastError();
            return PNETGPU_ENOMEM;
        }
        if (ctx->util_scratch) (void)hipFree(ctx->util_scratch);   // no staged call is in flight: each one syncs
        ctx->util_scratch = p;
        ctx->util_cap = cap;
    }
    *d = ctx->util_scratch;
    *stream = ctx->util_stream;
    return PNETGPU_OK;
}
static thread_local int g_last_hip_error = 0;
int last_hip_error() { return g_last_hip_error; }
void set_last_hip_error(int e) { g_last_hip_error = e; }
static thread_local const char* g_last_rx_kernel = "";
void set_last_rx_kernel(const char* name) { g_last_rx_kernel = name; }
const char* last_rx_kernel() { return g_last_rx_kernel; }
int hip_fail(hipError_t e) {
    g_last_hip_error = e != hipSuccess ? (int)e : (int)hipErrorUnknown;
    return PNETGPU_EHIP;
}
}  // namespace pnetgpu

namespace {

constexpr int kBlock = 256;

int64_t tuning(const pnetgpu_ctx* ctx, int key) { return ctx->tune[key]; }

// persistent slice grid: one resident wave of blocks (at most `want`)
int slice_grid(pnetgpu_ctx* ctx, int which, int pseudo, bool extra, uint64_t want) {
    // which 0 (strided): pseudo = strided_variant() in 0..7
    const int k = which == 0 || which == 3 ? pseudo : (pseudo == 0 ? 0 : pseudo == 4 ? 1 : 2);
    int& c = ctx->slice_per_cu[which][k][extra ? 1 : 0];
    if (c <= 0) c = pnetgpu::slice_blocks_per_cu(which, pseudo, extra);
    const int64_t v = tuning(ctx, PNETGPU_TUNE_SLICE_BLOCKS_PER_CU);
    const uint64_t cap = (uint64_t)ctx->cus * (uint64_t)(v > 0 ? v : c > 0 ? c : 1);
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(want, cap));
}
constexpr int kRunFrames = 64;      // frames per wave-run
// PNET_STATIC_PCT: share of a batch's runs assigned statically (100: no claims);
// PNET_CLAIM_COUNTERS: claim counters per launch (rx_config.h)

// Run scheduling of a persistent-grid launch (RunSched): a static grid-stride
// share, then claimed units, so that waves whose share ran slow (the younger
// waves of a SIMD, the slower XCDs: tools/wave_times.py) do not set the
// kernel's end. Launches of fewer than 8 units per wave stay static (1500-B
// frames at 4 runs per wave: claims measured even to +1 %).
// The counters are a block of the context's pool held by this launch alone,
// whatever its stream: a block is handed out only after the launch that held
// it last has finished (its last wave wrote the block's sequence number to
// pinned host memory, RunQueue::finish), so launches on any streams, reused
// stream handles and concurrent streams never share counters. With every block
// held by unfinished launches, or while the stream is being captured into a
// graph (a replayed launch would reuse the captured block and sequence number
// while an earlier replay may still hold it), the launch runs the static
// schedule: the same results without claims. *blk receives the block taken
// (-1: none) and *prev its previous sequence number, for sched_undo.
int plan_sched(pnetgpu_ctx* ctx, uint64_t nunits, uint64_t nwaves, void* stream, pnetgpu::RunSched* s, int* blk,
               uint32_t* prev) {
    *s = pnetgpu::RunSched{};
    *blk = -1;
    s->nstatic = nunits;
    const int64_t tp = tuning(ctx, PNETGPU_TUNE_STATIC_PCT);
    const int64_t static_pct = tp >= 0 ? tp : PNET_STATIC_PCT;
    if (static_pct >= 100 || nwaves == 0 || nunits < 8 * nwaves) return PNETGPU_OK;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(static_cast<hipStream_t>(stream), &cs) != hipSuccess) {
        (void)hipGetLastError();
        cs = hipStreamCaptureStatusActive;       // unknown: the safe choice
    }
    if (cs != hipStreamCaptureStatusNone) {
        ++ctx->captured_static;
        return PNETGPU_OK;
    }
    uint32_t b = kSchedBlocks;
    for (uint32_t i = 0; i < kSchedBlocks; ++i) {
        const uint32_t c = (ctx->next_block + i) % kSchedBlocks;
        if (__atomic_load_n(&ctx->done_host[c], __ATOMIC_ACQUIRE) == ctx->seq[c]) {
            b = c;
            break;
        }
    }
    if (b == kSchedBlocks) {
        ++ctx->static_fallbacks;
        return PNETGPU_OK;
    }
    ctx->next_block = (b + 1) % kSchedBlocks;
    *blk = (int)b;
    *prev = ctx->seq[b];
    if (++ctx->next_seq == ctx->seq[b]) ++ctx->next_seq;   // never the value the block's word already holds
    ctx->seq[b] = ctx->next_seq;
    ++ctx->claimed_launches;
    unsigned long long* ctr = ctx->d_sched + (size_t)b * kSchedStride;
    s->nstatic = (nunits * (uint64_t)static_pct / 100) / nwaves * nwaves;
    s->ctr = ctr;
    s->groups_done = ctr + (size_t)kMaxCtrs * kCtrStride;
    s->done_host = ctx->done_dev + b;
    s->seq = ctx->seq[b];
    const int64_t tn = tuning(ctx, PNETGPU_TUNE_CLAIM_COUNTERS);
    const uint64_t nctr = tn > 0 ? (uint64_t)tn : PNET_CLAIM_COUNTERS;
    // every counter needs home waves: wave ids [0, kClaimChunk nctr) cover them all
    const uint64_t homes = std::max<uint64_t>(1, nwaves / pnetgpu::kClaimChunk);
    s->nctr = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({nctr, kMaxCtrs, homes}));
    s->ctr_stride = (uint32_t)kCtrStride;
    return PNETGPU_OK;
}

// A launch that took a block failed to start: the block is free again.
void sched_undo(pnetgpu_ctx* ctx, int blk, uint32_t prev) {
    if (blk < 0) return;
    ctx->seq[blk] = prev;
    --ctx->claimed_launches;
}

// PNETGPU_<NAME> of each tuning key, read once when a context is created
const char* const kTuneEnv[PNETGPU_NTUNE] = {"PNETGPU_RX_KIND",        "PNETGPU_BLOCKS_PER_CU",
                                             "PNETGPU_STATIC_PCT",     "PNETGPU_CLAIM_COUNTERS",
                                             "PNETGPU_SLICE_BLOCKS_PER_CU", "PNETGPU_SLICE_KERNEL",
                                             "PNETGPU_SLICE_DENSE_SPAN",    "PNETGPU_DEBUG",
                                             "PNETGPU_SCHED_EPOCH"};

bool tuning_valid(int key, int64_t v) {
    if (v == -1) return true;   // the default
    switch (key) {
    case PNETGPU_TUNE_RX_KIND: return v == pnetgpu::kKindMixed || v == pnetgpu::kKindMtu || v == pnetgpu::kKindJumbo;
    case PNETGPU_TUNE_BLOCKS_PER_CU:
    case PNETGPU_TUNE_SLICE_BLOCKS_PER_CU: return v >= 1 && v <= 64;
    case PNETGPU_TUNE_STATIC_PCT: return v >= 0 && v <= 100;
    case PNETGPU_TUNE_CLAIM_COUNTERS: return v >= 1 && v <= (int64_t)kMaxCtrs;
    case PNETGPU_TUNE_SLICE_KERNEL: return v >= 1 && v <= 3;
    case PNETGPU_TUNE_SLICE_DENSE_SPAN: return v >= 0 && v <= 65536;
    case PNETGPU_TUNE_DEBUG: return v == 0 || v == 1;
    case PNETGPU_TUNE_SCHED_EPOCH: return v >= 0 && v <= (int64_t)UINT32_MAX;   // retired: accepted, ignored
    default: return false;
    }
}

void tuning_from_env(pnetgpu_ctx* c) {
    for (int k = 0; k < PNETGPU_NTUNE; ++k) {
        c->tune[k] = -1;
        const char* e = std::getenv(kTuneEnv[k]);
        if (!e || !*e) continue;
        int64_t v;
        if (k == PNETGPU_TUNE_SLICE_KERNEL && (e[0] == 'r' || e[0] == 'g' || e[0] == 't'))
            v = e[0] == 'r' ? 1 : e[0] == 'g' ? 2 : 3;   // run, group, tiny
        else v = std::strtoll(e, nullptr, 10);
        if (tuning_valid(k, v)) c->tune[k] = v;
    }
}

int set_device(const pnetgpu_ctx* ctx) {
    const hipError_t e = hipSetDevice(ctx->device);
    return e == hipSuccess ? PNETGPU_OK : pnetgpu::hip_fail(e);
}

// Aligns the frame base down to 16 B; offsets are shifted by the remainder.
void align_base(const uint8_t* data, uint64_t bytes, const uint8_t** al, uint64_t* delta,
                uint64_t* limit) {
    const uintptr_t p = reinterpret_cast<uintptr_t>(data);
    *delta = p & 15u;
    *al = reinterpret_cast<const uint8_t*>(p - *delta);
    *limit = bytes + *delta;
}

}  // namespace

extern "C" {

int pnetgpu_abi_version(void) { return PNETGPU_ABI_VERSION; }

const char* pnetgpu_strerror(int code) {
    switch (code) {
        case PNETGPU_OK: return "ok";
        case PNETGPU_EINVAL: return "invalid argument";
        case PNETGPU_ENODEV: return "no such HIP device";
        case PNETGPU_EHIP: return "HIP runtime or kernel launch failure";
        case PNETGPU_ENOMEM: return "out of memory";
        case PNETGPU_EFULL: return "batch full: submit first";
        case PNETGPU_EBUSY: return "every ring slot in flight: wait first";
        case PNETGPU_EEMPTY: return "nothing to return (no batch in flight, end of file, or timeout)";
        case PNETGPU_EFORMAT: return "malformed or unsupported capture / block format";
        case PNETGPU_ESYS: return "operating-system call failed (see errno)";
        default: return "unknown pnetgpu error";
    }
}

int pnetgpu_last_hip_error(void) { return pnetgpu::last_hip_error(); }

const char* pnetgpu_last_rx_kernel(void) { return pnetgpu::last_rx_kernel(); }

int pnetgpu_device_count(int* count) {
    if (!count) return PNETGPU_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        *count = 0;
        return PNETGPU_ENODEV;
    }
    *count = n;
    return PNETGPU_OK;
}

int pnetgpu_ctx_create(int device, pnetgpu_ctx** out) {
    if (!out) return PNETGPU_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return PNETGPU_ENODEV;
    if (hipSetDevice(device) != hipSuccess) return PNETGPU_EHIP;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return PNETGPU_EHIP;
    auto* c = new (std::nothrow) pnetgpu_ctx;
    if (!c) return PNETGPU_ENOMEM;
    c->device = device;
    c->cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    tuning_from_env(c);
    if (hipMalloc((void**)&c->d_sched, kSchedBytes) != hipSuccess ||
        hipHostMalloc((void**)&c->done_host, kSchedBlocks * sizeof(uint32_t),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        pnetgpu_ctx_destroy(c);
        return PNETGPU_ENOMEM;
    }
    if (hipHostGetDevicePointer((void**)&c->done_dev, c->done_host, 0) != hipSuccess || !c->done_dev) {
        pnetgpu_ctx_destroy(c);
        return PNETGPU_EHIP;
    }
    for (uint32_t i = 0; i < kSchedBlocks; ++i) c->done_host[i] = 0;   // == seq[i]: every block free
    if (hipMemset(c->d_sched, 0, kSchedBytes) != hipSuccess) {
        pnetgpu_ctx_destroy(c);
        return PNETGPU_EHIP;
    }
    *out = c;
    return PNETGPU_OK;
}

int pnetgpu_ctx_set_tuning(pnetgpu_ctx* ctx, int key, int64_t value) {
    if (!ctx || key < 0 || key >= PNETGPU_NTUNE || !tuning_valid(key, value)) return PNETGPU_EINVAL;
    ctx->tune[key] = value;
    return PNETGPU_OK;
}

int pnetgpu_ctx_get_tuning(const pnetgpu_ctx* ctx, int key, int64_t* value) {
    if (!ctx || !value || key < 0 || key >= PNETGPU_NTUNE) return PNETGPU_EINVAL;
    *value = ctx->tune[key];
    return PNETGPU_OK;
}

int pnetgpu_ctx_sched_conflicts(pnetgpu_ctx* ctx, uint64_t* count) {
    pnetgpu::set_last_hip_error(0);
    if (!ctx || !count) return PNETGPU_EINVAL;
    *count = 0;   // launches never share counters (plan_sched): nothing to report
    return PNETGPU_OK;
}

int pnetgpu_ctx_sched_stats(const pnetgpu_ctx* ctx, uint64_t stats[PNETGPU_NSCHED_STATS]) {
    if (!ctx || !stats) return PNETGPU_EINVAL;
    stats[PNETGPU_SCHED_CLAIMED] = ctx->claimed_launches;
    stats[PNETGPU_SCHED_STATIC_BUSY] = ctx->static_fallbacks;
    stats[PNETGPU_SCHED_STATIC_CAPTURED] = ctx->captured_static;
    uint64_t busy = 0;
    for (uint32_t i = 0; i < kSchedBlocks; ++i)
        busy += __atomic_load_n(&ctx->done_host[i], __ATOMIC_ACQUIRE) != ctx->seq[i];
    stats[PNETGPU_SCHED_BLOCKS_HELD] = busy;
    stats[PNETGPU_SCHED_BLOCKS] = kSchedBlocks;
    return PNETGPU_OK;
}

void pnetgpu_ctx_destroy(pnetgpu_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    // launches still in flight write their counter block and host word: wait
    // for exactly those (each held block's word reaching its sequence number),
    // not for every stream of the device; static and graph-captured launches
    // never touch the pool. A block not handed back within 30 s (a faulted
    // device) falls back to a device-wide synchronize, which reports the fault.
    if (ctx->d_sched && ctx->done_host) {
        bool held = true;
        for (int spin = 0; held && spin < 600000; ++spin) {
            held = false;
            for (uint32_t i = 0; i < kSchedBlocks && !held; ++i)
                held = __atomic_load_n(&ctx->done_host[i], __ATOMIC_ACQUIRE) != ctx->seq[i];
            if (held) {
                const timespec ts{0, 50000};
                nanosleep(&ts, nullptr);
            }
        }
        if (held) (void)hipDeviceSynchronize();
    }
    if (ctx->util_stream) (void)hipStreamSynchronize(ctx->util_stream);
    if (ctx->util_scratch) (void)hipFree(ctx->util_scratch);
    if (ctx->util_stream) (void)hipStreamDestroy(ctx->util_stream);
    if (ctx->d_sched) (void)hipFree(ctx->d_sched);
    if (ctx->done_host) (void)hipHostFree(ctx->done_host);
    delete ctx;
}

static int rx_common(pnetgpu_ctx* ctx, const pnetgpu_batch* b, const pnetgpu_rx_columns* cols, void* stream,
                     bool tx) {
    pnetgpu::set_last_hip_error(0);   // a stale error of an earlier call is not this one's
    if (!ctx || !b || !cols) return PNETGPU_EINVAL;
    if (b->n_frames == 0) return PNETGPU_OK;
    if (!b->data) return PNETGPU_EINVAL;
    if (b->stride == 0 && (!b->offsets || !b->lengths)) return PNETGPU_EINVAL;
    if ((cols->src_ipv6 && (reinterpret_cast<uintptr_t>(cols->src_ipv6) & 15)) ||
        (cols->dst_ipv6 && (reinterpret_cast<uintptr_t>(cols->dst_ipv6) & 15)))
        return PNETGPU_EINVAL;
    if (b->n_frames > (UINT64_MAX - kRunFrames) / 2) return PNETGPU_EINVAL;
    constexpr uint32_t kRxFlags = PNETGPU_RX_VLAN | PNETGPU_RX_IPV6_EXT | PNETGPU_RX_L3;
    constexpr uint32_t kHints = PNETGPU_DESC_HINT_LARGE | PNETGPU_DESC_HINT_JUMBO;
    if ((b->flags & ~(kRxFlags | PNETGPU_DESC_COMPACT | kHints)) || b->reserved) return PNETGPU_EINVAL;
    const uint32_t rxf = b->flags & kRxFlags;   // parse extensions only
    int rc = set_device(ctx);
    if (rc) return rc;

    pnetgpu::RxArgs a{};
    align_base(b->data, b->data_bytes, &a.data, &a.delta, &a.limit);
    a.n = b->n_frames;
    a.first = b->first_offset;
    a.stride = b->stride;
    a.frame_len = b->frame_len;
    a.offsets = b->offsets;
    a.lengths = b->lengths;
    a.cols = *cols;
    a.nruns = (a.n + kRunFrames - 1) / kRunFrames;
    a.flags = rxf;
    a.desc_compact = b->stride == 0 && (b->flags & PNETGPU_DESC_COMPACT) != 0;
    a.l3mode = (rxf & PNETGPU_RX_L3) != 0;
    a.field_cols = cols->eth_dst || cols->eth_src || cols->ip_version || cols->ip_header_length || cols->ip_dscp ||
                   cols->ip_ecn || cols->ip_total_length || cols->ip_identification || cols->ip_flags ||
                   cols->ip_fragment_offset || cols->ip6_traffic_class || cols->ip6_flow_label ||
                   cols->ip6_payload_length || cols->udp_length || cols->tcp_sequence || cols->tcp_acknowledgement ||
                   cols->tcp_data_offset || cols->tcp_reserved || cols->tcp_flags || cols->tcp_window ||
                   cols->tcp_urgent_ptr || cols->icmp_sequence;

    // Kernel choice. Small: fixed stride, every frame 16-B aligned, at most 64 B,
    // inside the buffer (the 64-B configs). Otherwise rx_kernel with the tail
    // shape of the batch's frame sizes: MTU or jumbo for fixed stride, mixed for
    // descriptor batches (their lengths are device-resident).
    int kind = pnetgpu::kKindMixed;
    if (!b->stride) {
        // the caller's size hint (PNETGPU_DESC_HINT_*): the lengths are device-resident
        if (b->flags & PNETGPU_DESC_HINT_JUMBO) kind = pnetgpu::kKindJumbo;
        else if (b->flags & PNETGPU_DESC_HINT_LARGE) kind = pnetgpu::kKindMtu;
    } else {
        const uint64_t base_sh = (a.delta + b->first_offset) & 15u;
        const uint64_t last_end = a.delta + b->first_offset + (b->n_frames - 1) * (uint64_t)b->stride + b->frame_len;
        const bool fits = b->n_frames <= (UINT64_MAX - a.delta - b->first_offset - b->frame_len) / b->stride &&
                          last_end <= a.limit;
        if (base_sh == 0 && b->stride % 16 == 0 && b->frame_len <= 64 && fits && rxf == 0)
            kind = pnetgpu::kKindSmall;
        else
            kind = b->frame_len >= 4096 ? pnetgpu::kKindJumbo : pnetgpu::kKindMtu;
    }
    // the context's tuning (pnetgpu_ctx_set_tuning; never the environment per call)
    const bool debug = tuning(ctx, PNETGPU_TUNE_DEBUG) > 0;
    const int64_t kind_v = tuning(ctx, PNETGPU_TUNE_RX_KIND);
    if (kind_v >= 0 && kind != pnetgpu::kKindSmall) kind = (int)kind_v;
    const int ext = rxf != 0 || a.field_cols;   // the EXT instantiations (launch_rx)
    int& per_cu_cached = ctx->per_cu[kind & 7][ext];
    if (per_cu_cached <= 0 || debug) {                             // first use of this kernel on ctx
        int numregs = 0, lds = 0;
        per_cu_cached = pnetgpu::rx_blocks_per_cu(kind, ext, &numregs, &lds);
        if (debug)
            std::fprintf(stderr, "[pnetgpu] rx kind=%d regs=%d lds=%d blocks/cu=%d cus=%d\n", kind, numregs, lds,
                         per_cu_cached, ctx->cus);
    }
    if (per_cu_cached <= 0) return pnetgpu::hip_fail(hipGetLastError());
    const int64_t per_cu_v = tuning(ctx, PNETGPU_TUNE_BLOCKS_PER_CU);
    const int per_cu = per_cu_v > 0 ? (int)per_cu_v : per_cu_cached;
    const uint64_t wpb = (uint64_t)pnetgpu::rx_waves_per_block(kind);
    const uint64_t want = (a.nruns + wpb - 1) / wpb;
    const uint64_t cap = (uint64_t)ctx->cus * (uint64_t)per_cu;
    const int blocks = (int)std::max<uint64_t>(1, std::min(want, cap));
    int blk;
    uint32_t prev;
    if (const int rc = plan_sched(ctx, a.nruns, (uint64_t)blocks * wpb, stream, &a.sched, &blk, &prev)) return rc;
    if (const int e = pnetgpu::launch_rx(a, kind, blocks, tx, static_cast<hipStream_t>(stream))) {
        sched_undo(ctx, blk, prev);
        pnetgpu::set_last_hip_error(e);
        if (debug)
            std::fprintf(stderr, "[pnetgpu] rx launch failed: %s (%d)\n", hipGetErrorString((hipError_t)e), e);
        return PNETGPU_EHIP;
    }
    return PNETGPU_OK;
}

uint32_t pnetgpu_desc_size_hint(const uint32_t* lengths, uint64_t n) {
    if (!lengths) return 0;
    uint64_t bytes = 0, jumbo_bytes = 0, large = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t l = lengths[i];
        bytes += l;
        if (l >= pnetgpu::kHintJumboMin) jumbo_bytes += l;
        if (l >= pnetgpu::kHintLargeMin) ++large;
    }
    return pnetgpu::desc_size_hint(n, bytes, large, jumbo_bytes);
}

int pnetgpu_rx_process(pnetgpu_ctx* ctx, const pnetgpu_batch* b, const pnetgpu_rx_columns* cols, void* stream) {
    return rx_common(ctx, b, cols, stream, false);
}

int pnetgpu_tx_fill_checksums(pnetgpu_ctx* ctx, const pnetgpu_batch* b, const pnetgpu_rx_columns* cols,
                              void* stream) {
    return rx_common(ctx, b, cols, stream, true);
}

// slice_run_kernel stages a run of 64 small sorted slices through LDS when
// they span at least this many bytes (up to 5 KiB): coalesced loads beat the
// per-lane gathers once the slices are >= ~32 B apart (each gather then
// touches one cache line per lane); below, the gathers share lines and the
// staging's latency costs more than it saves. PNETGPU_TUNE_SLICE_DENSE_SPAN
// overrides (0: always stage, 65536: never).
static uint32_t dense_span(const pnetgpu_ctx* ctx) {
    const int64_t v = tuning(ctx, PNETGPU_TUNE_SLICE_DENSE_SPAN);
    return v >= 0 ? (uint32_t)std::min<int64_t>(v, UINT32_MAX) : 2048u;
}

// The descriptor slice kernel of a batch (1 slice_run_kernel, 2 slice_kernel,
// 3 slice_tiny_kernel), by the buffer bytes per slice unless the tuning names
// one: tiny for util::checksum batches of at most kTinyBytesPerSlice, run up
// to 512, group above. Tiny takes util::checksum only (no pseudo-header, no
// extra slice); a tuned 3 elsewhere means run.
static int slice_choice(const pnetgpu_ctx* ctx, uint64_t data_bytes, uint64_t n, bool plain) {
    const int64_t k = tuning(ctx, PNETGPU_TUNE_SLICE_KERNEL);
    if (k == 3) return plain ? 3 : 1;
    if (k == 1 || k == 2) return (int)k;
    const uint64_t per = data_bytes / n;
    return plain && per <= pnetgpu::kTinyBytesPerSlice ? 3 : per <= 512 ? 1 : 2;
}

static int slices_common(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes, uint64_t n,
                         const uint64_t* offsets, const uint32_t* lengths, const uint32_t* skipwords,
                         const uint8_t* addrs, const uint8_t* protos, uint16_t* out, int pseudo,
                         void* stream, const uint64_t* extra_offsets = nullptr,
                         const uint32_t* extra_lengths = nullptr) {
    pnetgpu::set_last_hip_error(0);
    if (!ctx) return PNETGPU_EINVAL;
    if (n == 0) return PNETGPU_OK;
    if (!data || !offsets || !lengths || !skipwords || !out) return PNETGPU_EINVAL;
    if (pseudo && (!addrs || !protos)) return PNETGPU_EINVAL;
    int rc = set_device(ctx);
    if (rc) return rc;
    pnetgpu::SliceArgs a{};
    align_base(data, data_bytes, &a.data, &a.delta, &a.limit);
    a.n = n;
    a.offsets = offsets;
    a.lengths = lengths;
    a.skipwords = skipwords;
    a.addrs = addrs;
    a.protos = protos;
    a.extra_offsets = extra_offsets;
    a.extra_lengths = extra_lengths;
    a.out = out;
    a.dense_min = dense_span(ctx);
    // Kernel choice. The slice lengths are device-resident, so the host decides
    // by the BUFFER bytes per slice (data_bytes / n), which equals the bytes per
    // slice only for slices that tile the buffer: slice_run_kernel (one wave per
    // 64 slices, a slice of at most 4 granules summed by its own lane, longer
    // ones by 2/4/8/16-lane groups of their size class; 9.4x on the reference's
    // 20-B bench shape, 384-B slices 0.64 vs 0.39 of 8 TB/s) when the buffer
    // averages <= 512 B per slice (even at 768 B); slice_kernel (one 16-lane group
    // per slice, grid-stride; 7 % faster on 1-KiB slices) otherwise; *_adv
    // batches the same way (their extra slices summed as a second range). Short
    // slices spread through a large buffer (e.g. headers of MTU frames) thus
    // take slice_kernel; callers that know their slice sizes set
    // PNETGPU_TUNE_SLICE_KERNEL (1 run, 2 group), and uniform slices have
    // pnetgpu_checksum_slices_strided, which decides by the slice length itself.
    const int which = slice_choice(ctx, data_bytes, n, pseudo == 0 && !extra_offsets);
    const bool run = which != 2;
    const uint64_t per_block = run ? kBlock : kBlock / 16;
    const int blocks = slice_grid(ctx, which, which == 3 ? 0 : pseudo, extra_offsets != nullptr,
                                  (n + per_block - 1) / per_block);
    // scheduled units: slice_run_kernel's / slice_tiny_kernel's runs of 64 slices, slice_kernel's 4
    int blk;
    uint32_t prev;
    if ((rc = plan_sched(ctx, run ? (n + 63) / 64 : (n + 3) / 4, (uint64_t)blocks * 4, stream, &a.sched, &blk,
                         &prev)))
        return rc;
    if (const int e = pnetgpu::launch_slices(a, pseudo, which, blocks, static_cast<hipStream_t>(stream))) {
        sched_undo(ctx, blk, prev);
        pnetgpu::set_last_hip_error(e);
        return PNETGPU_EHIP;
    }
    return PNETGPU_OK;
}

int pnetgpu_checksum_slices_strided(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes, uint64_t n,
                                    uint64_t first_offset, uint32_t stride, uint32_t slice_len, uint32_t skipword,
                                    uint16_t* out, void* stream) {
    pnetgpu::set_last_hip_error(0);
    if (!ctx) return PNETGPU_EINVAL;
    if (n == 0) return PNETGPU_OK;
    if (!data || !out) return PNETGPU_EINVAL;
    // every slice inside [0, data_bytes): first + (n - 1) * stride + slice_len, overflow-safe
    if (first_offset > data_bytes || slice_len > data_bytes - first_offset) return PNETGPU_EINVAL;
    if (stride && n - 1 > (data_bytes - first_offset - slice_len) / stride) return PNETGPU_EINVAL;
    int rc = set_device(ctx);
    if (rc) return rc;
    pnetgpu::SliceArgs a{};
    align_base(data, data_bytes, &a.data, &a.delta, &a.limit);
    a.n = n;
    a.out = out;
    a.strided = 1;
    a.first = first_offset;
    a.stride = stride;
    a.slice_len = slice_len;
    a.skipword = skipword;
    a.dense_min = dense_span(ctx);
    // small uniform slices (<= 64 B at <= 64 B apart): runs staged through LDS;
    // otherwise the descriptor kernels with computed offsets (the same choice
    // as pnetgpu_checksum_slices, by the slice length the caller gave)
    const bool small = stride <= 64 && slice_len <= 64;
    const bool run = !small && slice_len <= 512;
    const uint64_t per_block = small || run ? kBlock : kBlock / 16;
    const int blocks = slice_grid(ctx, small ? 0 : run ? 1 : 2, small ? pnetgpu::strided_variant(slice_len, stride) : 0, false,
                                  (n + per_block - 1) / per_block);
    // scheduled units: slice_strided_kernel's blocks of R runs (R as the kernel
    // computes it), slice_run_kernel's runs, slice_kernel's 4 slices
    const uint64_t slices_per_unit =
        small ? 64u * (stride ? std::max(1u, std::min(16u, 4096u / (64u * stride))) : 16u) : run ? 64u : 4u;
    int blk;
    uint32_t prev;
    if ((rc = plan_sched(ctx, (n + slices_per_unit - 1) / slices_per_unit, (uint64_t)blocks * 4, stream, &a.sched,
                         &blk, &prev)))
        return rc;
    const int e = small ? pnetgpu::launch_slices_strided_small(a, blocks, static_cast<hipStream_t>(stream))
                        : pnetgpu::launch_slices(a, 0, run ? 1 : 2, blocks, static_cast<hipStream_t>(stream));
    if (e) {
        sched_undo(ctx, blk, prev);
        return pnetgpu::hip_fail((hipError_t)e);
    }
    return PNETGPU_OK;
}

int pnetgpu_checksum_slices_compact(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes, uint64_t n,
                                    const pnetgpu_slice_desc* desc, uint16_t* out, void* stream) {
    pnetgpu::set_last_hip_error(0);
    if (!ctx) return PNETGPU_EINVAL;
    if (n == 0) return PNETGPU_OK;
    if (!data || !desc || !out) return PNETGPU_EINVAL;
    int rc = set_device(ctx);
    if (rc) return rc;
    pnetgpu::SliceArgs a{};
    align_base(data, data_bytes, &a.data, &a.delta, &a.limit);
    a.n = n;
    a.offsets = reinterpret_cast<const uint64_t*>(desc);
    a.compact = 1;
    a.out = out;
    a.dense_min = dense_span(ctx);
    // the same choice as pnetgpu_checksum_slices (by the buffer bytes per slice)
    const int which = slice_choice(ctx, data_bytes, n, true);
    const bool run = which != 2;
    const uint64_t per_block = run ? kBlock : kBlock / 16;
    const int blocks = slice_grid(ctx, which, which == 3 ? 1 : 0, false, (n + per_block - 1) / per_block);
    int blk;
    uint32_t prev;
    if ((rc = plan_sched(ctx, run ? (n + 63) / 64 : (n + 3) / 4, (uint64_t)blocks * 4, stream, &a.sched, &blk,
                         &prev)))
        return rc;
    if (const int e = pnetgpu::launch_slices(a, 0, which, blocks, static_cast<hipStream_t>(stream))) {
        sched_undo(ctx, blk, prev);
        return pnetgpu::hip_fail((hipError_t)e);
    }
    return PNETGPU_OK;
}

int pnetgpu_checksum_slices(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes, uint64_t n,
                            const uint64_t* offsets, const uint32_t* lengths, const uint32_t* skipwords,
                            uint16_t* out, void* stream) {
    return slices_common(ctx, data, data_bytes, n, offsets, lengths, skipwords, nullptr, nullptr, out, 0,
                         stream);
}

int pnetgpu_ipv4_checksum_slices(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes, uint64_t n,
                                 const uint64_t* offsets, const uint32_t* lengths,
                                 const uint32_t* skipwords, const uint8_t* addrs, const uint8_t* protos,
                                 uint16_t* out, void* stream) {
    return slices_common(ctx, data, data_bytes, n, offsets, lengths, skipwords, addrs, protos, out, 4,
                         stream);
}

int pnetgpu_ipv6_checksum_slices(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes, uint64_t n,
                                 const uint64_t* offsets, const uint32_t* lengths,
                                 const uint32_t* skipwords, const uint8_t* addrs, const uint8_t* protos,
                                 uint16_t* out, void* stream) {
    return slices_common(ctx, data, data_bytes, n, offsets, lengths, skipwords, addrs, protos, out, 16,
                         stream);
}

int pnetgpu_ipv4_checksum_adv_slices(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes, uint64_t n,
                                     const uint64_t* offsets, const uint32_t* lengths, const uint32_t* skipwords,
                                     const uint64_t* extra_offsets, const uint32_t* extra_lengths,
                                     const uint8_t* addrs, const uint8_t* protos, uint16_t* out, void* stream) {
    if (n && (!extra_offsets || !extra_lengths)) return PNETGPU_EINVAL;
    return slices_common(ctx, data, data_bytes, n, offsets, lengths, skipwords, addrs, protos, out, 4, stream,
                         extra_offsets, extra_lengths);
}

int pnetgpu_ipv6_checksum_adv_slices(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes, uint64_t n,
                                     const uint64_t* offsets, const uint32_t* lengths, const uint32_t* skipwords,
                                     const uint64_t* extra_offsets, const uint32_t* extra_lengths,
                                     const uint8_t* addrs, const uint8_t* protos, uint16_t* out, void* stream) {
    if (n && (!extra_offsets || !extra_lengths)) return PNETGPU_EINVAL;
    return slices_common(ctx, data, data_bytes, n, offsets, lengths, skipwords, addrs, protos, out, 16, stream,
                         extra_offsets, extra_lengths);
}

}  // extern "C"
