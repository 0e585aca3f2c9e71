// ring.cpp — host batch producer (include/pnetgpu_ring.h): pinned host batches
// filled frame by frame, shipped and verified asynchronously on the GPU (the
// capture-file readers that feed it are in pcap.cpp).
#include <hip/hip_runtime.h>

#include <immintrin.h>
#include <time.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <deque>
#include <new>
#include <vector>

#include "host_pool.h"
#include "pnetgpu.h"
#include "pnetgpu_ring.h"
#include "rx_internal.h"

namespace {

// slots per ring: one filling, one held by the application, the rest in flight
// (on two streams alternating by submission, so H2D of batch k+1 overlaps the
// kernel and D2H of k)
constexpr int kDefaultSlots = PNETGPU_RING_DEFAULT_SLOTS;
constexpr int kMaxSlots = PNETGPU_RING_MAX_SLOTS;
constexpr int kNumCols = 38;       // the 16 record columns, then the 22 header-field columns (ABI v3)
constexpr uint64_t kDefaultCols = 0xFFFFull;
// element bytes of each pnetgpu_rx_columns column, in struct order (counters skipped)
constexpr uint32_t kColBytes[kNumCols] = {2, 2, 2, 2, 1, 1, 2, 2, 2, 2, 4, 4, 16, 16, 2, 1,
                                          8, 8, 1, 1, 1, 1, 2, 2, 1, 2, 1, 4, 2, 2, 4, 4, 1, 1, 1, 2, 2, 2};

enum SlotState { kFree = 0, kFilling, kInFlight, kHeld };

uint64_t now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

// what one pack pass took: frames, bytes, and the size-hint statistics
struct PackStats {
    uint64_t frames = 0, bytes = 0;
    uint32_t max_len = 0, min_len = UINT32_MAX;
    uint64_t n_large = 0, jumbo_bytes = 0;
    bool irregular = false;                  // submit_region: a frame off the batch's constant stride
    bool compact_skipped = false;            // pack_frames left the compact descriptors out
};

struct Slot {
    uint8_t* h_frames = nullptr;
    uint64_t* h_off = nullptr;
    uint32_t* h_len = nullptr;
    // the same descriptors in PNETGPU_DESC_COMPACT form (u32 / u16), written
    // alongside; shipped instead when the batch is < 4 GiB and every frame < 64 KiB
    uint32_t* h_off32 = nullptr;
    uint16_t* h_len16 = nullptr;
    uint32_t max_len = 0, min_len = UINT32_MAX;
    // > 0: every frame is max_len bytes at this constant stride from the first,
    // so the batch can ship as a fixed-stride batch without descriptors
    uint32_t stride = 0;
    // frames [0, compact_n) have their compact descriptors; the pushes leave
    // them out past it only while every frame of the slot has one length
    // (backfill_compact fills them in when a batch turns out to need them)
    uint32_t compact_n = 0;
    // size statistics of the batch for its PNETGPU_DESC_HINT_* (desc_size_hint)
    uint64_t n_large = 0, jumbo_bytes = 0;
    uint64_t frame_bytes = 0;               // sum of the frame lengths (bytes counts gaps in a region)
    uint8_t* d_frames = nullptr;
    uint64_t* d_off = nullptr;
    uint32_t* d_len = nullptr;
    // record columns of a batch packed back to back (each 256-B aligned, sized
    // for the batch's n) in one device block and one pinned block: the results
    // come back in a single D2H copy
    uint8_t* d_rec = nullptr;
    uint8_t* h_rec = nullptr;
    uint64_t col_off[kNumCols] = {};
    uint64_t rec_bytes = 0;
    hipEvent_t done = nullptr;
    // PNETGPU_RING_STAGE_TIMES: timing events before the H2D, after it, after
    // the kernel and after the D2H
    hipEvent_t stage[4] = {};
    bool timed = false;                      // this batch recorded them
    uint32_t n = 0;
    uint64_t bytes = 0;
    uint64_t id = 0;
    const uint8_t* frames_view = nullptr;   // what the waited batch's `frames` points at
    uint64_t col_mask = 0;                   // columns this batch computed
    size_t rec_cap = 0;                      // bytes of d_rec / h_rec
    SlotState state = kFree;
};

void** col_slot(pnetgpu_rx_columns& c, int k) {
    void** p[kNumCols] = {(void**)&c.status,    (void**)&c.ip_csum,   (void**)&c.l4_csum,   (void**)&c.ethertype,
                          (void**)&c.ip_proto,  (void**)&c.ttl,       (void**)&c.l4_offset, (void**)&c.l4_length,
                          (void**)&c.src_port,  (void**)&c.dst_port,  (void**)&c.src_ipv4,  (void**)&c.dst_ipv4,
                          (void**)&c.src_ipv6,  (void**)&c.dst_ipv6,  (void**)&c.vlan_tci,  (void**)&c.l3_offset,
                          (void**)&c.eth_dst, (void**)&c.eth_src, (void**)&c.ip_version, (void**)&c.ip_header_length,
                          (void**)&c.ip_dscp, (void**)&c.ip_ecn, (void**)&c.ip_total_length,
                          (void**)&c.ip_identification, (void**)&c.ip_flags, (void**)&c.ip_fragment_offset,
                          (void**)&c.ip6_traffic_class, (void**)&c.ip6_flow_label, (void**)&c.ip6_payload_length,
                          (void**)&c.udp_length, (void**)&c.tcp_sequence, (void**)&c.tcp_acknowledgement,
                          (void**)&c.tcp_data_offset, (void**)&c.tcp_reserved, (void**)&c.tcp_flags,
                          (void**)&c.tcp_window, (void**)&c.tcp_urgent_ptr, (void**)&c.icmp_sequence};
    return p[k];
}

}  // namespace

struct pnetgpu_ring {
    pnetgpu_ctx* ctx = nullptr;
    int device = 0;
    uint64_t cap_bytes = 0;
    uint32_t cap_frames = 0;
    uint32_t flags = 0;
    uint64_t col_mask = kDefaultCols;           // columns computed and copied back (bit k: struct order)
    Slot slots[kMaxSlots];
    int nslots = kDefaultSlots;
    int filling = -1;
    int held = -1;
    std::deque<int> inflight;
    uint64_t next_id = 0;
    pnetgpu_ring_stats stats{};
    // Batches alternate between two streams (of different priorities, so on
    // different hardware queues) by submission order (batch id % 2),
    // whatever slot they fill: consecutive batches overlap (one's H2D with the
    // other's kernel and D2H) and no two in flight share a stream. Per-slot
    // streams (round 5) put up to four copies on the link at once and left
    // batch pairs on one stream whenever the free slots came back out of
    // order; two alternating streams moved 75 GB/s of link traffic where
    // three or four moved 60-69 on the same box (tools/ring_factor_probe.py,
    // profiles/r06/e2e/).
    static constexpr int kStreams = 2;
    hipStream_t streams[kStreams] = {};
};


static void free_slot(Slot& s) {
    if (s.h_frames) (void)hipHostFree(s.h_frames);
    if (s.h_off) (void)hipHostFree(s.h_off);
    if (s.h_len) (void)hipHostFree(s.h_len);
    if (s.h_off32) (void)hipHostFree(s.h_off32);
    if (s.h_len16) (void)hipHostFree(s.h_len16);
    if (s.d_frames) (void)hipFree(s.d_frames);
    if (s.d_off) (void)hipFree(s.d_off);
    if (s.d_len) (void)hipFree(s.d_len);
    if (s.d_rec) (void)hipFree(s.d_rec);
    if (s.h_rec) (void)hipHostFree(s.h_rec);
    if (s.done) (void)hipEventDestroy(s.done);
    for (hipEvent_t e : s.stage)
        if (e) (void)hipEventDestroy(e);
    s = Slot{};
}

// Bytes of the packed record block for up to n frames: the counters, then
// every selected column, each start rounded up to 256 B.
static size_t rec_capacity(uint64_t n, uint64_t mask) {
    size_t b = 8ull * PNETGPU_NCOUNTERS;
    for (int k = 0; k < kNumCols; ++k)
        if ((mask >> k) & 1u) b += 256 + (size_t)kColBytes[k] * n;
    return b;
}

// Replaces the slot's record block with one of `bytes`: the new device and host
// buffers are allocated first and swapped in only when both exist, so a failed
// allocation leaves the slot (and the ring's column mask) exactly as it was.
static bool alloc_rec(Slot& s, size_t bytes) {
    uint8_t* d = nullptr;
    uint8_t* h = nullptr;
    if (hipMalloc((void**)&d, bytes) != hipSuccess) return false;
    if (hipHostMalloc((void**)&h, bytes, hipHostMallocDefault) != hipSuccess) {
        (void)hipFree(d);
        return false;
    }
    if (s.d_rec) (void)hipFree(s.d_rec);
    if (s.h_rec) (void)hipHostFree(s.h_rec);
    s.d_rec = d;
    s.h_rec = h;
    s.rec_cap = bytes;
    return true;
}

static int take_free_slot(pnetgpu_ring* r) {
    for (int i = 0; i < r->nslots; ++i) {
        if (r->slots[i].state == kFree) {
            r->slots[i].state = kFilling;
            r->slots[i].n = 0;
            r->slots[i].bytes = 0;
            r->slots[i].max_len = 0;
            r->slots[i].min_len = UINT32_MAX;
            r->slots[i].stride = 0;
            r->slots[i].compact_n = 0;
            r->slots[i].n_large = 0;
            r->slots[i].jumbo_bytes = 0;
            r->slots[i].frame_bytes = 0;
            return i;
        }
    }
    return -1;
}

// Whether a batch of frames of len bytes at a constant stride ships as a
// fixed-stride batch: where the fixed-stride kernel is the one the descriptor
// batch's size hint would reach anyway — frames of <= 64 B on a 16-B multiple
// stride without parse extensions (the small kernel), or of >= kHintLargeMin B
// (the MTU / jumbo shapes, split at the same 4096 B).
static bool ships_strided(uint32_t len, uint32_t stride, uint32_t flags) {
    constexpr uint32_t kRxFlags = PNETGPU_RX_VLAN | PNETGPU_RX_IPV6_EXT | PNETGPU_RX_L3;
    return stride > 0 && stride >= len &&
           ((len <= 64 && stride % 16 == 0 && !(flags & kRxFlags)) || len >= pnetgpu::kHintLargeMin);
}

// The compact descriptors of frames [compact_n, upto) that the pushes left
// out: every frame of the slot up to there has the slot's one length, packed
// back to back, so frame i sits at i * len. Each frame is filled in once.
static void backfill_compact(Slot& s, uint64_t upto) {
    const uint32_t len = s.max_len;
    const uint64_t lo0 = s.compact_n, n = upto > lo0 ? upto - lo0 : 0;
    auto fill = [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo0 + lo; i < lo0 + hi; ++i) {
            s.h_off32[i] = (uint32_t)(i * len);
            s.h_len16[i] = (uint16_t)len;
        }
    };
    const unsigned nt = n >= (1u << 16) ? pnetgpu::host_threads() : 1u;
    if (nt > 1) pnetgpu::parallel_run(nt, [&](unsigned t) { fill(n * t / nt, n * (t + 1) / nt); });
    else fill(0, n);
    if (upto > s.compact_n) s.compact_n = (uint32_t)upto;
}

extern "C" {

int pnetgpu_ring_create_ex(pnetgpu_ctx* ctx, uint64_t batch_bytes, uint32_t batch_frames, uint32_t flags,
                           uint32_t nslots, pnetgpu_ring** out) {
    pnetgpu::set_last_hip_error(0);
    if (!ctx || !out || batch_bytes == 0 || batch_frames == 0) return PNETGPU_EINVAL;
    if (nslots < PNETGPU_RING_MIN_SLOTS || nslots > (uint32_t)kMaxSlots) return PNETGPU_EINVAL;
    if (flags & ~(PNETGPU_RX_VLAN | PNETGPU_RX_IPV6_EXT | PNETGPU_RX_L3 | PNETGPU_RING_STAGE_TIMES))
        return PNETGPU_EINVAL;
    *out = nullptr;
    auto* r = new (std::nothrow) pnetgpu_ring;
    if (!r) return PNETGPU_ENOMEM;
    r->ctx = ctx;
    r->device = pnetgpu::ctx_device(ctx);
    r->cap_bytes = batch_bytes;
    r->cap_frames = batch_frames;
    r->flags = flags;
    r->nslots = (int)nslots;
    if (hipSetDevice(r->device) != hipSuccess) {
        delete r;
        return pnetgpu::hip_fail(hipGetLastError());
    }
    bool ok = true;
    {
        // HIP multiplexes a process's streams onto GPU_MAX_HW_QUEUES hardware
        // queues (4 by default); two streams that land on one queue run every
        // operation of both in one order, and the ring's copy/copy-back overlap
        // is gone (54 GB/s of link traffic instead of 70-79, depending only on
        // how many streams the process made before the ring:
        // profiles/r06/e2e/hwq_probe*.txt). Queues are drawn per priority, so
        // the two streams get different priorities and never share one.
        int least = 0, greatest = 0;
        (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
        ok = hipStreamCreateWithPriority(&r->streams[0], hipStreamNonBlocking, least) == hipSuccess &&
             hipStreamCreateWithPriority(&r->streams[1], hipStreamNonBlocking, greatest) == hipSuccess;
    }
    for (int i = 0; i < r->nslots && ok; ++i) {
        Slot& s = r->slots[i];
        const size_t fb = batch_bytes + 32;    // granule tail
        ok = hipHostMalloc((void**)&s.h_frames, fb, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void**)&s.h_off, 8ull * batch_frames, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void**)&s.h_len, 4ull * batch_frames, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void**)&s.h_off32, 4ull * batch_frames, hipHostMallocDefault) == hipSuccess &&
             hipHostMalloc((void**)&s.h_len16, 2ull * batch_frames, hipHostMallocDefault) == hipSuccess &&
             hipMalloc((void**)&s.d_frames, fb) == hipSuccess &&
             hipMalloc((void**)&s.d_off, 8ull * batch_frames) == hipSuccess &&
             hipMalloc((void**)&s.d_len, 4ull * batch_frames) == hipSuccess &&
             hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess;
        for (int e = 0; e < 4 && ok && (flags & PNETGPU_RING_STAGE_TIMES); ++e)
            ok = hipEventCreate(&s.stage[e]) == hipSuccess;
        if (ok) ok = alloc_rec(s, rec_capacity(batch_frames, kDefaultCols));
        if (ok) std::memset(s.h_frames + batch_bytes, 0, 32);
    }
    if (!ok) {
        for (auto& s : r->slots) free_slot(s);
        for (auto& st : r->streams)
            if (st) (void)hipStreamDestroy(st);
        delete r;
        return PNETGPU_ENOMEM;
    }
    r->filling = take_free_slot(r);
    r->stats.host_threads = pnetgpu::host_threads();
    *out = r;
    return PNETGPU_OK;
}

int pnetgpu_ring_create(pnetgpu_ctx* ctx, uint64_t batch_bytes, uint32_t batch_frames, uint32_t flags,
                        pnetgpu_ring** out) {
    return pnetgpu_ring_create_ex(ctx, batch_bytes, batch_frames, flags, kDefaultSlots, out);
}

uint32_t pnetgpu_ring_slots(const pnetgpu_ring* r) { return r ? (uint32_t)r->nslots : 0u; }

void pnetgpu_ring_destroy(pnetgpu_ring* r) {
    if (!r) return;
    (void)hipSetDevice(r->device);
    for (auto& st : r->streams)
        if (st) (void)hipStreamSynchronize(st);
    for (auto& s : r->slots) free_slot(s);
    for (auto& st : r->streams)
        if (st) (void)hipStreamDestroy(st);
    delete r;
}

int pnetgpu_ring_push(pnetgpu_ring* r, const uint8_t* frame, uint32_t len) {
    if (!r || (!frame && len)) return PNETGPU_EINVAL;
    if (r->filling < 0 && (r->filling = take_free_slot(r)) < 0) return PNETGPU_EBUSY;
    Slot& s = r->slots[r->filling];
    if (s.n >= r->cap_frames || len > r->cap_bytes - s.bytes) return PNETGPU_EFULL;
    std::memcpy(s.h_frames + s.bytes, frame, len);
    s.h_off[s.n] = s.bytes;
    s.h_len[s.n] = len;
    // a frame that keeps a lazily described slot uniform stays undescribed
    const bool lazy = s.compact_n < s.n && len == s.max_len && s.min_len == s.max_len;
    if (!lazy) {
        backfill_compact(s, s.n);
        s.h_off32[s.n] = (uint32_t)s.bytes;
        s.h_len16[s.n] = (uint16_t)len;
        s.compact_n = s.n + 1;
    }
    s.max_len = std::max(s.max_len, len);
    s.min_len = std::min(s.min_len, len);
    s.n_large += len >= pnetgpu::kHintLargeMin;
    s.jumbo_bytes += len >= pnetgpu::kHintJumboMin ? len : 0;
    s.bytes += len;
    s.frame_bytes += len;
    s.n += 1;
    return PNETGPU_OK;
}

// Packs frames buf[offsets[i], +lengths[i]), i < m, back to back into dst from
// byte `at` (at most room_b bytes), with their descriptors at index 0 of the
// given arrays (off32 and len16 both NULL: no compact ones): the longest prefix that fits, the
// same cut as pushing one frame at a time. Returns the frames taken (0: the
// first frame alone does not fit) and fills *st.
//
// Large packs run on the persistent host pool (host_pool.h), descriptors
// included: one thread's copy into pinned memory tops out far below the PCIe
// link the batch is headed for, and a serial descriptor pass capped 64-B frames
// at ~330 Mframes/s end to end. Pass 1 sums each chunk's lengths; the caller
// finds the cut (all m frames, or the first chunk whose frames overflow, scanned
// to the exact frame); when the cut falls inside the push, pass 2 re-splits the
// frames below it evenly (1500-B frames fill a 64-MiB slot within the first of
// 16 chunks of a 2^20-frame push); the last pass writes every chunk's
// descriptors and copies its frames at its prefix offset (runs of frames
// adjacent in the source in one non-temporal copy). A pack of fewer than 2^16
// frames finds its cut serially and still copies in parallel from
// kParallelCopyMin bytes on.
constexpr uint64_t kParallelCopyMin = 4ull << 20;
static uint64_t pack_frames(const uint8_t* buf, const uint64_t* offsets, const uint32_t* lengths, uint64_t m,
                            uint64_t room_b, uint8_t* dst, uint64_t at, uint64_t* off64, uint32_t* len32,
                            uint32_t* off32, uint16_t* len16, PackStats* st, uint32_t skip_len = 0) {
    *st = PackStats{};
    // skip_len > 0: when every frame of the push is skip_len bytes the compact
    // descriptors are left out (the batch ships fixed-stride; st->compact_skipped)
    bool uniform = skip_len > 0 && off32;
    // one pass per chunk: descriptors, size statistics, and the copies of runs
    // of source-adjacent frames, each issued when the run ends
    auto fill_range = [&](uint64_t lo, uint64_t hi, uint64_t o) {
        PackStats cs;
        uint64_t run_src = lo < hi ? offsets[lo] : 0, run_dst = o, src_end = run_src;
        // Blocks of up to 64 frames, ending where the global frame index is a
        // multiple of 64 (the slot's arrays are 64-B aligned): the u64 / u32
        // descriptors of a block first, then its compact u32 / u16 ones, so
        // at most two non-temporal streams are open at once and each block
        // leaves whole lines behind (four interleaved streams cut the push's
        // rate by a third on the GPU boxes: profiles/r06/e2e/).
        for (uint64_t b0 = lo, b1; b0 < hi; b0 = b1) {
            b1 = std::min<uint64_t>(hi, b0 + 64 - ((reinterpret_cast<uintptr_t>(len32 + b0) >> 2) & 63));
            const uint64_t ob = o;
            for (uint64_t i = b0; i < b1; ++i) {
                const uint32_t len = lengths[i];
                const uint64_t so = offsets[i];
                if (so != src_end) {                   // not adjacent to the previous frame: copy that run
                    if (o > run_dst) pnetgpu::stage_copy(dst + run_dst, buf + run_src, o - run_dst);
                    run_src = so;
                    run_dst = o;
                }
                src_end = so + len;
                // non-temporal: the arrays are written once, in order, and read
                // next by the DMA engine or the consumer (no read-for-ownership)
                _mm_stream_si64(reinterpret_cast<long long*>(off64 + i), (long long)o);
                _mm_stream_si32(reinterpret_cast<int*>(len32 + i), (int)len);
                cs.max_len = std::max(cs.max_len, len);
                cs.min_len = std::min(cs.min_len, len);
                cs.n_large += len >= pnetgpu::kHintLargeMin;
                cs.jumbo_bytes += len >= pnetgpu::kHintJumboMin ? len : 0;
                o += len;
            }
            if (!off32) continue;
            uint64_t oc = ob;
            for (uint64_t i = b0; i < b1; ++i) {
                const uint32_t len = lengths[i];
                _mm_stream_si32(reinterpret_cast<int*>(off32 + i), (int)(uint32_t)oc);
                oc += len;
                // u16 lengths two at a time, one non-temporal u32 store at the
                // even index; a pair split by the range's ends is stored plainly
                if (reinterpret_cast<uintptr_t>(len16 + i) & 2) {
                    if (i > lo) _mm_stream_si32(reinterpret_cast<int*>(len16 + i - 1),
                                                (int)((lengths[i - 1] & 0xFFFFu) | (len << 16)));
                    else len16[i] = (uint16_t)len;
                } else if (i + 1 == hi) {
                    len16[i] = (uint16_t)len;
                }
            }
        }
        if (o > run_dst) pnetgpu::stage_copy(dst + run_dst, buf + run_src, o - run_dst);
        _mm_sfence();                                  // the streamed descriptors before the hand-over
        return cs;
    };
    const unsigned threads = pnetgpu::host_threads();
    uint64_t k = 0, bytes = 0, span = 0;   // the cut, its bytes, the frame range the chunks split
    unsigned nt = threads;
    std::vector<uint64_t> csum;
    if (m < (1u << 16) || threads <= 1) {
        // few frames: the cut in one serial scan of the lengths; the copies
        // still go parallel when they are large (7,456 jumbo frames fill a
        // 64-MiB slot, one thread's copy of which trails the link)
        while (k < m && lengths[k] <= room_b - bytes) {
            uniform = uniform && lengths[k] == skip_len;
            bytes += lengths[k++];
        }
        if (k == 0) return 0;
        if (uniform) {
            off32 = nullptr;
            len16 = nullptr;
            st->compact_skipped = true;
        }
        nt = bytes >= kParallelCopyMin ? (unsigned)std::min<uint64_t>(threads, (k + 15) / 16) : 1u;
        if (nt <= 1) {
            const bool skipped = st->compact_skipped;
            *st = fill_range(0, k, at);
            st->compact_skipped = skipped;
            st->frames = k;
            st->bytes = bytes;
            return k;
        }
        span = k;
        csum.assign(nt, 0);
        for (unsigned t = 0; t < nt; ++t)
            for (uint64_t i = k * t / nt, hi = k * (t + 1) / nt; i < hi; ++i) csum[t] += lengths[i];
    } else {
        csum.assign(nt, 0);
        std::vector<uint8_t> mixed(nt, 0);            // a chunk holding a frame other than skip_len
        pnetgpu::parallel_run(nt, [&](unsigned t) {
            uint64_t sum = 0;
            uint32_t lo_len = UINT32_MAX, hi_len = 0;
            for (uint64_t i = m * t / nt, hi = m * (t + 1) / nt; i < hi; ++i) {
                sum += lengths[i];
                lo_len = std::min(lo_len, lengths[i]);
                hi_len = std::max(hi_len, lengths[i]);
            }
            csum[t] = sum;
            mixed[t] = hi_len && (lo_len != hi_len || hi_len != skip_len);
        });
        for (unsigned t = 0; t < nt && uniform; ++t) uniform = !mixed[t];
        if (uniform) {
            off32 = nullptr;
            len16 = nullptr;
            st->compact_skipped = true;
        }
        unsigned c = 0;
        while (c < nt && bytes + csum[c] <= room_b) bytes += csum[c++];
        k = m;
        if (c < nt) {                                  // chunk c overflows: its exact cut
            k = m * c / nt;
            while (lengths[k] <= room_b - bytes) bytes += lengths[k++];
        }
        if (k == 0) return 0;
        span = m;
        if (k < m && k >= (uint64_t)nt * 64) {         // re-split [0, k) evenly
            span = k;
            pnetgpu::parallel_run(nt, [&](unsigned t) {
                uint64_t sum = 0;
                for (uint64_t i = k * t / nt, hi = k * (t + 1) / nt; i < hi; ++i) sum += lengths[i];
                csum[t] = sum;
            });
        }
    }
    std::vector<PackStats> cst(nt);
    pnetgpu::parallel_run(nt, [&](unsigned t) {
        const uint64_t lo = span * t / nt, hi = std::min(span * (t + 1) / nt, k);
        if (lo >= hi) return;
        uint64_t o = at;
        for (unsigned u = 0; u < t; ++u) o += csum[u];
        cst[t] = fill_range(lo, hi, o);
    });
    for (unsigned u = 0; u < nt; ++u) {
        st->max_len = std::max(st->max_len, cst[u].max_len);
        st->min_len = std::min(st->min_len, cst[u].min_len);
        st->n_large += cst[u].n_large;
        st->jumbo_bytes += cst[u].jumbo_bytes;
    }
    st->frames = k;
    st->bytes = bytes;
    return k;
}

int pnetgpu_ring_push_many(pnetgpu_ring* r, const uint8_t* buf, const uint64_t* offsets, const uint32_t* lengths,
                           uint64_t n, uint64_t* pushed) {
    if (!r || !pushed || (n && (!buf || !offsets || !lengths))) return PNETGPU_EINVAL;
    *pushed = 0;
    if (n == 0) return PNETGPU_OK;
    if (r->filling < 0 && (r->filling = take_free_slot(r)) < 0) return PNETGPU_EBUSY;
    const uint64_t t0 = now_ns();
    Slot& s = r->slots[r->filling];
    // While every frame of the slot has one length that ships fixed-stride, the
    // push leaves the compact descriptors out (they would never cross the link);
    // the first push that breaks the pattern backfills them for the frames before.
    const uint32_t slot_len = s.n == 0 ? lengths[0] : s.min_len == s.max_len ? s.max_len : 0;
    const uint32_t skip_len = slot_len && ships_strided(slot_len, slot_len, r->flags) ? slot_len : 0;
    PackStats st;
    const uint64_t k = pack_frames(buf, offsets, lengths, std::min<uint64_t>(n, r->cap_frames - s.n),
                                   r->cap_bytes - s.bytes, s.h_frames, s.bytes, s.h_off + s.n, s.h_len + s.n,
                                   s.h_off32 + s.n, s.h_len16 + s.n, &st, skip_len);
    if (k && !st.compact_skipped) {
        backfill_compact(s, s.n);                // the frames before this push (s.n not yet advanced)
        s.compact_n = s.n + (uint32_t)k;
    }
    r->stats.push_ns += now_ns() - t0;
    if (k == 0) return PNETGPU_EFULL;
    s.max_len = std::max(s.max_len, st.max_len);
    s.min_len = std::min(s.min_len, st.min_len);
    s.n_large += st.n_large;
    s.jumbo_bytes += st.jumbo_bytes;
    s.n += k;
    s.bytes += st.bytes;
    s.frame_bytes += st.bytes;
    *pushed = k;
    return PNETGPU_OK;
}

int pnetgpu_batch_pack(const uint8_t* buf, const uint64_t* offsets, const uint32_t* lengths, uint64_t n, uint8_t* dst,
                       uint64_t dst_cap, uint64_t* dst_offsets, uint32_t* dst_lengths, uint64_t* packed,
                       uint64_t* packed_bytes) {
    if (!packed || !packed_bytes || (n && (!buf || !offsets || !lengths || !dst || !dst_offsets || !dst_lengths)))
        return PNETGPU_EINVAL;
    *packed = *packed_bytes = 0;
    if (n == 0) return PNETGPU_OK;
    PackStats st;
    const uint64_t k = pack_frames(buf, offsets, lengths, n, dst_cap, dst, 0, dst_offsets, dst_lengths, nullptr,
                                   nullptr, &st);
    if (k == 0) return PNETGPU_EFULL;
    *packed = k;
    *packed_bytes = st.bytes;
    return PNETGPU_OK;
}

uint32_t pnetgpu_host_threads(void) { return pnetgpu::host_threads(); }

// Ship slot s: H2D of the frames from `src` (the slot's pinned batch, or a
// caller region for submit_region) and of the descriptors, receive kernel, D2H
// of every record column and the counters, completion event.
static int ship_slot(pnetgpu_ring* r, Slot& s, const uint8_t* src, uint64_t* id) {
    if (hipSetDevice(r->device) != hipSuccess) return pnetgpu::hip_fail(hipGetLastError());
    const hipStream_t st = r->streams[r->next_id % pnetgpu_ring::kStreams];
    // compact descriptors (6 B/frame over PCIe instead of 12) whenever they can
    // describe the batch; the full ones stay on the host for the waited batch view
    const bool compact = s.bytes <= UINT32_MAX && s.max_len <= UINT16_MAX;
    // Uniform frames at a constant stride ship as a fixed-stride batch, with no
    // descriptors on the link (6 of the 70 B a 64-B frame costs), where
    // ships_strided says so. The records are the same either way.
    const bool strided = s.stride > 0 && ships_strided(s.max_len, s.stride, r->flags);
    if (!strided) backfill_compact(s, s.n);   // frames the pushes left undescribed (e.g. a single frame)
    const void* h_off = compact ? (const void*)s.h_off32 : (const void*)s.h_off;
    const void* h_len = compact ? (const void*)s.h_len16 : (const void*)s.h_len;
    s.timed = (r->flags & PNETGPU_RING_STAGE_TIMES) != 0;
    if (s.timed && hipEventRecord(s.stage[0], st) != hipSuccess) return pnetgpu::hip_fail(hipGetLastError());
    // granule rule: the tail past the last frame is readable (32 zero bytes)
    const uint64_t desc_bytes = strided ? 0 : (compact ? 6ull : 12ull) * s.n;
    if (hipMemcpyAsync(s.d_frames, src, s.bytes, hipMemcpyHostToDevice, st) != hipSuccess ||
        (src != s.h_frames && hipMemsetAsync(s.d_frames + s.bytes, 0, 32, st) != hipSuccess) ||
        (!strided &&
         (hipMemcpyAsync(s.d_off, h_off, (compact ? 4ull : 8ull) * s.n, hipMemcpyHostToDevice, st) != hipSuccess ||
          hipMemcpyAsync(s.d_len, h_len, (compact ? 2ull : 4ull) * s.n, hipMemcpyHostToDevice, st) != hipSuccess)) ||
        hipMemsetAsync(s.d_rec, 0, 8ull * PNETGPU_NCOUNTERS, st) != hipSuccess ||
        (s.timed && hipEventRecord(s.stage[1], st) != hipSuccess))
        return pnetgpu::hip_fail(hipGetLastError());
    pnetgpu_batch b{};
    b.data = s.d_frames;
    b.data_bytes = s.bytes;
    b.n_frames = s.n;
    if (strided) {
        b.stride = s.stride;
        b.frame_len = s.max_len;
        b.flags = r->flags & ~PNETGPU_RING_STAGE_TIMES;
    } else {
        b.offsets = s.d_off;
        b.lengths = s.d_len;
        // the batch's size mix picks the kernel's tail shape (frames of >= 768 B:
        // MTU; mostly jumbo bytes: jumbo; else mixed); records are the same
        b.flags = (r->flags & ~PNETGPU_RING_STAGE_TIMES) | (compact ? PNETGPU_DESC_COMPACT : 0u) |
                  pnetgpu::desc_size_hint(s.n, s.frame_bytes, s.n_large, s.jumbo_bytes);
    }
    pnetgpu_rx_columns c{};
    uint64_t at = 8ull * PNETGPU_NCOUNTERS;          // the counters lead the record block
    for (int k = 0; k < kNumCols; ++k) {
        if (!((r->col_mask >> k) & 1u)) continue;
        at = (at + 255) & ~255ull;
        s.col_off[k] = at;
        *col_slot(c, k) = s.d_rec + at;
        at += (uint64_t)kColBytes[k] * s.n;
    }
    s.rec_bytes = at;
    c.counters = reinterpret_cast<uint64_t*>(s.d_rec);
    int rc = pnetgpu_rx_process(r->ctx, &b, &c, st);
    if (rc) return rc;
    s.col_mask = r->col_mask;
    if ((s.timed && hipEventRecord(s.stage[2], st) != hipSuccess) ||
        hipMemcpyAsync(s.h_rec, s.d_rec, at, hipMemcpyDeviceToHost, st) != hipSuccess ||   // counters + records
        (s.timed && hipEventRecord(s.stage[3], st) != hipSuccess) || hipEventRecord(s.done, st) != hipSuccess)
        return pnetgpu::hip_fail(hipGetLastError());
    r->stats.batches += 1;
    r->stats.frames += s.n;
    r->stats.bytes += s.bytes;
    r->stats.desc_bytes += desc_bytes;
    r->stats.stride_batches += strided;
    s.state = kInFlight;
    s.id = r->next_id++;
    if (id) *id = s.id;
    r->inflight.push_back(r->filling);
    r->filling = take_free_slot(r);
    return PNETGPU_OK;
}

int pnetgpu_ring_submit(pnetgpu_ring* r, uint64_t* id) {
    pnetgpu::set_last_hip_error(0);
    if (!r) return PNETGPU_EINVAL;
    if (id) *id = UINT64_MAX;
    if (r->filling < 0) return PNETGPU_OK;
    Slot& s = r->slots[r->filling];
    if (s.n == 0) return PNETGPU_OK;
    s.frames_view = s.h_frames;
    s.stride = s.n >= 2 && s.min_len == s.max_len ? s.max_len : 0;   // packed back to back
    const uint64_t t0 = now_ns();
    const int rc = ship_slot(r, s, s.h_frames, id);
    r->stats.submit_ns += now_ns() - t0;
    return rc;
}

int pnetgpu_ring_submit_region(pnetgpu_ring* r, const uint8_t* base, const uint64_t* offsets, const uint32_t* lengths,
                               uint64_t n, uint64_t* taken, uint64_t* id) {
    pnetgpu::set_last_hip_error(0);
    if (!r || !taken || (n && (!base || !offsets || !lengths))) return PNETGPU_EINVAL;
    *taken = 0;
    if (id) *id = UINT64_MAX;
    if (n == 0) return PNETGPU_OK;
    if (r->filling < 0 && (r->filling = take_free_slot(r)) < 0) return PNETGPU_EBUSY;
    Slot& s = r->slots[r->filling];
    if (s.n) return PNETGPU_EFULL;               // pushed frames are waiting: submit them first
    // the longest prefix of frames, ascending and non-overlapping, whose span fits the slot
    const uint64_t t_desc = now_ns();
    const uint64_t o0 = offsets[0];
    const uint64_t limit = std::min<uint64_t>(n, r->cap_frames);
    uint64_t k = 0, end = o0, fbytes = 0, large = 0, jumbo = 0;
    uint32_t mx = 0, mn = UINT32_MAX;
    bool irregular = false;
    // the stride a fixed-stride batch would have: frame i at o0 + i * S
    const uint64_t S = limit >= 2 && offsets[1] > o0 ? offsets[1] - o0 : 0;
    auto desc_range = [&](uint64_t lo, uint64_t hi) {   // descriptors + size statistics of [lo, hi)
        PackStats st;
        for (uint64_t i = lo; i < hi; ++i) {
            const uint32_t len = lengths[i];
            s.h_off[i] = offsets[i] - o0;
            s.h_len[i] = len;
            s.h_off32[i] = (uint32_t)(offsets[i] - o0);
            s.h_len16[i] = (uint16_t)len;
            st.max_len = std::max(st.max_len, len);
            st.min_len = std::min(st.min_len, len);
            st.irregular |= offsets[i] - o0 != i * S;
            st.bytes += len;
            st.n_large += len >= pnetgpu::kHintLargeMin;
            st.jumbo_bytes += len >= pnetgpu::kHintJumboMin ? len : 0;
        }
        return st;
    };
    bool done = false;
    const unsigned nt = limit >= (1u << 16) ? pnetgpu::host_threads() : 1u;
    if (nt > 1) {
        // Parallel form (a 64-B batch of 2^20 frames took ~1.4 ms on one thread,
        // the zero-copy producer's whole budget per batch): ascending frames have
        // ascending ends, so the cut is a binary search over the ends; then every
        // chunk of [0, cut] checks the order and the fit (the cut frame: order
        // only) while it writes its descriptors. Any anomaly (an overlap or a
        // descending frame) reruns the serial pass below, whose result is the
        // contract.
        auto fits = [&](uint64_t i) { return offsets[i] >= o0 && offsets[i] + lengths[i] - o0 <= r->cap_bytes; };
        uint64_t lo = 0, hi = limit;                     // largest prefix whose last frame fits
        while (lo < hi) {
            const uint64_t mid = lo + (hi - lo + 1) / 2;
            if (fits(mid - 1)) lo = mid;
            else hi = mid - 1;
        }
        const uint64_t kk = lo, checked = std::min(kk + 1, limit);
        if (kk > 0) {
            std::vector<PackStats> cst(nt);
            std::vector<uint8_t> bad(nt, 0);
            pnetgpu::parallel_run(nt, [&](unsigned t) {
                const uint64_t a = checked * t / nt, b = checked * (t + 1) / nt;
                for (uint64_t i = std::max<uint64_t>(a, 1); i < b; ++i)
                    if (offsets[i] < offsets[i - 1] + lengths[i - 1]) bad[t] = 1;
                for (uint64_t i = a; i < std::min(b, kk); ++i)
                    if (!fits(i)) bad[t] = 1;
                cst[t] = desc_range(a, std::min(b, kk));
            });
            bool ok = true;
            for (unsigned t = 0; t < nt; ++t) ok = ok && !bad[t];
            if (ok) {
                k = kk;
                end = offsets[k - 1] + lengths[k - 1];
                for (const PackStats& c : cst) {
                    mx = std::max(mx, c.max_len);
                    mn = std::min(mn, c.min_len);
                    irregular |= c.irregular;
                    fbytes += c.bytes;
                    large += c.n_large;
                    jumbo += c.jumbo_bytes;
                }
                done = true;
            }
        }
    }
    if (!done) {
        while (k < limit) {
            if (offsets[k] < end) return PNETGPU_EINVAL;   // frames must ascend without overlap
            const uint64_t fe = offsets[k] + lengths[k];
            if (fe - o0 > r->cap_bytes) break;
            end = fe;
            ++k;
        }
        const PackStats st = desc_range(0, k);
        mx = st.max_len;
        mn = st.min_len;
        irregular = st.irregular;
        fbytes = st.bytes;
        large = st.n_large;
        jumbo = st.jumbo_bytes;
    }
    r->stats.push_ns += now_ns() - t_desc;       // the descriptor pass (no frame copies here)
    if (k == 0) return PNETGPU_EFULL;            // the first frame alone exceeds batch_bytes
    s.n = (uint32_t)k;
    s.compact_n = (uint32_t)k;                   // the descriptor pass wrote them all
    s.bytes = end - o0;                          // the span shipped (gaps included)
    s.frame_bytes = fbytes;
    s.max_len = mx;
    s.min_len = mn;
    s.stride = k >= 2 && !irregular && mn == mx && S <= UINT32_MAX ? (uint32_t)S : 0;
    s.n_large = large;
    s.jumbo_bytes = jumbo;
    s.frames_view = base + o0;
    const uint64_t t0 = now_ns();
    const int rc = ship_slot(r, s, base + o0, id);
    r->stats.submit_ns += now_ns() - t0;
    if (rc) {   // nothing shipped: the slot is empty again (its pinned batch never held these frames)
        s.n = 0;
        s.bytes = s.frame_bytes = s.n_large = s.jumbo_bytes = 0;
        s.max_len = s.stride = s.compact_n = 0;
        s.min_len = UINT32_MAX;
        return rc;
    }
    *taken = k;
    return PNETGPU_OK;
}
static void release_held(pnetgpu_ring* r) {
    if (r->held >= 0) {
        r->slots[r->held].state = kFree;
        r->held = -1;
        if (r->filling < 0) r->filling = take_free_slot(r);
    }
}

int pnetgpu_ring_release(pnetgpu_ring* r) {
    if (!r) return PNETGPU_EINVAL;
    release_held(r);
    return PNETGPU_OK;
}

int pnetgpu_ring_wait(pnetgpu_ring* r, pnetgpu_ring_batch* out) {
    pnetgpu::set_last_hip_error(0);
    if (!r || !out) return PNETGPU_EINVAL;
    release_held(r);                             // the previous batch is released now
    if (r->inflight.empty()) return PNETGPU_EEMPTY;
    const int i = r->inflight.front();
    Slot& s = r->slots[i];
    // a failed wait leaves the batch in flight (the next wait tries it again)
    const uint64_t t0 = now_ns();
    const hipError_t e = hipEventSynchronize(s.done);
    r->stats.wait_ns += now_ns() - t0;
    if (e) return pnetgpu::hip_fail(e);
    if (s.timed) {
        float ms[3] = {0, 0, 0};
        bool ok = true;
        for (int k = 0; k < 3 && ok; ++k) ok = hipEventElapsedTime(&ms[k], s.stage[k], s.stage[k + 1]) == hipSuccess;
        if (ok) {
            r->stats.h2d_ms += ms[0];
            r->stats.kernel_ms += ms[1];
            r->stats.d2h_ms += ms[2];
            r->stats.timed_batches += 1;
        }
        s.timed = false;
    }
    r->inflight.pop_front();
    s.state = kHeld;
    r->held = i;
    out->id = s.id;
    out->n_frames = s.n;
    out->frames = s.frames_view;
    out->offsets = s.h_off;
    out->lengths = s.h_len;
    std::memset(&out->cols, 0, sizeof(out->cols));
    for (int k = 0; k < kNumCols; ++k)
        *col_slot(out->cols, k) = (s.col_mask >> k) & 1u ? static_cast<void*>(s.h_rec + s.col_off[k]) : nullptr;
    out->cols.counters = reinterpret_cast<uint64_t*>(s.h_rec);
    return PNETGPU_OK;
}

int pnetgpu_ring_set_columns(pnetgpu_ring* r, uint64_t column_mask) {
    pnetgpu::set_last_hip_error(0);
    if (!r || (column_mask >> kNumCols)) return PNETGPU_EINVAL;
    const size_t need = rec_capacity(r->cap_frames, column_mask);
    bool grow = false;
    Slot* const s0 = r->slots;
    Slot* const s1 = r->slots + r->nslots;
    for (const Slot* s = s0; s != s1; ++s) grow = grow || s->rec_cap < need;
    if (grow) {   // record blocks are resized only while no batch uses them
        for (const Slot* s = s0; s != s1; ++s)
            if (s->state == kInFlight || s->state == kHeld) return PNETGPU_EBUSY;
        if (hipSetDevice(r->device) != hipSuccess) return pnetgpu::hip_fail(hipGetLastError());
        for (Slot* s = s0; s != s1; ++s)
            if (s->rec_cap < need && !alloc_rec(*s, need)) return PNETGPU_ENOMEM;
    }
    r->col_mask = column_mask;
    return PNETGPU_OK;
}

int pnetgpu_ring_stats_get(const pnetgpu_ring* r, pnetgpu_ring_stats* out) {
    if (!r || !out) return PNETGPU_EINVAL;
    *out = r->stats;
    return PNETGPU_OK;
}

int pnetgpu_ring_stats_reset(pnetgpu_ring* r) {
    if (!r) return PNETGPU_EINVAL;
    const uint32_t threads = r->stats.host_threads;
    r->stats = pnetgpu_ring_stats{};
    r->stats.host_threads = threads;
    return PNETGPU_OK;
}

int pnetgpu_host_register(void* p, uint64_t bytes) {
    if (!p || !bytes) return PNETGPU_EINVAL;
    pnetgpu::set_last_hip_error(0);
    const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterDefault);
    return e == hipSuccess ? PNETGPU_OK : pnetgpu::hip_fail(e);
}

int pnetgpu_host_unregister(void* p) {
    if (!p) return PNETGPU_EINVAL;
    pnetgpu::set_last_hip_error(0);
    const hipError_t e = hipHostUnregister(p);
    return e == hipSuccess ? PNETGPU_OK : pnetgpu::hip_fail(e);
}

}  // extern "C"
