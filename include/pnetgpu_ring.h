/*
 * pnetgpu_ring.h — host-side batch producer for the receive engine.
 *
 * The reference hands the application one frame per DataLinkReceiver::next()
 * call (pnet_datalink/src/lib.rs:227-230; Linux AF_PACKET linux.rs:362-403,
 * pcap file replay pcap.rs:92,168-179), and the &[u8] is invalidated by the next
 * call. A pnetgpu_ring is the consumer that turns that stream into GPU batches:
 * pnetgpu_ring_push() copies each frame into a pinned host batch (descriptor
 * mode: offsets + lengths), pnetgpu_ring_submit() ships a full batch
 * asynchronously (hipMemcpyAsync H2D -> pnetgpu_rx_process -> D2H of every
 * result column) on one of the ring's two streams (alternating by submission;
 * created with different priorities, so HIP, which draws hardware queues per
 * priority, never serializes them on one queue),
 * and pnetgpu_ring_wait() hands back the
 * oldest finished batch's records in pinned host memory. Slots rotate (default
 * PNETGPU_RING_DEFAULT_SLOTS: one filling, one held by the application, the
 * rest in flight on alternating streams), so the H2D of one batch overlaps the
 * kernel and D2H of the previous ones and the application's host work.
 *
 * A batch whose frames all have one length at one constant stride (a capture
 * of fixed-size frames, TPACKET frame slots) ships as a fixed-stride batch with
 * no descriptors, wherever the fixed-stride kernel is the one its size hint
 * would pick: frames of <= 64 B on a stride that is a multiple of 16 with no
 * parse extensions (the small kernel), or of >= 768 B (the MTU / jumbo
 * shapes). Any other batch ships compact (u32 / u16) or full descriptors. The
 * records are identical either way; pnetgpu_ring_stats counts which.
 *
 * Validity: a waited batch (its frames and records) stays valid until the next
 * pnetgpu_ring_wait() or pnetgpu_ring_release() on the same ring.
 * Single-threaded use per ring.
 */
#ifndef PNETGPU_RING_H
#define PNETGPU_RING_H

#include <stdint.h>

#include "pnetgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PNETGPU_EFULL   (-5)   /* push: frame does not fit the filling batch -> submit first   */
#define PNETGPU_EBUSY   (-6)   /* push/submit: every slot is in flight or held -> wait first     */
#define PNETGPU_EEMPTY  (-7)   /* wait: nothing in flight; pcap_next: end of file               */
#define PNETGPU_EFORMAT (-8)   /* pcap/pcapng: malformed, or an unsupported link type          */

typedef struct pnetgpu_ring pnetgpu_ring;

/* Host view of one finished batch. Column pointers follow pnetgpu_rx_columns
 * (every column present, pinned host memory, n_frames elements each). */
typedef struct pnetgpu_ring_batch {
    uint64_t            id;         /* submission sequence number, from 0            */
    uint64_t            n_frames;
    const uint8_t*      frames;     /* the batch's frame bytes (pinned host)          */
    const uint64_t*     offsets;    /* frame i = frames[offsets[i], +lengths[i])      */
    const uint32_t*     lengths;
    pnetgpu_rx_columns  cols;       /* host pointers; counters has PNETGPU_NCOUNTERS  */
} pnetgpu_ring_batch;

#define PNETGPU_RING_MIN_SLOTS      2   /* one held + one filling: no batch in flight while held */
#define PNETGPU_RING_DEFAULT_SLOTS  4   /* held + filling + two in flight                         */
#define PNETGPU_RING_MAX_SLOTS     16

/* flags: PNETGPU_RX_* dispatch extensions applied to every batch;
 * PNETGPU_RING_DEFAULT_SLOTS slots of batch_bytes / batch_frames each */
int  pnetgpu_ring_create(pnetgpu_ctx* ctx, uint64_t batch_bytes, uint32_t batch_frames, uint32_t flags,
                         pnetgpu_ring** out);
/* The same with nslots slots (PNETGPU_RING_MIN_SLOTS..PNETGPU_RING_MAX_SLOTS,
 * else PNETGPU_EINVAL): nslots - 2 batches stay in flight while the application
 * holds one and fills another. Each slot pins batch_bytes of host memory and
 * allocates as much device memory. */
int  pnetgpu_ring_create_ex(pnetgpu_ctx* ctx, uint64_t batch_bytes, uint32_t batch_frames, uint32_t flags,
                            uint32_t nslots, pnetgpu_ring** out);
/* Slot count of a ring (0 for NULL). */
uint32_t pnetgpu_ring_slots(const pnetgpu_ring* ring);
void pnetgpu_ring_destroy(pnetgpu_ring* ring);

/* Ring-only create flag (never passed to the kernel): time each batch's device
 * stages with HIP events (H2D of frames + descriptors, receive kernel, D2H of
 * the records), summed in pnetgpu_ring_stats. Costs four event records a batch. */
#define PNETGPU_RING_STAGE_TIMES   0x10000u

/* Where a ring's time went, summed since creation or the last reset. Host times
 * are wall time on the calling thread inside the named calls; device times are
 * per-batch stage durations on the slot streams (they overlap across slots). */
typedef struct pnetgpu_ring_stats {
    uint64_t batches;         /* batches shipped (submit / submit_region)                     */
    uint64_t frames;          /* frames in them                                               */
    uint64_t bytes;           /* bytes shipped host -> device (the frame spans)               */
    uint64_t push_ns;         /* push_many: descriptors + copies; submit_region: descriptors */
    uint64_t submit_ns;       /* inside submit / submit_region: enqueueing H2D, kernel, D2H   */
    uint64_t wait_ns;         /* inside pnetgpu_ring_wait, blocked on the oldest batch        */
    uint64_t timed_batches;   /* batches whose device stages were timed                       */
    uint64_t desc_bytes;      /* descriptor bytes shipped host -> device (none for stride batches) */
    double   h2d_ms;          /* PNETGPU_RING_STAGE_TIMES only: H2D of frames + descriptors   */
    double   kernel_ms;       /*   the receive kernel                                         */
    double   d2h_ms;          /*   D2H of counters + record columns                           */
    uint32_t host_threads;    /* threads push_many's passes use (pnetgpu_host_threads)        */
    uint32_t stride_batches;  /* batches shipped as fixed-stride batches: uniform frames at a
                               * constant stride, no descriptors (pnetgpu_ring_submit)       */
} pnetgpu_ring_stats;
int pnetgpu_ring_stats_get(const pnetgpu_ring* ring, pnetgpu_ring_stats* out);
/* Zero every sum (host_threads is kept). */
int pnetgpu_ring_stats_reset(pnetgpu_ring* ring);

/* Host threads the producers' parallel passes use, the caller included:
 * PNETGPU_HOST_THREADS if set (1..64), else min(16, CPUs in the process's
 * affinity mask, its cgroup CPU quota rounded down). The workers are created
 * once per process, on the first large pass, and sleep between passes. */
uint32_t pnetgpu_host_threads(void);

/* Host batch builder without a ring (no HIP call): copies frames
 * buf[offsets[i], +lengths[i]) back to back into dst (dst_cap bytes), writing
 * dst_offsets[i] / dst_lengths[i], and stops at n frames or when the next frame
 * does not fit: *packed frames, *packed_bytes bytes. PNETGPU_EFULL if the first
 * frame alone exceeds dst_cap. The same pass as pnetgpu_ring_push_many, for a
 * caller staging batches in its own pinned memory for pnetgpu_rx_process. */
int pnetgpu_batch_pack(const uint8_t* buf, const uint64_t* offsets, const uint32_t* lengths, uint64_t n,
                       uint8_t* dst, uint64_t dst_cap, uint64_t* dst_offsets, uint32_t* dst_lengths,
                       uint64_t* packed, uint64_t* packed_bytes);

/* Copy one frame into the filling batch: 0, PNETGPU_EFULL or PNETGPU_EBUSY. */
int pnetgpu_ring_push(pnetgpu_ring* ring, const uint8_t* frame, uint32_t len);
/* Copy n frames (frame i = buf[offsets[i], +lengths[i]) on the host) until the
 * batch is full; *pushed = how many were taken (may be < n: then submit).
 * Frames adjacent in buf are copied by one memcpy, and pushes of >= 2^16 frames
 * are split over pnetgpu_host_threads() threads of a persistent pool
 * (descriptors, the cut where the batch fills and the copies); the batch holds
 * the same frames in the same order as n single pushes would. */
int pnetgpu_ring_push_many(pnetgpu_ring* ring, const uint8_t* buf, const uint64_t* offsets,
                           const uint32_t* lengths, uint64_t n, uint64_t* pushed);
/* Ship the filling batch (no-op returning 0 with *id = UINT64_MAX if empty);
 * pushed frames sit back to back, so uniform ones ship fixed-stride. */
int pnetgpu_ring_submit(pnetgpu_ring* ring, uint64_t* id);
/* Zero-copy submit: ship frames base[offsets[i], +lengths[i]) straight from the
 * caller's memory (one H2D of their span; no copy into the ring's pinned batch).
 * The frames must ascend without overlapping; the longest prefix whose span and
 * count fit the ring's batch is taken (*taken; then call again with the rest).
 * The region must stay unchanged and alive until the batch has been waited, and
 * the waited batch's `frames` points into it (offsets rebased to offsets[0]).
 * With memory registered through pnetgpu_host_register (e.g. an mmap of a pcap
 * file or of an AF_PACKET TPACKET ring) the copy is a direct DMA; pageable memory
 * works too, at the HIP runtime's staged-copy rate. Returns 0, PNETGPU_EBUSY
 * (wait first), PNETGPU_EFULL (frames were pushed into the filling batch: submit
 * them first; or the first frame exceeds batch_bytes) or PNETGPU_EINVAL. */
int pnetgpu_ring_submit_region(pnetgpu_ring* ring, const uint8_t* base, const uint64_t* offsets,
                               const uint32_t* lengths, uint64_t n, uint64_t* taken, uint64_t* id);
/* Columns later submissions compute and copy back: bit k selects the k-th
 * column of pnetgpu_rx_columns in struct order, counters not counted (status =
 * bit 0 ... l3_offset = bit 15, eth_dst = bit 16 ... icmp_sequence = bit 37);
 * default the 16 record columns (0xFFFF). A waited batch's unselected columns
 * are NULL. Fewer columns = fewer result bytes over PCIe (bits 0-15: 61 B/frame;
 * the IPv4 set, bits 0-11: 26 B/frame; all 38: 114 B/frame). Growing the record
 * returns PNETGPU_EBUSY while a batch is in flight or held. */
int pnetgpu_ring_set_columns(pnetgpu_ring* ring, uint64_t column_mask);
/* column_mask bits: the 16 record columns, then the header-field columns */
#define PNETGPU_COLS_RECORD            0xFFFFull     /* status ... l3_offset (the default) */
#define PNETGPU_COLS_IPV4_RECORD       0x0FFFull     /* status ... dst_ipv4: 26 B/frame   */
#define PNETGPU_COL_ETH_DST            (1ull << 16)
#define PNETGPU_COL_ETH_SRC            (1ull << 17)
#define PNETGPU_COL_IP_VERSION         (1ull << 18)
#define PNETGPU_COL_IP_HEADER_LENGTH   (1ull << 19)
#define PNETGPU_COL_IP_DSCP            (1ull << 20)
#define PNETGPU_COL_IP_ECN             (1ull << 21)
#define PNETGPU_COL_IP_TOTAL_LENGTH    (1ull << 22)
#define PNETGPU_COL_IP_IDENTIFICATION  (1ull << 23)
#define PNETGPU_COL_IP_FLAGS           (1ull << 24)
#define PNETGPU_COL_IP_FRAGMENT_OFFSET (1ull << 25)
#define PNETGPU_COL_IP6_TRAFFIC_CLASS  (1ull << 26)
#define PNETGPU_COL_IP6_FLOW_LABEL     (1ull << 27)
#define PNETGPU_COL_IP6_PAYLOAD_LENGTH (1ull << 28)
#define PNETGPU_COL_UDP_LENGTH         (1ull << 29)
#define PNETGPU_COL_TCP_SEQUENCE       (1ull << 30)
#define PNETGPU_COL_TCP_ACKNOWLEDGEMENT (1ull << 31)
#define PNETGPU_COL_TCP_DATA_OFFSET    (1ull << 32)
#define PNETGPU_COL_TCP_RESERVED       (1ull << 33)
#define PNETGPU_COL_TCP_FLAGS          (1ull << 34)
#define PNETGPU_COL_TCP_WINDOW         (1ull << 35)
#define PNETGPU_COL_TCP_URGENT_PTR     (1ull << 36)
#define PNETGPU_COL_ICMP_SEQUENCE      (1ull << 37)
/* Page-lock existing host memory for direct DMA (hipHostRegister) and undo it. */
int pnetgpu_host_register(void* p, uint64_t bytes);
int pnetgpu_host_unregister(void* p);
/* Block for the oldest submitted batch: 0 (fills *out) or PNETGPU_EEMPTY.
 * Releases the batch the previous wait returned. */
int pnetgpu_ring_wait(pnetgpu_ring* ring, pnetgpu_ring_batch* out);
/* Release the batch the last wait returned now (its views become invalid), so
 * its slot can take frames before the next wait: a consumer that is done with a
 * batch releases it and keeps filling while the other slots are in flight. No-op
 * when nothing is held. */
int pnetgpu_ring_release(pnetgpu_ring* ring);

/* Capture-file reader (the pcap.rs:92 from_file receiver, which reads through
 * libpcap's offline reader): classic pcap (microsecond or nanosecond magic,
 * either byte order) and pcapng (sections in either byte order; Enhanced,
 * Simple and obsolete Packet Blocks; every interface of the file with the first
 * one's link type, as libpcap requires; other block types skipped). The
 * streaming reader takes LINKTYPE_ETHERNET. next() returns the captured bytes
 * of each record, valid until the following call. */
typedef struct pnetgpu_pcap pnetgpu_pcap;
int  pnetgpu_pcap_open(const char* path, pnetgpu_pcap** out);
int  pnetgpu_pcap_next(pnetgpu_pcap* p, const uint8_t** frame, uint32_t* len);
void pnetgpu_pcap_close(pnetgpu_pcap* p);
/* Index an in-memory capture image, classic pcap or pcapng (e.g. an mmap of the whole file) for
 * pnetgpu_ring_submit_region: from byte *pos (0 = start of file) fill up to cap
 * record descriptors (offset of each record's captured bytes in img, its
 * captured length), *n = records found, *pos = where the next call resumes
 * (img_bytes at the end; for pcapng a block boundary). pcapng's section state
 * at *pos comes from the blocks before it: a call that continues the calling
 * thread's previous scan (same img and img_bytes, *pos where that call
 * stopped, and the same first 28 bytes and block header at *pos) resumes with
 * the state it stopped with, any other call re-reads the block headers before
 * *pos — so an image must not be rewritten in place between the calls of one
 * scan except from its first bytes on. PNETGPU_EFORMAT for a bad
 * header, an unsupported link type, a truncated record or block, or (pcapng)
 * a block whose two length fields differ or a packet naming an undescribed
 * interface. Link types: Ethernet (1) and raw IP (101, 228, 229) — check
 * pnetgpu_pcap_info for the receive flags the records need. */
int pnetgpu_pcap_scan(const uint8_t* img, uint64_t img_bytes, uint64_t* pos, uint64_t* offsets, uint32_t* lengths,
                      uint64_t cap, uint64_t* n);
/* The image's link type and the pnetgpu_batch / ring flags its records need:
 * LINKTYPE_ETHERNET (1) -> 0; LINKTYPE_RAW (101), LINKTYPE_IPV4 (228),
 * LINKTYPE_IPV6 (229) -> PNETGPU_RX_L3 (frames begin at the IP header).
 * PNETGPU_EFORMAT for any other link type or a bad header. */
int pnetgpu_pcap_info(const uint8_t* img, uint64_t img_bytes, uint32_t* linktype, uint32_t* rx_flags);

#ifdef __cplusplus
}
#endif
#endif
