/*
 * pnetgpu.h — C-ABI of the MI355X packet parse-and-checksum engine.
 *
 * This is the drop-in boundary for libpnet's per-packet receive hot path
 * (SURVEY.md §8(b)). Plain pointers and sizes only: no HIP, torch or C++
 * types in any signature (streams are passed as `void*` = hipStream_t).
 *
 * Which reference interface each entry point replaces:
 *
 *   pnetgpu_rx_process        the per-frame receive chain a libpnet user runs on
 *                             every `DataLinkReceiver::next()` frame
 *                             (pnet_datalink/src/lib.rs:227-230):
 *                             EthernetPacket::new → get_ethertype →
 *                             Ipv4Packet::new / Ipv6Packet::new → ipv4::checksum →
 *                             payload() → UdpPacket/TcpPacket/IcmpPacket::new →
 *                             udp|tcp::ipv4_checksum / ipv6_checksum, icmp::checksum,
 *                             icmpv6::checksum  — examples/packetdump.rs:120-217,
 *                             pnet_packet/src/ipv4.rs:165-178, udp.rs:34-56,104-126,
 *                             tcp.rs:239-286, icmp.rs:70-75, icmpv6.rs:80-85,
 *                             generated accessors pnet_macros/src/decorator.rs:1563-1670,
 *                             payload bounds decorator.rs:713-769.
 *   pnetgpu_tx_fill_checksums the sender side: set_checksum(ipv4::checksum(..)),
 *                             set_checksum(udp|tcp::ipv4_checksum(..)) etc. as
 *                             benches/rs_sender.rs:38-39,70-71 does per frame.
 *   pnetgpu_checksum_slices   pnet_packet::util::checksum (pnet_packet/src/util.rs:76-82),
 *                             re-exported as pnet::util::checksum (src/util.rs:11-12),
 *                             over a batch of slices; _compact: 8-B descriptors;
 *                             _strided: uniform slices without descriptor arrays.
 *   pnetgpu_ipv4_checksum_slices  pnet_packet::util::ipv4_checksum with empty
 *                             extra_data (util.rs:92-117), batched.
 *   pnetgpu_ipv6_checksum_slices  pnet_packet::util::ipv6_checksum with empty
 *                             extra_data (util.rs:125-150), batched.
 *   pnetgpu_ipv4|ipv6_checksum_adv_slices  the same with extra_data: the
 *                             udp|tcp::*_checksum_adv wrappers (udp.rs:45-56,115-126,
 *                             tcp.rs:250-261,275-286).
 *
 * Semantics are bit-exact with the reference: every
 * checksum word and extracted field equals what the Rust code returns for the
 * same bytes, including its clamps and saturations (IHL clamp, payload bounds
 * min(start+len, buffer), odd trailing byte as high byte, skipped word).
 *
 * Conventions
 *   - Return: 0 on success, a negative PNETGPU_E* code otherwise. No exceptions
 *     cross the ABI. Work is enqueued on `stream` (NULL = the device's null
 *     stream) and is complete only once that stream is synchronised.
 *   - Ownership: the caller owns every buffer; the library never frees caller
 *     memory. Device pointers must be device-accessible on the context's GPU.
 *   - Granule rule: the engine reads frame bytes in aligned 16-byte granules,
 *     so the allocation behind `data` must be readable up to
 *     round_up(data + data_bytes, 16). (hipMalloc'd buffers always are.)
 *   - Threading: a context is bound to one device; calls on one context may be
 *     issued from one host thread at a time. Distinct contexts are independent.
 *     Any number of launches may be in flight, on any streams, and launches
 *     may be captured into HIP graphs and replayed: a launch that balances its
 *     runs by claims (run scheduling) holds a counter block of
 *     the context's pool that no unfinished launch holds, whatever the streams
 *     (its last wave hands the block back, zeroed, through pinned host
 *     memory); with all 64 blocks held, and for every launch captured into a
 *     graph, the launch runs the static schedule — the same results without
 *     claims (pnetgpu_ctx_sched_stats counts each case). No launch can see
 *     another's counters, so destroyed and reused stream handles need no care.
 *   - Malformed input never faults: frames whose descriptor falls outside
 *     [0, data_bytes) get PNET_ST_DESC_INVALID, short frames get the
 *     *_MALFORMED bits (the reference's `new()` returning None).
 */
#ifndef PNETGPU_H
#define PNETGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PNETGPU_ABI_VERSION 3

/* ---- return codes ------------------------------------------------------- */
#define PNETGPU_OK        0
#define PNETGPU_EINVAL   (-1)  /* bad argument (NULL, size overflow, ...)      */
#define PNETGPU_ENODEV   (-2)  /* no HIP device / device index out of range    */
#define PNETGPU_EHIP     (-3)  /* a HIP runtime call or kernel launch failed   */
#define PNETGPU_ENOMEM   (-4)

/* ---- per-frame status word (rx columns .status) ------------------------- */
#define PNET_ST_L3_MASK           0x0003u  /* 1 = IPv4 (ethertype 0x0800), 2 = IPv6 (0x86DD) */
#define PNET_ST_L3_IPV4           0x0001u
#define PNET_ST_L3_IPV6           0x0002u
#define PNET_ST_L4_SHIFT          2
#define PNET_ST_L4_MASK           0x001Cu  /* dispatch on next_level_protocol / next_header */
#define PNET_ST_L4_UDP            (1u << PNET_ST_L4_SHIFT)  /* 17 */
#define PNET_ST_L4_TCP            (2u << PNET_ST_L4_SHIFT)  /* 6  */
#define PNET_ST_L4_ICMP           (3u << PNET_ST_L4_SHIFT)  /* 1  */
#define PNET_ST_L4_ICMPV6         (4u << PNET_ST_L4_SHIFT)  /* 58 */
#define PNET_ST_ETH_MALFORMED     0x0020u  /* EthernetPacket::new == None (len < 14)   */
#define PNET_ST_L3_MALFORMED      0x0040u  /* Ipv4Packet::new (< 20) / Ipv6Packet::new (< 40) == None */
#define PNET_ST_L4_MALFORMED      0x0080u  /* Udp (< 8) / Tcp (< 20) / Icmp(v6) (< 4) new == None */
#define PNET_ST_IP_CSUM_OK        0x0100u  /* ipv4::checksum(&ip) == ip.get_checksum() */
#define PNET_ST_L4_CSUM_DONE      0x0200u  /* an L4 checksum was computed (l4_csum valid) */
#define PNET_ST_L4_CSUM_OK        0x0400u  /* computed L4 checksum == stored field       */
#define PNET_ST_UNKNOWN_ETHERTYPE 0x0800u
#define PNET_ST_UNKNOWN_PROTO     0x1000u
#define PNET_ST_VLAN              0x2000u  /* PNETGPU_RX_VLAN: one or more VLAN tags were peeled */
#define PNET_ST_FRAGMENT          0x4000u  /* PNETGPU_RX_IPV6_EXT: non-first IPv6 fragment, no L4 */
#define PNET_ST_DESC_INVALID      0x8000u  /* descriptor outside [0, data_bytes): not read */

/* ---- opt-in dispatch extensions (pnetgpu_batch.flags) --------------------
 * The reference's receive chain (packetdump.rs) dispatches Ethernet -> IP
 * directly. These flags follow the reference's other views first:
 *   PNETGPU_RX_VLAN      up to two VlanPacket views (vlan.rs:62-72) for
 *                        ethertypes 0x8100 / 0x88A8 / 0x9100 (ethernet.rs:102-112);
 *                        a truncated tag (< 4 B) sets VLAN | L3_MALFORMED.
 *   PNETGPU_RX_IPV6_EXT  up to four IPv6 extension headers (ipv6.rs:39-137):
 *                        Hop-by-Hop 0 / Destination 60 / Routing 43 (length
 *                        hdr_ext_len*8+8), Fragment 44 (8 B; a fragment with
 *                        offset (value & ~3) != 0 sets FRAGMENT and stops); a
 *                        truncated header sets L4_MALFORMED. ip_proto reports
 *                        the protocol after the walk; the L4 pseudo-header uses
 *                        the base header's addresses and the L4 slice length.
 *   PNETGPU_RX_L3        frames begin at the IP header (pnet_transport's Layer3
 *                        receive, pnet_transport/src/lib.rs:342-374, and raw-IP
 *                        captures): no Ethernet header; the version nibble picks
 *                        the chain (4 -> Ipv4Packet, 6 -> Ipv6Packet), anything
 *                        else or an empty frame sets UNKNOWN_ETHERTYPE. ethertype
 *                        reports 0x0800 / 0x86DD (0 otherwise), l3_offset 0;
 *                        PNETGPU_RX_VLAN has no effect. */
#define PNETGPU_RX_VLAN           0x1u
#define PNETGPU_RX_IPV6_EXT       0x2u
#define PNETGPU_RX_L3             0x4u

/* Compact descriptors (descriptor mode; ignored with stride > 0): `offsets`
 * points to uint32_t[n_frames] and `lengths` to uint16_t[n_frames] (cast to
 * the fields' types) — 6 B per frame instead of 12, the layout SURVEY.md
 * §8(b) suggested. For batches under 4 GiB with frames under 64 KiB; the
 * pinned ring (pnetgpu_ring.h) uses it whenever a batch qualifies. */
#define PNETGPU_DESC_COMPACT      0x100u

/* Frame-size hints (descriptor mode; ignored with stride > 0). A descriptor
 * batch's lengths are device-resident, so the library cannot see its size mix
 * and runs the mixed shape (built for IMIX-like batches). A caller that knows
 * its frames (the pinned ring does, from the lengths it pushes) may name the
 * shape the fixed-stride kinds use: measured on one MI355X box
 * (profiles/r05/shape/), packed 1500-B frames 0.33 ms mixed -> 0.28 ms MTU,
 * 9000-B frames 0.205 -> 0.176 ms jumbo, 64-B/9000-B frames at 7:1 0.122 ->
 * 0.109 ms jumbo — but IMIX 0.34 ms mixed -> 0.58 ms MTU, 1.29 ms jumbo, so
 * the hint must describe the batch. Without a hint the mixed shape streams
 * each run of 64 frames that are all 768 B - 4 KiB in the MTU order, and each
 * run of frames all >= 4 KiB in the jumbo order (1500-B frames 0.283 ms,
 * 9000-B 0.178 ms, profiles/r05/uni_runs/); the hint still saves the run
 * checks. Records are identical whatever the hint.
 * pnetgpu_desc_size_hint computes it from host-side lengths. */
#define PNETGPU_DESC_HINT_LARGE   0x200u  /* (nearly) every frame >= 768 B: the MTU shape       */
#define PNETGPU_DESC_HINT_JUMBO   0x400u  /* most bytes in frames >= 4 KiB: the jumbo shape      */

/* ---- batch-wide counters (rx columns .counters, uint64 each, accumulated) */
#define PNETGPU_CTR_FRAMES        0  /* frames with a valid descriptor            */
#define PNETGPU_CTR_BYTES         1  /* sum of their lengths                      */
#define PNETGPU_CTR_IPV4          2
#define PNETGPU_CTR_IPV6          3
#define PNETGPU_CTR_IP_CSUM_BAD   4  /* IPv4 parsed and header checksum mismatch  */
#define PNETGPU_CTR_L4_CSUM_BAD   5  /* L4 checksum computed and mismatch         */
#define PNETGPU_CTR_MALFORMED     6  /* any *_MALFORMED or DESC_INVALID           */
#define PNETGPU_CTR_UNKNOWN       7  /* unknown ethertype or protocol             */
#define PNETGPU_NCOUNTERS         8

typedef struct pnetgpu_ctx pnetgpu_ctx;

/*
 * A batch of Ethernet frames (no FCS) resident in device memory.
 *   stride > 0 : fixed-stride mode, frame i = data[first_offset + i*stride, +frame_len)
 *   stride == 0: descriptor mode,  frame i = data[offsets[i], +lengths[i])
 */
typedef struct pnetgpu_batch {
    const uint8_t*  data;         /* device pointer to frame bytes                 */
    uint64_t        data_bytes;   /* bytes of `data` frames may occupy             */
    uint64_t        n_frames;
    uint64_t        first_offset; /* stride mode only                              */
    uint32_t        stride;       /* > 0 selects fixed-stride mode                 */
    uint32_t        frame_len;    /* stride mode: length of every frame            */
    const uint64_t* offsets;      /* descriptor mode: device array [n_frames]      */
    const uint32_t* lengths;      /* descriptor mode: device array [n_frames]      */
    uint32_t        flags;        /* PNETGPU_RX_* dispatch extensions (0 = reference chain) */
    uint32_t        reserved;     /* must be 0                                     */
} pnetgpu_batch;

/*
 * Result columns (struct of arrays, one element per frame, device pointers).
 * Any column may be NULL (not written). Field values are those of the
 * reference's generated getters for the view the dispatch reached, 0 otherwise.
 */
typedef struct pnetgpu_rx_columns {
    uint16_t* status;     /* PNET_ST_* bits                                        */
    uint16_t* ip_csum;    /* ipv4::checksum(&ip) (IPv4 only)                       */
    uint16_t* l4_csum;    /* udp/tcp ipv4|ipv6_checksum, icmp::checksum, icmpv6::checksum */
    uint16_t* ethertype;  /* EthernetPacket::get_ethertype (inner one past VLAN tags) */
    uint8_t*  ip_proto;   /* get_next_level_protocol (v4) / get_next_header (v6)   */
    uint8_t*  ttl;        /* get_ttl (v4) / get_hop_limit (v6)                     */
    uint16_t* l4_offset;  /* frame offset of ip.payload() (0 when it is empty)     */
    uint16_t* l4_length;  /* ip.payload().len()                                    */
    uint16_t* src_port;   /* UDP/TCP get_source; ICMP(v6): type<<8 | code          */
    uint16_t* dst_port;   /* UDP/TCP get_destination; ICMP(v6): BE16 at +4 if len>=8 */
    uint32_t* src_ipv4;   /* get_source octets as a big-endian-valued u32          */
    uint32_t* dst_ipv4;
    uint8_t*  src_ipv6;   /* [n_frames][16] Ipv6 get_source octets (16-B aligned)   */
    uint8_t*  dst_ipv6;   /* [n_frames][16]                                        */
    uint16_t* vlan_tci;   /* outer VlanPacket TCI (pcp|dei|vid) when PNET_ST_VLAN  */
    uint8_t*  l3_offset;  /* frame offset of the IP header (14, or 18/22 past tags) */
    uint64_t* counters;   /* [PNETGPU_NCOUNTERS], atomically accumulated           */
    /* ---- header-field columns (ABI v3): the remaining generated getters of
     * each view, written only when requested. A column is 0 for a frame whose
     * dispatch did not construct that view (its new() returned None or was
     * never called). Multi-bit fields are the getters' values, not raw bytes. */
    uint64_t* eth_dst;             /* EthernetPacket get_destination: MacAddr octets as a BE-valued u48  (ethernet.rs:20-30) */
    uint64_t* eth_src;             /* EthernetPacket get_source                                         */
    uint8_t*  ip_version;          /* Ipv4Packet / Ipv6Packet get_version (u4)          (ipv4.rs:140, ipv6.rs:23) */
    uint8_t*  ip_header_length;    /* Ipv4 get_header_length (u4, the raw IHL)          (ipv4.rs:141)     */
    uint8_t*  ip_dscp;             /* Ipv4 get_dscp (u6)                                (ipv4.rs:142)     */
    uint8_t*  ip_ecn;              /* Ipv4 get_ecn (u2)                                 (ipv4.rs:143)     */
    uint16_t* ip_total_length;     /* Ipv4 get_total_length                             (ipv4.rs:144)     */
    uint16_t* ip_identification;   /* Ipv4 get_identification                           (ipv4.rs:145)     */
    uint8_t*  ip_flags;            /* Ipv4 get_flags (u3)                               (ipv4.rs:146)     */
    uint16_t* ip_fragment_offset;  /* Ipv4 get_fragment_offset (u13be)                  (ipv4.rs:147)     */
    uint8_t*  ip6_traffic_class;   /* Ipv6 get_traffic_class (u8 across the nibbles)    (ipv6.rs:24)      */
    uint32_t* ip6_flow_label;      /* Ipv6 get_flow_label (u20be)                       (ipv6.rs:25)      */
    uint16_t* ip6_payload_length;  /* Ipv6 get_payload_length                           (ipv6.rs:26)      */
    uint16_t* udp_length;          /* UdpPacket get_length                              (udp.rs:27)       */
    uint32_t* tcp_sequence;        /* TcpPacket get_sequence                            (tcp.rs:59)       */
    uint32_t* tcp_acknowledgement; /* TcpPacket get_acknowledgement                     (tcp.rs:60)       */
    uint8_t*  tcp_data_offset;     /* TcpPacket get_data_offset (u4)                    (tcp.rs:61)       */
    uint8_t*  tcp_reserved;        /* TcpPacket get_reserved (u4)                       (tcp.rs:62)       */
    uint8_t*  tcp_flags;           /* TcpPacket get_flags (u8)                          (tcp.rs:63)       */
    uint16_t* tcp_window;          /* TcpPacket get_window                              (tcp.rs:64)       */
    uint16_t* tcp_urgent_ptr;      /* TcpPacket get_urgent_ptr                          (tcp.rs:66)       */
    uint16_t* icmp_sequence;       /* Icmp(v6) echo get_sequence_number: BE16 at +6 for the echo types
                                    * only (ICMP 0/8, ICMPv6 128/129) when the slice holds >= 8 B, the
                                    * EchoRequest/EchoReply view (icmp.rs:221-232,303-314; icmpv6.rs:837-995);
                                    * 0 for every other type. Its identifier is dst_port                  */
} pnetgpu_rx_columns;

int         pnetgpu_abi_version(void);
const char* pnetgpu_strerror(int code);
/* The hipError_t behind the last PNETGPU_EHIP a kernel launch returned on the
 * calling thread (0 if none); PNETGPU_DEBUG=1 also prints it to stderr. */
int         pnetgpu_last_hip_error(void);
/* The kernel the last pnetgpu_rx_process / pnetgpu_tx_fill_checksums /
 * pnetgpu_*_slices launch on the calling thread used, named as rocprofv3 names
 * it (e.g. "rx_kernel<8, 4, 8, false, 0, true, false, false>",
 * "slice_tiny_kernel<true>"; "" before any launch): what a profile's kernel
 * row is, for measurement records. Static storage. */
const char* pnetgpu_last_rx_kernel(void);
int         pnetgpu_device_count(int* count);

int  pnetgpu_ctx_create(int device, pnetgpu_ctx** out);
void pnetgpu_ctx_destroy(pnetgpu_ctx* ctx);

/* ---- per-context tuning -------------------------------------------------
 * The kernels' measured defaults can be overridden per
 * context, for tests and measurement tools. Each key is read from the
 * environment variable PNETGPU_<NAME> once, in pnetgpu_ctx_create, and is
 * never re-read on a call: afterwards only pnetgpu_ctx_set_tuning changes it.
 * A value of -1 restores the default. */
#define PNETGPU_TUNE_RX_KIND             0  /* non-small receive batches: 0 mixed, 2 MTU, 3 jumbo shape   */
#define PNETGPU_TUNE_BLOCKS_PER_CU       1  /* receive grid: resident blocks per CU (> 0)                  */
#define PNETGPU_TUNE_STATIC_PCT          2  /* share of runs taken in grid-stride order, 0..100 (100: no claims; default 88) */
#define PNETGPU_TUNE_CLAIM_COUNTERS      3  /* claim counters per launch, 1..128 (default 64)              */
#define PNETGPU_TUNE_SLICE_BLOCKS_PER_CU 4  /* slice grids: resident blocks per CU (> 0)                   */
#define PNETGPU_TUNE_SLICE_KERNEL        5  /* descriptor slices: 1 slice_run_kernel, 2 slice_kernel,
                                             * 3 slice_tiny_kernel (util::checksum batches; others: 1)    */
#define PNETGPU_TUNE_SLICE_DENSE_SPAN    6  /* bytes a run of small slices must span to be LDS-staged (default 2048) */
#define PNETGPU_TUNE_DEBUG               7  /* 1: log each receive call's kernel and grid to stderr        */
#define PNETGPU_TUNE_SCHED_EPOCH         8  /* retired (per-stream epochs, ABI v3 before the counter pool):
                                             * 0..2^32-1 accepted and ignored                                 */
#define PNETGPU_NTUNE                    9
int pnetgpu_ctx_set_tuning(pnetgpu_ctx* ctx, int key, int64_t value);
int pnetgpu_ctx_get_tuning(const pnetgpu_ctx* ctx, int key, int64_t* value);

/* Kept for ABI v3 callers: claims that saw another launch's counters. Launches
 * never share counters (each holds its own pool block), so *count is always 0;
 * no device synchronisation. */
int pnetgpu_ctx_sched_conflicts(pnetgpu_ctx* ctx, uint64_t* count);

/* Run-scheduling counts of a context since its creation (host-side, no
 * synchronisation): stats[PNETGPU_SCHED_CLAIMED] launches that took a counter
 * block; [PNETGPU_SCHED_STATIC_BUSY] launches that ran static because every
 * block was held by an unfinished launch; [PNETGPU_SCHED_STATIC_CAPTURED]
 * launches captured into a graph (static by design); [PNETGPU_SCHED_BLOCKS_HELD]
 * blocks held right now; [PNETGPU_SCHED_BLOCKS] the pool size. Launches too
 * short to claim (fewer than 8 runs per wave, or STATIC_PCT 100) are in none. */
#define PNETGPU_SCHED_CLAIMED          0
#define PNETGPU_SCHED_STATIC_BUSY      1
#define PNETGPU_SCHED_STATIC_CAPTURED  2
#define PNETGPU_SCHED_BLOCKS_HELD      3
#define PNETGPU_SCHED_BLOCKS           4
#define PNETGPU_NSCHED_STATS           5
int pnetgpu_ctx_sched_stats(const pnetgpu_ctx* ctx, uint64_t stats[PNETGPU_NSCHED_STATS]);

/* The PNETGPU_DESC_HINT_* flag for a descriptor batch with these host-side
 * lengths: JUMBO when frames of >= 4096 B carry >= 80 % of the bytes, LARGE
 * when >= 15/16 of the frames are >= 768 B, else 0 (the mixed shape). Host
 * arithmetic over the lengths only (no device work); n = 0 gives 0. */
uint32_t pnetgpu_desc_size_hint(const uint32_t* lengths, uint64_t n);

/* Receive path: parse + verify every frame of `batch`, write `cols`. */
int pnetgpu_rx_process(pnetgpu_ctx* ctx, const pnetgpu_batch* batch,
                       const pnetgpu_rx_columns* cols, void* stream);

/* Transmit side: for every checksum the receive path computes (IPv4 header;
 * UDP/TCP over IPv4/IPv6; ICMP; ICMPv6 over IPv6), write the computed value
 * big-endian into the frame's stored field, in place — the
 * MutableIpv4Packet/MutableUdpPacket/... set_checksum(checksum(..)) calls of the
 * reference's packet builders (benches/rs_sender.rs:38-39,70-71; setters
 * pnet_macros/src/decorator.rs:1490-1530). `batch->data` must be writable and
 * frames must not overlap. `cols` (optional columns) report the frames as they
 * were BEFORE patching (status OK bits = "was already correct"). */
int pnetgpu_tx_fill_checksums(pnetgpu_ctx* ctx, const pnetgpu_batch* batch,
                              const pnetgpu_rx_columns* cols, void* stream);

/* out[i] = util::checksum(data[offsets[i], +lengths[i]), skipwords[i]).
 * Every *_slices entry point returns what a release build of the reference
 * returns for any slice length: its u32 sums wrap modulo 2^32 once a slice
 * (+ extra slice) passes 64 KiB (a debug build panics there instead). */
int pnetgpu_checksum_slices(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes,
                            uint64_t n, const uint64_t* offsets, const uint32_t* lengths,
                            const uint32_t* skipwords, uint16_t* out, void* stream);

/* Compact slice descriptor (8 B instead of the 16 B of the three arrays): for
 * buffers under 4 GiB and slices under 64 KiB. */
typedef struct pnetgpu_slice_desc {
    uint32_t offset;     /* slice start, bytes from `data`  */
    uint16_t length;     /* slice bytes                     */
    uint16_t skipword;   /* util::checksum's skipword       */
} pnetgpu_slice_desc;

/* out[i] = util::checksum(data[desc[i].offset, +desc[i].length), desc[i].skipword):
 * pnetgpu_checksum_slices with compact descriptors (one 8-B load per slice). */
int pnetgpu_checksum_slices_compact(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes,
                                    uint64_t n, const pnetgpu_slice_desc* desc, uint16_t* out,
                                    void* stream);

/* out[i] = util::checksum(data[first_offset + i*stride, +slice_len), skipword) for
 * i < n: uniform slices with no descriptor arrays (the reference's own bench
 * shape, pnet_packet/benches/checksum_benchmarks.rs:8-18, batched). Every
 * slice must lie inside [0, data_bytes) (else PNETGPU_EINVAL); slices may
 * overlap (stride < slice_len) and stride 0 repeats one slice. */
int pnetgpu_checksum_slices_strided(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes,
                                    uint64_t n, uint64_t first_offset, uint32_t stride,
                                    uint32_t slice_len, uint32_t skipword, uint16_t* out, void* stream);

/* out[i] = util::ipv4_checksum(slice_i, skipwords[i], &[], src_i, dst_i, protos[i]);
 * addrs: [n][8] = src octets || dst octets. */
int pnetgpu_ipv4_checksum_slices(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes,
                                 uint64_t n, const uint64_t* offsets, const uint32_t* lengths,
                                 const uint32_t* skipwords, const uint8_t* addrs,
                                 const uint8_t* protos, uint16_t* out, void* stream);

/* out[i] = util::ipv6_checksum(slice_i, skipwords[i], &[], src_i, dst_i, protos[i]);
 * addrs: [n][32] = src octets || dst octets. */
int pnetgpu_ipv6_checksum_slices(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes,
                                 uint64_t n, const uint64_t* offsets, const uint32_t* lengths,
                                 const uint32_t* skipwords, const uint8_t* addrs,
                                 const uint8_t* protos, uint16_t* out, void* stream);

/* The *_adv forms: util::ipv4_checksum / ipv6_checksum with a non-empty
 * extra_data slice per item (udp|tcp::ipv4_checksum_adv / ipv6_checksum_adv,
 * udp.rs:45-56,115-126, tcp.rs:250-261,275-286): extra slice i =
 * data[extra_offsets[i], +extra_lengths[i]), summed from its own start; an
 * odd-length extra drops its trailing byte (util.rs:114, udp.rs:42-44) while
 * the pseudo-header length counts it. */
int pnetgpu_ipv4_checksum_adv_slices(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes,
                                     uint64_t n, const uint64_t* offsets, const uint32_t* lengths,
                                     const uint32_t* skipwords, const uint64_t* extra_offsets,
                                     const uint32_t* extra_lengths, const uint8_t* addrs,
                                     const uint8_t* protos, uint16_t* out, void* stream);
int pnetgpu_ipv6_checksum_adv_slices(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes,
                                     uint64_t n, const uint64_t* offsets, const uint32_t* lengths,
                                     const uint32_t* skipwords, const uint64_t* extra_offsets,
                                     const uint32_t* extra_lengths, const uint8_t* addrs,
                                     const uint8_t* protos, uint16_t* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PNETGPU_H */
