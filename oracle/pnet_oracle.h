/*
 * pnet_oracle.h — CPU restatement of libpnet's per-packet receive path.
 *
 * TEST INFRASTRUCTURE ONLY. This is the parity oracle: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker (or as the timed CPU baseline). The product path
 * (libpnet_amd / libpnetgpu.so) never links, loads or calls anything here.
 *
 * It restates, scalar and literal, the semantics of the Rust reference
 * (libpnet v0.35.0 under /root/reference, which cannot be compiled here:
 * no Rust toolchain in the image — see DESIGN.md "Oracle"):
 *
 *   pnet_packet/src/util.rs:76-181     checksum / finalize / ipv4_checksum /
 *                                      ipv6_checksum / sum_be_words
 *   pnet_packet/src/ipv4.rs:138-178    Ipv4 layout + ipv4::checksum (IHL clamp)
 *   pnet_packet/src/ipv4.rs:226-243    options / payload length functions
 *   pnet_packet/src/ipv6.rs:21-37      Ipv6 layout (payload bounded by payload_length)
 *   pnet_packet/src/udp.rs:23-56,104-126   Udp layout + checksums (skipword 3)
 *   pnet_packet/src/tcp.rs:55-71,227-286   Tcp layout + checksums (skipword 8)
 *   pnet_packet/src/icmp.rs:55-75      Icmp layout + checksum (skipword 1)
 *   pnet_packet/src/icmpv6.rs:68-85    Icmpv6 checksum (IPv6 pseudo-header, skipword 1)
 *   pnet_packet/src/ethernet.rs:20-30  Ethernet layout
 *   pnet_macros/src/decorator.rs:593-600   new(): None below minimum_packet_size
 *   pnet_macros/src/decorator.rs:713-769   payload(): [start, min(end,len)), empty if len<=start
 *   examples/packetdump.rs:120-217     receive dispatch chain
 *
 * Parity pinning: every known-answer vector in the reference's own tests
 * (tests/golden/reference_kats.json, see tests/test_oracle_kat.py).
 */
#ifndef PNET_ORACLE_H
#define PNET_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status word — identical values to include/pnetgpu.h (checked by a CPU test) */
#define ORACLE_ST_L3_IPV4          0x0001u
#define ORACLE_ST_L3_IPV6          0x0002u
#define ORACLE_ST_L4_SHIFT         2
#define ORACLE_ST_L4_UDP           (1u << ORACLE_ST_L4_SHIFT)
#define ORACLE_ST_L4_TCP           (2u << ORACLE_ST_L4_SHIFT)
#define ORACLE_ST_L4_ICMP          (3u << ORACLE_ST_L4_SHIFT)
#define ORACLE_ST_L4_ICMPV6        (4u << ORACLE_ST_L4_SHIFT)
#define ORACLE_ST_ETH_MALFORMED    0x0020u
#define ORACLE_ST_L3_MALFORMED     0x0040u
#define ORACLE_ST_L4_MALFORMED     0x0080u
#define ORACLE_ST_IP_CSUM_OK       0x0100u
#define ORACLE_ST_L4_CSUM_DONE     0x0200u
#define ORACLE_ST_L4_CSUM_OK       0x0400u
#define ORACLE_ST_UNKNOWN_ETHERTYPE 0x0800u
#define ORACLE_ST_UNKNOWN_PROTO    0x1000u
#define ORACLE_ST_VLAN             0x2000u
#define ORACLE_ST_FRAGMENT         0x4000u
#define ORACLE_ST_DESC_INVALID     0x8000u

/* opt-in dispatch extensions (beyond packetdump.rs's chain) */
#define ORACLE_RX_VLAN      0x1u   /* follow 802.1Q/802.1ad/QinQ tags, vlan.rs:62-72 (<= 2)   */
#define ORACLE_RX_IPV6_EXT  0x2u   /* walk IPv6 extension headers, ipv6.rs:39-137 (<= 4)      */
#define ORACLE_RX_L3        0x4u   /* frames begin at the IP header (version nibble dispatch)  */

/* One receive record: the same fields as the GPU result columns. */
typedef struct oracle_rec {
    uint16_t status;
    uint16_t ip_csum;     /* ipv4::checksum(&ip)                         */
    uint16_t l4_csum;     /* udp/tcp ipv4|ipv6_checksum, icmp(v6)::checksum */
    uint16_t ethertype;
    uint8_t  ip_proto;    /* IPv4 next_level_protocol / IPv6 next_header */
    uint8_t  ttl;         /* IPv4 ttl / IPv6 hop_limit                   */
    uint16_t l4_offset;   /* frame offset of ip.payload() (0 if empty)   */
    uint16_t l4_length;   /* ip.payload().len()                          */
    uint16_t src_port;    /* UDP/TCP source; ICMP: type<<8|code          */
    uint16_t dst_port;    /* UDP/TCP destination; ICMP: BE16@4 if len>=8 */
    uint32_t src_ipv4;    /* octets as big-endian u32                    */
    uint32_t dst_ipv4;
    uint8_t  src_ipv6[16];
    uint8_t  dst_ipv6[16];
    uint16_t vlan_tci;    /* outer VLAN tag control information (RX_VLAN)   */
    uint8_t  l3_offset;   /* frame offset of the IP header                 */
    uint8_t  _pad;
    /* header-field getters (0 unless the dispatch constructed that view) */
    uint64_t eth_dst;             /* ethernet.rs:23 MacAddr octets, BE-valued u48 */
    uint64_t eth_src;             /* ethernet.rs:25                             */
    uint32_t tcp_sequence;        /* tcp.rs:59                                  */
    uint32_t tcp_acknowledgement; /* tcp.rs:60                                  */
    uint32_t ip6_flow_label;      /* ipv6.rs:25 u20be                           */
    uint16_t ip_total_length;     /* ipv4.rs:144                                */
    uint16_t ip_identification;   /* ipv4.rs:145                                */
    uint16_t ip_fragment_offset;  /* ipv4.rs:147 u13be                          */
    uint16_t ip6_payload_length;  /* ipv6.rs:26                                 */
    uint16_t udp_length;          /* udp.rs:27                                  */
    uint16_t tcp_window;          /* tcp.rs:64                                  */
    uint16_t tcp_urgent_ptr;      /* tcp.rs:66                                  */
    uint16_t icmp_sequence;       /* echo views only: ICMP 0/8, ICMPv6 128/129, slice >= 8 B */
    uint8_t  ip_version;          /* ipv4.rs:140 / ipv6.rs:23 u4                */
    uint8_t  ip_header_length;    /* ipv4.rs:141 u4                             */
    uint8_t  ip_dscp;             /* ipv4.rs:142 u6                             */
    uint8_t  ip_ecn;              /* ipv4.rs:143 u2                             */
    uint8_t  ip_flags;            /* ipv4.rs:146 u3                             */
    uint8_t  ip6_traffic_class;   /* ipv6.rs:24 u8 (across the nibbles)         */
    uint8_t  tcp_data_offset;     /* tcp.rs:61 u4                               */
    uint8_t  tcp_reserved;        /* tcp.rs:62 u4                               */
    uint8_t  tcp_flags;           /* tcp.rs:63 u8                               */
    uint8_t  _pad3[3];
} oracle_rec;

/* util.rs:158-181 */
uint32_t oracle_sum_be_words(const uint8_t* data, size_t len, size_t skipword);
/* util.rs:84-89 */
uint16_t oracle_finalize_checksum(uint32_t sum);
/* util.rs:76-82 */
uint16_t oracle_checksum(const uint8_t* data, size_t len, size_t skipword);
/* util.rs:92-117 */
uint16_t oracle_ipv4_checksum(const uint8_t* data, size_t len, size_t skipword,
                              const uint8_t* extra, size_t extra_len,
                              const uint8_t src[4], const uint8_t dst[4], uint8_t proto);
/* util.rs:125-150 */
uint16_t oracle_ipv6_checksum(const uint8_t* data, size_t len, size_t skipword,
                              const uint8_t* extra, size_t extra_len,
                              const uint8_t src[16], const uint8_t dst[16], uint8_t proto);

/* Receive dispatch for one Ethernet frame (packetdump.rs:120-217). */
void oracle_rx_frame(const uint8_t* frame, size_t len, oracle_rec* out);
/* Same with opt-in extensions (ORACLE_RX_*). */
void oracle_rx_frame_ex(const uint8_t* frame, size_t len, uint32_t flags, oracle_rec* out);

/*
 * Batch form over a frame buffer. stride > 0: frame i = buf[first + i*stride,
 * +frame_len); stride == 0: frame i = buf[offsets[i], +lengths[i]).
 * Frames outside [0, buf_len) get ORACLE_ST_DESC_INVALID and nothing else.
 * nthreads > 1 splits the batch into static index shards (std pthreads).
 */
void oracle_rx_batch(const uint8_t* buf, uint64_t buf_len, uint64_t n,
                     uint64_t first, uint32_t stride, uint32_t frame_len,
                     const uint64_t* offsets, const uint32_t* lengths,
                     oracle_rec* out, int nthreads);
void oracle_rx_batch_ex(const uint8_t* buf, uint64_t buf_len, uint64_t n,
                        uint64_t first, uint32_t stride, uint32_t frame_len,
                        const uint64_t* offsets, const uint32_t* lengths, uint32_t flags,
                        oracle_rec* out, int nthreads);

size_t oracle_rec_size(void);

/* Sender side (benches/rs_sender.rs:38-39,70-71): write every computed checksum
 * into its stored field in place; records describe the frames before patching. */
void oracle_tx_fill(uint8_t* buf, uint64_t buf_len, uint64_t n, uint64_t first, uint32_t stride,
                    uint32_t frame_len, const uint64_t* offsets, const uint32_t* lengths, uint32_t flags,
                    oracle_rec* out);

/* CPU baselines: the batch receive with persistent threads (each static shard
 * processed `reps` times by one of nthreads threads), and rs_sender.rs's
 * build_udp4_packet (benches/rs_sender.rs:25-72) for n 64-B frames at stride 64
 * (frame i: identification i, UDP source port 1234 + i). */
void oracle_rx_batch_reps(const uint8_t* buf, uint64_t buf_len, uint64_t n, uint64_t first, uint32_t stride,
                          uint32_t frame_len, const uint64_t* offsets, const uint32_t* lengths, uint32_t flags,
                          oracle_rec* out, int nthreads, int reps);
void oracle_rs_sender_build(uint8_t* buf, uint64_t n, int nthreads, int reps);
void oracle_checksum_slices_reps(const uint8_t* buf, uint64_t n, const uint64_t* offsets, const uint32_t* lengths,
                                 const uint32_t* skipwords, uint16_t* out, int nthreads, int reps);

/* Batched util::checksum over (offset, length, skipword) slices. */
void oracle_checksum_slices(const uint8_t* buf, uint64_t n, const uint64_t* offsets,
                            const uint32_t* lengths, const uint32_t* skipwords,
                            uint16_t* out);

#ifdef __cplusplus
}
#endif
#endif
