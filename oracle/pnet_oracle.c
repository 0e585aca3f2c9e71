/*
 * pnet_oracle.c — CPU restatement of libpnet's receive path (parity oracle).
 *
 * TEST INFRASTRUCTURE ONLY (see pnet_oracle.h). Scalar and literal on
 * purpose: each function follows the cited reference lines one-to-one so
 * that a reader can check it against the Rust source. It is also the
 * "port" CPU baseline timed by bench.py (cpu_baseline.kind = "port").
 */
#include "pnet_oracle.h"

#include <pthread.h>
#include <string.h>

/* ---- pnet_packet/src/util.rs ------------------------------------------ */

/* util.rs:158-181  fn sum_be_words(data: &[u8], skipword: usize) -> u32
 * (u32 arithmetic: wraps modulo 2^32 as the reference does in a release
 * build - overflow checks off; a debug build panics on such inputs) */
uint32_t oracle_sum_be_words(const uint8_t* data, size_t len, size_t skipword) {
    if (len == 0) return 0;                       /* :159-161 */
    const uint8_t* cur = data;
    size_t cur_len = len;
    uint32_t sum = 0;
    size_t i = 0;
    while (cur_len >= 2) {                        /* :166 */
        if (i != skipword) {                      /* :167 */
            sum += ((uint32_t)cur[0] << 8) | (uint32_t)cur[1];   /* :169 u16::from_be_bytes */
        }
        cur += 2;                                 /* :171 */
        cur_len -= 2;
        i += 1;                                   /* :172 */
    }
    if (i != skipword && (len & 1) != 0) {        /* :176 */
        sum += (uint32_t)data[len - 1] << 8;      /* :177 */
    }
    return sum;
}

/* util.rs:84-89  fn finalize_checksum(mut sum: u32) -> u16be */
uint16_t oracle_finalize_checksum(uint32_t sum) {
    while ((sum >> 16) != 0) {
        sum = (sum >> 16) + (sum & 0xFFFF);
    }
    return (uint16_t)~sum;
}

/* util.rs:76-82  pub fn checksum(data: &[u8], skipword: usize) -> u16be */
uint16_t oracle_checksum(const uint8_t* data, size_t len, size_t skipword) {
    if (len == 0) return 0;
    return oracle_finalize_checksum(oracle_sum_be_words(data, len, skipword));
}

/* util.rs:119-122  fn ipv4_word_sum(ip: &Ipv4Addr) -> u32 */
static uint32_t ipv4_word_sum(const uint8_t o[4]) {
    return (((uint32_t)o[0] << 8) | o[1]) + (((uint32_t)o[2] << 8) | o[3]);
}

/* util.rs:152-154  fn ipv6_word_sum(ip: &Ipv6Addr) -> u32  (segments().sum()) */
static uint32_t ipv6_word_sum(const uint8_t o[16]) {
    uint32_t s = 0;
    for (int k = 0; k < 8; ++k) s += ((uint32_t)o[2 * k] << 8) | o[2 * k + 1];
    return s;
}

/* util.rs:92-117  pub fn ipv4_checksum(...) -> u16be */
uint16_t oracle_ipv4_checksum(const uint8_t* data, size_t len, size_t skipword,
                              const uint8_t* extra, size_t extra_len,
                              const uint8_t src[4], const uint8_t dst[4], uint8_t proto) {
    uint32_t sum = 0;
    sum += ipv4_word_sum(src);                                    /* :103 */
    sum += ipv4_word_sum(dst);                                    /* :104 */
    sum += proto;                                                 /* :107 */
    sum += (uint32_t)(len + extra_len);                           /* :109-110 */
    sum += oracle_sum_be_words(data, len, skipword);              /* :113 */
    sum += oracle_sum_be_words(extra, extra_len, extra_len / 2);  /* :114 */
    return oracle_finalize_checksum(sum);                         /* :116 */
}

/* util.rs:125-150  pub fn ipv6_checksum(...) -> u16be */
uint16_t oracle_ipv6_checksum(const uint8_t* data, size_t len, size_t skipword,
                              const uint8_t* extra, size_t extra_len,
                              const uint8_t src[16], const uint8_t dst[16], uint8_t proto) {
    uint32_t sum = 0;
    sum += ipv6_word_sum(src);                                    /* :136 */
    sum += ipv6_word_sum(dst);                                    /* :137 */
    sum += proto;                                                 /* :140 */
    sum += (uint32_t)(len + extra_len);                           /* :142-143 */
    sum += oracle_sum_be_words(data, len, skipword);              /* :146 */
    sum += oracle_sum_be_words(extra, extra_len, extra_len / 2);  /* :147 */
    return oracle_finalize_checksum(sum);                         /* :149 */
}

/* ---- generated accessors (pnet_macros/src/decorator.rs:1563-1670) ----- */

static inline uint16_t be16(const uint8_t* p) { return (uint16_t)(((uint16_t)p[0] << 8) | p[1]); }
static inline uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* A borrowed byte slice, the PacketData::Borrowed of packet.rs:117-122. */
typedef struct { const uint8_t* p; size_t len; } slice_t;

/* ---- L4 handlers: packetdump.rs:31-98 plus the checksum wrappers ------- */

/* udp.rs:23-31 (min size 8), udp.rs:34-56 / 104-126 (skipword 3) */
/* tcp.rs:55-71 (min size 20), tcp.rs:239-286 (skipword 8)            */
/* icmp.rs:55-67 (min size 4),  icmp.rs:70-75 (skipword 1, no pseudo)  */
/* icmpv6.rs:68-77 (min size 4), icmpv6.rs:80-85 (IPv6 pseudo, skip 1) */
static void l4_dispatch(oracle_rec* r, int is_v6, uint8_t proto, slice_t l4,
                        const uint8_t* src, const uint8_t* dst) {
    switch (proto) {
    case 17: /* IpNextHeaderProtocols::Udp, ip.rs:79 */
        r->status |= ORACLE_ST_L4_UDP;
        if (l4.len < 8) { r->status |= ORACLE_ST_L4_MALFORMED; return; }  /* UdpPacket::new */
        r->src_port = be16(l4.p + 0);
        r->dst_port = be16(l4.p + 2);
        r->udp_length = be16(l4.p + 4);                   /* udp.rs:27 length: u16be */
        r->l4_csum = is_v6 ? oracle_ipv6_checksum(l4.p, l4.len, 3, NULL, 0, src, dst, 17)
                           : oracle_ipv4_checksum(l4.p, l4.len, 3, NULL, 0, src, dst, 17);
        r->status |= ORACLE_ST_L4_CSUM_DONE;
        if (r->l4_csum == be16(l4.p + 6)) r->status |= ORACLE_ST_L4_CSUM_OK;
        return;
    case 6: /* IpNextHeaderProtocols::Tcp, ip.rs:46 */
        r->status |= ORACLE_ST_L4_TCP;
        if (l4.len < 20) { r->status |= ORACLE_ST_L4_MALFORMED; return; }  /* TcpPacket::new */
        r->src_port = be16(l4.p + 0);
        r->dst_port = be16(l4.p + 2);
        r->tcp_sequence = be32(l4.p + 4);                 /* tcp.rs:59 sequence: u32be        */
        r->tcp_acknowledgement = be32(l4.p + 8);          /* tcp.rs:60 acknowledgement: u32be */
        r->tcp_data_offset = l4.p[12] >> 4;               /* tcp.rs:61 data_offset: u4 (high) */
        r->tcp_reserved = l4.p[12] & 0x0F;                /* tcp.rs:62 reserved: u4 (low)     */
        r->tcp_flags = l4.p[13];                          /* tcp.rs:63 flags: u8              */
        r->tcp_window = be16(l4.p + 14);                  /* tcp.rs:64 window: u16be          */
        r->tcp_urgent_ptr = be16(l4.p + 18);              /* tcp.rs:66 urgent_ptr: u16be      */
        r->l4_csum = is_v6 ? oracle_ipv6_checksum(l4.p, l4.len, 8, NULL, 0, src, dst, 6)
                           : oracle_ipv4_checksum(l4.p, l4.len, 8, NULL, 0, src, dst, 6);
        r->status |= ORACLE_ST_L4_CSUM_DONE;
        if (r->l4_csum == be16(l4.p + 16)) r->status |= ORACLE_ST_L4_CSUM_OK;
        return;
    case 1: /* IpNextHeaderProtocols::Icmp, ip.rs:31 */
        r->status |= ORACLE_ST_L4_ICMP;
        if (l4.len < 4) { r->status |= ORACLE_ST_L4_MALFORMED; return; }   /* IcmpPacket::new */
        r->src_port = be16(l4.p + 0);                     /* icmp_type << 8 | icmp_code */
        r->dst_port = l4.len >= 8 ? be16(l4.p + 4) : 0;   /* echo identifier, icmp.rs:221-232 */
        /* EchoReply (type 0) / EchoRequest (type 8) views only: packetdump.rs:52-75,
         * sequence_number icmp.rs:229/311; any other type builds no echo view */
        r->icmp_sequence = (l4.len >= 8 && (l4.p[0] == 0 || l4.p[0] == 8)) ? be16(l4.p + 6) : 0;
        r->l4_csum = oracle_checksum(l4.p, l4.len, 1);
        r->status |= ORACLE_ST_L4_CSUM_DONE;
        if (r->l4_csum == be16(l4.p + 2)) r->status |= ORACLE_ST_L4_CSUM_OK;
        return;
    case 58: /* IpNextHeaderProtocols::Icmpv6, ip.rs:205 */
        r->status |= ORACLE_ST_L4_ICMPV6;
        if (l4.len < 4) { r->status |= ORACLE_ST_L4_MALFORMED; return; }   /* Icmpv6Packet::new */
        r->src_port = be16(l4.p + 0);
        r->dst_port = l4.len >= 8 ? be16(l4.p + 4) : 0;
        /* Icmpv6 EchoRequest (128) / EchoReply (129) views only (icmpv6.rs:135-137,837-995) */
        r->icmp_sequence = (l4.len >= 8 && (l4.p[0] == 128 || l4.p[0] == 129)) ? be16(l4.p + 6) : 0;
        if (is_v6) { /* icmpv6::checksum needs IPv6 addresses; none exists over IPv4 */
            r->l4_csum = oracle_ipv6_checksum(l4.p, l4.len, 1, NULL, 0, src, dst, 58);
            r->status |= ORACLE_ST_L4_CSUM_DONE;
            if (r->l4_csum == be16(l4.p + 2)) r->status |= ORACLE_ST_L4_CSUM_OK;
        }
        return;
    default:
        r->status |= ORACLE_ST_UNKNOWN_PROTO;             /* packetdump.rs:139-152 */
        return;
    }
}

/* packetdump.rs:155-168 handle_ipv4_packet; ep = Ipv4 bytes at frame offset l3 */
static void handle_ipv4(oracle_rec* r, slice_t ep, size_t l3) {
    r->status |= ORACLE_ST_L3_IPV4;
    if (ep.len < 20) { r->status |= ORACLE_ST_L3_MALFORMED; return; }  /* Ipv4Packet::new, min 20 */
    const uint8_t* ip = ep.p;
    unsigned ihl = ip[0] & 0x0F;                          /* header_length: u4 */
    r->ip_version = ip[0] >> 4;                           /* ipv4.rs:140 version: u4 (high)  */
    r->ip_header_length = (uint8_t)ihl;                   /* ipv4.rs:141                     */
    r->ip_dscp = ip[1] >> 2;                              /* ipv4.rs:142 dscp: u6 (high)     */
    r->ip_ecn = ip[1] & 0x03;                             /* ipv4.rs:143 ecn: u2 (low)       */
    r->ip_total_length = be16(ip + 2);                    /* ipv4.rs:144                     */
    r->ip_identification = be16(ip + 4);                  /* ipv4.rs:145                     */
    r->ip_flags = ip[6] >> 5;                             /* ipv4.rs:146 flags: u3 (high)    */
    r->ip_fragment_offset = be16(ip + 6) & 0x1FFF;        /* ipv4.rs:147 u13be (low 13 bits) */
    /* ipv4.rs:165-178: clamp IHL*4 to [minimum_packet_size, packet().len()] */
    size_t hl = (size_t)ihl * 4;
    if (hl < 20) hl = 20;
    else if (hl > ep.len) hl = ep.len;
    r->ip_csum = oracle_checksum(ip, hl, 5);
    if (r->ip_csum == be16(ip + 10)) r->status |= ORACLE_ST_IP_CSUM_OK;

    r->ttl = ip[8];
    r->ip_proto = ip[9];
    r->src_ipv4 = be32(ip + 12);
    r->dst_ipv4 = be32(ip + 16);

    /* payload(): start = 20 + ipv4_options_length (ipv4.rs:226-231, saturating),
     * end = min(start + ipv4_payload_length (ipv4.rs:241-243), len)
     * (decorator.rs:728-753); empty if len <= start. */
    size_t opts = (size_t)ihl * 4 > 20 ? (size_t)ihl * 4 - 20 : 0;
    size_t start = 20 + opts;
    size_t total_length = be16(ip + 2);
    size_t plen = total_length > (size_t)ihl * 4 ? total_length - (size_t)ihl * 4 : 0;
    slice_t l4 = { NULL, 0 };
    if (ep.len > start) {
        size_t end = start + plen;
        if (end > ep.len) end = ep.len;
        l4.p = ip + start;
        l4.len = end - start;
        r->l4_offset = (uint16_t)(l3 + start);
        r->l4_length = (uint16_t)l4.len;
    }
    l4_dispatch(r, 0, ip[9], l4, ip + 12, ip + 16);
}

/* packetdump.rs:170-183 handle_ipv6_packet; with ORACLE_RX_IPV6_EXT the
 * extension headers of ipv6.rs:39-137 are walked first (at most 4):
 * Hop-by-Hop (0) / Destination (60): Extension, min 2 bytes, length
 * hdr_ext_len*8+8 (ipv6_extension_length + the 2 fixed bytes, ipv6.rs:56-58);
 * Routing (43): min 4, same length (ipv6.rs:75-77); Fragment (44): 8 bytes
 * (ipv6.rs:80-89), get_fragment_offset = value & !0x3 (ipv6.rs:95-97): a
 * non-first fragment carries no L4 header (PNET_ST_FRAGMENT, no dispatch).
 * A truncated extension header (its new() == None, or its length running past
 * the payload) sets L4_MALFORMED. */
static void handle_ipv6(oracle_rec* r, slice_t ep, size_t l3, uint32_t flags) {
    r->status |= ORACLE_ST_L3_IPV6;
    if (ep.len < 40) { r->status |= ORACLE_ST_L3_MALFORMED; return; }  /* Ipv6Packet::new, min 40 */
    const uint8_t* ip = ep.p;
    r->ip_version = ip[0] >> 4;                           /* ipv6.rs:23 version: u4            */
    r->ip6_traffic_class = (uint8_t)(((ip[0] & 0x0F) << 4) | (ip[1] >> 4));   /* ipv6.rs:24 */
    r->ip6_flow_label = ((uint32_t)(ip[1] & 0x0F) << 16) | be16(ip + 2);    /* ipv6.rs:25 u20be */
    r->ip6_payload_length = be16(ip + 4);                 /* ipv6.rs:26                        */
    r->ip_proto = ip[6];                                  /* next_header */
    r->ttl = ip[7];                                       /* hop_limit */
    memcpy(r->src_ipv6, ip + 8, 16);
    memcpy(r->dst_ipv6, ip + 24, 16);
    /* payload bounded by payload_length (ipv6.rs:34-36, #[length = "payload_length"]) */
    size_t payload_length = be16(ip + 4);
    slice_t pl = { NULL, 0 };
    if (ep.len > 40) {
        size_t end = 40 + payload_length;
        if (end > ep.len) end = ep.len;
        pl.p = ip + 40;
        pl.len = end - 40;
    }
    uint8_t next = ip[6];
    size_t pos = 0;
    if (flags & ORACLE_RX_IPV6_EXT) {
        for (int k = 0; k < 4; ++k) {
            if (next == 0 || next == 60 || next == 43) {
                size_t minl = next == 43 ? 4 : 2;
                if (pl.len - pos < minl) { r->ip_proto = next; r->status |= ORACLE_ST_L4_MALFORMED; return; }
                size_t el = (size_t)pl.p[pos + 1] * 8 + 8;
                if (el > pl.len - pos) { r->ip_proto = next; r->status |= ORACLE_ST_L4_MALFORMED; return; }
                next = pl.p[pos];
                pos += el;
            } else if (next == 44) {
                if (pl.len - pos < 8) { r->ip_proto = next; r->status |= ORACLE_ST_L4_MALFORMED; return; }
                unsigned fo = be16(pl.p + pos + 2);
                next = pl.p[pos];
                pos += 8;
                if ((fo & 0xFFFCu) != 0) {                /* not the first fragment */
                    r->ip_proto = next;
                    r->status |= ORACLE_ST_FRAGMENT;
                    if (pl.len > pos) {
                        r->l4_offset = (uint16_t)(l3 + 40 + pos);
                        r->l4_length = (uint16_t)(pl.len - pos);
                    }
                    return;
                }
            } else {
                break;
            }
        }
        r->ip_proto = next;
    }
    slice_t l4 = { NULL, 0 };
    if (pl.len > pos) {
        l4.p = pl.p + pos;
        l4.len = pl.len - pos;
        r->l4_offset = (uint16_t)(l3 + 40 + pos);
        r->l4_length = (uint16_t)l4.len;
    }
    l4_dispatch(r, 1, next, l4, ip + 8, ip + 24);
}

static int is_vlan_tpid(unsigned et) {       /* EtherTypes::Vlan / PBridge / QinQ, ethernet.rs:102-112 */
    return et == 0x8100 || et == 0x88A8 || et == 0x9100;
}

/* packetdump.rs:200-217 handle_ethernet_frame; with ORACLE_RX_VLAN up to two
 * VlanPacket views (vlan.rs:62-72: 4 bytes, inner ethertype at +2) are peeled
 * first and the IP header starts after them. */
void oracle_rx_frame_ex(const uint8_t* frame, size_t len, uint32_t flags, oracle_rec* r) {
    memset(r, 0, sizeof(*r));
    unsigned et;
    size_t l3;
    if (flags & ORACLE_RX_L3) {
        /* pnet_transport Layer3 receive (lib.rs:342-374): Ipv4Packet::new over the
         * whole buffer; IPv6 by the version nibble; the IP views as below */
        const unsigned ver = len ? frame[0] >> 4 : 0;
        et = ver == 4 ? 0x0800u : ver == 6 ? 0x86DDu : 0u;
        l3 = 0;
    } else {
        if (len < 14) { r->status = ORACLE_ST_ETH_MALFORMED; return; }  /* EthernetPacket::new, min 14 */
        for (int k = 0; k < 6; ++k) {                     /* ethernet.rs:23,25 MacAddr(u8 x 6) */
            r->eth_dst = (r->eth_dst << 8) | frame[k];
            r->eth_src = (r->eth_src << 8) | frame[6 + k];
        }
        et = be16(frame + 12);                            /* ethernet.rs:27-28 */
        l3 = 14;
    }
    if ((flags & (ORACLE_RX_VLAN | ORACLE_RX_L3)) == ORACLE_RX_VLAN) {
        for (int k = 0; k < 2 && is_vlan_tpid(et); ++k) {
            r->status |= ORACLE_ST_VLAN;
            if (len < l3 + 4) {                           /* VlanPacket::new == None */
                r->ethertype = (uint16_t)et;
                r->status |= ORACLE_ST_L3_MALFORMED;
                return;
            }
            if (k == 0) r->vlan_tci = be16(frame + l3);
            et = be16(frame + l3 + 2);
            l3 += 4;
        }
    }
    r->ethertype = (uint16_t)et;
    r->l3_offset = (uint8_t)l3;
    slice_t ep = { frame + l3, len - l3 };                /* payload: last field, unbounded */
    switch (et) {
    case 0x0800: handle_ipv4(r, ep, l3); break;          /* EtherTypes::Ipv4, ethernet.rs:68 */
    case 0x86DD: handle_ipv6(r, ep, l3, flags); break;   /* EtherTypes::Ipv6, ethernet.rs:88 */
    default: r->status |= ORACLE_ST_UNKNOWN_ETHERTYPE; break;
    }
}

void oracle_rx_frame(const uint8_t* frame, size_t len, oracle_rec* r) {
    oracle_rx_frame_ex(frame, len, 0, r);
}

/* ---- batch drivers ------------------------------------------------------ */

typedef struct {
    const uint8_t* buf; uint64_t buf_len; uint64_t lo, hi;
    uint64_t first; uint32_t stride, frame_len;
    const uint64_t* offsets; const uint32_t* lengths; oracle_rec* out; uint32_t flags;
} shard_t;

static void* rx_shard(void* arg) {
    shard_t* s = (shard_t*)arg;
    for (uint64_t i = s->lo; i < s->hi; ++i) {
        uint64_t off = s->stride ? s->first + i * (uint64_t)s->stride : s->offsets[i];
        uint64_t len = s->stride ? s->frame_len : s->lengths[i];
        if (off > s->buf_len || len > s->buf_len - off) {
            memset(&s->out[i], 0, sizeof(oracle_rec));
            s->out[i].status = ORACLE_ST_DESC_INVALID;
            continue;
        }
        oracle_rx_frame_ex(s->buf + off, (size_t)len, s->flags, &s->out[i]);
    }
    return NULL;
}

void oracle_rx_batch(const uint8_t* buf, uint64_t buf_len, uint64_t n,
                     uint64_t first, uint32_t stride, uint32_t frame_len,
                     const uint64_t* offsets, const uint32_t* lengths,
                     oracle_rec* out, int nthreads) {
    oracle_rx_batch_ex(buf, buf_len, n, first, stride, frame_len, offsets, lengths, 0, out, nthreads);
}

void oracle_rx_batch_ex(const uint8_t* buf, uint64_t buf_len, uint64_t n,
                        uint64_t first, uint32_t stride, uint32_t frame_len,
                        const uint64_t* offsets, const uint32_t* lengths, uint32_t flags,
                        oracle_rec* out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    shard_t sh[256];
    pthread_t th[256];
    for (int t = 0; t < nthreads; ++t) {
        shard_t s = { buf, buf_len, n * (uint64_t)t / nthreads, n * (uint64_t)(t + 1) / nthreads,
                      first, stride, frame_len, offsets, lengths, out, flags };
        sh[t] = s;
    }
    if (nthreads == 1) { rx_shard(&sh[0]); return; }
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, rx_shard, &sh[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

void oracle_checksum_slices(const uint8_t* buf, uint64_t n, const uint64_t* offsets,
                            const uint32_t* lengths, const uint32_t* skipwords,
                            uint16_t* out) {
    for (uint64_t i = 0; i < n; ++i)
        out[i] = oracle_checksum(buf + offsets[i], lengths[i], skipwords[i]);
}

size_t oracle_rec_size(void) { return sizeof(oracle_rec); }

/* Sender side: the set_checksum(checksum(..)) calls of the reference's packet
 * builders (benches/rs_sender.rs:38-39,70-71): every checksum the receive
 * dispatch computes is written big-endian into its field, in place. The record
 * describes the frame as it was before patching. */
void oracle_tx_fill(uint8_t* buf, uint64_t buf_len, uint64_t n, uint64_t first, uint32_t stride,
                    uint32_t frame_len, const uint64_t* offsets, const uint32_t* lengths, uint32_t flags,
                    oracle_rec* out) {
    for (uint64_t i = 0; i < n; ++i) {
        uint64_t off = stride ? first + i * (uint64_t)stride : offsets[i];
        uint64_t len = stride ? frame_len : lengths[i];
        oracle_rec* r = &out[i];
        if (off > buf_len || len > buf_len - off) {
            memset(r, 0, sizeof(*r));
            r->status = ORACLE_ST_DESC_INVALID;
            continue;
        }
        uint8_t* f = buf + off;
        oracle_rx_frame_ex(f, (size_t)len, flags, r);
        if ((r->status & (ORACLE_ST_L3_IPV4 | ORACLE_ST_L3_IPV6 | ORACLE_ST_L3_MALFORMED)) == ORACLE_ST_L3_IPV4) {
            f[r->l3_offset + 10] = (uint8_t)(r->ip_csum >> 8);   /* Ipv4 checksum field, header bytes 10-11 */
            f[r->l3_offset + 11] = (uint8_t)r->ip_csum;
        }
        if (r->status & ORACLE_ST_L4_CSUM_DONE) {
            unsigned kind = r->status & (7u << ORACLE_ST_L4_SHIFT);
            unsigned at = kind == ORACLE_ST_L4_UDP ? 6u : kind == ORACLE_ST_L4_TCP ? 16u : 2u;
            f[r->l4_offset + at] = (uint8_t)(r->l4_csum >> 8);
            f[r->l4_offset + at + 1] = (uint8_t)r->l4_csum;
        }
    }
}

/* ---- CPU baselines (bench.py's cpu_baseline / config0 legs) ---------------
 * Persistent threads: each of nthreads static index shards is processed `reps`
 * times by one thread, so short passes are not dominated by thread start-up. */

typedef struct {
    void (*fn)(void* arg, uint64_t lo, uint64_t hi);
    void* arg;
    uint64_t lo, hi;
    int reps;
} rep_job_t;

static void* rep_worker(void* p) {
    rep_job_t* j = (rep_job_t*)p;
    for (int r = 0; r < j->reps; ++r) j->fn(j->arg, j->lo, j->hi);
    return NULL;
}

static void run_sharded(void (*fn)(void*, uint64_t, uint64_t), void* arg, uint64_t n, int nthreads, int reps) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 1024) nthreads = 1024;
    static rep_job_t jobs[1024];
    static pthread_t th[1024];
    for (int t = 0; t < nthreads; ++t) {
        rep_job_t j = { fn, arg, n * (uint64_t)t / nthreads, n * (uint64_t)(t + 1) / nthreads, reps };
        jobs[t] = j;
    }
    if (nthreads == 1) { rep_worker(&jobs[0]); return; }
    int started = 0;
    for (int t = 0; t < nthreads; ++t)
        if (pthread_create(&th[t], NULL, rep_worker, &jobs[t]) == 0) ++started;
        else { rep_worker(&jobs[t]); th[t] = 0; }
    for (int t = 0; t < nthreads; ++t)
        if (th[t]) pthread_join(th[t], NULL);
    (void)started;
}

static void rx_range(void* arg, uint64_t lo, uint64_t hi) {
    shard_t s = *(shard_t*)arg;
    s.lo = lo;
    s.hi = hi;
    rx_shard(&s);
}

void oracle_rx_batch_reps(const uint8_t* buf, uint64_t buf_len, uint64_t n, uint64_t first, uint32_t stride,
                          uint32_t frame_len, const uint64_t* offsets, const uint32_t* lengths, uint32_t flags,
                          oracle_rec* out, int nthreads, int reps) {
    shard_t s = { buf, buf_len, 0, n, first, stride, frame_len, offsets, lengths, out, flags };
    run_sharded(rx_range, &s, n, nthreads, reps);
}

/* benches/rs_sender.rs:25-72: build_udp4_packet behind an Ethernet header
 * (rs_sender.rs:94-100), the IPv4 checksum after the IPv4 setters and the UDP
 * checksum after the payload, written big-endian by the setters. Frame i
 * carries identification i and UDP source port 1234 + i (16-bit) so that every
 * frame's checksums differ; frame 0 is rs_sender's own (0xB8CA / 0xB94C). */
static void rs_sender_frame(uint8_t* f, uint64_t i) {
    static const uint8_t dst[6] = {0x02, 0x00, 0x00, 0x00, 0x00, 0x01};
    static const uint8_t src[6] = {0x02, 0x00, 0x00, 0x00, 0x00, 0x02};
    memset(f, 0, 64);
    memcpy(f, dst, 6);                                   /* set_destination */
    memcpy(f + 6, src, 6);                               /* set_source */
    f[12] = 0x08; f[13] = 0x00;                          /* set_ethertype(EtherTypes::Ipv4) */
    uint8_t* ip = f + 14;
    ip[0] = (uint8_t)((4 << 4) | 5);                     /* set_version(4), set_header_length(5) */
    ip[2] = 0; ip[3] = 20 + 8 + 5;                       /* set_total_length(33) */
    ip[4] = (uint8_t)(i >> 8); ip[5] = (uint8_t)i;       /* identification */
    ip[8] = 4;                                           /* set_ttl(4) */
    ip[9] = 17;                                          /* IpNextHeaderProtocols::Udp */
    ip[12] = 127; ip[15] = 1;                            /* set_source(127.0.0.1) */
    ip[16] = 127; ip[19] = 1;                            /* set_destination(127.0.0.1) */
    const uint16_t ipc = oracle_checksum(ip, 20, 5);     /* ipv4::checksum (ipv4.rs:165-178) */
    ip[10] = (uint8_t)(ipc >> 8); ip[11] = (uint8_t)ipc;
    uint8_t* udp = ip + 20;
    const uint16_t sport = (uint16_t)(1234 + i);
    udp[0] = (uint8_t)(sport >> 8); udp[1] = (uint8_t)sport;   /* set_source */
    udp[2] = 1234 >> 8; udp[3] = 1234 & 0xFF;            /* set_destination(1234) */
    udp[4] = 0; udp[5] = 8 + 5;                          /* set_length(13) */
    memcpy(udp + 8, "rmesg", 5);
    const uint16_t uc = oracle_ipv4_checksum(udp, 13, 3, NULL, 0, ip + 12, ip + 16, 17);   /* udp.rs:34-56 */
    udp[6] = (uint8_t)(uc >> 8); udp[7] = (uint8_t)uc;
}

static void build_range(void* arg, uint64_t lo, uint64_t hi) {
    uint8_t* buf = (uint8_t*)arg;
    for (uint64_t i = lo; i < hi; ++i) rs_sender_frame(buf + 64 * i, i);
}

void oracle_rs_sender_build(uint8_t* buf, uint64_t n, int nthreads, int reps) {
    run_sharded(build_range, buf, n, nthreads, reps);
}

typedef struct {
    const uint8_t* buf; const uint64_t* offsets; const uint32_t* lengths; const uint32_t* skipwords; uint16_t* out;
} slices_t;

static void slices_range(void* arg, uint64_t lo, uint64_t hi) {
    const slices_t* s = (const slices_t*)arg;
    for (uint64_t i = lo; i < hi; ++i) s->out[i] = oracle_checksum(s->buf + s->offsets[i], s->lengths[i], s->skipwords[i]);
}

void oracle_checksum_slices_reps(const uint8_t* buf, uint64_t n, const uint64_t* offsets, const uint32_t* lengths,
                                 const uint32_t* skipwords, uint16_t* out, int nthreads, int reps) {
    slices_t s = { buf, offsets, lengths, skipwords, out };
    run_sharded(slices_range, &s, n, nthreads, reps);
}
