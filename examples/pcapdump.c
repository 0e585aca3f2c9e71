/*
 * pcapdump.c — libpnet's examples/packetdump.rs over a pcap or pcapng file, with the
 * per-packet work (Ethernet -> IPv4/IPv6 -> UDP/TCP/ICMP/ICMPv6 dispatch, the
 * views' bounds, header fields and checksums) done on the GPU through the
 * C-ABI. The host only indexes the file (pnetgpu_pcap_scan), ships the records
 * straight from the mapped file (pnetgpu_ring_submit_region) and prints one
 * line per frame from the result columns, in packetdump's formats
 * (packetdump.rs:31-217): the record columns plus the header-field columns
 * packetdump prints — Ethernet source/destination MacAddr, UDP get_length,
 * ICMP echo sequence_number (its identifier is dst_port). Only the ARP fields
 * (arp.rs:83-104; ARP is outside the GPU path) are read from the frame bytes.
 *
 * Raw-IP captures (LINKTYPE_RAW / IPV4 / IPV6, e.g. from a tun device) run with
 * PNETGPU_RX_L3: packetdump's tun branch (packetdump.rs:250-283) wraps such
 * packets in a zeroed Ethernet header chosen by IP version, so well-formed
 * packets print the same lines; a version other than 4 / 6 prints
 * "Unknown packet: IP version V".
 *
 * Where packetdump would panic (EthernetPacket::new(..).unwrap() on a frame
 * shorter than 14 B, packetdump.rs:291; Echo*Packet::new(..).unwrap() on a
 * 4..7-B echo message, :54,:65) this prints "Malformed Ethernet Frame" /
 * "Malformed ICMP Packet" and goes on.
 *
 * Live mode (-l IFACE) is packetdump's own loop on an interface
 * (packetdump.rs:285-300: datalink::channel, rx.next(), handle_ethernet_frame)
 * with the per-frame receive replaced by whole TPACKET_V3 blocks
 * (pnetgpu_afpacket.h): each retired block's frames go from the ring mapping
 * to the GPU in one submit, are printed once the batch is waited, and the
 * block is then given back to the kernel. Needs CAP_NET_RAW.
 *
 * usage: pcapdump [-i NAME] [-c] FILE.pcap|FILE.pcapng
 *        pcapdump [-i NAME] [-c] -l IFACE [-n COUNT] [-w MS]
 *   -i NAME  the "[interface]" label (default: pcap, or IFACE in live mode)
 *   -c       append the checksum verdicts to every IP line
 *   -l IFACE capture from IFACE instead of reading a file
 *   -n COUNT live: stop after COUNT frames
 *   -w MS    live: stop after MS ms without a retired block (default: wait on)
 */
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "pnetgpu.h"
#include "pnetgpu_afpacket.h"
#include "pnetgpu_ring.h"

/* the record columns + the header fields packetdump prints */
#define DUMP_COLUMNS (PNETGPU_COLS_RECORD | PNETGPU_COL_ETH_DST | PNETGPU_COL_ETH_SRC | PNETGPU_COL_UDP_LENGTH | \
                      PNETGPU_COL_ICMP_SEQUENCE)

static const char* g_name = "pcap";
static int g_csum = 0;
static int g_l3 = 0;   /* raw-IP capture: no Ethernet header */

static unsigned be16(const uint8_t* p) { return ((unsigned)p[0] << 8) | p[1]; }

static void fmt_mac(char* out, uint64_t m) {   /* column value: MacAddr octets as a BE-valued u48 */
    sprintf(out, "%02x:%02x:%02x:%02x:%02x:%02x", (unsigned)(m >> 40) & 255u, (unsigned)(m >> 32) & 255u,
            (unsigned)(m >> 24) & 255u, (unsigned)(m >> 16) & 255u, (unsigned)(m >> 8) & 255u, (unsigned)m & 255u);
}

static void fmt_v4(char* out, uint32_t be) {   /* column value: octets as a big-endian-valued u32 */
    sprintf(out, "%u.%u.%u.%u", be >> 24, (be >> 16) & 255u, (be >> 8) & 255u, be & 255u);
}

/* Rust's Ipv6Addr Display: ::ffff:a.b.c.d for IPv4-mapped, else the first
 * longest run (>= 2) of zero segments as "::", segments in lowercase hex. */
static void fmt_v6(char* out, const uint8_t* a) {
    unsigned s[8];
    for (int i = 0; i < 8; ++i) s[i] = be16(a + 2 * i);
    if (!s[0] && !s[1] && !s[2] && !s[3] && !s[4] && s[5] == 0xFFFF) {
        sprintf(out, "::ffff:%u.%u.%u.%u", a[12], a[13], a[14], a[15]);
        return;
    }
    int best = 0, best_len = 0, cur = 0, cur_len = 0;
    for (int i = 0; i < 8; ++i) {
        if (s[i] == 0) {
            if (cur_len == 0) cur = i;
            if (++cur_len > best_len) {
                best = cur;
                best_len = cur_len;
            }
        } else {
            cur_len = 0;
        }
    }
    char* p = out;
    if (best_len > 1) {
        for (int i = 0; i < best; ++i) p += sprintf(p, i ? ":%x" : "%x", s[i]);
        p += sprintf(p, "::");
        for (int i = best + best_len; i < 8; ++i) p += sprintf(p, i > best + best_len ? ":%x" : "%x", s[i]);
    } else {
        for (int i = 0; i < 8; ++i) p += sprintf(p, i ? ":%x" : "%x", s[i]);
    }
}

static void csum_suffix(char* out, unsigned st) {
    out[0] = 0;
    if (!g_csum) return;
    char* p = out;
    if ((st & PNET_ST_L3_MASK) == PNET_ST_L3_IPV4)
        p += sprintf(p, "; ip checksum %s", (st & PNET_ST_IP_CSUM_OK) ? "ok" : "bad");
    if (st & PNET_ST_L4_CSUM_DONE) sprintf(p, "; l4 checksum %s", (st & PNET_ST_L4_CSUM_OK) ? "ok" : "bad");
}

/* One frame of a waited batch, i = its index there. */
static void dump_frame(const pnetgpu_ring_batch* b, uint64_t i) {
    const pnetgpu_rx_columns* c = &b->cols;
    const uint8_t* f = b->frames + b->offsets[i];
    const uint32_t len = b->lengths[i];
    const unsigned st = c->status[i];
    char src[64], dst[64], sfx[64];
    if (st & PNET_ST_ETH_MALFORMED) {
        printf("[%s]: Malformed Ethernet Frame\n", g_name);
        return;
    }
    const unsigned l3 = st & PNET_ST_L3_MASK;
    if (l3 == 0 && g_l3) {   /* raw IP, neither version 4 nor 6 */
        printf("[%s]: Unknown packet: IP version %u; length: %u\n", g_name, len ? f[0] >> 4 : 0u, len);
        return;
    }
    if (l3 == 0) {   /* packetdump.rs:202-217: ARP, otherwise unknown */
        const unsigned et = c->ethertype[i];
        char sm[24], dm[24];
        fmt_mac(dm, c->eth_dst[i]);
        fmt_mac(sm, c->eth_src[i]);
        if (et == 0x0806) {
            if (len - 14 < 28) {
                printf("[%s]: Malformed ARP Packet\n", g_name);
                return;
            }
            const uint8_t* arp = f + 14;
            printf("[%s]: ARP packet: %s(%u.%u.%u.%u) > %s(%u.%u.%u.%u); operation: ArpOperation(%u)\n", g_name, sm,
                   arp[14], arp[15], arp[16], arp[17], dm, arp[24], arp[25], arp[26], arp[27], be16(arp + 6));
        } else {
            printf("[%s]: Unknown packet: %s > %s; ethertype: EtherType(%u) length: %u\n", g_name, sm, dm, et, len);
        }
        return;
    }
    if (st & PNET_ST_L3_MALFORMED) {
        printf("[%s]: Malformed %s Packet\n", g_name, l3 == PNET_ST_L3_IPV4 ? "IPv4" : "IPv6");
        return;
    }
    if (l3 == PNET_ST_L3_IPV4) {
        fmt_v4(src, c->src_ipv4[i]);
        fmt_v4(dst, c->dst_ipv4[i]);
    } else {
        fmt_v6(src, c->src_ipv6 + 16 * i);
        fmt_v6(dst, c->dst_ipv6 + 16 * i);
    }
    csum_suffix(sfx, st);
    const unsigned l4len = c->l4_length[i];
    const int bad = (st & PNET_ST_L4_MALFORMED) != 0;
    switch (st & PNET_ST_L4_MASK) {
    case PNET_ST_L4_UDP:
        if (bad) printf("[%s]: Malformed UDP Packet\n", g_name);
        else printf("[%s]: UDP Packet: %s:%u > %s:%u; length: %u%s\n", g_name, src, c->src_port[i], dst,
                    c->dst_port[i], c->udp_length[i], sfx);
        return;
    case PNET_ST_L4_TCP:
        if (bad) printf("[%s]: Malformed TCP Packet\n", g_name);
        else printf("[%s]: TCP Packet: %s:%u > %s:%u; length: %u%s\n", g_name, src, c->src_port[i], dst,
                    c->dst_port[i], l4len, sfx);
        return;
    case PNET_ST_L4_ICMP: {
        const unsigned type = c->src_port[i] >> 8;
        if (bad || ((type == 0 || type == 8) && l4len < 8)) {
            printf("[%s]: Malformed ICMP Packet\n", g_name);
        } else if (type == 0 || type == 8) {
            printf("[%s]: ICMP echo %s %s -> %s (seq=%u, id=%u)%s\n", g_name, type ? "request" : "reply", src, dst,
                   c->icmp_sequence[i], c->dst_port[i], sfx);
        } else {
            printf("[%s]: ICMP packet %s -> %s (type=IcmpType(%u))%s\n", g_name, src, dst, type, sfx);
        }
        return;
    }
    case PNET_ST_L4_ICMPV6:
        if (bad) printf("[%s]: Malformed ICMPv6 Packet\n", g_name);
        else printf("[%s]: ICMPv6 packet %s -> %s (type=Icmpv6Type(%u))%s\n", g_name, src, dst, c->src_port[i] >> 8,
                    sfx);
        return;
    default:
        printf("[%s]: Unknown %s packet: %s > %s; protocol: IpNextHeaderProtocol(%u) length: %u%s\n", g_name,
               l3 == PNET_ST_L3_IPV4 ? "IPv4" : "IPv6", src, dst, c->ip_proto[i], l4len, sfx);
    }
}

static int drain_one(pnetgpu_ring* ring) {
    pnetgpu_ring_batch b;
    const int rc = pnetgpu_ring_wait(ring, &b);
    if (rc) return rc;
    for (uint64_t i = 0; i < b.n_frames; ++i) dump_frame(&b, i);
    return 0;
}

/* Print every batch in flight (the frames submitted so far). */
static int drain_all(pnetgpu_ring* ring) {
    int rc;
    while (!(rc = drain_one(ring))) {
    }
    return rc == PNETGPU_EEMPTY ? 0 : rc;
}

/* Live capture: up to `count` frames (-1 = no limit); a wait of idle_ms
 * without a retired block ends the capture (-1 = wait on). */
static int live(const char* ifname, long long count, int idle_ms) {
    pnetgpu_afp* afp = NULL;
    int rc = pnetgpu_afp_open(ifname, 1u << 20, 64, 10, &afp);
    if (rc) {
        fprintf(stderr, "pcapdump: %s: %s\n", ifname, rc == PNETGPU_ESYS ? strerror(errno) : pnetgpu_strerror(rc));
        return 1;
    }
    const uint8_t* base = NULL;
    uint64_t bytes = 0;
    uint32_t block_bytes = 0, n_blocks = 0;
    rc = pnetgpu_afp_ring(afp, &base, &bytes, &block_bytes, &n_blocks);
    const int registered = !rc && pnetgpu_host_register((void*)base, bytes) == PNETGPU_OK;
    pnetgpu_ctx* ctx = NULL;
    pnetgpu_ring* ring = NULL;
    if (!rc) rc = pnetgpu_ctx_create(0, &ctx);
    if (!rc) rc = pnetgpu_ring_create(ctx, 64u << 20, 1u << 18, 0, &ring);
    if (!rc) rc = pnetgpu_ring_set_columns(ring, DUMP_COLUMNS);
    /* a TPACKET_V3 packet takes at least its 48-B header plus 16-B-aligned data */
    const uint64_t cap = block_bytes / 64u + 1u;
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * cap);
    uint32_t* lens = (uint32_t*)malloc(sizeof(uint32_t) * cap);
    if (!rc && (!offs || !lens)) rc = PNETGPU_ENOMEM;
    long long seen = 0;
    while (!rc && (count < 0 || seen < count)) {
        uint64_t n = 0;
        uint32_t blk = 0;
        rc = pnetgpu_afp_next_block(afp, idle_ms < 0 ? 1000 : idle_ms, offs, lens, NULL, cap, &n, &blk);
        if (rc == PNETGPU_EEMPTY) {
            rc = 0;
            if (idle_ms >= 0) break;
            continue;
        }
        if (rc) break;
        if (count >= 0 && (long long)n > count - seen) n = (uint64_t)(count - seen);
        for (uint64_t k = 0; !rc && k < n;) {
            uint64_t taken = 0;
            rc = pnetgpu_ring_submit_region(ring, base, offs + k, lens + k, n - k, &taken, NULL);
            if (rc == PNETGPU_EBUSY) rc = drain_one(ring);
            else k += taken;
        }
        if (!rc) rc = drain_all(ring);   /* the block is read until its batches are waited */
        if (!rc) rc = pnetgpu_afp_release_block(afp, blk);
        seen += (long long)n;
        fflush(stdout);
    }
    if (rc) fprintf(stderr, "pcapdump: %s\n", pnetgpu_strerror(rc));
    if (ring) pnetgpu_ring_destroy(ring);
    if (ctx) pnetgpu_ctx_destroy(ctx);
    if (registered) pnetgpu_host_unregister((void*)base);
    pnetgpu_afp_close(afp);
    free(offs);
    free(lens);
    return rc ? 1 : 0;
}

int main(int argc, char** argv) {
    int opt, named = 0, idle_ms = -1;
    const char* iface = NULL;
    long long count = -1;
    while ((opt = getopt(argc, argv, "i:cl:n:w:")) != -1) {
        if (opt == 'i') g_name = optarg, named = 1;
        else if (opt == 'c') g_csum = 1;
        else if (opt == 'l') iface = optarg;
        else if (opt == 'n') count = atoll(optarg);
        else if (opt == 'w') idle_ms = atoi(optarg);
        else return 2;
    }
    if (iface ? optind != argc || count < -1 : optind != argc - 1) {
        fprintf(stderr, "usage: pcapdump [-i NAME] [-c] FILE.pcap\n"
                        "       pcapdump [-i NAME] [-c] -l IFACE [-n COUNT] [-w MS]\n");
        return 2;
    }
    if (iface) {
        if (!named) g_name = iface;
        return live(iface, count, idle_ms);
    }
    const int fd = open(argv[optind], O_RDONLY);
    struct stat sb;
    if (fd < 0 || fstat(fd, &sb) != 0) {
        fprintf(stderr, "pcapdump: %s: %s\n", argv[optind], strerror(errno));
        return 1;
    }
    const uint64_t bytes = (uint64_t)sb.st_size;
    uint8_t* img = bytes ? (uint8_t*)mmap(NULL, bytes, PROT_READ, MAP_PRIVATE, fd, 0) : NULL;
    if (bytes && img == (uint8_t*)MAP_FAILED) {
        fprintf(stderr, "pcapdump: mmap: %s\n", strerror(errno));
        return 1;
    }
    /* direct DMA from the mapping when it can be page-locked, staged copies otherwise */
    const int registered = bytes && pnetgpu_host_register(img, bytes) == PNETGPU_OK;

    /* Ethernet captures take packetdump's chain; raw-IP ones (tun devices,
     * LINKTYPE_RAW / IPV4 / IPV6) start at the IP header: PNETGPU_RX_L3 */
    uint32_t linktype = 1, flags = 0;
    int rc = bytes ? pnetgpu_pcap_info(img, bytes, &linktype, &flags) : PNETGPU_OK;
    g_l3 = (flags & PNETGPU_RX_L3) != 0;
    pnetgpu_ctx* ctx = NULL;
    pnetgpu_ring* ring = NULL;
    if (!rc) rc = pnetgpu_ctx_create(0, &ctx);
    if (!rc) rc = pnetgpu_ring_create(ctx, 64u << 20, 1u << 18, flags, &ring);
    if (!rc) rc = pnetgpu_ring_set_columns(ring, DUMP_COLUMNS);
    enum { kCap = 1 << 16 };
    uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * kCap);
    uint32_t* lens = (uint32_t*)malloc(sizeof(uint32_t) * kCap);
    if (!offs || !lens) rc = PNETGPU_ENOMEM;
    uint64_t pos = 0;
    while (!rc && pos < bytes) {
        uint64_t n = 0;
        rc = pnetgpu_pcap_scan(img, bytes, &pos, offs, lens, kCap, &n);
        for (uint64_t k = 0; !rc && k < n;) {
            uint64_t taken = 0;
            rc = pnetgpu_ring_submit_region(ring, img, offs + k, lens + k, n - k, &taken, NULL);
            if (rc == PNETGPU_EBUSY) rc = drain_one(ring);   /* every slot in flight: print the oldest */
            else k += taken;
        }
    }
    while (!rc) rc = drain_one(ring);
    if (rc == PNETGPU_EEMPTY) rc = 0;
    if (rc) fprintf(stderr, "pcapdump: %s\n", pnetgpu_strerror(rc));
    if (ring) pnetgpu_ring_destroy(ring);
    if (ctx) pnetgpu_ctx_destroy(ctx);
    if (registered) pnetgpu_host_unregister(img);
    if (bytes) munmap(img, bytes);
    close(fd);
    free(offs);
    free(lens);
    return rc ? 1 : 0;
}
