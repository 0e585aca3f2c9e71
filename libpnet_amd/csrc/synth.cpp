// synth.cpp — seeded synthetic frame producer (include/pnetgpu_synth.h).
//
// Host-side data source for the benchmark and the GPU tests: it plays the role
// of the frame producer (a NIC ring / pnet_datalink receiver), building frames
// as the reference's own builders do (benches/rs_sender.rs:25-101 and the
// pnet_packet setters) and filling their checksums so they verify. It is not a
// checker: parity is always judged against oracle/, never against this file.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "pnetgpu.h"
#include "pnetgpu_synth.h"

namespace {

inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Rng {
    uint64_t s;
    uint64_t next() { return s = splitmix64(s); }
    uint32_t u32() { return (uint32_t)(next() >> 32); }
    void bytes(uint8_t* p, size_t n) {
        while (n >= 8) {
            uint64_t v = next();
            std::memcpy(p, &v, 8);
            p += 8;
            n -= 8;
        }
        if (n) {
            uint64_t v = next();
            std::memcpy(p, &v, n);
        }
    }
};

inline void put16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

// Internet checksum arithmetic used only to BUILD valid frames (RFC 1071 as in
// pnet_packet/src/util.rs); the parity checker is oracle/, not this.
uint32_t sum_be(const uint8_t* p, size_t n) {
    uint32_t s = 0;
    size_t i = 0;
    for (; i + 1 < n; i += 2) s += ((uint32_t)p[i] << 8) | p[i + 1];
    if (n & 1) s += (uint32_t)p[n - 1] << 8;
    return s;
}
uint16_t fin(uint32_t s) {
    while (s >> 16) s = (s & 0xFFFF) + (s >> 16);
    return (uint16_t)~s;
}

constexpr uint64_t kSeedBase = 0x9E3779B97F4A7C15ull;

uint64_t frame_seed(uint64_t seed, int workload, uint64_t i) {
    return splitmix64(seed ^ kSeedBase ^ ((uint64_t)workload << 56) ^ splitmix64(i));
}

// IMIX size class: 64/576/1500 B at 7:4:1 (BASELINE.json configs[3])
uint32_t imix_len(uint64_t seed, uint64_t i) {
    const uint32_t r = (uint32_t)(frame_seed(seed, 99, i) % 12);
    return r < 7 ? 64u : (r < 11 ? 576u : 1500u);
}

struct Built {
    int ip_bad, l4_bad;
};

void eth_header(uint8_t* f, Rng& r, uint16_t ethertype, bool zero_macs) {
    if (zero_macs) std::memset(f, 0, 12);
    else r.bytes(f, 12);
    put16(f + 12, ethertype);
}

// IPv4 header (IHL 5) at f+14 with checksum (ipv4::checksum, skipword 5)
void ipv4_header(uint8_t* ip, Rng& r, uint8_t proto, uint16_t total_len, bool rs_sender) {
    std::memset(ip, 0, 20);
    ip[0] = 0x45;
    put16(ip + 2, total_len);
    if (rs_sender) {           // benches/rs_sender.rs:29-36
        ip[8] = 4;
        ip[9] = proto;
        ip[12] = 127; ip[15] = 1;
        ip[16] = 127; ip[19] = 1;
    } else {
        ip[1] = (uint8_t)(r.u32() & 0xFC);
        put16(ip + 4, r.u32() & 0xFFFF);
        ip[6] = 0x40;          // DF
        ip[8] = (uint8_t)(32 + (r.u32() & 63));
        ip[9] = proto;
        r.bytes(ip + 12, 8);
    }
    put16(ip + 10, fin(sum_be(ip, 20)));
}

uint32_t pseudo_v4(const uint8_t* ip, uint8_t proto, uint32_t l4len) {
    return sum_be(ip + 12, 8) + proto + l4len;
}
uint32_t pseudo_v6(const uint8_t* ip6, uint8_t proto, uint32_t l4len) {
    return sum_be(ip6 + 8, 32) + proto + l4len;
}

// L4 segment at l4 (length n >= header) with checksum given the pseudo-header sum
void udp_seg(uint8_t* l4, uint32_t n, uint32_t data_len, Rng& r, uint32_t pseudo, bool rs_sender) {
    if (rs_sender) {           // benches/rs_sender.rs:44-72
        put16(l4, 1234);
        put16(l4 + 2, 1234);
        std::memcpy(l4 + 8, "rmesg", 5);
    } else {
        put16(l4, r.u32() & 0xFFFF);
        put16(l4 + 2, r.u32() & 0xFFFF);
        r.bytes(l4 + 8, data_len);
    }
    put16(l4 + 4, 8 + data_len);
    put16(l4 + 6, 0);
    put16(l4 + 6, fin(pseudo + sum_be(l4, n)));
}

void tcp_seg(uint8_t* l4, uint32_t n, Rng& r, uint32_t pseudo) {
    r.bytes(l4, 12);           // ports, seq, ack
    l4[12] = 5 << 4;           // data offset 5, no options
    l4[13] = (uint8_t)(r.u32() & 0x3F) | 0x10;
    put16(l4 + 14, r.u32() & 0xFFFF);
    put16(l4 + 16, 0);
    put16(l4 + 18, 0);
    r.bytes(l4 + 20, n - 20);
    put16(l4 + 16, fin(pseudo + sum_be(l4, n)));
}

void icmp_echo(uint8_t* l4, uint32_t n, Rng& r) {
    l4[0] = 8;                 // echo request (icmp.rs:303-314)
    l4[1] = 0;
    put16(l4 + 2, 0);
    put16(l4 + 4, r.u32() & 0xFFFF);
    put16(l4 + 6, r.u32() & 0xFFFF);
    r.bytes(l4 + 8, n - 8);
    put16(l4 + 2, fin(sum_be(l4, n)));
}

// Builds frame i of `workload` into f (length len). Returns which checksum the
// optional corruption breaks.
Built build(int workload, uint64_t seed, uint64_t i, uint32_t corrupt_ppm, uint8_t* f, uint32_t len) {
    Rng r{frame_seed(seed, workload, i)};
    std::memset(f, 0, len);
    Built b{0, 0};
    uint32_t l4off = 0, l4hdr = 0, l4end = 0;
    bool v4 = true;
    switch (workload) {
        case PNETGPU_SYNTH_RS_SENDER:
        case PNETGPU_SYNTH_UDP64: {
            const bool rs = workload == PNETGPU_SYNTH_RS_SENDER;
            eth_header(f, r, 0x0800, rs);
            ipv4_header(f + 14, r, 17, 20 + 8 + 5, rs);   // 17 bytes of Ethernet padding follow
            udp_seg(f + 34, 13, 5, r, pseudo_v4(f + 14, 17, 13), rs);
            l4off = 34; l4hdr = 8; l4end = 47;
            break;
        }
        case PNETGPU_SYNTH_TCP1500: {
            eth_header(f, r, 0x0800, false);
            ipv4_header(f + 14, r, 6, (uint16_t)(len - 14), false);
            tcp_seg(f + 34, len - 34, r, pseudo_v4(f + 14, 6, len - 34));
            l4off = 34; l4hdr = 20; l4end = len;
            break;
        }
        case PNETGPU_SYNTH_UDP1500: {
            // rs_sender.rs:54-72's frame at full MTU: Eth 14 | IPv4 20 (total_length
            // 1486) | UDP 8 (length 1466) | 1458 random data bytes, no padding
            eth_header(f, r, 0x0800, false);
            ipv4_header(f + 14, r, 17, (uint16_t)(len - 14), false);
            const uint32_t n = len - 34;
            udp_seg(f + 34, n, n - 8, r, pseudo_v4(f + 14, 17, n), false);
            l4off = 34; l4hdr = 8; l4end = len;
            break;
        }
        case PNETGPU_SYNTH_IMIX: {
            eth_header(f, r, 0x0800, false);
            const uint32_t k = (uint32_t)(r.next() % 3);
            const uint8_t proto = k == 0 ? 17 : (k == 1 ? 6 : 1);
            ipv4_header(f + 14, r, proto, (uint16_t)(len - 14), false);
            const uint32_t n = len - 34;
            if (proto == 17) { udp_seg(f + 34, n, n - 8, r, pseudo_v4(f + 14, 17, n), false); l4hdr = 8; }
            else if (proto == 6) { tcp_seg(f + 34, n, r, pseudo_v4(f + 14, 6, n)); l4hdr = 20; }
            else { icmp_echo(f + 34, n, r); l4hdr = 8; }
            l4off = 34; l4end = len;
            break;
        }
        case PNETGPU_SYNTH_UDP6_JUMBO: {
            v4 = false;
            eth_header(f, r, 0x86DD, false);
            uint8_t* ip6 = f + 14;
            const uint32_t n = len - 54;
            ip6[0] = 0x60;
            put16(ip6 + 4, n);
            ip6[6] = 17;
            ip6[7] = 64;
            r.bytes(ip6 + 8, 32);
            udp_seg(f + 54, n, n - 8, r, pseudo_v6(ip6, 17, n), false);
            l4off = 54; l4hdr = 8; l4end = len;
            break;
        }
        default: break;
    }
    if (corrupt_ppm && (splitmix64(r.next()) % 1000000u) < corrupt_ppm) {
        const uint64_t x = r.next();
        const uint8_t flip = (uint8_t)(1 + (x & 0xFF) % 255);
        if (v4 && ((x >> 8) & 1)) {
            f[14 + 4 + (uint32_t)((x >> 16) % 5)] ^= flip;   // id / flags / frag / ttl
            b.ip_bad = 1;
        } else {
            const uint32_t lo = l4off + l4hdr, span = l4end - lo;
            f[lo + (uint32_t)((x >> 16) % span)] ^= flip;   // L4 payload byte
            b.l4_bad = 1;
        }
    }
    return b;
}

bool layout(int workload, uint64_t first, uint64_t n, uint64_t seed, uint64_t* total, uint32_t* stride,
            uint32_t* flen) {
    switch (workload) {
        case PNETGPU_SYNTH_RS_SENDER:
        case PNETGPU_SYNTH_UDP64: *stride = 64; break;
        case PNETGPU_SYNTH_TCP1500:
        case PNETGPU_SYNTH_UDP1500: *stride = 1500; break;
        case PNETGPU_SYNTH_UDP6_JUMBO: *stride = 9000; break;
        case PNETGPU_SYNTH_IMIX: *stride = 0; break;
        default: return false;
    }
    *flen = *stride;
    uint64_t bytes = 0;
    if (*stride) {
        bytes = n * (uint64_t)*stride;
    } else {
        for (uint64_t i = first; i < first + n; ++i) bytes += imix_len(seed, i);
    }
    *total = (bytes + 15) / 16 * 16 + 16;
    return true;
}

template <class F>
void parallel_for(uint64_t n, int nthreads, F fn) {
    nthreads = std::max(1, std::min(nthreads, 256));
    if (nthreads == 1 || n < 4096) {
        fn(0, n, 0);
        return;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back(fn, n * t / nthreads, n * (t + 1) / nthreads, t);
    for (auto& x : th) x.join();
}

}  // namespace

extern "C" {

int pnetgpu_synth_layout_range(int workload, uint64_t first, uint64_t n, uint64_t seed, uint64_t* total_bytes,
                               uint32_t* stride, uint32_t* frame_len) {
    if (!total_bytes || !stride || !frame_len || n > UINT64_MAX - first) return PNETGPU_EINVAL;
    return layout(workload, first, n, seed, total_bytes, stride, frame_len) ? PNETGPU_OK : PNETGPU_EINVAL;
}

int pnetgpu_synth_layout(int workload, uint64_t n, uint64_t seed, uint64_t* total_bytes, uint32_t* stride,
                         uint32_t* frame_len) {
    return pnetgpu_synth_layout_range(workload, 0, n, seed, total_bytes, stride, frame_len);
}

int pnetgpu_synth_lengths(int workload, uint64_t first, uint64_t n, uint64_t seed, uint32_t* lengths) {
    uint64_t total = 0;
    uint32_t stride = 0, flen = 0;
    if (!lengths || n > UINT64_MAX - first || !layout(workload, 0, 0, seed, &total, &stride, &flen))
        return PNETGPU_EINVAL;
    for (uint64_t i = 0; i < n; ++i) lengths[i] = stride ? stride : imix_len(seed, first + i);
    return PNETGPU_OK;
}

int pnetgpu_synth_fill_range(int workload, uint64_t first, uint64_t n, uint64_t seed, uint32_t corrupt_ppm,
                             uint8_t* buf, uint64_t buf_bytes, uint64_t* offsets, uint32_t* lengths,
                             uint64_t expect[PNETGPU_SYNTH_NEXP], int nthreads) {
    uint64_t total = 0;
    uint32_t stride = 0, flen = 0;
    if (!buf || n > UINT64_MAX - first || !layout(workload, first, n, seed, &total, &stride, &flen) ||
        buf_bytes < total)
        return PNETGPU_EINVAL;
    if (stride == 0 && (!offsets || !lengths)) return PNETGPU_EINVAL;
    if (stride == 0) {
        uint64_t pos = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t l = imix_len(seed, first + i);
            offsets[i] = pos;
            lengths[i] = l;
            pos += l;
        }
    }
    std::memset(buf + (total >= 32 ? total - 32 : 0), 0, total >= 32 ? 32 : total);  // readable zero tail
    std::vector<uint64_t> ipb(256, 0), l4b(256, 0), byt(256, 0);
    parallel_for(n, nthreads, [&](uint64_t lo, uint64_t hi, int t) {
        uint64_t a = 0, b = 0, c = 0;
        for (uint64_t i = lo; i < hi; ++i) {
            const uint64_t off = stride ? i * stride : offsets[i];
            const uint32_t l = stride ? stride : lengths[i];
            Built r = build(workload, seed, first + i, corrupt_ppm, buf + off, l);   // frame first + i of the batch
            a += r.ip_bad;
            b += r.l4_bad;
            c += l;
        }
        ipb[t] = a; l4b[t] = b; byt[t] = c;
    });
    if (expect) {
        expect[PNETGPU_SYNTH_EXP_IP_BAD] = expect[PNETGPU_SYNTH_EXP_L4_BAD] = expect[PNETGPU_SYNTH_EXP_BYTES] = 0;
        for (int t = 0; t < 256; ++t) {
            expect[PNETGPU_SYNTH_EXP_IP_BAD] += ipb[t];
            expect[PNETGPU_SYNTH_EXP_L4_BAD] += l4b[t];
            expect[PNETGPU_SYNTH_EXP_BYTES] += byt[t];
        }
    }
    return PNETGPU_OK;
}

int pnetgpu_synth_fill(int workload, uint64_t n, uint64_t seed, uint32_t corrupt_ppm, uint8_t* buf,
                       uint64_t buf_bytes, uint64_t* offsets, uint32_t* lengths,
                       uint64_t expect[PNETGPU_SYNTH_NEXP], int nthreads) {
    return pnetgpu_synth_fill_range(workload, 0, n, seed, corrupt_ppm, buf, buf_bytes, offsets, lengths, expect,
                                    nthreads);
}

}  // extern "C"
