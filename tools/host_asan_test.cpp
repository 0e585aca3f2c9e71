// host_asan_test.cpp — AddressSanitizer/UBSan run of the library's HOST code
// (no GPU needed): the synthetic-frame producer, the batch producer's parallel
// pack (fuzzed, on the host pool's threads), the classic-pcap and pcapng
// readers and in-memory indexers (fuzzed), the TPACKET_V3 block walk (fuzzed: it parses memory the
// OS kernel writes) and the C-ABI's argument validation. Linked from objects built with
// -fsanitize=address,undefined (libpnet_amd/Makefile target `asan-test`), so
// the sanitizer runtime comes with the executable itself.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pnetgpu.h"
#include "pnetgpu_afpacket.h"
#include "pnetgpu_ring.h"
#include "pnetgpu_synth.h"
#include "pnetgpu_util.h"

static int failures = 0;
static uint32_t rnd();
#define CHECK(c)                                                              \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++failures;                                                       \
        }                                                                     \
    } while (0)

static void put32(std::vector<uint8_t>& b, uint32_t v, bool be) {
    for (int i = 0; i < 4; ++i) b.push_back((uint8_t)(be ? v >> (24 - 8 * i) : v >> (8 * i)));
}
static void put16(std::vector<uint8_t>& b, uint16_t v, bool be) {
    b.push_back((uint8_t)(be ? v >> 8 : v));
    b.push_back((uint8_t)(be ? v : v >> 8));
}

static std::string write_pcap(const char* name, bool be, bool ns, const std::vector<std::vector<uint8_t>>& frames,
                              size_t truncate_to = 0) {
    std::vector<uint8_t> b;
    put32(b, ns ? 0xA1B23C4Du : 0xA1B2C3D4u, be);
    put16(b, 2, be);
    put16(b, 4, be);
    put32(b, 0, be);
    put32(b, 0, be);
    put32(b, 65535, be);
    put32(b, 1, be);   // LINKTYPE_ETHERNET
    for (const auto& f : frames) {
        put32(b, 1, be);
        put32(b, 2, be);
        put32(b, (uint32_t)f.size(), be);
        put32(b, (uint32_t)f.size() + 4, be);
        b.insert(b.end(), f.begin(), f.end());
    }
    if (truncate_to && truncate_to < b.size()) b.resize(truncate_to);
    std::string path = std::string("/tmp/pnet_asan_") + name + ".pcap";
    FILE* fp = std::fopen(path.c_str(), "wb");
    std::fwrite(b.data(), 1, b.size(), fp);
    std::fclose(fp);
    return path;
}

static void test_synth() {
    for (int w = 0; w <= 4; ++w) {
        for (uint64_t n : {1ull, 63ull, 1000ull}) {
            uint64_t total = 0;
            uint32_t stride = 0, flen = 0;
            CHECK(pnetgpu_synth_layout(w, n, 7, &total, &stride, &flen) == 0);
            std::vector<uint8_t> buf(total);
            std::vector<uint64_t> offs(n);
            std::vector<uint32_t> lens(n);
            uint64_t exp[PNETGPU_SYNTH_NEXP] = {};
            CHECK(pnetgpu_synth_fill(w, n, 7, 300000, buf.data(), buf.size(), offs.data(), lens.data(), exp, 3) == 0);
            CHECK(exp[PNETGPU_SYNTH_EXP_BYTES] > 0);
            // a buffer one byte short is refused, not overrun
            if (total > 0)
                CHECK(pnetgpu_synth_fill(w, n, 7, 0, buf.data(), total - 1, offs.data(), lens.data(), exp, 1) != 0);
        }
    }
    uint64_t total = 0;
    uint32_t stride = 0, flen = 0;
    CHECK(pnetgpu_synth_layout(99, 10, 1, &total, &stride, &flen) != 0);
}

static void test_pcap() {
    std::vector<std::vector<uint8_t>> frames;
    for (int i = 0; i < 50; ++i) frames.emplace_back((size_t)(i * 37 % 1600), (uint8_t)i);
    for (int be = 0; be < 2; ++be) {
        for (int ns = 0; ns < 2; ++ns) {
            const std::string p = write_pcap("ok", be, ns, frames);
            pnetgpu_pcap* pc = nullptr;
            CHECK(pnetgpu_pcap_open(p.c_str(), &pc) == 0);
            const uint8_t* f = nullptr;
            uint32_t len = 0;
            size_t k = 0;
            int rc;
            while ((rc = pnetgpu_pcap_next(pc, &f, &len)) == 0) {
                CHECK(k < frames.size() && len == frames[k].size());
                if (k < frames.size() && len == frames[k].size() && len) CHECK(std::memcmp(f, frames[k].data(), len) == 0);
                ++k;
            }
            CHECK(rc == PNETGPU_EEMPTY && k == frames.size());
            pnetgpu_pcap_close(pc);
        }
    }
    // truncated inside a record: the reader stops without reading past the file
    const std::string t = write_pcap("trunc", false, false, frames, 24 + 16 + 10 + 16 + 3);
    pnetgpu_pcap* pc = nullptr;
    if (pnetgpu_pcap_open(t.c_str(), &pc) == 0) {
        const uint8_t* f = nullptr;
        uint32_t len = 0;
        int n = 0;
        while (pnetgpu_pcap_next(pc, &f, &len) == 0 && n < 100) ++n;
        CHECK(n <= 2);
        pnetgpu_pcap_close(pc);
    }
    // not a pcap file / missing file
    const std::string g = "/tmp/pnet_asan_garbage.pcap";
    FILE* fp = std::fopen(g.c_str(), "wb");
    std::fputs("definitely not a capture file", fp);
    std::fclose(fp);
    CHECK(pnetgpu_pcap_open(g.c_str(), &pc) == PNETGPU_EFORMAT);
    CHECK(pnetgpu_pcap_open("/tmp/pnet_asan_does_not_exist.pcap", &pc) != 0);
}

static void test_abi_validation() {
    CHECK(pnetgpu_abi_version() == PNETGPU_ABI_VERSION);
    for (int c = 0; c >= -9; --c) CHECK(pnetgpu_strerror(c) != nullptr && std::strlen(pnetgpu_strerror(c)) > 0);
    CHECK(pnetgpu_strerror(-1000) != nullptr);
    pnetgpu_batch b{};
    pnetgpu_rx_columns cols{};
    CHECK(pnetgpu_rx_process(nullptr, &b, &cols, nullptr) == PNETGPU_EINVAL);
    CHECK(pnetgpu_tx_fill_checksums(nullptr, &b, &cols, nullptr) == PNETGPU_EINVAL);
    uint16_t out[4];
    uint64_t off[4] = {0, 1, 2, 3};
    uint32_t len[4] = {1, 1, 1, 1}, skip[4] = {0, 0, 0, 0};
    uint8_t data[16] = {};
    CHECK(pnetgpu_checksum_slices(nullptr, data, 16, 4, off, len, skip, out, nullptr) == PNETGPU_EINVAL);
    CHECK(pnetgpu_checksum_slices_strided(nullptr, data, 16, 4, 0, 4, 4, 0, out, nullptr) == PNETGPU_EINVAL);
    pnetgpu_slice_desc cd[4] = {{0, 1, 0}, {1, 1, 0}, {2, 1, 0}, {3, 1, 0}};
    CHECK(pnetgpu_checksum_slices_compact(nullptr, data, 16, 4, cd, out, nullptr) == PNETGPU_EINVAL);
    CHECK(pnetgpu_checksum_slices_compact(nullptr, data, 16, 0, cd, out, nullptr) == PNETGPU_EINVAL);
    CHECK(pnetgpu_last_rx_kernel() != nullptr && std::strlen(pnetgpu_last_rx_kernel()) == 0);   // no launch yet
    CHECK(pnetgpu_last_hip_error() == 0);
    CHECK(pnetgpu_ipv4_checksum_adv_slices(nullptr, data, 16, 4, off, len, skip, off, len, data, data, out,
                                           nullptr) == PNETGPU_EINVAL);
    pnetgpu_ring* r = nullptr;
    CHECK(pnetgpu_ring_create(nullptr, 1 << 20, 1024, 0, &r) == PNETGPU_EINVAL);
    pnetgpu_ctx* ctx = nullptr;
    CHECK(pnetgpu_ctx_create(-1, &ctx) != 0);
    pnetgpu_ctx_destroy(nullptr);
    pnetgpu_ring_destroy(nullptr);
    pnetgpu_pcap_close(nullptr);
    // host-memory util entry points (pnetgpu_util.h): argument checks before any HIP call
    uint8_t a4[4] = {};
    CHECK(pnetgpu_util_checksum(nullptr, data, 16, 0, out) == PNETGPU_EINVAL);
    CHECK(pnetgpu_util_ipv4_checksum(nullptr, data, 16, 0, nullptr, 0, a4, a4, 17, out) == PNETGPU_EINVAL);
    CHECK(pnetgpu_util_ipv6_checksum(nullptr, data, 16, 0, nullptr, 0, a4, a4, 17, out) == PNETGPU_EINVAL);
    CHECK(pnetgpu_checksum_slices_host(nullptr, data, 16, 4, off, len, skip, out) == PNETGPU_EINVAL);
    CHECK(pnetgpu_batch_pack(nullptr, off, len, 4, data, 16, off, len, nullptr, nullptr) == PNETGPU_EINVAL);
}

// pnetgpu_batch_pack (the pnetgpu_ring_push_many pass on the persistent host
// pool) over random frame layouts and capacities: the frames taken are the
// longest prefix that fits, copied byte for byte to their packed offsets, and
// nothing is written past the destination (ASan guards its end).
static void test_pack_fuzz() {
    CHECK(pnetgpu_host_threads() >= 1);
    for (int round = 0; round < 40; ++round) {
        const uint64_t n = round % 4 == 0 ? 70000 + rnd() % 40000 : 1 + rnd() % 3000;
        std::vector<uint64_t> offs(n), doff(n, ~0ull);
        std::vector<uint32_t> lens(n), dlen(n, ~0u);
        uint64_t at = 0, total = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint32_t r = rnd() % 100;
            lens[i] = r < 60 ? 64 : r < 90 ? 576 : r < 98 ? 1500 : 9000;
            at += (rnd() % 4 == 0) ? rnd() % 40 : 0;     // gaps: copies break inside chunks
            offs[i] = at;
            at += lens[i];
            total += lens[i];
        }
        std::vector<uint8_t> src(at);
        for (auto& b : src) b = (uint8_t)rnd();
        const uint64_t cap = round % 3 == 0 ? total : 1 + rnd() % (total + 1);
        std::vector<uint8_t> dst(cap);
        uint64_t k = 0, bytes = 0;
        const int rc = pnetgpu_batch_pack(src.data(), offs.data(), lens.data(), n, dst.data(), cap, doff.data(),
                                          dlen.data(), &k, &bytes);
        uint64_t want = 0, wb = 0;
        while (want < n && lens[want] <= cap - wb) wb += lens[want++];
        CHECK(want == 0 ? rc == PNETGPU_EFULL : rc == PNETGPU_OK);
        CHECK(k == want && bytes == wb);
        uint64_t o = 0;
        for (uint64_t i = 0; i < k; ++i) {
            CHECK(doff[i] == o && dlen[i] == lens[i]);
            CHECK(std::memcmp(dst.data() + o, src.data() + offs[i], lens[i]) == 0);
            o += lens[i];
        }
        CHECK(k == n || doff[k] == ~0ull);              // nothing past the cut
    }
}

// Random mutations of valid TPACKET_V3 blocks and pcap images: every call
// returns a code, and every descriptor it reports lies inside the buffer.
static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    rng_state ^= rng_state << 13;
    rng_state ^= rng_state >> 7;
    rng_state ^= rng_state << 17;
    return (uint32_t)rng_state;
}

static void test_walk_fuzz() {
    const uint32_t kBlock = 8192;
    int ok_blocks = 0;
    for (int iter = 0; iter < 3000; ++iter) {
        std::vector<uint8_t> blk(kBlock, 0);
        const uint32_t n = rnd() % 40;
        uint32_t p = 48, last = 48;
        uint32_t placed = 0;
        for (uint32_t k = 0; k < n; ++k) {
            const uint32_t snap = rnd() % 300, mac = 66;
            if (p + mac + snap > kBlock) break;
            const uint32_t nxt = (mac + snap + 15) & ~15u;
            std::memcpy(&blk[p], &nxt, 4);
            std::memcpy(&blk[p + 12], &snap, 4);
            std::memcpy(&blk[p + 24], &mac, 2);
            last = p;
            p += nxt;
            ++placed;
        }
        if (placed) {
            const uint32_t zero = 0;
            std::memcpy(&blk[last], &zero, 4);
        }
        const uint32_t first = 48, blk_len = placed ? std::min<uint32_t>(p, kBlock) : 48;
        std::memcpy(&blk[12], &placed, 4);
        std::memcpy(&blk[16], &first, 4);
        std::memcpy(&blk[20], &blk_len, 4);
        const int flips = (int)(rnd() % 4);                 // 0: intact
        for (int f = 0; f < flips; ++f) blk[rnd() % std::min<uint32_t>(kBlock, p + 64)] = (uint8_t)rnd();
        uint64_t offs[64];
        uint32_t lens[64], st[64];
        uint64_t got = 0;
        const int rc = pnetgpu_tpacket3_walk(blk.data(), kBlock, 0, offs, lens, st, 64, &got);
        if (flips == 0) CHECK(rc == 0 && got == placed);
        if (rc == 0) {
            ++ok_blocks;
            for (uint64_t k = 0; k < got; ++k) CHECK(offs[k] + lens[k] <= kBlock);
        }
    }
    CHECK(ok_blocks > 1000);
    uint64_t got = 0;
    CHECK(pnetgpu_tpacket3_walk(nullptr, 8192, 0, nullptr, nullptr, nullptr, 0, &got) == PNETGPU_EINVAL);
}

static void test_scan_fuzz() {
    std::vector<std::vector<uint8_t>> frames;
    for (int i = 0; i < 30; ++i) frames.push_back(std::vector<uint8_t>(rnd() % 200, (uint8_t)i));
    const std::string path = write_pcap("fuzz", false, false, frames);
    FILE* f = std::fopen(path.c_str(), "rb");
    std::vector<uint8_t> img(1 << 16);
    img.resize(std::fread(img.data(), 1, img.size(), f));
    std::fclose(f);
    for (int iter = 0; iter < 3000; ++iter) {
        std::vector<uint8_t> m = img;
        const int flips = 1 + (int)(rnd() % 3);
        for (int k = 0; k < flips; ++k) m[rnd() % m.size()] = (uint8_t)rnd();
        const uint64_t cut = rnd() % 3 == 0 ? rnd() % m.size() : m.size();
        uint64_t pos = 0, n = 0, offs[16];
        uint32_t lens[16];
        for (int guard = 0; guard < 100 && pos < cut; ++guard) {
            if (pnetgpu_pcap_scan(m.data(), cut, &pos, offs, lens, 16, &n) != 0) break;
            for (uint64_t k = 0; k < n; ++k) CHECK(offs[k] + lens[k] <= cut);
            if (n == 0) break;
        }
        uint32_t lt = 0, fl = 0;
        (void)pnetgpu_pcap_info(m.data(), cut, &lt, &fl);
    }
}

// pcapng image: SHB, two IDBs, EPB / SPB / PB packets, a skipped block
static std::vector<uint8_t> pcapng_image(bool be, const std::vector<std::vector<uint8_t>>& frames) {
    std::vector<uint8_t> b;
    auto block = [&](uint32_t type, const std::vector<uint8_t>& body) {
        std::vector<uint8_t> padded = body;
        while (padded.size() % 4) padded.push_back(0);
        const uint32_t n = 12 + (uint32_t)padded.size();
        put32(b, type, be);
        put32(b, n, be);
        b.insert(b.end(), padded.begin(), padded.end());
        put32(b, n, be);
    };
    std::vector<uint8_t> shb;
    put32(shb, 0x1A2B3C4Du, be);
    put16(shb, 1, be);
    put16(shb, 0, be);
    put32(shb, 0xFFFFFFFFu, be);
    put32(shb, 0xFFFFFFFFu, be);
    block(0x0A0D0D0Au, shb);
    for (int i = 0; i < 2; ++i) {
        std::vector<uint8_t> idb;
        put16(idb, 1, be);
        put16(idb, 0, be);
        put32(idb, i ? 0u : 150u, be);
        block(1, idb);
    }
    block(0x40000BADu, std::vector<uint8_t>(7, 0x5A));
    for (size_t i = 0; i < frames.size(); ++i) {
        const auto& f = frames[i];
        std::vector<uint8_t> body;
        const uint32_t kind = (uint32_t)(i % 3);
        if (kind == 0) {                                   // EPB
            put32(body, (uint32_t)(i % 2), be);
            put32(body, 0, be);
            put32(body, (uint32_t)i, be);
            put32(body, (uint32_t)f.size(), be);
            put32(body, (uint32_t)f.size(), be);
            body.insert(body.end(), f.begin(), f.end());
            block(6, body);
        } else if (kind == 1) {                            // SPB
            put32(body, (uint32_t)f.size(), be);
            body.insert(body.end(), f.begin(), f.end());
            block(3, body);
        } else {                                           // obsolete PB
            put16(body, (uint16_t)(i % 2), be);
            put16(body, 0, be);
            put32(body, 0, be);
            put32(body, (uint32_t)i, be);
            put32(body, (uint32_t)f.size(), be);
            put32(body, (uint32_t)f.size(), be);
            body.insert(body.end(), f.begin(), f.end());
            block(2, body);
        }
    }
    return b;
}

// The pcapng indexer and streaming reader over mutated and truncated images:
// every descriptor stays inside the image, nothing reads past it (ASan).
static void test_pcapng_fuzz() {
    std::vector<std::vector<uint8_t>> frames;
    for (int i = 0; i < 40; ++i) frames.push_back(std::vector<uint8_t>(rnd() % 200, (uint8_t)i));
    for (int be = 0; be < 2; ++be) {
        const std::vector<uint8_t> img = pcapng_image(be != 0, frames);
        uint64_t pos = 0, n = 0, offs[64];
        uint32_t lens[64];
        CHECK(pnetgpu_pcap_scan(img.data(), img.size(), &pos, offs, lens, 64, &n) == PNETGPU_OK);
        CHECK(n == frames.size() && pos == img.size());
        for (uint64_t k = 0; k < n; ++k)
            CHECK(lens[k] == std::min<uint32_t>((uint32_t)frames[k].size(), k % 3 == 1 ? 150u : 0xFFFFFFFFu));
        for (int iter = 0; iter < 3000; ++iter) {
            std::vector<uint8_t> m = img;
            const int flips = 1 + (int)(rnd() % 3);
            for (int k = 0; k < flips; ++k) m[rnd() % m.size()] = (uint8_t)rnd();
            const uint64_t cut = rnd() % 3 == 0 ? rnd() % m.size() : m.size();
            uint64_t p = 0, got = 0;
            for (int guard = 0; guard < 100 && p < cut; ++guard) {
                if (pnetgpu_pcap_scan(m.data(), cut, &p, offs, lens, 7, &got) != 0) break;
                for (uint64_t k = 0; k < got; ++k) CHECK(offs[k] + lens[k] <= cut);
                if (got == 0) break;
            }
            uint32_t lt = 0, fl = 0;
            (void)pnetgpu_pcap_info(m.data(), cut, &lt, &fl);
            if (iter % 30 == 0) {                            // the streaming reader on the same bytes
                const std::string path = "/tmp/pnet_asan_ng.pcapng";
                FILE* f = std::fopen(path.c_str(), "wb");
                std::fwrite(m.data(), 1, cut, f);
                std::fclose(f);
                pnetgpu_pcap* r = nullptr;
                if (pnetgpu_pcap_open(path.c_str(), &r) == PNETGPU_OK) {
                    const uint8_t* fr;
                    uint32_t len;
                    for (int guard = 0; guard < 200 && pnetgpu_pcap_next(r, &fr, &len) == PNETGPU_OK; ++guard)
                        if (len) CHECK(fr[len - 1] == fr[len - 1]);   // touches the last byte (ASan)
                    pnetgpu_pcap_close(r);
                }
            }
        }
    }
}

int main() {
    test_synth();
    test_pcap();
    test_abi_validation();
    test_pack_fuzz();
    test_walk_fuzz();
    test_scan_fuzz();
    test_pcapng_fuzz();
    std::printf("%s (%d failures)\n", failures ? "FAILED" : "ok", failures);
    return failures ? 1 : 0;
}
