// pack_compact_check.cpp — the ring push's pack (ring.cpp pack_frames) with the
// compact descriptor arrays it ships (u32 offsets, u16 lengths), on the CPU:
// pushes of 1..120k frames starting at any descriptor index (the slot's fill
// level), fixed and mixed lengths, with and without source gaps, cut by the
// slot's byte room. Every compact descriptor must equal its u64 / u32 one, and
// nothing outside the push's index range may be written. Built by
// libpnet_amd/Makefile `compact-check` (ring.cpp is included for its static
// pack_frames); exits non-zero on any mismatch.
#include "../libpnet_amd/csrc/ring.cpp"

#include <cstdio>
#include <random>

int main() {
    std::mt19937_64 rng(5);
    int bad = 0;
    for (int trial = 0; trial < 60; ++trial) {
        const uint64_t m = trial % 3 == 0 ? 70000 + rng() % 50000 : 1 + rng() % 5000;
        const uint64_t start = rng() % 100;
        std::vector<uint32_t> lens(m);
        std::vector<uint64_t> offs(m);
        uint64_t o = 0;
        for (uint64_t i = 0; i < m; ++i) {
            lens[i] = trial % 2 ? 64 : 20 + rng() % 1500;
            offs[i] = o;
            o += lens[i] + (trial % 4 == 1 ? rng() % 3 : 0);
        }
        std::vector<uint8_t> src(o + 64);
        for (auto& b : src) b = (uint8_t)rng();
        const uint64_t room = trial % 5 == 0 ? o / 2 : o + 64;
        std::vector<uint8_t> dst(room + 64);
        std::vector<uint64_t> o64(start + m + 1, ~0ull);
        std::vector<uint32_t> l32(start + m + 1, ~0u), o32(start + m + 1, 0xDEADBEEFu);
        std::vector<uint16_t> l16(start + m + 1, 0xBEEF);
        PackStats st;
        const uint64_t k = pack_frames(src.data(), offs.data(), lens.data(), m, room, dst.data(), 0, o64.data() + start,
                                       l32.data() + start, o32.data() + start, l16.data() + start, &st);
        uint64_t at = 0;
        for (uint64_t i = 0; i < k && !bad; ++i) {
            const uint64_t j = start + i;
            if (o64[j] != at || l32[j] != lens[i] || o32[j] != (uint32_t)at || l16[j] != (uint16_t)lens[i] ||
                std::memcmp(dst.data() + at, src.data() + offs[i], lens[i])) {
                std::printf("trial %d: frame %lu wrong\n", trial, (unsigned long)i);
                ++bad;
            }
            at += lens[i];
        }
        for (uint64_t j : {start + k, start ? start - 1 : start + k})
            if (l16[j] != 0xBEEF || o32[j] != 0xDEADBEEFu || l32[j] != ~0u || o64[j] != ~0ull) {
                std::printf("trial %d: wrote outside the push at %lu\n", trial, (unsigned long)j);
                ++bad;
            }
        if (k == 0 || st.bytes != at) {
            std::printf("trial %d: k=%lu bytes=%lu\n", trial, (unsigned long)k, (unsigned long)st.bytes);
            ++bad;
        }
    }
    // skip_len: a push whose frames all have that length leaves the compact
    // arrays untouched (and says so); any other length in it writes them all
    for (int trial = 0; trial < 12; ++trial) {
        const uint64_t m = trial % 2 ? 70000 + rng() % 50000 : 1 + rng() % 5000;
        const bool odd = trial % 3 == 2;                  // one frame of another length
        std::vector<uint32_t> lens(m, 64);
        if (odd) lens[rng() % m] = 60;
        std::vector<uint64_t> offs(m);
        for (uint64_t i = 0; i < m; ++i) offs[i] = i * 64;
        std::vector<uint8_t> src(m * 64 + 64, 3), dst(m * 64 + 64);
        std::vector<uint64_t> o64(m);
        std::vector<uint32_t> l32(m), o32(m, 0xDEADBEEFu);
        std::vector<uint16_t> l16(m, 0xBEEF);
        PackStats st;
        const uint64_t k = pack_frames(src.data(), offs.data(), lens.data(), m, m * 64, dst.data(), 0, o64.data(),
                                       l32.data(), o32.data(), l16.data(), &st, 64);
        const bool untouched = o32[0] == 0xDEADBEEFu && l16[0] == 0xBEEF && o32[k - 1] == 0xDEADBEEFu;
        const bool written = o32[k - 1] == (uint32_t)o64[k - 1] && l16[k - 1] == (uint16_t)l32[k - 1];
        if (k != m || st.compact_skipped == odd || (odd ? !written : !untouched)) {
            std::printf("skip trial %d: k=%lu skipped=%d odd=%d\n", trial, (unsigned long)k, st.compact_skipped, odd);
            ++bad;
        }
    }
    std::printf("pack_compact_check: %s (%u host threads)\n", bad ? "FAILED" : "ok", pnetgpu::host_threads());
    return bad != 0;
}
