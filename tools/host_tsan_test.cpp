// host_tsan_test.cpp — ThreadSanitizer run of the batch producer's parallel
// pack (pnetgpu_batch_pack = the pnetgpu_ring_push_many pass) on the
// persistent host pool (csrc/host_pool.cpp), no GPU needed: large pushes of
// mixed 64/1500-B frames with gaps, while a second thread packs the same
// frames into its own batch at the same time (one of the two finds the pool
// busy and runs serially). Built with -fsanitize=thread by
// libpnet_amd/Makefile `tsan-test`; exits non-zero on a wrong batch, and TSan
// reports any data race.
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "pnetgpu_ring.h"

int main() {
    unsigned s = 1;
    auto rnd = [&] {
        s = s * 1103515245u + 12345u;
        return s >> 8;
    };
    int bad = 0;
    for (int round = 0; round < 30; ++round) {
        const uint64_t n = 70000 + rnd() % 50000;
        std::vector<uint64_t> o(n), d(n), d2(n);
        std::vector<uint32_t> l(n), dl(n), l2(n);
        uint64_t at = 0;
        for (uint64_t i = 0; i < n; ++i) {
            l[i] = (rnd() % 3) ? 64 : 1500;
            at += rnd() % 3 == 0 ? 8 : 0;
            o[i] = at;
            at += l[i];
        }
        std::vector<uint8_t> src(at), dst(at), dst2(at);
        for (auto& b : src) b = (uint8_t)rnd();
        uint64_t k = 0, b = 0, k2 = 0, b2 = 0;
        std::thread t2([&] {
            pnetgpu_batch_pack(src.data(), o.data(), l.data(), n, dst2.data(), at / 2, d2.data(), l2.data(), &k2, &b2);
        });
        pnetgpu_batch_pack(src.data(), o.data(), l.data(), n, dst.data(), at, d.data(), dl.data(), &k, &b);
        t2.join();
        bad += k != n || k2 == 0 || k2 >= n;
        for (uint64_t i = 0; i < k; ++i) bad += std::memcmp(dst.data() + d[i], src.data() + o[i], l[i]) != 0;
        for (uint64_t i = 0; i < k2; ++i) bad += std::memcmp(dst2.data() + d2[i], src.data() + o[i], l[i]) != 0;
    }
    std::printf("%s (%d bad, %u host threads)\n", bad ? "FAILED" : "ok", bad, pnetgpu_host_threads());
    return bad ? 1 : 0;
}
