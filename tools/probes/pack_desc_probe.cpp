// pack_desc_probe — the ring's pack (ring.cpp pack_frames) with and without the
// compact descriptor arrays it also writes (u32 offsets, u16 lengths), into
// malloc'd, hipHostMalloc'd or mmap'd + registered memory: what slows the push?
// 2^20 64-B frames per pack from a 256-MiB source, best-of-rounds GB/s of frame
// bytes. CPU only (hipHostMalloc needs a GPU: that leg is skipped without one).
//
//   make -C libpnet_amd && hipcc -O3 -std=c++17 -Iinclude -Ilibpnet_amd/csrc -c \
//     tools/probes/pack_desc_probe.cpp -o /tmp/pdp.o && hipcc --offload-arch=gfx950 /tmp/pdp.o \
//     -Llibpnet_amd -lpnetgpu -Wl,-rpath,$PWD/libpnet_amd -lpthread -o /tmp/pdp && /tmp/pdp
#include "../../libpnet_amd/csrc/ring.cpp"

#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// kind 0: aligned_alloc; 1: hipHostMalloc; 2: mmap + hipHostRegister;
// 3: mmap + MADV_HUGEPAGE + hipHostRegister
static const char* kKinds[] = {"malloc", "hipHostMalloc", "mmap+register", "mmap+thp+register"};
template <class T>
static T* alloc(size_t n, int kind) {
    void* p = nullptr;
    const size_t b = (n * sizeof(T) + (2u << 20) - 1) & ~size_t((2u << 20) - 1);
    if (kind == 1) {
        if (hipHostMalloc(&p, b, hipHostMallocDefault) != hipSuccess) return nullptr;
    } else if (kind >= 2) {
        p = mmap(nullptr, b, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) return nullptr;
        if (kind == 3) madvise(p, b, MADV_HUGEPAGE);
    } else {
        p = std::aligned_alloc(4096, b);
    }
    std::memset(p, 1, b);
    if (kind >= 2 && hipHostRegister(p, b, hipHostRegisterDefault) != hipSuccess) return nullptr;
    return static_cast<T*>(p);
}

int main() {
    const uint64_t n = 1 << 20, total = 4 * n;
    std::vector<uint8_t> src(total * 64, 7);
    std::vector<uint64_t> offs(total);
    std::vector<uint32_t> lens(total, 64);
    for (uint64_t i = 0; i < total; ++i) offs[i] = i * 64;
    int ndev = 0;
    const bool gpu = hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0;
    std::printf("host_threads %u gpu %d\n", pnetgpu::host_threads(), gpu ? 1 : 0);
    for (int pinned = 0; pinned <= (gpu ? 3 : 0); ++pinned) {
        uint8_t* dst = alloc<uint8_t>(64ull << 20, pinned);
        uint64_t* o64 = alloc<uint64_t>(n, pinned);
        uint32_t* l32 = alloc<uint32_t>(n, pinned);
        uint32_t* o32 = alloc<uint32_t>(n, pinned);
        uint16_t* l16 = alloc<uint16_t>(n, pinned);
        if (!dst || !o64 || !l32 || !o32 || !l16) {
            std::printf("%s: allocation failed\n", kKinds[pinned]);
            continue;
        }
        for (int compact = 0; compact <= 1; ++compact) {
            double best = 0;
            for (int round = 0; round < 5; ++round) {
                uint64_t bytes = 0, i = 0;
                const double t0 = now();
                while (now() - t0 < 0.5) {
                    PackStats st;
                    const uint64_t k = pack_frames(src.data(), offs.data() + i, lens.data() + i, n, 64ull << 20, dst,
                                                   0, o64, l32, compact ? o32 : nullptr, compact ? l16 : nullptr,
                                                   &st);
                    bytes += st.bytes;
                    i = (i + k) % total;
                }
                best = std::max(best, bytes / (now() - t0) / 1e9);
            }
            std::printf("%s compact=%d  %.1f GB/s\n", kKinds[pinned], compact, best);
        }
    }
    return 0;
}
