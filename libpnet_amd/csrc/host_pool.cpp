// host_pool.cpp — persistent fork-join pool for the batch producers (host_pool.h).
//
// Round 5 split large pushes over fresh std::threads per call, sized from
// hardware_concurrency() (256 on the GPU hosts) and synchronised with
// yield-spinning barriers: under the hosts' 16-CPU cgroup quota, 16 spinning
// threads plus the caller and the HIP runtime's own threads got throttled, and
// the pinned-ring producer ran at 0.80x of the plain PCIe pipeline. Here the
// workers are created once, sleep on a condition variable between passes, and
// the pool is sized from the affinity mask and the cgroup quota.
#include "host_pool.h"

#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

namespace pnetgpu {
namespace {

constexpr unsigned kMaxDefaultThreads = 16;
constexpr unsigned kMaxThreads = 64;

// quota / period of one cgroup cpu controller file, as a CPU count (0: none)
double read_quota_v2(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return 0;
    char q[32] = {0};
    unsigned long long p = 0;
    const int got = std::fscanf(f, "%31s %llu", q, &p);
    std::fclose(f);
    if (got != 2 || p == 0 || std::strcmp(q, "max") == 0) return 0;
    return std::strtod(q, nullptr) / (double)p;
}

double read_quota_v1(const std::string& dir) {
    long long q = -1, p = 0;
    if (FILE* f = std::fopen((dir + "/cpu.cfs_quota_us").c_str(), "r")) {
        if (std::fscanf(f, "%lld", &q) != 1) q = -1;
        std::fclose(f);
    }
    if (FILE* f = std::fopen((dir + "/cpu.cfs_period_us").c_str(), "r")) {
        if (std::fscanf(f, "%lld", &p) != 1) p = 0;
        std::fclose(f);
    }
    return q > 0 && p > 0 ? (double)q / (double)p : 0;
}

// The smallest CPU quota on the way from this process's cgroup up to the
// hierarchy root (cgroup v2 cpu.max, else v1 cpu.cfs_quota_us); 0 if unlimited.
double cgroup_quota() {
    double best = 0;
    auto take = [&](double q) {
        if (q > 0 && (best == 0 || q < best)) best = q;
    };
    std::string v2path, v1path;
    if (FILE* f = std::fopen("/proc/self/cgroup", "r")) {
        char line[1024];
        while (std::fgets(line, sizeof line, f)) {
            std::string s(line);
            while (!s.empty() && (s.back() == '\n' || s.back() == '\r')) s.pop_back();
            const size_t a = s.find(':'), b = a == std::string::npos ? a : s.find(':', a + 1);
            if (b == std::string::npos) continue;
            const std::string ctrl = s.substr(a + 1, b - a - 1), path = s.substr(b + 1);
            if (s.compare(0, a, "0") == 0 && ctrl.empty()) v2path = path;
            if (ctrl == "cpu" || ctrl.find("cpu,") == 0 || ctrl.find(",cpu") != std::string::npos) v1path = path;
        }
        std::fclose(f);
    }
    for (std::string p = v2path;; p = p.substr(0, p.find_last_of('/'))) {   // the group, then its parents
        take(read_quota_v2("/sys/fs/cgroup" + p + "/cpu.max"));
        if (p.empty() || p == "/") break;
    }
    take(read_quota_v2("/sys/fs/cgroup/cpu.max"));
    for (const char* mnt : {"/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"}) {
        take(read_quota_v1(mnt));
        if (!v1path.empty() && v1path != "/") take(read_quota_v1(std::string(mnt) + v1path));
    }
    return best;
}

unsigned compute_threads() {
    if (const char* e = std::getenv("PNETGPU_HOST_THREADS")) {
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 1) return (unsigned)std::min<long>(v, kMaxThreads);
    }
    unsigned n = kMaxDefaultThreads;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = std::min(n, (unsigned)std::max(1, CPU_COUNT(&set)));
    const double q = cgroup_quota();
    if (q > 0) n = std::min(n, (unsigned)std::max(1.0, q));
    return std::max(1u, n);
}

class Pool {
public:
    explicit Pool(unsigned nthreads) : nthreads_(nthreads) {}

    // the workers start on the first pass; a thread that cannot be created
    // leaves the pool smaller (a pool of none runs every part on the caller)
    void start() {
        if (started_) return;
        started_ = true;
        for (unsigned id = 1; id < nthreads_; ++id) {
            try {
                workers_.emplace_back([this, id] { loop(id); });
            } catch (...) {
                break;
            }
        }
    }

    void run(unsigned nt, const std::function<void(unsigned)>& fn) {
        std::unique_lock<std::mutex> use(use_mu_, std::try_to_lock);
        if (use.owns_lock()) start();
        const unsigned avail = use.owns_lock() ? 1 + (unsigned)workers_.size() : 1;
        if (nt <= 1 || avail <= 1) {
            for (unsigned t = 0; t < nt; ++t) fn(t);
            return;
        }
        // more parts than threads: the caller runs the surplus after its own
        const unsigned par = std::min(nt, avail);
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &fn;
            job_nt_ = par;
            remaining_ = par - 1;
            ++gen_;
        }
        cv_work_.notify_all();
        fn(0);
        for (unsigned t = par; t < nt; ++t) fn(t);
        std::unique_lock<std::mutex> g(mu_);
        cv_done_.wait(g, [&] { return remaining_ == 0; });
        job_ = nullptr;
    }

    unsigned workers() const { return (unsigned)workers_.size(); }
    unsigned nthreads() const { return nthreads_; }

private:
    void loop(unsigned id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)>* job;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_work_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (id >= job_nt_) continue;
                job = job_;
            }
            (*job)(id);
            std::lock_guard<std::mutex> g(mu_);
            if (--remaining_ == 0) cv_done_.notify_one();
        }
    }

    const unsigned nthreads_;
    bool started_ = false;
    std::vector<std::thread> workers_;
    std::mutex use_mu_;                 // one pass at a time
    std::mutex mu_;
    std::condition_variable cv_work_, cv_done_;
    const std::function<void(unsigned)>* job_ = nullptr;
    unsigned job_nt_ = 0, remaining_ = 0;
    uint64_t gen_ = 0;
};

std::mutex g_pool_mu;
Pool* g_pool = nullptr;   // never destroyed: workers stay parked until the process exits
unsigned g_threads = 0;

// a forked child has none of the parent's workers: it starts a pool of its own
void after_fork_child() {
    g_pool = nullptr;
    new (&g_pool_mu) std::mutex();
}

Pool* pool() {
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (!g_pool) {
        static bool registered = false;
        if (!registered) {
            pthread_atfork(nullptr, nullptr, after_fork_child);
            registered = true;
        }
        if (!g_threads) g_threads = compute_threads();
        g_pool = new (std::nothrow) Pool(g_threads);
    }
    return g_pool;
}

__attribute__((target("avx2"))) void copy_nt_avx2(uint8_t* dst, const uint8_t* src, size_t n) {
    // head: up to the destination's next 32-B boundary
    const size_t head = (32 - ((uintptr_t)dst & 31)) & 31;
    std::memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    size_t i = 0;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256((const __m256i*)(src + i));
        const __m256i b = _mm256_loadu_si256((const __m256i*)(src + i + 32));
        const __m256i c = _mm256_loadu_si256((const __m256i*)(src + i + 64));
        const __m256i d = _mm256_loadu_si256((const __m256i*)(src + i + 96));
        _mm256_stream_si256((__m256i*)(dst + i), a);
        _mm256_stream_si256((__m256i*)(dst + i + 32), b);
        _mm256_stream_si256((__m256i*)(dst + i + 64), c);
        _mm256_stream_si256((__m256i*)(dst + i + 96), d);
    }
    std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();
}

}  // namespace

unsigned host_threads() {
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (!g_threads) g_threads = compute_threads();
    return g_threads;
}

unsigned host_workers_started() {
    std::lock_guard<std::mutex> g(g_pool_mu);
    return g_pool ? g_pool->workers() : 0;
}

void parallel_run(unsigned nt, const std::function<void(unsigned)>& fn) {
    Pool* p = pool();
    if (!p) {
        for (unsigned t = 0; t < nt; ++t) fn(t);
        return;
    }
    p->run(nt, fn);
}

void stage_copy(uint8_t* dst, const uint8_t* src, size_t n) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (n >= (64u << 10) && avx2)
        copy_nt_avx2(dst, src, n);
    else
        std::memcpy(dst, src, n);
}

}  // namespace pnetgpu
