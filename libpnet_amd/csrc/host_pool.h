// host_pool.h — the host threads behind the batch producers' parallel passes
// (pnetgpu_ring_push_many, pnetgpu_batch_pack): one persistent fork-join pool
// per process, sized from what the process may actually run on.
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>

namespace pnetgpu {

// Threads a parallel pass uses, the caller included: PNETGPU_HOST_THREADS if
// set (1..64), else min(16, CPUs in the affinity mask, the cgroup's cpu.max /
// cfs quota rounded down), at least 1. Read once per process.
unsigned host_threads();
// Worker threads the pool has started so far (host_threads() - 1 once used, 0 before).
unsigned host_workers_started();

// Runs fn(t) for t in [0, nt) and returns when every part has returned: part 0
// on the calling thread, the others on the pool's persistent workers, which
// sleep on a condition variable between passes (no spinning). nt is clamped to
// host_threads(). While another thread's pass holds the pool, or when no
// worker could be started, the parts run one after another on the caller.
void parallel_run(unsigned nt, const std::function<void(unsigned)>& fn);

// memcpy for batch staging: large copies into memory the CPU will not read
// again (pinned batches the DMA engine reads) use non-temporal stores, which
// skip the read-for-ownership of every destination line; ends with a store fence.
void stage_copy(uint8_t* dst, const uint8_t* src, size_t n);

}  // namespace pnetgpu
