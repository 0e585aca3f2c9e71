// util_host.cpp — pnet_packet::util's free functions over host memory
// (include/pnetgpu_util.h): the host bytes and descriptors are staged into the
// context's device scratch on its own stream, summed by the slice kernels of
// pnetgpu_*_slices (rx_slices.h), and the words copied back; each call is
// synchronous. No CPU arithmetic on the checksum path: the GPU computes every
// word, as for the device-pointer entry points.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "pnetgpu.h"
#include "pnetgpu_util.h"
#include "rx_internal.h"

namespace {

constexpr uint64_t kMaxSlice = 0xFFFFFFFFull;   // the slice kernels' u32 lengths

uint64_t up16(uint64_t x) { return (x + 15) & ~15ull; }

// The reference's usize skipword as the kernels' u32: any word at or past the
// end of a slice (< 4 GiB) skips nothing, and 2 * 0x7FFFFFFF still fits 32 bits.
uint32_t skip32(uint64_t skipword) { return (uint32_t)std::min<uint64_t>(skipword, 0x7FFFFFFFull); }

// One staged call: `items` host ranges copied to their scratch offsets, the
// launch, the result words back, then the stream drained.
struct Copy {
    uint64_t at;
    const void* src;
    uint64_t bytes;
};

template <class Launch>
int staged(pnetgpu_ctx* ctx, uint64_t scratch_bytes, const Copy* copies, int ncopies, uint64_t out_at,
           uint64_t out_bytes, uint16_t* out, Launch launch) {
    uint8_t* d = nullptr;
    hipStream_t st = nullptr;
    if (const int rc = pnetgpu::ctx_util_scratch(ctx, scratch_bytes, &d, &st)) return rc;
    for (int i = 0; i < ncopies; ++i)
        if (copies[i].bytes &&
            hipMemcpyAsync(d + copies[i].at, copies[i].src, copies[i].bytes, hipMemcpyHostToDevice, st) != hipSuccess)
            return pnetgpu::hip_fail(hipGetLastError());
    if (const int rc = launch(d, st)) {
        (void)hipStreamSynchronize(st);        // the copies above may still read caller memory
        return rc;
    }
    if (hipMemcpyAsync(out, d + out_at, out_bytes, hipMemcpyDeviceToHost, st) != hipSuccess) {
        const hipError_t e = hipGetLastError();
        (void)hipStreamSynchronize(st);
        return pnetgpu::hip_fail(e);
    }
    if (const hipError_t e = hipStreamSynchronize(st)) return pnetgpu::hip_fail(e);
    return PNETGPU_OK;
}

// util::ipv4_checksum / ipv6_checksum of one slice (alen = 4 / 16)
int pseudo_one(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t len, uint64_t skipword, const uint8_t* extra,
               uint64_t extra_len, const uint8_t* src, const uint8_t* dst, uint8_t proto, uint16_t* out, int alen) {
    pnetgpu::set_last_hip_error(0);
    if (!ctx || !out || !src || !dst || (len && !data) || (extra_len && !extra)) return PNETGPU_EINVAL;
    if (len > kMaxSlice || extra_len > kMaxSlice) return PNETGPU_EINVAL;
    // scratch: slice | extra slice | descriptors | addresses | protocol | result
    struct Desc {
        uint64_t off, eoff;
        uint32_t len, skip, elen, pad;
    } h{};
    const uint64_t e_at = up16(len);
    const uint64_t data_bytes = e_at + extra_len;
    const uint64_t desc_at = up16(data_bytes) + 16;       // the granule tail of the data stays readable
    const uint64_t addr_at = desc_at + sizeof(Desc);
    const uint64_t proto_at = addr_at + 32;
    const uint64_t out_at = up16(proto_at + 1);
    h.off = 0;
    h.len = (uint32_t)len;
    h.skip = skip32(skipword);
    h.eoff = e_at;
    h.elen = (uint32_t)extra_len;
    uint8_t addrs[32] = {};
    std::memcpy(addrs, src, alen);
    std::memcpy(addrs + alen, dst, alen);
    const Copy copies[] = {{0, data, len}, {e_at, extra, extra_len}, {desc_at, &h, sizeof h},
                           {addr_at, addrs, 2ull * alen}, {proto_at, &proto, 1}};
    const int pseudo = alen == 4 ? 4 : 16;
    return staged(ctx, out_at + 16, copies, 5, out_at, 2, out, [&](uint8_t* d, hipStream_t st) {
        const uint64_t* off = reinterpret_cast<const uint64_t*>(d + desc_at + offsetof(Desc, off));
        const uint64_t* eoff = reinterpret_cast<const uint64_t*>(d + desc_at + offsetof(Desc, eoff));
        const uint32_t* ln = reinterpret_cast<const uint32_t*>(d + desc_at + offsetof(Desc, len));
        const uint32_t* sk = reinterpret_cast<const uint32_t*>(d + desc_at + offsetof(Desc, skip));
        const uint32_t* el = reinterpret_cast<const uint32_t*>(d + desc_at + offsetof(Desc, elen));
        uint16_t* o = reinterpret_cast<uint16_t*>(d + out_at);
        if (extra_len == 0)
            return pseudo == 4 ? pnetgpu_ipv4_checksum_slices(ctx, d, data_bytes, 1, off, ln, sk, d + addr_at,
                                                              d + proto_at, o, st)
                               : pnetgpu_ipv6_checksum_slices(ctx, d, data_bytes, 1, off, ln, sk, d + addr_at,
                                                              d + proto_at, o, st);
        return pseudo == 4 ? pnetgpu_ipv4_checksum_adv_slices(ctx, d, data_bytes, 1, off, ln, sk, eoff, el,
                                                              d + addr_at, d + proto_at, o, st)
                           : pnetgpu_ipv6_checksum_adv_slices(ctx, d, data_bytes, 1, off, ln, sk, eoff, el,
                                                              d + addr_at, d + proto_at, o, st);
    });
}

}  // namespace

extern "C" {

int pnetgpu_util_checksum(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t len, uint64_t skipword, uint16_t* out) {
    pnetgpu::set_last_hip_error(0);
    if (!ctx || !out || (len && !data)) return PNETGPU_EINVAL;
    if (len > kMaxSlice) return PNETGPU_EINVAL;
    const uint64_t off = 0;
    const uint32_t ln = (uint32_t)len, sk = skip32(skipword);
    return pnetgpu_checksum_slices_host(ctx, data, len, 1, &off, &ln, &sk, out);
}

int pnetgpu_util_ipv4_checksum(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t len, uint64_t skipword,
                               const uint8_t* extra, uint64_t extra_len, const uint8_t* source,
                               const uint8_t* destination, uint8_t next_level_protocol, uint16_t* out) {
    return pseudo_one(ctx, data, len, skipword, extra, extra_len, source, destination, next_level_protocol, out, 4);
}

int pnetgpu_util_ipv6_checksum(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t len, uint64_t skipword,
                               const uint8_t* extra, uint64_t extra_len, const uint8_t* source,
                               const uint8_t* destination, uint8_t next_level_protocol, uint16_t* out) {
    return pseudo_one(ctx, data, len, skipword, extra, extra_len, source, destination, next_level_protocol, out, 16);
}

int pnetgpu_checksum_slices_host(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes, uint64_t n,
                                 const uint64_t* offsets, const uint32_t* lengths, const uint32_t* skipwords,
                                 uint16_t* out) {
    pnetgpu::set_last_hip_error(0);
    if (!ctx) return PNETGPU_EINVAL;
    if (n == 0) return PNETGPU_OK;
    if (!offsets || !lengths || !skipwords || !out || (data_bytes && !data)) return PNETGPU_EINVAL;
    for (uint64_t i = 0; i < n; ++i)   // host descriptors: checked before anything is staged
        if (offsets[i] > data_bytes || lengths[i] > data_bytes - offsets[i]) return PNETGPU_EINVAL;
    if (n > (UINT64_MAX - data_bytes) / 32) return PNETGPU_EINVAL;
    // scratch: buffer | offsets | lengths | skipwords | results
    const uint64_t off_at = up16(data_bytes) + 16;
    const uint64_t len_at = up16(off_at + 8 * n);
    const uint64_t skip_at = up16(len_at + 4 * n);
    const uint64_t out_at = up16(skip_at + 4 * n);
    const Copy copies[] = {{0, data, data_bytes}, {off_at, offsets, 8 * n}, {len_at, lengths, 4 * n},
                           {skip_at, skipwords, 4 * n}};
    return staged(ctx, out_at + 2 * n + 16, copies, 4, out_at, 2 * n, out, [&](uint8_t* d, hipStream_t st) {
        return pnetgpu_checksum_slices(ctx, d, data_bytes, n, reinterpret_cast<const uint64_t*>(d + off_at),
                                       reinterpret_cast<const uint32_t*>(d + len_at),
                                       reinterpret_cast<const uint32_t*>(d + skip_at),
                                       reinterpret_cast<uint16_t*>(d + out_at), st);
    });
}

}  // extern "C"
