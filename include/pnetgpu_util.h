/*
 * pnetgpu_util.h — pnet_packet::util's free functions over HOST memory.
 *
 * The reference's checksum helpers take a host slice and return the word
 * (pnet_packet/src/util.rs:76-150, re-exported as pnet::util,
 * src/util.rs:11-12):
 *
 *   util::checksum(data: &[u8], skipword: usize) -> u16                 util.rs:76-82
 *   util::ipv4_checksum(data, skipword, extra_data, &Ipv4Addr, &Ipv4Addr,
 *                       IpNextHeaderProtocol) -> u16                     util.rs:92-117
 *   util::ipv6_checksum(data, skipword, extra_data, &Ipv6Addr, &Ipv6Addr,
 *                       IpNextHeaderProtocol) -> u16                     util.rs:125-150
 *
 * A caller replacing one of those calls with one of these needs no device
 * memory of its own: the bytes are staged through the context's device
 * scratch on the context's own stream, summed by the same slice kernels as
 * pnetgpu_*_slices (pnetgpu.h), and the call returns with *out set
 * (synchronous). One call costs a launch and two small copies, so these serve
 * API parity and small workloads; batches belong on pnetgpu_rx_process, the
 * *_slices entry points, or pnetgpu_checksum_slices_host below.
 *
 * Lengths: a slice (and an extra slice) must be shorter than 4 GiB
 * (PNETGPU_EINVAL otherwise); skipword is the reference's usize, any value
 * (a word past the slice skips nothing). Results equal a release build of
 * the reference for every length (u32 sums wrap past 64 KiB, pnetgpu.h).
 * One host thread at a time per context, as for every context call.
 */
#ifndef PNETGPU_UTIL_H
#define PNETGPU_UTIL_H

#include <stdint.h>

#include "pnetgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* *out = util::checksum(data[0, len), skipword) */
int pnetgpu_util_checksum(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t len, uint64_t skipword, uint16_t* out);

/* *out = util::ipv4_checksum(data[0, len), skipword, extra[0, extra_len), source,
 * destination, next_level_protocol); source / destination: 4 octets each;
 * extra may be NULL when extra_len is 0. */
int pnetgpu_util_ipv4_checksum(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t len, uint64_t skipword,
                               const uint8_t* extra, uint64_t extra_len, const uint8_t* source,
                               const uint8_t* destination, uint8_t next_level_protocol, uint16_t* out);

/* *out = util::ipv6_checksum(...); source / destination: 16 octets each. */
int pnetgpu_util_ipv6_checksum(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t len, uint64_t skipword,
                               const uint8_t* extra, uint64_t extra_len, const uint8_t* source,
                               const uint8_t* destination, uint8_t next_level_protocol, uint16_t* out);

/* out[i] = util::checksum(data[offsets[i], +lengths[i]), skipwords[i]) for i < n,
 * every array in host memory: the buffer and descriptors go over in one staged
 * copy each, one launch, the n words come back; synchronous. Every slice must
 * lie inside [0, data_bytes) (PNETGPU_EINVAL otherwise). */
int pnetgpu_checksum_slices_host(pnetgpu_ctx* ctx, const uint8_t* data, uint64_t data_bytes, uint64_t n,
                                 const uint64_t* offsets, const uint32_t* lengths, const uint32_t* skipwords,
                                 uint16_t* out);

#ifdef __cplusplus
}
#endif
#endif /* PNETGPU_UTIL_H */
