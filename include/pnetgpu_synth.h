/*
 * pnetgpu_synth.h — seeded synthetic frame producer for the BASELINE.json
 * workloads (the in-memory stand-in for a NIC ring / pnet_datalink's
 * DataLinkReceiver, in the spirit of pnet_datalink/src/dummy.rs).
 *
 * Frames are built the way the reference builds them (benches/rs_sender.rs:25-101
 * for Eth/IPv4/UDP; pnet_packet setters for TCP/ICMP/IPv6) with random field
 * values from splitmix64(seed ^ frame index), so the bytes are identical for any
 * thread count. A fraction of frames get exactly one flipped byte, either in
 * the IPv4 header's id/flags/ttl bytes (IPv4 checksum mismatch only) or in the
 * L4 payload (L4 checksum mismatch only); the producer reports how many.
 */
#ifndef PNETGPU_SYNTH_H
#define PNETGPU_SYNTH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PNETGPU_SYNTH_RS_SENDER   0  /* config 1: the rs_sender 64-B frame, verbatim copies */
#define PNETGPU_SYNTH_UDP64       1  /* config 2: 64-B Eth/IPv4/UDP, random fields          */
#define PNETGPU_SYNTH_TCP1500     2  /* config 3: 1500-B Eth/IPv4/TCP                        */
#define PNETGPU_SYNTH_IMIX        3  /* config 4: 64/576/1500 B at 7:4:1, UDP/TCP/ICMP echo  */
#define PNETGPU_SYNTH_UDP6_JUMBO  4  /* config 5: 9000-B Eth/IPv6/UDP                         */
#define PNETGPU_SYNTH_UDP1500     5  /* north_star's 1500-B Eth/IPv4/UDP (1458 data bytes)    */

/* expect[] slots written by pnetgpu_synth_fill */
#define PNETGPU_SYNTH_EXP_IP_BAD  0
#define PNETGPU_SYNTH_EXP_L4_BAD  1
#define PNETGPU_SYNTH_EXP_BYTES   2
#define PNETGPU_SYNTH_NEXP        3

/* Bytes needed for n frames (tail-padded to 16 B) and the fixed stride (0 = descriptor mode). */
int pnetgpu_synth_layout(int workload, uint64_t n, uint64_t seed, uint64_t* total_bytes,
                         uint32_t* stride, uint32_t* frame_len);

/* Fill buf (>= total_bytes) and, in descriptor mode, offsets/lengths [n].
 * corrupt_ppm: corrupted frames per million. nthreads >= 1. */
int pnetgpu_synth_fill(int workload, uint64_t n, uint64_t seed, uint32_t corrupt_ppm,
                       uint8_t* buf, uint64_t buf_bytes, uint64_t* offsets, uint32_t* lengths,
                       uint64_t expect[PNETGPU_SYNTH_NEXP], int nthreads);

/* The same for frames [first, first + n) of a batch (frame i depends only on
 * seed and i): one shard of a global batch, byte-identical to those frames of
 * the whole batch. pnetgpu_synth_lengths writes the frame lengths of that range
 * without building anything (a byte-balanced split of IMIX, shard_by_bytes). */
int pnetgpu_synth_layout_range(int workload, uint64_t first, uint64_t n, uint64_t seed, uint64_t* total_bytes,
                               uint32_t* stride, uint32_t* frame_len);
int pnetgpu_synth_fill_range(int workload, uint64_t first, uint64_t n, uint64_t seed, uint32_t corrupt_ppm,
                             uint8_t* buf, uint64_t buf_bytes, uint64_t* offsets, uint32_t* lengths,
                             uint64_t expect[PNETGPU_SYNTH_NEXP], int nthreads);
int pnetgpu_synth_lengths(int workload, uint64_t first, uint64_t n, uint64_t seed, uint32_t* lengths);

#ifdef __cplusplus
}
#endif
#endif
