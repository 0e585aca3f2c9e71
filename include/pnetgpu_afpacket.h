/*
 * pnetgpu_afpacket.h — Linux AF_PACKET TPACKET_V3 receive ring as a batch
 * producer for pnetgpu_ring_submit_region: the kernel writes packets into a
 * memory-mapped block ring, each retired block is walked on the host (a few
 * header reads per packet, no copies) and its frames are shipped straight
 * from the mapping into HBM.
 *
 * Replaces, for batch consumers, the per-packet receive loop of
 * pnet_datalink's Linux channel (pnet_datalink/src/linux.rs:362-403: one
 * recvfrom into a 4096-B buffer per next(), buffer invalidated by the next
 * call; pnet_datalink/src/lib.rs:227-230 DataLinkReceiver::next). Frames are
 * the same Ethernet frames (captured bytes, tp_snaplen).
 *
 * Opening a packet socket needs CAP_NET_RAW; pnetgpu_afp_open returns
 * PNETGPU_ESYS with errno preserved when it is denied. Single-threaded use per
 * pnetgpu_afp (one consumer walks and releases the blocks in ring order);
 * distinct rings (e.g. one per PACKET_FANOUT member) are independent.
 */
#ifndef PNETGPU_AFPACKET_H
#define PNETGPU_AFPACKET_H

#include <stdint.h>

#include "pnetgpu.h"
#include "pnetgpu_ring.h"   /* PNETGPU_EEMPTY / EFULL / EFORMAT */

#ifdef __cplusplus
extern "C" {
#endif

#define PNETGPU_ESYS (-9)   /* an OS call failed; errno holds the reason */

typedef struct pnetgpu_afp pnetgpu_afp;

/* Open a TPACKET_V3 receive ring on interface `ifname` (NULL or "" = every
 * interface): n_blocks blocks of block_bytes (a power of two, >= 4096, a
 * multiple of the page size); the kernel retires a partly filled block after
 * retire_ms. PNETGPU_EINVAL for bad sizes or an unknown interface. */
int  pnetgpu_afp_open(const char* ifname, uint32_t block_bytes, uint32_t n_blocks, uint32_t retire_ms,
                      pnetgpu_afp** out);
void pnetgpu_afp_close(pnetgpu_afp* afp);
/* The ring mapping: block k starts at base + k * block_bytes. Register it
 * (pnetgpu_host_register(base, bytes)) for direct DMA. */
int  pnetgpu_afp_ring(pnetgpu_afp* afp, const uint8_t** base, uint64_t* bytes, uint32_t* block_bytes,
                      uint32_t* n_blocks);
/* Wait up to timeout_ms (-1 = forever) for the next retired block, in ring
 * order, and describe its packets: offsets relative to the ring base (for
 * pnetgpu_ring_submit_region(ring, base, ...)), lengths = captured bytes,
 * tp_status (may be NULL; TP_STATUS_CSUMNOTREADY marks packets whose L4
 * checksum the sending host left to offload). *block = the block's index.
 * PNETGPU_EEMPTY on timeout, PNETGPU_EFULL if the block holds more than cap
 * packets, PNETGPU_EFORMAT for an inconsistent block. */
int  pnetgpu_afp_next_block(pnetgpu_afp* afp, int timeout_ms, uint64_t* offsets, uint32_t* lengths,
                            uint32_t* tp_status, uint64_t cap, uint64_t* n, uint32_t* block);
/* Give a block back to the kernel once the batch holding its frames has been
 * waited (the ring slot no longer reads it). Blocks are released in order. */
int  pnetgpu_afp_release_block(pnetgpu_afp* afp, uint32_t block);
/* Join PACKET_FANOUT group `group_id` (the reference's Config::linux_fanout,
 * pnet_datalink/src/linux.rs:156-200 and lib.rs:110-128): rings opened on the
 * same interface with the same group share its traffic — one ring per GPU
 * rank. type: PNETGPU_FANOUT_*; flags: PNETGPU_FANOUT_FLAG_* (defrag, rollover). */
#define PNETGPU_FANOUT_HASH      0u
#define PNETGPU_FANOUT_LB        1u
#define PNETGPU_FANOUT_CPU       2u
#define PNETGPU_FANOUT_ROLLOVER  3u
#define PNETGPU_FANOUT_RND       4u
#define PNETGPU_FANOUT_QM        5u
#define PNETGPU_FANOUT_FLAG_ROLLOVER 0x1000u
#define PNETGPU_FANOUT_FLAG_DEFRAG   0x8000u
int  pnetgpu_afp_fanout(pnetgpu_afp* afp, uint16_t group_id, uint32_t type, uint32_t flags);
/* Promiscuous mode on the bound interface (the reference's Config::promiscuous). */
int  pnetgpu_afp_promiscuous(pnetgpu_afp* afp, int on);
/* Socket statistics (PACKET_STATISTICS: packets seen / dropped since the last call). */
int  pnetgpu_afp_stats(pnetgpu_afp* afp, uint64_t* packets, uint64_t* drops);

/* Walk one TPACKET_V3 block image of block_bytes (no socket needed):
 * descriptors of its packets, offsets relative to block_offset (the block's
 * own offset inside whatever buffer is shipped). Same errors as next_block. */
int  pnetgpu_tpacket3_walk(const uint8_t* block, uint64_t block_bytes, uint64_t block_offset, uint64_t* offsets,
                           uint32_t* lengths, uint32_t* tp_status, uint64_t cap, uint64_t* n);

#ifdef __cplusplus
}
#endif

#endif  // PNETGPU_AFPACKET_H
