// afpacket.cpp — AF_PACKET TPACKET_V3 receive ring as a batch producer
// (include/pnetgpu_afpacket.h). The reference receives one frame per
// recvfrom() into a reused 4096-B buffer (pnet_datalink/src/linux.rs:362-403);
// here the kernel fills a mapped block ring, a retired block is walked for its
// packets' (offset, captured length) and those descriptors go to
// pnetgpu_ring_submit_region, which DMAs the frames from the mapping itself.
#include <errno.h>
#include <linux/if_ether.h>
#include <linux/if_packet.h>
#include <net/if.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>
#include <arpa/inet.h>

#include <cstdint>
#include <cstring>
#include <new>

#include "pnetgpu_afpacket.h"

struct pnetgpu_afp {
    int fd = -1;
    uint8_t* map = nullptr;
    uint64_t map_bytes = 0;
    uint32_t block_bytes = 0;
    uint32_t n_blocks = 0;
    uint32_t next = 0;       // next block to hand out (ring order)
    int ifindex = 0;         // bound interface (0 = all)
};

namespace {

// Block descriptor / packet header fields, read as plain loads at their
// <linux/if_packet.h> offsets (tpacket_block_desc, tpacket3_hdr).
template <class T>
T rd(const uint8_t* p) {
    T v;
    std::memcpy(&v, p, sizeof v);
    return v;
}

constexpr uint64_t kBlkStatus = offsetof(tpacket_block_desc, hdr) + offsetof(tpacket_hdr_v1, block_status);
constexpr uint64_t kBlkNum = offsetof(tpacket_block_desc, hdr) + offsetof(tpacket_hdr_v1, num_pkts);
constexpr uint64_t kBlkFirst = offsetof(tpacket_block_desc, hdr) + offsetof(tpacket_hdr_v1, offset_to_first_pkt);
constexpr uint64_t kBlkLen = offsetof(tpacket_block_desc, hdr) + offsetof(tpacket_hdr_v1, blk_len);

uint32_t block_status(const uint8_t* blk) {
    return __atomic_load_n(reinterpret_cast<const uint32_t*>(blk + kBlkStatus), __ATOMIC_ACQUIRE);
}

}  // namespace

extern "C" {

int pnetgpu_tpacket3_walk(const uint8_t* block, uint64_t block_bytes, uint64_t block_offset, uint64_t* offsets,
                          uint32_t* lengths, uint32_t* tp_status, uint64_t cap, uint64_t* n) {
    if (!block || !n || (cap && (!offsets || !lengths))) return PNETGPU_EINVAL;
    *n = 0;
    if (block_bytes < sizeof(tpacket_block_desc)) return PNETGPU_EFORMAT;
    const uint32_t num = rd<uint32_t>(block + kBlkNum);
    const uint64_t blk_len = rd<uint32_t>(block + kBlkLen);
    uint64_t p = rd<uint32_t>(block + kBlkFirst);
    if (blk_len > block_bytes) return PNETGPU_EFORMAT;
    if (num > cap) return PNETGPU_EFULL;
    for (uint32_t k = 0; k < num; ++k) {
        if (p + sizeof(tpacket3_hdr) > blk_len) return PNETGPU_EFORMAT;
        const uint8_t* h = block + p;
        const uint64_t mac = rd<uint16_t>(h + offsetof(tpacket3_hdr, tp_mac));
        const uint64_t snap = rd<uint32_t>(h + offsetof(tpacket3_hdr, tp_snaplen));
        if (p + mac + snap > blk_len) return PNETGPU_EFORMAT;
        offsets[k] = block_offset + p + mac;
        lengths[k] = (uint32_t)snap;
        if (tp_status) tp_status[k] = rd<uint32_t>(h + offsetof(tpacket3_hdr, tp_status));
        const uint32_t nx = rd<uint32_t>(h + offsetof(tpacket3_hdr, tp_next_offset));
        if (k + 1 < num) {
            if (nx == 0 || nx < mac + snap) return PNETGPU_EFORMAT;   // packets ascend, never overlap
            p += nx;
        }
    }
    *n = num;
    return PNETGPU_OK;
}

int pnetgpu_afp_open(const char* ifname, uint32_t block_bytes, uint32_t n_blocks, uint32_t retire_ms,
                     pnetgpu_afp** out) {
    if (!out) return PNETGPU_EINVAL;
    *out = nullptr;
    const long page = sysconf(_SC_PAGESIZE);
    if (block_bytes < 4096 || (block_bytes & (block_bytes - 1)) || block_bytes % (uint32_t)page || n_blocks == 0)
        return PNETGPU_EINVAL;
    unsigned ifindex = 0;
    if (ifname && *ifname && (ifindex = if_nametoindex(ifname)) == 0) return PNETGPU_EINVAL;
    const int fd = socket(AF_PACKET, SOCK_RAW, htons(ETH_P_ALL));
    if (fd < 0) return PNETGPU_ESYS;
    auto fail = [&](int rc) {
        const int e = errno;
        close(fd);
        errno = e;
        return rc;
    };
    int v = TPACKET_V3;
    if (setsockopt(fd, SOL_PACKET, PACKET_VERSION, &v, sizeof v) != 0) return fail(PNETGPU_ESYS);
    tpacket_req3 req{};
    req.tp_block_size = block_bytes;
    req.tp_block_nr = n_blocks;
    req.tp_frame_size = 2048;                                  // V3 packs packets; only sizes the count
    req.tp_frame_nr = (block_bytes / 2048) * n_blocks;
    req.tp_retire_blk_tov = retire_ms;
    if (setsockopt(fd, SOL_PACKET, PACKET_RX_RING, &req, sizeof req) != 0) return fail(PNETGPU_ESYS);
    const uint64_t bytes = (uint64_t)block_bytes * n_blocks;
    void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) return fail(PNETGPU_ESYS);
    sockaddr_ll sll{};
    sll.sll_family = AF_PACKET;
    sll.sll_protocol = htons(ETH_P_ALL);
    sll.sll_ifindex = (int)ifindex;
    if (bind(fd, reinterpret_cast<sockaddr*>(&sll), sizeof sll) != 0) {
        const int e = errno;
        munmap(m, bytes);
        close(fd);
        errno = e;
        return PNETGPU_ESYS;
    }
    auto* a = new (std::nothrow) pnetgpu_afp;
    if (!a) {
        munmap(m, bytes);
        close(fd);
        return PNETGPU_ENOMEM;
    }
    a->fd = fd;
    a->map = static_cast<uint8_t*>(m);
    a->map_bytes = bytes;
    a->block_bytes = block_bytes;
    a->n_blocks = n_blocks;
    a->ifindex = (int)ifindex;
    *out = a;
    return PNETGPU_OK;
}

void pnetgpu_afp_close(pnetgpu_afp* a) {
    if (!a) return;
    if (a->map) munmap(a->map, a->map_bytes);
    if (a->fd >= 0) close(a->fd);
    delete a;
}

int pnetgpu_afp_ring(pnetgpu_afp* a, const uint8_t** base, uint64_t* bytes, uint32_t* block_bytes,
                     uint32_t* n_blocks) {
    if (!a) return PNETGPU_EINVAL;
    if (base) *base = a->map;
    if (bytes) *bytes = a->map_bytes;
    if (block_bytes) *block_bytes = a->block_bytes;
    if (n_blocks) *n_blocks = a->n_blocks;
    return PNETGPU_OK;
}

int pnetgpu_afp_next_block(pnetgpu_afp* a, int timeout_ms, uint64_t* offsets, uint32_t* lengths,
                           uint32_t* tp_status, uint64_t cap, uint64_t* n, uint32_t* block) {
    if (!a || !n || !block) return PNETGPU_EINVAL;
    *n = 0;
    const uint8_t* blk = a->map + (uint64_t)a->next * a->block_bytes;
    if (!(block_status(blk) & TP_STATUS_USER)) {
        pollfd pfd{a->fd, POLLIN | POLLERR, 0};
        const int r = poll(&pfd, 1, timeout_ms);
        if (r < 0) return errno == EINTR ? PNETGPU_EEMPTY : PNETGPU_ESYS;
        if (!(block_status(blk) & TP_STATUS_USER)) return PNETGPU_EEMPTY;
    }
    const int rc = pnetgpu_tpacket3_walk(blk, a->block_bytes, (uint64_t)a->next * a->block_bytes, offsets, lengths,
                                         tp_status, cap, n);
    if (rc) return rc;
    *block = a->next;
    a->next = a->next + 1 == a->n_blocks ? 0 : a->next + 1;
    return PNETGPU_OK;
}

int pnetgpu_afp_release_block(pnetgpu_afp* a, uint32_t block) {
    if (!a || block >= a->n_blocks) return PNETGPU_EINVAL;
    uint8_t* blk = a->map + (uint64_t)block * a->block_bytes;
    __atomic_store_n(reinterpret_cast<uint32_t*>(blk + kBlkStatus), (uint32_t)TP_STATUS_KERNEL, __ATOMIC_RELEASE);
    return PNETGPU_OK;
}

int pnetgpu_afp_fanout(pnetgpu_afp* a, uint16_t group_id, uint32_t type, uint32_t flags) {
    if (!a || type > PNETGPU_FANOUT_QM || (flags & ~(PNETGPU_FANOUT_FLAG_ROLLOVER | PNETGPU_FANOUT_FLAG_DEFRAG)))
        return PNETGPU_EINVAL;
    const unsigned arg = (unsigned)group_id | ((type | flags) << 16);
    return setsockopt(a->fd, SOL_PACKET, PACKET_FANOUT, &arg, sizeof arg) == 0 ? PNETGPU_OK : PNETGPU_ESYS;
}

int pnetgpu_afp_promiscuous(pnetgpu_afp* a, int on) {
    if (!a || a->ifindex == 0) return PNETGPU_EINVAL;      // needs one bound interface
    packet_mreq mr{};
    mr.mr_ifindex = a->ifindex;
    mr.mr_type = PACKET_MR_PROMISC;
    const int opt = on ? PACKET_ADD_MEMBERSHIP : PACKET_DROP_MEMBERSHIP;
    return setsockopt(a->fd, SOL_PACKET, opt, &mr, sizeof mr) == 0 ? PNETGPU_OK : PNETGPU_ESYS;
}

int pnetgpu_afp_stats(pnetgpu_afp* a, uint64_t* packets, uint64_t* drops) {
    if (!a) return PNETGPU_EINVAL;
    tpacket_stats_v3 st{};
    socklen_t len = sizeof st;
    if (getsockopt(a->fd, SOL_PACKET, PACKET_STATISTICS, &st, &len) != 0) return PNETGPU_ESYS;
    if (packets) *packets = st.tp_packets;
    if (drops) *drops = st.tp_drops;
    return PNETGPU_OK;
}

}  // extern "C"
