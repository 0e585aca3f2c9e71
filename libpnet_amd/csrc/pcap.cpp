// pcap.cpp — capture-file readers for the batch producer (include/pnetgpu_ring.h):
// pnet_datalink's pcap backend (pnet_datalink/src/pcap.rs:92-105 from_file,
// :168-179 next) goes through libpcap's offline reader, which takes both the
// classic pcap format and pcapng. Both are read here without dependencies:
// a streaming reader (one record per call, like DataLinkReceiver::next) and an
// in-memory indexer that turns a file image into (offset, length) descriptors
// for zero-copy submits. Host code only; no frame byte is interpreted.
//
// pcapng (the block format): a file is a sequence of sections, each opened by
// a Section Header Block (type 0x0A0D0D0A) whose byte-order magic 0x1A2B3C4D
// fixes the section's byte order; Interface Description Blocks (type 1) give
// each interface's link type and snap length; packets come in Enhanced Packet
// Blocks (6: interface id, timestamp, captured and original length, data),
// Simple Packet Blocks (3: original length, data up to interface 0's snap
// length) or the obsolete Packet Block (2). Every block is
// [type u32][total length u32][body][total length u32], 4-B aligned; other
// block types (name resolution, statistics, custom, ...) are skipped. Like
// libpcap, every interface of a file must have the first interface's link type.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "pnetgpu.h"
#include "pnetgpu_ring.h"

namespace {

constexpr uint32_t kShb = 0x0A0D0D0Au;   // also the first 4 bytes of a pcapng file
constexpr uint32_t kIdb = 1, kPb = 2, kSpb = 3, kEpb = 6;
constexpr uint32_t kBom = 0x1A2B3C4Du;
constexpr uint32_t kMaxRecord = 1u << 26;   // a captured length above this is a corrupt file

uint32_t rd32(const uint8_t* p, bool swap) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}
uint16_t rd16(const uint8_t* p, bool swap) {
    uint16_t v;
    std::memcpy(&v, p, 2);
    return swap ? __builtin_bswap16(v) : v;
}

bool is_pcapng(const uint8_t* head) { return rd32(head, false) == kShb; }

// Link types a batch can be parsed from, and the receive flags they need.
int linktype_flags(uint32_t lt, uint32_t* flags) {
    if (lt == 1u) *flags = 0;
    else if (lt == 101u || lt == 228u || lt == 229u) *flags = PNETGPU_RX_L3;
    else return PNETGPU_EFORMAT;
    return PNETGPU_OK;
}

// The section and interface state of a pcapng reader.
struct NgState {
    bool swap = false;
    bool have_linktype = false;
    uint32_t linktype = 0;          // of the file's first interface (all must match)
    std::vector<uint32_t> snaplen;  // per interface of the current section (0: unlimited)
};

// One pcapng block of `body_len` body bytes (type already read). Updates the
// state for SHB / IDB; for a packet block sets *data / *caplen (data = nullptr
// for any other block). Returns PNETGPU_OK or PNETGPU_EFORMAT.
int ng_block(NgState& st, uint32_t type, const uint8_t* body, uint32_t body_len, const uint8_t** data,
             uint32_t* caplen) {
    *data = nullptr;
    *caplen = 0;
    if (type == kShb) {
        if (body_len < 16) return PNETGPU_EFORMAT;
        const uint32_t bom = rd32(body, false);
        if (bom == kBom) st.swap = false;
        else if (bom == __builtin_bswap32(kBom)) st.swap = true;
        else return PNETGPU_EFORMAT;
        if (rd16(body + 4, st.swap) != 1u) return PNETGPU_EFORMAT;   // major version 1
        st.snaplen.clear();                                          // a new section: new interfaces
        return PNETGPU_OK;
    }
    if (type == kIdb) {
        if (body_len < 8) return PNETGPU_EFORMAT;
        const uint32_t lt = rd16(body, st.swap);
        if (!st.have_linktype) {
            st.have_linktype = true;
            st.linktype = lt;
        } else if (lt != st.linktype) {
            return PNETGPU_EFORMAT;     // libpcap: every interface must share the first's link type
        }
        st.snaplen.push_back(rd32(body + 4, st.swap));
        return PNETGPU_OK;
    }
    if (type == kEpb || type == kPb) {
        if (body_len < 20) return PNETGPU_EFORMAT;
        const uint32_t ifid = type == kEpb ? rd32(body, st.swap) : rd16(body, st.swap);
        const uint32_t cap = rd32(body + 12, st.swap);
        if (ifid >= st.snaplen.size() || cap > kMaxRecord || cap > body_len - 20) return PNETGPU_EFORMAT;
        *data = body + 20;
        *caplen = cap;
        return PNETGPU_OK;
    }
    if (type == kSpb) {
        if (body_len < 4 || st.snaplen.empty()) return PNETGPU_EFORMAT;
        uint32_t cap = rd32(body, st.swap);                          // the original length
        if (st.snaplen[0] && cap > st.snaplen[0]) cap = st.snaplen[0];
        if (cap > kMaxRecord || cap > body_len - 4) return PNETGPU_EFORMAT;
        *data = body + 4;
        *caplen = cap;
        return PNETGPU_OK;
    }
    return PNETGPU_OK;   // any other block: skipped
}

// Walks the blocks of an in-memory pcapng image from byte 0: calls
// fn(data_offset, caplen) for every packet at or after byte `from` (at most
// `cap` of them: returns when that many were taken), stops at `from` with
// want_info (the first IDB's link type). *next = where the walk stopped (a
// block boundary, or img_bytes).
template <class F>
int ng_walk(const uint8_t* img, uint64_t img_bytes, uint64_t from, uint64_t cap, bool want_info, NgState& st,
            uint64_t* next, F fn, uint64_t start = 0) {
    uint64_t p = start, taken = 0;
    while (p < img_bytes) {
        if (img_bytes - p < 12) return PNETGPU_EFORMAT;              // truncated block header
        const uint32_t type = rd32(img + p, st.swap);
        // the SHB's length is read in the byte order its own magic gives
        bool swap = st.swap;
        if (rd32(img + p, false) == kShb) {
            const uint32_t bom = rd32(img + p + 8, false);
            if (bom == kBom) swap = false;
            else if (bom == __builtin_bswap32(kBom)) swap = true;
            else return PNETGPU_EFORMAT;
        }
        const uint32_t len = rd32(img + p + 4, swap);
        if (len < 12 || len % 4 || len > img_bytes - p || rd32(img + p + len - 4, swap) != len)
            return PNETGPU_EFORMAT;
        const uint32_t t = rd32(img + p, false) == kShb ? kShb : type;
        const uint8_t* data;
        uint32_t caplen;
        if (const int rc = ng_block(st, t, img + p + 8, len - 12, &data, &caplen)) return rc;
        if (want_info && st.have_linktype) {
            *next = p;
            return PNETGPU_OK;
        }
        if (data && p >= from) {
            if (taken == cap) {
                *next = p;
                return PNETGPU_OK;
            }
            fn((uint64_t)(data - img), caplen);
            ++taken;
        }
        p += len;
    }
    *next = img_bytes;
    return want_info && !st.have_linktype ? PNETGPU_EFORMAT : PNETGPU_OK;
}

// The state a pcapng scan stopped with, so that the next call of a scan in
// batches (*pos = where the previous call stopped, same image) resumes there
// instead of walking the block headers from byte 0 again (which made a scan of
// n packets in batches of k cost n^2 / k block reads). Per thread: a scan's
// calls come from one thread; any other call walks from byte 0 as before.
// A resumed call must be the same image, not another one of the same size that
// the allocator placed at the same address: the image's first 28 bytes (its
// SHB header) and the 12 bytes of the block at pos are matched too.
struct NgResume {
    const uint8_t* img = nullptr;
    uint64_t img_bytes = 0, pos = 0;
    uint8_t head[28] = {}, at[12] = {};
    NgState st;
    static size_t head_len(uint64_t img_bytes) { return (size_t)std::min<uint64_t>(28, img_bytes); }
    static size_t at_len(uint64_t img_bytes, uint64_t pos) {
        return pos < img_bytes ? (size_t)std::min<uint64_t>(12, img_bytes - pos) : 0;
    }
    bool matches(const uint8_t* i, uint64_t n, uint64_t p) const {
        return p && img == i && img_bytes == n && pos == p && std::memcmp(head, i, head_len(n)) == 0 &&
               std::memcmp(at, i + p, at_len(n, p)) == 0;
    }
    void keep(const uint8_t* i, uint64_t n, uint64_t p, const NgState& s) {
        img = i;
        img_bytes = n;
        pos = p;
        st = s;
        std::memcpy(head, i, head_len(n));
        std::memcpy(at, i + p, at_len(n, p));
    }
};
thread_local NgResume g_resume;

// Classic pcap global header of an in-memory image: byte order and link type.
int classic_header(const uint8_t* img, uint64_t img_bytes, bool* swap, uint32_t* linktype) {
    if (img_bytes < 24) return PNETGPU_EFORMAT;
    uint32_t magic;
    std::memcpy(&magic, img, 4);
    if (magic == 0xa1b2c3d4u || magic == 0xa1b23c4du) *swap = false;
    else if (magic == 0xd4c3b2a1u || magic == 0x4d3cb2a1u) *swap = true;
    else return PNETGPU_EFORMAT;
    *linktype = rd32(img + 20, *swap);
    return PNETGPU_OK;
}

}  // namespace

struct pnetgpu_pcap {
    FILE* f = nullptr;
    bool ng = false;
    bool swap = false;          // classic: the file's byte order
    NgState st;                 // pcapng: section / interface state
    std::vector<uint8_t> buf;   // the current record (classic) or block (pcapng)
};

extern "C" {

int pnetgpu_pcap_open(const char* path, pnetgpu_pcap** out) {
    if (!path || !out) return PNETGPU_EINVAL;
    *out = nullptr;
    FILE* f = std::fopen(path, "rb");
    if (!f) return PNETGPU_EINVAL;
    auto* p = new (std::nothrow) pnetgpu_pcap;
    if (!p) {
        std::fclose(f);
        return PNETGPU_ENOMEM;
    }
    p->f = f;
    uint8_t gh[24];
    int rc = PNETGPU_OK;
    if (std::fread(gh, 1, 4, f) != 4) {
        rc = PNETGPU_EFORMAT;
    } else if (is_pcapng(gh)) {
        p->ng = true;                    // blocks are read by next(); it starts at the SHB
        std::rewind(f);
    } else if (std::fread(gh + 4, 1, 20, f) != 20) {
        rc = PNETGPU_EFORMAT;
    } else {
        uint32_t lt = 0;
        rc = classic_header(gh, 24, &p->swap, &lt);
        if (!rc && lt != 1u) rc = PNETGPU_EFORMAT;   // LINKTYPE_ETHERNET
    }
    if (rc) {
        pnetgpu_pcap_close(p);
        return rc;
    }
    *out = p;
    return PNETGPU_OK;
}

int pnetgpu_pcap_next(pnetgpu_pcap* p, const uint8_t** frame, uint32_t* len) {
    if (!p || !frame || !len) return PNETGPU_EINVAL;
    if (!p->ng) {
        uint8_t rh[16];
        const size_t got = std::fread(rh, 1, 16, p->f);
        if (got == 0) return PNETGPU_EEMPTY;
        if (got != 16) return PNETGPU_EFORMAT;
        const uint32_t incl = rd32(rh + 8, p->swap);
        if (incl > kMaxRecord) return PNETGPU_EFORMAT;
        p->buf.resize(incl ? incl : 1);
        if (incl && std::fread(p->buf.data(), 1, incl, p->f) != incl) return PNETGPU_EFORMAT;
        *frame = p->buf.data();
        *len = incl;
        return PNETGPU_OK;
    }
    for (;;) {                                     // pcapng: blocks until the next packet
        uint8_t bh[12];
        const size_t got = std::fread(bh, 1, 12, p->f);
        if (got == 0) return PNETGPU_EEMPTY;
        if (got != 12) return PNETGPU_EFORMAT;
        uint32_t type = rd32(bh, p->st.swap);
        bool swap = p->st.swap;
        if (rd32(bh, false) == kShb) {
            type = kShb;
            const uint32_t bom = rd32(bh + 8, false);
            if (bom == kBom) swap = false;
            else if (bom == __builtin_bswap32(kBom)) swap = true;
            else return PNETGPU_EFORMAT;
        }
        const uint32_t blen = rd32(bh + 4, swap);
        if (blen < 12 || blen % 4 || blen > kMaxRecord + 64) return PNETGPU_EFORMAT;
        p->buf.resize(blen);
        std::memcpy(p->buf.data(), bh, 12);
        if (std::fread(p->buf.data() + 12, 1, blen - 12, p->f) != blen - 12) return PNETGPU_EFORMAT;
        if (rd32(p->buf.data() + blen - 4, swap) != blen) return PNETGPU_EFORMAT;
        const uint8_t* data;
        uint32_t caplen;
        if (const int rc = ng_block(p->st, type, p->buf.data() + 8, blen - 12, &data, &caplen)) return rc;
        if (type == kIdb && p->st.linktype != 1u) return PNETGPU_EFORMAT;   // the reader is Ethernet-only
        if (data) {
            *frame = data;
            *len = caplen;
            return PNETGPU_OK;
        }
    }
}

int pnetgpu_pcap_info(const uint8_t* img, uint64_t img_bytes, uint32_t* linktype, uint32_t* rx_flags) {
    if (!img || !linktype || !rx_flags) return PNETGPU_EINVAL;
    uint32_t lt = 0;
    if (img_bytes >= 4 && is_pcapng(img)) {
        NgState st;
        uint64_t next = 0;
        const int rc = ng_walk(img, img_bytes, 0, 0, true, st, &next, [](uint64_t, uint32_t) {});
        if (rc) return rc;
        lt = st.linktype;
    } else {
        bool swap;
        if (const int rc = classic_header(img, img_bytes, &swap, &lt)) return rc;
    }
    if (const int rc = linktype_flags(lt, rx_flags)) return rc;
    *linktype = lt;
    return PNETGPU_OK;
}

int pnetgpu_pcap_scan(const uint8_t* img, uint64_t img_bytes, uint64_t* pos, uint64_t* offsets, uint32_t* lengths,
                      uint64_t cap, uint64_t* n) {
    if (!img || !pos || !n || (cap && (!offsets || !lengths))) return PNETGPU_EINVAL;
    *n = 0;
    uint32_t flags;
    if (img_bytes >= 4 && is_pcapng(img)) {
        // the section / interface state at *pos comes from the blocks before it:
        // the walk starts at byte 0 and takes packets from *pos on (block
        // headers only until then)
        NgState st;
        uint64_t start = 0;
        if (g_resume.matches(img, img_bytes, *pos)) {
            st = g_resume.st;     // *pos is a block boundary this thread's last scan of the image stopped at
            start = *pos;
        }
        uint64_t k = 0, next = 0;
        const int rc = ng_walk(img, img_bytes, *pos, cap, false, st, &next, [&](uint64_t off, uint32_t len) {
            offsets[k] = off;
            lengths[k] = len;
            ++k;
        }, start);
        g_resume.img = nullptr;
        if (rc) return rc;
        if (k && linktype_flags(st.linktype, &flags)) return PNETGPU_EFORMAT;
        g_resume.keep(img, img_bytes, next, st);
        *n = k;
        *pos = next;
        return PNETGPU_OK;
    }
    bool swap;
    uint32_t linktype;
    if (const int rc = classic_header(img, img_bytes, &swap, &linktype)) return rc;
    if (const int rc = linktype_flags(linktype, &flags)) return rc;
    uint64_t p = *pos < 24 ? 24 : *pos;
    uint64_t k = 0;
    while (k < cap && p < img_bytes) {
        if (img_bytes - p < 16) return PNETGPU_EFORMAT;      // truncated record header
        const uint32_t incl = rd32(img + p + 8, swap);
        if (incl > kMaxRecord || incl > img_bytes - p - 16) return PNETGPU_EFORMAT;
        offsets[k] = p + 16;
        lengths[k] = incl;
        p += 16ull + incl;
        ++k;
    }
    *n = k;
    *pos = p;
    return PNETGPU_OK;
}

void pnetgpu_pcap_close(pnetgpu_pcap* p) {
    if (!p) return;
    if (p->f) std::fclose(p->f);
    delete p;
}

}  // extern "C"
