/*
 * rs_sender.c — the build+checksum half of libpnet's benches/rs_sender.rs on
 * the GPU, as a plain C program against the C-ABI.
 *
 * rs_sender.rs builds one 64-B Ethernet/IPv4/UDP frame ("rmesg", 127.0.0.1 ->
 * 127.0.0.1, ports 1234, ttl 4) and computes its checksums with
 * ipv4::checksum and udp::ipv4_checksum before every send (rs_sender.rs:25-72).
 * Here a batch of n such frames — frame 0 exactly rs_sender's, the others
 * with their own IPv4 identification and UDP source port so every checksum
 * differs — is built with zero checksum fields, filled on the GPU by
 * pnetgpu_tx_fill_checksums, verified by pnetgpu_rx_process (the receive
 * kernels recompute and compare every field the TX kernels wrote), and
 * optionally written to a pcap file (what would go to the wire).
 * Frame 0's fields must come out as 0xB8CA (IPv4) and 0xB94C (UDP).
 *
 * usage: rs_sender [n_frames] [out.pcap]
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pnetgpu.h"

#define CHECK(call)                                                                          \
    do {                                                                                     \
        int rc_ = (call);                                                                    \
        if (rc_) {                                                                           \
            fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_,        \
                    pnetgpu_strerror(rc_));                                                  \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)
#define HCHECK(call)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess) {                                                              \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

enum { kFrame = 64 };

/* rs_sender.rs's frame with both checksum fields zero; i varies ip id and udp sport */
static void build_frame(uint8_t* f, uint64_t i) {
    static const uint8_t dst[6] = {0x02, 0x00, 0x00, 0x00, 0x00, 0x01};
    static const uint8_t src[6] = {0x02, 0x00, 0x00, 0x00, 0x00, 0x02};
    memset(f, 0, kFrame);
    memcpy(f, dst, 6);
    memcpy(f + 6, src, 6);
    f[12] = 0x08;                                      /* EtherTypes::Ipv4 */
    uint8_t* ip = f + 14;
    ip[0] = 0x45;                                      /* version 4, IHL 5 */
    ip[3] = 20 + 8 + 5;                                /* total_length 33 */
    ip[4] = (uint8_t)(i >> 8), ip[5] = (uint8_t)i;     /* identification (0 for frame 0) */
    ip[8] = 4;                                         /* ttl */
    ip[9] = 17;                                        /* IpNextHeaderProtocols::Udp */
    ip[12] = 127, ip[15] = 1;                          /* 127.0.0.1 */
    ip[16] = 127, ip[19] = 1;                          /* 127.0.0.1 */
    uint8_t* udp = ip + 20;
    const unsigned sport = 1234 + (unsigned)(i % 50000);
    udp[0] = (uint8_t)(sport >> 8), udp[1] = (uint8_t)sport;
    udp[2] = 0x04, udp[3] = 0xD2;                      /* 1234 */
    udp[5] = 8 + 5;                                    /* length 13 */
    memcpy(udp + 8, "rmesg", 5);
}

static int write_pcap(const char* path, const uint8_t* frames, uint64_t n) {
    FILE* fp = fopen(path, "wb");
    if (!fp) return 1;
    const uint32_t gh[6] = {0xa1b2c3d4u, 0x00040002u, 0, 0, 65535, 1};   /* LINKTYPE_ETHERNET */
    fwrite(gh, 4, 6, fp);
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t rh[4] = {1700000000u, (uint32_t)(i % 1000000), kFrame, kFrame};
        fwrite(rh, 4, 4, fp);
        fwrite(frames + i * kFrame, 1, kFrame, fp);
    }
    return fclose(fp) != 0;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], NULL, 10) : 1000000;
    const char* out = argc > 2 ? argv[2] : NULL;
    if (n == 0) return 2;
    uint8_t* host = (uint8_t*)malloc(n * kFrame);
    if (!host) return 1;
    for (uint64_t i = 0; i < n; ++i) build_frame(host + i * kFrame, i);

    pnetgpu_ctx* ctx = NULL;
    CHECK(pnetgpu_ctx_create(0, &ctx));
    uint8_t* d_frames = NULL;
    uint16_t* d_status = NULL;
    uint64_t* d_ctr = NULL;
    HCHECK(hipMalloc((void**)&d_frames, n * kFrame + 64));
    HCHECK(hipMalloc((void**)&d_status, 2 * n));
    HCHECK(hipMalloc((void**)&d_ctr, 8 * PNETGPU_NCOUNTERS));
    HCHECK(hipMemcpy(d_frames, host, n * kFrame, hipMemcpyHostToDevice));

    pnetgpu_batch b;
    memset(&b, 0, sizeof b);
    b.data = d_frames;
    b.data_bytes = n * kFrame;
    b.n_frames = n;
    b.stride = kFrame;
    b.frame_len = kFrame;
    pnetgpu_rx_columns tx;
    memset(&tx, 0, sizeof tx);
    tx.status = d_status;

    /* checksum fill: once to load the kernel, then timed (filling is idempotent) */
    CHECK(pnetgpu_tx_fill_checksums(ctx, &b, &tx, NULL));
    hipEvent_t e0, e1;
    HCHECK(hipEventCreate(&e0));
    HCHECK(hipEventCreate(&e1));
    HCHECK(hipEventRecord(e0, NULL));
    CHECK(pnetgpu_tx_fill_checksums(ctx, &b, &tx, NULL));
    HCHECK(hipEventRecord(e1, NULL));
    HCHECK(hipEventSynchronize(e1));
    float ms = 0;
    HCHECK(hipEventElapsedTime(&ms, e0, e1));

    /* verify: the receive path recomputes every field the fill wrote */
    pnetgpu_rx_columns rx;
    memset(&rx, 0, sizeof rx);
    rx.status = d_status;
    rx.counters = d_ctr;
    HCHECK(hipMemset(d_ctr, 0, 8 * PNETGPU_NCOUNTERS));
    CHECK(pnetgpu_rx_process(ctx, &b, &rx, NULL));
    uint64_t ctr[PNETGPU_NCOUNTERS];
    HCHECK(hipMemcpy(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost));
    HCHECK(hipMemcpy(host, d_frames, n * kFrame, hipMemcpyDeviceToHost));

    const unsigned ipc = ((unsigned)host[24] << 8) | host[25], udpc = ((unsigned)host[40] << 8) | host[41];
    printf("filled %llu frames in %.3f ms (%.1f Mpkts/s); frame 0: ipv4 checksum 0x%04X, udp checksum 0x%04X\n",
           (unsigned long long)n, ms, n / (ms * 1e3), ipc, udpc);
    printf("verify: frames %llu ipv4 %llu ip_csum_bad %llu l4_csum_bad %llu malformed %llu\n",
           (unsigned long long)ctr[PNETGPU_CTR_FRAMES], (unsigned long long)ctr[PNETGPU_CTR_IPV4],
           (unsigned long long)ctr[PNETGPU_CTR_IP_CSUM_BAD], (unsigned long long)ctr[PNETGPU_CTR_L4_CSUM_BAD],
           (unsigned long long)ctr[PNETGPU_CTR_MALFORMED]);
    int ok = ipc == 0xB8CA && udpc == 0xB94C && ctr[PNETGPU_CTR_FRAMES] == n && ctr[PNETGPU_CTR_IPV4] == n &&
             ctr[PNETGPU_CTR_IP_CSUM_BAD] == 0 && ctr[PNETGPU_CTR_L4_CSUM_BAD] == 0 && ctr[PNETGPU_CTR_MALFORMED] == 0;
    if (out && write_pcap(out, host, n)) {
        fprintf(stderr, "rs_sender: cannot write %s\n", out);
        ok = 0;
    }
    pnetgpu_ctx_destroy(ctx);
    (void)hipFree(d_frames);
    (void)hipFree(d_status);
    (void)hipFree(d_ctr);
    free(host);
    printf("%s\n", ok ? "OK" : "MISMATCH");
    return ok ? 0 : 1;
}
