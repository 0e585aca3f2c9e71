/*
 * rx_verify.c — the C-ABI from a plain C host program (no Python, no PyTorch):
 * what a libpnet application binds through FFI. Builds a
 * synthetic batch of 64-B Eth/IPv4/UDP frames with planted corruptions, then
 *   1. device-resident: hipMemcpy H2D -> pnetgpu_rx_process -> counters;
 *   2. zero-copy producer: the host buffer registered (pnetgpu_host_register)
 *      and shipped by pnetgpu_ring_submit_region through a 6-slot ring
 *      (pnetgpu_ring_create_ex), each batch released once its records are read;
 *   3. a descriptor batch of 1500-B UDP frames (compact u32/u16 descriptors)
 *      with the size hint pnetgpu_desc_size_hint gives for their lengths;
 * and checks that exactly the planted corruptions were flagged every way.
 * Build: make -C libpnet_amd examples    Run: libpnet_amd/build/rx_verify [n_frames]
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pnetgpu.h"
#include "pnetgpu_ring.h"
#include "pnetgpu_synth.h"

#define CHECK(call)                                                                    \
    do {                                                                               \
        int rc_ = (call);                                                              \
        if (rc_) {                                                                     \
            fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_,  \
                    pnetgpu_strerror(rc_));                                            \
            return 1;                                                                  \
        }                                                                              \
    } while (0)
#define HCHECK(call)                                                                   \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #call,            \
                    hipGetErrorString(e_));                                            \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], NULL, 10) : (1u << 20);
    if (pnetgpu_abi_version() != PNETGPU_ABI_VERSION) {
        fprintf(stderr, "ABI mismatch: library %d, header %d\n", pnetgpu_abi_version(), PNETGPU_ABI_VERSION);
        return 1;
    }
    uint64_t bytes = 0, expect[PNETGPU_SYNTH_NEXP];
    uint32_t stride = 0, flen = 0;
    CHECK(pnetgpu_synth_layout(PNETGPU_SYNTH_UDP64, n, 7, &bytes, &stride, &flen));
    uint8_t* host = (uint8_t*)malloc(bytes);
    if (!host) return 1;
    CHECK(pnetgpu_synth_fill(PNETGPU_SYNTH_UDP64, n, 7, 20000, host, bytes, NULL, NULL, expect, 8));

    pnetgpu_ctx* ctx = NULL;
    CHECK(pnetgpu_ctx_create(0, &ctx));

    /* 1. device-resident batch */
    uint8_t* d_frames = NULL;
    uint16_t* d_status = NULL;
    uint64_t* d_ctr = NULL;
    HCHECK(hipMalloc((void**)&d_frames, bytes));
    HCHECK(hipMalloc((void**)&d_status, 2 * n));
    HCHECK(hipMalloc((void**)&d_ctr, 8 * PNETGPU_NCOUNTERS));
    HCHECK(hipMemcpy(d_frames, host, bytes, hipMemcpyHostToDevice));
    HCHECK(hipMemset(d_ctr, 0, 8 * PNETGPU_NCOUNTERS));
    pnetgpu_batch b;
    memset(&b, 0, sizeof b);
    b.data = d_frames;
    b.data_bytes = bytes;
    b.n_frames = n;
    b.stride = stride;
    b.frame_len = flen;
    pnetgpu_rx_columns cols;
    memset(&cols, 0, sizeof cols);
    cols.status = d_status;
    cols.counters = d_ctr;
    CHECK(pnetgpu_rx_process(ctx, &b, &cols, NULL));
    uint64_t ctr[PNETGPU_NCOUNTERS];
    HCHECK(hipMemcpy(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost));
    printf("device batch: frames %llu ip_csum_bad %llu (planted %llu) l4_csum_bad %llu (planted %llu)\n",
           (unsigned long long)ctr[PNETGPU_CTR_FRAMES], (unsigned long long)ctr[PNETGPU_CTR_IP_CSUM_BAD],
           (unsigned long long)expect[PNETGPU_SYNTH_EXP_IP_BAD], (unsigned long long)ctr[PNETGPU_CTR_L4_CSUM_BAD],
           (unsigned long long)expect[PNETGPU_SYNTH_EXP_L4_BAD]);
    int ok = ctr[PNETGPU_CTR_FRAMES] == n && ctr[PNETGPU_CTR_IP_CSUM_BAD] == expect[PNETGPU_SYNTH_EXP_IP_BAD] &&
             ctr[PNETGPU_CTR_L4_CSUM_BAD] == expect[PNETGPU_SYNTH_EXP_L4_BAD];

    /* 2. zero-copy producer over the registered host buffer */
    uint64_t* offs = (uint64_t*)malloc(8 * n);
    uint32_t* lens = (uint32_t*)malloc(4 * n);
    if (!offs || !lens) return 1;
    for (uint64_t i = 0; i < n; ++i) {
        offs[i] = i * stride;
        lens[i] = flen;
    }
    CHECK(pnetgpu_host_register(host, bytes));
    pnetgpu_ring* ring = NULL;
    CHECK(pnetgpu_ring_create_ex(ctx, 16u << 20, 1u << 18, 0, 6, &ring));
    CHECK(pnetgpu_ring_set_columns(ring, 0x0FFFu));   /* the IPv4 record */
    uint64_t done = 0, seen = 0, ipbad = 0, l4bad = 0;
    for (;;) {
        if (done < n) {
            uint64_t taken = 0;
            int rc = pnetgpu_ring_submit_region(ring, host, offs + done, lens + done, n - done, &taken, NULL);
            if (rc == 0) {
                done += taken;
                continue;
            }
            if (rc != PNETGPU_EBUSY) CHECK(rc);
        }
        pnetgpu_ring_batch rb;
        int rc = pnetgpu_ring_wait(ring, &rb);
        if (rc == PNETGPU_EEMPTY) break;
        CHECK(rc);
        seen += rb.n_frames;
        ipbad += rb.cols.counters[PNETGPU_CTR_IP_CSUM_BAD];
        l4bad += rb.cols.counters[PNETGPU_CTR_L4_CSUM_BAD];
        CHECK(pnetgpu_ring_release(ring));   /* done with it: its slot refills now */
    }
    printf("zero-copy ring: frames %llu ip_csum_bad %llu l4_csum_bad %llu\n", (unsigned long long)seen,
           (unsigned long long)ipbad, (unsigned long long)l4bad);
    ok = ok && seen == n && ipbad == expect[PNETGPU_SYNTH_EXP_IP_BAD] && l4bad == expect[PNETGPU_SYNTH_EXP_L4_BAD];

    pnetgpu_ring_destroy(ring);
    CHECK(pnetgpu_host_unregister(host));

    /* 3. 1500-B UDP frames as a compact-descriptor batch with their size hint */
    const uint64_t m = n / 16 ? n / 16 : 1;
    uint64_t mbytes = 0, mexp[PNETGPU_SYNTH_NEXP];
    uint32_t mstride = 0, mlen = 0;
    CHECK(pnetgpu_synth_layout(PNETGPU_SYNTH_UDP1500, m, 8, &mbytes, &mstride, &mlen));
    uint8_t* mh = (uint8_t*)malloc(mbytes);
    uint32_t* moff = (uint32_t*)malloc(4 * m);
    uint16_t* mlen16 = (uint16_t*)malloc(2 * m);
    uint32_t* mlen32 = (uint32_t*)malloc(4 * m);
    if (!mh || !moff || !mlen16 || !mlen32) return 1;
    CHECK(pnetgpu_synth_fill(PNETGPU_SYNTH_UDP1500, m, 8, 20000, mh, mbytes, NULL, NULL, mexp, 8));
    for (uint64_t i = 0; i < m; ++i) {
        moff[i] = (uint32_t)(i * mstride);
        mlen16[i] = (uint16_t)mlen;
        mlen32[i] = mlen;
    }
    const uint32_t hint = pnetgpu_desc_size_hint(mlen32, m);
    uint8_t* dm = NULL;
    void *dmo = NULL, *dml = NULL;
    HCHECK(hipMalloc((void**)&dm, mbytes));
    HCHECK(hipMalloc(&dmo, 4 * m));
    HCHECK(hipMalloc(&dml, 2 * m));
    HCHECK(hipMemcpy(dm, mh, mbytes, hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(dmo, moff, 4 * m, hipMemcpyHostToDevice));
    HCHECK(hipMemcpy(dml, mlen16, 2 * m, hipMemcpyHostToDevice));
    HCHECK(hipMemset(d_ctr, 0, 8 * PNETGPU_NCOUNTERS));
    memset(&b, 0, sizeof b);
    b.data = dm;
    b.data_bytes = mbytes;
    b.n_frames = m;
    b.offsets = (const uint64_t*)dmo;   /* PNETGPU_DESC_COMPACT: u32 offsets, u16 lengths */
    b.lengths = (const uint32_t*)dml;
    b.flags = PNETGPU_DESC_COMPACT | hint;
    CHECK(pnetgpu_rx_process(ctx, &b, &cols, NULL));
    HCHECK(hipMemcpy(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost));
    printf("1500-B descriptor batch (hint 0x%x, %s): frames %llu ip_csum_bad %llu (planted %llu) l4_csum_bad %llu "
           "(planted %llu)\n", hint, pnetgpu_last_rx_kernel(), (unsigned long long)ctr[PNETGPU_CTR_FRAMES],
           (unsigned long long)ctr[PNETGPU_CTR_IP_CSUM_BAD], (unsigned long long)mexp[PNETGPU_SYNTH_EXP_IP_BAD],
           (unsigned long long)ctr[PNETGPU_CTR_L4_CSUM_BAD], (unsigned long long)mexp[PNETGPU_SYNTH_EXP_L4_BAD]);
    ok = ok && hint == PNETGPU_DESC_HINT_LARGE && ctr[PNETGPU_CTR_FRAMES] == m &&
         ctr[PNETGPU_CTR_IP_CSUM_BAD] == mexp[PNETGPU_SYNTH_EXP_IP_BAD] &&
         ctr[PNETGPU_CTR_L4_CSUM_BAD] == mexp[PNETGPU_SYNTH_EXP_L4_BAD];
    uint64_t st[PNETGPU_NSCHED_STATS];
    CHECK(pnetgpu_ctx_sched_stats(ctx, st));
    printf("run scheduling: %llu launches claimed, %llu static (busy), %llu static (captured), pool %llu\n",
           (unsigned long long)st[PNETGPU_SCHED_CLAIMED], (unsigned long long)st[PNETGPU_SCHED_STATIC_BUSY],
           (unsigned long long)st[PNETGPU_SCHED_STATIC_CAPTURED], (unsigned long long)st[PNETGPU_SCHED_BLOCKS]);
    (void)hipFree(dm);
    (void)hipFree(dmo);
    (void)hipFree(dml);
    free(mh);
    free(moff);
    free(mlen16);
    free(mlen32);
    pnetgpu_ctx_destroy(ctx);
    (void)hipFree(d_frames);
    (void)hipFree(d_status);
    (void)hipFree(d_ctr);
    free(offs);
    free(lens);
    free(host);
    printf("%s\n", ok ? "OK" : "MISMATCH");
    return ok ? 0 : 1;
}
