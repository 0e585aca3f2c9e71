/*
 * util_checksum.c — pnet::util's checksum functions from plain C on host bytes
 * (include/pnetgpu_util.h): what a Rust or C call site of
 * `util::checksum(&data, skipword)` / `util::ipv4_checksum(..)` /
 * `util::ipv6_checksum(..)` (pnet_packet/src/util.rs:76-150) becomes, with no
 * device memory of its own. Prints the word as 0xHHHH.
 *
 *   util_checksum HEXDATA SKIPWORD
 *   util_checksum -4 HEXDATA SKIPWORD SRC_HEX(4 B) DST_HEX(4 B) PROTO [EXTRA_HEX]
 *   util_checksum -6 HEXDATA SKIPWORD SRC_HEX(16 B) DST_HEX(16 B) PROTO [EXTRA_HEX]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pnetgpu.h"
#include "pnetgpu_util.h"

static int unhex(const char* s, uint8_t* out, size_t cap, size_t* n) {
    const size_t len = strlen(s);
    if (len % 2 || len / 2 > cap) return -1;
    for (size_t i = 0; i < len / 2; ++i) {
        unsigned v;
        if (sscanf(s + 2 * i, "%2x", &v) != 1) return -1;
        out[i] = (uint8_t)v;
    }
    *n = len / 2;
    return 0;
}

int main(int argc, char** argv) {
    static uint8_t data[1 << 16], extra[1 << 12];
    uint8_t src[16], dst[16];
    size_t n = 0, ne = 0, ns = 0, nd = 0;
    int version = 0, a = 1;
    if (argc > 1 && (!strcmp(argv[1], "-4") || !strcmp(argv[1], "-6"))) {
        version = argv[1][1] - '0';
        a = 2;
    }
    const int need = version ? a + 5 : a + 2;
    if (argc < need || unhex(argv[a], data, sizeof data, &n)) {
        fprintf(stderr, "usage: util_checksum [-4|-6] HEXDATA SKIPWORD [SRC DST PROTO [EXTRA]]\n");
        return 2;
    }
    const unsigned long long skip = strtoull(argv[a + 1], NULL, 0);
    pnetgpu_ctx* ctx = NULL;
    int rc = pnetgpu_ctx_create(0, &ctx);
    if (rc) {
        fprintf(stderr, "pnetgpu_ctx_create: %s\n", pnetgpu_strerror(rc));
        return 1;
    }
    uint16_t out = 0;
    if (!version) {
        rc = pnetgpu_util_checksum(ctx, data, n, skip, &out);
    } else {
        const size_t alen = version == 4 ? 4 : 16;
        if (unhex(argv[a + 2], src, sizeof src, &ns) || unhex(argv[a + 3], dst, sizeof dst, &nd) || ns != alen ||
            nd != alen || (argc > a + 5 && unhex(argv[a + 5], extra, sizeof extra, &ne))) {
            fprintf(stderr, "bad address or extra data\n");
            pnetgpu_ctx_destroy(ctx);
            return 2;
        }
        const uint8_t proto = (uint8_t)strtoul(argv[a + 4], NULL, 0);
        rc = version == 4 ? pnetgpu_util_ipv4_checksum(ctx, data, n, skip, extra, ne, src, dst, proto, &out)
                          : pnetgpu_util_ipv6_checksum(ctx, data, n, skip, extra, ne, src, dst, proto, &out);
    }
    if (rc) {
        fprintf(stderr, "checksum: %s\n", pnetgpu_strerror(rc));
        pnetgpu_ctx_destroy(ctx);
        return 1;
    }
    printf("0x%04X\n", out);
    pnetgpu_ctx_destroy(ctx);
    return 0;
}
