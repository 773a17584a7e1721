/* RFC 1321 MD5, plain C — TEST INFRASTRUCTURE ONLY (oracle/).
 *
 * Restates the message digest the reference obtains from OTP
 * `crypto:hash(md5, IoList)` (src/synctree.erl:252,258).  Pinned by the RFC 1321
 * appendix A.5 test suite in tests/test_oracle_c.py.  Independent of the HIP
 * device MD5 in riak_ensemble_amd/csrc so that each checks the other.
 */
#ifndef ORACLE_MD5_REF_H
#define ORACLE_MD5_REF_H
#include <stdint.h>
#include <string.h>

typedef struct {
    uint32_t s[4];
    uint64_t len;
    uint8_t buf[64];
    uint32_t fill;
} md5r_ctx;

static const uint32_t md5r_K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613, 0xfd469501,
    0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821,
    0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a,
    0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70,
    0x289b7ec6, 0xeaa127fa, 0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
    0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const uint8_t md5r_R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                                   5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                                   4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                                   6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static inline uint32_t md5r_rol(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

static void md5r_block(uint32_t s[4], const uint8_t *p) {
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
        m[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) | ((uint32_t)p[4 * i + 2] << 16) |
               ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = s[0], b = s[1], c = s[2], d = s[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        uint32_t t = d;
        d = c;
        c = b;
        b = b + md5r_rol(a + f + md5r_K[i] + m[g], md5r_R[i]);
        a = t;
    }
    s[0] += a; s[1] += b; s[2] += c; s[3] += d;
}

static inline void md5r_init(md5r_ctx *c) {
    c->s[0] = 0x67452301; c->s[1] = 0xefcdab89; c->s[2] = 0x98badcfe; c->s[3] = 0x10325476;
    c->len = 0; c->fill = 0;
}

static inline void md5r_update(md5r_ctx *c, const uint8_t *p, size_t n) {
    c->len += n;
    if (c->fill) {
        size_t take = 64 - c->fill;
        if (take > n) take = n;
        memcpy(c->buf + c->fill, p, take);
        c->fill += (uint32_t)take; p += take; n -= take;
        if (c->fill == 64) { md5r_block(c->s, c->buf); c->fill = 0; }
    }
    while (n >= 64) { md5r_block(c->s, p); p += 64; n -= 64; }
    if (n) { memcpy(c->buf, p, n); c->fill = (uint32_t)n; }
}

static inline void md5r_final(md5r_ctx *c, uint8_t out[16]) {
    /* RFC 1321 §3.1-3.2: 0x80, zeros to 56 mod 64, 64-bit little-endian bit length */
    uint64_t bits = c->len * 8;
    c->buf[c->fill++] = 0x80;
    if (c->fill > 56) {
        memset(c->buf + c->fill, 0, 64 - c->fill);
        md5r_block(c->s, c->buf);
        c->fill = 0;
    }
    memset(c->buf + c->fill, 0, 56 - c->fill);
    for (int i = 0; i < 8; i++) c->buf[56 + i] = (uint8_t)(bits >> (8 * i));
    md5r_block(c->s, c->buf);
    for (int i = 0; i < 4; i++) {
        out[4 * i] = (uint8_t)c->s[i]; out[4 * i + 1] = (uint8_t)(c->s[i] >> 8);
        out[4 * i + 2] = (uint8_t)(c->s[i] >> 16); out[4 * i + 3] = (uint8_t)(c->s[i] >> 24);
    }
}

static inline void md5r(const uint8_t *p, size_t n, uint8_t out[16]) {
    md5r_ctx c;
    md5r_init(&c);
    md5r_update(&c, p, n);
    md5r_final(&c, out);
}
#endif
