// leveldb_fmt.h — device encoder of the synctree_leveldb on-disk format
// (SURVEY.md §8f rank 2).
//
// synctree_leveldb stores every node {Level, Bucket} of a tree as one LevelDB
// record (src/synctree_leveldb.erl:104-109, 134-152):
//   key   = <<0:8, TreeId/binary, Level:8, (binary:encode_unsigned(Bucket))/binary>>
//   value = term_to_binary(Node)
// with Node = TopHash (a 17-byte binary) at {0,0}, [{ChildId, Hash17}] for an
// inner node (levels 1..H), [{Key, Value}] for a segment (level H+1).
//
// term_to_binary (ERTS external term format, version 131, uncompressed) on
// that domain:
//   binary            109, Len:32, Bytes
//   list              108, Count:32, Elements..., 106 (NIL); [] is 106 alone
//   2-tuple           104, 2, A, B
//   integer 0..255    97, B
//   integer int32     98, V:32/signed
//   other integers    110, N, Sign, N little-endian magnitude bytes
//   atom              119, Len:8, Utf8 (Len < 256) | 118, Len:16, Utf8
// (atoms: the UTF-8 forms term_to_binary emits from OTP 26; binary_to_term of
// every OTP since R16 reads them.  The decoder on the restore side also reads
// the Latin-1 ATOM_EXT / SMALL_ATOM_EXT forms older releases wrote.)
//
// One record index space r in [0, nslots) matching the slot layout
// (DevTree.base): r = 0 is {0,0} (value: the stored top hash, slot 1);
// r in [base[L], base[L+1]) for L in 1..H is inner node (L, r - base[L])
// whose content is the W slots at base[L+1] + Bucket*W; r in
// [base[H+1], nslots) is segment r - base[H+1] (CSR content).  Records come
// out in that (Level, Bucket) order; a LevelDB write batch of distinct keys
// does not depend on it.
//
// All kernels are HBM-bound byte formatting (no MD5):
//   k_snap_entry_sizes  one lane per segment entry: its ETF length
//   k_snap_sizes        one lane per record: present flag, key and value length
//   k_snap_write        one lane per record: key, list header / NIL, inner
//                       nodes' children, the {0,0} hash
//   k_snap_entries      one lane per segment entry: {Key, Value} bytes
// (three rocPRIM scans between them give the offsets).  Node content is read
// once and every output byte written once.
#pragma once
#include "st_kernels.h"

__host__ __device__ inline uint32_t etf_int_size(int64_t v) {
    if (v >= 0 && v < 256) return 2;
    if (v >= -2147483648LL && v <= 2147483647LL) return 5;
    uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    uint32_t n = 0;
    while (m) { n++; m >>= 8; }
    return 3 + n;
}

__device__ inline uint8_t *etf_int_write(uint8_t *p, int64_t v) {
    if (v >= 0 && v < 256) {
        p[0] = 97; p[1] = (uint8_t)v;
        return p + 2;
    }
    if (v >= -2147483648LL && v <= 2147483647LL) {
        const uint32_t u = (uint32_t)(int32_t)v;
        p[0] = 98; p[1] = (uint8_t)(u >> 24); p[2] = (uint8_t)(u >> 16); p[3] = (uint8_t)(u >> 8); p[4] = (uint8_t)u;
        return p + 5;
    }
    uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    uint32_t n = 0;
    p[0] = 110; p[2] = v < 0 ? 1 : 0;
    while (m) { p[3 + n] = (uint8_t)m; n++; m >>= 8; }
    p[1] = (uint8_t)n;
    return p + 3 + n;
}

__device__ inline uint8_t *etf_u32be(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
    return p + 4;
}

// binary:encode_unsigned/1 length (0 -> <<0>>)
__host__ __device__ inline uint32_t enc_unsigned_len(uint64_t b) {
    uint32_t n = 1;
    while (b >> (8 * n) && n < 8) n++;
    return n;
}

// int64 value of a device integer key record (tag, BE bytes with the sign bit
// flipped for ordering: st_kernels.h key records)
__device__ inline int64_t krec_int(const uint8_t *p) {
    uint64_t u = 0;
    for (int i = 0; i < 8; i++) u = (u << 8) | p[1 + i];
    return (int64_t)(u ^ 0x8000000000000000ull);
}

// ETF size of the key of record bytes p[0..len)
__device__ inline uint32_t etf_key_size(const uint8_t *p, uint64_t len) {
    if (p[0] == KEYTAG_INT) return etf_int_size(krec_int(p));
    const uint64_t l = len - 1;
    if (p[0] == KEYTAG_ATOM) return (uint32_t)(l < 256 ? 2 + l : 3 + l);
    return (uint32_t)(5 + l);
}

__device__ inline uint8_t *etf_key_write(uint8_t *o, const uint8_t *p, uint64_t len) {
    if (p[0] == KEYTAG_INT) return etf_int_write(o, krec_int(p));
    const uint32_t l = (uint32_t)(len - 1);
    if (p[0] == KEYTAG_ATOM) {
        if (l < 256) { o[0] = 119; o[1] = (uint8_t)l; o += 2; }
        else { o[0] = 118; o[1] = (uint8_t)(l >> 8); o[2] = (uint8_t)l; o += 3; }
    } else {
        o[0] = 109; o = etf_u32be(o + 1, l);
    }
    for (uint32_t i = 0; i < l; i++) o[i] = p[1 + i];
    return o + l;
}

// level of record r (1..H+1); r >= 1
__device__ inline uint32_t snap_level(const DevTree &t, uint64_t r) {
    uint32_t L = 1;
    while (L <= t.H && r >= t.base[L + 1]) L++;
    return L;
}

// ETF bytes of every segment entry {Key, Value}: 2 + key + 5 + |Value|
__global__ void k_snap_entry_sizes(DevTree t, uint64_t n, uint64_t *es) {
    for (uint64_t e = gtid(); e <= n; e += gstride()) {
        if (e == n) { es[e] = 0; break; }
        const uint64_t k0 = t.koff[e];
        es[e] = 2 + etf_key_size(t.kheap + k0, t.koff[e + 1] - k0) + 5 + (t.voff[e + 1] - t.voff[e]);
    }
}

// Per record: present flag, key length, value length.  eo: exclusive scan of
// k_snap_entry_sizes (n + 1 entries).
__global__ void k_snap_sizes(DevTree t, uint32_t idlen, uint64_t R, const uint64_t *eo, uint64_t *pres, uint64_t *klen,
                             uint64_t *vlen) {
    for (uint64_t r = gtid(); r <= R; r += gstride()) {
        uint64_t p = 0, kl = 0, vl = 0;
        if (r == 0) {
            if (t.tag[1] & TAG_PRESENT) { p = 1; kl = 3 + idlen; vl = 23; }
        } else if (r < R) {
            const uint32_t L = snap_level(t, r);
            const uint64_t b = r - t.base[L];
            if (L <= t.H) {
                const uint64_t c0 = t.base[L + 1] + b * t.W;
                uint64_t cnt = 0, body = 0;
                for (uint32_t j = 0; j < t.W; j++)
                    if (t.tag[c0 + j] & TAG_PRESENT) {
                        cnt++;
                        body += 2 + etf_int_size((int64_t)(b * t.W + j)) + 22;
                    }
                if (cnt) { p = 1; vl = 7 + body; }
            } else {
                const uint64_t e0 = t.seg_off[b], e1 = t.seg_off[b + 1];
                if (e1 > e0) { p = 1; vl = 7 + eo[e1] - eo[e0]; }
            }
            if (p) kl = 2 + idlen + enc_unsigned_len(b);
        }
        pres[r] = p; klen[r] = kl; vlen[r] = vl;
    }
}

// Write every present record at its scanned offsets; rank[r] numbers the
// present records (output koff/voff entries).  Segment records get their
// list header and NIL here; k_snap_entries writes their entries.
__global__ void k_snap_write(DevTree t, const uint8_t *id, uint32_t idlen, uint64_t R, const uint64_t *rank,
                             const uint64_t *ko, const uint64_t *vo, const uint64_t *eo, uint8_t *kout, uint8_t *vout,
                             uint64_t *okoff, uint64_t *ovoff) {
    for (uint64_t r = gtid(); r < R; r += gstride()) {
        if (rank[r + 1] == rank[r]) continue;
        const uint64_t n = rank[r];
        okoff[n] = ko[r];
        ovoff[n] = vo[r];
        const uint32_t L = r == 0 ? 0 : snap_level(t, r);
        const uint64_t b = r == 0 ? 0 : r - t.base[L];
        // key <<0, Id, Level, encode_unsigned(Bucket)>>
        uint8_t *k = kout + ko[r];
        k[0] = 0;
        for (uint32_t i = 0; i < idlen; i++) k[1 + i] = id[i];
        k[1 + idlen] = (uint8_t)L;
        const uint32_t bl = enc_unsigned_len(b);
        for (uint32_t i = 0; i < bl; i++) k[2 + idlen + i] = (uint8_t)(b >> (8 * (bl - 1 - i)));
        uint8_t *v = vout + vo[r];
        v[0] = 131;
        if (L == 0) {
            v[1] = 109; v = etf_u32be(v + 2, 17);
            const uint4 m = t.md5[1];
            v[0] = (uint8_t)t.tag[1];
            const uint32_t w[4] = {m.x, m.y, m.z, m.w};
            for (int q = 0; q < 16; q++) v[1 + q] = (uint8_t)(w[q >> 2] >> (8 * (q & 3)));
            continue;
        }
        if (L <= t.H) {
            const uint64_t c0 = t.base[L + 1] + b * t.W;
            uint32_t cnt = 0;
            for (uint32_t j = 0; j < t.W; j++) cnt += (t.tag[c0 + j] & TAG_PRESENT) ? 1 : 0;
            v[1] = 108; v = etf_u32be(v + 2, cnt);
            for (uint32_t j = 0; j < t.W; j++) {
                const uint16_t tg = t.tag[c0 + j];
                if (!(tg & TAG_PRESENT)) continue;
                v[0] = 104; v[1] = 2;
                v = etf_int_write(v + 2, (int64_t)(b * t.W + j));
                v[0] = 109; v = etf_u32be(v + 1, 17);
                const uint4 m = t.md5[c0 + j];
                v[0] = (uint8_t)tg;
                const uint32_t w[4] = {m.x, m.y, m.z, m.w};
                for (int q = 0; q < 16; q++) v[1 + q] = (uint8_t)(w[q >> 2] >> (8 * (q & 3)));
                v += 17;
            }
            v[0] = 106;
            continue;
        }
        const uint64_t e0 = t.seg_off[b], e1 = t.seg_off[b + 1];
        v[1] = 108; v = etf_u32be(v + 2, (uint32_t)(e1 - e0));
        v[eo[e1] - eo[e0]] = 106;
    }
}

// One lane per segment entry: {Key, Value} at the record's value offset +
// 6 (list header) + the entry's offset within its segment.  Consecutive
// entries land in consecutive output bytes, so a wave's stores stay within
// a few cache lines.
__global__ void k_snap_entries(DevTree t, uint64_t n, uint64_t sb, const uint64_t *vo, const uint64_t *eo,
                               uint8_t *vout) {
    for (uint64_t e = gtid(); e < n; e += gstride()) {
        // segment of entry e: last s with seg_off[s] <= e (segments are non-empty here)
        uint64_t lo = 0, hi = t.S;
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (t.seg_off[mid] <= e) lo = mid; else hi = mid;
        }
        uint8_t *v = vout + vo[sb + lo] + 6 + (eo[e] - eo[t.seg_off[lo]]);
        v[0] = 104; v[1] = 2;
        const uint64_t k0 = t.koff[e];
        v = etf_key_write(v + 2, t.kheap + k0, t.koff[e + 1] - k0);
        const uint64_t v0 = t.voff[e], vl = t.voff[e + 1] - v0;
        v[0] = 109; v = etf_u32be(v + 1, (uint32_t)vl);
        for (uint64_t i = 0; i < vl; i++) v[i] = t.vheap[v0 + i];
    }
}
