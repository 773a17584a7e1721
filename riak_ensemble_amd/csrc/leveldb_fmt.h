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
// (three exclusive scans between them give the offsets: the library's
// three-launch scan, synctree_hip.hip exclusive_scan).  Node content is read
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

// Is a UTF-8 atom text representable in Latin-1 (every code point < 256)?
// Its Latin-1 length in *n.
__device__ inline bool utf8_latin1(const uint8_t *u, uint64_t l, uint32_t *n) {
    uint32_t c = 0;
    for (uint64_t i = 0; i < l; i++) {
        const uint8_t b = u[i];
        if (b < 0x80) { c++; continue; }
        if ((b == 0xC2 || b == 0xC3) && i + 1 < l) { c++; i++; continue; }
        return false;
    }
    *n = c;
    return true;
}

// ETF size of the key of record bytes p[0..len).  Atoms: ATOM_EXT (Latin-1)
// as term_to_binary writes them before OTP 26 (the reference's era, R16 -
// OTP 19: SURVEY §8c), the UTF-8 forms otherwise or with ST_FLAG_ATOM_UTF8.
// Term records carry their term_to_binary bytes (term_key.h).
__device__ inline uint32_t etf_key_size(const uint8_t *p, uint64_t len, uint32_t flags) {
    if (p[0] == KEYTAG_INT && len == 9) return etf_int_size(krec_int(p));
    if (krec_is_term(p, len)) {
        uint64_t ea, sa;
        uint32_t el, sl;
        krec_term_parts(p, len, &ea, &el, &sa, &sl);
        return el - 1;   // without the version byte
    }
    const uint64_t l = len - 1;
    if (p[0] == KEYTAG_ATOM) {
        uint32_t n;
        if (!(flags & ST_FLAG_ATOM_UTF8) && utf8_latin1(p + 1, l, &n)) return 3 + n;
        return (uint32_t)(l < 256 ? 2 + l : 3 + l);
    }
    return (uint32_t)(5 + l);
}

__device__ inline uint8_t *etf_key_write(uint8_t *o, const uint8_t *p, uint64_t len, uint32_t flags) {
    if (p[0] == KEYTAG_INT && len == 9) return etf_int_write(o, krec_int(p));
    if (krec_is_term(p, len)) {
        uint64_t ea, sa;
        uint32_t el, sl;
        krec_term_parts(p, len, &ea, &el, &sa, &sl);
        for (uint32_t i = 1; i < el; i++) o[i - 1] = p[ea + i];
        return o + el - 1;
    }
    const uint32_t l = (uint32_t)(len - 1);
    if (p[0] == KEYTAG_ATOM) {
        uint32_t n;
        if (!(flags & ST_FLAG_ATOM_UTF8) && utf8_latin1(p + 1, l, &n)) {
            o[0] = 100; o[1] = (uint8_t)(n >> 8); o[2] = (uint8_t)n; o += 3;
            for (uint32_t i = 0; i < l; i++) {
                const uint8_t b = p[1 + i];
                if (b < 0x80) *o++ = b;
                else { *o++ = (uint8_t)(((b & 0x1F) << 6) | (p[2 + i] & 0x3F)); i++; }
            }
            return o;
        }
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
        es[e] = 2 + etf_key_size(t.kheap + k0, t.koff[e + 1] - k0, t.flags) + 5 + (t.voff[e + 1] - t.voff[e]);
    }
}

// Per record: present flag, key length, value length.  eo: exclusive scan of
// k_snap_entry_sizes (n + 1 entries).
__global__ void k_snap_sizes(DevTree t, uint32_t idlen, uint64_t R, const uint64_t *eo, const uint8_t *erec,
                             uint64_t *pres, uint64_t *klen, uint64_t *vlen) {
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
                const uint64_t e0 = t.seg_off[b], e1 = t.seg_end[b];
                if (e1 > e0) { p = 1; vl = 7 + eo[e1] - eo[e0]; }
            }
            // an empty node the backend holds as [] (a raw store of [], or the
            // segment a corrupt/2 emptied, synctree.erl:246-247)
            if (!p && erec && erec[r]) { p = 1; vl = 2; }
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
            if (!cnt) { v[1] = 106; continue; }   // []
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
        const uint64_t e0 = t.seg_off[b], e1 = t.seg_end[b];
        if (e1 == e0) { v[1] = 106; continue; }   // []
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
        v = etf_key_write(v + 2, t.kheap + k0, t.koff[e + 1] - k0, t.flags);
        const uint64_t v0 = t.voff[e], vl = t.voff[e + 1] - v0;
        v[0] = 109; v = etf_u32be(v + 1, (uint32_t)vl);
        for (uint64_t i = 0; i < vl; i++) v[i] = t.vheap[v0 + i];
    }
}

// ---------------------------------------------------------------------------
// Restore: binary_to_term of the records on the device.
#define DK_DEPTH 48   // open tuples / lists of one key the device decodes (deeper keys: the host's)
//
// bad = malformed bytes (the reference's binary_to_term raises and fetch/3
// answers Default: the node is absent); dom = a well-formed term the device
// tree cannot hold (the whole restore fails with ST_EINVAL); host = a key
// this decoder leaves to the host's (term_key.h segment_from_etf): maps,
// FLOAT_EXT, keys nested deeper than DK_DEPTH.
struct DEtf {
    const uint8_t *p, *e;
    bool bad, dom, host;
    __device__ DEtf(const uint8_t *a, const uint8_t *b) : p(a), e(b), bad(false), dom(false), host(false) {}
    __device__ bool need(uint64_t n) {
        if (bad || (uint64_t)(e - p) < n) bad = true;
        return !bad;
    }
    __device__ uint32_t u8() { return need(1) ? *p++ : 0; }
    __device__ uint32_t u16() {
        if (!need(2)) return 0;
        const uint32_t v = ((uint32_t)p[0] << 8) | p[1];
        p += 2;
        return v;
    }
    __device__ uint32_t u32() {
        if (!need(4)) return 0;
        const uint32_t v = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
        p += 4;
        return v;
    }
    // a standard ETF tag outside the node domain, or garbage
    __device__ void other(uint32_t tg) {
        if (tg == 70 || tg == 77 || tg == 80 || tg == 88 || tg == 90 || (tg >= 97 && tg <= 120)) dom = true;
        else bad = true;
    }
    __device__ bool integer(int64_t &v) {
        const uint32_t tg = u8();
        if (bad) return false;
        if (tg == 97) { v = u8(); return !bad; }
        if (tg == 98) { v = (int32_t)u32(); return !bad; }
        if (tg == 110) {
            const uint32_t n = u8(), sign = u8();
            if (!need(n)) return false;
            uint64_t m = 0;
            bool big = false;
            for (uint32_t i = 0; i < n; i++) {
                if (i < 8) m |= (uint64_t)p[i] << (8 * i);
                else big |= p[i] != 0;
            }
            p += n;
            if (big || (!sign && m > 0x7FFFFFFFFFFFFFFFull) || (sign && m > 0x8000000000000000ull)) { dom = true; return false; }
            v = sign ? (int64_t)(0 - m) : (int64_t)m;
            return true;
        }
        other(tg);
        return false;
    }
    __device__ bool binary(const uint8_t *&b, uint32_t &len) {
        const uint32_t tg = u8();
        if (bad) return false;
        if (tg != 109) { other(tg); return false; }
        len = u32();
        if (!need(len)) return false;
        b = p;
        p += len;
        return true;
    }
    __device__ bool list(uint32_t &n) {
        const uint32_t tg = u8();
        if (bad) return false;
        if (tg == 106) { n = 0; return true; }
        if (tg != 108) { other(tg); return false; }
        n = u32();
        return !bad;
    }
    __device__ bool tuple2() {
        const uint32_t tg = u8();
        if (bad) return false;
        if (tg != 104) { other(tg); return false; }
        if (u8() != 2) { dom = !bad; return false; }
        return true;
    }
    __device__ bool nil() {
        const uint32_t tg = u8();
        if (bad) return false;
        if (tg != 106) { dom = true; return false; }   // an improper list
        return true;
    }
    __device__ bool version() {
        const uint32_t v = u8();
        if (!bad && v != 131) bad = true;
        if (!bad && p < e && *p == 80) { dom = true; return false; }   // compressed term
        return !bad;
    }
    __device__ bool end() {
        if (!bad && p != e) bad = true;   // trailing bytes: binary_to_term/1 raises badarg
        return !bad;
    }
    // Key term -> device key record (term_key.h): the plain form for int64,
    // atom and binary keys (integers as sign-flipped big-endian, Latin-1
    // atoms converted to UTF-8), the term record [SK][ETF][Seg][etf_len]
    // [seg_len] for every other key the host accepts (tuples, lists,
    // floats, integers outside int64, nested atoms / binaries).  dst NULL:
    // only the record length.
    __device__ bool key(uint8_t *dst, uint32_t &rlen) {
        if (!need(1)) return false;
        const uint32_t tg = *p;
        if (tg == 97 || tg == 98 || tg == 110 || tg == 111) {
            const uint8_t *t0 = p;
            int64_t v;
            if (tg == 111 || !integer(v)) {   // a bignum beyond int64: a term record
                if (bad) return false;
                p = t0;
                dom = false;
                return term_key(dst, rlen);
            }
            if (dst) {
                const uint64_t u = (uint64_t)v ^ 0x8000000000000000ull;
                dst[0] = KEYTAG_INT;
                for (int i = 0; i < 8; i++) dst[1 + i] = (uint8_t)(u >> (8 * (7 - i)));
            }
            rlen = 9;
            return true;
        }
        if (tg == 100 || tg == 115 || tg == 118 || tg == 119) {
            p++;
            const uint32_t len = (tg == 100 || tg == 118) ? u16() : u8();
            if (!need(len)) return false;
            const bool latin = tg == 100 || tg == 115;
            uint32_t o = 1;
            for (uint32_t i = 0; i < len; i++) {
                const uint8_t c = p[i];
                if (latin && c >= 0x80) {
                    if (dst) { dst[o] = (uint8_t)(0xC0 | (c >> 6)); dst[o + 1] = (uint8_t)(0x80 | (c & 0x3F)); }
                    o += 2;
                } else {
                    if (dst) dst[o] = c;
                    o++;
                }
            }
            if (dst) dst[0] = KEYTAG_ATOM;
            p += len;
            rlen = o;
            return true;
        }
        if (tg != 109) return term_key(dst, rlen);
        const uint8_t *b;
        uint32_t len;
        if (!binary(b, len)) return false;
        if (dst) {
            dst[0] = KEYTAG_BINARY;
            for (uint32_t i = 0; i < len; i++) dst[1 + i] = b[i];
        }
        rlen = 1 + len;
        return true;
    }

    // ---- term records (term_key.h, restated for the device: an explicit
    // stack instead of recursion, DK_DEPTH open tuples / lists at most)
    __device__ void sk_put(uint8_t *dst, uint32_t &o, uint32_t b) {
        if (dst) dst[o] = (uint8_t)b;
        o++;
    }
    __device__ void sk_int64(uint8_t *dst, uint32_t &o, int64_t v) {
        const uint64_t u = (uint64_t)v ^ 0x8000000000000000ull;
        sk_put(dst, o, KEYTAG_INT);
        for (int i = 7; i >= 0; i--) sk_put(dst, o, (uint32_t)(u >> (8 * i)) & 0xFF);
    }
    // |v| = mag[0..n) little-endian; the SK of the integer (int64 form when it fits)
    __device__ void sk_bigmag(uint8_t *dst, uint32_t &o, bool neg, const uint8_t *le, uint32_t n, uint32_t shift_bytes,
                              uint64_t lo64) {
        // n significant little-endian bytes (le[n-1] != 0) followed by shift_bytes zero bytes below them
        const uint32_t tot = n + shift_bytes;
        const bool fits = tot < 8 || (tot == 8 && (le[n - 1] < 0x80 || (neg && le[n - 1] == 0x80 && lo64 == 0x8000000000000000ull)));
        if (tot == 0) { sk_int64(dst, o, 0); return; }
        if (fits) { sk_int64(dst, o, neg ? (int64_t)(0 - lo64) : (int64_t)lo64); return; }
        if (tot > 255) { dom = true; return; }   // beyond the record's one-byte length (host alike)
        sk_put(dst, o, neg ? KEYTAG_NUMLO : KEYTAG_NUMHI);
        sk_put(dst, o, neg ? 255 - tot : tot);
        for (uint32_t i = 0; i < n; i++) sk_put(dst, o, neg ? (uint32_t)(uint8_t)~le[n - 1 - i] : le[n - 1 - i]);
        for (uint32_t i = 0; i < shift_bytes; i++) sk_put(dst, o, neg ? 0xFF : 0x00);
    }
    __device__ void sk_escaped(uint8_t *dst, uint32_t &o, uint32_t tag, const uint8_t *b, uint32_t n, bool latin) {
        sk_put(dst, o, tag);
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t c = b[i];
            if (latin && c >= 0x80) { sk_put(dst, o, 0xC0 | (c >> 6)); sk_put(dst, o, 0x80 | (c & 0x3F)); continue; }
            sk_put(dst, o, c);
            if (c == 0) sk_put(dst, o, 0xFF);
        }
        sk_put(dst, o, 0);
        sk_put(dst, o, 1);
    }
    __device__ void sk_float(uint8_t *dst, uint32_t &o, double v) {
        const double two63 = 9223372036854775808.0;
        if (v >= -two63 && v < two63) {
            const double f = floor(v);
            const double r = v - f;
            sk_int64(dst, o, (int64_t)f);
            if (r == 0.0) return;   // integral (and -0.0): the SK of the equal integer
            const uint64_t bits = (uint64_t)__double_as_longlong(r);
            sk_put(dst, o, SK_FLOAT);
            for (int i = 7; i >= 0; i--) sk_put(dst, o, (uint32_t)(bits >> (8 * i)) & 0xFF);
            return;
        }
        int ex;
        const double m = frexp(fabs(v), &ex);                 // |v| = m * 2^ex, m in [0.5, 1)
        const uint64_t mant = (uint64_t)ldexp(m, 53);         // 53-bit integer
        const uint32_t shift = (uint32_t)(ex - 53);           // >= 11 here
        const uint64_t x = mant << (shift & 7);               // <= 60 bits
        uint8_t le[8];
        uint32_t n = 0;
        for (uint64_t y = x; y; y >>= 8) le[n++] = (uint8_t)y;
        sk_bigmag(dst, o, v < 0, le, n, shift >> 3, 0);
    }
    // One term at p (a key, not in the plain domain) -> its term record.
    __device__ bool term_key(uint8_t *dst, uint32_t &rlen) {
        const uint8_t *t0 = p;
        uint32_t o = 0;
        uint32_t kind[DK_DEPTH], rem[DK_DEPTH];   // open containers: 0 tuple, 1 list, 2 list tail
        int sp = 0;
        bool top = true, big = false;
        uint64_t big_lo = 0;
        for (;;) {
            const uint32_t tg = u8();
            if (bad) return false;
            bool opened = false;
            switch (tg) {
            case 97: sk_int64(dst, o, (int64_t)u8()); break;
            case 98: sk_int64(dst, o, (int64_t)(int32_t)u32()); break;
            case 110: case 111: {
                const uint32_t n = tg == 110 ? u8() : u32();
                const uint32_t sign = u8();
                if (!need(n)) return false;
                uint32_t m = n;
                while (m && p[m - 1] == 0) m--;   // significant magnitude bytes
                uint64_t lo = 0;
                for (uint32_t i = 0; i < 8 && i < n; i++) lo |= (uint64_t)p[i] << (8 * i);
                sk_bigmag(dst, o, sign != 0 && m, p, m, 0, lo);
                if (top && !(m < 8 || (m == 8 && (p[7] < 0x80 || (sign && lo == 0x8000000000000000ull))))) {
                    big = true;   // ensure_binary(Integer) = <<Key:64>>: the low 64 bits, two's complement
                    big_lo = sign ? 0 - lo : lo;
                }
                p += n;
                break;
            }
            case 70: {
                if (!need(8)) return false;
                uint64_t b = 0;
                for (int i = 0; i < 8; i++) b = (b << 8) | p[i];
                p += 8;
                const double v = __longlong_as_double((long long)b);
                if (!isfinite(v)) { bad = true; return false; }   // binary_to_term refuses non-finite floats
                sk_float(dst, o, v);
                break;
            }
            case 100: case 115: case 118: case 119: {
                const uint32_t n = (tg == 100 || tg == 118) ? u16() : u8();
                if (!need(n)) return false;
                sk_escaped(dst, o, KEYTAG_ATOM, p, n, tg == 100 || tg == 115);
                p += n;
                break;
            }
            case 109: {
                const uint32_t n = u32();
                if (!need(n)) return false;
                sk_escaped(dst, o, KEYTAG_BINARY, p, n, false);
                p += n;
                break;
            }
            case 104: case 105: {
                const uint32_t n = tg == 104 ? u8() : u32();
                if (bad) return false;
                sk_put(dst, o, KEYTAG_TUPLE);
                for (int i = 3; i >= 0; i--) sk_put(dst, o, (n >> (8 * i)) & 0xFF);
                if (n) {
                    if (sp == DK_DEPTH) { host = true; return false; }
                    kind[sp] = 0; rem[sp] = n; sp++;
                    opened = true;
                }
                break;
            }
            case 106: sk_put(dst, o, KEYTAG_NIL); break;
            case 107: {
                const uint32_t n = u16();
                if (!need(n)) return false;
                sk_put(dst, o, KEYTAG_LIST);
                for (uint32_t i = 0; i < n; i++) sk_int64(dst, o, p[i]);
                p += n;
                sk_put(dst, o, SK_LIST_END);
                break;
            }
            case 108: {
                const uint32_t n = u32();
                if (bad) return false;
                if (n == 0) { dom = true; return false; }   // never written by term_to_binary
                if (sp == DK_DEPTH) { host = true; return false; }
                sk_put(dst, o, KEYTAG_LIST);
                kind[sp] = 1; rem[sp] = n; sp++;
                opened = true;
                break;
            }
            case 99: case 116: host = true; return false;   // FLOAT_EXT, maps: the host's decoder
            default:
                other(tg);   // pids, ports, refs, funs, bitstrings: outside the key domain
                return false;
            }
            if (dom) return false;
            top = false;
            if (opened) continue;
            // the term is complete: close the containers it completes
            while (sp > 0) {
                const int q = sp - 1;
                if (kind[q] == 2) { sp--; continue; }   // a list's improper tail ends the list
                if (--rem[q]) break;                    // more elements
                if (kind[q] == 0) { sp--; continue; }   // a tuple ends
                if (!need(1)) return false;             // a list's elements ended: its tail
                const uint32_t t = *p;
                if (t == 106) { p++; sk_put(dst, o, SK_LIST_END); sp--; continue; }
                if (t == 108) {                         // the tail is a list: the same list goes on
                    p++;
                    rem[q] = u32();
                    if (bad) return false;
                    if (rem[q] == 0) { dom = true; return false; }
                    break;
                }
                if (t == 107) {                         // a string tail: small integers, then []
                    p++;
                    const uint32_t n = u16();
                    if (!need(n)) return false;
                    for (uint32_t i = 0; i < n; i++) sk_int64(dst, o, p[i]);
                    p += n;
                    sk_put(dst, o, SK_LIST_END);
                    sp--;
                    continue;
                }
                sk_put(dst, o, t == 109 ? SK_TAIL_HIGH : SK_TAIL_LOW);   // improper tail: compared as a term
                kind[q] = 2;
                break;
            }
            if (sp == 0) break;
        }
        // [SK][ETF = 131 ++ the term's bytes][Seg][etf_len u16 LE][seg_len u16 LE]
        const uint32_t etf_len = 1 + (uint32_t)(p - t0);
        if (etf_len > 0xFFFE) { dom = true; return false; }
        if (dst) {
            dst[o] = 131;
            for (uint32_t i = 1; i < etf_len; i++) dst[o + i] = t0[i - 1];
        }
        uint32_t r = o + etf_len;
        if (big) {
            if (dst) for (int i = 0; i < 8; i++) dst[r + i] = (uint8_t)(big_lo >> (8 * (7 - i)));
            r += 8;
        }
        const uint32_t seg_len = big ? 8u : 0xFFFFu;
        if (dst) {
            dst[r] = (uint8_t)(etf_len & 0xFF); dst[r + 1] = (uint8_t)(etf_len >> 8);
            dst[r + 2] = (uint8_t)(seg_len & 0xFF); dst[r + 3] = (uint8_t)(seg_len >> 8);
        }
        rlen = r + 4;
        return true;
    }
};

// Counters of one restore: [0] nodes loaded, [1] undecodable nodes skipped,
// [2] domain error flag, [3] lowest record slot with a domain error.
#define RST_LOADED 0
#define RST_SKIPPED 1
#define RST_DOM 2
#define RST_DOMSLOT 3
#define RST_HOST 4      // segments handed to the host decoder (segok 2)

__device__ inline void rst_dom(unsigned long long *ctr, uint64_t r) {
    atomicOr(&ctr[RST_DOM], 1ull);
    atomicMin(&ctr[RST_DOMSLOT], (unsigned long long)r);
}

__device__ inline void set_entry_dev(uint16_t &tag, uint4 &m, const uint8_t *h17) {
    tag = (uint16_t)(TAG_PRESENT | h17[0]);
    uint32_t w[4];
    for (int k = 0; k < 4; k++)
        w[k] = (uint32_t)h17[1 + 4 * k] | ((uint32_t)h17[2 + 4 * k] << 8) | ((uint32_t)h17[3 + 4 * k] << 16) |
               ((uint32_t)h17[4 + 4 * k] << 24);
    m = make_uint4(w[0], w[1], w[2], w[3]);
}

// One lane per record: its node slot r (db_key/3 inverted for this tree id
// and geometry); the last record of a key wins (atomicMax of index + 1).
// Other trees' records and keys db_key/3 never produces are ignored.
__global__ void k_rest_keys(DevTree t, const uint8_t *id, uint32_t idlen, uint64_t n, const uint8_t *kh,
                            const uint64_t *ko, unsigned long long *recof) {
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const uint8_t *k = kh + ko[i];
        const uint64_t kl = ko[i + 1] - ko[i];
        if (kl < 3 + (uint64_t)idlen || k[0] != 0) continue;
        bool same = true;
        for (uint32_t q = 0; q < idlen; q++) same &= k[1 + q] == id[q];
        if (!same) continue;
        const uint32_t L = k[1 + idlen];
        const uint8_t *bb = k + 2 + idlen;
        const uint64_t bl = kl - 2 - idlen;
        if (bl > 8 || (bl > 1 && bb[0] == 0) || L > t.H + 1) continue;
        uint64_t b = 0;
        for (uint64_t q = 0; q < bl; q++) b = (b << 8) | bb[q];
        if (L == 0 ? b != 0 : b >= t.base[L + 1] - t.base[L]) continue;
        atomicMax(&recof[L == 0 ? 0 : t.base[L] + b], (unsigned long long)(i + 1));
    }
}

// One lane per node slot r: decode its record (if any).  {0,0} and inner
// nodes go straight into the staging slot arrays (stag/smd, zeroed); a
// segment is validated and sized (entries, key-record bytes, value bytes).
__global__ void k_rest_nodes(DevTree t, uint64_t R, const unsigned long long *recof, const uint8_t *vh,
                             const uint64_t *vo, uint16_t *stag, uint4 *smd, uint64_t *ecnt, uint64_t *kcnt,
                             uint64_t *vcnt, uint8_t *segok, uint8_t *serec, unsigned long long *ctr) {
    const uint64_t sb = t.base[t.H + 1];
    for (uint64_t r = gtid(); r < R; r += gstride()) {
        const bool seg = r >= sb;
        if (seg) { ecnt[r - sb] = 0; kcnt[r - sb] = 0; vcnt[r - sb] = 0; segok[r - sb] = 0; }
        const unsigned long long i1 = recof[r];
        if (!i1) continue;
        const uint64_t i = i1 - 1;
        DEtf in(vh + vo[i], vh + vo[i + 1]);
        bool good = in.version();
        if (r == 0) {
            const uint8_t *h = nullptr;
            uint32_t len = 0;
            good = good && in.binary(h, len) && in.end();
            if (good && len != 17) in.dom = true;
            if (in.dom) { rst_dom(ctr, r); continue; }
            if (!good) { atomicAdd(&ctr[RST_SKIPPED], 1ull); continue; }
            set_entry_dev(stag[1], smd[1], h);
            set_entry_dev(stag[0], smd[0], h);   // reload_top_hash (synctree.erl:172-175)
            atomicAdd(&ctr[RST_LOADED], 1ull);
            continue;
        }
        if (!seg) {
            const uint32_t L = snap_level(t, r);
            const uint64_t b = r - t.base[L], c0 = t.base[L + 1] + b * t.W;
            uint32_t cnt = 0;
            good = good && in.list(cnt);
            const uint8_t *first = in.p;
            int64_t prevc = -1;
            for (uint32_t j = 0; good && j < cnt; j++) {
                int64_t c = 0;
                const uint8_t *h;
                uint32_t len = 0;
                good = in.tuple2() && in.integer(c) && in.binary(h, len);
                if (good && (len != 17 || c < (int64_t)(b * t.W) || c >= (int64_t)((b + 1) * t.W) || c <= prevc)) in.dom = true;
                if (in.dom) break;
                prevc = c;
            }
            if (good && !in.dom && cnt) good = in.nil();
            good = good && !in.dom && in.end();
            if (in.dom) { rst_dom(ctr, r); continue; }
            if (!good) { atomicAdd(&ctr[RST_SKIPPED], 1ull); continue; }
            if (cnt == 0) serec[r] = 1;      // a [] record
            DEtf w(first, vh + vo[i + 1]);   // second pass: store the validated children
            for (uint32_t j = 0; j < cnt; j++) {
                int64_t c = 0;
                const uint8_t *h;
                uint32_t len;
                w.tuple2(); w.integer(c); w.binary(h, len);
                const uint64_t s = c0 + ((uint64_t)c - b * t.W);
                set_entry_dev(stag[s], smd[s], h);
            }
            atomicAdd(&ctr[RST_LOADED], 1ull);
            continue;
        }
        uint32_t cnt = 0;
        uint64_t kb = 0, vb = 0;
        good = good && in.list(cnt);
        for (uint32_t j = 0; good && j < cnt; j++) {
            uint32_t kl = 0, len = 0;
            const uint8_t *v;
            good = in.tuple2() && in.key(nullptr, kl) && in.binary(v, len);
            if (in.dom || in.host) break;
            kb += kl;
            vb += len;
        }
        if (in.host) { segok[r - sb] = 2; atomicAdd(&ctr[RST_HOST], 1ull); continue; }
        if (good && !in.dom && cnt) good = in.nil();
        good = good && !in.dom && in.end();
        if (in.dom) { rst_dom(ctr, r); continue; }
        if (!good) { atomicAdd(&ctr[RST_SKIPPED], 1ull); continue; }   // fetch/3 answers []
        ecnt[r - sb] = cnt; kcnt[r - sb] = kb; vcnt[r - sb] = vb;
        segok[r - sb] = 1;
        if (cnt == 0) serec[r] = 1;
        atomicAdd(&ctr[RST_LOADED], 1ull);
    }
}

// One lane per validated segment: its entries' key records and values into
// the new CSR at the scanned offsets; keys must be strictly ascending (an
// orddict), else a domain error.
__global__ void k_rest_segments(DevTree t, const unsigned long long *recof, const uint8_t *vh, const uint64_t *vo,
                                const uint8_t *segok, const uint64_t *seg_off, const uint64_t *kbase,
                                const uint64_t *vbase, uint64_t *koff, uint8_t *kheap, uint64_t *voff, uint8_t *vheap,
                                unsigned long long *ctr) {
    const uint64_t sb = t.base[t.H + 1];
    for (uint64_t s = gtid(); s < t.S; s += gstride()) {
        if (segok[s] != 1) continue;
        const uint64_t i = recof[sb + s] - 1;
        DEtf in(vh + vo[i], vh + vo[i + 1]);
        uint32_t cnt = 0;
        in.version();
        in.list(cnt);
        uint64_t e = seg_off[s], kp = kbase[s], vp = vbase[s];
        uint64_t pk = 0, pl = 0;
        for (uint32_t j = 0; j < cnt; j++, e++) {
            uint32_t kl = 0, len = 0;
            const uint8_t *v;
            in.tuple2();
            in.key(kheap + kp, kl);
            in.binary(v, len);
            if (j && rec_cmp(kheap + pk, pl, kheap + kp, kl) >= 0)   // strictly ascending in Erlang term order
                rst_dom(ctr, sb + s);
            koff[e] = kp;
            voff[e] = vp;
            for (uint32_t q = 0; q < len; q++) vheap[vp + q] = v[q];
            pk = kp; pl = kl;
            kp += kl;
            vp += len;
        }
    }
}

// The segments the host decoded (hs[i], entries [he[i], he[i+1]) of the
// host's key records hk / values hv with end offsets hko / hvo, one leading
// 0): sizes before the scans, entries after them.
__global__ void k_rest_host_sizes(uint64_t n, const uint64_t *hs, const uint64_t *he, const uint64_t *hko,
                                  const uint64_t *hvo, uint64_t *ec, uint64_t *kc, uint64_t *vc) {
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const uint64_t s = hs[i], a = he[i], b = he[i + 1];
        ec[s] = b - a;
        kc[s] = hko[b] - hko[a];
        vc[s] = hvo[b] - hvo[a];
    }
}

__global__ void k_rest_host_write(uint64_t n, const uint64_t *hs, const uint64_t *he, const uint64_t *hko,
                                  const uint64_t *hvo, const uint8_t *hk, const uint8_t *hv, const uint64_t *seg_off,
                                  const uint64_t *kbase, const uint64_t *vbase, uint64_t *koff, uint8_t *kheap,
                                  uint64_t *voff, uint8_t *vheap) {
    for (uint64_t i = gtid(); i < n; i += gstride()) {
        const uint64_t s = hs[i], a = he[i], b = he[i + 1];
        const uint64_t e = seg_off[s], kp = kbase[s], vp = vbase[s], k0 = hko[a], v0 = hvo[a];
        for (uint64_t j = a; j < b; j++) {
            koff[e + j - a] = kp + hko[j] - k0;
            voff[e + j - a] = vp + hvo[j] - v0;
        }
        for (uint64_t q = k0; q < hko[b]; q++) kheap[kp + q - k0] = hk[q];
        for (uint64_t q = v0; q < hvo[b]; q++) vheap[vp + q - v0] = hv[q];
    }
}
