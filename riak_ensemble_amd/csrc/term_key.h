// term_key.h — host-side key records for term_to_binary keys (ST_KEY_TERM).
//
// The reference hashes a key that is not an integer, atom or binary through
// term_to_binary (ensure_binary/1, src/synctree.erl:261-268), and keeps the
// entries of a segment in Erlang term order (orddict:store, :206).  The
// device orders key records with memcmp, so a term key becomes
//
//     [SK(Key)] [ETF] [Seg] [etf_len u16 LE] [seg_len u16 LE]
//
// SK is a self-delimiting, order-preserving encoding of the term (memcmp of
// two SKs = Erlang term order, defined below); ETF = term_to_binary(Key) as
// given by the caller (leveldb snapshots copy it); Seg = ensure_binary(Key),
// the bytes get_segment/2 hashes (seg_len 0xFFFF: Seg = ETF, the
// term_to_binary case; integers outside int64 hash <<Key:64>>, their low 64
// bits).  The plain records of the int64 / atom / binary domain keep their
// short form (tag + payload), with tags that interleave with the SK classes:
//
//   0x0F  integer < -2^63   [0x0F][255 - n][~magnitude, n bytes BE]
//   0x10  int64             [0x10][8 bytes BE, sign bit flipped]
//         float in [-2^63, 2^63): [0x10][floor as above][0xFE][frac, 8 bytes],
//         an integral float (frac 0) without the [0xFE][frac] part
//   0x11  integer >= 2^63   [0x11][n][magnitude, n bytes BE]
//         (floats beyond int64 are integral: the SK of the equal integer)
//   0x20  atom              [0x20][utf8, escaped][00 01]
//   0x30  tuple             [0x30][arity u32 BE][SK(e1)]...[SK(en)]
//   0x34  map               [0x34][size u32 BE][SKX(k1)]...[SKX(kn)][SK(v1)]...[SK(vn)]
//                           with k1 < ... < kn in map-key order
//   0x38  nil               [0x38]
//   0x40  list              [0x40][SK(h1)]...[end]; end = [03] for a proper
//                           list, [02][SK(T)] for a tail T < nil (number,
//                           atom, tuple), [F0][SK(T)] for a binary tail
//   0x50  binary            [0x50][bytes, escaped][00 01]
//
// Escaping (nested atoms / binaries only): 0x00 -> 00 FF, end -> 00 01.
// ERTS type order: number < atom < (reference < fun < port < pid) < tuple <
// map < nil < list < bitstring; the bracketed types are rejected.  Maps order
// by size, then their keys in map-key order, then their values in key order;
// map keys compare EXACTLY (=:=, "integers are less than floats" in map-key
// order: 1 and 1.0 are two keys, every integer sorts before every float).
// SKX, the exact form used for map keys (and everything under them), is the
// SK with numbers split by type: integers as above, floats as
// [0x18][IEEE bits, order-preserving] (-0.0 as 0.0).  Numbers
// compare by value, and an integer and a float of equal value (1 and 1.0,
// also nested: {1} and {1.0}) have the SAME SK: they are equal keys (==), as
// orddict:store/erase, lists:keyfind and orddict_delta treat them; the key
// comparison (krec_order_len in st_kernels.h) looks at the SK bytes only, and
// a store of one form replaces an entry of the other (orddict:store keeps the
// new key).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#define KEYTAG_NUMLO 0x0F
#define KEYTAG_INT 0x10
#define KEYTAG_NUMHI 0x11
#define KEYTAG_ATOM 0x20
#define KEYTAG_XFLOAT 0x18
#define KEYTAG_TUPLE 0x30
#define KEYTAG_MAP 0x34
#define KEYTAG_NIL 0x38
#define KEYTAG_LIST 0x40
#define KEYTAG_BINARY 0x50
#define SK_TAIL_LOW 0x02
#define SK_LIST_END 0x03
#define SK_TAIL_HIGH 0xF0
#define SK_FLOAT 0xFE

namespace termkey {

struct Etf {
    const uint8_t *p, *e;
    std::string err;
    int depth = 0;
    bool dom = false;   // err is a well-formed term outside the key domain (not malformed bytes)
    bool need(size_t n) {
        if ((size_t)(e - p) < n) { if (err.empty()) err = "truncated term_to_binary"; return false; }
        return true;
    }
    uint32_t u8() { return *p++; }
    uint32_t u16() { uint32_t v = ((uint32_t)p[0] << 8) | p[1]; p += 2; return v; }
    uint32_t u32() { uint32_t v = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; p += 4; return v; }
};

// the standard ETF tags: a term the decoder does not take is outside the
// domain (pids, ports, refs, funs, bitstrings, compressed terms); any other
// byte is garbage
inline bool etf_known_tag(uint32_t tag) {
    return tag == 70 || tag == 77 || tag == 80 || tag == 88 || tag == 90 || (tag >= 97 && tag <= 120);
}

// magnitude bytes (big-endian, no leading zeros) + sign -> SK
inline void sk_integer(std::vector<uint8_t> &o, bool neg, const std::vector<uint8_t> &mag) {
    size_t n = mag.size();
    // fits int64?  |v| <= 2^63 - 1, or v = -2^63
    bool fits = n < 8 || (n == 8 && (mag[0] < 0x80 || (neg && mag[0] == 0x80 &&
                                                          std::all_of(mag.begin() + 1, mag.end(), [](uint8_t b) { return b == 0; }))));
    if (fits) {
        uint64_t m = 0;
        for (uint8_t b : mag) m = (m << 8) | b;
        const uint64_t u = (neg ? (uint64_t)(0 - m) : m) ^ 0x8000000000000000ull;
        o.push_back(KEYTAG_INT);
        for (int i = 7; i >= 0; i--) o.push_back((uint8_t)(u >> (8 * i)));
        return;
    }
    if (neg) {
        o.push_back(KEYTAG_NUMLO);
        o.push_back((uint8_t)(255 - n));
        for (uint8_t b : mag) o.push_back((uint8_t)~b);
    } else {
        o.push_back(KEYTAG_NUMHI);
        o.push_back((uint8_t)n);
        o.insert(o.end(), mag.begin(), mag.end());
    }
}

inline void sk_escaped(std::vector<uint8_t> &o, uint8_t tag, const uint8_t *b, size_t n) {
    o.push_back(tag);
    for (size_t i = 0; i < n; i++) {
        o.push_back(b[i]);
        if (b[i] == 0) o.push_back(0xFF);
    }
    o.push_back(0);
    o.push_back(1);
}

inline void latin1_to_utf8(const uint8_t *b, size_t n, std::vector<uint8_t> &u) {
    for (size_t i = 0; i < n; i++) {
        if (b[i] < 0x80) u.push_back(b[i]);
        else { u.push_back((uint8_t)(0xC0 | (b[i] >> 6))); u.push_back((uint8_t)(0x80 | (b[i] & 0x3F))); }
    }
}

inline void sk_float(std::vector<uint8_t> &o, double v) {
    const double two63 = 9223372036854775808.0;
    if (v >= -two63 && v < two63) {
        const double f = std::floor(v);
        const double r = v - f;   // exact, in [0, 1)
        const int64_t fi = (int64_t)f;
        const uint64_t u = (uint64_t)fi ^ 0x8000000000000000ull;
        o.push_back(KEYTAG_INT);
        for (int i = 7; i >= 0; i--) o.push_back((uint8_t)(u >> (8 * i)));
        if (r == 0.0) return;   // integral (and -0.0): the SK of the equal integer
        uint64_t bits;
        std::memcpy(&bits, &r, 8);
        o.push_back(SK_FLOAT);
        for (int i = 7; i >= 0; i--) o.push_back((uint8_t)(bits >> (8 * i)));
        return;
    }
    // integral: mantissa * 2^exp with exp >= 0
    int ex;
    const double m = std::frexp(std::fabs(v), &ex);   // |v| = m * 2^ex, m in [0.5, 1)
    const uint64_t mant = (uint64_t)std::ldexp(m, 53);  // 53-bit integer
    const int shift = ex - 53;                            // >= 11 here
    // magnitude = mant << shift, as big-endian bytes
    std::vector<uint8_t> le;   // little-endian bytes
    uint64_t carry = mant;
    int bits = shift;
    while (bits >= 8) { le.push_back(0); bits -= 8; }
    unsigned __int128 x = (unsigned __int128)carry << bits;
    while (x) { le.push_back((uint8_t)x); x >>= 8; }
    std::vector<uint8_t> mag(le.rbegin(), le.rend());
    sk_integer(o, v < 0, mag);   // integral: the SK of the equal integer
}

// term -> SK; returns the ERTS type class of the term (for list tails), or -1
enum Cls { C_NUM = 0, C_ATOM = 1, C_TUPLE = 2, C_NIL = 3, C_LIST = 4, C_BIN = 5, C_MAP = 6 };

inline int sk_term(Etf &in, std::vector<uint8_t> &o, bool top, bool exact, bool *is_int64, int64_t *ival,
                   bool *is_big, std::vector<uint8_t> *bigmag, bool *bigneg);

// a float in the exact (map-key) order: above every integer, by value
inline void skx_float(std::vector<uint8_t> &o, double v) {
    if (v == 0.0) v = 0.0;   // -0.0 =:= 0.0
    uint64_t b;
    std::memcpy(&b, &v, 8);
    b = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
    o.push_back(KEYTAG_XFLOAT);
    for (int i = 7; i >= 0; i--) o.push_back((uint8_t)(b >> (8 * i)));
}

inline bool sk_bigint(Etf &in, uint32_t n, std::vector<uint8_t> &mag, bool &neg) {
    if (!in.need(1 + (size_t)n)) return false;
    neg = in.u8() != 0;
    mag.clear();
    for (uint32_t i = 0; i < n; i++) mag.push_back(in.p[n - 1 - i]);   // LE -> BE
    in.p += n;
    size_t z = 0;
    while (z < mag.size() && mag[z] == 0) z++;
    mag.erase(mag.begin(), mag.begin() + z);
    if (mag.empty()) neg = false;
    return true;
}

inline int sk_list_rest(Etf &in, std::vector<uint8_t> &o, bool exact);

inline int sk_term(Etf &in, std::vector<uint8_t> &o, bool top, bool exact, bool *is_int64, int64_t *ival,
                   bool *is_big, std::vector<uint8_t> *bigmag, bool *bigneg) {
    if (++in.depth > 200) { in.err = "term nested too deeply"; return -1; }
    if (!in.need(1)) return -1;
    const uint32_t tag = in.u8();
    int cls = -1;
    switch (tag) {
    case 97:   // SMALL_INTEGER_EXT
    case 98: { // INTEGER_EXT
        int64_t v;
        if (tag == 97) { if (!in.need(1)) return -1; v = in.u8(); }
        else { if (!in.need(4)) return -1; v = (int32_t)in.u32(); }
        const uint64_t u = (uint64_t)v ^ 0x8000000000000000ull;
        o.push_back(KEYTAG_INT);
        for (int i = 7; i >= 0; i--) o.push_back((uint8_t)(u >> (8 * i)));
        if (is_int64) { *is_int64 = true; *ival = v; }
        cls = C_NUM;
        break;
    }
    case 110:   // SMALL_BIG_EXT
    case 111: { // LARGE_BIG_EXT
        uint32_t n;
        if (tag == 110) { if (!in.need(1)) return -1; n = in.u8(); }
        else { if (!in.need(4)) return -1; n = in.u32(); }
        std::vector<uint8_t> mag;
        bool neg;
        if (!sk_bigint(in, n, mag, neg)) return -1;
        const size_t at = o.size();
        sk_integer(o, neg, mag);
        if (o[at] == KEYTAG_INT) {
            if (is_int64) {
                uint64_t u = 0;
                for (int i = 1; i <= 8; i++) u = (u << 8) | o[at + i];
                *is_int64 = true;
                *ival = (int64_t)(u ^ 0x8000000000000000ull);
            }
        } else if (is_big) {
            *is_big = true;
            *bigmag = mag;
            *bigneg = neg;
        }
        cls = C_NUM;
        break;
    }
    case 70: { // NEW_FLOAT_EXT
        if (!in.need(8)) return -1;
        uint64_t b = 0;
        for (int i = 0; i < 8; i++) b = (b << 8) | in.p[i];
        in.p += 8;
        double v;
        std::memcpy(&v, &b, 8);
        if (!std::isfinite(v)) { in.err = "non-finite float"; return -1; }
        if (exact) skx_float(o, v);
        else sk_float(o, v);
        cls = C_NUM;
        break;
    }
    case 99: { // FLOAT_EXT: 31-byte "%.20e" string
        if (!in.need(31)) return -1;
        char buf[32];
        std::memcpy(buf, in.p, 31);
        buf[31] = 0;
        in.p += 31;
        char *end = nullptr;
        const double v = std::strtod(buf, &end);
        if (end == buf || !std::isfinite(v)) { in.err = "bad FLOAT_EXT"; return -1; }
        if (exact) skx_float(o, v);
        else sk_float(o, v);
        cls = C_NUM;
        break;
    }
    case 100: case 115: case 118: case 119: {   // atoms
        uint32_t n;
        if (tag == 100 || tag == 118) { if (!in.need(2)) return -1; n = in.u16(); }
        else { if (!in.need(1)) return -1; n = in.u8(); }
        if (!in.need(n)) return -1;
        std::vector<uint8_t> u;
        if (tag == 100 || tag == 115) latin1_to_utf8(in.p, n, u);
        else u.assign(in.p, in.p + n);
        in.p += n;
        if (top) { o.push_back(KEYTAG_ATOM); o.insert(o.end(), u.begin(), u.end()); }
        else sk_escaped(o, KEYTAG_ATOM, u.data(), u.size());
        cls = C_ATOM;
        break;
    }
    case 104: case 105: {   // tuples
        uint32_t n;
        if (tag == 104) { if (!in.need(1)) return -1; n = in.u8(); }
        else { if (!in.need(4)) return -1; n = in.u32(); }
        o.push_back(KEYTAG_TUPLE);
        for (int i = 3; i >= 0; i--) o.push_back((uint8_t)(n >> (8 * i)));
        for (uint32_t i = 0; i < n; i++)
            if (sk_term(in, o, false, exact, nullptr, nullptr, nullptr, nullptr, nullptr) < 0) return -1;
        cls = C_TUPLE;
        break;
    }
    case 106:   // NIL_EXT
        o.push_back(KEYTAG_NIL);
        cls = C_NIL;
        break;
    case 107: { // STRING_EXT: a list of small integers
        if (!in.need(2)) return -1;
        const uint32_t n = in.u16();
        if (!in.need(n)) return -1;
        o.push_back(KEYTAG_LIST);
        for (uint32_t i = 0; i < n; i++) {
            const uint64_t u = (uint64_t)in.p[i] ^ 0x8000000000000000ull;
            o.push_back(KEYTAG_INT);
            for (int k = 7; k >= 0; k--) o.push_back((uint8_t)(u >> (8 * k)));
        }
        in.p += n;
        o.push_back(SK_LIST_END);
        cls = C_LIST;
        break;
    }
    case 108: { // LIST_EXT
        in.p--;
        o.push_back(KEYTAG_LIST);
        if (sk_list_rest(in, o, exact) < 0) return -1;
        cls = C_LIST;
        break;
    }
    case 109: { // BINARY_EXT
        if (!in.need(4)) return -1;
        const uint32_t n = in.u32();
        if (!in.need(n)) return -1;
        if (top) { o.push_back(KEYTAG_BINARY); o.insert(o.end(), in.p, in.p + n); }
        else sk_escaped(o, KEYTAG_BINARY, in.p, n);
        in.p += n;
        cls = C_BIN;
        break;
    }
    case 116: { // MAP_EXT: Arity, then Arity key/value pairs in any order
        if (!in.need(4)) return -1;
        const uint32_t n = in.u32();
        if ((uint64_t)n * 2 > (uint64_t)(in.e - in.p)) { in.err = "truncated term_to_binary"; return -1; }
        std::vector<std::vector<uint8_t>> ks(n), vs(n);
        std::vector<uint32_t> ord(n);
        for (uint32_t i = 0; i < n; i++) {
            ord[i] = i;
            if (sk_term(in, ks[i], false, true, nullptr, nullptr, nullptr, nullptr, nullptr) < 0) return -1;
            if (sk_term(in, vs[i], false, exact, nullptr, nullptr, nullptr, nullptr, nullptr) < 0) return -1;
        }
        std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return ks[a] < ks[b]; });
        for (uint32_t i = 1; i < n; i++)
            if (ks[ord[i - 1]] == ks[ord[i]]) { in.err = "map with a repeated key"; return -1; }
        o.push_back(KEYTAG_MAP);
        for (int i = 3; i >= 0; i--) o.push_back((uint8_t)(n >> (8 * i)));
        for (uint32_t i : ord) o.insert(o.end(), ks[i].begin(), ks[i].end());
        for (uint32_t i : ord) o.insert(o.end(), vs[i].begin(), vs[i].end());
        cls = C_MAP;
        break;
    }
    default:
        // the standard tags of pids, ports, refs, funs, bitstrings, compressed
        // terms: well-formed terms outside the domain; anything else is garbage
        in.dom = etf_known_tag(tag);
        in.err = in.dom ? "term type outside the key domain (pid/port/ref/fun/bitstring)" : "unknown term_to_binary tag";
        return -1;
    }
    in.depth--;
    return cls;
}

// the elements and tail of a LIST_EXT at in.p (tag included); a tail that
// is itself a list continues the same list
inline int sk_list_rest(Etf &in, std::vector<uint8_t> &o, bool exact) {
    for (;;) {
        if (!in.need(5)) return -1;
        const uint32_t tag = in.u8();
        if (tag != 108) { in.err = "internal: expected LIST_EXT"; return -1; }
        const uint32_t n = in.u32();
        for (uint32_t i = 0; i < n; i++)
            if (sk_term(in, o, false, exact, nullptr, nullptr, nullptr, nullptr, nullptr) < 0) return -1;
        if (!in.need(1)) return -1;
        const uint32_t t = *in.p;
        if (t == 106) { in.p++; o.push_back(SK_LIST_END); return 0; }
        if (t == 108) continue;
        if (t == 107) {   // a string tail: more small-integer elements, then []
            in.p++;
            if (!in.need(2)) return -1;
            const uint32_t m = in.u16();
            if (!in.need(m)) return -1;
            for (uint32_t i = 0; i < m; i++) {
                const uint64_t u = (uint64_t)in.p[i] ^ 0x8000000000000000ull;
                o.push_back(KEYTAG_INT);
                for (int k = 7; k >= 0; k--) o.push_back((uint8_t)(u >> (8 * k)));
            }
            in.p += m;
            o.push_back(SK_LIST_END);
            return 0;
        }
        // improper tail: compared with the other list's rest as a term
        std::vector<uint8_t> tail;
        const int c = sk_term(in, tail, false, exact, nullptr, nullptr, nullptr, nullptr, nullptr);
        if (c < 0) return -1;
        o.push_back(c == C_BIN ? SK_TAIL_HIGH : SK_TAIL_LOW);
        o.insert(o.end(), tail.begin(), tail.end());
        return 0;
    }
}

// One term at in.p (no version byte) -> its device key record (plain form
// for int64, atom and binary keys); the ETF part of a term record is 131 ++
// the term's bytes.  Returns "" on success or the reason (in.dom: a
// well-formed term outside the key domain, else malformed bytes).
inline std::string record_from_term(Etf &in, std::vector<uint8_t> &rec) {
    const uint8_t *t0 = in.p;
    std::vector<uint8_t> sk;
    bool is64 = false, big = false, bneg = false;
    int64_t iv = 0;
    std::vector<uint8_t> bmag;
    const int cls = sk_term(in, sk, true, false, &is64, &iv, &big, &bmag, &bneg);
    if (cls < 0) return in.err;
    rec.insert(rec.end(), sk.begin(), sk.end());
    if (is64 || cls == C_ATOM || cls == C_BIN) return "";   // the plain domain
    const size_t n = 1 + (size_t)(in.p - t0);
    if (n > 0xFFFE) { in.dom = true; return "term_to_binary key longer than 65534 bytes"; }
    rec.push_back(131);
    rec.insert(rec.end(), t0, in.p);
    uint32_t seg_len = 0xFFFF;
    if (big) {   // ensure_binary(Integer) = <<Key:64>>: the low 64 bits, two's complement
        uint64_t lo = 0;
        const size_t m = bmag.size();
        for (size_t i = m > 8 ? m - 8 : 0; i < m; i++) lo = (lo << 8) | bmag[i];
        if (bneg) lo = 0 - lo;
        for (int i = 7; i >= 0; i--) rec.push_back((uint8_t)(lo >> (8 * i)));
        seg_len = 8;
    }
    rec.push_back((uint8_t)(n & 0xFF));
    rec.push_back((uint8_t)(n >> 8));
    rec.push_back((uint8_t)(seg_len & 0xFF));
    rec.push_back((uint8_t)(seg_len >> 8));
    return "";
}

// term_to_binary(Key) bytes -> device key record.  "" or the reason.
inline std::string record_from_etf(const uint8_t *etf, size_t n, std::vector<uint8_t> &rec) {
    if (n < 2 || etf[0] != 131) return "not a term_to_binary (version 131) encoding";
    if (n > 0xFFFE) return "term_to_binary key longer than 65534 bytes";
    Etf in{etf + 1, etf + n, std::string()};
    std::vector<uint8_t> r;
    const std::string e = record_from_term(in, r);
    if (!e.empty()) return e;
    if (in.p != in.e) return "trailing bytes after the term";
    rec.insert(rec.end(), r.begin(), r.end());
    return "";
}

// A synctree_leveldb segment node, term_to_binary([{Key, Value}]) with
// binary values (synctree_leveldb.erl:111-123, the host half of the
// device restore for the segments its decoder hands over: map keys,
// FLOAT_EXT, nesting deeper than its stack).  Appends the key records and
// values; koff/voff get one end offset per entry.  Key order is the
// caller's to check.
enum SegStatus { SEG_OK = 0, SEG_BAD = 1, SEG_DOM = 2 };
inline int segment_from_etf(const uint8_t *b, size_t n, std::vector<uint8_t> &krec, std::vector<uint64_t> &koff,
                            std::vector<uint8_t> &val, std::vector<uint64_t> &voff) {
    Etf in{b, b + n, std::string()};
    auto other = [](uint32_t tg) { return etf_known_tag(tg) ? SEG_DOM : SEG_BAD; };
    if (!in.need(1) || in.u8() != 131) return SEG_BAD;
    if (in.p < in.e && *in.p == 80) return SEG_DOM;   // compressed
    if (!in.need(1)) return SEG_BAD;
    uint32_t tg = in.u8(), cnt = 0;
    if (tg == 108) {
        if (!in.need(4)) return SEG_BAD;
        cnt = in.u32();
    } else if (tg != 106) return other(tg);
    for (uint32_t j = 0; j < cnt; j++) {
        if (!in.need(1)) return SEG_BAD;
        if ((tg = in.u8()) != 104) return other(tg);
        if (!in.need(1)) return SEG_BAD;
        if (in.u8() != 2) return SEG_DOM;
        in.depth = 0;
        if (!record_from_term(in, krec).empty()) return in.dom ? SEG_DOM : SEG_BAD;
        koff.push_back(krec.size());
        if (!in.need(1)) return SEG_BAD;
        if ((tg = in.u8()) != 109) return other(tg);
        if (!in.need(4)) return SEG_BAD;
        const uint32_t len = in.u32();
        if (!in.need(len)) return SEG_BAD;
        val.insert(val.end(), in.p, in.p + len);
        in.p += len;
        voff.push_back(val.size());
    }
    if (cnt) {
        if (!in.need(1)) return SEG_BAD;
        if (in.u8() != 106) return SEG_DOM;   // an improper list
    }
    return in.p == in.e ? SEG_OK : SEG_BAD;
}

}  // namespace termkey
