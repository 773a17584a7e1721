// small_path.h — the per-key latency path of insert/3 and get/2 (SURVEY §8f
// rank 4; src/synctree.erl:189-227): a batch of at most SB_MAX keys is served
// by ONE workgroup in ONE launch.  The host writes the call's request (keys,
// values, the tree view) into a slot of fine-grained host memory; the kernel
// copies it into LDS and writes self-validating result records straight into
// mapped host memory, which the host spins on: a call costs one launch and no
// stream synchronisation.
//
// Segments changed by small inserts are not merged into the CSR at once: the
// new content of a segment goes to an OVERLAY record (ov.idx[s] -> offset in
// ov.heap, a bump-allocated device heap), and the segment's path is rehashed in
// the slot arrays immediately.  Only the small kernels read through the
// overlay; every other entry point first merges the overlay into the CSR
// (flush_overlay in synctree_hip.hip: one ingest with replace flags), so the
// bulk kernels never see it.
//
// Overlay record at ov.heap + off (16-byte aligned):
//   u32 n, kbytes, vbytes, pad; u32 koff[n+1]; u32 voff[n+1];
//   key records [kbytes]; values [vbytes]
// (key records: the CSR's tag + ensure_binary encoding; values contiguous, so
// a segment's hash input is one byte range, as in the CSR).
#pragma once
#include "st_kernels.h"

#define SB_MAX 16        // keys per small batch
#define SB_KB 512        // key-record bytes per small batch
#define SB_VB 512        // value bytes per small batch (insert)
#define SB_OUT_VB 4096   // value bytes a small get returns
#define SB_SEG_CAP 1024  // entries of one segment a small insert rewrites (larger: bulk path)
#define SB_VERIFY 96     // threads that verify path nodes (SB_MAX keys x 6 levels)
#define SB_GVAL 128      // get: value bytes per key prefetched into LDS (longer: read at the end)

struct SmallIn {
    uint32_t n, op;       // op: 0 = get/2, 1 = insert/3
    uint32_t dbg, seq;    // dbg: phase stamps into SmallOut.stamp (ST_SMALL_STAMPS); seq: the call's
                          // sequence number (never 0), echoed in every result record
    uint32_t koff[SB_MAX + 1];
    uint32_t voff[SB_MAX + 1];
    uint8_t kb[SB_KB];
    uint8_t vb[SB_VB];
};

// Result block (fine-grained host memory).  The GPU's writes to host memory
// are not seen by the host in program order even across a system-scope fence
// (round 2: a call read an earlier call's status words after the later
// sequence word had arrived), so no result depends on the order of two
// stores: every result is ONE self-validating 16-byte record written with a
// single store -- {seq, word, x, check(seq, word, x)} -- and the value bytes
// a get returns are covered by an FNV-1a sum in their key's record.  The host
// spins until the header and every key's record carry this call's seq and a
// valid check (and the value sums match); a record of an earlier call, or a
// torn one, never validates.
//   hdr:    word = retry | new_entries << 1
//   rec[i]: word = status | clevel << 8 | vlen << 16;
//           x = cbucket (corrupted) or the FNV-1a of the value bytes (get, found)
// Host copy of a validated result block (synctree_hip.hip small_collect).
struct SmallRes {
    int32_t status[SB_MAX];
    uint32_t clevel[SB_MAX];
    uint64_t cbucket[SB_MAX];
    uint32_t voff[SB_MAX + 1];   // get: key i's value is vbytes[voff[i] .. voff[i+1])
    uint32_t new_entries;
    bool retry;                  // not served (overlay full, segment too large): the bulk path serves the call
};
#define SMALL_SLOTS 2

struct SmallOut {
    uint4 hdr;
    uint4 rec[SB_MAX];
    uint64_t stamp[16];        // diagnostic phase stamps, in.dbg only, read after a stream sync: [k] wall (100 MHz), [8 + k] shader clock
    uint8_t vbytes[SB_OUT_VB]; // get: key i's value at the sum of the earlier keys' vlen
};

__host__ __device__ __forceinline__ uint32_t small_check(uint32_t seq, uint32_t w, uint32_t x) {
    uint32_t h = seq * 0x9E3779B1u ^ 0x85EBCA77u;
    h = (h ^ w) * 0xC2B2AE3Du;
    h = (h ^ (h >> 15) ^ x) * 0x27D4EB2Fu;
    return (h ^ (h >> 13)) | 1u;   // never 0: a zeroed record does not validate
}
__host__ __device__ __forceinline__ uint32_t fnv1a_step(uint32_t h, uint8_t b) { return (h ^ b) * 16777619u; }
#define FNV1A_INIT 2166136261u

__device__ __forceinline__ void put_rec(uint4 *dst, uint32_t seq, uint32_t w, uint32_t x) {
    *dst = make_uint4(seq, w, x, small_check(seq, w, x));   // one 16-byte store
}
// the key's record after its result words are final; the header last, after
// a barrier and a system-scope release (the host validates each anyway)
__device__ __forceinline__ void key_rec(SmallOut *out, uint32_t i, uint32_t seq, int32_t status, uint32_t clevel,
                                        uint32_t vlen, uint32_t x) {
    put_rec(&out->rec[i], seq, (uint32_t)status | (clevel << 8) | (vlen << 16), x);
}
__device__ __forceinline__ void hdr_rec(SmallOut *out, uint32_t seq, uint32_t retry, uint32_t new_entries) {
    __threadfence_system();
    put_rec(&out->hdr, seq, retry | (new_entries << 1), 0u);
}

struct Overlay {   // device pointers: global memory (ST_GAS, st_kernels.h)
    uint64_t ST_GAS *idx;              // [S], ~0 = segment not in the overlay
    uint8_t ST_GAS *heap;
    unsigned long long ST_GAS *used;   // bump pointer (device)
    uint64_t cap;
};

// One call's whole input, written by the host into a per-tree slot of
// fine-grained host memory before the launch; the kernel's only arguments are
// the slot and result-block pointers (no large by-value argument block).
struct SmallReq {
    DevTree t;
    Overlay ov;
    SmallIn in;
};

// get_segment/2 (synctree.erl:251-253) of one key record (tag + payload)
__device__ __forceinline__ uint64_t record_segment(const uint8_t *p, uint64_t len, uint64_t segmask) {
    uint32_t d[4];
    if (p[0] == KEYTAG_INT && len == 9) {
        uint32_t m[16];
        uint32_t x0 = 0, x1 = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) { x0 |= (uint32_t)p[1 + i] << (8 * i); x1 |= (uint32_t)p[5 + i] << (8 * i); }
        m[0] = x0 ^ 0x80u;   // unflip the sign bit: message = <<Key:64/big>>
        m[1] = x1;
        m[2] = 0x80u;
#pragma unroll
        for (int w = 3; w < 16; w++) m[w] = 0u;
        m[14] = 64u;
        stmd5::init(d);
        stmd5::compress_lat(d, m);
    } else {
        const uint8_t *sp;
        uint64_t sl;
        krec_seg_bytes(p, len, &sp, &sl);
        stmd5::md5_global_pf(sp, sl, d);
    }
    const uint64_t lo = ((uint64_t)__builtin_bswap32(d[2]) << 32) | (uint64_t)__builtin_bswap32(d[3]);
    return lo & segmask;
}

// Read-only view of one segment's content: its overlay record if it has one,
// else its CSR range.
struct SegView {
    uint64_t n, e0;
    const uint8_t *kh, *vh;          // key / value byte bases
    const uint64_t *ko64, *vo64;     // CSR: absolute offsets (index e0 + i)
    const uint32_t *ko32, *vo32;     // overlay: relative offsets
    __device__ __forceinline__ uint64_t koff(uint64_t i) const { return ko32 ? ko32[i] : ko64[e0 + i]; }
    __device__ __forceinline__ uint64_t voff(uint64_t i) const { return vo32 ? vo32[i] : vo64[e0 + i]; }
    __device__ __forceinline__ const uint8_t *key(uint64_t i) const { return kh + koff(i); }
    __device__ __forceinline__ uint64_t klen(uint64_t i) const { return koff(i + 1) - koff(i); }
    __device__ __forceinline__ const uint8_t *val(uint64_t i) const { return vh + voff(i); }
    __device__ __forceinline__ uint64_t vlen(uint64_t i) const { return voff(i + 1) - voff(i); }
};

__device__ __forceinline__ SegView seg_view(const DevTree &t, const Overlay &ov, uint64_t s) {
    SegView v;
    const uint64_t o = ov.idx[s];
    if (o != ~0ull) {
        const uint32_t *h = reinterpret_cast<const uint32_t *>(ov.heap + o);
        const uint32_t n = h[0], kb = h[1];
        v.n = n;
        v.e0 = 0;
        v.ko32 = h + 4;
        v.vo32 = h + 4 + (n + 1);
        v.kh = reinterpret_cast<const uint8_t *>(h + 4 + 2 * (n + 1));
        v.vh = v.kh + kb;
        v.ko64 = v.vo64 = nullptr;
    } else {
        v.e0 = t.seg_off[s];
        v.n = t.seg_end[s] - v.e0;
        v.kh = t.kheap;
        v.vh = t.vheap;
        v.ko64 = t.koff;
        v.vo64 = t.voff;
        v.ko32 = v.vo32 = nullptr;
    }
    return v;
}

__device__ __forceinline__ uint64_t ov_record_bytes(uint64_t n, uint64_t kb, uint64_t vb) {
    return (16 + 8 * (n + 1) + kb + vb + 15) & ~15ull;
}

// verify_hash of segment s (synctree.erl:322-340) through the overlay
__device__ __forceinline__ bool verify_segment_ov(const DevTree &t, const Overlay &ov, uint64_t s) {
    const uint32_t L = t.H + 1;
    const uint64_t slot = t.base[L] + s;
    const uint64_t eslot = (L == 1) ? 0 : slot;
    const uint16_t et = t.tag[eslot];
    const uint4 e = t.md5[eslot];   // loaded up front, with the segment's offsets
    const SegView v = seg_view(t, ov, s);
    if (!(et & TAG_PRESENT)) return v.n == 0;
    uint32_t d[4];
    const uint64_t a = v.voff(0);
    stmd5::md5_global_pf(v.vh + a, v.voff(v.n) - a, d);
    return (et == TAG_PRESENT) && e.x == d[0] && e.y == d[1] && e.z == d[2] && e.w == d[3];
}

// lower_bound of key record k among the segment's keys
__device__ __forceinline__ uint64_t seg_lower_bound(const SegView &v, const uint8_t *k, uint64_t kl, bool *eq) {
    uint64_t lo = 0, hi = v.n;
    while (lo < hi) {
        const uint64_t m = (lo + hi) >> 1;
        if (rec_cmp(v.key(m), v.klen(m), k, kl) < 0) lo = m + 1; else hi = m;
    }
    *eq = lo < v.n && rec_cmp(v.key(lo), v.klen(lo), k, kl) == 0;
    return lo;
}

// Dynamic LDS of k_small: SB_VERIFY node-staging regions, then per wave a
// merge plan of SB_SEG_CAP + SB_MAX output entries (source, key length, value
// length).
__host__ __device__ __forceinline__ uint32_t small_lds_bytes(uint32_t W) {
    return SB_VERIFY * lane_region_bytes(W) + 4 * (SB_SEG_CAP + SB_MAX) * 12;
}

// insert/3 of ONE key (the per-key latency case, peer_tree do_insert,
// riak_ensemble_peer_tree.erl:224-234), speculatively: wave 0 verifies the
// root->segment path (get_path, synctree.erl:302-320) while wave 2 prefetches
// the path nodes' child entries, writes the segment's new overlay record
// (orddict:store, :206), hashes it from an LDS copy of its values and hashes
// the new path bottom-up from LDS (update_path, :201-209) -- all without
// touching the tree.  Only if the path verified are the overlay index and
// the path's slot entries committed; a corrupted path commits nothing
// ({corrupted, L, B}, :193-194); the overlay space of the discarded record is
// reclaimed at the next flush.
#define SB_STAMP(k) do { if (in.dbg && threadIdx.x == 0) { out->stamp[k] = __builtin_amdgcn_s_memrealtime(); out->stamp[8 + (k)] = __builtin_amdgcn_s_memtime(); } } while (0)
#define SB_STAMPW(k) do { if (in.dbg && (threadIdx.x & 63) == 0) { out->stamp[k] = __builtin_amdgcn_s_memrealtime(); out->stamp[8 + (k)] = __builtin_amdgcn_s_memtime(); } } while (0)
#define S1_VBUF 4096   // value bytes of a segment hashed from LDS (larger: bulk path)
#define S1_PATH 192    // path child entries (H x W <= 192 for W <= 32, S <= 2^31)
// LDS flags between the waves of the one-key insert (workgroup scope)
__device__ __forceinline__ void lds_flag_set(uint32_t *f) {
    __hip_atomic_store(f, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_flag_wait(uint32_t *f) {
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) __builtin_amdgcn_s_sleep(1);
}
// exclusive prefix sum over the 64 lanes of a wave
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t x) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t v = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) v += y;
    }
    return v - x;
}

#define S1_NEW 0x80000000u
__device__ __forceinline__ void small_insert_one(const DevTree &t, const Overlay &ov, const SmallIn &in, SmallOut *out, uint8_t *dyn,
                                 const uint8_t *kb, const uint8_t *vb, uint64_t s, uint32_t *bad) {
    __shared__ uint64_t s1_off;
    __shared__ uint32_t s1_news, s1_retry, s1_n, s1_kb, s1_vb, s1_plan_ready, s1_pre_ready;
    __shared__ uint4 s1_new[ST_MAXLEV + 2];    // new entry per level (H+1 = the segment)
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t H = t.H, L1 = H + 1, W = t.W;
    // wave 3's plan area of the dynamic LDS: path entries, the value copy, a message region
    uint8_t *area = dyn + SB_VERIFY * lane_region_bytes(W) + 3 * (SB_SEG_CAP + SB_MAX) * 12;
    uint4 *pe = reinterpret_cast<uint4 *>(area);                       // [H][W]
    uint16_t *pt = reinterpret_cast<uint16_t *>(pe + S1_PATH);         // [H][W]
    uint8_t *vbuf = reinterpret_cast<uint8_t *>(pt + S1_PATH);         // S1_VBUF + 64
    uint8_t *regs = vbuf + S1_VBUF + 64;                               // H x lane_region_bytes(W)
    __shared__ uint32_t s1_pre[ST_MAXLEV + 2][4];                      // per level: prefix state
    __shared__ uint32_t s1_p[ST_MAXLEV + 2], s1_len[ST_MAXLEV + 2];     // changed entry's offset, length
    // the merged entry list (source entry or S1_NEW, key / value offsets in the new record)
    uint32_t *plan = reinterpret_cast<uint32_t *>(dyn + SB_VERIFY * lane_region_bytes(W)) + 2 * 3 * (SB_SEG_CAP + SB_MAX);
    uint32_t *pk = plan + (SB_SEG_CAP + SB_MAX), *pv = pk + (SB_SEG_CAP + SB_MAX);
    if (tid == 0) { s1_retry = 0; s1_news = 0; s1_plan_ready = 0; s1_pre_ready = 0; }
    __syncthreads();
    SB_STAMP(1);
    const uint8_t *k = kb + in.koff[0];
    const uint64_t kl = in.koff[1] - in.koff[0];
    const uint32_t vl = in.voff[1] - in.voff[0];
    if (wave == 0) {
        if (lane < L1) {   // path verification, level lane + 1
            const uint32_t l = lane + 1;
            bool good;
            if (l == L1) good = verify_segment_ov(t, ov, s);
            else good = verify_inner_node(t, l, s >> (t.shift * (L1 - l)), dyn + lane * lane_region_bytes(W));
            if (!good) atomicMin(&bad[0], l);
        }
        if (lane == 0 && in.dbg) { out->stamp[2] = __builtin_amdgcn_s_memrealtime(); out->stamp[10] = __builtin_amdgcn_s_memtime(); }
    } else if (wave == 1) {
        // path nodes' child entries (level l node b_l, children base[l+1] +
        // b_l*W + j); lanes 1..H: level `lane`'s node message with the path
        // child's entry as a placeholder, and the MD5 state over the blocks
        // before that entry (they do not depend on the new hashes below it)
        for (uint32_t x = lane; x < H * W; x += 64) {
            const uint32_t l = x / W + 1, j = x % W;
            const uint64_t bl = s >> (t.shift * (L1 - l));
            const uint64_t c = t.base[l + 1] + bl * W + j;
            pe[x] = t.md5[c];
            pt[x] = t.tag[c];
        }
        wave_sync_lds();
        if (lane >= 1 && lane <= H) {
            const uint32_t l = lane;
            const uint32_t j = (uint32_t)((s >> (t.shift * (L1 - (l + 1)))) % W);
            uint8_t *reg = regs + (l - 1) * lane_region_bytes(W);
            MsgWriter mw;
            mw.init(reg);
            uint32_t before = 0;
            for (uint32_t q = 0; q < W; q++) {
                const bool pres = q == j || (pt[(l - 1) * W + q] & TAG_PRESENT);
                if (!pres) continue;
                if (q < j) before++;
                mw.entry(q == j ? (uint32_t)TAG_PRESENT : pt[(l - 1) * W + q], pe[(l - 1) * W + q]);
            }
            const uint32_t len = mw.finish();
            s1_p[l] = 17 * before;
            s1_len[l] = len;
            uint32_t st[4];
            stmd5::md5_lds_prefix(reg, (17 * before) / 64, st);
            s1_pre[l][0] = st[0]; s1_pre[l][1] = st[1]; s1_pre[l][2] = st[2]; s1_pre[l][3] = st[3];
        }
        wave_sync_lds();
        if (lane == 0) lds_flag_set(&s1_pre_ready);
    } else if (wave == 2) {
        // the merged entry list (orddict:store, synctree.erl:206) and the new
        // segment's values in LDS; then the new segment hash and the path
        // bottom-up (update_path, :201-209) on lane 0
        const SegView v = seg_view(t, ov, s);
        const uint64_t n = v.n;
        if (n < 64) {   // a lane per old entry: lower_bound by ballot, offsets by prefix sums
            uint32_t kli = 0, vli = 0;
            int c = 1;
            if (lane < n) {
                kli = (uint32_t)v.klen(lane);
                vli = (uint32_t)v.vlen(lane);
                c = rec_cmp(v.key(lane), kli, k, kl);
            }
            const uint32_t pos = (uint32_t)__popcll(__ballot(lane < n && c < 0));
            const bool eq = __ballot(lane < n && c == 0) != 0;
            const uint32_t out_n = (uint32_t)n + (eq ? 0u : 1u);
            const bool act = lane < out_n;
            const uint32_t src = lane < pos ? lane : (lane == pos ? S1_NEW : (eq ? lane : lane - 1));
            const uint32_t sk = __shfl(kli, (int)(src & 63), 64), sv = __shfl(vli, (int)(src & 63), 64);
            const uint32_t a = !act ? 0u : (src == S1_NEW ? (uint32_t)kl : sk);
            const uint32_t b = !act ? 0u : (src == S1_NEW ? vl : sv);
            const uint32_t pa = wave_excl_sum(a), pb = wave_excl_sum(b);
            const uint32_t ta = __shfl(pa + a, 63, 64), tb = __shfl(pb + b, 63, 64);
            if (act) { plan[lane] = src; pk[lane] = pa; pv[lane] = pb; }
            if (lane == 0) {
                pk[out_n] = ta; pv[out_n] = tb;
                s1_n = out_n; s1_kb = ta; s1_vb = tb;
                s1_news = eq ? 0 : 1;
                if (tb > S1_VBUF) s1_retry = 1;
            }
            if (act && tb <= S1_VBUF) {
                const uint8_t *vs = src == S1_NEW ? vb + in.voff[0] : v.val(src);
                for (uint32_t q = 0; q < b; q++) vbuf[pb + q] = vs[q];
            }
            wave_sync_lds();
        } else {        // larger segments: lane 0 walks the list
            if (lane == 0) {
                bool eq;
                const uint64_t pos = seg_lower_bound(v, k, kl, &eq);
                uint64_t out_n = 0, kbytes = 0, vbytes = 0;
                bool fits = n + 1 <= SB_SEG_CAP;
                for (uint64_t x = 0; x < n + 1 && fits; x++) {
                    uint32_t src, a, b;
                    if (x < pos) { src = (uint32_t)x; a = (uint32_t)v.klen(x); b = (uint32_t)v.vlen(x); }
                    else if (x == pos) { src = S1_NEW; a = (uint32_t)kl; b = vl; }
                    else {
                        const uint64_t y = eq ? x : x - 1;
                        if (y >= n) break;
                        src = (uint32_t)y; a = (uint32_t)v.klen(y); b = (uint32_t)v.vlen(y);
                    }
                    plan[out_n] = src; pk[out_n] = (uint32_t)kbytes; pv[out_n] = (uint32_t)vbytes;
                    kbytes += a; vbytes += b; out_n++;
                }
                pk[out_n] = (uint32_t)kbytes; pv[out_n] = (uint32_t)vbytes;
                s1_n = (uint32_t)out_n; s1_kb = (uint32_t)kbytes; s1_vb = (uint32_t)vbytes;
                s1_news = eq ? 0 : 1;
                if (!fits || vbytes > S1_VBUF) s1_retry = 1;
            }
            wave_sync_lds();
            if (!s1_retry)
                for (uint32_t q = lane; q < s1_n; q += 64) {
                    const uint32_t src = plan[q];
                    const uint8_t *vs = src == S1_NEW ? vb + in.voff[0] : v.val(src);
                    for (uint32_t b = pv[q]; b < pv[q + 1]; b++) vbuf[b] = vs[b - pv[q]];
                }
            wave_sync_lds();
        }
        if (lane == 0) lds_flag_set(&s1_plan_ready);
        if (lane == 0 && in.dbg) { out->stamp[3] = __builtin_amdgcn_s_memrealtime(); out->stamp[11] = __builtin_amdgcn_s_memtime(); }
        if (!s1_retry && lane == 0) {
            uint32_t d[4];
            stmd5::md5_lds(vbuf, s1_vb, d);   // the new segment hash
            uint4 e = make_uint4(d[0], d[1], d[2], d[3]);
            s1_new[L1] = e;
            lds_flag_wait(&s1_pre_ready);
            for (uint32_t l = H; l >= 1; l--) {   // patch the child's entry, resume each node's MD5
                uint8_t *reg = regs + (l - 1) * lane_region_bytes(W);
                uint8_t *q = reg + s1_p[l];
                q[0] = 0;   // ?H_MD5
                const uint32_t w4[4] = {e.x, e.y, e.z, e.w};
#pragma unroll
                for (int b = 0; b < 16; b++) q[1 + b] = (uint8_t)(w4[b >> 2] >> (8 * (b & 3)));
                stmd5::md5_lds_resume(reg, s1_len[l], s1_p[l] / 64, s1_pre[l], d);
                e = make_uint4(d[0], d[1], d[2], d[3]);
                s1_new[l] = e;
            }
            if (in.dbg) { out->stamp[4] = __builtin_amdgcn_s_memrealtime(); out->stamp[12] = __builtin_amdgcn_s_memtime(); }
        }
    } else {
        // wave 3: the segment's new overlay record (header, offset tables,
        // key and value bytes) while wave 2 hashes; committed only if the
        // path verified
        if (lane == 0) lds_flag_wait(&s1_plan_ready);
        wave_sync_lds();
        if (!s1_retry) {
            const uint32_t m = s1_n, kbn = s1_kb, vbn = s1_vb;
            uint64_t off = 0;
            if (lane == 0) {
                const uint64_t bytes = ov_record_bytes(m, kbn, vbn);
                off = atomicAdd(ov.used, (unsigned long long)bytes);
                if (off + bytes > ov.cap) s1_retry = 1;
                else s1_off = off;
            }
            off = __shfl(off, 0, 64);
            wave_sync_lds();
            if (!s1_retry) {
                uint32_t *h = reinterpret_cast<uint32_t *>(ov.heap + off);
                uint32_t *ko = h + 4, *vo = h + 4 + (m + 1);
                uint8_t *kd = reinterpret_cast<uint8_t *>(h + 4 + 2 * (m + 1));
                uint8_t *vd = kd + kbn;
                if (lane == 0) { h[0] = m; h[1] = kbn; h[2] = vbn; h[3] = 0; }
                const SegView v = seg_view(t, ov, s);
                for (uint32_t q = lane; q <= m; q += 64) {
                    ko[q] = pk[q];
                    vo[q] = pv[q];
                    if (q == m) continue;
                    const uint32_t src = plan[q];
                    const uint8_t *ks = src == S1_NEW ? k : v.key(src);
                    for (uint32_t b = pk[q]; b < pk[q + 1]; b++) kd[b] = ks[b - pk[q]];
                    for (uint32_t b = pv[q]; b < pv[q + 1]; b++) vd[b] = vbuf[b];
                }
            }
        }
    }
    __syncthreads();
    SB_STAMP(5);
    const bool ok = bad[0] == ~0u;
    if (s1_retry) {   // nothing was committed: the host takes the bulk path
        if (tid == 0) hdr_rec(out, in.seq, 1u, 0u);
        return;
    }
    if (ok) {   // commit: the overlay record and the path's entries
        if (tid == 0) ov.idx[s] = s1_off;
        if (tid < L1) {
            const uint32_t l = tid + 1;
            const uint64_t slot = t.base[l] + (s >> (t.shift * (L1 - l)));
            t.md5[slot] = s1_new[l];
            t.tag[slot] = TAG_PRESENT;
            if (l == 1) { t.md5[0] = s1_new[l]; t.tag[0] = TAG_PRESENT; }
        }
    }
    if (tid == 0) {
        if (ok) key_rec(out, 0, in.seq, ST_OK, 0, 0, 0);
        else key_rec(out, 0, in.seq, ST_CORRUPTED, bad[0], 0, (uint32_t)(s >> (t.shift * (L1 - bad[0]))));
    }
    SB_STAMP(6);
    __syncthreads();
    SB_STAMP(7);
    if (tid == 0) hdr_rec(out, in.seq, 0u, ok ? s1_news : 0u);
}

// The small-batch kernel (one workgroup of 256 threads, 4 waves).
//  1. key -> segment (lane per key; key records copied from the kernel
//     arguments into LDS first)
//  2. path verification: thread per (key, level) verifies node (level,
//     bucket) of the key's path against its parent's entry (get_path,
//     synctree.erl:302-320); a key's first failing level is its {corrupted,
//     Level, Bucket}
//  3. get: lane per key: orddict_find in the segment, value bytes to `out`.
//     insert: wave per distinct touched segment: orddict:store of the batch's
//     keys of that segment in batch order (last writer wins) into a new
//     overlay record (sizes and space reserved for every segment first, so a
//     batch that does not fit changes nothing); then the dirty path bottom-up,
//     one thread per distinct node, a barrier per level (update_path,
//     synctree.erl:201-209).
// `out` is mapped pinned host memory: the host reads it after the stream sync.
__device__ __forceinline__ void small_body(const SmallReq *req, SmallOut *out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
    // the request (host memory) into LDS: one round trip, dword per thread
    __shared__ __attribute__((aligned(16))) SmallReq rq;
    static_assert(sizeof(SmallReq) % 4 == 0, "request is copied in dwords");
    const uint32_t ST_GAS *rqw = (const uint32_t ST_GAS *)req;   // global loads (k_small_multi reads req from memory)
    for (uint32_t i = threadIdx.x; i < sizeof(SmallReq) / 4; i += blockDim.x) reinterpret_cast<uint32_t *>(&rq)[i] = rqw[i];
    __syncthreads();
    const DevTree &t = rq.t;
    const Overlay &ov = rq.ov;
    const SmallIn &in = rq.in;
    __shared__ uint8_t kb[SB_KB + 64];
    __shared__ uint8_t vb[SB_VB + 64];
    __shared__ uint64_t seg[SB_MAX];
    __shared__ uint32_t bad[SB_MAX];            // first failing level (~0 = none)
    __shared__ uint32_t grp[SB_MAX];            // key -> group (distinct segment) index
    __shared__ uint32_t keep[SB_MAX];           // insert: last writer of its key (and path verified)
    __shared__ uint64_t gseg[SB_MAX];
    __shared__ uint64_t goff[SB_MAX];           // overlay offset of the group's new record
    __shared__ uint32_t gn[SB_MAX], gkb[SB_MAX], gvb[SB_MAX], gnew[SB_MAX];
    __shared__ uint64_t dnode[SB_MAX];
    __shared__ uint32_t ngrp, nd, retry;
    __shared__ uint32_t vlen_out[SB_MAX + 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t n = in.n, L1 = t.H + 1;
    SB_STAMP(0);
    for (uint32_t i = tid; i < in.koff[n]; i += blockDim.x) kb[i] = in.kb[i];
    for (uint32_t i = tid; in.op == 1 && i < in.voff[n]; i += blockDim.x) vb[i] = in.vb[i];
    if (tid < SB_MAX) { bad[tid] = ~0u; keep[tid] = 0; }
    if (tid == 0) { ngrp = 0; nd = 0; retry = 0; }
    __syncthreads();
    const uint16_t top_tag = t.tag[0];   // issued before the key hash: its latency hides under it
    if (tid < n) seg[tid] = record_segment(kb + in.koff[tid], in.koff[tid + 1] - in.koff[tid], t.S - 1);
    __syncthreads();
    const bool undefined_top = (top_tag & TAG_PRESENT) == 0;
    if (in.op == 0 && undefined_top) {   // get/2: undefined top => notfound (synctree.erl:216-218)
        if (tid < n) key_rec(out, tid, in.seq, ST_NOTFOUND, 0, 0, 0);
        __syncthreads();
        if (tid == 0) hdr_rec(out, in.seq, 0u, 0u);
        return;
    }
    if (in.op == 1 && n == 1) {   // insert/3 of one key: the speculative path below
        small_insert_one(t, ov, in, out, dyn, kb, vb, seg[0], bad);
        return;
    }
    // ---- 2. path verification: thread x = key * L1 + (level - 1); for a
    // get, wave 2 looks the keys up at the same time (the answer is used only
    // if the key's path verified)
    __shared__ const uint8_t *gsrc[SB_MAX];
    __shared__ uint32_t glen[SB_MAX], gfound[SB_MAX];
    // Inner path nodes on threads [0, SB_VERIFY), the segments on wave 3: the
    // segment MD5 (global memory) and the inner-node MD5 (LDS) in one wave
    // would run one after the other, as two branches.
    if (tid < SB_VERIFY) {
        for (uint32_t x = tid; x < n * t.H; x += SB_VERIFY) {
            const uint32_t i = x / t.H, l = x % t.H + 1;
            if (!verify_inner_node(t, l, seg[i] >> (t.shift * (L1 - l)), dyn + tid * lane_region_bytes(t.W)))
                atomicMin(&bad[i], l);
        }
    } else if (tid >= 192) {
        for (uint32_t i = tid - 192; i < n; i += 64)
            if (!verify_segment_ov(t, ov, seg[i])) atomicMin(&bad[i], L1);
    }
    __shared__ uint8_t gval[SB_MAX][SB_GVAL];   // values found, prefetched while the paths verify
    if (in.op == 0 && tid >= 128 && tid < 128 + n) {   // orddict_find (synctree.erl:342-348)
        const uint32_t i = tid - 128;
        const SegView v = seg_view(t, ov, seg[i]);
        bool eq;
        const uint64_t at = seg_lower_bound(v, kb + in.koff[i], in.koff[i + 1] - in.koff[i], &eq);
        const uint32_t len = eq ? (uint32_t)v.vlen(at) : 0;
        const uint8_t *src = eq ? v.val(at) : nullptr;
        gfound[i] = eq ? 1 : 0;
        glen[i] = len;
        gsrc[i] = src;
        if (len <= SB_GVAL)
            for (uint32_t b = 0; b < len; b++) gval[i][b] = src[b];
    }
    __syncthreads();
    SB_STAMP(2);
    // each key's verification and lookup results, read ONCE into its thread's
    // registers right after they are complete; the result words below come
    // from these copies (an intermittent failure showed a key's LDS word
    // changing between the barrier above and the status write)
    uint32_t my_bad = ~0u, my_found = 0, my_len = 0;
    uint64_t my_seg = 0;
    const uint8_t *my_src = nullptr;
    if (tid < n) {
        my_bad = bad[tid];
        my_seg = seg[tid];
        if (in.op == 0) { my_found = gfound[tid]; my_len = glen[tid]; my_src = gsrc[tid]; }
    }
    if (in.op == 0) {
        // ---- 3 (get): the verified answers
        uint32_t len = 0;
        const uint8_t *src = nullptr;
        if (tid < n) {
            if (my_bad == ~0u && my_found) {
                len = my_len;
                src = my_src;
            }
            vlen_out[tid + 1] = len;
        }
        __syncthreads();
        if (tid == 0) {
            vlen_out[0] = 0;
            for (uint32_t i = 1; i <= n; i++) vlen_out[i] += vlen_out[i - 1];
            retry = vlen_out[n] > SB_OUT_VB;
        }
        __syncthreads();
        if (tid < n && !retry) {   // this key's value bytes, then its record (with their FNV-1a)
            uint32_t h = FNV1A_INIT;
            if (src && len <= SB_GVAL) src = gval[tid];   // the LDS copy
            if (src)
                for (uint32_t b = 0; b < len; b++) {
                    const uint8_t c = src[b];
                    out->vbytes[vlen_out[tid] + b] = c;
                    h = fnv1a_step(h, c);
                }
            if (my_bad != ~0u)
                key_rec(out, tid, in.seq, ST_CORRUPTED, my_bad, 0, (uint32_t)(my_seg >> (t.shift * (L1 - my_bad))));
            else
                key_rec(out, tid, in.seq, my_found ? ST_OK : ST_NOTFOUND, 0, len, my_found ? h : 0u);
        }
        SB_STAMP(6);
        __syncthreads();
        SB_STAMP(7);
        if (tid == 0) hdr_rec(out, in.seq, retry, 0u);
        return;
    }
    // ---- 3 (insert): groups = distinct verified segments, last writer per key
    if (tid == 0) {
        for (uint32_t i = 0; i < n; i++) {
            if (bad[i] != ~0u) continue;
            uint32_t g = 0;
            while (g < ngrp && gseg[g] != seg[i]) g++;
            if (g == ngrp) { gseg[g] = seg[i]; ngrp++; }
            grp[i] = g;
            keep[i] = 1;
            for (uint32_t j = i + 1; j < n; j++)   // a later write of the same key wins
                if (seg[j] == seg[i] && rec_cmp(kb + in.koff[i], in.koff[i + 1] - in.koff[i], kb + in.koff[j],
                                                in.koff[j + 1] - in.koff[j]) == 0) { keep[i] = 0; break; }
        }
    }
    __syncthreads();
    // sizes of every group's new record, space reserved before anything is
    // written (pass 0); then every record written (pass 1).  The merge plan of
    // a group (its output entries' sources and lengths) is rebuilt in each
    // pass by the group's wave (lane 0): a wave's plan area holds one group.
    uint32_t *plan = reinterpret_cast<uint32_t *>(dyn + SB_VERIFY * lane_region_bytes(t.W)) + wave * 3 * (SB_SEG_CAP + SB_MAX);
    uint32_t *pk = plan + (SB_SEG_CAP + SB_MAX), *pv = pk + (SB_SEG_CAP + SB_MAX);
    for (int pass = 0; pass < 2; pass++) {
        for (uint32_t g = wave; g < ngrp; g += 4) {
            const SegView v = seg_view(t, ov, gseg[g]);
            if (lane == 0) {
                // batch keys of the group in key order (<= SB_MAX, insertion sort)
                uint32_t m = 0, idx[SB_MAX];
                for (uint32_t i = 0; i < n; i++)
                    if (keep[i] && grp[i] == g) {
                        uint32_t q = m++;
                        while (q > 0 && rec_cmp(kb + in.koff[idx[q - 1]], in.koff[idx[q - 1] + 1] - in.koff[idx[q - 1]],
                                                kb + in.koff[i], in.koff[i + 1] - in.koff[i]) > 0) {
                            idx[q] = idx[q - 1];
                            q--;
                        }
                        idx[q] = i;
                    }
                // merged order: old entries and batch keys (bit 31), equal keys replaced
                uint64_t x = 0, out_n = 0, kbytes = 0, vbytes = 0, news = 0;
                bool fits = true;
                auto emit = [&](uint32_t src, uint32_t kl, uint32_t vl) {
                    if (out_n >= SB_SEG_CAP) { fits = false; return; }
                    plan[out_n] = src;
                    pk[out_n] = kl;
                    pv[out_n] = vl;
                    kbytes += kl;
                    vbytes += vl;
                    out_n++;
                };
                for (uint32_t r = 0; r < m && fits; r++) {
                    const uint32_t i = idx[r];
                    const uint8_t *k = kb + in.koff[i];
                    const uint64_t kl = in.koff[i + 1] - in.koff[i];
                    bool eq;
                    const uint64_t pos = seg_lower_bound(v, k, kl, &eq);
                    for (; x < pos && fits; x++) emit((uint32_t)x, (uint32_t)v.klen(x), (uint32_t)v.vlen(x));
                    emit(0x80000000u | i, (uint32_t)kl, in.voff[i + 1] - in.voff[i]);
                    if (eq) x++;
                    else news++;
                }
                for (; x < v.n && fits; x++) emit((uint32_t)x, (uint32_t)v.klen(x), (uint32_t)v.vlen(x));
                if (pass == 0) {
                    if (!fits) {
                        atomicOr(&retry, 1u);
                    } else {
                        const uint64_t bytes = ov_record_bytes(out_n, kbytes, vbytes);
                        const uint64_t off = atomicAdd(ov.used, (unsigned long long)bytes);
                        if (off + bytes > ov.cap) atomicOr(&retry, 1u);
                        goff[g] = off;
                        gn[g] = (uint32_t)out_n;
                        gkb[g] = (uint32_t)kbytes;
                        gvb[g] = (uint32_t)vbytes;
                        gnew[g] = (uint32_t)news;
                    }
                } else {   // header and offset tables; lengths -> offsets in LDS too
                    uint32_t *h = reinterpret_cast<uint32_t *>(ov.heap + goff[g]);
                    const uint32_t mm = gn[g];
                    uint32_t *ko = h + 4, *vo = h + 4 + (mm + 1);
                    h[0] = mm; h[1] = gkb[g]; h[2] = gvb[g]; h[3] = 0;
                    uint32_t a = 0, c = 0;
                    for (uint32_t q = 0; q < mm; q++) {
                        const uint32_t kq = pk[q], vq = pv[q];
                        ko[q] = a; vo[q] = c; pk[q] = a; pv[q] = c;
                        a += kq; c += vq;
                    }
                    ko[mm] = a; vo[mm] = c; pk[mm] = a; pv[mm] = c;
                }
            }
            if (pass == 1) {   // entry bytes, lane per entry; offsets from the LDS plan (never read
                               // back from the record just written: no global read-after-write)
                wave_sync_lds();
                uint32_t *h = reinterpret_cast<uint32_t *>(ov.heap + goff[g]);
                const uint32_t mm = gn[g];
                uint8_t *kd = reinterpret_cast<uint8_t *>(h + 4 + 2 * (mm + 1));
                uint8_t *vd = kd + gkb[g];
                for (uint32_t q = lane; q < mm; q += 64) {
                    const uint32_t src = plan[q];
                    const uint8_t *ks, *vs;
                    if (src & 0x80000000u) {
                        const uint32_t i = src & 0x7fffffffu;
                        ks = kb + in.koff[i];
                        vs = vb + in.voff[i];
                    } else {
                        ks = v.key(src);
                        vs = v.val(src);
                    }
                    const uint32_t k0 = pk[q], kn = pk[q + 1] - k0, v0 = pv[q], vn = pv[q + 1] - v0;
                    for (uint32_t b = 0; b < kn; b++) kd[k0 + b] = ks[b];
                    for (uint32_t b = 0; b < vn; b++) vd[v0 + b] = vs[b];
                }
                wave_sync_lds();
            }
        }
        __syncthreads();
        if (pass == 0 && retry) {   // nothing was written: the host takes the bulk path
            if (tid == 0) hdr_rec(out, in.seq, 1u, 0u);
            return;
        }
    }
    // Global data written by other threads of this workgroup is read back
    // below (the new records, then each level's new entries): an agent-scope
    // release/acquire around each barrier also drops this CU's L1 lines, so
    // no read is served from a line cached before the write.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    // the new records replace the segments' content; rehash the dirty paths
    if (tid < ngrp) ov.idx[gseg[tid]] = goff[tid];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (tid < ngrp) {   // level H+1: the segment entries
        const uint64_t s = gseg[tid], slot = t.base[L1] + s;
        const SegView v = seg_view(t, ov, s);
        uint32_t d[4];
        const uint64_t a = v.voff(0);
        stmd5::md5_global_pf(v.vh + a, v.voff(v.n) - a, d);
        const uint4 e = make_uint4(d[0], d[1], d[2], d[3]);
        t.md5[slot] = e;
        t.tag[slot] = TAG_PRESENT;
        if (L1 == 1) { t.md5[0] = e; t.tag[0] = TAG_PRESENT; }
    }
    for (uint32_t l = L1 - 1; l >= 1; l--) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (tid == 0) {
            uint32_t c = 0;
            for (uint32_t g = 0; g < ngrp; g++) {
                const uint64_t b = gseg[g] >> (t.shift * (L1 - l));
                uint32_t q = 0;
                while (q < c && dnode[q] != b) q++;
                if (q == c) dnode[c++] = b;
            }
            nd = c;
        }
        __syncthreads();
        if (tid < nd) {
            const uint64_t b = dnode[tid], slot = t.base[l] + b;
            uint8_t *reg = dyn + tid * lane_region_bytes(t.W);
            const uint32_t len = stage_inner(t, l, b, reg);
            uint32_t d[4];
            stmd5::md5_lds(reg, len, d);   // an insert never empties a node: len > 0
            const uint4 e = make_uint4(d[0], d[1], d[2], d[3]);
            t.md5[slot] = e;
            t.tag[slot] = TAG_PRESENT;
            if (l == 1) { t.md5[0] = e; t.tag[0] = TAG_PRESENT; }
        }
    }
    __syncthreads();
    if (tid < n) {
        if (my_bad != ~0u)
            key_rec(out, tid, in.seq, ST_CORRUPTED, my_bad, 0, (uint32_t)(my_seg >> (t.shift * (L1 - my_bad))));
        else
            key_rec(out, tid, in.seq, ST_OK, 0, 0, 0);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t c = 0;
        for (uint32_t g = 0; g < ngrp; g++) c += gnew[g];
        hdr_rec(out, in.seq, 0u, c);
    }
}

// Overlay flush, step 1: per segment, the number of overlay entries and
// their key / value bytes (0 for segments without an overlay record).
__global__ void k_ov_sizes(Overlay ov, uint64_t S, uint64_t *cnt, uint64_t *kbytes, uint64_t *vbytes, uint8_t *rep) {
    for (uint64_t s = gtid(); s <= S; s += gstride()) {
        if (s == S) { cnt[s] = kbytes[s] = vbytes[s] = 0; break; }
        const uint64_t o = ov.idx[s];
        if (o == ~0ull) { cnt[s] = kbytes[s] = vbytes[s] = 0; rep[s] = 0; continue; }
        const uint32_t *h = reinterpret_cast<const uint32_t *>(ov.heap + o);
        cnt[s] = h[0];
        kbytes[s] = h[1];
        vbytes[s] = h[2];
        rep[s] = 1;
    }
}

// Diagnostic (ST_OV_CHECK & 256): overlay index entries whose record is not
// a plausible one (offset at or past the fill level, or an empty record):
// a[0] count, a[1] lowest segment, a[2] highest segment, a[3] one offset.
__global__ void k_ov_audit(Overlay ov, uint64_t S, unsigned long long *a) {
    const unsigned long long used = *ov.used;
    for (uint64_t s = gtid(); s < S; s += gstride()) {
        const uint64_t o = ov.idx[s];
        if (o == ~0ull) continue;
        const bool bad = o >= used || reinterpret_cast<const uint32_t *>(ov.heap + o)[0] == 0;
        if (!bad) continue;
        atomicAdd(&a[0], 1ull);
        atomicMin(&a[1], (unsigned long long)s);
        atomicMax(&a[2], (unsigned long long)s);
        a[3] = o;
    }
}

// Overlay flush, step 2: the overlay entries as one ingest batch (segment
// order), with their segment ids (seg_given).
__global__ void k_ov_gather(Overlay ov, uint64_t S, const uint64_t *eoff, const uint64_t *koff0, const uint64_t *voff0,
                            uint8_t *krec, uint64_t *koff, uint8_t *vheap, uint64_t *voff, uint32_t *segs) {
    for (uint64_t s = gtid(); s < S; s += gstride()) {
        const uint64_t o = ov.idx[s];
        if (o == ~0ull) continue;
        const uint32_t *h = reinterpret_cast<const uint32_t *>(ov.heap + o);
        const uint32_t n = h[0], kbn = h[1];
        const uint32_t *ko = h + 4, *vo = h + 4 + (n + 1);
        const uint8_t *kd = reinterpret_cast<const uint8_t *>(h + 4 + 2 * (n + 1)), *vd = kd + kbn;
        const uint64_t e = eoff[s];
        for (uint32_t i = 0; i < n; i++) {
            koff[e + i] = koff0[s] + ko[i];
            voff[e + i] = voff0[s] + vo[i];
            segs[e + i] = (uint32_t)s;
        }
        copy_bytes(krec + koff0[s], kd, kbn);
        copy_bytes(vheap + voff0[s], vd, h[2]);
    }
}

__global__ void k_ov_terminate(uint64_t n, const uint64_t *ktot, const uint64_t *vtot, uint64_t *koff, uint64_t *voff) {
    if (gtid() == 0) { koff[n] = *ktot; voff[n] = *vtot; }
}

// After corrupt/2 (synctree.erl:241-247): if the key's segment is now empty
// the backend holds [] for it (erec).  One thread.
__global__ void k_erec_emptied(DevTree t, const uint8_t *krec, const uint64_t *koff, uint8_t *erec) {
    if (threadIdx.x != 0) return;
    const uint64_t s = record_segment(krec + koff[0], koff[1] - koff[0], t.S - 1);
    if (t.seg_off[s] == t.seg_end[s]) erec[t.base[t.H + 1] + s] = 1;
}

__global__ void __launch_bounds__(256) k_small(const SmallReq *req, SmallOut *out) { small_body(req, out); }

// Many trees' per-key batches in ONE launch (st_insert1_multi / st_get1_multi):
// workgroup b serves items[b], one tree's batch of <= SB_MAX keys (its own
// request slot and result block; no two items of a launch share a tree).
struct SmallItem {
    const SmallReq *req;
    SmallOut *out;
};
__global__ void __launch_bounds__(256) k_small_multi(const SmallItem *items) {
    const SmallItem it = items[blockIdx.x];
    small_body(it.req, it.out);
}
