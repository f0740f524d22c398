// mrgpu_map.hip — Map-side kernels other than the wc pipeline (mrgpu_wc.hip):
//
// grep (MapReduce/mrapps/dgrep.go:18-36): streaming literal search (exact
//   per-byte SWAR first-byte filter, LDS verify); each hit's line (strings.Split
//   on "\n") is resolved and inserted, deduplicated by content, into the LongTable.
// wc words longer than 16 bytes (wc_long_kernel): decoded forward from their
//   start, counted in the LongTable.
// collect: the HBM tables' distinct keys -> records with partition =
//   ihash(key) % nReduce (mr/worker.go:33-37,76), appended at ctr->nrec.
#include <climits>

#include "mrgpu_device.h"

namespace mrg {

// Words longer than 16 bytes (wc.go:21-34 for the words the map kernel's 16-byte
// keys cannot hold): one lane per occurrence decodes the word forward from its
// start (Go acceptance ranges, IsLetter from LDS tables) and hashes its bytes
// (FNV-1a-64).  Occurrences are then counted in a per-workgroup LDS table keyed
// by the hash and confirmed by a bytewise compare against the slot's first
// occurrence, so the HBM LongTable sees one insert per (workgroup, distinct
// word) instead of one per occurrence: a Zipf-hot long word otherwise serializes
// on its slot's atomics (mixed-script text has many words over 16 bytes: C2u's
// 31 M occurrences took 136 ms that way).  Lost claim races and a full table
// fall back to a direct HBM insert (exact either way).
constexpr int kLongWG = 1024;    // one workgroup per CU
constexpr int kLongSlots = 4096;  // 96 KB of LDS table
constexpr unsigned long long kRepUnpub = ~0ull;
struct alignas(16) LongLds {
    unsigned long long h[kLongSlots];    // hash | 1 (0: empty)
    unsigned long long rep[kLongSlots];  // input offset of the slot's first occurrence (kRepUnpub until published)
    uint32_t len[kLongSlots];
    uint32_t cnt[kLongSlots];
    uint32_t l2[kLetterUnique * 8];
    uint8_t l1[kLetterLdsPages];
};

// Byte j (0..31) of a 32-byte register window (two 16-byte blocks).
__device__ __forceinline__ uint32_t win_byte(const uint4& a, const uint4& b, uint32_t j) {
    const uint32_t d = j >> 2;
    const uint32_t w = d == 0 ? a.x : d == 1 ? a.y : d == 2 ? a.z : d == 3 ? a.w : d == 4 ? b.x : d == 5 ? b.y : d == 6 ? b.z : b.w;
    return (w >> (8 * (j & 3))) & 0xFFu;
}
__device__ __forceinline__ uint4 ld16_bounded(const uint8_t* in, uint64_t n, uint64_t at) {  // at: 16-byte aligned
    if (at + 16 <= n) return *(const uint4*)(in + at);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < 16; k++)
        if (at + k < n) w[k >> 2] |= (uint32_t)in[at + k] << (8 * (k & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ void __launch_bounds__(kLongWG) wc_long_kernel(const uint8_t* __restrict__ in, uint64_t n, Tables t,
                                                          LetterTables lt, uint64_t nlist) {
    __shared__ LongLds A;
    if (nlist == ~0ull) {  // the map's list length, read here (workgroup-uniform)
        const uint64_t m = t.ctr->nlist;
        nlist = m < t.list_cap ? m : t.list_cap;
        if (nlist == 0) return;
    }
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLongSlots; i += kLongWG) {
        A.h[i] = 0;
        A.rep[i] = kRepUnpub;
        A.cnt[i] = 0;
    }
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLetterUnique * 8; i += kLongWG) A.l2[i] = lt.l2[i];
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLetterLdsPages; i += kLongWG) A.l1[i] = lt.l1[i];
    __syncthreads();
    const LdsLetters L{(const lds_u8*)A.l1, (const lds_u32*)A.l2, nullptr};
    // this workgroup's contiguous share of the list
    const uint64_t per = (nlist + gridDim.x - 1) / gridDim.x;
    const uint64_t b = (uint64_t)blockIdx.x * per, e = b + per < nlist ? b + per : nlist;
    for (uint64_t i = b + threadIdx.x; i < e; i += kLongWG) {
        const uint64_t s = t.list[i];
        if (s == kListHole) continue;  // the unused rest of a map wave's reserved range
        // decode forward through a 32-byte register window of aligned 16-byte
        // loads (the next block requested a block ahead), not a chain of byte loads
        uint64_t wb = s & ~15ull;
        uint4 w0 = ld16_bounded(in, n, wb), w1 = ld16_bounded(in, n, wb + 16);
        uint64_t q = s, h = kFnv64Off;
        while (q < n) {
            if (q - wb >= 16) {  // slide: the rune at q and its 3 successors stay inside the window
                wb += 16;
                w0 = w1;
                w1 = ld16_bounded(in, n, wb + 16);
            }
            const uint32_t j = (uint32_t)(q - wb);
            const uint32_t c0 = win_byte(w0, w1, j);
            uint32_t vl = 1;
            bool let;
            if (c0 < 0x80u) {
                let = ((c0 | 0x20u) - 0x61u) < 26u;
                if (let) h = fnv1a64_step(h, c0);
            } else {
                const uint32_t c1 = q + 1 < n ? win_byte(w0, w1, j + 1) : 0, c2 = q + 2 < n ? win_byte(w0, w1, j + 2) : 0,
                               c3 = q + 3 < n ? win_byte(w0, w1, j + 3) : 0;
                vl = (uint32_t)utf8_valid_len(c0, c1, c2, c3);
                let = vl != 0 && is_letter_lds(utf8_decode(c0, c1, c2, c3, (int)vl), L);
                if (let) {
                    h = fnv1a64_step(h, c0);
                    if (vl > 1) h = fnv1a64_step(h, c1);
                    if (vl > 2) h = fnv1a64_step(h, c2);
                    if (vl > 3) h = fnv1a64_step(h, c3);
                }
            }
            if (!let) break;
            q += vl;
        }
        const uint32_t len = (uint32_t)(q - s);
        const unsigned long long hk = h | 1ull;
        bool done = false;
        uint32_t slot = (uint32_t)(hk >> 20) & (kLongSlots - 1);
        for (int probe = 0; probe < 16 && !done; probe++, slot = (slot + 1) & (kLongSlots - 1)) {
            unsigned long long cur = __hip_atomic_load(&A.h[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (cur == 0) {
                cur = atomicCAS(&A.h[slot], 0ull, hk);
                if (cur == 0) {  // claimed: publish the representative, then count
                    A.len[slot] = len;
                    __hip_atomic_store(&A.rep[slot], (unsigned long long)s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    atomicAdd(&A.cnt[slot], 1u);
                    done = true;
                    break;
                }
            }
            if (cur == hk) {
                const unsigned long long r = __hip_atomic_load(&A.rep[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (r == kRepUnpub) break;  // being published: never wait here, insert directly
                if (A.len[slot] == len && (r == s || bytes_equal(in + r, in + s, len))) {
                    atomicAdd(&A.cnt[slot], 1u);
                    done = true;
                }
            }
        }
        if (!done) long_insert(t, h, in + s, len, 1);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLongSlots; i += kLongWG) {
        const uint32_t c = A.cnt[i];
        if (c) long_insert(t, A.h[i], in + A.rep[i], A.len[i], c);
    }
}

// Words of 17-32 bytes handed over by the map kernel as 32-byte zero-padded key
// records (the map read them from its LDS window; no decode of the input here),
// in one region per map wave.  They are counted by hash bucket, so that every
// occurrence of a key meets ONE workgroup's LDS table and the HBM LongTable sees
// one insert per distinct key (round 4 counted them per map workgroup: a
// workgroup of C2u saw ~40 K distinct words, its 4096-slot table overflowed,
// and ~4 M records plus ~1 M table entries per split went to the LongTable by
// CAS, 3.2 ms):
//   1. lrec_hist_kernel: per map workgroup, its records per bucket (LDS
//      histogram, bucket = 8 bits of a fold of the record's words), and each
//      record's bucket as a byte (the scatter reads 1 byte, not 32, per record);
//   2. lrec_scan_kernel: bucket-major exclusive offsets over (bucket, workgroup);
//   3. lrec_scatter_kernel: each record's index at its bucket's next position;
//   4. wc_lrec_kernel: one workgroup per range of the bucket-ordered records
//      counts them in an LDS table (slot from a cheap mix of the 32 bytes,
//      confirmed by comparing the two records' 32 bytes: equal zero-padded
//      records <=> equal keys, letters are never 0x00) and writes each distinct
//      key once as a partial with its FNV-1a-64 (the hash wc_long_kernel and
//      the LongTable use, so a word that reached the table by either path meets
//      itself there); its representative is the record itself (the collect
//      copies the key bytes from it).  Exact: a full table inserts the record
//      directly;
//   5. lrec_merge_kernel: one workgroup per bucket merges the partials of the
//      ranges the bucket spans and inserts each distinct key once.
constexpr uint32_t kLrecBuckets = 256;
#ifndef MRG_LREC_SLOTS
#define MRG_LREC_SLOTS 1024
#endif
constexpr int kLrecSlots = MRG_LREC_SLOTS;
struct alignas(16) LrecLds {
    unsigned long long h[kLrecSlots];    // hash | 1 (0: not yet written)
    unsigned long long rep[kLrecSlots];  // address of the slot's first record (0: empty; the claim)
    uint32_t len[kLrecSlots];
    uint32_t cnt[kLrecSlots];
    u32x4 key[kLrecSlots][2];            // the representative's 32 bytes (valid once h is written)
};

__device__ __forceinline__ uint32_t lrec_bucket(const uint4& a, const uint4& b) {
    return fold32(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w) >> 24;
}

// One LDS add for the lanes sharing the first active lane's bucket
// (a Zipf-hot long word puts most of a workgroup's records in one bucket: one
// same-address atomic per lane serialized), one per lane for the rest.
// Returns each lane's position (the add's old value + its rank among the
// lanes of one add).
__device__ __forceinline__ uint32_t lrec_bucket_add(uint32_t* cnt, uint32_t b, bool active, bool want_pos) {
    const uint64_t act = __ballot(active);
    if (act == 0) return 0;
    const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)b, (int)__builtin_ctzll(act));
    const uint64_t m = __ballot(active && b == b0);
    uint32_t base = 0;
    if (active && mbcnt64(m) == 0 && b == b0) base = atomicAdd(&cnt[b0], (uint32_t)__popcll(m));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)__builtin_ctzll(m));
    uint32_t pos = base + mbcnt64(m);
    if (active && b != b0) pos = want_pos ? atomicAdd(&cnt[b], 1u) : (atomicAdd(&cnt[b], 1u), 0u);
    return pos;
}

__global__ void __launch_bounds__(kLongWG) lrec_hist_kernel(Tables t, uint32_t nwg) {
    __shared__ uint32_t hist[kLrecBuckets];
    const uint32_t g = blockIdx.x, cap = t.lrec_cap;
    for (uint32_t b = threadIdx.x; b < kLrecBuckets; b += kLongWG) hist[b] = 0;
    __syncthreads();
    for (int r = 0; r < kWavesPerWG; r++) {
        const uint4* recs = t.lrec + ((uint64_t)g * kWavesPerWG + r) * cap * 2;
        const uint32_t nr = min(t.lrec_cnt[g * kWavesPerWG + r], cap);
        for (uint32_t i0 = 0; i0 < nr; i0 += kLongWG) {  // (workgroup-uniform trip count: whole waves in the adds)
            const uint32_t i = i0 + threadIdx.x;
            const bool act = i < nr;
            const uint32_t b = act ? lrec_bucket(recs[2 * i], recs[2 * i + 1]) : 0u;
            if (act) t.lrec_bkt[((uint64_t)g * kWavesPerWG + r) * cap + i] = (uint8_t)b;
            lrec_bucket_add(hist, b, act, false);
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < kLrecBuckets; b += kLongWG) t.lrec_off[(uint64_t)b * nwg + g] = hist[b];
}

// Exclusive scan of the kLrecBuckets x nwg counts in place (one workgroup,
// a multiple of 4 entries per thread read as uint4), the total at
// [kLrecBuckets * nwg].
__global__ void __launch_bounds__(1024) lrec_scan_kernel(uint32_t* off, uint32_t nwg, const uint32_t* wave_cnt) {
    __shared__ uint32_t part[1024];
    const uint32_t E = kLrecBuckets * nwg, tid = threadIdx.x;
    // no records at all (every ASCII split of short words): the counts are all
    // zero, so are their exclusive prefixes; only the total is written (the
    // scan over the 256 x nwg counts took ~32 us per C2 step)
    bool any = false;
    for (uint32_t i = tid; i < nwg * kWavesPerWG; i += 1024) any |= wave_cnt[i] != 0;
    if (!__syncthreads_or(any)) {
        if (tid == 0) off[E] = 0;
        return;
    }
    // thread tid owns entries [tid * per, +per), per a multiple of 4 (E = 256 nwg)
    const uint32_t per = ((E + 1023) / 1024 + 3) & ~3u;
    uint4* o4 = (uint4*)off;
    // two passes over the thread's entries (the second reads them from L2): held
    // in registers they spilled to scratch
    uint32_t sum = 0;
    for (uint32_t q = 0; q < per; q += 4) {
        const uint32_t i = tid * per + q;
        if (i < E) {
            const uint4 v = o4[i / 4];
            sum += v.x + v.y + v.z + v.w;
        }
    }
    part[tid] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan of the thread sums
        const uint32_t x = tid >= d ? part[tid - d] : 0u;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    uint32_t run = part[tid] - sum;
    for (uint32_t q = 0; q < per; q += 4) {
        const uint32_t i = tid * per + q;
        if (i < E) {
            const uint4 v = o4[i / 4];
            uint4 e;
            e.x = run; run += v.x;
            e.y = run; run += v.y;
            e.z = run; run += v.z;
            e.w = run; run += v.w;
            o4[i / 4] = e;
        }
    }
    if (tid == 1023) off[E] = part[1023];
}

__global__ void __launch_bounds__(kLongWG) lrec_scatter_kernel(Tables t, uint32_t nwg) {
    __shared__ uint32_t cur[kLrecBuckets];
    const uint32_t g = blockIdx.x, cap = t.lrec_cap;
    for (uint32_t b = threadIdx.x; b < kLrecBuckets; b += kLongWG) cur[b] = t.lrec_off[(uint64_t)b * nwg + g];
    __syncthreads();
    for (int r = 0; r < kWavesPerWG; r++) {
        const uint64_t region = (uint64_t)g * kWavesPerWG + r;
        const uint32_t nr = min(t.lrec_cnt[g * kWavesPerWG + r], cap);
        for (uint32_t i0 = 0; i0 < nr; i0 += kLongWG) {
            const uint32_t i = i0 + threadIdx.x;
            const bool act = i < nr;
            const uint32_t b = act ? t.lrec_bkt[region * cap + i] : 0u;
            const uint32_t pos = lrec_bucket_add(cur, b, act, true);
            if (act) t.lrec_idx[pos] = (uint32_t)(region * cap + i);
        }
    }
}

// FNV-1a-64 and length of a zero-padded 32-byte record's key.
__device__ __forceinline__ uint64_t lrec_fnv(const uint4& a, const uint4& b, uint32_t& len) {
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint64_t h = kFnv64Off;
    len = 0;
    for (int x = 0; x < 32; x++) {
        const uint32_t c = (w[x >> 2] >> (8 * (x & 3))) & 0xFFu;
        if (c == 0) break;
        h = fnv1a64_step(h, c);
        len++;
    }
    return h;
}

// Count `run` occurrences of the key of record me (bytes a, b; FNV-1a-64 h,
// len bytes): the LDS table, or the LongTable directly when 16 probes find no
// room (len 0: h is a table-local hash, not yet the key's FNV-1a-64 and length,
// computed here for that insert).  A slot is claimed by CAS on its representative's address, so the
// claim publishes it (a prober never meets a claimed slot it cannot compare
// with: round 4's hash-first claim sent racing lanes of a hot word to the
// LongTable); the hash, written after the claim, only skips byte compares.
__device__ __forceinline__ void lrec_count(LrecLds& A, const Tables& t, const uint4& a, const uint4& b, uint64_t h,
                                           uint32_t len, unsigned long long me, uint32_t run, uint32_t& direct) {
    const unsigned long long hk = h | 1ull;
    uint32_t slot = (uint32_t)(hk >> 20) & (kLrecSlots - 1);
    for (int probe = 0; probe < 16; probe++, slot = (slot + 1) & (kLrecSlots - 1)) {
        unsigned long long r = __hip_atomic_load(&A.rep[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (r == 0) {
            r = atomicCAS(&A.rep[slot], 0ull, me);
            if (r == 0) {  // claimed (and published): key bytes, length and hash for the others, then count
                A.key[slot][0] = to_v4(a);
                A.key[slot][1] = to_v4(b);
                A.len[slot] = len;
                __hip_atomic_store(&A.h[slot], hk, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                atomicAdd(&A.cnt[slot], run);
                return;
            }
        }
        const unsigned long long hs = __hip_atomic_load(&A.h[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (hs != 0 && hs != hk) continue;  // another key
        uint4 ra, rb;
        if (hs != 0) {  // the bytes from LDS (no global round trip per probe)
            ra = from_v4(A.key[slot][0]);
            rb = from_v4(A.key[slot][1]);
        } else {  // claimed, not yet published: the representative itself
            const uint4* rr = (const uint4*)(uintptr_t)r;
            ra = rr[0];
            rb = rr[1];
        }
        if (ra.x == a.x && ra.y == a.y && ra.z == a.z && ra.w == a.w && rb.x == b.x && rb.y == b.y && rb.z == b.z &&
            rb.w == b.w) {
            atomicAdd(&A.cnt[slot], run);
            return;
        }
    }
    if (len == 0) h = lrec_fnv(a, b, len);
    long_insert(t, h, (const uint8_t*)(uintptr_t)me, len, run);
    direct++;
}

// A cheap 64-bit mix of a record's 32 bytes: the LDS table's slot and compare
// hash (the FNV-1a-64 the LongTable needs is computed once per distinct key
// when the partials are written; per record, its byte loop was the kernel's
// main instruction cost).
__device__ __forceinline__ uint64_t lrec_mix(const uint4& a, const uint4& b) {
    const uint64_t x0 = ((uint64_t)a.y << 32 | a.x) ^ __builtin_rotateleft64((uint64_t)b.y << 32 | b.x, 17);
    const uint64_t x1 = ((uint64_t)a.w << 32 | a.z) ^ __builtin_rotateleft64((uint64_t)b.w << 32 | b.z, 29);
    return short_hash64(x0, x1) * 0x9E3779B97F4A7C15ull;
}

// A key cached in a thread's registers with its count so far.
struct LrecKey {
    uint4 a, b;
    uint64_t h;
    uint32_t run;
    unsigned long long rep;
    __device__ __forceinline__ bool same(const uint4& x, const uint4& y) const {
        return a.x == x.x && a.y == x.y && a.z == x.z && a.w == x.w && b.x == y.x && b.y == y.y && b.z == y.z && b.w == y.w;
    }
};

// The bucket-ordered records in kLrecGrid equal contiguous ranges, one per
// workgroup (a Zipf-hot long word is most of its bucket: ~6 M of C2u's 28 M
// records in one bucket; a range rarely spans more than one bucket, so its
// table holds few distinct keys); each thread walks a contiguous share of the
// range, kLrecBatch records per step with all their loads in flight, and counts
// runs of equal records in registers before the table (the hot word's runs
// are long; it is also kept in a two-key register cache).  A workgroup writes
// its distinct keys with their counts as partials; lrec_merge_kernel then
// merges each bucket's partials (from the ranges its records span) and inserts
// every distinct key into the LongTable ONCE (inserting them from every range
// put ~1000 concurrent inserts of a hot word on one LongTable slot: 1.4 ms).
// (1024 ranges of a 1024-slot table: C2u wc_lrec 0.786 -> 0.751 ms, merge
// unchanged, against 512 x 2048; profiles/ab_r05_lrec_grid.txt)
#ifndef MRG_LREC_GRID
#define MRG_LREC_GRID 1024
#endif
#ifndef MRG_LREC_BATCH
#define MRG_LREC_BATCH 2
#endif
constexpr uint32_t kLrecGrid = MRG_LREC_GRID, kLrecBatch = MRG_LREC_BATCH;
static_assert(kLrecGrid <= 1024 && (uint64_t)kLrecGrid * kLrecSlots <= 512ull * 4096, "the partials buffer (kLrecPartBytes)");
static_assert(sizeof(LrecLds) <= 160 * 1024, "LDS");
__global__ void __launch_bounds__(kLongWG) wc_lrec_kernel(Tables t, uint32_t nwg) {
    __shared__ LrecLds A;
    const uint64_t T = t.lrec_off[(uint64_t)kLrecBuckets * nwg];  // all records
    const uint32_t s0 = (uint32_t)(T * blockIdx.x / kLrecGrid), s1 = (uint32_t)(T * (blockIdx.x + 1) / kLrecGrid);
    if (s0 == s1) {  // (fewer records than ranges: an empty range still says so to lrec_merge_kernel)
        if (threadIdx.x == 0) t.lrec_pcnt[blockIdx.x] = 0;
        return;
    }
    uint32_t direct = 0;
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLrecSlots; i += kLongWG) {
        A.h[i] = 0;
        A.rep[i] = 0;
        A.cnt[i] = 0;
    }
    __syncthreads();
    const uint32_t per = (s1 - s0 + kLongWG - 1) / kLongWG;
    const uint32_t k0 = min(s0 + threadIdx.x * per, s1), k1 = min(k0 + per, s1);
    // two cached keys per thread (the most recent first): a hot word (~half of
    // its bucket's records) stays cached between the other words, so it reaches
    // the LDS counter once per thread, not once per run (its runs average ~2)
    LrecKey c0 = {}, c1 = {};
    for (uint32_t kb = k0; kb < k1; kb += kLrecBatch) {
        uint32_t ix[kLrecBatch];
        uint4 ra[kLrecBatch], rb[kLrecBatch];
#pragma unroll
        for (uint32_t q = 0; q < kLrecBatch; q++) ix[q] = kb + q < k1 ? t.lrec_idx[kb + q] : 0u;
#pragma unroll
        for (uint32_t q = 0; q < kLrecBatch; q++) {
            const uint4* rec = t.lrec + 2ull * ix[q];
            ra[q] = kb + q < k1 ? rec[0] : make_uint4(0, 0, 0, 0);
            rb[q] = kb + q < k1 ? rec[1] : make_uint4(0, 0, 0, 0);
        }
        // (fully unrolled: a runtime trip count indexed ra/rb dynamically and put
        // them in scratch, 288 B per lane)
#pragma unroll
        for (uint32_t q = 0; q < kLrecBatch; q++) {
            const uint4 a = ra[q], b = rb[q];
            if (kb + q >= k1) {
            } else if (c0.run && c0.same(a, b)) {
                c0.run++;
            } else if (c1.run && c1.same(a, b)) {
                const LrecKey x = c1;
                c1 = c0;
                c0 = x;
                c0.run++;
            } else {
                if (c1.run) lrec_count(A, t, c1.a, c1.b, c1.h, 0, c1.rep, c1.run, direct);
                c1 = c0;
                c0.a = a;
                c0.b = b;
                c0.h = lrec_mix(a, b);
                c0.rep = (unsigned long long)(uintptr_t)(t.lrec + 2ull * ix[q]);
                c0.run = 1;
            }
        }
    }
    if (c0.run) lrec_count(A, t, c0.a, c0.b, c0.h, 0, c0.rep, c0.run, direct);
    if (c1.run) lrec_count(A, t, c1.a, c1.b, c1.h, 0, c1.rep, c1.run, direct);
    if (t.dbg) {  // (MRG_DEBUG_TIMES diagnostics: records that missed the LDS table)
        const uint64_t d = wave_sum(direct);
        if ((threadIdx.x & 63) == 0 && d) atomicAdd(&t.ctr->lds_miss, (unsigned long long)d);
    }
    __syncthreads();
    // this range's distinct keys -> partials [range][i], their count at pcount[range]
    LrecPart* part = t.lrec_part + (uint64_t)blockIdx.x * kLrecSlots;
    __shared__ uint32_t np;
    if (threadIdx.x == 0) np = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLrecSlots; i += kLongWG) {
        const uint32_t c = A.cnt[i];
        if (c) {  // the key's FNV-1a-64 and length from its bytes
            const uint4 a = from_v4(A.key[i][0]), b = from_v4(A.key[i][1]);
            uint32_t len;
            const uint64_t h = lrec_fnv(a, b, len);
            const uint32_t o = atomicAdd(&np, 1u);
            part[o] = LrecPart{A.rep[i], h, len, c, lrec_bucket(a, b), 0};
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) t.lrec_pcnt[blockIdx.x] = np;
}

// First record index of range r (wc_lrec_kernel's split of the T records).
__device__ __forceinline__ uint64_t lrec_range_start(uint64_t T, uint32_t r) { return T * r / kLrecGrid; }

// One workgroup per bucket: the partials of every range its records span (a
// wave per range), those of this bucket counted in an LDS table, then one
// LongTable insert per distinct key.
__global__ void __launch_bounds__(kLongWG) lrec_merge_kernel(Tables t, uint32_t nwg) {
    __shared__ LrecLds A;
    const uint32_t bk = blockIdx.x;
    const uint64_t T = t.lrec_off[(uint64_t)kLrecBuckets * nwg];
    const uint64_t bs = t.lrec_off[(uint64_t)bk * nwg], be = t.lrec_off[(uint64_t)(bk + 1) * nwg];
    if (bs == be) return;
    // ranges holding records bs and be - 1
    uint32_t r0 = (uint32_t)min<uint64_t>(bs * kLrecGrid / T, kLrecGrid - 1), r1 = (uint32_t)min<uint64_t>((be - 1) * kLrecGrid / T, kLrecGrid - 1);
    while (r0 + 1 < kLrecGrid && lrec_range_start(T, r0 + 1) <= bs) r0++;
    while (r0 > 0 && lrec_range_start(T, r0) > bs) r0--;
    while (r1 + 1 < kLrecGrid && lrec_range_start(T, r1 + 1) <= be - 1) r1++;
    while (r1 > 0 && lrec_range_start(T, r1) > be - 1) r1--;
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLrecSlots; i += kLongWG) {
        A.h[i] = 0;
        A.rep[i] = 0;
        A.cnt[i] = 0;
    }
    __syncthreads();
    uint32_t direct = 0;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t r = r0 + wv; r <= r1; r += kLongWG / 64) {
        const LrecPart* part = t.lrec_part + (uint64_t)r * kLrecSlots;
        for (uint32_t i = lane, n = t.lrec_pcnt[r]; i < n; i += 64) {
            const LrecPart p = part[i];
            if (p.bucket != bk) continue;
            const uint4* rr = (const uint4*)(uintptr_t)p.rep;
            lrec_count(A, t, rr[0], rr[1], p.h, p.len, p.rep, p.cnt, direct);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < (uint32_t)kLrecSlots; i += kLongWG) {
        const uint32_t c = A.cnt[i];
        if (c) long_insert(t, A.h[i], (const uint8_t*)(uintptr_t)A.rep[i], A.len[i], c);
    }
}

void launch_wc_lrec(const Tables& t, uint32_t nwg, hipStream_t s) {
    if (!t.lrec || !nwg) return;
    lrec_hist_kernel<<<nwg, kLongWG, 0, s>>>(t, nwg);
    lrec_scan_kernel<<<1, 1024, 0, s>>>(t.lrec_off, nwg, t.lrec_cnt);
    lrec_scatter_kernel<<<nwg, kLongWG, 0, s>>>(t, nwg);
    wc_lrec_kernel<<<kLrecGrid, kLongWG, 0, s>>>(t, nwg);
    lrec_merge_kernel<<<kLrecBuckets, kLongWG, 0, s>>>(t, nwg);
}

// ------------------------------------------------------------ grep kernels
// Pattern occurrence search.  Every occurrence start p (with p + plen <= n) is
// appended to the list; grep_resolve_kernel resolves its line.
__device__ __forceinline__ uint32_t eq_mask16(uint4 v, uint32_t rep) {
    // exact per-byte equality with the broadcast byte (no borrow false positives)
    uint32_t m = 0;
    uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t x = ws[k] ^ rep;
        uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // 0x80 where byte == 0
        m |= (((z >> 7) * 0x10204080u) >> 28) << (4 * k);
    }
    return m;
}

// Streaming literal search.  Each wave streams its chunks through a private
// two-slot LDS ring, one buffer_load_dwordx4 ... lds per chunk (64 lanes x 16 B:
// lanes 0-59 the chunk's 960 own bytes, lanes 60-63 a 64-byte look-ahead),
// issued one chunk ahead.  The DMA is inline asm, invisible to hipcc's waitcnt
// pass, and the loop issues no other VMEM instruction on its common path, so the
// wait for a chunk is a counted vmcnt(1) — a compiler-visible load or a global
// pattern read in the loop would make hipcc wait vmcnt(0) and serialize the
// prefetch (measured: 7.0 ms per 10 GB that way).  The pattern sits in LDS.
// Candidates: positions whose next four bytes equal the pattern's first four
// (patterns of 1-3 bytes: the first two, per-byte SWAR compares), verified in
// LDS for patterns of <= 65 bytes (longer
// ones read HBM and drain with vmcnt(0)).  Matches are buffered per wave in LDS
// and flushed to the list with ONE cursor atomic per flush: a same-address
// device atomic per match serializes at the memory side (~12 ns each; C3's
// ~600 K matches cost 7 ms that way, the whole kernel time).
constexpr uint32_t kGrepOwn = 960;  // own bytes per chunk (lanes 0-59)
// LDS ring slots per wave: kGrepSlots - 1 chunk DMAs in flight while one chunk
// is scanned.  3 slots and a 128-entry match buffer keep two workgroups per CU
// (64 KiB of LDS each); C3 map 2.09 -> 2.05 ms against 2 slots and 256 entries,
// 3 slots with 256 entries (one workgroup per CU) 2.31 ms
// (profiles/ab_r05_grep_ring.txt)
#ifndef MRG_GREP_SLOTS
#define MRG_GREP_SLOTS 3
#endif
constexpr uint32_t kGrepSlots = MRG_GREP_SLOTS;
#ifndef MRG_GREP_BUF
#define MRG_GREP_BUF 128
#endif
constexpr uint32_t kGrepBuf = MRG_GREP_BUF;  // buffered matches per wave
// flushed once fewer than this many entries are free (a chunk rarely adds more)
constexpr uint32_t kGrepFlushRoom = kGrepBuf / 2 < 64 ? kGrepBuf / 2 : 64;
typedef int gi32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void grep_dma(const uint8_t* in, uint64_t n, uint64_t cs, uint32_t lane, uint32_t lds_base) {
    // descriptor base = the window start rounded down to 1 GiB: 32-bit offsets
    const uint64_t base = cs & ~((1ull << 30) - 1);
    const uint64_t r = n - base;  // wraps if base >= n
    const uint32_t rhi = (uint32_t)(r >> 32), rlo = (uint32_t)r;
    const uint32_t nrec = (int32_t)rhi < 0 ? 0u : (rhi != 0 || rlo > 0xFFFFFF00u) ? 0xFFFFFF00u : rlo;
    const uint64_t b = (uint64_t)(in + base);
    const gi32x4 rs = {(int)__builtin_amdgcn_readfirstlane((uint32_t)b),
                       (int)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32) & 0xFFFFu),
                       (int)__builtin_amdgcn_readfirstlane(nrec), 0x00020000};
    const uint32_t voff = (uint32_t)(cs - base) + 16u * lane;
    lds_base = __builtin_amdgcn_readfirstlane(lds_base);
    asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs), "s"(lds_base)
                 : "memory", "m0");
}

// grep_dma as a stream: the descriptor (base = the window start rounded down
// to 1 GiB, range = bytes to the split's end) is recomputed only when the
// offset passes 3 GiB; a chunk's DMA is one 32-bit add.
struct GrepStream {
    uint32_t base_lo, base_hi, nrec, voff;
    __device__ __forceinline__ void set(const uint8_t* in, uint64_t n, uint64_t cs) {
        const uint64_t base = cs & ~((1ull << 30) - 1);
        const uint64_t r = n - base;  // wraps if base >= n
        const uint32_t rhi = (uint32_t)(r >> 32), rlo = (uint32_t)r;
        nrec = (int32_t)rhi < 0 ? 0u : (rhi != 0 || rlo > 0xFFFFFF00u) ? 0xFFFFFF00u : rlo;
        const uint64_t b = (uint64_t)(in + base);
        base_lo = (uint32_t)b;
        base_hi = (uint32_t)(b >> 32) & 0xFFFFu;
        voff = (uint32_t)(cs - base);
    }
    __device__ __forceinline__ void issue(uint32_t lane, uint32_t lds_base) const {
        const gi32x4 rs = {(int)__builtin_amdgcn_readfirstlane(base_lo), (int)__builtin_amdgcn_readfirstlane(base_hi),
                           (int)__builtin_amdgcn_readfirstlane(nrec), 0x00020000};
        lds_base = __builtin_amdgcn_readfirstlane(lds_base);
        asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff + 16u * lane), "s"(rs),
                     "s"(lds_base)
                     : "memory", "m0");
    }
};

// Of a chunk's occurrences (lane l: 16-bit masks `hit` and `nl` ('\n') of its
// 16 bytes), keep the first of each line: an occurrence is dropped when an
// earlier one of the chunk has no '\n' between them (the pattern holds no
// '\n').  The last occurrence / newline of the lanes below come from a wave
// prefix max.
__device__ __attribute__((noinline)) uint32_t first_hit_per_line(uint32_t hit, uint32_t nl, uint32_t lane) {
    int lh = hit ? (int)(16 * lane + 31 - __builtin_clz(hit)) : -1;
    int ln = nl ? (int)(16 * lane + 31 - __builtin_clz(nl)) : -1;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {  // inclusive prefix max
        const int a = __shfl_up(lh, off), b = __shfl_up(ln, off);
        if (lane >= (uint32_t)off) {
            lh = max(lh, a);
            ln = max(ln, b);
        }
    }
    int ph = __shfl_up(lh, 1), pn = __shfl_up(ln, 1);  // exclusive: the lanes below
    if (lane == 0) ph = pn = -1;
    bool open = ph > pn;  // the line this lane starts in already has an occurrence
    uint32_t keep = 0;
    for (int b = 0; b < 16; b++) {
        if ((nl >> b) & 1u) open = false;
        if ((hit >> b) & 1u) {
            if (!open) keep |= 1u << b;
            open = true;
        }
    }
    return keep;
}

__global__ void __launch_bounds__(kThreads) grep_map_kernel(const uint8_t* __restrict__ in, uint64_t n, uint64_t cbeg,
                                                            uint64_t nchunks, const uint8_t* __restrict__ pat,
                                                            uint32_t plen, Tables t) {
    __shared__ uint4 ring[kWavesPerWG][kGrepSlots][kChunk / 16];
    __shared__ uint8_t P[kAhead + 16];
    __shared__ unsigned long long mbuf[kWavesPerWG][kGrepBuf];  // buffered match positions
    __shared__ uint32_t mcnt[kWavesPerWG];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (tid < plen && tid < (uint32_t)sizeof(P)) P[tid] = pat[tid];
    if (tid < kWavesPerWG) mcnt[tid] = 0;
    __syncthreads();
    lds_u32* wcnt = (lds_u32*)&mcnt[wv];
    auto flush = [&]() {  // the wave's buffered matches -> the list (one atomic)
        const uint32_t cnt = min(*wcnt, (uint32_t)kGrepBuf);
        if (cnt == 0) return;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(&t.ctr->nlist, (unsigned long long)cnt);
        base = __shfl(base, 0);
        for (uint32_t i = lane; i < cnt; i += 64) {
            if (base + i < t.list_cap) t.list[base + i] = mbuf[wv][i];
            else set_status(t.ctr, kStListFull);
        }
        wave_sync();
        if (lane == 0) *wcnt = 0;
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        wave_sync();
    };
    const bool in_lds = plen <= (uint32_t)kAhead + 1;
    const uint32_t p0 = P[0], p1 = plen > 1 ? P[1] : 0u, p2 = plen > 2 ? P[2] : 0u, p3 = plen > 3 ? P[3] : 0u;
    const uint32_t rep0 = p0 * 0x01010101u, rep1 = p1 * 0x01010101u;
    // Chunk indices are 32-bit (the launcher checks) and the DMA offsets advance
    // by one 32-bit add per chunk (GrepStream): scalar work the loop no longer
    // redoes per chunk in 64 bits.
    const uint32_t stride = gridDim.x * kWavesPerWG;
    const uint32_t c0 = (uint32_t)cbeg + blockIdx.x * kWavesPerWG + wv, nch = (uint32_t)nchunks;
    const uint32_t slot0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)ring[wv][0];
    const uint64_t cstep = (uint64_t)stride * kGrepOwn;
    const uint32_t cstep32 = (uint32_t)cstep;  // < 2^24
#pragma unroll
    for (uint32_t q = 0; q + 1 < kGrepSlots; q++)
        grep_dma(in, n, (uint64_t)(c0 + q * stride) * kGrepOwn, lane, slot0 + q * kChunk);
    GrepStream ds;
    ds.set(in, n, (uint64_t)c0 * kGrepOwn + (kGrepSlots - 1) * cstep);
    // the chunks whose window [cs, cs + kChunk) holds the dword with the split's
    // last n % 4 bytes (none when n % 4 == 0)
    const uint64_t n4 = n & ~3ull;
    const uint32_t tail_lo = (n & 3) == 0 ? ~0u : n4 < kChunk ? 0u : (uint32_t)((n4 - kChunk) / kGrepOwn + 1);
    const uint32_t tail_hi = (n & 3) == 0 ? 0u : (uint32_t)(n4 / kGrepOwn);
    const uint32_t tail_span = (n & 3) == 0 ? 0u : tail_hi - tail_lo;  // (n % 4 == 0: c - ~0u <= 0 only for c = ~0u: never)
    uint32_t k = 0;
    uint64_t cs = (uint64_t)c0 * kGrepOwn;
    for (uint32_t c = c0; c < nch; c += stride, cs += cstep, k = k == kGrepSlots - 1 ? 0u : k + 1u) {
        // the chunk kGrepSlots - 1 strides ahead into the slot the previous one left
        const uint32_t kn = k == 0 ? kGrepSlots - 1 : k - 1u;
        ds.issue(lane, slot0 + kn * kChunk);
        ds.voff += cstep32;
        if (ds.voff >= (3u << 30)) ds.set(in, n, cs + kGrepSlots * cstep);  // rare: the window moved 2 GiB past the base
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kGrepSlots - 1) : "memory");  // this chunk's DMA has landed
        if (c - tail_lo <= tail_span) {  // c in [tail_lo, tail_hi]: one unsigned compare
            // the split's last n % 4 bytes sit in a dword the range check zero-filled
            if (lane < (uint32_t)(n & 3)) ((lds_u8*)ring[wv][k])[n4 - cs + lane] = in[n4 + lane];
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            wave_sync();
        }
        const lds_uint4* b4 = (const lds_uint4*)ring[wv][k];
        const lds_u8* bb = (const lds_u8*)b4;
        const uint4 v = from_v4(b4[lane]);
        uint32_t m, q0;  // candidate starts of this lane's bytes; pattern bytes they already match
        if (plen >= 4) {
            // 4-byte prefix filter as 32-bit compares: the word at each of the 16
            // start offsets (v_alignbyte of the lane's dwords and the next lane's
            // first) against the pattern's first four bytes, the compare results
            // straight into lane masks OR-ed by the scalar unit (7 VALU a dword);
            // the exact per-offset mask only for lanes with a candidate.  (A
            // zero-byte test of OR-ed shifted XORs per dword, ~10 VALU a dword,
            // measured 0.08 ms slower per 10 GB; per-byte masks of the first two
            // bytes ~70 VALU a lane and a candidate loop in most chunks: 0.19 ms.)
            const uint32_t p4 = p0 | p1 << 8 | p2 << 16 | p3 << 24;
            const uint32_t nx = (uint32_t)__shfl_down((int)v.x, 1);  // the next lane's first dword
            const uint32_t w[5] = {v.x, v.y, v.z, v.w, nx};
            uint64_t cand = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                cand |= __ballot(w[j] == p4);
#pragma unroll
                for (int b = 1; b < 4; b++) cand |= __ballot(__builtin_amdgcn_alignbyte(w[j + 1], w[j], b) == p4);
            }
            m = 0;
            if (lane < kGrepOwn / 16 && __builtin_amdgcn_inverse_ballot_w64(cand)) {
#pragma unroll
                for (int j = 0; j < 4; j++)
#pragma unroll
                    for (int b = 0; b < 4; b++)
                        if ((b == 0 ? w[j] : __builtin_amdgcn_alignbyte(w[j + 1], w[j], b)) == p4) m |= 1u << (4 * j + b);
            }
            q0 = 4;
        } else {
            m = lane < kGrepOwn / 16 ? eq_mask16(v, rep0) : 0u;
            if (plen > 1) {
                const uint32_t m1 = eq_mask16(v, rep1);
                const uint32_t nb = (uint32_t)__shfl_down((int)(m1 & 1u), 1);  // next lane's byte 0 (lane 59 -> 60: look-ahead)
                m &= (m1 >> 1) | (nb << 15);
            }
            q0 = 2;
        }
        bool any = false;  // a rare path issued other VMEM instructions: drain before the next DMA wait
        uint32_t vm = 0;   // verified occurrences starting in this lane's bytes
        while (m) {
            const uint32_t bit = __builtin_ctz(m);
            m &= m - 1;
            const uint32_t at = 16 * lane + bit;
            const uint64_t pos = cs + at;
            if (pos + plen > n) continue;
            bool ok = true;
            if (in_lds) {
                for (uint32_t q = q0; q < plen; q++)
                    if (bb[at + q] != P[q]) { ok = false; break; }
            } else {
                for (uint32_t q = q0; q < plen; q++)
                    if (in[pos + q] != pat[q]) { ok = false; break; }
                any = true;
            }
            if (ok) vm |= 1u << bit;
        }
        // Only the first occurrence of each line within the chunk goes on: later
        // ones name the same line (a line with k occurrences would otherwise be
        // resolved k times).  Rare in text, so only chunks with two or more pay.
        const uint64_t lanes_hit = __ballot(vm != 0);
        if ((lanes_hit & (lanes_hit - 1)) != 0 || __ballot((vm & (vm - 1)) != 0) != 0)
            vm = first_hit_per_line(vm, eq_mask16(v, 0x0A0A0A0Au), lane);
        while (vm) {
            const uint32_t bit = __builtin_ctz(vm);
            vm &= vm - 1;
            const uint64_t pos = cs + 16 * lane + bit;
            const uint32_t at_m = __hip_atomic_fetch_add(wcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (at_m < (uint32_t)kGrepBuf) {
                mbuf[wv][at_m] = pos;
            } else {  // buffer full inside one chunk (pathological): append directly
                __hip_atomic_fetch_add(wcnt, ~0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                list_append(t, pos);
                any = true;
            }
        }
        if (__ballot(any)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // rare paths: drain
        wave_sync();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this slot's LDS reads are done before it is refilled
        // (the buffer only grows in chunks with a match: no LDS read of the count
        // in the others)
        if (lanes_hit != 0 && *wcnt >= kGrepBuf - kGrepFlushRoom) flush();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last prefetch lands before the workgroup exits
    flush();
}

// Empty pattern: every line (strings.Split yields len(sep-count)+1 lines).
__global__ void grep_all_lines_kernel(const uint8_t* __restrict__ in, uint64_t n, Tables t) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
        if (i == 0) list_append(t, 0);
        else if (in[i - 1] == '\n') list_append(t, i);
    }
}

// The 16-byte aligned block holding input byte q: its bytes and the input index
// of its byte 0 (negative, or its tail past n, when the split is not 16-byte
// aligned; an aligned block never crosses a page, and the bytes outside
// [0, n) are masked off).
__device__ __forceinline__ uint4 block16(const uint8_t* in, int64_t q, int64_t& bi) {
    const uintptr_t a = (uintptr_t)(in + q);
    const uintptr_t ab = a & ~(uintptr_t)15;
    bi = q - (int64_t)(a - ab);
    return *(const uint4*)ab;
}
// Offset (relative to in) of the 16-byte-aligned block holding byte q.
__device__ __forceinline__ int64_t block_start(const uint8_t* in, int64_t q) {
    const uintptr_t a = (uintptr_t)(in + q);
    return q - (int64_t)(a - (a & ~(uintptr_t)15));
}

// long_insert (mrgpu_device.h) without its fill counters: returns whether this
// lane claimed a new slot, and the caller counts claims once per wave.
__device__ __forceinline__ bool long_try_insert_counted(const Tables& t, uint64_t h, const uint8_t* rep, uint64_t len,
                                                        uint64_t* slot = nullptr) {
    h |= 1ull;
    bool pending = true, claimed = false;
    uint32_t tries = 0;
    while (__ballot(pending)) {  // wave-uniform: reconverges between attempts
        if (pending) {
            const int r = long_try(t, h, rep, len, 1, slot);
            if (r == kFull) set_status(t.ctr, kStLongFull);
            claimed = r == kClaimed;
            pending = r == kRetry;
            if (pending && ++tries > kMaxRetries) { set_status(t.ctr, kStSpin); pending = false; }
        }
    }
    return claimed;
}

// ------------------------------------------------------------ grep lines
// Line resolution, linear in the input.  The hits are sorted by position.  Hit
// i's line starts after the last '\n' before it; if there is none between the
// previous hit and this one, both lie in one line and hit i is dropped.  So
// the backward scans cover disjoint byte ranges (each at most up to the
// previous hit), only the first hit of a line scans forward to its end, and
// the lines are hashed once per occurrence of the line.  A lane scans at most
// kLineScan bytes each way; a hit whose bounds lie further (long lines) goes
// to grep_resolve_long_kernel, one workgroup per hit with coalesced 4 KiB
// steps.  The lines sit at random HBM offsets, so this is bound by
// memory-level parallelism: a lane per hit keeps 64 independent misses in
// flight per wave, each step one aligned 16-byte load.
constexpr int64_t kLineScan = 4096;

// Position of the last '\n' in [lo, p), scanning down from p: -1 if there is
// none, -2 if none within kLineScan bytes.
__device__ int64_t last_nl_before(const uint8_t* in, int64_t lo, int64_t p) {
    int64_t q = p;
    while (q > lo) {
        if (p - q >= kLineScan) return -2;
        int64_t bi;
        const uint4 v = block16(in, q - 1, bi);
        uint32_t m = eq_mask16(v, 0x0A0A0A0Au) & ((2u << (uint32_t)(q - 1 - bi)) - 1u);  // bytes < q
        if (bi < lo) m &= ~((1u << (uint32_t)(lo - bi)) - 1u);                            // bytes >= lo
        if (m) return bi + 31 - __builtin_clz(m);
        q = bi;
    }
    return -1;
}

// Whether the pattern occurs at input offset x (x + plen <= n checked).
__device__ __forceinline__ bool occurs_at(const uint8_t* in, int64_t n, int64_t x, const uint8_t* pat, uint32_t plen) {
    if (x < 0 || x + (int64_t)plen > n) return false;
    for (uint32_t q = 0; q < plen; q++)
        if (in[x + q] != pat[q]) return false;
    return true;
}

// Unsorted hits: the line start of hit p, found like last_nl_before(in, 0, p),
// and whether the line has an occurrence of the pattern starting before the
// hit's chunk [cs, cs + kGrepOwn).  Such an occurrence belongs to an earlier
// chunk, which emitted this same line occurrence (grep_map_kernel keeps the
// first hit of each line per chunk), so this hit is dropped: every line
// occurrence is resolved exactly once, by the first chunk holding a hit in it
// (its record count is then the number of times the line occurs, as
// dgrep.go:30-33 emits one KeyValue per matching line).  The scan stops at the
// first '\n' or earlier occurrence below p, so over a long line with hits in
// many chunks the scans cover disjoint byte ranges (linear).
// Returns the '\n' position, -1 (none: the split's first line), -2 (beyond
// kLineScan) or -3 (an earlier chunk's occurrence: drop).
__device__ int64_t line_start_first_chunk(const uint8_t* in, int64_t n, int64_t p, int64_t cs, const uint8_t* pat,
                                          uint32_t plen) {
    const uint32_t rep0 = (uint32_t)pat[0] * 0x01010101u;
    int64_t q = p;
    while (q > 0) {
        if (p - q >= kLineScan) return -2;
        int64_t bi;
        const uint4 v = block16(in, q - 1, bi);
        const uint32_t below = (2u << (uint32_t)(q - 1 - bi)) - 1u;  // bytes < q
        const uint32_t valid = bi < 0 ? ~((1u << (uint32_t)(-bi)) - 1u) : ~0u;  // bytes >= 0
        const uint32_t nl = eq_mask16(v, 0x0A0A0A0Au) & below & valid;
        const int64_t top_nl = nl ? bi + 31 - __builtin_clz(nl) : -1;
        if (bi < cs) {  // occurrences starting below the chunk, above the newline
            uint32_t m = eq_mask16(v, rep0) & below & valid;
            if (cs - bi < 16) m &= (1u << (uint32_t)(cs - bi)) - 1u;
            if (top_nl >= 0) m &= ~((2u << (uint32_t)(top_nl - bi)) - 1u);
            while (m) {
                const uint32_t b = 31 - __builtin_clz(m);
                m &= ~(1u << b);
                if (occurs_at(in, n, bi + b, pat, plen)) return -3;
            }
        }
        if (nl) return top_nl;
        q = bi;
    }
    return -1;
}

// Position of the first '\n' in [q0, n): n if there is none, -2 if none within
// kLineScan bytes.
__device__ int64_t first_nl_from(const uint8_t* in, int64_t n, int64_t q0) {
    for (int64_t q = q0; q < n;) {
        if (q - q0 >= kLineScan) return -2;
        int64_t bi;
        const uint4 v = block16(in, q, bi);
        uint32_t m = eq_mask16(v, 0x0A0A0A0Au) & ~((1u << (uint32_t)(q - bi)) - 1u);
        if (n - bi < 16) m &= (1u << (uint32_t)(n - bi)) - 1u;
        if (m) return bi + __builtin_ctz(m);
        q = bi + 16;
    }
    return n;
}

// Workgroup size of the grep line kernels: their shared cursors (lines, table
// fill, records) take one device atomic per 1024 items.  Same-address atomics
// serialize at ~25 ns each: one per wave cost C3 ~0.15 ms per kernel.
constexpr int kLineWG = 1024, kLineWaves = kLineWG / 64;

// Append the (s, e) line pairs (one cursor atomic per workgroup) and deferred
// hit indices (rare: one per wave that has any) of a workgroup.
__device__ __forceinline__ void put_line(const Tables& t, uint64_t cap, bool keep, uint64_t s, uint64_t e, bool defer,
                                         uint64_t i, unsigned long long* scratch) {
    const unsigned long long o = block_alloc<kLineWaves>(&t.ctr->nlines, keep ? 1u : 0u, scratch);
    if (keep) {
        if (o < cap) {
            t.lines[2 * o] = s;
            t.lines[2 * o + 1] = e;
        } else {
            set_status(t.ctr, kStListFull);
        }
    }
    const unsigned long long d = wave_alloc(&t.ctr->ndefer, defer);
    if (defer) {
        if (d < cap) t.defer[d] = i;
        else set_status(t.ctr, kStListFull);
    }
}

// One lane per hit.  plen == 0: the hits are line starts (empty pattern).
// sorted: the hits are in position order, and a hit whose line has an earlier
// hit (no '\n' since it) is dropped; unsorted (the map kernel's order, no sort
// pass: C3 ~0.13 ms of radix passes), every hit resolves its own line, and the
// LongTable's insert merges the rare repeats (a line with hits in two chunks).
__global__ void __launch_bounds__(kLineWG) grep_resolve_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                               const uint8_t* __restrict__ pat, uint32_t plen,
                                                               Tables t, uint64_t cap, const unsigned long long* dn,
                                                               bool sorted) {
    __shared__ unsigned long long scratch[kLineWaves + 1];
    __shared__ unsigned long long wg_bytes;
    if (threadIdx.x == 0) wg_bytes = 0;  // (put_line's barriers order this before the adds below)
    // dn: the hit count read here (the map kernel's cursor, no host round trip);
    // the workgroups stride over it in whole-workgroup steps (put_line's barriers)
    const uint64_t nhits = dn ? (*dn < cap ? *dn : cap) : cap;
    for (uint64_t base = (uint64_t)blockIdx.x * kLineWG; base < nhits; base += (uint64_t)gridDim.x * kLineWG) {
        const uint64_t i = base + threadIdx.x;
        bool keep = false, defer = false;
        int64_t s = 0, e = 0;
        if (i < nhits) {
            const int64_t p = (int64_t)t.hits[i];
            if (plen == 0) {
                s = p;
                keep = true;
            } else {
                const int64_t lo = i == 0 || !sorted ? 0 : (int64_t)t.hits[i - 1] + 1;
                const int64_t q = sorted ? last_nl_before(in, lo, p)
                                         : line_start_first_chunk(in, (int64_t)n, p, p - p % (int64_t)kGrepOwn, pat, plen);
                if (q == -2) defer = true;
                else if (q >= 0) { s = q + 1; keep = true; }
                else if (q == -1 && lo == 0) { s = 0; keep = true; }  // no '\n' before the hit: the split's first line
                // else: no '\n' since the previous hit (sorted), or an earlier chunk's
                // occurrence in the line (unsorted): that hit names this line
            }
            if (keep) {
                e = first_nl_from(in, (int64_t)n, p + plen);
                if (e == -2) { keep = false; defer = true; }
            }
        }
        put_line(t, cap, keep, (uint64_t)s, (uint64_t)e, defer, i, scratch);
        // the lines' bytes (the record arena's bound)
        const uint64_t lb = wave_sum(keep ? (uint64_t)(e - s) : 0ull);
        if ((threadIdx.x & 63) == 0 && lb) atomicAdd(&wg_bytes, (unsigned long long)lb);
    }
    __syncthreads();
    if (threadIdx.x == 0 && wg_bytes) atomicAdd(&t.ctr->line_bytes, wg_bytes);  // one device atomic per workgroup
}

// Deferred hits: one 256-thread workgroup each, 16 bytes per lane per step
// (4 KiB steps of aligned blocks), block-wide max / min of the newline found.
__global__ void __launch_bounds__(256) grep_resolve_long_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                                const uint8_t* __restrict__ pat, uint32_t plen,
                                                                Tables t, uint64_t ndefer_h, uint64_t cap, bool sorted,
                                                                bool dev_count) {
    // dev_count: the deferred count read here (no host round trip; none: every
    // workgroup returns at once)
    const uint64_t ndefer = dev_count ? (t.ctr->ndefer < cap ? t.ctr->ndefer : cap) : ndefer_h;
    __shared__ long long red[4];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uintptr_t base = (uintptr_t)in;
    auto block_max = [&](long long v) -> long long {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v = max(v, (long long)__shfl_xor(v, off));
        if (lane == 0) red[wv] = v;
        __syncthreads();
        v = max(max(red[0], red[1]), max(red[2], red[3]));
        __syncthreads();
        return v;
    };
    for (uint64_t d = blockIdx.x; d < ndefer; d += gridDim.x) {
        const uint64_t i = t.defer[d];
        const int64_t p = (int64_t)t.hits[i];
        int64_t s = p;
        bool keep = true;
        if (plen != 0) {
            const int64_t lo = i == 0 || !sorted ? 0 : (int64_t)t.hits[i - 1] + 1;
            // unsorted: occurrences starting below the hit's chunk end the scan
            // too (line_start_first_chunk: an earlier chunk resolves this line)
            const int64_t cs = sorted ? 0 : p - p % (int64_t)kGrepOwn;
            // aligned blocks from the one holding p - 1 downwards: block k starts at
            // input offset top - 16 k.  Events: 2 x ('\n' position), 2 x (occurrence
            // start) + 1; the highest event below p decides.
            const int64_t top = (int64_t)(((base + (uint64_t)p - 1) & ~(uintptr_t)15) - base);
            long long found = -1;
            for (int64_t step = 0; found < 0; step++) {
                const int64_t bo = top - 16 * (256 * step + (int64_t)tid);  // this lane's block
                const int64_t hi_end = top - 16 * 256 * step + 16;          // first block of the step ends here
                if (hi_end <= lo) break;
                long long mine = -1;
                if (bo + 16 > lo && bo < p) {
                    const uint4 v = *(const uint4*)(in + bo);
                    uint32_t m = eq_mask16(v, 0x0A0A0A0Au);
                    for (int b = 15; b >= 0; b--)
                        if (((m >> b) & 1u) && bo + b >= lo && bo + b < p) { mine = 2 * (bo + b); break; }
                    if (bo < cs) {
                        uint32_t c = eq_mask16(v, (uint32_t)pat[0] * 0x01010101u);
                        for (int b = 15; b >= 0; b--)
                            if (((c >> b) & 1u) && bo + b >= 0 && bo + b < cs && 2 * (bo + b) + 1 > mine &&
                                occurs_at(in, (int64_t)n, bo + b, pat, plen)) {
                                mine = 2 * (bo + b) + 1;
                                break;
                            }
                    }
                }
                found = block_max(mine);
            }
            if (found >= 0 && (found & 1)) keep = false;  // an earlier chunk's occurrence in this line
            else if (found >= 0) s = found / 2 + 1;
            else if (lo == 0) s = 0;
            else keep = false;
        }
        int64_t e = (int64_t)n;
        if (keep) {
            const int64_t q0 = p + plen;
            const int64_t first = (int64_t)((base + (uint64_t)q0) & ~(uintptr_t)15) - (int64_t)base;
            for (int64_t step = 0;; step++) {
                const int64_t bo = first + 16 * (256 * step + (int64_t)tid);
                if (first + 16 * 256 * step >= (int64_t)n) break;
                long long mine = LLONG_MAX;
                if (bo < (int64_t)n && bo + 16 > q0) {
                    const uint4 v = *(const uint4*)(in + bo);
                    uint32_t m = eq_mask16(v, 0x0A0A0A0Au);
                    for (int b = 0; b < 16; b++)
                        if (((m >> b) & 1u) && bo + b >= q0 && bo + b < (int64_t)n) { mine = bo + b; break; }
                }
                const long long f = -block_max(-mine);
                if (f != LLONG_MAX) { e = f; break; }
            }
        }
        if (tid == 0 && keep) {
            atomicAdd(&t.ctr->line_bytes, (unsigned long long)(e - s));
            const unsigned long long o = atomicAdd(&t.ctr->nlines, 1ull);
            if (o < cap) {
                t.lines[2 * o] = (uint64_t)s;
                t.lines[2 * o + 1] = (uint64_t)e;
            } else {
                set_status(t.ctr, kStListFull);
            }
        }
    }
}

// Line content hash for the LongTable: FNV-1a-64 of every byte, or for a line
// longer than kHashAll of its first and last kHashEdge bytes and its length
// (equal lines hash equally, and slot matches are confirmed bytewise anyway).
constexpr uint64_t kHashAll = 8192, kHashEdge = 2048;
__device__ uint64_t hash_bytes(const uint8_t* in, int64_t s, int64_t e, uint64_t h) {
    // 64 bytes per step: the four aligned 16-byte loads are issued together (one
    // memory round trip per step, not per 16 bytes: long lines dominated the
    // kernel); only blocks holding bytes before e are read
    for (int64_t q = s; q < e;) {
        const int64_t bi = block_start(in, q);
        const uint8_t* ab = in + bi;
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = bi + 16 * k < e ? *(const uint4*)(ab + 16 * k) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const int64_t p = bi + 16 * k + j;
                if (p >= q && p < e) h = fnv1a64_step(h, (w[j >> 2] >> (8 * (j & 3))) & 0xFFu);
            }
        }
        q = bi + 64;
    }
    return h;
}

// A line's FNV-1a-32 (the partition hash, worker.go:76) in one pass over its
// bytes, and from it and the length the line's LongTable hash.  The table
// confirms every hash match bytewise, so the hash only has to be a function of
// the bytes; it is used by grep_insert_kernel's table alone (records merged
// later are re-inserted into clean tables with hash_bytes).  An FNV-1a-64 chain
// beside the 32-bit one doubled the kernel's multiplies (C3 insert 0.45 ms).
// 32-bit position arithmetic within each 64-byte block.
__device__ __forceinline__ uint64_t hash_line(const uint8_t* in, int64_t s, int64_t e, uint32_t& h32) {
    uint32_t g = 2166136261u;
    for (int64_t q = s; q < e;) {
        const int64_t bi = block_start(in, q);
        const uint8_t* ab = in + bi;
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = bi + 16 * k < e ? *(const uint4*)(ab + 16 * k) : make_uint4(0, 0, 0, 0);
        const uint32_t lo = (uint32_t)(q - bi);                      // 0..15
        const uint32_t span = (uint32_t)((e - bi < 64 ? e - bi : 64) - (int64_t)lo);  // block positions [lo, lo + span)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const uint32_t c = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                if ((uint32_t)(16 * k + j) - lo < span) g = fnv1a32_step(g, c);
            }
        }
        q = bi + 64;
    }
    h32 = g;
    uint64_t x = ((uint64_t)g << 32) | (uint32_t)(e - s);
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    return x ^ (x >> 33);
}

// The first 16 bytes of a line (zero-padded past len) as little-endian k0 / k1:
// the aligned 16-byte blocks holding them (a block is read only if it holds a
// byte of the line) funnel-shifted by the start's byte offset.
__device__ __forceinline__ void line_prefix16(const uint8_t* in, int64_t s, uint64_t len, uint64_t& k0, uint64_t& k1) {
    k0 = k1 = 0;
    if (len == 0) return;
    const uintptr_t a = (uintptr_t)(in + s), ab = a & ~(uintptr_t)15;
    const uint32_t sh = (uint32_t)(a - ab);
    const uint64_t want = len < 16 ? len : 16;
    const uint4 v0 = *(const uint4*)ab;
    const uint4 v1 = ab + 16 < a + want ? *(const uint4*)(ab + 16) : make_uint4(0, 0, 0, 0);
    const uint64_t q0 = (uint64_t)v0.y << 32 | v0.x, q1 = (uint64_t)v0.w << 32 | v0.z;
    const uint64_t q2 = (uint64_t)v1.y << 32 | v1.x, q3 = (uint64_t)v1.w << 32 | v1.z;
    const bool hi = sh >= 8;
    const uint32_t r = 8 * (sh & 7);
    const uint64_t a0 = hi ? q1 : q0, a1 = hi ? q2 : q1, a2 = hi ? q3 : q2;
    k0 = r ? (a0 >> r) | (a1 << (64 - r)) : a0;
    k1 = r ? (a1 >> r) | (a2 << (64 - r)) : a1;
    if (len < 8) {
        k0 &= (1ull << (8 * len)) - 1;
        k1 = 0;
    } else if (len < 16) {
        k1 &= (1ull << (8 * (len - 8))) - 1;
    }
}

// One lane per resolved line: hash, insert into the LongTable (the first
// occurrence claims the slot).  emit: the claiming lane also writes the line's
// record at a workgroup's share of ctr->nrec / ctr->arena (one cursor pair per
// workgroup) and the wave copies the claimed lines' bytes into the arena, one
// line at a time with coalesced stores — the collect pass over the table
// (C3: 0.26 ms + two host round trips) is not needed.  The record's count
// (the line's occurrences: mr-X-r holds one KV per occurrence, worker.go:80-92)
// is the slot's, read by grep_counts_kernel once every insert is in.
// (t.dbg, MRG_DEBUG_TIMES: per workgroup 4 stamps: start, table inserts done,
// cursors reserved, lines copied)
__device__ __forceinline__ void ins_stamp(const Tables& t, int k) {
    if (t.dbg && threadIdx.x == 0) t.dbg[4 * blockIdx.x + k] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void grep_insert_line(const uint8_t* __restrict__ in, const Tables& t, uint64_t i,
                                                 uint64_t nlines, bool emit, unsigned long long* scratch) {
    ins_stamp(t, 0);
    bool claimed = false;
    uint64_t len = 0, k0 = 0, k1 = 0;
    uint32_t h32 = 0;
    int64_t s = 0;
    uint64_t slot = 0;
    if (i < nlines) {
        s = (int64_t)t.lines[2 * i];
        const int64_t e = (int64_t)t.lines[2 * i + 1];
        len = (uint64_t)(e - s);
        uint64_t h;
        if (len <= kHashAll) {
            h = hash_line(in, s, e, h32);
        } else {
            h = hash_bytes(in, s, s + (int64_t)kHashEdge, kFnv64Off);
            h = hash_bytes(in, e - (int64_t)kHashEdge, e, h);
            h = fnv1a64_step(h ^ len, 0xA5u);
        }
        claimed = long_try_insert_counted(t, h, in + s, len, &slot);
        if (emit && claimed) {
            line_prefix16(in, s, len, k0, k1);
            if (len > kHashAll) {  // (rare: a very long line's partition hash)
                h32 = 2166136261u;
                for (uint64_t x = 0; x < len; x++) h32 = fnv1a32_step(h32, in[s + x]);
            }
        }
    }
    // fill counters once per workgroup (same-address device atomics serialize)
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t ik = claimed ? 1u : 0u, ib = claimed ? len : 0;  // inclusive wave scans
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t yk = __shfl_up(ik, off), yb = __shfl_up(ib, off);
        if (lane >= (uint32_t)off) { ik += yk; ib += yb; }
    }
    if (lane == 63) {
        scratch[wv] = ik;
        scratch[kLineWaves + wv] = ib;
    }
    __syncthreads();
    ins_stamp(t, 1);
    if (threadIdx.x == 0) {
        unsigned long long kk = 0, bb = 0;
        for (int w = 0; w < kLineWaves; w++) {  // -> exclusive prefixes per wave
            const unsigned long long xk = scratch[w], xb = scratch[kLineWaves + w];
            scratch[w] = kk;
            scratch[kLineWaves + w] = bb;
            kk += xk;
            bb += xb;
        }
        unsigned long long rb = 0, ab = 0;
        if (kk) {
            // emit: the record cursors count exactly the claims and their bytes,
            // so they stand in for long_used / long_bytes (grep_counts_kernel
            // copies them over): two same-address atomics per workgroup step, not four
            unsigned long long used;
            if (emit) {
                rb = atomicAdd(&t.ctr->nrec, kk);
                ab = atomicAdd(&t.ctr->arena, bb);
                used = rb + kk;
            } else {
                atomicAdd(&t.ctr->long_bytes, bb);
                used = atomicAdd(&t.ctr->long_used, kk) + kk;
            }
            if (used * 10 > (t.lo_mask + 1) * 7) set_status(t.ctr, kStLongFull);
        }
        scratch[2 * kLineWaves] = rb;
        scratch[2 * kLineWaves + 1] = ab;
    }
    __syncthreads();
    ins_stamp(t, 2);
    if (!emit) return;  // (workgroup-uniform)
    const uint64_t o = scratch[2 * kLineWaves] + scratch[wv] + ik - (claimed ? 1u : 0u);
    const uint64_t off = scratch[2 * kLineWaves + 1] + scratch[kLineWaves + wv] + ib - (claimed ? len : 0);
    bool ok = false;
    if (claimed) {
        if (o < t.out_cap && off + len <= t.out.arena_n) {
            ok = true;
            t.out.k0[o] = k0;
            t.out.k1[o] = k1;
            t.out.len[o] = (uint32_t)len;
            t.out.cnt[o] = slot;  // the slot's index until grep_counts_kernel reads its final count
            t.out.part[o] = (h32 & 0x7fffffffu) % t.nreduce;
            t.out.koff[o] = off;
        } else {
            set_status(t.ctr, kStRecFull);
        }
    }
    // The claimed lines' bytes by the whole wave, four lines per step with all
    // four lines' loads issued before their stores (a line at a time left one
    // load round trip per line on each wave's critical path: insert 0.28 ->
    // 0.45 ms on C3).
    constexpr int kCopyLines = 4;
    uint64_t m = __ballot(ok);
    while (m) {
        uint64_t src[kCopyLines], dst[kCopyLines];
        uint32_t l[kCopyLines], lmax = 0;
#pragma unroll
        for (int k = 0; k < kCopyLines; k++) {
            src[k] = dst[k] = 0;
            l[k] = 0;
            if (m) {
                const uint32_t j = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
                src[k] = readlane64((uint64_t)s, j);
                dst[k] = readlane64(off, j);
                l[k] = (uint32_t)__builtin_amdgcn_readlane((uint32_t)len, j);
                lmax = l[k] > lmax ? l[k] : lmax;
            }
        }
        for (uint32_t x0 = 0; x0 < lmax; x0 += 64) {
            const uint32_t x = x0 + lane;
            uint8_t b[kCopyLines];
#pragma unroll
            for (int k = 0; k < kCopyLines; k++) b[k] = x < l[k] ? in[src[k] + x] : (uint8_t)0;
#pragma unroll
            for (int k = 0; k < kCopyLines; k++)
                if (x < l[k]) t.out.arena[dst[k] + x] = b[k];
        }
    }
    if (t.dbg) {
        __syncthreads();
        ins_stamp(t, 3);
    }
}

// nlines, or with dn the line count read here (the resolution's cursor, no
// host round trip): the workgroups stride over it in whole-workgroup steps.
__global__ void __launch_bounds__(kLineWG) grep_insert_kernel(const uint8_t* __restrict__ in, Tables t, uint64_t nlines,
                                                              const unsigned long long* dn, bool emit) {
    __shared__ unsigned long long scratch[2 * kLineWaves + 2];
    const uint64_t n = dn ? (*dn < nlines ? *dn : nlines) : nlines;
    for (uint64_t base = (uint64_t)blockIdx.x * kLineWG; base < n; base += (uint64_t)gridDim.x * kLineWG) {
        grep_insert_line(in, t, base + threadIdx.x, n, emit, scratch);
        __syncthreads();  // scratch reused by the next step
    }
}

// ------------------------------------------------------------ collect
// ShortTable: every claim appends its slot index to the claim list (sh_list), so
// record i is the list's i-th slot, written at base + i with no shared cursor.
// The ShortTable's claimed slots (its claim list, ctr->short_used entries) as
// records at ctr->nrec; nrec_add_kernel then advances ctr->nrec past them.
__global__ void collect_short_kernel(Tables t) {
    const uint64_t used = t.ctr->short_used;
    const uint64_t n = used < t.sh_mask + 1 ? used : t.sh_mask + 1;
    const uint64_t base = t.ctr->nrec;  // (nothing moves it during this kernel)
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t o = base + i;
        if (o >= t.out_cap) { set_status(t.ctr, kStRecFull); continue; }
        const ShortSlot s = t.sh[t.sh_list[i]];
        const uint32_t len = key_len_short(s.k0, s.k1);
        t.out.k0[o] = s.k0;
        t.out.k1[o] = s.k1;
        t.out.len[o] = len;
        t.out.cnt[o] = s.count;
        t.out.part[o] = short_partition(s.k0, s.k1, len, t.nreduce);
        t.out.koff[o] = ~0ull;
    }
}

__global__ void nrec_add_kernel(Tables t) {
    const uint64_t used = t.ctr->short_used;
    t.ctr->nrec += used < t.sh_mask + 1 ? used : t.sh_mask + 1;
}

// One LongTable record: key bytes copied to the arena at `off` by aligned
// 16-byte blocks (the representative sits at a random input offset: one load
// per block, not a chain of byte loads), prefix words and partition from them.
// Record o of a LongTable key, its bytes copied to the arena at off: the first
// 16 bytes as k0/k1 and the partition from FNV-1a-32 of all bytes
// (worker.go:76), read in aligned 16-byte blocks.  Returns false (and sets
// kStRecFull) when the record or arena buffer is too small.
// copy_bytes = false: the arena bytes are left to the caller (collect_long_kernel
// copies each record's bytes with the whole wave: 64 consecutive bytes per store
// instruction instead of 64 scattered ones).
template <bool copy_bytes = true>
__device__ __forceinline__ bool emit_long_rec(const Tables& t, const LongSlot& s, uint64_t o, uint64_t off, uint64_t len) {
    if (o >= t.out_cap || off + len > t.out.arena_n) { set_status(t.ctr, kStRecFull); return false; }
    uint32_t h = 2166136261u;
    uint64_t k0 = 0, k1 = 0;
    for (int64_t q = 0; q < (int64_t)len;) {  // 64 bytes (four loads in flight) per step, as hash_bytes
        const int64_t bi = block_start(s.rep, q);
        const uint8_t* ab = s.rep + bi;
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++)
            v[k] = bi + 16 * k < (int64_t)len ? *(const uint4*)(ab + 16 * k) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
            for (int j = 0; j < 16; j++) {
                const int64_t p = bi + 16 * k + j;
                if (p < q || p >= (int64_t)len) continue;
                const uint32_t b = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                if (copy_bytes) t.out.arena[off + p] = (uint8_t)b;  // (stores do not wait)
                h = fnv1a32_step(h, b);
                if (p < 8) k0 |= (uint64_t)b << (8 * p);
                else if (p < 16) k1 |= (uint64_t)b << (8 * (p - 8));
            }
        }
        q = bi + 64;
    }
    t.out.k0[o] = k0;
    t.out.k1[o] = k1;
    t.out.len[o] = (uint32_t)len;
    t.out.cnt[o] = s.count;
    t.out.part[o] = (h & 0x7fffffffu) % t.nreduce;
    t.out.koff[o] = off;
    return true;
}

// LongTable -> records.  Each wave takes kCollectSlots x 64 slots per step and
// reserves their records and arena bytes with ONE pair of cursor atomics
// (same-address device atomics serialize at the memory side: one pair per 64
// slots of a 1 M-slot table cost ~0.6 ms).
// Latency-bound (each key's bytes sit at a random input offset): many waves with
// few slots each beat few waves with many (8 slots per lane: C3 collect 0.4 ms).
constexpr int kCollectSlots = 2;
__global__ void __launch_bounds__(kLineWG) collect_long_kernel(Tables t) {
    __shared__ unsigned long long scratch[2 * kLineWaves + 2];
    if (t.ctr->long_used == 0) return;  // (launched without a host read of the count; workgroup-uniform)
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t n = t.lo_mask + 1;
    constexpr uint64_t kStep = 64 * kCollectSlots;
    const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    // the loop bound is workgroup-uniform (whole workgroups step together): every
    // thread reaches the barriers
    const uint64_t wg0 = (uint64_t)blockIdx.x * kLineWaves * kStep;
    for (uint64_t g0 = wg0; g0 < n; g0 += nw * kStep) {
        const uint64_t w0 = g0 + wv * kStep;
        LongSlot sl[kCollectSlots];
        uint32_t c = 0;
        uint64_t bytes = 0;
#pragma unroll
        for (int k = 0; k < kCollectSlots; k++) {
            const uint64_t i = w0 + 64 * k + lane;
            sl[k] = i < n ? t.lo[i] : LongSlot{0, nullptr, 0, 0};
            const bool valid = sl[k].hash != 0 && sl[k].rep != nullptr && sl[k].len != 0;
            if (!valid) sl[k].len = 0;  // len + 1 of a valid slot is >= 1
            c += valid;
            bytes += valid ? sl[k].len - 1 : 0;
        }
        // inclusive wave scans of the record and byte counts
        uint64_t ic = c, ib = bytes;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint64_t yc = __shfl_up(ic, off), yb = __shfl_up(ib, off);
            if (lane >= (uint32_t)off) { ic += yc; ib += yb; }
        }
        // one cursor pair per workgroup step: wave totals -> LDS -> exclusive
        // prefix per wave and one atomic each
        if (lane == 63) {
            scratch[wv] = ic;
            scratch[kLineWaves + wv] = ib;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned long long rc = 0, rb = 0;
            for (int w = 0; w < kLineWaves; w++) {
                const unsigned long long xc = scratch[w], xb = scratch[kLineWaves + w];
                scratch[w] = rc;
                scratch[kLineWaves + w] = rb;
                rc += xc;
                rb += xb;
            }
            scratch[2 * kLineWaves] = rc ? atomicAdd(&t.ctr->nrec, rc) : 0ull;
            scratch[2 * kLineWaves + 1] = rc ? atomicAdd(&t.ctr->arena, rb) : 0ull;
            if (rc) atomicAdd(&t.ctr->nlong_rec, rc);
        }
        __syncthreads();
        const uint64_t rbase = scratch[2 * kLineWaves] + scratch[wv], abase = scratch[2 * kLineWaves + 1] + scratch[kLineWaves + wv];
        __syncthreads();
        uint64_t o = rbase + ic - c, off = abase + ib - bytes;
        uint64_t offk[kCollectSlots];
        bool okk[kCollectSlots];
#pragma unroll
        for (int k = 0; k < kCollectSlots; k++) {
            offk[k] = off;
            okk[k] = false;
            if (sl[k].len == 0) continue;
            const uint64_t len = sl[k].len - 1;
            okk[k] = emit_long_rec<false>(t, sl[k], o, off, len);
            o++;
            off += len;
        }
        // The records' key bytes into the arena, one record at a time by the whole
        // wave (coalesced byte loads and stores; each lane writing its own records'
        // bytes made 64 scattered byte stores per instruction: C3 collect 0.26 ms).
#pragma unroll
        for (int k = 0; k < kCollectSlots; k++) {
            uint64_t m = __ballot(okk[k]);
            while (m) {
                const uint32_t j = (uint32_t)__builtin_ctzll(m);
                m &= m - 1;
                const uint64_t rep = readlane64((uint64_t)sl[k].rep, j), dst = readlane64(offk[k], j);
                const uint32_t len = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(sl[k].len - 1), j);
                const uint8_t* src = (const uint8_t*)rep;
                for (uint32_t x = lane; x < len; x += 64) t.out.arena[dst + x] = src[x];
            }
        }
    }
}

// Re-aggregate records (merge / import / exchange receive).
__global__ void insert_recs_kernel(Recs src, Tables t) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < src.n; i += stride) {
        const uint64_t ko = src.koff[i];
        if (ko == ~0ull) {
            short_insert(t, src.k0[i], src.k1[i], src.cnt[i]);
        } else {
            const uint8_t* p = src.arena + ko;
            const uint32_t len = src.len[i];
            uint64_t h = kFnv64Off;
            for (uint32_t k = 0; k < len; k++) h = fnv1a64_step(h, p[k]);
            long_insert(t, h, p, len, src.cnt[i]);
        }
    }
}

// Zero everything a map run accumulates into, in one launch (each separate
// hipMemsetAsync is its own ~4 us dispatch): the counters, the bucket flags,
// the spill stream lengths, the LongTable, and the ShortTable unless known clean.
__global__ void clear_tables_kernel(Tables t, bool short_table) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i0 < sizeof(Counters) / 8) reinterpret_cast<unsigned long long*>(t.ctr)[i0] = 0;
    if (t.bflag)
        for (uint64_t i = i0; i < (uint64_t)t.sp.nb; i += stride) t.bflag[i] = 0;
    if (t.sp.counts) {  // counts and counts8 are contiguous (make_tables)
        const uint64_t nc = 2ull * t.sp.nb * t.sp.nwg;
        for (uint64_t i = i0; i < nc; i += stride) t.sp.counts[i] = 0;
    }
    if (t.lrec_cnt && i0 < (uint64_t)kMaxMapWGs * kWavesPerWG) t.lrec_cnt[i0] = 0;  // (regions the map does not use stay 0)
    if (short_table)
        for (uint64_t i = i0; i <= t.sh_mask; i += stride) t.sh[i] = ShortSlot{0, kUnwritten, 0, 0};
    for (uint64_t i = i0; i <= t.lo_mask; i += stride) t.lo[i] = LongSlot{0, nullptr, 0, 0};
}

// ------------------------------------------------------------ launchers
int map_grid_size(int device) {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0) ncu = 256;
    return ncu;  // one 1024-thread workgroup per CU (LDS-bound), persistent over chunks
}

__global__ void clear_long_kernel(Tables t) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t i = i0; i <= t.lo_mask; i += stride) t.lo[i] = LongSlot{0, nullptr, 0, 0};
    if (i0 == 0) {
        // the insert's own status bits only: a hit-list overflow flagged by the
        // map kernel must survive to the counter read after the insert (grep's
        // speculative sizes read nothing in between)
        t.ctr->status &= ~(uint32_t)(kStLongFull | kStRecFull | kStSpin);
        t.ctr->long_used = 0;
        t.ctr->long_bytes = 0;
        t.ctr->nrec = 0;
        t.ctr->arena = 0;
    }
}

void clear_long_table(const Tables& t, hipStream_t s) { clear_long_kernel<<<2048, 256, 0, s>>>(t); }

void clear_tables(const Tables& t, bool short_table, hipStream_t s) {
    static_assert(sizeof(Counters) % 8 == 0 && sizeof(Counters) / 8 <= 256, "counters cleared by the first threads");
    clear_tables_kernel<<<2048, 256, 0, s>>>(t, short_table);
}

void launch_wc_long(const uint8_t* in, uint64_t n, const Tables& t, LetterTables lt, uint64_t nlist, hipStream_t s) {
    if (nlist == 0) return;
    // one workgroup per CU (LDS-bound), each with a contiguous share of the list
    // (nlist = ~0, read on the device: every CU)
    uint64_t g = nlist == ~0ull ? ~0ull : (nlist + kLongWG * 4 - 1) / (kLongWG * 4);
    const uint64_t ncu = (uint64_t)map_grid_size(0);
    if (g > ncu) g = ncu;
    wc_long_kernel<<<(unsigned)g, kLongWG, 0, s>>>(in, n, t, lt, nlist);
}

void launch_grep_map(const uint8_t* in, uint64_t n, const uint8_t* d_pat, uint32_t plen, const Tables& t, int grid,
                     hipStream_t s, uint64_t cbeg, uint64_t cend) {
    static_assert(kGrepOwn == kGrepChunkBytes, "chunk size");
    uint64_t nchunks = (n + kGrepOwn - 1) / kGrepOwn;
    if (cend < nchunks) nchunks = cend;
    if (nchunks <= cbeg || plen == 0) return;
    uint64_t g = (nchunks - cbeg + kWavesPerWG - 1) / kWavesPerWG;
    const uint64_t gmax = (uint64_t)grid * 2;
    if (g > gmax) g = gmax;
    // (32-bit chunk indices in the kernel: mrg_map refuses splits past them)
    grep_map_kernel<<<(unsigned)g, kThreads, 0, s>>>(in, n, cbeg, nchunks, d_pat, plen, t);
}

void launch_grep_all_lines(const uint8_t* in, uint64_t n, const Tables& t, int grid, hipStream_t s) {
    grep_all_lines_kernel<<<grid * 4, 256, 0, s>>>(in, n, t);
}

void launch_grep_resolve(const uint8_t* in, uint64_t n, const uint8_t* d_pat, uint32_t plen, const Tables& t,
                         uint64_t nhits, bool dev_count, bool sorted, hipStream_t s) {
    if (nhits == 0) return;
    uint64_t g = (nhits + kLineWG - 1) / kLineWG;
    if (dev_count && g > 1024) g = 1024;  // (nhits = the list's capacity: the workgroups stride)
    grep_resolve_kernel<<<(unsigned)g, kLineWG, 0, s>>>(in, n, d_pat, plen, t, nhits,
                                                        dev_count ? &t.ctr->nlist : nullptr, sorted);
}

void launch_grep_resolve_long(const uint8_t* in, uint64_t n, const uint8_t* d_pat, uint32_t plen, const Tables& t,
                              uint64_t ndefer, uint64_t nhits, bool dev_count, bool sorted, hipStream_t s) {
    if (!dev_count && ndefer == 0) return;
    const uint64_t g = dev_count ? 1024 : ndefer < 4096 ? ndefer : 4096;
    grep_resolve_long_kernel<<<(unsigned)g, 256, 0, s>>>(in, n, d_pat, plen, t, ndefer, nhits, sorted, dev_count);
}

// The emitted records' counts: cnt held the claimed slot's index.
__global__ void grep_counts_kernel(Tables t) {
    const uint64_t n = t.ctr->nrec < t.out_cap ? t.ctr->nrec : t.out_cap;
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // (the insert counted its claims in the record cursors only)
        t.ctr->long_used = t.ctr->nrec;
        t.ctr->long_bytes = t.ctr->arena;
    }
    for (uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; o < n; o += (uint64_t)gridDim.x * blockDim.x)
        t.out.cnt[o] = t.lo[t.out.cnt[o] & t.lo_mask].count;
}

void launch_grep_insert(const uint8_t* in, const Tables& t, uint64_t nlines, bool dev_count, bool emit, hipStream_t s) {
    if (nlines == 0) return;
    uint64_t g = (nlines + kLineWG - 1) / kLineWG;
#ifndef MRG_GREP_INS_GRID
#define MRG_GREP_INS_GRID 1024
#endif
    if (dev_count && g > MRG_GREP_INS_GRID) g = MRG_GREP_INS_GRID;  // (nlines = the capacity: the workgroups stride)
    grep_insert_kernel<<<(unsigned)g, kLineWG, 0, s>>>(in, t, nlines, dev_count ? &t.ctr->nlines : nullptr, emit);
    if (emit) {
        const uint64_t g = (nlines + 255) / 256;
        grep_counts_kernel<<<(unsigned)(g < 2048 ? g : 2048), 256, 0, s>>>(t);
    }
}

__global__ void collect_mark_kernel(Counters* ctr) { ctr->nrec_base = ctr->nrec; }
__global__ void collect_undo_kernel(Counters* ctr) {
    ctr->nrec = ctr->nrec_base;
    ctr->arena = 0;
    ctr->nlong_rec = 0;
    ctr->status &= ~(uint32_t)kStRecFull;
}
void launch_collect_undo(const Tables& t, hipStream_t s) { collect_undo_kernel<<<1, 1, 0, s>>>(t.ctr); }

int launch_collect(const Tables& t, bool long_table, hipStream_t s) {
    collect_mark_kernel<<<1, 1, 0, s>>>(t.ctr);
    collect_short_kernel<<<512, 256, 0, s>>>(t);
    nrec_add_kernel<<<1, 1, 0, s>>>(t);
    if (long_table) {
        const uint64_t steps = (t.lo_mask + 1 + 64 * kCollectSlots - 1) / (64 * kCollectSlots);  // wave steps
        const uint64_t g = (steps + kLineWaves - 1) / kLineWaves < 512 ? (steps + kLineWaves - 1) / kLineWaves : 512;
        collect_long_kernel<<<(unsigned)g, kLineWG, 0, s>>>(t);
    }
    return (int)hipGetLastError();
}

void launch_insert_recs(const Recs& src, const Tables& t, hipStream_t s) {
    if (src.n == 0) return;
    uint64_t g = (src.n + 255) / 256;
    if (g > 4096) g = 4096;
    insert_recs_kernel<<<(unsigned)g, 256, 0, s>>>(src, t);
}

}  // namespace mrg
