// mrgpu_reduce.hip — Reduce side: sort.Sort(ByKey) + group + Reduce + Fprintf.
//
// Reference: MapReduce/mr/worker.go:123-146 (and main/mrsequential.go:59-84).
// Input records are already grouped (one record per distinct key with its
// count), so "group + reducef(len(values))" is the record itself; what remains
// is the bytewise key order and the "%v %v\n" formatting.
//
// Order: Go string '<' is unsigned bytewise with a shorter prefix first.  Keys
// are sorted by (partition, first 16 bytes zero-padded, big-endian) with
// stable LSD radix passes; a strictly smaller padded prefix implies a smaller
// key, so that order is exact whenever prefixes differ.  Runs of equal
// prefixes (keys > 16 bytes, or grep lines containing NUL bytes) are then
// ordered by a full bytewise comparison inside each run.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <algorithm>

#include "mrgpu_device.h"
#include "mrgpu_scan.h"

namespace mrg {

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        size_t c = n < 4096 ? 4096 : n + n / 4;
        hipError_t e = hipMalloc(&p, c);
        if (e == hipSuccess) cap = c;
        return e;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct ReduceWs {
    DBuf perm_a, perm_b, key_a, key_b, lineoff, out, flags, sel, offs, ext, tiek, bins, runs;
    uint64_t* h_pinned = nullptr;  // small pinned staging
    int digit_bits = 0;            // radix digit of the key passes: 10, or 8 (0 = 8; mrgpu_sort.hip)
    bool fold_part = true;         // wc: partition folded into the top bits of the k0 sort key
    bool grep_k1 = true;           // grep: radix passes over the first 16 key bytes (else 8, more ties)
    bool compact_ties = true;      // tied runs merge-sorted on compact key copies (TieKey)
    // single-key wc sorts by the hand-written sample sort below instead of the
    // radix passes: exact, but measured slower (C2 reduce 0.70 vs 0.42 ms, C5 4.4 vs
    // 2.5 ms: its LDS bitonic bin sorts and scattered writes), so off by default
    bool bin_sort = false;
    // the wc single-key pass sorts only the key's top 32 bits ((partition, first
    // key bits): four 8-bit onesweep passes over u32 keys instead of six 10-bit
    // passes over u64 ones); keys tied on them are ordered by fix_ties
    bool prefix32 = true;
    // (compatibility option: the radix passes are always the hand-written LSD sort,
    // mrgpu_sort.hip; rocPRIM's onesweep was the alternative until round 4)
    bool own_sort = true;
    // grep (16-byte passes): tied runs ordered by rank per run (waves / workgroups)
    // instead of one merge sort of every tied key
    bool tie_rank = true;
    // grep (every partition): the bucketed sort fused with the output
    // (grep_bin_reduce); off: the radix passes + tie ranking + line writer
    int grep_bins = 1;  // see reduce_format
    // grep bins: the previous reduce's splitters, reused for a reduce of similar
    // size whose bins all fit the LDS sort (a worker's map tasks are alike; the
    // 8192-key sample sort is the bin path's largest serial step, ~146 us)
    DBuf gb_spl;
    uint32_t gb_nbins = 0, gb_pbits = 0;
    uint64_t gb_n = 0;
    bool gb_ok = false, gb_warm = true;
    RadixWs* rx = nullptr;
    ScanWs scan;                   // look-back state of the hand-written scans (mrgpu_scan.h)
};

void reduce_ws_set(ReduceWs* w, int digit_bits, int fold_part, int grep_k1) {
    if (digit_bits == 0 || digit_bits == 8 || digit_bits == 10) w->digit_bits = digit_bits;
    if (fold_part >= 0) w->fold_part = fold_part != 0;
    if (grep_k1 >= 0) w->grep_k1 = grep_k1 != 0;
}

void reduce_ws_set_compact_ties(ReduceWs* w, bool on) { w->compact_ties = on;
}

void reduce_ws_set_bin_sort(ReduceWs* w, bool on) { w->bin_sort = on; }
void reduce_ws_set_prefix32(ReduceWs* w, bool on) { w->prefix32 = on; }
void reduce_ws_set_own_sort(ReduceWs* w, bool on) { w->own_sort = on; }
void reduce_ws_set_tie_rank(ReduceWs* w, bool on) { w->tie_rank = on; }
void reduce_ws_set_grep_bins(ReduceWs* w, int v) {
    if (v < 0) {  // -1: bins with fresh splitters every reduce (no warm start)
        w->grep_bins = 1;
        w->gb_warm = false;
        return;
    }
    w->grep_bins = v;
    w->gb_warm = true;
}

ReduceWs* reduce_ws_new() {
    ReduceWs* w = new ReduceWs();
    w->rx = radix_ws_new();
    if (hipHostMalloc((void**)&w->h_pinned, 4096 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess) w->h_pinned = nullptr;
    return w;
}

void reduce_ws_free(ReduceWs* w) {
    if (!w) return;
    DBuf* bs[] = {&w->perm_a, &w->perm_b, &w->key_a, &w->key_b, &w->lineoff, &w->out, &w->flags, &w->sel, &w->offs, &w->ext, &w->tiek, &w->bins, &w->runs, &w->gb_spl};
    for (DBuf* b : bs) b->release();
    if (w->h_pinned) hipHostFree(w->h_pinned);
    radix_ws_free(w->rx);
    w->scan.release();
    delete w;
}

// flags[1]: a bin of the bucketed sort was too large (the sort falls back to
// rocPRIM), flags[2]: tied runs found, flags[3]: long runs (flags[0]: unused).

__global__ void iota_kernel(uint32_t* p, uint64_t n) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = (uint32_t)i;
}

// Long keys (grep lines) carry key bytes 16-63 as kExtWords big-endian words
// (ext_words_kernel): the comparison sort's compares become independent 8-byte
// loads.
constexpr int kExtWords = 6;

// The first 8 key bytes of an ASCII key (every byte < 0x80) in 56 bits: the
// low 7 bits of each byte, first byte highest (order-preserving, lossless).
__device__ __forceinline__ uint64_t pack7(uint64_t k0) {
    uint64_t v = 0;
#pragma unroll
    for (int b = 0; b < 8; b++) v = (v << 7) | ((k0 >> (8 * b)) & 0x7Full);
    return v;
}

// which: 0 = len, 1 = bswap(k1), 2 = bswap(k0), 3 = part, 4 = part in the top
// `fold` bits over bswap(k0) >> fold (the first 64 - fold key bits), 5 = part
// over pack7(k0) (ASCII keys: 56 + fold bits, nothing dropped); 6 / 7 = the
// top 32 bits of the 5 / 4 key (u32; for 6, fold = the partition bits).
__global__ void gather_key_kernel(Recs r, const uint32_t* perm, uint64_t n, int which, uint64_t* k64, uint32_t* k32,
                                  uint32_t fold = 0) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint32_t j = perm ? perm[i] : (uint32_t)i;
        if (which == 0) k32[i] = r.len[j];
        else if (which == 1) k64[i] = __builtin_bswap64(r.k1[j]);
        else if (which == 2) k64[i] = __builtin_bswap64(r.k0[j]);
        else if (which == 4) k64[i] = ((uint64_t)r.part[j] << (64 - fold)) | (__builtin_bswap64(r.k0[j]) >> fold);
        else if (which == 5) k64[i] = ((uint64_t)r.part[j] << 56) | pack7(r.k0[j]);
        else if (which == 6)  // top 32 bits of the (56 + fold)-bit packed key (fold = the partition bits here)
            k32[i] = (uint32_t)((((uint64_t)r.part[j] << 56) | pack7(r.k0[j])) >> (24 + fold));
        else if (which == 7) k32[i] = (uint32_t)((((uint64_t)r.part[j] << (64 - fold)) | (__builtin_bswap64(r.k0[j]) >> fold)) >> 32);
        else k32[i] = r.part[j];
    }
}

// tie[i] = 1 when sorted position i has the same sort key as i - 1 (the single
// folded / packed key pass: equal keys are equal (partition, prefix)).  The
// "any tie" flag (read by grep's all-runs path) takes one atomic per workgroup:
// a per-wave check and atomic on one address made this 30 us instead of 5 at
// C2's 1e6 keys.  The u32 variant (ASCII wc keys only) sets no flag.
__global__ void mark_ties_sorted_kernel(const uint64_t* keys, uint64_t n, uint8_t* tie, unsigned long long* flags) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    int any = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint8_t t = i > 0 && keys[i] == keys[i - 1] ? 1 : 0;  // (coalesced: no record gathers)
        tie[i] = t;
        any |= t;
    }
    // flags[2] = "some run is tied" (grep's folded single pass reads it): one
    // atomic per workgroup (block-uniform: every thread reaches the barrier)
    if (__syncthreads_or(any) && threadIdx.x == 0) atomicOr(&flags[2], 1ull);
}

// The same on sorted u32 keys (the 32-bit prefix pass).
__global__ void mark_ties_sorted32_kernel(const uint32_t* keys, uint64_t n, uint8_t* tie, unsigned long long* flags) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        tie[i] = i > 0 && keys[i] == keys[i - 1] ? 1 : 0;
    }
}

// Big-endian 8-byte word of key bytes [pos, pos + 8), zero past the key's end.
__device__ __forceinline__ uint64_t key_word_be(const uint8_t* p, uint32_t pos, uint32_t len) {
    uint64_t w = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) w |= (pos + k < len ? (uint64_t)p[pos + k] : 0ull) << (56 - 8 * k);
    return w;
}

// Bytewise order (worker.go:27, shorter prefix first) by 8-byte words: the
// first 16 bytes are the records' k0/k1 (zero-padded), the rest come from the
// arena.  Comparing zero-padded words and then lengths is exactly bytewise order:
// a word can only differ at a padding position of the shorter key if the longer
// key has a nonzero byte there, and then the shorter key is the smaller.
__device__ int rec_cmp(const Recs& r, uint32_t a, uint32_t b) {
    const uint64_t a0 = __builtin_bswap64(r.k0[a]), b0 = __builtin_bswap64(r.k0[b]);
    if (a0 != b0) return a0 < b0 ? -1 : 1;
    const uint64_t a1 = __builtin_bswap64(r.k1[a]), b1 = __builtin_bswap64(r.k1[b]);
    if (a1 != b1) return a1 < b1 ? -1 : 1;
    const uint32_t la = r.len[a], lb = r.len[b];
    if (la > 16 && lb > 16) {
        const uint8_t* pa = r.arena + r.koff[a];
        const uint8_t* pb = r.arena + r.koff[b];
        const uint32_t mx = la > lb ? la : lb;
        for (uint32_t pos = 16; pos < mx; pos += 8) {
            const uint64_t wa = key_word_be(pa, pos, la), wb = key_word_be(pb, pos, lb);
            if (wa != wb) return wa < wb ? -1 : 1;
        }
    }
    // equal zero-padded words: the shorter key is a prefix of the longer one (if
    // one key has <= 16 bytes, the other's bytes past it up to 16 are zero)
    return (la > lb) - (la < lb);
}

// Key bytes 16-63 of each record as kExtWords big-endian words (zero past the
// key's end), read by the tied-run comparator.
__global__ void ext_words_kernel(Recs r, uint64_t* ext) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < r.n; j += stride) {
        const uint32_t len = r.len[j];
        uint64_t wd[kExtWords] = {};
        if (len > 16) {
            // key bytes [16, min(len, 64)) by the (at most four) aligned 16-byte
            // blocks of the arena holding them, all loads issued before any is used
            // (one memory round trip per record, not one per block; an aligned
            // block never crosses a page, and only blocks holding key bytes are read)
            const uint8_t* p = r.arena + r.koff[j];
            const int64_t end = len < 16 + 8 * kExtWords ? (int64_t)len : 16 + 8 * kExtWords;
            const uintptr_t a = (uintptr_t)(p + 16), ab = a & ~(uintptr_t)15;
            const int64_t bi0 = 16 - (int64_t)(a - ab);  // key index of block 0's first byte
            uint4 v[4];
#pragma unroll
            for (int blk = 0; blk < 4; blk++)
                v[blk] = bi0 + 16 * blk < end ? *(const uint4*)(ab + 16 * blk) : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int blk = 0; blk < 4; blk++) {
                const uint32_t w4[4] = {v[blk].x, v[blk].y, v[blk].z, v[blk].w};
#pragma unroll
                for (int b = 0; b < 16; b++) {
                    const int64_t k = bi0 + 16 * blk + b;
                    if (k < 16 || k >= end) continue;
                    const uint64_t byte = (w4[b >> 2] >> (8 * (b & 3))) & 0xFFu;
#pragma unroll
                    for (int w = 0; w < kExtWords; w++)  // register-indexed: select, no scratch
                        if ((k - 16) >> 3 == w) wd[w] |= byte << (56 - 8 * ((k - 16) & 7));
                }
            }
        }
#pragma unroll
        for (int w = 0; w < kExtWords; w++) ext[kExtWords * j + w] = wd[w];
    }
}

// rec_cmp with key bytes 16-63 from the ext words: the common case is a handful
// of independent 8-byte loads instead of a chain of arena byte loads.
__device__ int rec_cmp_ext(const Recs& r, const uint64_t* ext, uint32_t a, uint32_t b) {
    const uint64_t a0 = __builtin_bswap64(r.k0[a]), b0 = __builtin_bswap64(r.k0[b]);
    if (a0 != b0) return a0 < b0 ? -1 : 1;
    const uint64_t a1 = __builtin_bswap64(r.k1[a]), b1 = __builtin_bswap64(r.k1[b]);
    if (a1 != b1) return a1 < b1 ? -1 : 1;
    const uint64_t* ea = ext + kExtWords * (uint64_t)a;
    const uint64_t* eb = ext + kExtWords * (uint64_t)b;
#pragma unroll
    for (int w = 0; w < kExtWords; w++)
        if (ea[w] != eb[w]) return ea[w] < eb[w] ? -1 : 1;
    constexpr uint32_t kCovered = 16 + 8 * kExtWords;
    const uint32_t la = r.len[a], lb = r.len[b];
    if (la > kCovered && lb > kCovered) {
        const uint8_t* pa = r.arena + r.koff[a];
        const uint8_t* pb = r.arena + r.koff[b];
        const uint32_t mx = la > lb ? la : lb;
        for (uint32_t pos = kCovered; pos < mx; pos += 8) {
            const uint64_t wa = key_word_be(pa, pos, la), wb = key_word_be(pb, pos, lb);
            if (wa != wb) return wa < wb ? -1 : 1;
        }
    }
    // equal zero-padded words up to here: the shorter key is a prefix of the longer
    return (la > lb) - (la < lb);
}

// fold > 0: the sort key held only the first 64 - fold bits of the key
__device__ __forceinline__ bool same_prefix(const Recs& r, uint32_t a, uint32_t b, bool with_k1, uint32_t fold) {
    if (r.part[a] != r.part[b]) return false;
    if (fold) return (__builtin_bswap64(r.k0[a]) >> fold) == (__builtin_bswap64(r.k0[b]) >> fold);
    return r.k0[a] == r.k0[b] && (!with_k1 || r.k1[a] == r.k1[b]);
}

// tie[i] = 1 when sorted position i has the same (part, prefix) as i-1, the
// prefix being the first 8 key bytes (sorted without the k1 pass) or all 16:
// distinct keys with equal zero-padded prefixes are only ordered by a full
// bytewise comparison.
__global__ void mark_ties_kernel(Recs r, const uint32_t* perm, uint64_t n, uint8_t* tie, unsigned long long* flags,
                                 bool with_k1, uint32_t fold) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint8_t t = 0;
        if (i > 0 && same_prefix(r, perm[i - 1], perm[i], with_k1, fold)) t = 1;
        tie[i] = t;
        if (__ballot(t) && (threadIdx.x & 63) == 0 && flags[2] == 0) atomicOr(&flags[2], 1ull);
    }
}

// grep after the 16-byte passes: tie[i] = 1 when sorted position i has the
// same (partition, first 16 key bytes) as i - 1 (mark_ties_kernel with k1), and
// in the same pass the positions that start a group (tie[i] == 0) compacted in
// order into bpos, their count in *nb: a thread takes 16 consecutive positions,
// the tiles chain by decoupled look-back (mrgpu_scan.h).  One launch in place of
// the tie marks + rocPRIM's select over a counting iterator.
__global__ void __launch_bounds__(kScanThreads) mark_ties_bounds_kernel(Recs r, const uint32_t* __restrict__ perm,
                                                                        uint64_t n, uint8_t* __restrict__ tie,
                                                                        unsigned long long* flags, uint32_t* bpos,
                                                                        uint32_t* nb, ScanState st) {
    __shared__ unsigned long long red[kScanThreads / 64];
    __shared__ unsigned long long pre;
    __shared__ uint32_t tile_w;
    const uint32_t t = scan_take_tile(st, &tile_w);
    const uint64_t i0 = (uint64_t)t * kScanTile + (uint64_t)threadIdx.x * kScanPer;
    uint32_t prev = i0 > 0 && i0 <= n ? perm[i0 - 1] : 0u;
    uint32_t tb = 0, bb = 0;  // tie / boundary bits of the 16 positions
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++) {
        const uint64_t i = i0 + k;
        if (i < n) {
            const uint32_t cur = perm[i];
            const bool tk = i > 0 && same_prefix(r, prev, cur, true, 0u);
            tb |= (tk ? 1u : 0u) << k;
            bb |= (tk ? 0u : 1u) << k;
            prev = cur;
        }
    }
    if (i0 + kScanPer <= n) {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; q++)
            w[q] = ((tb >> (4 * q)) & 1u) | (((tb >> (4 * q + 1)) & 1u) << 8) | (((tb >> (4 * q + 2)) & 1u) << 16) |
                   (((tb >> (4 * q + 3)) & 1u) << 24);
        *(uint4*)(tie + i0) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
        for (uint32_t k = 0; i0 + k < n; k++) tie[i0 + k] = (uint8_t)((tb >> k) & 1u);
    }
    if (__ballot(tb != 0) && (threadIdx.x & 63) == 0 && flags[2] == 0) atomicOr(&flags[2], 1ull);
    uint64_t tot;
    const uint64_t ex = block_excl_scan_u64((uint64_t)__popc(bb), red, &tot);
    if (threadIdx.x < 64) {
        const uint64_t p = scan_lookback(st, t, tot);
        if (threadIdx.x == 0) pre = p;
    }
    __syncthreads();
    uint64_t o = pre + ex;
    for (uint32_t m = bb; m; m &= m - 1) bpos[o++] = (uint32_t)(i0 + __builtin_ctz(m));
    if (i0 < n && i0 + kScanPer >= n) *nb = (uint32_t)o;  // the thread holding the last position: the count
}

// Positions i with f[i] != 0, compacted in order into pos, their count in
// *count (the members of long tied runs for the merge sort): one look-back
// launch in place of rocPRIM's select.
__global__ void __launch_bounds__(kScanThreads) flag_positions_kernel(const uint8_t* __restrict__ f, uint64_t n,
                                                                      uint32_t* pos, uint32_t* count, ScanState st) {
    __shared__ unsigned long long red[kScanThreads / 64];
    __shared__ unsigned long long pre;
    __shared__ uint32_t tile_w;
    const uint32_t t = scan_take_tile(st, &tile_w);
    const uint64_t i0 = (uint64_t)t * kScanTile + (uint64_t)threadIdx.x * kScanPer;
    uint32_t bb = 0;
    // (f may start at any byte, e.g. lng = tie + n: the 16-byte load only where aligned)
    if (i0 + kScanPer <= n && ((uintptr_t)(f + i0) & 15u) == 0) {
        const uint4 v = *(const uint4*)(f + i0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int b = 0; b < 4; b++) bb |= (((w[q] >> (8 * b)) & 0xFFu) != 0 ? 1u : 0u) << (4 * q + b);
    } else {
        for (uint32_t k = 0; k < kScanPer && i0 + k < n; k++) bb |= (f[i0 + k] != 0 ? 1u : 0u) << k;
    }
    uint64_t tot;
    const uint64_t ex = block_excl_scan_u64((uint64_t)__popc(bb), red, &tot);
    if (threadIdx.x < 64) {
        const uint64_t p = scan_lookback(st, t, tot);
        if (threadIdx.x == 0) pre = p;
    }
    __syncthreads();
    uint64_t o = pre + ex;
    for (uint32_t m = bb; m; m &= m - 1) pos[o++] = (uint32_t)(i0 + __builtin_ctz(m));
    if (i0 < n && i0 + kScanPer >= n) *count = (uint32_t)o;
}

// Insertion sort of each tied run by full bytewise comparison.  A run longer
// than max_run is left alone and flags[3] set; its first max_run + 1 members are
// marked in `lng` here (bounded work per thread), the rest by
// mark_long_tail_kernel.  The caller then sorts with the k1 pass (16-byte
// prefixes), or merge-sorts the marked members by full comparison
// (sort_long_runs).
__global__ void fix_ties_kernel(Recs r, uint32_t* perm, uint64_t n, const uint8_t* tie, uint64_t max_run,
                                unsigned long long* flags, uint8_t* lng) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i + 1 < n; i += stride) {
        if (tie[i] || !tie[i + 1]) continue;
        uint64_t e = i + 1;
        while (e < n && tie[e] && e - i <= max_run) e++;
        if (e - i > max_run) {
            if (flags[3] == 0) atomicOr(&flags[3], 1ull);
            for (uint64_t a = i; a < e; a++) lng[a] = 1;  // e = i + max_run + 1 here
            continue;
        }
        for (uint64_t a = i + 1; a < e; a++) {
            uint32_t v = perm[a];
            uint64_t b = a;
            while (b > i && rec_cmp(r, perm[b - 1], v) > 0) {
                perm[b] = perm[b - 1];
                b--;
            }
            perm[b] = v;
        }
    }
}

// The members of fix_ties_kernel's long runs (max_run = kTailWindow) past the
// first kTailWindow + 1: position a is one iff tie[a - 63 .. a] are all set (its
// run then started at a - 64 or earlier, so it is longer than 64).  One thread
// per 64 positions: the tie bytes of [b - 64, b + 64) folded into a 128-bit
// mask, runs of 64 set bits found by shift-and doubling.
constexpr uint32_t kTailWindow = 64;
__device__ __forceinline__ uint64_t tie_bits8(const uint8_t* tie, int64_t p, uint64_t n) {
    if (p < 0) return 0;
    uint64_t w;
    if ((uint64_t)p + 8 <= n) {
        w = *(const uint64_t*)(tie + p);
    } else {
        w = 0;
        for (uint64_t q = 0; q < 8 && (uint64_t)p + q < n; q++) w |= (uint64_t)tie[p + q] << (8 * q);
    }
    // byte q != 0 -> bit q
    w = (w | (w >> 4)) & 0x0F0F0F0F0F0F0F0Full;
    w = (w | (w >> 2)) & 0x0303030303030303ull;
    w = (w | (w >> 1)) & 0x0101010101010101ull;
    return (w * 0x0102040810204080ull) >> 56;
}
__global__ void mark_long_tail_kernel(const uint8_t* tie, uint64_t n, uint8_t* lng) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t * 64 < n; t += stride) {
        const int64_t b = (int64_t)(t * 64);
        uint64_t lo = 0, hi = 0;
        for (int q = 0; q < 8; q++) {
            lo |= tie_bits8(tie, b - 64 + 8 * q, n) << (8 * q);
            hi |= tie_bits8(tie, b + 8 * q, n) << (8 * q);
        }
        // x &= x << k over the 128-bit (hi:lo), k = 1, 2, ..., 32: bit p stays set
        // iff bits p - 63 .. p are all set
        for (int k = 1; k < 64; k <<= 1) {
            hi &= (hi << k) | (lo >> (64 - k));
            lo &= lo << k;
        }
        for (int q = 0; q < 8 && hi; q++, hi >>= 8) {
            const uint64_t p = (uint64_t)b + 8 * q;
            for (int j = 0; j < 8; j++)
                if (((hi >> j) & 1) && p + j < n) lng[p + j] = 1;
        }
    }
}

// Every member of a tied run (lng[i] != 0), for keys whose runs are best
// merge-sorted as a whole (grep lines: long keys, runs of any length).
__global__ void mark_all_ties_kernel(const uint8_t* tie, uint64_t n, uint8_t* lng) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        lng[i] = tie[i] | (i + 1 < n ? tie[i + 1] : (uint8_t)0);
}

// (partition, key) order of two records: the order the whole sort produces.
struct FullLess {
    Recs r;
    const uint64_t* ext;  // kExtWords per record, or nullptr
    __device__ bool operator()(const uint32_t& a, const uint32_t& b) const {
        if (r.part[a] != r.part[b]) return r.part[a] < r.part[b];
        return (ext ? rec_cmp_ext(r, ext, a, b) : rec_cmp(r, a, b)) < 0;
    }
};

// The merge sort of tied records compares copies of their keys laid out
// contiguously in sort-input order (80 bytes each: the first 64 key bytes as
// big-endian words, partition, length, record index), not the records' scattered
// fields: a comparison touches one or two cache lines per key instead of four.
struct alignas(16) TieKey {
    uint64_t w[2 + kExtWords];
    uint32_t part, len, rec, pad;
};

__global__ void tie_keys_kernel(Recs r, const uint64_t* ext, const uint32_t* va, const uint32_t* d_m, TieKey* K,
                                uint32_t* ia) {
    const uint32_t m = *d_m;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const uint32_t j = va[i];
        TieKey k;
        k.w[0] = __builtin_bswap64(r.k0[j]);
        k.w[1] = __builtin_bswap64(r.k1[j]);
#pragma unroll
        for (int w = 0; w < kExtWords; w++) k.w[2 + w] = ext[(uint64_t)kExtWords * j + w];
        k.part = r.part[j];
        k.len = r.len[j];
        k.rec = j;
        k.pad = 0;
        K[i] = k;
        ia[i] = i;
    }
}

struct CompactLess {
    const TieKey* K;
    Recs r;
    __device__ bool operator()(const uint32_t& a, const uint32_t& b) const {
        const TieKey& A = K[a];
        const TieKey& B = K[b];
        if (A.part != B.part) return A.part < B.part;
#pragma unroll
        for (int w = 0; w < 2 + kExtWords; w++)
            if (A.w[w] != B.w[w]) return A.w[w] < B.w[w];
        constexpr uint32_t kCovered = 16 + 8 * kExtWords;
        if (A.len > kCovered && B.len > kCovered) {  // equal first 64 bytes: the rest from the arena
            const uint8_t* pa = r.arena + r.koff[A.rec];
            const uint8_t* pb = r.arena + r.koff[B.rec];
            const uint32_t mx = A.len > B.len ? A.len : B.len;
            for (uint32_t pos = kCovered; pos < mx; pos += 8) {
                const uint64_t wa = key_word_be(pa, pos, A.len), wb = key_word_be(pb, pos, B.len);
                if (wa != wb) return wa < wb;
            }
        }
        return A.len < B.len;
    }
};

__global__ void untie_perm_kernel(const uint32_t* va, const uint32_t* ib, const uint32_t* d_m, uint32_t* vb) {
    const uint32_t m = *d_m;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) vb[i] = va[ib[i]];
}

__global__ void gather_perm_kernel(const uint32_t* perm, const uint32_t* pos, const uint32_t* d_m, uint32_t* v) {
    const uint32_t m = *d_m;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) v[i] = perm[pos[i]];
}
__global__ void scatter_perm_kernel(uint32_t* perm, const uint32_t* pos, const uint32_t* d_m, const uint32_t* v) {
    const uint32_t m = *d_m;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) perm[pos[i]] = v[i];
}

// decimal digits of v: compares against the powers of ten, no divisions
__device__ __forceinline__ uint32_t ndigits(uint64_t v) {
    uint32_t d = 1;
    uint64_t p = 10;
#pragma unroll
    for (int k = 1; k < 20; k++, p *= 10) d += v >= p ? 1u : 0u;
    return d;
}

// The decimal digits of v (d of them) at o[0, d), most significant first.
template <class OutPtr>
__device__ __forceinline__ void put_digits(OutPtr o, uint64_t v, uint32_t d) {
    if (v < (1ull << 32)) {  // 32-bit divisions for every count below 2^32
        uint32_t w = (uint32_t)v;
        for (uint32_t k = d; k > 0; k--) {
            o[k - 1] = (uint8_t)('0' + w % 10u);
            w /= 10u;
        }
    } else {
        for (uint32_t k = d; k > 0; k--) {
            o[k - 1] = (uint8_t)('0' + v % 10);
            v /= 10;
        }
    }
}

// Line lengths and their exclusive scan in one pass (worker.go:144 /
// mrsequential.go:81: "key value\n" per distinct key, in sorted order):
// off[i] = byte offset of sorted line i, off[n] = the output's total bytes.  A
// thread takes 16 consecutive lines; the tiles chain by decoupled look-back
// (mrgpu_scan.h), so this is one launch with no scratch memsets (it replaced a
// line-length kernel + rocPRIM's exclusive scan).
template <int kApp>
__global__ void __launch_bounds__(kScanThreads) line_offsets_kernel(Recs r, const uint32_t* __restrict__ perm, uint64_t n,
                                                                    uint64_t* __restrict__ off, ScanState st) {
    __shared__ unsigned long long red[kScanThreads / 64];
    __shared__ unsigned long long pre;
    __shared__ uint32_t tile_w;
    const uint32_t t = scan_take_tile(st, &tile_w);
    const uint64_t i0 = (uint64_t)t * kScanTile + (uint64_t)threadIdx.x * kScanPer;
    uint32_t j[kScanPer];
    if (i0 + kScanPer <= n) {
        const uint4* p4 = (const uint4*)(perm + i0);
#pragma unroll
        for (uint32_t q = 0; q < kScanPer / 4; q++) {
            const uint4 v = p4[q];
            j[4 * q] = v.x; j[4 * q + 1] = v.y; j[4 * q + 2] = v.z; j[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (uint32_t k = 0; k < kScanPer; k++) j[k] = i0 + k < n ? perm[i0 + k] : 0u;
    }
    uint64_t l[kScanPer];
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++) {
        uint64_t v = 0;
        if (i0 + k < n) {
            const uint64_t len = r.len[j[k]];
            v = kApp == 1 ? len + 2 + ndigits(r.cnt[j[k]]) : 2 * len + 2;
        }
        l[k] = v;
        sum += v;
    }
    uint64_t tot;
    const uint64_t ex = block_excl_scan_u64(sum, red, &tot);
    if (threadIdx.x < 64) {
        const uint64_t p = scan_lookback(st, t, tot);
        if (threadIdx.x == 0) pre = p;
    }
    __syncthreads();
    uint64_t o = pre + ex;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++) {
        if (i0 + k < n) off[i0 + k] = o;
        o += l[k];
    }
    if (i0 < n && i0 + kScanPer >= n) off[n] = o;  // the thread holding the last line: the total
}

// Output lines ("key count\n" for wc, "line line\n" for grep): a block's 256
// consecutive lines are one contiguous output range; each thread writes its line
// into LDS, then the block copies the range out with 16-byte stores (byte stores
// only at the range's two ends, which neighbouring blocks share).  A range longer
// than the LDS buffer (very long keys) is written directly, byte by byte.
constexpr uint32_t kWlLines = 256;  // threads per workgroup
// lines per workgroup step: grep's output lines (the line twice, ~160 B at C3)
// overflowed 256 lines' staging, and an unstaged block stores byte by byte
// (slow into device memory, slower into pinned host memory)
template <int kApp>
constexpr uint32_t wl_lines() { return kApp == 1 ? 256u : 128u; }
// skip (grep_bin_reduce): when *skip is set, a bin was too large for its sort,
// so perm is incomplete and nothing is written (the caller redoes the reduce)
template <int kApp>
__global__ void __launch_bounds__(kWlLines) write_lines_staged_kernel(Recs r, const uint32_t* perm, uint64_t n,
                                                                        const uint64_t* off, uint8_t* out,
                                                                        const unsigned long long* skip) {
    if (skip && *skip) return;
    constexpr uint32_t kWlBytes = kApp == 1 ? 16384 : 49152;  // C2 lines ~14 B, C3 lines ~120 B
    __shared__ __attribute__((aligned(16))) uint8_t buf[kWlBytes];
    const uint32_t tid = threadIdx.x;
    constexpr uint32_t L = wl_lines<kApp>();
    for (uint64_t i0 = (uint64_t)blockIdx.x * L; i0 < n; i0 += (uint64_t)gridDim.x * L) {
        const uint64_t iend = i0 + L < n ? i0 + L : n;
        const uint64_t start = off[i0], end = off[iend];  // off[n] = the total
        const uint64_t a0 = start & ~15ull;
        const bool staged = end - a0 <= kWlBytes;  // block-uniform
        const uint64_t i = i0 + tid;
        if (i < iend) {
            const uint32_t j = perm[i];
            const uint32_t len = r.len[j];
            const uint64_t k0 = r.k0[j], k1 = r.k1[j];
            const uint8_t* kb = len > 16 ? r.arena + r.koff[j] : nullptr;
            const uint64_t v = r.cnt[j];
            const uint32_t d = kApp == 1 ? ndigits(v) : 0u;
            auto emit = [&](auto o) {
                if (kApp != 1 && kb) {  // grep: the line twice, its arena bytes read in aligned 16-byte blocks
                    for (int64_t q = 0; q < (int64_t)len;) {
                        const uintptr_t a = (uintptr_t)(kb + q), ab = a & ~(uintptr_t)15;
                        const int64_t bi = q - (int64_t)(a - ab);
                        const uint4 v4 = *(const uint4*)ab;
                        const uint32_t w4[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
                        for (int b = 0; b < 16; b++) {
                            const int64_t k = bi + b;
                            if (k < q || k >= (int64_t)len) continue;
                            const uint8_t c = (uint8_t)(w4[b >> 2] >> (8 * (b & 3)));
                            o[k] = c;
                            o[len + 1 + k] = c;
                        }
                        q = bi + 16;
                    }
                    o[len] = ' ';
                    o[2 * len + 1] = '\n';
                    return;
                }
                for (uint32_t k = 0; k < len; k++)
                    o[k] = kb ? kb[k] : (uint8_t)((k < 8 ? k0 : k1) >> (8 * (k & 7)));
                o[len] = ' ';
                if (kApp == 1) {
                    put_digits(o + len + 1, v, d);
                    o[len + 1 + d] = '\n';
                } else {
                    for (uint32_t k = 0; k < len; k++) o[len + 1 + k] = o[k];
                    o[2 * len + 1] = '\n';
                }
            };
            if (staged) emit(buf + (off[i] - a0));
            else emit(out + off[i]);
        }
        if (staged) {
            __syncthreads();
            const uint32_t nq = (uint32_t)((end - a0 + 15) / 16);
            for (uint32_t q = tid; q < nq; q += kWlLines) {
                const uint64_t ga = a0 + 16ull * q;
                if (ga >= start && ga + 16 <= end) {
                    *(uint4*)(out + ga) = *(const uint4*)(buf + 16 * q);
                } else {
                    for (uint32_t b = 0; b < 16; b++)
                        if (ga + b >= start && ga + b < end) out[ga + b] = buf[16 * q + b];
                }
            }
            __syncthreads();
        }
    }
}

// offsets[p] = byte offset of the first line of partition p (lower bound on sorted part).
// offsets[nparts] = the output's total bytes (last line's offset + length);
// with one_part the output is one partition: offsets = {0, total}.
__global__ void part_offsets_kernel(Recs r, const uint32_t* perm, uint64_t n, const uint64_t* off, uint32_t nparts,
                                    bool one_part, uint64_t* offsets) {
    uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p > nparts) return;
    const uint64_t total = off[n];
    if (p == nparts) { offsets[p] = total; return; }
    if (one_part) { offsets[p] = 0; return; }
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (r.part[perm[mid]] < p) lo = mid + 1; else hi = mid;
    }
    offsets[p] = lo < n ? off[lo] : total;
}

// Records of one partition (or owner): one cursor atomic per wave (wave_alloc),
// not per record (same-address device atomics serialize).  The loop bound is
// wave-uniform, so every lane reaches the ballot.
__global__ void select_kernel(Recs src, uint32_t mod, uint32_t want, Recs dst, unsigned long long* cnt) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); b < src.n; b += stride) {
        const uint64_t i = b + (threadIdx.x & 63u);
        const bool take = i < src.n && src.part[i] % mod == want;
        const unsigned long long o = wave_alloc(cnt, take);
        if (!take) continue;
        dst.k0[o] = src.k0[i];
        dst.k1[o] = src.k1[i];
        dst.len[o] = src.len[i];
        dst.cnt[o] = src.cnt[i];
        dst.part[o] = src.part[i];
        dst.koff[o] = src.koff[i];
    }
}

// ------------------------------------------------------------ bucketed sort
// The wc reduce's single 64-bit key pass ((partition, packed or folded key
// prefix) per distinct key; keys + record indices), hand-written for the sizes
// that matter (1e6 - 1e7 keys), in place of rocPRIM's onesweep (six or seven
// ~25 us digit passes, each with two look-back memsets).  A sample sort:
//   1. bin_sample_kernel: one workgroup sorts an evenly spaced sample of S keys
//      in LDS (bitonic) and keeps every (S / nbins)-th as a splitter: the
//      partition and key-prefix bits are far from uniform (10 partitions of
//      16 bit patterns, 52 letters of 128, Zipf), so bins are cut by rank;
//   2. bin_count_kernel: each of G workgroups bins its contiguous range of keys
//      by binary search over the splitters in LDS (a key's bin = the number of
//      splitters <= it: equal keys share a bin), keeps the bin per key, and
//      writes its LDS histogram as H[group][bin];
//   3. bin_offsets_kernel: per bin, the exclusive prefix over the groups (a
//      coalesced column walk) and the bin total; bin_starts_kernel: exclusive
//      scan of the totals;
//   4. bin_scatter_kernel: each group places its keys at its bins' cursors (an
//      LDS atomic per key; order inside a bin is free);
//   5. bin_sort_kernel: workgroups stride over the bins and sort each in LDS
//      (bitonic network over (key, index)): bins of <= 2048 keys by 256-thread
//      workgroups, larger ones (<= 8192) by 1024-thread ones.
// Equal keys end up adjacent in any order: tie runs are ordered by full key
// comparison afterwards (fix_ties), exactly as after the radix sort.  A bin of
// more than 8192 keys (thousands of keys tied on their first 8 bytes) sets
// flags[1], and the caller repeats the pass with the radix passes.
// Measured (MI355X, rocprofv3): C2 (1e6 keys) sample 81 us, count 12, offsets
// 58, scatter 25, bin sorts 92 us = 0.70 ms reduce against onesweep's 0.42; C5
// (1e7) 1.6 ms of sort kernels against ~1.8 ms.  Option sort_bins=1 (tests run
// both); the default stays the radix passes.
constexpr uint32_t kBinMax = 8192;        // bins at most (LDS: splitters + histogram)
constexpr uint32_t kBinGroups = 256;      // count / scatter workgroups at most
constexpr uint32_t kBinSample = 16384;    // sample keys at most (one LDS bitonic sort)
constexpr uint32_t kBinSmall = 2048, kBinBig = 8192;

// Bitonic sort of P (a power of two) (key, value) pairs in LDS by NT threads.
template <uint32_t NT, class KT>
__device__ __forceinline__ void lds_bitonic(KT* K, uint32_t* V, uint32_t P) {
    for (uint32_t k = 2; k <= P; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < P / 2; i += NT) {
                const uint32_t a = 2 * i - (i & (j - 1)), c = a + j;  // pair (a, a + j), a's bit j clear
                const auto ka = K[a], kc = K[c];
                if ((ka > kc) == ((a & k) == 0)) {
                    K[a] = kc;
                    K[c] = ka;
                    if (V) {
                        const uint32_t t = V[a];
                        V[a] = V[c];
                        V[c] = t;
                    }
                }
            }
        }
    __syncthreads();
}

__global__ void __launch_bounds__(1024) bin_sample_kernel(const uint64_t* keys, uint64_t n, uint32_t S, uint32_t nbins,
                                                          uint64_t* spl) {
    __shared__ uint64_t K[kBinSample];
    for (uint32_t i = threadIdx.x; i < S; i += 1024) K[i] = keys[(uint64_t)i * n / S];
    lds_bitonic<1024, uint64_t>(K, nullptr, S);
    for (uint32_t j = threadIdx.x; j + 1 < nbins; j += 1024) spl[j] = K[(uint64_t)(j + 1) * S / nbins];
}

// the number of splitters <= k (nbins - 1 splitters, sorted)
__device__ __forceinline__ uint32_t bin_of(const uint64_t* sp, uint32_t nbins, uint64_t k) {
    uint32_t lo = 0, cnt = nbins - 1;  // upper bound over sp[0, nbins - 1)
    while (cnt) {
        const uint32_t half = cnt >> 1;
        if (sp[lo + half] <= k) {
            lo += half + 1;
            cnt -= half + 1;
        } else {
            cnt = half;
        }
    }
    return lo;
}

__global__ void __launch_bounds__(1024) bin_count_kernel(const uint64_t* keys, uint64_t n, const uint64_t* spl,
                                                         uint32_t nbins, uint16_t* kbin, uint32_t* H) {
    __shared__ uint64_t sp[kBinMax];
    __shared__ uint32_t h[kBinMax];
    for (uint32_t i = threadIdx.x; i < nbins; i += 1024) {
        h[i] = 0;
        if (i + 1 < nbins) sp[i] = spl[i];
    }
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b = (uint64_t)blockIdx.x * per, e = b + per < n ? b + per : n;
    for (uint64_t i = b + threadIdx.x; i < e; i += 1024) {
        const uint32_t bin = bin_of(sp, nbins, keys[i]);
        kbin[i] = (uint16_t)bin;
        atomicAdd(&h[bin], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbins; i += 1024) H[(uint64_t)blockIdx.x * nbins + i] = h[i];
}

// H[g][bin] -> exclusive prefix over g (in place, a coalesced column walk); tot[bin] = the bin's size
__global__ void bin_offsets_kernel(uint32_t* H, uint32_t G, uint32_t nbins, uint32_t* tot) {
    const uint32_t bin = blockIdx.x * blockDim.x + threadIdx.x;
    if (bin >= nbins) return;
    uint32_t run = 0;
    for (uint32_t g = 0; g < G; g++) {
        uint32_t* p = H + (uint64_t)g * nbins + bin;
        const uint32_t v = *p;
        *p = run;
        run += v;
    }
    tot[bin] = run;
}

// start[bin] = exclusive scan of tot (one workgroup)
__global__ void __launch_bounds__(1024) bin_starts_kernel(const uint32_t* tot, uint32_t nbins, uint32_t* start) {
    __shared__ uint32_t part[1024];
    const uint32_t per = (nbins + 1023) / 1024, t = threadIdx.x;
    uint32_t a = 0;
    for (uint32_t q = 0; q < per; q++)
        if (t * per + q < nbins) a += tot[t * per + q];
    part[t] = a;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const uint32_t x = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    uint32_t run = part[t] - a;
    for (uint32_t q = 0; q < per; q++)
        if (t * per + q < nbins) {
            start[t * per + q] = run;
            run += tot[t * per + q];
        }
}

__global__ void __launch_bounds__(1024) bin_scatter_kernel(const uint64_t* keys, uint64_t n, const uint16_t* kbin,
                                                           uint32_t nbins, const uint32_t* H, const uint32_t* start,
                                                           uint64_t* kout, uint32_t* vout) {
    __shared__ uint32_t cur[kBinMax];
    for (uint32_t i = threadIdx.x; i < nbins; i += 1024) cur[i] = start[i] + H[(uint64_t)blockIdx.x * nbins + i];
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b = (uint64_t)blockIdx.x * per, e = b + per < n ? b + per : n;
    for (uint64_t i = b + threadIdx.x; i < e; i += 1024) {
        const uint32_t pos = atomicAdd(&cur[kbin[i]], 1u);
        kout[pos] = keys[i];
        vout[pos] = (uint32_t)i;  // the keys were gathered in record order
    }
}

// Sort bins of size (lo, CAP] in place; workgroups stride over the bins.  Padding
// keys are ~0, which no real key equals (key bytes are never 0xFF); a bin over
// the largest CAP flags the fallback.
template <uint32_t CAP, uint32_t NT>
__global__ void __launch_bounds__(NT) bin_sort_kernel(uint64_t* keys, uint32_t* vals, const uint32_t* start,
                                                      const uint32_t* tot, uint32_t nbins, uint32_t lo, bool flag_over,
                                                      unsigned long long* flags) {
    __shared__ uint64_t K[CAP];
    __shared__ uint32_t V[CAP];
    for (uint32_t bin = blockIdx.x; bin < nbins; bin += gridDim.x) {
        const uint32_t m = tot[bin];
        if (m > CAP) {
            if (flag_over && threadIdx.x == 0) atomicOr(&flags[1], 1ull);
            continue;
        }
        if (m <= lo || m < 2) continue;
        uint32_t P = 2;
        while (P < m) P <<= 1;
        const uint64_t s0 = start[bin];
        for (uint32_t i = threadIdx.x; i < P; i += NT) {
            K[i] = i < m ? keys[s0 + i] : ~0ull;
            V[i] = i < m ? vals[s0 + i] : 0u;
        }
        lds_bitonic<NT, uint64_t>(K, V, P);
        for (uint32_t i = threadIdx.x; i < m; i += NT) {
            keys[s0 + i] = K[i];
            vals[s0 + i] = V[i];
        }
        __syncthreads();  // LDS reused by the workgroup's next bin
    }
}

// keys gathered in record order -> kout sorted, vout the record indices.
// Scratch in ws->bins.
static int bin_sort_pass(ReduceWs* ws, const uint64_t* keys, uint64_t* kout, uint32_t* vout, uint64_t n,
                         unsigned long long* flags, hipStream_t s) {
    uint32_t nbins = 256;
    while (nbins < kBinMax && (uint64_t)nbins * 700 < n) nbins <<= 1;
    uint32_t S = 4 * nbins;
    if (S > kBinSample) S = kBinSample;
    while (S > n && S > 2) S >>= 1;  // (tiny inputs: a sample of distinct positions)
    const uint32_t G = (uint32_t)std::min<uint64_t>(kBinGroups, (n + 4095) / 4096);
    const size_t hbytes = (size_t)G * nbins * 4, kb = (n * 2 + 15) & ~15ull;
    if (hipError_t e = ws->bins.ensure(hbytes + 2 * (size_t)nbins * 4 + (size_t)nbins * 8 + kb + 64)) return (int)e;
    uint32_t* H = ws->bins.as<uint32_t>();
    uint32_t* tot = H + (size_t)G * nbins;
    uint32_t* start = tot + nbins;
    uint64_t* spl = (uint64_t*)(start + nbins);
    uint16_t* kbin = (uint16_t*)(spl + nbins);
    bin_sample_kernel<<<1, 1024, 0, s>>>(keys, n, S, nbins, spl);
    bin_count_kernel<<<G, 1024, 0, s>>>(keys, n, spl, nbins, kbin, H);
    bin_offsets_kernel<<<(nbins + 255) / 256, 256, 0, s>>>(H, G, nbins, tot);
    bin_starts_kernel<<<1, 1024, 0, s>>>(tot, nbins, start);
    bin_scatter_kernel<<<G, 1024, 0, s>>>(keys, n, kbin, nbins, H, start, kout, vout);
    bin_sort_kernel<kBinSmall, 256><<<nbins < 2048 ? nbins : 2048, 256, 0, s>>>(kout, vout, start, tot, nbins, 0, false,
                                                                                  flags);
    bin_sort_kernel<kBinBig, 1024><<<256, 1024, 0, s>>>(kout, vout, start, tot, nbins, kBinSmall, true, flags);
    return (int)hipGetLastError();
}

static inline unsigned grid_for(uint64_t n) {
    uint64_t g = (n + 255) / 256;
    if (g < 1) g = 1;
    if (g > 4096) g = 4096;
    return (unsigned)g;
}

#define RCHK(x)                                   \
    do {                                          \
        hipError_t _e = (x);                      \
        if (_e != hipSuccess) return (int)_e;     \
    } while (0)

// The radix passes are the hand-written ones of mrgpu_sort.hip (no library
// sort on any path: round 5 removed rocPRIM's onesweep, the option own_sort = 0
// is kept for compatibility and runs the same passes).
template <class K>
static int sort_pass(ReduceWs* ws, K* keys_in, K* keys_out, uint32_t* v_in, uint32_t* v_out, uint64_t n, unsigned bits,
                     hipStream_t s) {
    if constexpr (sizeof(K) == 8) return radix_sort_pairs_u64(ws->rx, keys_in, keys_out, v_in, v_out, n, bits, s);
    else return radix_sort_pairs_u32(ws->rx, keys_in, keys_out, v_in, v_out, n, bits, s);
}

int sort_u64_keys(ReduceWs* ws, uint64_t* k_in, uint64_t* k_out, uint64_t n, unsigned bits, hipStream_t s) {
    return radix_sort_keys_u64(ws->rx, k_in, k_out, n, bits, s);
}

// In-place sort of device keys (4 or 8 bytes) with optional u32 values
// (mrg_sort_pairs, a test hook): through the same dispatch as the reduce.
int sort_in_place(ReduceWs* ws, int key_bytes, void* keys, uint32_t* vals, uint64_t n, unsigned bits, hipStream_t s) {
    if (n == 0) return 0;
    if ((key_bytes != 4 && key_bytes != 8) || (!vals && key_bytes != 8)) return (int)hipErrorInvalidValue;
    radix_ws_set_digit_bits(ws->rx, ws->digit_bits);
    void* ko = nullptr;
    uint32_t* vo = nullptr;
    RCHK(hipMalloc(&ko, n * key_bytes));
    if (vals && hipMalloc((void**)&vo, n * 4) != hipSuccess) {
        (void)hipFree(ko);
        return (int)hipErrorOutOfMemory;
    }
    int e;
    if (key_bytes == 4) e = sort_pass<uint32_t>(ws, (uint32_t*)keys, (uint32_t*)ko, vals, vo, n, bits, s);
    else if (vals) e = sort_pass<uint64_t>(ws, (uint64_t*)keys, (uint64_t*)ko, vals, vo, n, bits, s);
    else e = sort_u64_keys(ws, (uint64_t*)keys, (uint64_t*)ko, n, bits, s);
    if (!e) e = (int)hipMemcpyAsync(keys, ko, n * key_bytes, hipMemcpyDeviceToDevice, s);
    if (!e && vals) e = (int)hipMemcpyAsync(vals, vo, n * 4, hipMemcpyDeviceToDevice, s);
    if (!e) e = (int)hipStreamSynchronize(s);
    (void)hipFree(ko);
    if (vo) (void)hipFree(vo);
    return e;
}

int sort_u32_pairs(ReduceWs* ws, uint32_t* k_in, uint32_t* k_out, uint32_t* v_in, uint32_t* v_out, uint64_t n,
                   unsigned bits, hipStream_t s) {
    return sort_pass<uint32_t>(ws, k_in, k_out, v_in, v_out, n, bits, s);
}

// ---- comparison merge sort of u32 items (hand-written; replaces rocPRIM's) --
// Items are record / key indices ordered by a comparator over device memory
// (FullLess, CompactLess).  The keys they name are distinct, so the order is
// total and stability is moot.  Two stages:
//  - tile_sort_kernel: one 1024-thread workgroup sorts kSortTile items by a
//    bitonic network in LDS (the padding past m compares above every item);
//  - merge_pass_kernel: sorted runs of width w merged pairwise into runs of 2w,
//    one item per thread: its rank in the partner run by binary search (left
//    items count the partner's smaller items, right items the partner's items
//    not greater), so each item lands at its own position with no shared
//    cursor — ceil(log2(m / kSortTile)) passes.
constexpr uint32_t kSortTile = 2048;

template <class Less>
__global__ void __launch_bounds__(1024) tile_sort_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                         uint32_t m, Less less) {
    __shared__ uint32_t it[kSortTile];
    const uint32_t base = blockIdx.x * kSortTile;
    for (uint32_t i = threadIdx.x; i < kSortTile; i += 1024) it[i] = base + i < m ? in[base + i] : ~0u;
    __syncthreads();
    for (uint32_t size = 2; size <= kSortTile; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t t = threadIdx.x; t < kSortTile / 2; t += 1024) {
                const uint32_t i = 2 * t - (t & (stride - 1)), j = i + stride;
                const uint32_t A = it[i], B = it[j];
                // A > B; ~0u is padding, above every item
                const bool gt = A == ~0u ? B != ~0u : B != ~0u && less(B, A);
                if (gt == ((i & size) == 0)) {
                    it[i] = B;
                    it[j] = A;
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = threadIdx.x; i < kSortTile; i += 1024)
        if (base + i < m) out[base + i] = it[i];
}

template <class Less>
__global__ void __launch_bounds__(256) merge_pass_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                         uint32_t m, uint32_t w, Less less) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
        const uint64_t blk = i / (2ull * w) * (2ull * w);
        const uint64_t mid = blk + w < m ? blk + w : m, end = blk + 2ull * w < m ? blk + 2ull * w : m;
        const uint32_t x = in[i];
        uint64_t pos;
        if (i < mid) {  // left run: the partner's items less than x come first
            uint64_t lo = mid, hi = end;
            while (lo < hi) {
                const uint64_t md = (lo + hi) >> 1;
                if (less(in[md], x)) lo = md + 1;
                else hi = md;
            }
            pos = (i - blk) + (lo - mid);
        } else {  // right run: the partner's items not greater than x come first
            uint64_t lo = blk, hi = mid;
            while (lo < hi) {
                const uint64_t md = (lo + hi) >> 1;
                if (!less(x, in[md])) lo = md + 1;
                else hi = md;
            }
            pos = (i - mid) + (lo - blk);
        }
        out[blk + pos] = x;
    }
}

// Sorts a[0, m) (device, m known on the host); b is scratch of m items.
// Returns the buffer holding the result (a or b).
template <class Less>
static uint32_t* merge_sort_u32(uint32_t* a, uint32_t* b, uint32_t m, Less less, hipStream_t s) {
    if (m == 0) return a;
    const uint32_t tiles = (m + kSortTile - 1) / kSortTile;
    tile_sort_kernel<<<tiles, 1024, 0, s>>>(a, b, m, less);
    uint32_t *src = b, *dst = a;
    const unsigned g = (unsigned)std::min<uint64_t>(((uint64_t)m + 255) / 256, 4096);
    for (uint64_t w = kSortTile; w < m; w <<= 1) {
        merge_pass_kernel<<<g, 256, 0, s>>>(src, dst, m, (uint32_t)w, less);
        std::swap(src, dst);
    }
    return src;
}

// The members of long tied runs (lng[i] != 0): compacted in order, merge-sorted
// by full (partition, key) comparison, written back to the same positions.  The
// runs are contiguous and already in (partition, prefix) order, which the full
// order refines, so sorting all marked members together keeps every run in its
// own positions.  Scratch: sel (positions), key_b (values, two halves).
static int sort_long_runs(ReduceWs* ws, const Recs& r, uint32_t* perm, uint64_t n, const uint8_t* lng, const uint64_t* ext,
                          hipStream_t s) {
    RCHK(ws->sel.ensure(n * 4 + 1024));
    RCHK(ws->offs.ensure(64));
    uint32_t* pos = ws->sel.as<uint32_t>();
    uint32_t* d_m = ws->offs.as<uint32_t>();
    {
        const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
        ScanState st;
        RCHK(ws->scan.prepare(ntiles, s, &st));
        flag_positions_kernel<<<(unsigned)ntiles, kScanThreads, 0, s>>>(lng, n, pos, d_m, st);
    }
    RCHK(hipMemcpyAsync(ws->h_pinned + 8, d_m, 4, hipMemcpyDeviceToHost, s));
    RCHK(hipStreamSynchronize(s));
    const uint32_t m = (uint32_t)(ws->h_pinned[8] & 0xFFFFFFFFu);
    if (m == 0) return 0;
    static const bool dbg = getenv("MRG_DEBUG_TIES") != nullptr;
    hipEvent_t ev[2];
    if (dbg) {
        for (auto& e : ev) (void)hipEventCreate(&e);
        (void)hipEventRecord(ev[0], s);
    }
    uint32_t* va = ws->key_b.as<uint32_t>();
    uint32_t* vb = va + n;
    const unsigned g = (unsigned)((m + 255) / 256 < 4096 ? (m + 255) / 256 : 4096);
    gather_perm_kernel<<<g, 256, 0, s>>>(perm, pos, d_m, va);
    const uint32_t* sorted;
    if (ext && ws->compact_ties) {
        RCHK(ws->tiek.ensure((size_t)m * (sizeof(TieKey) + 8) + 64));
        TieKey* K = ws->tiek.as<TieKey>();
        uint32_t* ia = (uint32_t*)(K + m);
        uint32_t* ib = ia + m;
        tie_keys_kernel<<<g, 256, 0, s>>>(r, ext, va, d_m, K, ia);
        const uint32_t* io = merge_sort_u32(ia, ib, m, CompactLess{K, r}, s);
        untie_perm_kernel<<<g, 256, 0, s>>>(va, io, d_m, vb);
        sorted = vb;
    } else {
        sorted = merge_sort_u32(va, vb, m, FullLess{r, ext}, s);
    }
    scatter_perm_kernel<<<g, 256, 0, s>>>(perm, pos, d_m, sorted);
    if (dbg) {  // (MRG_DEBUG_TIES: the long runs' sort, gather to scatter, by HIP events)
        (void)hipEventRecord(ev[1], s);
        RCHK(hipStreamSynchronize(s));
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
        fprintf(stderr, "[ties] long runs: %u members merge-sorted in %.1f us\n", m, 1e3 * ms);
        for (auto& e : ev) (void)hipEventDestroy(e);
    }
    return 0;
}

// ---- grep's tied runs (keys equal in (partition, first 16 bytes)) ----------
// After the 16-byte radix sort, C3 has ~90 K tied keys in ~13 K runs: 12 K runs
// of 2-8 keys, ~1.2 K of 9-64, ~120 of 65-1422 (10 GB, R = 10).  Each run is
// ordered on its own, by rank: a key's position in its run = how many run
// members compare less (keys are distinct, so ranks are a permutation):
//  - runs of <= 64 keys: one wave per run, a key per lane, the other members'
//    words broadcast by readlane (no LDS, no barriers);
//  - runs of 65-2048 keys: one 1024-thread workgroup per run, a bitonic sort of
//    member indices over the members' words staged in LDS;
//  - longer runs: marked in `lng` for the merge sort (sort_long_runs).
// Compared: key bytes 16-63 (the ext words), then bytes 64+ from the arena when
// both keys are longer, then the length — the order rec_cmp_ext gives.
constexpr uint32_t kSmallRun = 64, kMidRun = 2048;

__device__ __forceinline__ int tied_cmp(const Recs& r, const uint64_t* ea, uint32_t la, uint32_t ra, const uint64_t* eb,
                                        uint32_t lb, uint32_t rb) {
#pragma unroll
    for (int w = 0; w < kExtWords; w++)
        if (ea[w] != eb[w]) return ea[w] < eb[w] ? -1 : 1;
    constexpr uint32_t kCovered = 16 + 8 * kExtWords;
    if (la > kCovered && lb > kCovered) {
        const uint8_t* pa = r.arena + r.koff[ra];
        const uint8_t* pb = r.arena + r.koff[rb];
        const uint32_t mx = la > lb ? la : lb;
        for (uint32_t pos = kCovered; pos < mx; pos += 8) {
            const uint64_t wa = key_word_be(pa, pos, la), wb = key_word_be(pb, pos, lb);
            if (wa != wb) return wa < wb ? -1 : 1;
        }
    }
    return (la > lb) - (la < lb);
}

// One wave per 64 consecutive group boundaries (bpos: sorted positions that
// start a (partition, prefix) group; cnt[0]'s low half = how many): the wave
// ranks each run of 2-64 keys among them in turn — a key per lane, the other
// members' words broadcast by readlane — and lists runs of 65-kMidRun keys in
// `mid` (cnt[2]); longer runs are listed as kLongChunk-key pieces in `lchunk`
// (cnt[3], marked in lng by mark_chunks_kernel) and flag flags[3].
constexpr uint32_t kLongChunk = 4096;
__global__ void __launch_bounds__(256) rank_small_runs_kernel(Recs r, const uint64_t* ext, uint32_t* perm,
                                                              const uint32_t* bpos, uint64_t n, uint2* mid,
                                                              uint2* lchunk, unsigned long long* cnt,
                                                              unsigned long long* flags) {
    const uint64_t nb = *(const uint32_t*)cnt;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; c * 64 < nb; c += nwaves) {
        const uint64_t j = c * 64 + lane;
        uint32_t bs = 0, bk = 0;
        if (j < nb) {
            bs = bpos[j];
            bk = (uint32_t)((j + 1 < nb ? (uint64_t)bpos[j + 1] : n) - bs);
        }
        if (bk > kSmallRun && bk <= kMidRun) mid[atomicAdd(cnt + 2, 1ull)] = make_uint2(bs, bk);
        if (bk > kMidRun) {
            const uint32_t pieces = (bk + kLongChunk - 1) / kLongChunk;
            const uint64_t at = atomicAdd(cnt + 3, (unsigned long long)pieces);
            for (uint32_t q = 0; q < pieces; q++)
                lchunk[at + q] = make_uint2(bs + q * kLongChunk, std::min(kLongChunk, bk - q * kLongChunk));
            atomicOr(&flags[3], 1ull);
        }
        uint64_t todo = __ballot(bk >= 2 && bk <= kSmallRun);
        while (todo) {
            const uint32_t q = (uint32_t)__builtin_ctzll(todo);
            todo &= todo - 1;
            const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)bs, (int)q);
            const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)bk, (int)q);
            const bool have = lane < k;
            const uint32_t rec = have ? perm[s + lane] : 0u;
            uint64_t e[kExtWords];
#pragma unroll
            for (int w = 0; w < kExtWords; w++) e[w] = have ? ext[(uint64_t)kExtWords * rec + w] : 0ull;
            const uint32_t len = have ? r.len[rec] : 0u;
            uint32_t rank = 0;
            for (uint32_t m = 0; m < k; m++) {
                uint64_t em[kExtWords];
#pragma unroll
                for (int w = 0; w < kExtWords; w++) em[w] = readlane64(e[w], m);
                const uint32_t lm = (uint32_t)__builtin_amdgcn_readlane((int)len, (int)m);
                const uint32_t rm = (uint32_t)__builtin_amdgcn_readlane((int)rec, (int)m);
                // (not against itself: equal words would walk the arena tail)
                if (have && m != lane && tied_cmp(r, em, lm, rm, e, len, rec) < 0) rank++;
            }
            if (have) perm[s + rank] = rec;
        }
    }
}

// The long runs' members, a listed piece per workgroup iteration.
__global__ void __launch_bounds__(256) mark_chunks_kernel(const uint2* lchunk, const unsigned long long* cnt,
                                                          uint8_t* lng) {
    const uint64_t np = cnt[3];
    for (uint64_t c = blockIdx.x; c < np; c += gridDim.x) {
        const uint2 sk = lchunk[c];
        for (uint32_t a = threadIdx.x; a < sk.y; a += blockDim.x) lng[(uint64_t)sk.x + a] = 1;
    }
}

// A run of 65-kMidRun keys per workgroup: a bitonic sort of (first ext word,
// member) items in LDS; items with equal first words compare all words.
struct MidItem {
    uint64_t w;
    uint32_t m, pad;
};
struct MidRunLds {
    MidItem it[kMidRun];
    uint64_t e[kMidRun][kExtWords];
    uint32_t len[kMidRun];
    uint32_t rec[kMidRun];
};

__global__ void __launch_bounds__(1024) rank_mid_runs_kernel(Recs r, const uint64_t* ext, uint32_t* perm,
                                                             const uint2* mid, const unsigned long long* cnt) {
    __shared__ MidRunLds L;
    const uint64_t nruns = cnt[2];
    const uint32_t tid = threadIdx.x;
    for (uint64_t run = blockIdx.x; run < nruns; run += gridDim.x) {
        const uint2 sk = mid[run];
        const uint32_t s = sk.x, k = sk.y;
        uint32_t P = 1;
        while (P < k) P <<= 1;
        for (uint32_t m = tid; m < P; m += 1024) {
            MidItem x;
            x.m = m;  // m >= k: padding, above every member
            x.pad = 0;
            x.w = ~0ull;
            if (m < k) {
                const uint32_t rec = perm[s + m];
                L.rec[m] = rec;
                L.len[m] = r.len[rec];
#pragma unroll
                for (int w = 0; w < kExtWords; w++) L.e[m][w] = ext[(uint64_t)kExtWords * rec + w];
                x.w = L.e[m][0];
            }
            L.it[m] = x;
        }
        __syncthreads();
        for (uint32_t size = 2; size <= P; size <<= 1) {
            for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                for (uint32_t t = tid; t < (P >> 1); t += 1024) {
                    const uint32_t i = 2 * t - (t & (stride - 1));
                    const uint32_t j = i + stride;
                    const MidItem A = L.it[i], B = L.it[j];
                    bool gt;  // item A > item B
                    if (A.w != B.w) {
                        gt = A.w > B.w;
                    } else if (A.m >= k || B.m >= k) {
                        gt = A.m >= k && (B.m < k || A.m > B.m);
                    } else {
                        uint64_t ea[kExtWords], eb[kExtWords];
#pragma unroll
                        for (int w = 0; w < kExtWords; w++) {
                            ea[w] = L.e[A.m][w];
                            eb[w] = L.e[B.m][w];
                        }
                        gt = tied_cmp(r, ea, L.len[A.m], L.rec[A.m], eb, L.len[B.m], L.rec[B.m]) > 0;
                    }
                    if (gt == ((i & size) == 0)) {
                        L.it[i] = B;
                        L.it[j] = A;
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t m = tid; m < k; m += 1024) perm[s + m] = L.rec[L.it[m].m];
        __syncthreads();  // LDS reused by the next run
    }
}

// Orders grep's tied runs after the 16-byte sort (perm = its result; the tie
// marks are written to `tie` by the boundary pass here).  Runs over kMidRun keys are marked in lng and flags[3] is set: the
// caller reads the flag and merge-sorts them (sort_long_runs).
static int rank_tied_runs(ReduceWs* ws, const Recs& r, uint32_t* perm, uint64_t n, uint8_t* tie, uint8_t* lng,
                          const uint64_t* ext, unsigned long long* flags, hipStream_t s) {
    const uint64_t nmid = n / kSmallRun + 2, nlong = n / kLongChunk + n / (kMidRun + 1) + 2;
    RCHK(ws->runs.ensure(64 + (nmid + nlong) * 8));
    unsigned long long* cnt = ws->runs.as<unsigned long long>();
    uint2* mid = (uint2*)(cnt + 8);
    uint2* lchunk = mid + nmid;
    uint32_t* d_nb = (uint32_t*)cnt;  // cnt[0]'s low half
    uint32_t* bpos = ws->key_b.as<uint32_t>();
    RCHK(hipMemsetAsync(cnt, 0, 64, s));
    {  // tie marks + the group boundaries, one look-back launch
        const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
        ScanState st;
        RCHK(ws->scan.prepare(ntiles, s, &st));
        mark_ties_bounds_kernel<<<(unsigned)ntiles, kScanThreads, 0, s>>>(r, perm, n, tie, flags, bpos, d_nb, st);
    }
    static const bool dbg = getenv("MRG_DEBUG_TIES") != nullptr;
    hipEvent_t ev[3];
    if (dbg) {
        for (auto& e : ev) (void)hipEventCreate(&e);
        (void)hipEventRecord(ev[0], s);
    }
    const unsigned g = (unsigned)std::min<uint64_t>((n / 64 + 4) / 4 + 1, 2048);  // 4 waves per block
    rank_small_runs_kernel<<<g, 256, 0, s>>>(r, ext, perm, bpos, n, mid, lchunk, cnt, flags);
    mark_chunks_kernel<<<1024, 256, 0, s>>>(lchunk, cnt, lng);
    if (dbg) (void)hipEventRecord(ev[1], s);
    rank_mid_runs_kernel<<<256, 1024, 0, s>>>(r, ext, perm, mid, cnt);
    if (dbg) {
        (void)hipEventRecord(ev[2], s);
        (void)hipEventSynchronize(ev[2]);
        unsigned long long h[3];
        (void)hipMemcpy(h, cnt, 24, hipMemcpyDeviceToHost);
        float t[2];
        for (int i = 0; i < 2; i++) (void)hipEventElapsedTime(&t[i], ev[i], ev[i + 1]);
        fprintf(stderr, "[ties] n %llu bounds %llu mid %llu: small %.1f us mid %.1f us\n", (unsigned long long)n,
                h[0] & 0xFFFFFFFFull, h[2], 1e3 * t[0], 1e3 * t[1]);
        for (auto& e : ev) (void)hipEventDestroy(e);
    }
    return 0;
}

int select_recs(ReduceWs* ws, const Recs& src, uint32_t mod, uint32_t want, Recs* dst, hipStream_t s) {
    // dst arrays must be preallocated by the caller with src.n capacity; arena shared with src.
    unsigned long long* cnt = nullptr;
    RCHK(ws->flags.ensure(64));
    cnt = ws->flags.as<unsigned long long>();
    RCHK(hipMemsetAsync(cnt, 0, 8, s));
    if (src.n) select_kernel<<<grid_for(src.n), 256, 0, s>>>(src, mod, want, *dst, cnt);
    RCHK(hipMemcpyAsync(ws->h_pinned, cnt, 8, hipMemcpyDeviceToHost, s));
    RCHK(hipStreamSynchronize(s));
    dst->n = ws->h_pinned[0];
    dst->arena = src.arena;
    dst->arena_n = src.arena_n;
    return 0;
}

uint64_t reduce_out_bound(const Recs& r, int app) {
    // a wc line is key + ' ' + <= 20 digits + '\n', a grep line key + ' ' + key + '\n';
    // key bytes past 16 live in the arena
    const uint64_t key_bound = 16 * r.n + r.arena_n;
    return app == 1 ? key_bound + 22 * r.n + 16 : 2 * key_bound + 2 * r.n + 16;
}

// hout (pinned host memory of hout_cap bytes, or null): the output lines are
// written there directly by the formatting kernel (its stores cross PCIe at the
// copy engine's rate, measured 54.8 GB/s, so the write and the transfer overlap
// and the separate device-to-host copy and its host round trip disappear).
// ---- grep: bucketed sort fused with the output ---------------------------
// C3's reduce ended with ~1.45 ms of PCIe: the 78 MB of "L L\n" lines written
// into pinned host memory by write_lines_staged_kernel, after ~0.8 ms of sort
// (17 radix passes, the tied runs ranked) in which the link was idle.  Here the
// lines are cut into bins by rank (sampled splitters over (partition, first key
// bits), as the wc sample sort: equal keys share a bin, bins are contiguous
// ranges of the sorted order), each bin's byte offset comes from a scan of the
// bins' line bytes, and one kernel then sorts each bin in LDS by full bytewise
// order and writes its lines straight out: workgroups that finish sorting a bin
// write while others still sort, so the sort runs under the link's time.
//   gb_key_kernel      key64 = (partition, first 64 - pbits bits of the key)
//   bin_sample_kernel  splitters (shared with the wc sample sort)
//   gb_count_kernel    bin per key; per group: keys and line bytes per bin
//   gb_offsets_kernel  per bin: prefix over the groups, totals (one wave a bin)
//   gb_starts_kernel   exclusive scans of the bins' keys and bytes
//   gb_scatter_kernel  record indices grouped by bin
//   gb_sort_emit_kernel  per bin: LDS bitonic sort (partition, bytes 0-23 from
//                      registers, then rec_cmp_ext), line offsets, lines out
//   gb_part_offsets_kernel  partition offsets from the first line of each
// A bin over kGbCap keys (more than kGbCap lines sharing partition and first
// key bits, e.g. log lines behind one timestamp) flags flags[1]: the caller
// redoes the reduce with the radix passes (its output overwrites everything).
// bins of 2049-4096 keys (gbx_sort_emit_kernel takes the smaller ones): 1024
// threads, 152 KB of LDS, tied keys compared through rec_cmp_ext
constexpr uint32_t kGbCap = 2048;
constexpr uint32_t kGbBigThreads = 1024, kGbBigCap = 4096, kGbBigStage = 12288;
constexpr uint32_t kGbBinMax = 4096;     // bins at most (count kernel LDS: 112 KB)
constexpr uint32_t kGbGroups = 128;      // count / scatter workgroups at most

struct GbEnt {
    uint64_t a, b, c;  // key bytes 0-7, 8-15, 16-23 as big-endian words (zero-padded)
    uint32_t part, idx;
};

// Key128 (hi, lo): (partition, the first 128 - pbits key bits), big-endian:
// lines tie on it about as often as on their first 16 bytes (C3: runs of at
// most ~1.4 K), where an 8-byte prefix put tens of thousands of lines behind
// one Zipf-frequent first word into one bin.
struct Key128 {
    uint64_t hi, lo;
};
__device__ __forceinline__ bool k128_le(const Key128& a, const Key128& b) {
    return a.hi < b.hi || (a.hi == b.hi && a.lo <= b.lo);
}
__device__ __forceinline__ bool k128_gt(const Key128& a, const Key128& b) {
    return a.hi > b.hi || (a.hi == b.hi && a.lo > b.lo);
}

__global__ void gb_key_kernel(Recs r, uint32_t pbits, Key128* key) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.n; i += stride) {
        const uint64_t A = __builtin_bswap64(r.k0[i]), B = __builtin_bswap64(r.k1[i]);
        Key128 k;
        if (pbits) {
            k.hi = ((uint64_t)r.part[i] << (64 - pbits)) | (A >> pbits);
            k.lo = (A << (64 - pbits)) | (B >> pbits);
        } else {
            k.hi = A;
            k.lo = B;
        }
        key[i] = k;
    }
}

// Splitters: one workgroup sorts an evenly spaced sample of S keys in LDS
// (bitonic) and keeps every (S / nbins)-th.
#ifndef MRG_GB_SAMPLE
#define MRG_GB_SAMPLE 8192
#endif
#ifndef MRG_GB_PER_BIN
#define MRG_GB_PER_BIN 256
#endif
constexpr uint32_t kGbSample = MRG_GB_SAMPLE;  // (A/B: 4096 cost 70 us, 8192 ~140 us)
constexpr uint32_t kGbPerBin = MRG_GB_PER_BIN;  // mean keys a bin
__global__ void __launch_bounds__(1024) gb_sample_kernel(const Key128* keys, uint64_t n, uint32_t S, uint32_t nbins,
                                                         Key128* spl) {
    __shared__ Key128 K[kGbSample];
    for (uint32_t i = threadIdx.x; i < S; i += 1024) K[i] = keys[(uint64_t)i * n / S];
    for (uint32_t k = 2; k <= S; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < S / 2; i += 1024) {
                const uint32_t a = 2 * i - (i & (j - 1)), c = a + j;
                const Key128 ka = K[a], kc = K[c];
                if (k128_gt(ka, kc) == ((a & k) == 0)) {
                    K[a] = kc;
                    K[c] = ka;
                }
            }
        }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j + 1 < nbins; j += 1024) spl[j] = K[(uint64_t)(j + 1) * S / nbins];
}

// the number of splitters <= k (nbins - 1 sorted splitters): equal keys share a bin
__device__ __forceinline__ uint32_t gb_bin_of(const Key128* sp, uint32_t nbins, const Key128& k) {
    uint32_t lo = 0, cnt = nbins - 1;
    while (cnt) {
        const uint32_t half = cnt >> 1;
        if (k128_le(sp[lo + half], k)) {
            lo += half + 1;
            cnt -= half + 1;
        } else {
            cnt = half;
        }
    }
    return lo;
}

__global__ void __launch_bounds__(1024) gb_count_kernel(Recs r, const Key128* key, const Key128* spl,
                                                        uint32_t nbins, uint16_t* kbin, uint32_t* H,
                                                        unsigned long long* HB) {
    __shared__ Key128 sp[kGbBinMax];
    __shared__ uint32_t h[kGbBinMax];
    __shared__ unsigned long long hb[kGbBinMax];
    for (uint32_t i = threadIdx.x; i < nbins; i += 1024) {
        h[i] = 0;
        hb[i] = 0;
        if (i + 1 < nbins) sp[i] = spl[i];
    }
    __syncthreads();
    const uint64_t n = r.n, per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b = (uint64_t)blockIdx.x * per, e = b + per < n ? b + per : n;
    for (uint64_t i = b + threadIdx.x; i < e; i += 1024) {
        const uint32_t bin = gb_bin_of(sp, nbins, key[i]);
        kbin[i] = (uint16_t)bin;
        atomicAdd(&h[bin], 1u);
        atomicAdd(&hb[bin], 2ull * r.len[i] + 2ull);  // "L L\n" (dgrep.go:44-46, worker.go:144)
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbins; i += 1024) {
        H[(uint64_t)blockIdx.x * nbins + i] = h[i];
        HB[(uint64_t)blockIdx.x * nbins + i] = hb[i];
    }
}

// One wave per bin: the prefix over the G groups of its key and byte counts
// (in place), the totals in tot / btot.
__global__ void __launch_bounds__(256) gb_offsets_kernel(uint32_t* H, unsigned long long* HB, uint32_t G,
                                                         uint32_t nbins, uint32_t* tot, unsigned long long* btot) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t bin = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (bin >= nbins) return;
    uint32_t run = 0;
    unsigned long long brun = 0;
    for (uint32_t g0 = 0; g0 < G; g0 += 64) {
        const uint32_t g = g0 + lane;
        const uint64_t at = (uint64_t)g * nbins + bin;
        const uint32_t v = g < G ? H[at] : 0u;
        const unsigned long long bv = g < G ? HB[at] : 0ull;
        const uint64_t iv = wave_incl_scan_u64(v), ib = wave_incl_scan_u64(bv);
        if (g < G) {
            H[at] = run + (uint32_t)(iv - v);
            HB[at] = brun + (ib - bv);
        }
        run += (uint32_t)__shfl(iv, 63);
        brun += __shfl(ib, 63);
    }
    if (lane == 0) {
        tot[bin] = run;
        btot[bin] = brun;
    }
}

// start / bstart = exclusive scans of tot / btot (one workgroup); bstart[nbins]
// = the output's total bytes
__global__ void __launch_bounds__(1024) gb_starts_kernel(const uint32_t* tot, const unsigned long long* btot,
                                                         uint32_t nbins, uint32_t* start,
                                                         unsigned long long* bstart) {
    __shared__ unsigned long long pa[1024], pb[1024];
    const uint32_t per = (nbins + 1023) / 1024, t = threadIdx.x;
    unsigned long long a = 0, bb = 0;
    for (uint32_t q = 0; q < per; q++)
        if (t * per + q < nbins) {
            a += tot[t * per + q];
            bb += btot[t * per + q];
        }
    pa[t] = a;
    pb[t] = bb;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {
        const unsigned long long x = t >= d ? pa[t - d] : 0ull, y = t >= d ? pb[t - d] : 0ull;
        __syncthreads();
        pa[t] += x;
        pb[t] += y;
        __syncthreads();
    }
    unsigned long long run = pa[t] - a, brun = pb[t] - bb;
    for (uint32_t q = 0; q < per; q++)
        if (t * per + q < nbins) {
            start[t * per + q] = (uint32_t)run;
            bstart[t * per + q] = brun;
            run += tot[t * per + q];
            brun += btot[t * per + q];
        }
    if (t == 1023) bstart[nbins] = pb[1023];
}

__global__ void __launch_bounds__(1024) gb_scatter_kernel(uint64_t n, const uint16_t* kbin, uint32_t nbins,
                                                          const uint32_t* H, const uint32_t* start, uint32_t* idx) {
    __shared__ uint32_t cur[kGbBinMax];
    for (uint32_t i = threadIdx.x; i < nbins; i += 1024) cur[i] = start[i] + H[(uint64_t)blockIdx.x * nbins + i];
    __syncthreads();
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b = (uint64_t)blockIdx.x * per, e = b + per < n ? b + per : n;
    for (uint64_t i = b + threadIdx.x; i < e; i += 1024) idx[atomicAdd(&cur[kbin[i]], 1u)] = (uint32_t)i;
}

// Bytewise order (worker.go:27 ByKey, partition first): bytes 0-23 from the
// entries, then rec_cmp_ext.  Padding entries (idx ~0) sort last.
__device__ __forceinline__ bool gb_less(const Recs& r, const uint64_t* ext, const GbEnt& x, const GbEnt& y) {
    if (x.part != y.part) return x.part < y.part;
    if (x.a != y.a) return x.a < y.a;
    if (x.b != y.b) return x.b < y.b;
    if (x.c != y.c) return x.c < y.c;
    if (x.idx == ~0u || y.idx == ~0u) return x.idx != ~0u && y.idx == ~0u;
    return rec_cmp_ext(r, ext, x.idx, y.idx) < 0;
}

// One output line "L L\n" (grep: the key twice) at o.
template <class OutPtr>
__device__ __forceinline__ void gb_emit_line(const Recs& r, uint32_t j, OutPtr o) {
    const uint32_t len = r.len[j];
    if (len > 16) {  // arena bytes by aligned 16-byte blocks
        const uint8_t* kb = r.arena + r.koff[j];
        for (int64_t q = 0; q < (int64_t)len;) {
            const uintptr_t a = (uintptr_t)(kb + q), ab = a & ~(uintptr_t)15;
            const int64_t bi = q - (int64_t)(a - ab);
            const uint4 v4 = *(const uint4*)ab;
            const uint32_t w4[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
            for (int bb = 0; bb < 16; bb++) {
                const int64_t k = bi + bb;
                if (k < q || k >= (int64_t)len) continue;
                const uint8_t c = (uint8_t)(w4[bb >> 2] >> (8 * (bb & 3)));
                o[k] = c;
                o[len + 1 + k] = c;
            }
            q = bi + 16;
        }
    } else {
        const uint64_t k0 = r.k0[j], k1 = r.k1[j];
        for (uint32_t k = 0; k < len; k++) {
            const uint8_t c = (uint8_t)((k < 8 ? k0 : k1) >> (8 * (k & 7)));
            o[k] = c;
            o[len + 1 + k] = c;
        }
    }
    o[len] = ' ';
    o[2 * len + 1] = '\n';
}

// Bins of (lo, CAP] keys; a bin over the big variant's CAP flags flags[1].
// EMIT: the bin's lines are written here (staged in LDS); else its sorted
// record indices and global line offsets go to perm_out / off_out for
// write_lines_staged_kernel.
template <uint32_t CAP, uint32_t NT, uint32_t STAGE, bool EMIT>
__global__ void __launch_bounds__(NT) gb_sort_emit_kernel(Recs r, const uint64_t* ext, const uint32_t* idx,
                                                          const uint32_t* start, const uint32_t* tot,
                                                          const unsigned long long* bstart, uint32_t nbins,
                                                          uint32_t lo_keys, bool flag_over, uint8_t* out,
                                                          uint32_t* perm_out, uint64_t* off_out,
                                                          unsigned long long* poff, unsigned long long* flags) {
    __shared__ GbEnt E[CAP];
    __shared__ uint32_t loff[CAP + 1];  // line offsets inside the bin
    __shared__ __attribute__((aligned(16))) uint8_t stage[STAGE];
    __shared__ unsigned long long red[NT / 64];
    constexpr uint32_t PER = CAP / NT, kGbStage = STAGE;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (uint32_t bin = blockIdx.x; bin < nbins; bin += gridDim.x) {
        const uint32_t m = tot[bin];
        if (m <= lo_keys) continue;
        if (m > CAP) {
            if (flag_over && tid == 0) atomicOr(&flags[1], 1ull);
            continue;
        }
        if (flag_over && tid == 0) atomicOr(&flags[0], 1ull);  // a bin past the LDS sort's size: resample next time
        uint32_t P = 1;
        while (P < m) P <<= 1;
        const uint32_t s0 = start[bin];
        for (uint32_t i = tid; i < P; i += NT) {
            GbEnt x;
            if (i < m) {
                const uint32_t j = idx[s0 + i];
                x.a = __builtin_bswap64(r.k0[j]);
                x.b = __builtin_bswap64(r.k1[j]);
                x.c = r.len[j] > 16 ? ext[(uint64_t)kExtWords * j] : 0ull;
                x.part = r.part[j];
                x.idx = j;
            } else {
                x.a = x.b = x.c = ~0ull;
                x.part = ~0u;
                x.idx = ~0u;
            }
            E[i] = x;
        }
        // bitonic network over P entries (swaps of whole entries)
        for (uint32_t k = 2; k <= P; k <<= 1)
            for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
                __syncthreads();
                for (uint32_t i = tid; i < P / 2; i += NT) {
                    const uint32_t a = 2 * i - (i & (jj - 1)), c = a + jj;
                    const GbEnt xa = E[a], xc = E[c];
                    const bool up = (a & k) == 0;
                    if (gb_less(r, ext, xc, xa) == up) {
                        E[a] = xc;
                        E[c] = xa;
                    }
                }
            }
        __syncthreads();
        // line offsets in the bin: thread t takes items [PER t, PER t + PER)
        uint64_t l[PER], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t i = PER * tid + q;
            l[q] = i < m ? 2ull * r.len[E[i].idx] + 2ull : 0ull;
            sum += l[q];
        }
        const uint64_t incl = wave_incl_scan_u64(sum);
        if (lane == 63) red[w] = incl;
        __syncthreads();
        uint64_t pre = 0;
#pragma unroll
        for (uint32_t q = 0; q < NT / 64; q++) pre += q < w ? red[q] : 0ull;
        uint64_t o = pre + incl - sum;
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t i = PER * tid + q;
            if (i < m) loff[i] = (uint32_t)o;
            o += l[q];
        }
        if (tid == NT - 1) loff[m] = (uint32_t)(pre + incl);  // the bin's byte total
        __syncthreads();
        const uint64_t gbase = bstart[bin];
        // the first line of each partition (partitions are contiguous in the sorted order)
        for (uint32_t i = tid; i < m; i += NT)
            if (i == 0 || E[i].part != E[i - 1].part) atomicMin(&poff[E[i].part], gbase + loff[i]);
        if constexpr (!EMIT) {
            for (uint32_t i = tid; i < m; i += NT) {
                perm_out[s0 + i] = E[i].idx;
                off_out[s0 + i] = gbase + loff[i];
            }
            __syncthreads();  // LDS reused by the workgroup's next bin
            continue;
        }
        // lines out, in steps of as many lines as the staging buffer holds
        for (uint32_t i0 = 0; i0 < m;) {
            const uint64_t gs = gbase + loff[i0];
            const uint64_t a0 = gs & ~15ull;
            // lines [i0, i1): the most (<= NT) whose bytes fit the stage from a0
            uint32_t lo = i0 + 1, hi = i0 + NT < m ? i0 + NT : m;  // i1 in [lo, hi]
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (gbase + loff[mid] - a0 <= kGbStage) lo = mid;
                else hi = mid - 1;
            }
            const uint32_t i1 = lo;
            const uint64_t ge = gbase + loff[i1];
            const bool staged = ge - a0 <= kGbStage;  // (false: one line longer than the stage)
            const uint32_t i = i0 + tid;
            if (i < i1) {
                const uint64_t go = gbase + loff[i];
                if (staged) gb_emit_line(r, E[i].idx, stage + (go - a0));
                else gb_emit_line(r, E[i].idx, out + go);
            }
            if (staged) {
                __syncthreads();
                const uint32_t nq = (uint32_t)((ge - a0 + 15) / 16);
                for (uint32_t q = tid; q < nq; q += NT) {
                    const uint64_t ga = a0 + 16ull * q;
                    if (ga >= gs && ga + 16 <= ge) {
                        *(uint4*)(out + ga) = *(const uint4*)(stage + 16 * q);
                    } else {
                        for (uint32_t bb = 0; bb < 16; bb++)
                            if (ga + bb >= gs && ga + bb < ge) out[ga + bb] = stage[16 * q + bb];
                    }
                }
            }
            __syncthreads();
            i0 = i1;
        }
    }
}

// Bins of at most kGbxCap keys (nearly all of them): gb_sort_emit_kernel with
// every compared word in LDS.  An entry holds key bytes 0-23 and the bin-local
// slot of its record; the slot's key bytes 24-63 (ext words 1-5), length and
// record index sit in LDS beside the entries, so lines tied on their first 24
// bytes (C3: lines behind a Zipf-frequent first word and the pattern) compare
// without a global load; only keys equal in their first 64 bytes read the
// arena.  (The first version compared ties through rec_cmp_ext in global
// memory: its per-bin sorts took ~0.5 ms of C3's reduce in total.)
constexpr uint32_t kGbxCap = 2048, kGbxThreads = 1024, kGbxStage = 16384;
constexpr uint32_t kGbxWords = 3;  // ext words 1-3 (key bytes 24-47) in LDS; 4-5 read from ext when tied
struct GbxEnt {
    uint64_t a, b, c;  // key bytes 0-7, 8-15, 16-23, big-endian words (zero-padded)
    uint32_t part, slot;
};

template <bool EMIT>
__global__ void __launch_bounds__(kGbxThreads) gbx_sort_emit_kernel(Recs r, const uint64_t* ext, const uint32_t* idx,
                                                                     const uint32_t* start, const uint32_t* tot,
                                                                     const unsigned long long* bstart, uint32_t nbins,
                                                                     uint8_t* out, uint32_t* perm_out,
                                                                     uint64_t* off_out, unsigned long long* poff) {
    constexpr uint32_t CAP = kGbxCap, NT = kGbxThreads, PER = CAP / NT, NX = kGbxWords;
    __shared__ GbxEnt E[CAP];
    __shared__ uint64_t X[CAP * NX];  // key bytes 24-63 of slot s at X[NX s, NX s + NX)
    __shared__ uint32_t LEN[CAP], IDX[CAP];
    __shared__ uint32_t loff[CAP + 1];
    __shared__ __attribute__((aligned(16))) uint8_t stage[EMIT ? kGbxStage : 16];
    __shared__ unsigned long long red[NT / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    // bytewise order (worker.go:27 ByKey, partition first), exactly rec_cmp_ext's
    auto less = [&](const GbxEnt& x, const GbxEnt& y) -> bool {
        if (x.part != y.part) return x.part < y.part;
        if (x.a != y.a) return x.a < y.a;
        if (x.b != y.b) return x.b < y.b;
        if (x.c != y.c) return x.c < y.c;
        if (x.slot == ~0u || y.slot == ~0u) return x.slot != ~0u && y.slot == ~0u;  // padding last
#pragma unroll
        for (uint32_t q = 0; q < NX; q++) {
            const uint64_t ex = X[NX * x.slot + q], ey = X[NX * y.slot + q];
            if (ex != ey) return ex < ey;
        }
        const uint32_t ia = IDX[x.slot], ib = IDX[y.slot];
#pragma unroll
        for (uint32_t q = 1 + NX; q < (uint32_t)kExtWords; q++) {  // (tied through byte 47: rare)
            const uint64_t ex = ext[(uint64_t)kExtWords * ia + q], ey = ext[(uint64_t)kExtWords * ib + q];
            if (ex != ey) return ex < ey;
        }
        constexpr uint32_t kCovered = 16 + 8 * kExtWords;
        const uint32_t la = LEN[x.slot], lb = LEN[y.slot];
        if (la > kCovered && lb > kCovered) {
            const uint8_t* pa = r.arena + r.koff[ia];
            const uint8_t* pb = r.arena + r.koff[ib];
            const uint32_t mx = la > lb ? la : lb;
            for (uint32_t pos = kCovered; pos < mx; pos += 8) {
                const uint64_t wa = key_word_be(pa, pos, la), wb = key_word_be(pb, pos, lb);
                if (wa != wb) return wa < wb;
            }
        }
        return la < lb;
    };
    for (uint32_t bin = blockIdx.x; bin < nbins; bin += gridDim.x) {
        const uint32_t m = tot[bin];
        if (m == 0 || m > CAP) continue;  // (larger bins: gb_sort_emit_kernel)
        uint32_t P = 1;
        while (P < m) P <<= 1;
        const uint32_t s0 = start[bin];
        for (uint32_t i = tid; i < P; i += NT) {
            GbxEnt x;
            if (i < m) {
                const uint32_t j = idx[s0 + i];
                const uint64_t* e = ext + (uint64_t)kExtWords * j;
                x.a = __builtin_bswap64(r.k0[j]);
                x.b = __builtin_bswap64(r.k1[j]);
                x.c = e[0];  // (zero for keys of <= 16 bytes: ext_words_kernel)
#pragma unroll
                for (uint32_t q = 0; q < NX; q++) X[NX * i + q] = e[1 + q];
                x.part = r.part[j];
                x.slot = i;
                LEN[i] = r.len[j];
                IDX[i] = j;
            } else {
                x.a = x.b = x.c = ~0ull;
                x.part = ~0u;
                x.slot = ~0u;
            }
            E[i] = x;
        }
        for (uint32_t k = 2; k <= P; k <<= 1)
            for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
                __syncthreads();
                for (uint32_t i = tid; i < P / 2; i += NT) {
                    const uint32_t a = 2 * i - (i & (jj - 1)), c = a + jj;
                    const GbxEnt xa = E[a], xc = E[c];
                    if (less(xc, xa) == ((a & k) == 0)) {
                        E[a] = xc;
                        E[c] = xa;
                    }
                }
            }
        __syncthreads();
        uint64_t l[PER], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t i = PER * tid + q;
            l[q] = i < m ? 2ull * LEN[E[i].slot] + 2ull : 0ull;
            sum += l[q];
        }
        const uint64_t incl = wave_incl_scan_u64(sum);
        if (lane == 63) red[w] = incl;
        __syncthreads();
        uint64_t pre = 0;
#pragma unroll
        for (uint32_t q = 0; q < NT / 64; q++) pre += q < w ? red[q] : 0ull;
        uint64_t o = pre + incl - sum;
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t i = PER * tid + q;
            if (i < m) loff[i] = (uint32_t)o;
            o += l[q];
        }
        if (tid == NT - 1) loff[m] = (uint32_t)(pre + incl);
        __syncthreads();
        const uint64_t gbase = bstart[bin];
        for (uint32_t i = tid; i < m; i += NT)
            if (i == 0 || E[i].part != E[i - 1].part) atomicMin(&poff[E[i].part], gbase + loff[i]);
        if constexpr (!EMIT) {
            for (uint32_t i = tid; i < m; i += NT) {
                perm_out[s0 + i] = IDX[E[i].slot];
                off_out[s0 + i] = gbase + loff[i];
            }
        } else {
            for (uint32_t i0 = 0; i0 < m;) {
                const uint64_t gs = gbase + loff[i0];
                const uint64_t a0 = gs & ~15ull;
                uint32_t lo = i0 + 1, hi = i0 + NT < m ? i0 + NT : m;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi + 1) >> 1;
                    if (gbase + loff[mid] - a0 <= kGbxStage) lo = mid;
                    else hi = mid - 1;
                }
                const uint32_t i1 = lo;
                const uint64_t ge = gbase + loff[i1];
                const bool staged = ge - a0 <= kGbxStage;
                const uint32_t i = i0 + tid;
                if (i < i1) {
                    const uint64_t go = gbase + loff[i];
                    const uint32_t j = IDX[E[i].slot];
                    if (staged) gb_emit_line(r, j, stage + (go - a0));
                    else gb_emit_line(r, j, out + go);
                }
                if (staged) {
                    __syncthreads();
                    const uint32_t nq = (uint32_t)((ge - a0 + 15) / 16);
                    for (uint32_t q = tid; q < nq; q += NT) {
                        const uint64_t ga = a0 + 16ull * q;
                        if (ga >= gs && ga + 16 <= ge) {
                            *(uint4*)(out + ga) = *(const uint4*)(stage + 16 * q);
                        } else {
                            for (uint32_t bb = 0; bb < 16; bb++)
                                if (ga + bb >= gs && ga + bb < ge) out[ga + bb] = stage[16 * q + bb];
                        }
                    }
                }
                __syncthreads();
                i0 = i1;
            }
        }
        __syncthreads();  // LDS reused by the workgroup's next bin
    }
}

__global__ void gb_total_kernel(const unsigned long long* total, uint64_t* off_n) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *off_n = *total;
}

// offsets[p] = byte offset of partition p's first line (the next non-empty
// partition's, or the total, when p has none); offsets[nparts] = the total.
__global__ void gb_part_offsets_kernel(const unsigned long long* poff, const unsigned long long* total, uint32_t nparts,
                                       uint64_t* offsets) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    uint64_t next = *total;
    offsets[nparts] = next;
    for (uint32_t p = nparts; p-- > 0;) {
        if (poff[p] != ~0ull) next = poff[p];
        offsets[p] = next;
    }
}

// The fused grep reduce; returns 0, or a HIP error.  *over = a bin was too
// large (nothing usable was written: the caller runs the radix path).
static int grep_bin_reduce(ReduceWs* ws, const Recs& r, uint32_t nreduce, uint8_t* out, uint64_t* h_offsets,
                           bool* over, bool emit, hipStream_t s) {
    const uint64_t n = r.n;
    uint32_t pbits = 0;
    while (nreduce > 1 && (1ull << pbits) < nreduce) pbits++;
    // ~512 keys a bin on average and >= 4 samples a bin (bins cut by sampled
    // rank: fewer samples a bin spread the sizes past kGbxCap)
    uint32_t nbins = 1;
    while (nbins < kGbBinMax && (uint64_t)nbins * kGbPerBin < n) nbins <<= 1;
    uint32_t S = 8 * nbins;
    if (S > kGbSample) S = kGbSample;
    while (S > n && S > 2) S >>= 1;
    const uint32_t G = (uint32_t)std::min<uint64_t>(kGbGroups, (n + 4095) / 4096);
    // scratch: key64 (key_b), idx (perm_a); bins: H, HB, tot, btot, start, bstart, spl, kbin, poff
    const size_t hb = (size_t)G * nbins * 4, hbb = (size_t)G * nbins * 8;
    const size_t need = hbb + hb + (size_t)nbins * (4 + 8 + 4 + 8) + 8 + n * 2 + 16 + (size_t)(nreduce + 1) * 8 + 256;
    RCHK(ws->bins.ensure(need));
    uint8_t* p8 = ws->bins.as<uint8_t>();
    unsigned long long* HB = (unsigned long long*)p8;            p8 += hbb;
    unsigned long long* btot = (unsigned long long*)p8;          p8 += (size_t)nbins * 8;
    unsigned long long* bstart = (unsigned long long*)p8;        p8 += (size_t)nbins * 8 + 8;
    unsigned long long* poff = (unsigned long long*)p8;          p8 += (size_t)(nreduce + 1) * 8;
    uint32_t* H = (uint32_t*)p8;                                  p8 += hb;
    uint32_t* tot = (uint32_t*)p8;                                p8 += (size_t)nbins * 4;
    uint32_t* start = (uint32_t*)p8;                              p8 += (size_t)nbins * 4;
    uint16_t* kbin = (uint16_t*)p8;
    Key128* key = ws->ext.as<Key128>() + (size_t)n * kExtWords / 2;  // (ext holds n x kExtWords words, then these)
    uint32_t* idx = ws->perm_a.as<uint32_t>();
    unsigned long long* flags = ws->flags.as<unsigned long long>();
    const uint32_t nparts = nreduce;
    RCHK(hipMemsetAsync(poff, 0xFF, (size_t)nparts * 8, s));
    gb_key_kernel<<<grid_for(n), 256, 0, s>>>(r, pbits, key);
    RCHK(ws->gb_spl.ensure((size_t)kGbBinMax * sizeof(Key128)));
    Key128* spl = ws->gb_spl.as<Key128>();
    const bool reuse = ws->gb_warm && ws->gb_ok && nbins == ws->gb_nbins && pbits == ws->gb_pbits &&
                       n >= ws->gb_n / 2 && n <= 2 * ws->gb_n;
    if (!reuse) gb_sample_kernel<<<1, 1024, 0, s>>>(key, n, S, nbins, spl);
    gb_count_kernel<<<G, 1024, 0, s>>>(r, key, spl, nbins, kbin, H, HB);
    gb_offsets_kernel<<<(nbins + 3) / 4, 256, 0, s>>>(H, HB, G, nbins, tot, btot);
    gb_starts_kernel<<<1, 1024, 0, s>>>(tot, btot, nbins, start, bstart);
    gb_scatter_kernel<<<G, 1024, 0, s>>>(n, kbin, nbins, H, start, idx);
    uint32_t* perm = ws->perm_b.as<uint32_t>();
    uint64_t* off = ws->lineoff.as<uint64_t>();
    const uint64_t* ext = ws->ext.as<uint64_t>();
    if (emit) {  // the lines written by the sorting workgroups
        gbx_sort_emit_kernel<true><<<nbins < 256 ? nbins : 256, kGbxThreads, 0, s>>>(r, ext, idx, start, tot, bstart,
                                                                                   nbins, out, perm, off, poff);
        gb_sort_emit_kernel<kGbBigCap, kGbBigThreads, kGbBigStage, true><<<nbins < 256 ? nbins : 256, kGbBigThreads, 0,
                                                                          s>>>(
            r, ext, idx, start, tot, bstart, nbins, kGbCap, true, out, perm, off, poff, flags);
    } else {  // sorted order + line offsets, then the line writer over all of them
        gbx_sort_emit_kernel<false><<<nbins < 256 ? nbins : 256, kGbxThreads, 0, s>>>(r, ext, idx, start, tot, bstart,
                                                                                    nbins, out, perm, off, poff);
        gb_sort_emit_kernel<kGbBigCap, kGbBigThreads, 16, false><<<nbins < 256 ? nbins : 256, kGbBigThreads, 0, s>>>(
            r, ext, idx, start, tot, bstart, nbins, kGbCap, true, out, perm, off, poff, flags);
        gb_total_kernel<<<1, 64, 0, s>>>(bstart + nbins, off + n);
        const unsigned g = (unsigned)std::min<uint64_t>((n + wl_lines<2>() - 1) / wl_lines<2>(), 8192);
        write_lines_staged_kernel<2><<<g, kWlLines, 0, s>>>(r, perm, n, off, out, flags + 1);
    }
    gb_part_offsets_kernel<<<1, 64, 0, s>>>(poff, bstart + nbins, nparts, ws->offs.as<uint64_t>());
    RCHK(hipGetLastError());
    RCHK(hipMemcpyAsync(h_offsets, ws->offs.p, (size_t)(nparts + 1) * 8, hipMemcpyDeviceToHost, s));
    RCHK(hipMemcpyAsync(ws->h_pinned + 8, flags, 16, hipMemcpyDeviceToHost, s));  // flags 0 (big bins), 1 (over)
    RCHK(hipStreamSynchronize(s));
    *over = ws->h_pinned[9] != 0;
    ws->gb_ok = ws->h_pinned[8] == 0 && ws->h_pinned[9] == 0;
    ws->gb_nbins = nbins;
    ws->gb_pbits = pbits;
    ws->gb_n = n;
    return 0;
}

int reduce_format(ReduceWs* ws, const Recs& r, int app, uint32_t nreduce, uint32_t only_part, uint8_t** d_out,
                  uint64_t* out_n, uint64_t* h_offsets, hipStream_t s, bool ascii_keys, uint8_t* hout, uint64_t hout_cap) {
    const uint64_t n = r.n;
    const bool all = only_part == 0xFFFFFFFFu;
    const uint32_t nparts = all ? nreduce : 1;
    if (n == 0) {
        for (uint32_t p = 0; p <= nparts; p++) h_offsets[p] = 0;
        *out_n = 0;
        RCHK(ws->out.ensure(16));
        *d_out = ws->out.as<uint8_t>();
        return 0;
    }
    RCHK(ws->flags.ensure(64));
    unsigned long long* flags = ws->flags.as<unsigned long long>();
    RCHK(ws->perm_a.ensure(n * 4));
    RCHK(ws->perm_b.ensure(n * 4));
    RCHK(ws->key_a.ensure(n * 8));
    RCHK(ws->key_b.ensure(n * 8));
    RCHK(ws->lineoff.ensure(n * 8 + 8));
    // Output bytes, bounded up front so nothing waits for the exact total
    const uint64_t bound = reduce_out_bound(r, app);
    const bool to_host = hout != nullptr && bound <= hout_cap;
    if (!to_host) RCHK(ws->out.ensure(bound));
    RCHK(ws->offs.ensure((size_t)(nparts + 1) * 8));
    RCHK(hipMemsetAsync(flags, 0, 32, s));

    uint32_t* pa = ws->perm_a.as<uint32_t>();
    uint32_t* pb = ws->perm_b.as<uint32_t>();
    // grep keys are whole lines (> 16 bytes, often sharing their first words):
    // sort with the k1 pass from the start; ties merge-sort on the ext words
    // (measured: two more 64-bit radix passes over bytes 16-31 cost more, ~16
    // launches, than the larger merge sort they save)
    const bool grep = app != 1;
    const bool k1_first = grep && ws->grep_k1;
    // radix digits (mrgpu_sort.hip): 8 bits; option sort_digit_bits = 10 for
    // 10-bit ones (fewer, wider passes: measured no faster)
    radix_ws_set_digit_bits(ws->rx, ws->digit_bits);
    const uint64_t* ext = nullptr;
    if (grep) {
        RCHK(ws->ext.ensure(n * 8 * kExtWords + n * 16 + 16));  // (+ grep_bin_reduce's 16-byte keys)
        ext_words_kernel<<<grid_for(n), 256, 0, s>>>(r, ws->ext.as<uint64_t>());
        ext = ws->ext.as<uint64_t>();
    }
    // grep, every partition, lines written into pinned host memory: the
    // bucketed sort fused with the output (above), whose sorting runs under the
    // PCIe time; the radix path below when a bin was too large, and for a device
    // output buffer (mrg_run_job_async: the transfer overlaps the next job on
    // another stream, and with nothing to hide under, the bin sorts measured
    // slower than the radix passes: C3 pipelined 2557 vs 2664 GB/s)
    // (grep_bins: 0 radix path; 1 bins fused with the output into host memory
    // (default), radix for a device buffer; 2 / 3 bins for any output: sorted
    // order then the line writer / fused, for tests and A/B)
    if (grep && all && (ws->grep_bins >= 2 || (to_host && ws->grep_bins == 1)) && n <= 0xFFFFFFFFull) {
        bool over = false;
        uint8_t* o = to_host ? hout : ws->out.as<uint8_t>();
        if (int e = grep_bin_reduce(ws, r, nreduce, o, h_offsets, &over, ws->grep_bins != 2, s)) return e;
        if (!over) {
            *d_out = o;
            *out_n = h_offsets[nparts];
            return 0;
        }
        RCHK(hipMemsetAsync(flags, 0, 32, s));
    }
    auto pass32 = [&](int which, unsigned bits) -> int {
        gather_key_kernel<<<grid_for(n), 256, 0, s>>>(r, pa, n, which, nullptr, ws->key_a.as<uint32_t>());
        int e = sort_pass<uint32_t>(ws, ws->key_a.as<uint32_t>(), ws->key_b.as<uint32_t>(), pa, pb, n, bits, s);
        std::swap(pa, pb);
        return e;
    };
    auto pass64 = [&](int which, uint32_t fold = 0, bool first = false, unsigned bits = 64) -> int {
        // first: the permutation is the identity (keys gathered in record order)
        gather_key_kernel<<<grid_for(n), 256, 0, s>>>(r, first ? nullptr : pa, n, which, ws->key_a.as<uint64_t>(),
                                                      nullptr, fold);
        if (first) iota_kernel<<<grid_for(n), 256, 0, s>>>(pa, n);
        int e = sort_pass<uint64_t>(ws, ws->key_a.as<uint64_t>(), ws->key_b.as<uint64_t>(), pa, pb, n, bits, s);
        std::swap(pa, pb);
        return e;
    };
    // partition bits folded into the k0 key's top (wc without the k1 pass): one
    // 64-bit pass orders (partition, first 64 - pbits key bits); keys equal there
    // are tied runs for fix_ties
    uint32_t pbits = 0;
    if (all && nreduce > 1)
        while ((1ull << pbits) < nreduce) pbits++;
    const uint32_t fold = ws->fold_part && pbits > 0 && pbits <= 16 ? pbits : 0;
    // ASCII keys (the map saw no byte >= 0x80): (partition, 7 bits per byte of the
    // first 8 bytes) loses nothing and sorts 56 + pbits bits
    const bool packed = ws->fold_part && ascii_keys && pbits <= 8 && !grep;
    bool keys_sorted = false;  // key_b holds the sort keys of the single (partition, prefix) pass
    bool keys32 = false;       // ... as u32 (the 32-bit prefix pass)
    // Stable LSD passes: (k1), k0, partition.  The k1 pass (bytes 8-15) is
    // skipped at first: keys that share their first 8 bytes form short tied runs
    // that fix_ties orders by full comparison; if a run is long (many keys with
    // one 8-byte prefix), everything is sorted again with the k1 pass.
    // the single-key pass by the hand-written bucketed sort (bins of the
    // partition and the first key bits); the radix passes when a bin overflowed
    bool use_bins = ws->bin_sort;
    auto bin_pass = [&](int which, uint32_t fold_bits) -> int {
        gather_key_kernel<<<grid_for(n), 256, 0, s>>>(r, nullptr, n, which, ws->key_a.as<uint64_t>(), nullptr, fold_bits);
        int e = bin_sort_pass(ws, ws->key_a.as<uint64_t>(), ws->key_b.as<uint64_t>(), pb, n, flags, s);
        std::swap(pa, pb);
        return e;
    };
    auto sort_all = [&](bool with_k1) -> int {
        int e;
        keys_sorted = !with_k1 && (packed || fold);
        // (ASCII keys only: 28 bits are their first 4 characters; a UTF-8 key's
        // first 3.5 bytes are ~2 Greek or Cyrillic letters, and C2u's tied runs then
        // took the slow long-run path: reduce 0.52 -> 1.57 ms)
        keys32 = keys_sorted && ws->prefix32 && !use_bins && packed;
        if (keys32) {  // top 32 bits of the (partition, prefix) key: u32 pairs, 4 passes
            gather_key_kernel<<<grid_for(n), 256, 0, s>>>(r, nullptr, n, packed ? 6 : 7, nullptr, ws->key_a.as<uint32_t>(),
                                                          packed ? pbits : fold);
            iota_kernel<<<grid_for(n), 256, 0, s>>>(pa, n);
            e = sort_pass<uint32_t>(ws, ws->key_a.as<uint32_t>(), ws->key_b.as<uint32_t>(), pa, pb, n, 32, s);
            std::swap(pa, pb);
            return e;
        }
        if (!with_k1 && packed) return use_bins ? bin_pass(5, 0) : pass64(5, 0, true, 56 + pbits);
        if (!with_k1 && fold) return use_bins ? bin_pass(4, fold) : pass64(4, fold, true);
        if (with_k1) {
            if ((e = pass64(1, 0, true))) return e;
            if ((e = pass64(2))) return e;
        } else if ((e = pass64(2, 0, true))) {
            return e;
        }
        if (pbits && (e = pass32(3, pbits))) return e;
        return 0;
    };
    // Tied runs of up to kMaxRun are insertion-sorted in place (one thread per
    // run); longer ones are marked.  Returns whether any run was long; with
    // `merge`, the long runs are then merge-sorted by full comparison.
    constexpr uint64_t kMaxRun = kTailWindow;  // mark_long_tail_kernel's window
    auto fix_ties = [&](bool with_k1, bool merge, bool* any_long, bool all_runs = false) -> int {
        uint8_t* tie = ws->key_a.as<uint8_t>();
        uint8_t* lng = tie + n;
        RCHK(hipMemsetAsync(lng, 0, n, s));
        RCHK(hipMemsetAsync(flags + 2, 0, 16, s));
        if (!with_k1 && keys32) mark_ties_sorted32_kernel<<<grid_for(n), 256, 0, s>>>(ws->key_b.as<uint32_t>(), n, tie, flags);
        else if (!with_k1 && keys_sorted) mark_ties_sorted_kernel<<<grid_for(n), 256, 0, s>>>(ws->key_b.as<uint64_t>(), n, tie, flags);
        else mark_ties_kernel<<<grid_for(n), 256, 0, s>>>(r, pa, n, tie, flags, with_k1, with_k1 ? 0u : fold);
        if (all_runs) {  // every tied run goes to the merge sort (no per-run insertion sort)
            mark_all_ties_kernel<<<grid_for(n), 256, 0, s>>>(tie, n, lng);
            RCHK(hipMemcpyAsync(ws->h_pinned + 3, flags + 2, 8, hipMemcpyDeviceToHost, s));
            RCHK(hipStreamSynchronize(s));
            *any_long = ws->h_pinned[3] != 0;
            return *any_long ? sort_long_runs(ws, r, pa, n, lng, ext, s) : 0;
        }
        fix_ties_kernel<<<grid_for(n), 256, 0, s>>>(r, pa, n, tie, kMaxRun, flags, lng);
        if (merge) mark_long_tail_kernel<<<grid_for((n + 63) / 64), 256, 0, s>>>(tie, n, lng);
        RCHK(hipMemcpyAsync(ws->h_pinned + 1, flags + 1, 24, hipMemcpyDeviceToHost, s));  // flags 1-3
        RCHK(hipStreamSynchronize(s));
        *any_long = ws->h_pinned[3] != 0;
        if (*any_long && merge) return sort_long_runs(ws, r, pa, n, lng, ext, s);
        return 0;
    };
    int e;
    if ((e = sort_all(k1_first))) return e;
    // grep after the 16-byte passes: tied runs ranked per run, speculatively (the
    // output is written, then the long-run flag read: only runs over kMidRun keys
    // redo the output after a merge sort)
    const bool rank_ties = grep && k1_first && ws->tie_rank;
    if (rank_ties) {
        uint8_t* tie = ws->key_a.as<uint8_t>();
        RCHK(hipMemsetAsync(tie + n, 0, n, s));
        RCHK(hipMemsetAsync(flags + 2, 0, 16, s));
        // (the tie marks are made by rank_tied_runs' boundary pass)
        if ((e = rank_tied_runs(ws, r, pa, n, tie, tie + n, ext, flags, s))) return e;
    } else if (grep) {  // every tied run (equal first 16, or with !grep_k1 first 8 - pbits / 8, bytes) merge-sorted
        bool any_long = false;
        if ((e = fix_ties(k1_first, true, &any_long, true))) return e;
    }
    uint8_t* out = to_host ? hout : ws->out.as<uint8_t>();
    // line lengths, their scan, the lines, the partition offsets (copied to the host)
    auto emit_output = [&]() -> int {
        uint64_t* off = ws->lineoff.as<uint64_t>();  // n + 1 offsets
        const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
        ScanState st;
        RCHK(ws->scan.prepare(ntiles, s, &st));
        if (app != 1) line_offsets_kernel<2><<<(unsigned)ntiles, kScanThreads, 0, s>>>(r, pa, n, off, st);
        else line_offsets_kernel<1><<<(unsigned)ntiles, kScanThreads, 0, s>>>(r, pa, n, off, st);
        if (app != 1) {
            const unsigned g = (unsigned)std::min<uint64_t>((n + wl_lines<2>() - 1) / wl_lines<2>(), 8192);
            write_lines_staged_kernel<2><<<g, kWlLines, 0, s>>>(r, pa, n, off, out, nullptr);
        } else {
            const unsigned g = (unsigned)std::min<uint64_t>((n + wl_lines<1>() - 1) / wl_lines<1>(), 8192);
            write_lines_staged_kernel<1><<<g, kWlLines, 0, s>>>(r, pa, n, off, out, nullptr);
        }
        part_offsets_kernel<<<(nparts + 1 + 255) / 256, 256, 0, s>>>(r, pa, n, off, nparts, !all, ws->offs.as<uint64_t>());
        RCHK(hipMemcpyAsync(h_offsets, ws->offs.p, (size_t)(nparts + 1) * 8, hipMemcpyDeviceToHost, s));
        return 0;
    };
    if (!grep) {
        // Speculative: the single key pass's tied runs are fixed and the output is
        // written without a host check in between; the fix-up's flags come back
        // with the partition offsets (one host round trip for the whole reduce).
        // Only if a run was long (or a bin overflowed) is the output redone.
        // (lng is not cleared here: it is read only by the long-run path below,
        // which clears and recomputes it.)
        uint8_t* tie = ws->key_a.as<uint8_t>();
        if (keys32) mark_ties_sorted32_kernel<<<grid_for(n), 256, 0, s>>>(ws->key_b.as<uint32_t>(), n, tie, flags);
        else if (keys_sorted) mark_ties_sorted_kernel<<<grid_for(n), 256, 0, s>>>(ws->key_b.as<uint64_t>(), n, tie, flags);
        else mark_ties_kernel<<<grid_for(n), 256, 0, s>>>(r, pa, n, tie, flags, false, fold);
        fix_ties_kernel<<<grid_for(n), 256, 0, s>>>(r, pa, n, tie, kMaxRun, flags, tie + n);
        if ((e = emit_output())) return e;
        RCHK(hipMemcpyAsync(ws->h_pinned + 1, flags + 1, 24, hipMemcpyDeviceToHost, s));  // flags 1-3
        RCHK(hipStreamSynchronize(s));
        const bool bins_over = use_bins && keys_sorted && ws->h_pinned[1];
        bool any_long = ws->h_pinned[3] != 0;
        if (bins_over || any_long) {
            // keys of 9-16 bytes sharing an 8-byte prefix in a long run: sort again with
            // the k1 pass (cheaper than a comparison sort); any other long run (keys
            // > 16 bytes; 8-byte keys differing in the folded-away bits): comparison
            // merge sort of the run members
            // (a run over 64 needs 65 distinct keys sharing the sort key's prefix:
            // 9-16-byte keys, or longer ones; <= 8-byte keys differ within 2^fold)
            if (bins_over) {  // a bin overflowed: the whole pass again with the radix passes
                use_bins = false;
                RCHK(hipMemsetAsync(flags + 1, 0, 8, s));
                if ((e = sort_all(false))) return e;
                if ((e = fix_ties(false, false, &any_long))) return e;
            }
            if (any_long) {
                if ((e = sort_all(true))) return e;
                if ((e = fix_ties(true, true, &any_long))) return e;
            }
            if ((e = emit_output())) return e;
        }
    } else if (rank_ties) {
        if ((e = emit_output())) return e;
        RCHK(hipMemcpyAsync(ws->h_pinned + 3, flags + 3, 8, hipMemcpyDeviceToHost, s));
        RCHK(hipStreamSynchronize(s));
        if (ws->h_pinned[3]) {  // runs over kMidRun keys: merge-sorted, the output redone
            uint8_t* tie = ws->key_a.as<uint8_t>();
            if ((e = sort_long_runs(ws, r, pa, n, tie + n, ext, s))) return e;
            if ((e = emit_output())) return e;
        }
    } else if ((e = emit_output())) {
        return e;
    }
    RCHK(hipStreamSynchronize(s));
    *d_out = out;
    *out_n = h_offsets[nparts];
    return 0;
}

}  // namespace mrg
