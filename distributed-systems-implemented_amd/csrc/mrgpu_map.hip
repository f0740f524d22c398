// mrgpu_map.hip — Map side of the MI355X MapReduce hot path (gfx950).
//
// wc (MapReduce/mrapps/wc.go:21-34 + mr/worker.go:72-78):
//   One wave owns a 2 KiB chunk of input at a time (plus a 16 B look-back and a
//   64 B look-ahead halo).  Lanes load 16 B each (two coalesced 1 KiB wave loads),
//   stage the bytes in the wave's LDS slice and classify them:
//     * ASCII chunks (wave-uniform test): SWAR letter test, 4 bytes per op;
//     * otherwise a Go-exact UTF-8 decode (utf8.DecodeRune acceptance ranges,
//       invalid byte = U+FFFD width 1) + unicode.IsLetter via a two-level bitmap.
//   A word is a maximal run of letter bytes (strings.FieldsFunc with
//   !unicode.IsLetter).  Word starts are compacted with ballot/mbcnt prefix sums
//   into an LDS list, then each lane takes one word: its length comes from the
//   letter bitmaps (ctz), its <= 16 key bytes are packed into two u64 with
//   v_alignbyte, and the word is counted in the workgroup's LDS hash table (the
//   combiner: every wc value is "1", so Reduce(len(values)) == sum of counts).
//   Misses (table full) and the final LDS flush go to the HBM ShortTable; words
//   longer than 16 bytes go to a list handled by wc_long_kernel.
//   ihash (FNV-1a) is computed once per *distinct* key in collect_kernel — the
//   partition is a pure function of the key, so this equals the per-KV
//   ihash(kv.Key) % NReduce of worker.go:76 with W/U times fewer hashes.
//
// grep (MapReduce/mrapps/dgrep.go:18-36): streaming literal search (first-byte
//   SWAR filter, LDS verify); each hit's line (strings.Split on "\n") is
//   resolved and inserted, deduplicated by content, into the LongTable.
#include "mrgpu_internal.h"

namespace mrg {

constexpr int kChunk = 1024;                      // bytes per wave-chunk (16 B per lane)
constexpr int kBack = 16;
constexpr int kAhead = 64;
constexpr int kBuf = kBack + kChunk + kAhead;  // 1104, multiple of 16
constexpr int kWavesPerWG = 16;
constexpr int kThreads = kWavesPerWG * kWave;
constexpr int kListCap = kChunk / 2;              // max word starts in a chunk
constexpr int kLdsSets = 1536;                    // map-side combiner (per workgroup): 4-way sets
constexpr int kAggThreads = 512;
constexpr int kAggSets = 960;                     // bucket aggregator (half the LDS: 2 workgroups per CU)
constexpr int kGlobalProbes = 4096;

struct alignas(16) WaveLds {
    uint8_t buf[kBuf];
    uint16_t list[kListCap];
};

// LDS hash table, 4-way set associative: the 4 k0 of a set are 32 contiguous
// bytes (two ds_read_b128), so a lookup is a handful of VALU ops and no probe
// loop.  A way is claimed by CAS on its k0 (0 -> key), then k1 is published
// (k1 == kUnwritten until then; 0xFF bytes never occur in a UTF-8 key).
template <int NSETS>
struct alignas(16) STable {
    unsigned long long k0[NSETS * 4];
    unsigned long long k1[NSETS * 4];
    uint32_t cnt[NSETS * 4];
};

struct alignas(16) MapLds {
    WaveLds w[kWavesPerWG];
    STable<kLdsSets> T;
    uint32_t cur[kSpillBuckets];     // records appended to this workgroup's 16-byte stream of each bucket
    uint32_t cur8[kSpillBuckets];    // ... and to its 8-byte stream
};

struct alignas(16) AggLds {
    STable<kAggSets> T;
    uint32_t nmiss;  // keys appended to the bucket's miss list
};

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ const uint8_t* ld_agent_ptr(const uint8_t* const* p) {
    return __hip_atomic_load(const_cast<const uint8_t**>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void set_status(Counters* c, uint32_t bits) { atomicOr(&c->status, bits); }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Exclusive prefix sum over the wave of c (0 <= c < 32) by ballot bit-planes.
__device__ __forceinline__ uint32_t wave_excl_scan5(uint32_t c, uint32_t* total) {
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 5; k++) {
        uint64_t b = __ballot((c >> k) & 1u);
        base += mbcnt64(b) << k;
        tot += (uint32_t)__popcll(b) << k;
    }
    *total = tot;
    return base;
}

// 4 ASCII bytes -> 4-bit letter mask ([A-Za-z]); requires every byte < 0x80.
__device__ __forceinline__ uint32_t ascii_letters4(uint32_t x) {
    uint32_t y = x | 0x20202020u;
    uint32_t t = (y + 0x1F1F1F1Fu) & ~(y + 0x05050505u) & 0x80808080u;
    return ((t >> 7) * 0x10204080u) >> 28;
}
__device__ __forceinline__ uint32_t ascii_mask16(uint4 v) {
    return ascii_letters4(v.x) | (ascii_letters4(v.y) << 4) | (ascii_letters4(v.z) << 8) | (ascii_letters4(v.w) << 12);
}

__device__ __forceinline__ bool is_letter_cp(uint32_t cp, LetterTables lt) {
    if (cp < 0x80) return ((cp | 0x20u) - 0x61u) < 26u;
    uint32_t idx = lt.l1[cp >> 8];
    return (lt.l2[idx * 8 + ((cp >> 5) & 7)] >> (cp & 31)) & 1u;
}

// Go utf8 acceptance: length of the valid sequence starting with bytes c0..c3, or 0.
__device__ __forceinline__ int utf8_valid_len(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    if (c0 < 0x80) return 1;
    if (c0 < 0xC2 || c0 > 0xF4) return 0;
    uint32_t lo = 0x80, hi = 0xBF;
    if (c0 == 0xE0) lo = 0xA0;
    else if (c0 == 0xED) hi = 0x9F;
    else if (c0 == 0xF0) lo = 0x90;
    else if (c0 == 0xF4) hi = 0x8F;
    if (c1 < lo || c1 > hi) return 0;
    if (c0 < 0xE0) return 2;
    if ((c2 & 0xC0) != 0x80) return 0;
    if (c0 < 0xF0) return 3;
    if ((c3 & 0xC0) != 0x80) return 0;
    return 4;
}

__device__ __forceinline__ uint32_t utf8_decode(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, int n) {
    if (n == 1) return c0;
    if (n == 2) return ((c0 & 0x1F) << 6) | (c1 & 0x3F);
    if (n == 3) return ((c0 & 0x0F) << 12) | ((c1 & 0x3F) << 6) | (c2 & 0x3F);
    return ((c0 & 0x07) << 18) | ((c1 & 0x3F) << 12) | ((c2 & 0x3F) << 6) | (c3 & 0x3F);
}

// Letter mask of the W bytes at b[q0 .. q0+W) with Go decoding semantics.
// Needs b[q0-6 .. q0+W+3) addressable (zeros outside the input act as
// non-continuation terminators, matching Go's truncated-sequence rule).
// Rune starts use the local rule: byte q starts a rune unless a valid sequence
// of length > k starts at q-k, k in {1,2,3}.
template <int W>
__device__ uint32_t utf8_letter_mask(const uint8_t* b, int q0, LetterTables lt) {
    uint32_t mask = 0;
    int vl1 = 0, vl2 = 0, vl3 = 0;  // valid lengths at q-1, q-2, q-3
    for (int q = q0 - 6; q < q0 + W; q++) {
        uint32_t c0 = b[q], c1 = b[q + 1], c2 = b[q + 2], c3 = b[q + 3];
        int vl = utf8_valid_len(c0, c1, c2, c3);
        if (q >= q0 - 3) {
            bool start = !(vl1 >= 2 || vl2 >= 3 || vl3 >= 4);
            if (start) {
                bool let = vl > 0 && is_letter_cp(utf8_decode(c0, c1, c2, c3, vl), lt);
                if (let) {
                    for (int k = 0; k < vl; k++) {
                        int pos = q + k - q0;
                        if (pos >= 0 && pos < W) mask |= 1u << pos;
                    }
                }
            }
        }
        vl3 = vl2; vl2 = vl1; vl1 = vl;
    }
    return mask;
}

__device__ __forceinline__ uint32_t fold32(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    uint32_t x = w0 ^ __builtin_rotateleft32(w1, 7) ^ __builtin_rotateleft32(w2, 13) ^ __builtin_rotateleft32(w3, 21);
    return x * 0x9E3779B1u;
}

__device__ __forceinline__ uint64_t short_hash64(uint64_t k0, uint64_t k1) {
    uint64_t h = (k0 ^ (k1 * 0x9E3779B97F4A7C15ull)) * 0xD6E8FEB86659FD93ull;
    return h ^ (h >> 32);
}

__device__ __forceinline__ uint64_t fnv1a64_step(uint64_t h, uint32_t b) { return (h ^ b) * 1099511628211ull; }
constexpr uint64_t kFnv64Off = 14695981039346656037ull;

// ------------------------------------------------------- HBM table inserts
// Lock-free insert of a short key.  Claim = CAS on k0 (0 -> key); the claimer
// then publishes k1.  A prober that matches k0 before k1 is visible never waits
// inside the probe loop: the compiler may place the claimer's publish on the
// loop's exit path, after every other lane of its wave left the loop, so an
// in-loop wait can stall a whole wave (measured: ~100 ms per 10 GB).  Instead
// *_try returns kRetry and *_insert re-runs it from a wave-uniform outer loop,
// which only iterates after the claimer's stores have executed.  All shared
// words use agent-scope atomics (sc1: coherent across the 8 XCD L2s).
enum : int { kDone = 0, kRetry = 1, kFull = 2 };
constexpr uint32_t kMaxRetries = 1u << 20;

__device__ int short_try(const Tables& t, uint64_t k0, uint64_t k1, uint64_t cnt) {
    uint64_t i = short_hash64(k0, k1) & t.sh_mask;
    for (uint32_t probes = 0; probes <= (uint32_t)kGlobalProbes; probes++) {
        ShortSlot* s = &t.sh[i];
        uint64_t cur = ld_agent(&s->k0);
        if (cur == 0) {
            uint64_t prev = atomicCAS((unsigned long long*)&s->k0, 0ull, (unsigned long long)k0);
            if (prev == 0) {
                st_agent(&s->k1, k1);
                atomicAdd((unsigned long long*)&s->count, (unsigned long long)cnt);
                unsigned long long used = atomicAdd(&t.ctr->short_used, 1ull);
                if (used * 10 > (t.sh_mask + 1) * 7) set_status(t.ctr, kStShortFull);
                return kDone;
            }
            cur = prev;
        }
        if (cur == k0) {
            uint64_t v = ld_agent(&s->k1);
            if (v == kUnwritten) return kRetry;
            if (v == k1) {
                atomicAdd((unsigned long long*)&s->count, (unsigned long long)cnt);
                return kDone;
            }
        }
        i = (i + 1) & t.sh_mask;
    }
    return kFull;
}

__device__ void short_insert(const Tables& t, uint64_t k0, uint64_t k1, uint64_t cnt) {
    bool pending = true;
    uint32_t tries = 0;
    while (__ballot(pending)) {  // wave-uniform: reconverges between attempts
        if (pending) {
            const int r = short_try(t, k0, k1, cnt);
            if (r == kFull) set_status(t.ctr, kStShortFull);
            pending = r == kRetry;
            if (pending && ++tries > kMaxRetries) { set_status(t.ctr, kStSpin); pending = false; }
        }
    }
}

// Long keys: claim = CAS on hash; publish len+1 and rep separately; a prober
// that needs them before both are visible retries from the outer loop.
__device__ int long_try(const Tables& t, uint64_t h, const uint8_t* rep, uint64_t len, uint64_t cnt) {
    uint64_t i = (h * 0x9E3779B97F4A7C15ull >> 17) & t.lo_mask;
    for (uint32_t probes = 0; probes <= (uint32_t)kGlobalProbes; probes++) {
        LongSlot* s = &t.lo[i];
        uint64_t cur = ld_agent(&s->hash);
        if (cur == 0) {
            uint64_t prev = atomicCAS((unsigned long long*)&s->hash, 0ull, (unsigned long long)h);
            if (prev == 0) {
                st_agent(&s->len, len + 1);
                __hip_atomic_store(const_cast<const uint8_t**>(&s->rep), rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicAdd((unsigned long long*)&s->count, (unsigned long long)cnt);
                atomicAdd(&t.ctr->long_bytes, (unsigned long long)len);
                unsigned long long used = atomicAdd(&t.ctr->long_used, 1ull);
                if (used * 10 > (t.lo_mask + 1) * 7) set_status(t.ctr, kStLongFull);
                return kDone;
            }
            cur = prev;
        }
        if (cur == h) {
            const uint8_t* r = ld_agent_ptr(&s->rep);
            const uint64_t lp1 = ld_agent(&s->len);
            if (r == nullptr || lp1 == 0) return kRetry;
            if (lp1 == len + 1) {
                bool eq = true;
                for (uint64_t k = 0; k < len; k++)
                    if (r[k] != rep[k]) { eq = false; break; }
                if (eq) {
                    atomicAdd((unsigned long long*)&s->count, (unsigned long long)cnt);
                    return kDone;
                }
            }
        }
        i = (i + 1) & t.lo_mask;
    }
    return kFull;
}

__device__ void long_insert(const Tables& t, uint64_t h, const uint8_t* rep, uint64_t len, uint64_t cnt) {
    h |= 1ull;
    bool pending = true;
    uint32_t tries = 0;
    while (__ballot(pending)) {
        if (pending) {
            const int r = long_try(t, h, rep, len, cnt);
            if (r == kFull) set_status(t.ctr, kStLongFull);
            pending = r == kRetry;
            if (pending && ++tries > kMaxRetries) { set_status(t.ctr, kStSpin); pending = false; }
        }
    }
}

__device__ __forceinline__ void list_append(const Tables& t, uint64_t v) {
    unsigned long long idx = atomicAdd(&t.ctr->nlist, 1ull);
    if (idx < t.list_cap) t.list[idx] = v;
    else set_status(t.ctr, kStListFull);
}

// ------------------------------------------------------------ LDS table
// Count `add` occurrences of key (k0,k1) in a workgroup LDS table.  One probe,
// no loop: the key is looked up in the first way of its set whose k0 matches.
// Returns false (a miss: the caller spills or forwards the key, where it is
// still counted exactly) when that way holds a different k1 (another key with
// the same first 8 bytes in the same set: ~4/NSETS of such pairs), when it is
// claimed but not yet published, when the key is absent and its set is full,
// or when a claim CAS races — the table never waits on another lane (see
// short_try).  Kept branch-light on purpose: each divergent `if` costs a
// handful of SALU exec-mask instructions per wave, and the map kernel is
// issue-bound.
template <int NSETS>
__device__ __forceinline__ bool st_lookup_add(STable<NSETS>& T, uint64_t k0, uint64_t k1, uint32_t h, uint32_t add,
                                              uint32_t& base, uint32_t& empty, uint32_t& m_out) {
    // Explicit LDS address space: through a generic (or volatile) pointer hipcc
    // emits flat_load ... sc0 sc1 + s_waitcnt vmcnt(0), i.e. every lookup would
    // wait for all of the wave's outstanding HBM loads and stores.
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    typedef const __attribute__((address_space(3))) u64x2 lds_u64x2;
    typedef const __attribute__((address_space(3))) unsigned long long lds_u64;
    base = __umulhi(h, NSETS) * 4;
    const u64x2 a = *(lds_u64x2*)(&T.k0[base]);
    const u64x2 b = *(lds_u64x2*)(&T.k0[base + 2]);
    const uint32_t m = (a.x == k0 ? 1u : 0u) | (a.y == k0 ? 2u : 0u) | (b.x == k0 ? 4u : 0u) | (b.y == k0 ? 8u : 0u);
    const uint32_t z = (a.x == 0 ? 1u : 0u) | (a.y == 0 ? 2u : 0u) | (b.x == 0 ? 4u : 0u) | (b.y == 0 ? 8u : 0u);
    const uint32_t slot = base + (__builtin_ctz(m | 16u) & 3u);
    const uint64_t v = *(lds_u64*)(&T.k1[slot]);  // read unconditionally (way 0 when m == 0)
    const bool hit = (m != 0) & (v == k1);
    empty = m != 0 ? 0u : z;  // claimable ways, only when the key's k0 is absent from the set
    m_out = m | (z << 4);     // 0: the key's k0 is absent and the set is full
    if (hit) atomicAdd(&T.cnt[slot], add);
    return hit;
}

// Claim the first empty way of the set for the key (after st_lookup_add found
// its k0 absent).  False when the CAS races with another lane's claim.
template <int NSETS>
__device__ __forceinline__ bool st_claim(STable<NSETS>& T, uint64_t k0, uint64_t k1, uint32_t base, uint32_t empty,
                                         uint32_t add) {
    const uint32_t es = base + __builtin_ctz(empty);
    if (atomicCAS(&T.k0[es], 0ull, (unsigned long long)k0) != 0ull) return false;
    __hip_atomic_store(&T.k1[es], (unsigned long long)k1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    atomicAdd(&T.cnt[es], add);
    return true;
}

template <int NSETS>
__device__ __forceinline__ bool st_insert(STable<NSETS>& T, uint64_t k0, uint64_t k1, uint32_t h, uint32_t add) {
    uint32_t base, empty, m;
    bool ok = st_lookup_add(T, k0, k1, h, add, base, empty, m);
    if (empty != 0) ok = st_claim(T, k0, k1, base, empty, add);
    return ok;
}

// Two-choice variant (bucket aggregator, whose table is about half full): a
// key whose first set is full and does not hold its k0 lives in a second set.
// Ways are never freed, so once the first set is full a key absent from it can
// never appear there later — lookups and claims agree on the key's set.
template <int NSETS>
__device__ __forceinline__ bool st_insert2(STable<NSETS>& T, uint64_t k0, uint64_t k1, uint32_t h, uint32_t add) {
    uint32_t base, empty, m;
    bool ok = st_lookup_add(T, k0, k1, h, add, base, empty, m);
    if (empty != 0) {
        ok = st_claim(T, k0, k1, base, empty, add);
    } else if (m == 0) {  // first set full, key absent
        const uint32_t h2 = __builtin_amdgcn_alignbit(h, h, 16) * 0xC2B2AE3Du;
        ok = st_lookup_add(T, k0, k1, h2, add, base, empty, m);
        if (empty != 0) ok = st_claim(T, k0, k1, base, empty, add);
    }
    return ok;
}

template <int NSETS>
__device__ __forceinline__ void st_init(STable<NSETS>& T, uint32_t tid, uint32_t nthreads) {
    for (uint32_t i = tid; i < (uint32_t)NSETS * 4; i += nthreads) {
        T.k0[i] = 0;
        T.k1[i] = kUnwritten;
        T.cnt[i] = 0;
    }
}

// Add every occupied way of the table to the HBM ShortTable.
template <int NSETS>
__device__ __forceinline__ void st_flush(STable<NSETS>& T, const Tables& t, uint32_t tid, uint32_t nthreads) {
    for (uint32_t i = tid; i < (uint32_t)NSETS * 4; i += nthreads) {
        const uint64_t k0 = T.k0[i];
        if (k0 != 0) short_insert(t, k0, T.k1[i], T.cnt[i]);
    }
}

// Spill bucket from the combiner hash h = fold32(key): top byte of a second
// multiplicative hash, so keys of one bucket still spread over all sets of the
// aggregator's table (which indexes by the top bits of h).
__device__ __forceinline__ uint32_t spill_bucket(uint32_t h) {
    static_assert(kSpillBuckets == 512, "bucket = top 9 bits");
    return (h * 0x85EBCA6Bu) >> 23;
}

// ------------------------------------------------------------ chunk loading
struct ChunkRegs {
    uint4 a, h;  // a: chunk bytes [16l, 16l+16); h: halo piece (lanes 0-3 look-ahead, lane 4 look-back)
};

__device__ __forceinline__ uint4 load16_bounded(const uint8_t* in, uint64_t n, int64_t off) {
    uint32_t w[4] = {0, 0, 0, 0};
    for (int k = 0; k < 16; k++) {
        int64_t o = off + k;
        if (o >= 0 && (uint64_t)o < n) w[k >> 2] |= (uint32_t)in[o] << (8 * (k & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void load_chunk(const uint8_t* __restrict__ in, uint64_t n, uint64_t cs, uint32_t lane,
                                           ChunkRegs& r) {
    if (cs + kChunk + kAhead <= n && cs >= (uint64_t)kBack) {
        const uint4* p = reinterpret_cast<const uint4*>(in + cs);
        r.a = p[lane];
        if (lane < 4) r.h = p[64 + lane];
        else if (lane == 4) r.h = p[-1];
        else r.h = make_uint4(0, 0, 0, 0);
    } else {
        r.a = load16_bounded(in, n, (int64_t)cs + 16 * lane);
        if (lane < 4) r.h = load16_bounded(in, n, (int64_t)cs + kChunk + 16 * lane);
        else if (lane == 4) r.h = load16_bounded(in, n, (int64_t)cs - 16);
        else r.h = make_uint4(0, 0, 0, 0);
    }
}

__device__ __forceinline__ void stage_chunk(WaveLds& W, const ChunkRegs& r, uint32_t lane) {
    uint4* b4 = reinterpret_cast<uint4*>(W.buf);
    b4[1 + lane] = r.a;
    if (lane < 4) b4[65 + lane] = r.h;
    else if (lane == 4) b4[0] = r.h;
}

// ------------------------------------------------------------ wc map kernel
// Each wave walks its chunks independently (grid stride over waves, one chunk
// prefetched ahead); the only workgroup barriers are at start and end.
template <uint32_t mode>
__global__ void __launch_bounds__(kThreads) wc_map_kernel(const uint8_t* __restrict__ in, uint64_t n, uint64_t nchunks,
                                                          Tables t, LetterTables lt) {
    // mode (benchmark ablation only, compile-time; results are wrong unless 0):
    // 1 = read input only, 2 = tokenize only (no per-word work), 4 = per-word key
    // extraction without the table, 16 = drop combiner misses (no spill append),
    // 32 = spill without the store
    __shared__ MapLds L;
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63;
    const uint32_t wv = tid >> 6;
    WaveLds& W = L.w[wv];

    st_init(L.T, tid, kThreads);
    for (uint32_t b = tid; b < (uint32_t)kSpillBuckets; b += kThreads) L.cur[b] = L.cur8[b] = 0;
    __syncthreads();

    const uint64_t stride = (uint64_t)gridDim.x * kWavesPerWG;
    const uint64_t c0 = (uint64_t)blockIdx.x * kWavesPerWG + wv;
    const uint64_t my_stream0 = (uint64_t)blockIdx.x * t.sp.sub_keys;  // + b*nwg*sub_keys
    const uint64_t my_stream8 = (uint64_t)blockIdx.x * t.sp.sub8;
    const uint32_t bstride = t.sp.nwg * (uint32_t)t.sp.sub_keys;  // < 2^32 (ensure_spill)
    const uint32_t bstride8 = t.sp.nwg * (uint32_t)t.sp.sub8;
    const uint32_t sub = (uint32_t)t.sp.sub_keys, sub8 = (uint32_t)t.sp.sub8;
    uint64_t ovf = 0, utf8_chunks = 0, acc = 0;
    ChunkRegs cur, nxt;
    if (c0 < nchunks) load_chunk(in, n, c0 * kChunk, lane, cur);

    for (uint64_t c = c0; c < nchunks; c += stride) {
        {
            const uint64_t cs = c * kChunk;
            if (c + stride < nchunks) load_chunk(in, n, (c + stride) * kChunk, lane, nxt);  // prefetch next round
            if constexpr ((mode & 1) != 0) {
                acc ^= cur.a.x ^ cur.a.y ^ cur.a.z ^ cur.a.w ^ cur.h.x;
                cur = nxt;
                continue;
            }

            stage_chunk(W, cur, lane);
            uint32_t hi = (cur.a.x | cur.a.y | cur.a.z | cur.a.w | cur.h.x | cur.h.y | cur.h.z | cur.h.w) & 0x80808080u;
            const bool ascii = __ballot(hi != 0) == 0;
            uint32_t mA, mH = 0;
            if (ascii) {
                mA = ascii_mask16(cur.a);
                if (lane < 5) mH = ascii_mask16(cur.h);
            } else {
                utf8_chunks++;
                wave_sync();
                mA = utf8_letter_mask<16>(W.buf, kBack + 16 * lane, lt);
                if (lane < 3) mH = utf8_letter_mask<16>(W.buf, kBack + kChunk + 16 * lane, lt);
                else if (lane == 4) mH = utf8_letter_mask<8>(W.buf, 8, lt) << 8;  // look-back bits 8..15
            }
            // word starts (letter byte whose predecessor is not a letter byte) and
            // lengths (ctz over this piece + the next two pieces' masks), packed
            // into the list as start | min(len, 31) << 11
            const uint32_t lm1 = (lane + 63) & 63, lp1 = (lane + 1) & 63, lp2 = (lane + 2) & 63;
            const uint32_t prevA_m = __shfl(mA, (int)lm1);
            const uint32_t back = __shfl(mH, 4);
            const uint32_t x1 = __shfl(mA, (int)lp1), z1 = __shfl(mH, (int)lp1);
            const uint32_t x2 = __shfl(mA, (int)lp2), z2 = __shfl(mH, (int)lp2);
            const uint64_t winA = (uint64_t)mA | ((uint64_t)(lane < 63 ? x1 : z1) << 16) |
                                  ((uint64_t)(lane < 62 ? x2 : z2) << 32);
            const uint32_t pa = (lane == 0 ? back : prevA_m) >> 15 & 1u;
            uint32_t SA = mA & ~((mA << 1) | pa) & 0xFFFFu;
            uint32_t total;
            uint32_t j = wave_excl_scan5(__popc(SA), &total);
            while (SA) {
                const uint32_t bit = __builtin_ctz(SA);
                const uint32_t len = min((uint32_t)__builtin_ctzll(~(winA >> bit)), 31u);
                W.list[j++] = (uint16_t)((16 * lane + bit) | (len << 11));
                SA &= SA - 1;
            }
            wave_sync();
            if constexpr ((mode & 2) != 0) {
                acc += total;
                cur = nxt;
                continue;
            }

            for (uint32_t w = lane; w < total; w += 64) {
                const uint32_t e = W.list[w];
                const uint32_t s = e & 0x7FFu, len = e >> 11;
                if (len > 16) {
                    list_append(t, cs + s);
                    continue;
                }
                const uint32_t q = kBack + s;
                const uint32_t* d = reinterpret_cast<const uint32_t*>(W.buf + (q & ~3u));
                const uint32_t sh = q & 3u;
                const uint32_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
                const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
                const uint32_t w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
                const uint32_t w2 = __builtin_amdgcn_alignbyte(d3, d2, sh);
                const uint32_t w3 = __builtin_amdgcn_alignbyte(d4, d3, sh);
                uint64_t k0 = ((uint64_t)w1 << 32) | w0;
                uint64_t k1 = ((uint64_t)w3 << 32) | w2;
                // keep the first len bytes (1 <= len <= 16), branch-free
                const uint32_t l1 = len > 8 ? len - 8 : 0u;
                k0 &= len >= 8 ? ~0ull : ~(~0ull << (8 * len));
                k1 &= l1 >= 8 ? ~0ull : ~(~0ull << (8 * l1));
                const uint32_t h = fold32((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32));
                if constexpr ((mode & 4) != 0) {
                    acc += h;
                    continue;
                }
                const bool hit = st_insert(L.T, k0, k1, h, 1);
                if constexpr ((mode & 16) != 0) { acc += hit; continue; }
                if (!hit) {  // append to this workgroup's stream of the key's bucket
                    const uint32_t b = spill_bucket(h);
                    const bool small = k1 == 0;  // key of at most 8 bytes: 8-byte record
                    const uint32_t pos = atomicAdd(small ? &L.cur8[b] : &L.cur[b], 1u);
                    if (pos < (small ? sub8 : sub)) {
                        if constexpr ((mode & 32) != 0) acc += (uint32_t)k0;
                        else if (small) t.sp.pool8[my_stream8 + (uint64_t)b * bstride8 + pos] = k0;
                        else t.sp.pool[my_stream0 + (uint64_t)b * bstride + pos] =
                            make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32));
                    } else {
                        short_insert(t, k0, k1, 1);
                        ovf++;
                    }
                }
            }
            wave_sync();
            cur = nxt;
        }
    }

    __syncthreads();
    unsigned long long spilled = 0;
    for (uint32_t b = tid; b < (uint32_t)kSpillBuckets; b += kThreads) {
        const uint32_t k = min(L.cur[b], sub), k8 = min(L.cur8[b], sub8);
        t.sp.counts[(uint64_t)b * t.sp.nwg + blockIdx.x] = k;
        t.sp.counts8[(uint64_t)b * t.sp.nwg + blockIdx.x] = k8;
        spilled += k + k8;
    }
    if (spilled) atomicAdd(&t.ctr->spilled, spilled);
    st_flush(L.T, t, tid, kThreads);
    if (ovf) atomicAdd(&t.ctr->spill_ovf, (unsigned long long)ovf);
    if (acc == 0x5eed5eedull) atomicAdd(&t.ctr->pad[0], 1ull);  // keeps ablation builds honest (no DCE)
    if (utf8_chunks && lane == 0) atomicAdd(&t.ctr->chunks_utf8, (unsigned long long)utf8_chunks);
}

// Bucket aggregation: one workgroup per spill bucket counts its keys in an LDS
// table (a bucket holds ~1/512 of the distinct spilled keys), then adds the
// per-key totals to the HBM ShortTable — one HBM atomic per distinct key per
// bucket instead of one per occurrence.  The bucket's nwg streams (one per map
// workgroup) are walked as one sequence of kAggGroup-record groups with the
// next group's loads in flight while the current one is inserted.
constexpr uint32_t kAggUnroll = 4;
constexpr uint32_t kAggGroup = kAggUnroll * kAggThreads;

__device__ __forceinline__ void agg_load(const uint4* blk, uint32_t i, uint32_t f, uint4& r) {
    r = i < f ? blk[i] : make_uint4(0, 0, 0, 0);
}
__device__ __forceinline__ void agg_load(const uint64_t* blk, uint32_t i, uint32_t f, uint4& r) {
    const uint64_t k = i < f ? blk[i] : 0;
    r = make_uint4((uint32_t)k, (uint32_t)(k >> 32), 0, 0);
}

template <uint32_t amode, typename Rec>
__device__ __forceinline__ void agg_streams(AggLds& A, const Tables& t, const Rec* pool, const uint32_t* counts,
                                            uint64_t sub, uint64_t& miss) {
    const uint32_t nwg = t.sp.nwg, tid = threadIdx.x;
    // (g, base, f): current stream, first record of the group, records in the stream
    uint32_t g = 0, base = 0, f = nwg ? counts[0] : 0;
    while (g < nwg && base >= f) { g++; f = g < nwg ? counts[g] : 0; }
    uint4 cur[kAggUnroll], nxt[kAggUnroll];
    if (g < nwg) {
#pragma unroll
        for (uint32_t u = 0; u < kAggUnroll; u++) agg_load(pool + (uint64_t)g * sub, base + u * kAggThreads + tid, f, cur[u]);
    }
    while (g < nwg) {
        uint32_t g2 = g, base2 = base + kAggGroup, f2 = f;
        while (g2 < nwg && base2 >= f2) { g2++; base2 = 0; f2 = g2 < nwg ? counts[g2] : 0; }
        if (g2 < nwg) {
#pragma unroll
            for (uint32_t u = 0; u < kAggUnroll; u++)
                agg_load(pool + (uint64_t)g2 * sub, base2 + u * kAggThreads + tid, f2, nxt[u]);
        }
#pragma unroll
        for (uint32_t u = 0; u < kAggUnroll; u++) {
            const uint4 k = cur[u];
            if ((k.x | k.y) != 0) {  // else past the stream's end (keys have k0 != 0)
                const uint64_t k0 = ((uint64_t)k.y << 32) | k.x, k1 = ((uint64_t)k.w << 32) | k.z;
                const uint32_t h = fold32(k.x, k.y, k.z, k.w);
                if constexpr ((amode & 128) != 0) {
                    miss += h;
                } else if constexpr ((amode & 256) != 0) {
                    uint32_t base, empty, mm;
                    miss += st_lookup_add(A.T, k0, k1, h, 0, base, empty, mm) + empty;
                } else if (!st_insert2(A.T, k0, k1, h, 1)) {
                    const uint32_t pos = atomicAdd(&A.nmiss, 1u);  // defer: no HBM round trip in the loop
                    if (pos < t.sp.amiss_cap)
                        t.sp.amiss[(uint64_t)blockIdx.x * t.sp.amiss_cap + pos] =
                            make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32));
                    else
                        short_insert(t, k0, k1, 1);
                    miss++;
                }
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < kAggUnroll; u++) cur[u] = nxt[u];
        g = g2; base = base2; f = f2;
    }
}

// amode (benchmark ablation only, compile-time; results are wrong unless 0):
// 128 = read + hash the records only, 256 = table lookups without adds/claims
template <uint32_t amode>
__global__ void __launch_bounds__(kAggThreads) wc_agg_kernel(Tables t) {
    __shared__ AggLds A;
    const uint32_t tid = threadIdx.x;
    st_init(A.T, tid, kAggThreads);
    if (tid == 0) A.nmiss = 0;
    __syncthreads();
    const uint64_t b = blockIdx.x;
    uint64_t miss = 0;
    agg_streams<amode>(A, t, t.sp.pool8 + b * t.sp.nwg * t.sp.sub8, t.sp.counts8 + b * t.sp.nwg, t.sp.sub8, miss);
    agg_streams<amode>(A, t, t.sp.pool + b * t.sp.nwg * t.sp.sub_keys, t.sp.counts + b * t.sp.nwg, t.sp.sub_keys, miss);
    __syncthreads();
    st_flush(A.T, t, tid, kAggThreads);
    const uint32_t nm = min(A.nmiss, t.sp.amiss_cap);
    for (uint32_t i = tid; i < nm; i += kAggThreads) {  // deferred misses, all lanes in flight
        const uint4 k = t.sp.amiss[b * t.sp.amiss_cap + i];
        short_insert(t, ((uint64_t)k.y << 32) | k.x, ((uint64_t)k.w << 32) | k.z, 1);
    }
    if (amode != 0 && miss == 0x5eed5eedull) atomicAdd(&t.ctr->pad[0], 1ull);  // no DCE in ablation builds
    else if (amode == 0 && miss) atomicAdd(&t.ctr->agg_miss, (unsigned long long)miss);
}

// Words longer than 16 bytes: decode forward from the start (one lane per word).
__global__ void wc_long_kernel(const uint8_t* __restrict__ in, uint64_t n, Tables t, LetterTables lt, uint64_t nlist) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlist) return;
    const uint64_t s = t.list[i];
    uint64_t q = s, h = kFnv64Off;
    while (q < n) {
        uint32_t c0 = in[q];
        uint32_t c1 = q + 1 < n ? in[q + 1] : 0, c2 = q + 2 < n ? in[q + 2] : 0, c3 = q + 3 < n ? in[q + 3] : 0;
        int vl = utf8_valid_len(c0, c1, c2, c3);
        if (vl == 0 || !is_letter_cp(utf8_decode(c0, c1, c2, c3, vl), lt)) break;
        for (int k = 0; k < vl; k++) h = fnv1a64_step(h, in[q + k]);
        q += vl;
    }
    long_insert(t, h, in + s, q - s, 1);
}

// ------------------------------------------------------------ grep kernels
// Pattern occurrence search.  Every occurrence start p (with p + plen <= n) is
// appended to the list; grep_lines_kernel resolves its line.
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

__global__ void __launch_bounds__(kThreads) grep_map_kernel(const uint8_t* __restrict__ in, uint64_t n, uint64_t nchunks,
                                                            const uint8_t* __restrict__ pat, uint32_t plen, Tables t) {
    __shared__ WaveLds Wl[kWavesPerWG];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63;
    WaveLds& W = Wl[tid >> 6];
    const uint32_t p0 = pat[0];
    const uint32_t rep = p0 * 0x01010101u;
    const bool in_lds = plen <= (uint32_t)kAhead;
    const uint64_t stride = (uint64_t)gridDim.x * kWavesPerWG;
    uint64_t c = (uint64_t)blockIdx.x * kWavesPerWG + (tid >> 6);
    ChunkRegs cur, nxt;
    if (c < nchunks) load_chunk(in, n, c * kChunk, lane, cur);
    for (; c < nchunks; c += stride) {
        const uint64_t cs = c * kChunk;
        if (c + stride < nchunks) load_chunk(in, n, (c + stride) * kChunk, lane, nxt);
        stage_chunk(W, cur, lane);
        wave_sync();
        {
            uint32_t m = eq_mask16(cur.a, rep);
            const uint32_t base = 16 * lane;
            while (m) {
                const uint32_t bit = __builtin_ctz(m);
                m &= m - 1;
                const uint64_t pos = cs + base + bit;
                if (pos + plen > n) continue;
                bool ok = true;
                if (in_lds) {
                    const uint8_t* q = W.buf + kBack + base + bit;
                    for (uint32_t k = 1; k < plen; k++)
                        if (q[k] != pat[k]) { ok = false; break; }
                } else {
                    for (uint32_t k = 1; k < plen; k++)
                        if (in[pos + k] != pat[k]) { ok = false; break; }
                }
                if (ok) list_append(t, pos);
            }
        }
        wave_sync();
        cur = nxt;
    }
}

// Empty pattern: every line (strings.Split yields len(sep-count)+1 lines).
__global__ void grep_all_lines_kernel(const uint8_t* __restrict__ in, uint64_t n, Tables t) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
        if (i == 0) list_append(t, 0);
        else if (in[i - 1] == '\n') list_append(t, i);
    }
}

// Resolve the line of each hit: [last '\n' before p]+1 .. next '\n' at/after p.
// plen == 0 means the list already holds line starts.
__global__ void grep_lines_kernel(const uint8_t* __restrict__ in, uint64_t n, uint32_t plen, Tables t, uint64_t nlist) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlist) return;
    const uint64_t p = t.list[i];
    uint64_t s = p;
    if (plen > 0)
        while (s > 0 && in[s - 1] != '\n') s--;
    uint64_t e = p;
    while (e < n && in[e] != '\n') e++;
    uint64_t h = kFnv64Off;
    for (uint64_t k = s; k < e; k++) h = fnv1a64_step(h, in[k]);
    long_insert(t, h, in + s, e - s, 1);
}

// ------------------------------------------------------------ collect
__device__ __forceinline__ uint32_t key_len_short(uint64_t k0, uint64_t k1) {
    if (k1) return 8 + (uint32_t)((71 - __builtin_clzll(k1)) >> 3);
    return (uint32_t)((71 - __builtin_clzll(k0)) >> 3);
}

__global__ void collect_short_kernel(Tables t, Recs r, uint32_t nreduce) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= t.sh_mask; i += stride) {
        const ShortSlot s = t.sh[i];
        if (s.k0 == 0) continue;
        const uint32_t len = key_len_short(s.k0, s.k1);
        uint32_t h = 2166136261u;
        for (uint32_t k = 0; k < len; k++) {
            const uint64_t w = k < 8 ? s.k0 : s.k1;
            h = fnv1a32_step(h, (uint32_t)(w >> (8 * (k & 7))) & 0xFFu);
        }
        const unsigned long long o = atomicAdd(&t.ctr->nrec, 1ull);
        r.k0[o] = s.k0;
        r.k1[o] = s.k1;
        r.len[o] = len;
        r.cnt[o] = s.count;
        r.part[o] = (h & 0x7fffffffu) % nreduce;
        r.koff[o] = ~0ull;
    }
}

__global__ void collect_long_kernel(Tables t, Recs r, uint32_t nreduce) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= t.lo_mask; i += stride) {
        const LongSlot s = t.lo[i];
        if (s.hash == 0 || s.rep == nullptr || s.len == 0) continue;
        const uint64_t len = s.len - 1;
        const unsigned long long off = atomicAdd(&t.ctr->arena, (unsigned long long)len);
        uint32_t h = 2166136261u;
        uint64_t k0 = 0, k1 = 0;
        for (uint64_t k = 0; k < len; k++) {
            const uint32_t b = s.rep[k];
            r.arena[off + k] = (uint8_t)b;
            h = fnv1a32_step(h, b);
            if (k < 8) k0 |= (uint64_t)b << (8 * k);
            else if (k < 16) k1 |= (uint64_t)b << (8 * (k - 8));
        }
        const unsigned long long o = atomicAdd(&t.ctr->nrec, 1ull);
        atomicAdd(&t.ctr->nlong_rec, 1ull);
        r.k0[o] = k0;
        r.k1[o] = k1;
        r.len[o] = (uint32_t)len;
        r.cnt[o] = s.count;
        r.part[o] = (h & 0x7fffffffu) % nreduce;
        r.koff[o] = off;
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

__global__ void clear_tables_kernel(Tables t) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= t.sh_mask; i += stride)
        t.sh[i] = ShortSlot{0, kUnwritten, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= t.lo_mask; i += stride)
        t.lo[i] = LongSlot{0, nullptr, 0, 0};
}

// ------------------------------------------------------------ launchers
int map_grid_size(int device) {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0) ncu = 256;
    return ncu;  // one 512-thread workgroup per CU (LDS-bound), persistent over chunks
}

void clear_tables(const Tables& t, hipStream_t s) {
    hipMemsetAsync(t.ctr, 0, sizeof(Counters), s);
    if (t.sp.counts) hipMemsetAsync(t.sp.counts, 0, (size_t)2 * kSpillBuckets * t.sp.nwg * sizeof(uint32_t), s);
    clear_tables_kernel<<<2048, 256, 0, s>>>(t);
}

uint32_t wc_map_grid(uint64_t n, int grid) {
    const uint64_t nchunks = (n + kChunk - 1) / kChunk;
    uint64_t g = (nchunks + kWavesPerWG - 1) / kWavesPerWG;
    if (g > (uint64_t)grid) g = (uint64_t)grid;
    return (uint32_t)(g ? g : 1);
}

void launch_wc_map(const uint8_t* in, uint64_t n, const Tables& t, LetterTables lt, int grid, int mode, hipStream_t s) {
    const uint64_t nchunks = (n + kChunk - 1) / kChunk;
    if (nchunks == 0) return;
    const uint64_t g = wc_map_grid(n, grid);
    switch (mode) {
#define MRG_MAP_MODE(M) \
    case M: wc_map_kernel<M><<<(unsigned)g, kThreads, 0, s>>>(in, n, nchunks, t, lt); break;
        MRG_MAP_MODE(1) MRG_MAP_MODE(2) MRG_MAP_MODE(4) MRG_MAP_MODE(16) MRG_MAP_MODE(32)
#undef MRG_MAP_MODE
        default: wc_map_kernel<0><<<(unsigned)g, kThreads, 0, s>>>(in, n, nchunks, t, lt); break;
    }
}

void launch_wc_agg(const Tables& t, int mode, hipStream_t s) {
    if (mode & 128) wc_agg_kernel<128><<<kSpillBuckets, kAggThreads, 0, s>>>(t);
    else if (mode & 256) wc_agg_kernel<256><<<kSpillBuckets, kAggThreads, 0, s>>>(t);
    else wc_agg_kernel<0><<<kSpillBuckets, kAggThreads, 0, s>>>(t);
}

void launch_wc_long(const uint8_t* in, uint64_t n, const Tables& t, LetterTables lt, uint64_t nlist, hipStream_t s) {
    if (nlist == 0) return;
    wc_long_kernel<<<(unsigned)((nlist + 255) / 256), 256, 0, s>>>(in, n, t, lt, nlist);
}

void launch_grep_map(const uint8_t* in, uint64_t n, const uint8_t* d_pat, uint32_t plen, const Tables& t, int grid,
                     hipStream_t s) {
    const uint64_t nchunks = (n + kChunk - 1) / kChunk;
    if (nchunks == 0 || plen == 0) return;
    uint64_t g = (nchunks + kWavesPerWG - 1) / kWavesPerWG;
    uint64_t gmax = (uint64_t)grid * 4;
    if (g > gmax) g = gmax;
    grep_map_kernel<<<(unsigned)g, kThreads, 0, s>>>(in, n, nchunks, d_pat, plen, t);
}

void launch_grep_all_lines(const uint8_t* in, uint64_t n, const Tables& t, int grid, hipStream_t s) {
    grep_all_lines_kernel<<<grid * 4, 256, 0, s>>>(in, n, t);
}

void launch_grep_lines(const uint8_t* in, uint64_t n, uint32_t plen, const Tables& t, uint64_t nlist, hipStream_t s) {
    if (nlist == 0) return;
    grep_lines_kernel<<<(unsigned)((nlist + 255) / 256), 256, 0, s>>>(in, n, plen, t, nlist);
}

void launch_collect(const Tables& t, Recs r, uint32_t nreduce, hipStream_t s) {
    collect_short_kernel<<<1024, 256, 0, s>>>(t, r, nreduce);
    collect_long_kernel<<<256, 256, 0, s>>>(t, r, nreduce);
}

void launch_insert_recs(const Recs& src, const Tables& t, hipStream_t s) {
    if (src.n == 0) return;
    uint64_t g = (src.n + 255) / 256;
    if (g > 4096) g = 4096;
    insert_recs_kernel<<<(unsigned)g, 256, 0, s>>>(src, t);
}

}  // namespace mrg
