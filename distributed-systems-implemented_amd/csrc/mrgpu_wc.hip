// mrgpu_wc.hip — the wc Map pipeline on gfx950 (MapReduce/mrapps/wc.go:21-34 +
// mr/worker.go:72-78 + the grouping half of worker.go:123-146).
//
// Stages (one launch each, all on the context stream):
//   0. sample_gather + wc_map (no dictionary) + wc_agg (sample mode) +
//      dict_build: the hottest keys of an evenly spaced sample of the split
//      become a static two-choice LDS dictionary (mrgpu_internal.h).
//   1. wc_map_kernel: one wave per 1 KiB chunk at a time.  Lanes load 16 B
//      each (coalesced dwordx4), classify letters (ASCII SWAR, or a Go-exact
//      UTF-8 decode + IsLetter bitmap), find word starts and lengths from the
//      letter bitmaps (DPP whole-wave shifts for the neighbour lanes), compact
//      them into an LDS list, then each lane takes 3 words at a time (all their
//      LDS reads in flight together): the key bytes come from the staged chunk
//      with aligned 8-byte LDS reads, the dictionary lookup is two aligned 16 B
//      reads, a hit is one LDS add, a miss is appended to the key's spill bucket
//      stream (8-byte records for keys <= 8 bytes, 16-byte otherwise).
//   2. wc_agg_kernel: one workgroup per spill bucket counts the bucket's keys in
//      an LDS table.  Every key of the bucket reaches this one workgroup
//      (bucket = f(key)), so its table holds exact totals and is emitted
//      directly as records — unless a key of the bucket also went to the HBM
//      table (a stream or table overflow), in which case the bucket is merged
//      through the HBM table instead, so no key is ever emitted twice.
//   3. dict_emit_kernel: per dictionary slot, the sum of the map workgroups'
//      counts -> one record.  Dictionary keys never spill (the lookup is a
//      pure function of the key), so these records are disjoint from stage 2.
// ihash (FNV-1a) % nReduce is computed once per distinct key at emission: the
// partition is a pure function of the key, so this equals worker.go:76's
// per-KV ihash.  Every wc value is "1", so Reduce(len(values)) = sum of counts
// (mrapps/wc.go:41-44): the combining is exact.
#include "mrgpu_device.h"

namespace mrg {

constexpr int kBatch = 3;                     // words per lane in flight
constexpr int kBatchWords = kBatch * kWave;   // 192 words of a chunk per pass
constexpr int kAggThreads = 512;

// A chunk owns kOwn input bytes; its LDS slot is one 1 KiB DMA of the bytes
// [start - 16, start + 1008): 16 bytes of look-back (lane 0), the 992 owned
// bytes (lanes 1-62) and 16 bytes of look-ahead (lane 63: a word starting in
// lane 62 ends, or is known to exceed 16 bytes, within lane 63; a UTF-8 rune
// starting in lane 63's last 3 bytes is completed from global memory on the
// rare non-ASCII path).  Neighbouring slots overlap by 32 bytes (re-read from
// L2, not HBM).
constexpr int kSlotBytes = 1024;
// A slot is followed by room for the 4 input bytes after its window: a UTF-8
// rune starting in the look-ahead lane's last 3 bytes needs them, and they are
// read from global memory only for such a chunk (a one-lane DMA per chunk for
// them measured +11 % on C5's store-bound map kernel).  Slots are 16-byte aligned.
constexpr int kSlotTail = 4;
constexpr int kSlotStride = kSlotBytes + 16;
constexpr int kOwnLanes = 62;
constexpr uint64_t kOwn = 16 * kOwnLanes;  // 992
constexpr int kRing = 3;                    // LDS slots per wave: current, in flight, free (the word list)
static_assert(kListCap * 2 <= kSlotBytes, "the word list lives in the free slot");

// NW waves per workgroup, NB spill buckets.  16 waves x 256 buckets is the
// default (512 streams per workgroup: fewer partially written lines competing
// for an XCD's 4 MB L2 than 512 buckets' 1024: C2 map 8.64 -> 8.29 ms);
// high-cardinality splits use 2048 buckets, whose cursors take the LDS of 4
// waves' rings (12 waves per workgroup).
// The mask table sits at LDS offset 0 (its address is (entry >> 6) & 0x1F0, no
// base); the dictionary's set offsets are then constant-displaced, which the
// ds_read offset field absorbs.
constexpr int kMaskLens = 32;  // kmask[len], len = 0..31 (> 16 = "more than 16 bytes", never used as a key)
// kS (high-cardinality splits): the 8-byte spill records are write-combined in
// LDS, 4 per stream (stage8), and leave as 32-byte writes (see the map kernel);
// the dictionary is then the mini geometry (DictMini), its LDS holds them.
template <int NW, int NB, bool kS = false>
struct alignas(16) MapLdsT {
    using Geo = std::conditional_t<kS, DictMini, DictFull>;
    uint4 kmask[kMaskLens];                     // kmask[len]: the first min(len, 16) of 16 key bytes
    uint4 dset[Geo::kSets];                     // dictionary image
    uint8_t ring[NW][kRing][kSlotStride];
    uint32_t dcnt[Geo::kSlots + kWave];         // dictionary counts of this workgroup (+ per-lane miss dummies)
    unsigned long long stage8[kS ? NB : 0][4];  // kS: the records of each 8-byte stream not yet written
    uint16_t fl[kS ? NB : 0];                   // kS: stream position of stage8[b][0] (low 16 bits)
    // spill cursors: [0, NB) 8-byte streams, [NB, 2 NB) 16-byte streams, then per-lane dummies for hits
    uint32_t curs[2 * NB + kWave];
    uint32_t lt2[kLetterUnique * 8];            // letter tables (non-ASCII chunks): l2 pages
    // letters among code points < U+0800 (2-byte runes: one table read), except
    // in the default 256-bucket layout (the others have no LDS left: l1 / l2 there)
    static constexpr bool kB2 = NB == kSpillBucketsLo;
    uint32_t lb2[kB2 ? 64 : 1];
    uint8_t lt1[kLetterLdsPages];               // l1 of the pages that hold letters
};
static_assert(kSlotBytes == 1024 && kMaskLens * 16 <= 512, "kmask index fits 0x1F0");
static_assert(sizeof(MapLdsT<kWavesPerWG, kSpillBuckets>) <= 160 * 1024, "map LDS budget");
static_assert(sizeof(MapLdsT<kWavesPerWG, kSpillBucketsLo>) <= 160 * 1024, "map LDS budget (256 buckets)");
static_assert(sizeof(MapLdsT<12, kSpillBucketsHi>) <= 160 * 1024, "map LDS budget (high-cardinality)");
static_assert(sizeof(MapLdsT<kWavesPerWG, kSpillBucketsHi, true>) <= 160 * 1024, "map LDS budget (staged)");

// v_ffbl_b32 as the hardware defines it: index of the lowest set bit, 0xFFFFFFFF for 0
// (__builtin_ctz(0) is undefined and the defined variants add a compare and select)
__device__ __forceinline__ uint32_t ffbl_raw(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// The two candidate dictionary sets of a key (hash h; mid = key of 9-16 bytes),
// as byte offsets of dset (16-byte sets at LDS offset 0): short keys take set
// a = h >> 20 and a ^ x, x = ((h >> 4) & 4095) | 1; mid keys the same bits
// masked to 8 (a = (h >> 20) & 255), in the 256 sets after the 4096 short ones
// (DictFull; DictMini: 9 and 6 bits).
// Computed pre-scaled by 16 with two masks, not three selects and two shifts.
template <class G = DictFull>
__device__ __forceinline__ void dict_set_addrs(uint32_t h, bool mid, uint32_t& a1, uint32_t& a2) {
    const uint32_t m = mid ? (uint32_t)(G::kMid - 1) << 4 : (uint32_t)(G::kShort - 1) << 4;
    const uint32_t off = mid ? (uint32_t)G::kShort * 16u : 0u;
    const uint32_t A = h >> 16;           // a << 4 in bits 4..15
    const uint32_t X = (h & ~15u) | 16u;  // x << 4 in bits 4..15 (bit 4 forced: a2 != a1)
    // (a & b) | c as v_bitop3_b32 (truth table 0xEA): a plain VALU op on gfx950,
    // where v_and_or_b32 issues at the 4-cycle rate (tools/ubench/valu_probe.hip)
    a1 = __builtin_amdgcn_bitop3_b32(A, m, off, 0xEA);
    a2 = __builtin_amdgcn_bitop3_b32(A ^ X, m, off, 0xEA);
}
template <class G = DictFull>
__device__ __forceinline__ void dict_sets(uint32_t h, bool mid, uint32_t& s1, uint32_t& s2) {
    uint32_t a1, a2;
    dict_set_addrs<G>(h, mid, a1, a2);
    s1 = a1 >> 4;
    s2 = a2 >> 4;
}

// Spill bucket of a key: bits 11..18 (256 buckets), 11..19 (512) or 10..20 (2048) of its hash.
// The bucket aggregator's tables index their first set by the top 11 bits
// (21..31), so the bucket bits must stay below bit 21: a shared bit fixes one
// set-index bit within a bucket and halves the first-choice sets (measured with
// 2048 buckets taken from bits 11..21: 2.3 % of C5's records found both their
// sets full and went to the next round).
template <int NB>
__device__ __forceinline__ uint32_t spill_bucket(uint32_t h) {
    static_assert(NB == 256 || NB == 512 || NB == 2048, "bucket = 8, 9 or 11 bits");
    return NB == 256 ? (h >> 11) & 255u : NB == 512 ? (h >> 11) & 511u : (h >> 10) & 2047u;
}

// ------------------------------------------------------------ wc map kernel
// One wave per 992-byte chunk at a time, every wave independent.  The input is
// streamed into a private ring of three 1 KiB LDS slots with one
// buffer_load_dwordx4...lds per chunk (lane l: bytes [start-16+16l, +16): lane 0
// = look-back, lanes 1-62 = the 992 owned bytes, lane 63 = look-ahead; the
// descriptor's range check zero-fills before/after the split), issued two
// chunks ahead.  gfx9 counts loads and stores on one in-order vmcnt, and hipcc
// waits vmcnt(0) as soon as a loop's VMEM count is not static, so the loop's
// VMEM instructions are fixed: the DMA is inline asm (invisible to hipcc's
// waitcnt pass) and the spill appends of a chunk are exactly two range-checked
// buffer stores (its misses compacted in LDS first; lanes with nothing to store
// use an out-of-range offset).  The wait for chunk c's DMA is then vmcnt(kVmemPerIter): only the
// previous iteration's stores and DMA may still be in flight.  Rare paths with
// other memory operations (words > 16 bytes, chunks of more than kBatchWords
// words, HBM-table overflow, UTF-8 table lookups) drain with vmcnt(0).
constexpr uint32_t kOutOfRange = 0xFFFFFFF0u;
constexpr int kVmemPerIter = 3;  // per chunk: one 8-byte and one 16-byte spill store, one DMA

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ i32x4 raw_rsrc(const void* base, uint32_t nrec) {
    const uint64_t b = (uint64_t)base;
    return (i32x4){(int)(uint32_t)b, (int)((uint32_t)(b >> 32) & 0xFFFFu), (int)nrec, 0x00020000};
}
// 64 lanes x 16 B: lane l's bytes at rsrc + voff -> LDS [lds_base + 16 l]
// kPol (benchmark variants of the input loads' cache policy): 0 default, 1 nt,
// 2 sc1, 3 sc0 sc1
template <int kPol = 0>
__device__ __forceinline__ void dma_chunk(i32x4 rsrc, uint32_t voff, uint32_t lds_base) {
    // operands are wave-uniform; readfirstlane puts them in SGPRs for the asm "s" constraints
    rsrc = (i32x4){__builtin_amdgcn_readfirstlane(rsrc.x), __builtin_amdgcn_readfirstlane(rsrc.y),
                   __builtin_amdgcn_readfirstlane(rsrc.z), __builtin_amdgcn_readfirstlane(rsrc.w)};
    lds_base = __builtin_amdgcn_readfirstlane(lds_base);
    if constexpr (kPol == 1)
        asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen nt lds" ::"v"(voff), "s"(rsrc), "s"(lds_base)
                     : "memory", "m0");
    else if constexpr (kPol == 2)
        asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen sc1 lds" ::"v"(voff), "s"(rsrc), "s"(lds_base)
                     : "memory", "m0");
    else if constexpr (kPol == 3)
        asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen sc0 sc1 lds" ::"v"(voff), "s"(rsrc),
                     "s"(lds_base)
                     : "memory", "m0");
    else
        asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc), "s"(lds_base)
                     : "memory", "m0");
}
__device__ __forceinline__ void wait_vmem_iter() {
    static_assert(kVmemPerIter == 3, "update the immediate");
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
}
// The same after an iteration that issued kVmemWide spill stores (a chunk with
// more than 64 dictionary misses appends from its word slots: 2 stores per
// batch slot, no drain), + its DMA.
constexpr int kVmemWide = 2 * kBatch;
__device__ __forceinline__ void wait_vmem_iter_wide() {
    static_assert(kVmemWide + 1 == 7, "update the immediate");
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
}
__device__ __forceinline__ void wait_vmem_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// The counted wait after an iteration that issued xv VMEM operations beyond
// the loop's base count B (long-word record and list stores, appends from the
// word slots): vmcnt(B + x) for the largest x in {0, 1, 2, 4} not above xv (a
// smaller count only waits longer).  A short compare chain: a full switch over
// xv compiled to a jump table whose SGPRs pushed 8 more of the loop's scalars
// into VGPR-lane spills.
template <int N>
__device__ __forceinline__ void vmcnt_imm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
template <int B>
__device__ __forceinline__ void wait_vmem_extra(uint32_t xv) {
    if (xv >= 4) vmcnt_imm<B + 4>();
    else if (xv >= 2) vmcnt_imm<B + 2>();
    else if (xv == 1) vmcnt_imm<B + 1>();
    else vmcnt_imm<B>();
}

// The staged (kS) loop: the flush's 4 stores and the DMA follow the awaited DMA
__device__ __forceinline__ void wait_vmem_iter_staged() { asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); }
// kS: a write-combining round every kFlushEvery chunk trips (a round is two
// workgroup barriers, which cost more than its stores: 2.2 of 11.4 ms per 10 GB
// of C5, profiles/mapprobe_r06_c5_staged_modes.txt); between rounds a group past
// its 4 records stores the rest directly.  2 measured 4 % faster than 1, 3 the
// same as 2.
#ifndef MRG_FLUSH_EVERY
#define MRG_FLUSH_EVERY 2
#endif
constexpr uint32_t kFlushEvery = MRG_FLUSH_EVERY;

// kS: an 8-byte record bound for stream position pos of bucket b (o8: its store
// offset, kOutOfRange if the lane has none) joins the stream's LDS group when
// its position lies in the group [fl[b], fl[b] + 4); otherwise it is stored
// directly.  Returns the offset the lane still stores at.
template <class LT>
__device__ __forceinline__ uint32_t stage_or_store(LT& L, uint32_t b, uint32_t pos, uint64_t key, uint32_t o8) {
    const uint32_t d = (pos - (uint32_t)L.fl[b]) & 0xFFFFu;
    const bool st = o8 != kOutOfRange && d < 4u;
    if (st) *(lds_u64*)&L.stage8[b][d] = key;
    return st ? kOutOfRange : o8;
}

// Issue the DMA of chunk c (any c: chunks past the split read as zeros).
// cs = the chunk's first owned byte (chunk index * kOwn)
template <int kPol = 0>
// The descriptor base is the window start rounded down to 1 GiB (a chunk's
// window never crosses its base's range), so this is 32-bit scalar arithmetic.
// For the split's first chunk the base is 0 and lane 0's offset (-16) wraps past
// the range: its look-back reads zeros, like everything at or past n.
__device__ __forceinline__ void dma_for_chunk(const uint8_t* in, uint64_t n, uint64_t cs, uint32_t lane, uint32_t lds_base) {
    const uint64_t base = cs == 0 ? 0 : ((cs - kBack) & ~((1ull << 30) - 1));
    const uint64_t r = n - base;  // bytes from the base to the end of the split (wraps if base >= n)
    const uint32_t rhi = (uint32_t)(r >> 32), rlo = (uint32_t)r;
    const uint32_t nrec = (int32_t)rhi < 0 ? 0u : (rhi != 0 || rlo > 0xFFFFFF00u) ? 0xFFFFFF00u : rlo;
    dma_chunk<kPol>(raw_rsrc(in + base, nrec), (uint32_t)(cs - base) - kBack + 16u * lane, lds_base);
}

// The map loop's rare paths (long words, full spill streams) read the Tables
// fields they need through this laundered reference: hipcc cannot hoist those
// kernarg loads out of the branch, so the pointers stay out of the SGPRs the
// hot path needs (hoisted, they pushed the loop's DMA scalars into VGPR-lane
// spills reloaded every chunk).
// (The reference is formed from the kernarg segment pointer: the kernel's
// arguments are laid out like the members of MapArgs; taking the parameter's
// own address would copy the struct to scratch.)
struct MapArgs {
    const uint8_t* in;
    uint64_t n;
    uint32_t cbeg, cend, ctail;
    int resume;
    Tables t;
    LetterTables lt;
};
// cold(): a generic reference (rare paths: flat loads, drained anyway);
// cold_list(): the long-word list's base and capacity by scalar loads (the
// single-pass long-word path runs on most chunks of mixed-script text, where a
// flat load would drain the DMA pipeline).
#ifndef MRG_NO_COLD_REF
__device__ __forceinline__ const Tables& cold(const Tables&) {
    const char* p = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const Tables*)(p + offsetof(MapArgs, t));
}
__device__ __forceinline__ void cold_list(const Tables&, uint64_t*& list, uint64_t& cap) {
    typedef const __attribute__((address_space(4))) char* kptr;
    kptr p = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    const __attribute__((address_space(4))) Tables* tp = (const __attribute__((address_space(4))) Tables*)(p + offsetof(MapArgs, t));
    list = tp->list;
    cap = tp->list_cap;
}
#else
__device__ __forceinline__ const Tables& cold(const Tables& t) { return t; }
__device__ __forceinline__ void cold_list(const Tables& t, uint64_t*& list, uint64_t& cap) {
    list = t.list;
    cap = t.list_cap;
}
#endif
// the split's address and size, for the loop's rare paths (scalar loads)
__device__ __forceinline__ void cold_input(const uint8_t*& in, uint64_t& n) {
    typedef const __attribute__((address_space(4))) char* kptr;
    kptr p = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    const __attribute__((address_space(4))) MapArgs* ap = (const __attribute__((address_space(4))) MapArgs*)p;
    in = ap->in;
    n = ap->n;
}

// The map loop's DMA stream, advanced incrementally: the descriptor (base =
// the window start rounded down to 1 GiB, range = bytes to the split's end)
// changes only when the window offset passes 3 GiB, so a chunk's DMA costs one
// 32-bit add instead of recomputing the 64-bit base and range (~30 scalar
// instructions per chunk).  rebase() reads the split's address and size from
// the kernarg segment (a rare path: they need no SGPRs in the loop).
struct DmaStream {
    uint32_t base_lo, base_hi, nrec;  // descriptor words 0-2 (word 3 is constant)
    uint32_t voff;                    // offset of the window start (chunk start - 16) from the base
    __device__ __forceinline__ void set(const uint8_t* in, uint64_t n, uint64_t cs) {
        const uint64_t base = cs == 0 ? 0 : ((cs - kBack) & ~((1ull << 30) - 1));
        const uint64_t r = n - base;
        const uint32_t rhi = (uint32_t)(r >> 32), rlo = (uint32_t)r;
        nrec = (int32_t)rhi < 0 ? 0u : (rhi != 0 || rlo > 0xFFFFFF00u) ? 0xFFFFFF00u : rlo;
        const uint64_t b = (uint64_t)(in + base);
        base_lo = (uint32_t)b;
        base_hi = (uint32_t)(b >> 32) & 0xFFFFu;
        voff = (uint32_t)(cs - base) - kBack;
    }
    template <int kPol>
    __device__ __forceinline__ void issue(uint32_t lane, uint32_t lds_base) const {
        dma_chunk<kPol>((i32x4){(int)base_lo, (int)base_hi, (int)nrec, 0x00020000}, voff + 16u * lane, lds_base);
    }
};

// Long-word list: each map wave reserves kLongReserve entries at a time; the
// unused rest of a range is closed with kListHole entries (skipped by
// wc_long_kernel).
constexpr uint32_t kLongReserve = 256;
// the 2048-bucket layout drains its spill stores after each chunk (measured
// faster for the slot-wise appends: its 4096 streams per workgroup then leave L2
// less fragmented); whether the staged >64-miss appends do the same
#ifndef MRG_STAGE2_DRAIN
#define MRG_STAGE2_DRAIN 1
#endif
constexpr bool kStage2Drain = MRG_STAGE2_DRAIN != 0;
// UTF-8 chunks: leads decoded wave-compacted (utf8_mask16_wave) or by the
// per-lane loop (utf8_mask16)
#ifndef MRG_UTF8_WAVE
#define MRG_UTF8_WAVE 1
#endif
// word starts into the chunk's list one per loop turn (default) or two
#ifndef MRG_LIST_PAIRS
#define MRG_LIST_PAIRS 0
#endif
// Wave priority MRG_PRIO while a batch issues its list, key-byte and
// dictionary-set reads, 0 after: the SIMD's arbiter then issues a wave's
// dependent LDS round trips ahead of the other waves' compute, so more of them
// are in flight (C2 map 6.64-6.71 -> 6.54-6.57 ms, C5 -0.1 ms per 10 GB;
// profiles/ab_r06_prio.txt; priority 3 no better)
#ifndef MRG_PRIO
#define MRG_PRIO 1
#endif
// (A/B) the bucket aggregator's first-set lookups and count adds at this priority
#ifndef MRG_AGG_PRIO
#define MRG_AGG_PRIO 0
#endif
// (A/B) where: 0 the batch's reads (default), 1 through the dictionary count
// adds, 2 static (odd waves 1, even 0, no toggling), 3 the reads and the fast
// path's staging + cursor adds, 4 from the batch's reads to the chunk's end
#ifndef MRG_PRIO_MODE
#define MRG_PRIO_MODE 4
#endif
__device__ __forceinline__ void list_close(const Tables& t, uint64_t lbase, uint32_t lleft, uint32_t lane) {
    for (uint32_t g = 0; g < lleft; g += kWave)
        if (g + lane < lleft && lbase + g + lane < t.list_cap) t.list[lbase + g + lane] = kListHole;
}

// input loads are non-temporal (measured ~2 % faster than the default policy);
// the other policies are benchmark variants (map_mode 0x100 = default, 0x4000 =
// sc1, 0x8000 = sc0 sc1)
constexpr int dma_policy(uint32_t mode) { return (mode & 0x100) ? 0 : (mode & 0x4000) ? 2 : (mode & 0x8000) ? 3 : 1; }

template <uint32_t mode, int NW = kWavesPerWG, int NB = kSpillBuckets, bool kS = false, bool kLean = false>
__global__ void __launch_bounds__(kThreads) wc_map_kernel(const uint8_t* __restrict__ in, uint64_t n, uint32_t cbeg,
                                                          uint32_t cend, uint32_t ctail, int resume, Tables t,
                                                          LetterTables lt) {
    // mode (benchmark ablation only, compile-time; results are wrong unless 0):
    // 1 = stream input only, 2 = tokenize only (no per-word work), 4 = per-word
    // key extraction without the dictionary, 16 = no spill append (misses dropped),
    // 32 = spill cursors but no stores, 8 = dictionary counters not updated,
    // 64 = non-ASCII chunks classified by the ASCII rule (no rune decoding);
    // 0x100 / 0x4000 / 0x8000 (exact) = input loads with the default policy /
    // sc1 / sc0 sc1 instead of nt; staged kernel only: 0x10000 = the write-combining
    // round without its stores, 0x20000 = no round.  (Measured and removed, DESIGN.md §6: the 4
    // hottest keys counted by ballots into SGPRs; key bytes by three aligned
    // 8-byte reads; a single-choice dictionary lookup.)
    __shared__ MapLdsT<NW, NB, kS> L;
    static_assert(!kS || (NB == kSpillBucketsHi && NW == kWavesPerWG), "staged spill: the 2048-bucket layout, 16 waves");
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR) for the DMA operands
    if constexpr (MRG_PRIO != 0 && MRG_PRIO_MODE == 2) {
        if (wv & 1u) __builtin_amdgcn_s_setprio(1);
    }
    lds_uint4* dset = (lds_uint4*)L.dset;
    lds_u32* dcnt = (lds_u32*)L.dcnt;
    lds_u32* curs = (lds_u32*)L.curs;
    const lds_uint4* kmask4 = (const lds_uint4*)L.kmask;
    if (t.dbg && tid == 0) t.dbg[2 * (NB + blockIdx.x)] = __builtin_amdgcn_s_memrealtime();

    using Geo = typename MapLdsT<NW, NB, kS>::Geo;
    const bool use_dict = t.dict != nullptr;
    // NW (waves per workgroup) < kWavesPerWG only for the occupancy benchmark (map_mode 0x1000 / 0x2000)
    constexpr uint32_t kT = NW * kWave;
    for (uint32_t i = tid; i < (uint32_t)Geo::kSets; i += kT) dset[i] = use_dict ? to_v4(t.dict[i]) : (u32x4){0, 0, 0, 0};
    // chunks [cbeg, cend) of the split; resume: an earlier launch mapped chunks
    // before cbeg (host input streamed piece by piece), so this workgroup's spill
    // cursors and dictionary counts continue from what it wrote
    for (uint32_t i = tid; i < (uint32_t)Geo::kSlots + kWave; i += kT)
        dcnt[i] = resume && use_dict && i < (uint32_t)Geo::kSlots ? t.dict_cnt[(uint64_t)blockIdx.x * Geo::kSlots + i] : 0u;
    for (uint32_t b = tid; b < 2u * NB + kWave; b += kT) {
        uint32_t v = 0;
        if (resume && b < (uint32_t)NB) v = t.sp.counts8[(uint64_t)b * t.sp.nwg + blockIdx.x];
        else if (resume && b < 2u * NB) v = t.sp.counts[(uint64_t)(b - NB) * t.sp.nwg + blockIdx.x];
        curs[b] = v;
        if (kS && b < (uint32_t)NB) L.fl[b] = (uint16_t)v;  // everything before the cursor is written
    }
    for (uint32_t i = tid; i < (uint32_t)kLetterUnique * 8; i += kT) L.lt2[i] = lt.l2[i];
    for (uint32_t i = tid; i < (uint32_t)kLetterLdsPages; i += kT) L.lt1[i] = lt.l1[i];
    if (MapLdsT<NW, NB, kS>::kB2 && tid < 64) L.lb2[tid] = lt.b2[tid];
    const LdsLetters lds_lt{(const lds_u8*)L.lt1, (const lds_u32*)L.lt2,
                            MapLdsT<NW, NB, kS>::kB2 ? (const lds_u32*)L.lb2 : nullptr};
    if (tid < kMaskLens * 4) {  // byte masks: dword d of kmask[len] keeps clamp(len - 4d, 0, 4) bytes
        const int nb = min(max((int)(tid >> 2) - 4 * (int)(tid & 3), 0), 4);
        ((uint32_t*)L.kmask)[tid] = nb == 4 ? 0xFFFFFFFFu : (1u << (8 * nb)) - 1u;
    }
    __syncthreads();

    // chunk indices are 32-bit (the launcher checks): scalar compares, no 64-bit VALU ones
    const uint32_t stride = gridDim.x * NW;
    const uint32_t c0 = cbeg + blockIdx.x * NW + wv;
    const uint32_t sub = (uint32_t)t.sp.sub_keys, sub8 = (uint32_t)t.sp.sub8;
    // this workgroup's spill streams: [g][bucket][sub] (a workgroup's stores stay
    // within a few MiB, so they hit few TLB pages; mrgpu_internal.h Spill)
    const __amdgpu_buffer_rsrc_t rs8 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(t.sp.pool8 + (uint64_t)blockIdx.x * NB * sub8), (short)0, (int)(NB * sub8 * 8u),
        0x00020000);
    const __amdgpu_buffer_rsrc_t rs16 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(t.sp.pool + (uint64_t)blockIdx.x * NB * sub), (short)0, (int)(NB * sub * 16u),
        0x00020000);
    uint32_t ovf = 0, utf8_chunks = 0;
    // this wave's 32-byte long-word records so far (its own region: no atomic)
    // (in a VGPR, uniform: an SGPR live across the loop would be spilled)
    uint32_t lrec_w = resume && t.lrec ? t.lrec_cnt[blockIdx.x * kWavesPerWG + wv] : 0u;
    asm volatile("" : "+v"(lrec_w));
    uint64_t acc = 0;
    // this wave's reserved range of the long-word list: [lbase, lbase + lleft)
    uint64_t lbase = 0;
    uint32_t lleft = 0;
    const uint32_t ring0 = lds_addr(L.ring[wv][0]);
    static_assert(sizeof(L.ring) >= 4 * kWavesPerWG * sizeof(unsigned long long), "block_add4 scratch aliases the ring");

    // prologue: chunk c0 landed before the loop, chunk c0 + stride in flight
    // byte offsets advance by addition (64-bit scalar multiplies per iteration are not free)
    const uint64_t cstep = (uint64_t)stride * kOwn;
    dma_for_chunk<dma_policy(mode)>(in, n, (uint64_t)c0 * kOwn, lane, ring0);
    wait_vmem_all();
    dma_for_chunk<dma_policy(mode)>(in, n, (uint64_t)c0 * kOwn + cstep, lane, ring0 + kSlotStride);
    // the stream of the chunk two strides ahead (the loop's DMA)
    DmaStream ds;
    ds.set(in, n, (uint64_t)c0 * kOwn + 2 * cstep);
    const uint32_t cstep32 = (uint32_t)cstep;  // < 2^23: one add per chunk
    uint32_t k = 0;  // ring slot of the current chunk
    uint64_t cs = (uint64_t)c0 * kOwn;  // the current chunk's first own byte = slot byte 16 (slot byte i = input cs - 16 + i)
    // kf = the free slot (the word list now, chunk c + 2*stride next) = the slot
    // before k; both rotate as loop-carried scalars
    uint32_t kf = kRing - 1;
    // VMEM operations the previous iteration issued after the DMA now awaited,
    // beyond the base count (2 spill stores + the DMA; kS: 4 flush stores + the
    // DMA): kVmemWide - 2 after appends from the word slots, plus long-word record
    // and list stores.  Only operations it certainly issued are counted (an
    // uncounted one only lengthens the wait).  One scalar: the loop's SGPRs are
    // scarce (hipcc spills the excess to VGPR lanes, reloaded every chunk).
    uint32_t xv = 0;
    // kS: every wave runs the workgroup's trip count (its barriers), a chunk past
    // cend counting as empty
    const uint32_t cw0 = cbeg + blockIdx.x * NW;
    const uint32_t ktrips = kS && cw0 < cend ? (cend - cw0 + stride - 1) / stride : 0u;
    uint32_t trip = 0;
    for (uint32_t c = c0; kS ? trip < ktrips : c < cend;
         c += stride, cs += cstep, kf = k, k = k == kRing - 1 ? 0 : k + 1, trip++) {
        // chunk c's DMA (issued two iterations ago) has landed
        if constexpr (kS && (mode & 0x20000) == 0 && kFlushEvery == 1) wait_vmem_extra<5>(xv);
        else wait_vmem_extra<kVmemPerIter>(xv);  // (kFlushEvery > 1: a round adds its stores to xv)
        xv = 0;
        lds_u8* buf = (lds_u8*)L.ring[wv][k];
        const uint32_t bufa = ring0 + k * kSlotStride;  // = lds_addr(buf)
        lds_uint4* b4 = (lds_uint4*)buf;
        lds_u16* list = (lds_u16*)L.ring[wv][kf];
        if (c >= ctail) {  // the window reaches the split's last n % 4 bytes (ctail = ~0u: none)
            // the split's last n % 4 bytes sit in a dword the range check zero-filled
            const uint8_t* cin;
            uint64_t cn;
            cold_input(cin, cn);
            const int64_t p = (int64_t)(cn & ~3ull) + lane - ((int64_t)cs - kBack);
            if (lane < (uint32_t)(cn & 3) && p >= 0 && p < kSlotBytes + kSlotTail) buf[p] = cin[(cn & ~3ull) + lane];
            wait_vmem_all();
            wave_sync();
        }
        if constexpr ((mode & 1) != 0) {
            acc += buf[16 + lane];
        } else {
            // lane l holds slot bytes [16l, 16l+16): lane 0 = look-back, lanes 1-62 the
            // chunk's own 992 bytes, lane 63 = look-ahead
            const uint4 ca = from_v4(b4[lane]);
            const uint32_t hi = (ca.x | ca.y | ca.z | ca.w) & 0x80808080u;
            const bool ascii = __ballot(hi != 0) == 0;
            uint32_t mA;
            if (ascii || (mode & 64) != 0) {  // (mode 64, ablation: no rune decoding)
                mA = ascii_mask16(ca);
            } else {
                // UTF-8: ASCII letters by SWAR, one loop turn per lead byte, letter
                // tables in LDS.  A lead in the window's last 3 bytes whose sequence
                // runs past it needs the input bytes after the window: read then
                // (one lane; drained, so the counted wait still holds), else no
                // memory operation.
                utf8_chunks++;
                const uint32_t tl = lane == 63 ? ca.w >> 8 : 0u;  // slot bytes 1021..1023
                const uint32_t cross = ((tl & 0xF8u) >= 0xF0u ? 1u : 0u) | ((tl >> 8 & 0xF0u) >= 0xE0u ? 1u : 0u) |
                                       ((tl >> 16 & 0xE0u) >= 0xC0u ? 1u : 0u);
                if (__ballot(cross != 0)) {
                    if (lane < (uint32_t)kSlotTail) {
                        const uint8_t* cin;
                        uint64_t cn;
                        cold_input(cin, cn);
                        const uint64_t p = cs - kBack + kSlotBytes + lane;
                        buf[kSlotBytes + lane] = p < cn ? cin[p] : (uint8_t)0;
                    }
                    wait_vmem_all();
                    wave_sync();
                }
                if constexpr (MRG_UTF8_WAVE && !kLean) mA = utf8_mask16_wave(buf, lane, (lds_u8*)L.ring[wv][kf], lds_lt);
                else mA = utf8_mask16(buf, 16 * lane, lane == 0, lds_lt);
            }
            if (kS && c >= cend) mA = 0;  // a trip past this wave's last chunk: nothing to count
            // Word starts (a letter byte whose predecessor is not one) in the owned lanes
            // and lengths (ctz over this lane's mask and the next lane's), packed into the
            // list as slot position | len << 10 (a u16: len > 16 means a long word; no
            // terminator in the window gives ctz = -1, i.e. 63 in the u16's top bits and
            // 31 in the 5-bit mask-table index).  Neighbour masks by DPP.
            const uint32_t x1 = wave_shl1_z(mA);
            const uint32_t pv = wave_shr1_z(mA);
            // Non-letters of this lane's 16 bytes and the next lane's.  A word starts at
            // bit <= 15, so one of <= 16 bytes ends by bit 31; the length is the
            // distance to the next non-letter (v_ffbl: -1 when there is none, a word of
            // more than 16 bytes; the mask table has 32 entries, so any length indexes
            // it without a clamp).
            const uint32_t nl = ~(mA | (x1 << 16));
            // lanes 1..kOwnLanes as a constant lane mask (a compare result is
            // loop-invariant: hoisted, it was spilled to VGPR lanes and reloaded)
            static_assert(kOwnLanes == 62, "owned-lane mask");
            const bool owned = __builtin_amdgcn_inverse_ballot_w64(0x7FFFFFFFFFFFFFFEull);
            uint32_t SA = owned ? (mA & ~((mA << 1) | ((pv >> 15) & 1u)) & 0xFFFFu) : 0u;
            const uint32_t nsa = __popc(SA);
            const uint32_t incl = wave_incl_scan_dpp(nsa);
            const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
            uint32_t j = incl - nsa;
            const uint32_t pos0 = 16 * lane;
#if MRG_LIST_PAIRS
            // two starts per loop turn: the loop runs max-over-lanes(starts) / 2
            // turns, its control (compare, exec update, branch) paid once per pair
            // (A/B variant: C2's map kernel 6.95 vs 6.69 ms one per turn)
            while (SA) {
                const uint32_t b1 = ffbl_raw(SA);
                SA &= SA - 1;
                const uint32_t b2 = ffbl_raw(SA);  // -1: this lane had one start left
                const uint32_t e1 = (pos0 + b1) | (ffbl_raw(nl >> b1) << 10);  // len -1: no terminator in the window
                const uint32_t e2 = (pos0 + b2) | (ffbl_raw(nl >> (b2 & 31u)) << 10);
                list[j] = (uint16_t)e1;
                if (SA) list[j + 1] = (uint16_t)e2;
                SA &= SA - 1;
                j += 2;
            }
#else
            while (SA) {
                const uint32_t bit = __builtin_ctz(SA);
                const uint32_t len = ffbl_raw(nl >> bit);  // -1 when no terminator in the window
                list[j++] = (uint16_t)((pos0 + bit) | (len << 10));
                SA &= SA - 1;
            }
#endif
            wave_sync();
            if constexpr ((mode & 2) != 0) {
                acc += total;
            } else {
                // passes of kBatchWords words: a 992-byte chunk of text has ~170; a chunk
                // with more words drains after each extra pass (its VMEM count differs)
                const uint32_t passes = total == 0 ? 1u : (total + kBatchWords - 1) / kBatchWords;
                for (uint32_t pass = 0; pass < passes; pass++) {
                    const uint32_t base = pass * kBatchWords;
                    // The batch runs in phases so that every LDS round trip of the
                    // kBatch words is in flight at once (list entries -> key bytes ->
                    // dictionary sets -> counters / spill cursors), with no branches
                    // on per-lane outcomes: misses add to a per-lane dummy counter and
                    // hits bump a per-lane dummy cursor.
                    uint32_t e[kBatch];
                    if constexpr (MRG_PRIO != 0 && MRG_PRIO_MODE != 2) __builtin_amdgcn_s_setprio(MRG_PRIO);
        #pragma unroll
                    for (int u = 0; u < kBatch; u++) {
                        const uint32_t w = base + lane + 64u * u;
                        // slots past the list read stale LDS (w <= 575: inside the workgroup's
                        // allocation); every use below is masked by valid = w < total
                        e[u] = list[w];
                    }
                    // the 20 bytes [s & ~3, +20) of each key: five dword reads (the same LDS
                    // cycles as three aligned 8-byte reads, without their 8-byte-phase selects)
                    uint32_t g0[kBatch], g1[kBatch], g2[kBatch], g3[kBatch], g4[kBatch];
                    u32x4 km[kBatch];  // the key's byte mask, from the length (same round trip)
        #pragma unroll
                    for (int u = 0; u < kBatch; u++) {
                        const lds_u32* p4 = (const lds_u32*)(uintptr_t)(bufa + (e[u] & 0x3FCu));
                        g0[u] = p4[0]; g1[u] = p4[1]; g2[u] = p4[2]; g3[u] = p4[3]; g4[u] = p4[4];
                        km[u] = kmask4[__builtin_amdgcn_ubfe(e[u], 10, 5)];  // 32 entries: any 5-bit length
                    }
                    uint64_t k0[kBatch], k1[kBatch];
                    uint32_t hh[kBatch];
                    // lane masks straight from the compares, taken once before the
                    // long-word branch (a per-lane bool lives across a branch as a 0/1
                    // VGPR and is re-compared after it)
                    uint64_t mOk[kBatch], mLng[kBatch], mMid[kBatch];
        #pragma unroll
                    for (int u = 0; u < kBatch; u++) {
                        // w = base + 64 u + lane < total <=> lane + 64 u < total - base (lane + 64 u
                        // is loop-invariant, total - base a scalar; passes cover total: no wrap)
                        const uint32_t len = e[u] >> 10;
                        const uint64_t mValid = __ballot(lane + 64u * u < total - base), mLe16 = __ballot(len <= 16);
                        mOk[u] = mValid & mLe16;
                        mLng[u] = mValid & ~mLe16;
                        // 16 key bytes at [s, s+16)
                        const uint32_t sh = e[u];  // v_alignbyte uses only the low 2 bits of its shift
                        const uint32_t a0 = g0[u], a1 = g1[u], a2 = g2[u], a3 = g3[u], a4 = g4[u];
                        const uint32_t w0 = __builtin_amdgcn_alignbyte(a1, a0, sh);
                        const uint32_t w1 = __builtin_amdgcn_alignbyte(a2, a1, sh);
                        const uint32_t w2 = __builtin_amdgcn_alignbyte(a3, a2, sh);
                        const uint32_t w3 = __builtin_amdgcn_alignbyte(a4, a3, sh);
                        // keep the first min(len, 16) bytes
                        k0[u] = ((uint64_t)(w1 & km[u].y) << 32) | (w0 & km[u].x);
                        k1[u] = ((uint64_t)(w3 & km[u].w) << 32) | (w2 & km[u].z);
                        hh[u] = fold32((uint32_t)k0[u], (uint32_t)(k0[u] >> 32), (uint32_t)k1[u], (uint32_t)(k1[u] >> 32));
                        mMid[u] = __ballot(k1[u] != 0);
                    }
                    // words of more than 16 bytes: their starts go to the list, resolved by
                    // wc_long_kernel from the input.  Mixed-script text has them in most
                    // chunks (C2u: ~3 per chunk), so each wave appends into its own
                    // reserved range of the list (one device atomic per kLongReserve
                    // words: a same-address atomic per chunk serialized the whole kernel,
                    // 207 ms per 10 GB), with one store per chunk: the starts are staged
                    // in the list slot, whose entries are all read by now (one pass).
                    // The extra stores are counted (xv) by the next iteration's wait.
                    if (kLean && (mLng[0] | mLng[1] | mLng[2])) {
                        // kLean (splits whose predecessor was all ASCII): every long word
                        // through the start-offset list, the round-3 code, which keeps
                        // the loop's scalars out of VGPR-lane spills (the record path
                        // below costs the ASCII loop ~2 %)
                        if (passes == 1) {
                            lds_u64* lst = (lds_u64*)L.ring[wv][kf];
                            uint32_t nlong = 0;
        #pragma unroll
                            for (int u = 0; u < kBatch; u++) {
                                if (__builtin_amdgcn_inverse_ballot_w64(mLng[u]))
                                    lst[nlong + mbcnt64(mLng[u])] = cs - kBack + (e[u] & 0x3FFu);
                                nlong += (uint32_t)__popcll(mLng[u]);
                            }
                            const Tables& tc = cold(t);
                            if (nlong > lleft) {  // a fresh range (rare): close the old one, one atomic, drain
                                list_close(tc, lbase, lleft, lane);
                                const uint32_t want = kLongReserve;
                                unsigned long long b0 = 0;
                                if (lane == 0) b0 = atomicAdd(&tc.ctr->nlist, (unsigned long long)want);
                                lbase = readfirstlane64(b0);
                                lleft = want;
                                if (lbase + want > tc.list_cap && lane == 0) set_status(tc.ctr, kStListFull);
                                wait_vmem_all();
                            }
                            uint64_t* lptr;
                            uint64_t lcap;
                            cold_list(t, lptr, lcap);
                            const uint64_t room = lbase < lcap ? lcap - lbase : 0;
                            const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
                                (void*)(lptr + lbase), (short)0, (int)(room < (0xFFFFFF00ull >> 3) ? room * 8u : 0xFFFFFF00ull),
                                0x00020000);
                            const unsigned long long v = lst[lane];  // nlong <= 59 (> 16-byte words of 992 bytes)
                            __builtin_amdgcn_raw_buffer_store_b64((u32x2){(uint32_t)v, (uint32_t)(v >> 32)}, rsl,
                                                                  lane < nlong ? lane * 8u : kOutOfRange, 0, 0);
                            xv += 1;
                            lbase += nlong;
                            lleft -= nlong;
                        } else {  // several passes (> 192 words): the list slot is still needed
        #pragma unroll
                            for (int u = 0; u < kBatch; u++)
                                if (__builtin_amdgcn_inverse_ballot_w64(mLng[u])) list_append(cold(t), cs - kBack + (e[u] & 0x3FFu));
                            wait_vmem_all();
                        }
                    } else if (mLng[0] | mLng[1] | mLng[2]) {
                        if (passes == 1) {
                            // Words of 17-32 bytes that end inside the window leave as
                            // 32-byte key records, read here from the slot (wc_lrec_kernel
                            // counts them: no second decode of the input); longer words and
                            // words running past the window take the start-offset list.
                            // The batch's long words are first compacted into the list slot
                            // (its entries are all read by now: one pass), so one lane per
                            // long word does the rest in a single round (per word slot, a
                            // round for the one or two long words of each 64 cost ~3x).
                            // The length comes from the letter masks of the word's lane and
                            // the next two (ds_bpermute; lanes past 63 are unknown bytes,
                            // taken as letters, so a word reaching them falls back).
                            lds_u16* lst16 = (lds_u16*)L.ring[wv][kf];
                            uint32_t nlong = 0;
        #pragma unroll
                            for (int u = 0; u < kBatch; u++) {
                                if (__builtin_amdgcn_inverse_ballot_w64(mLng[u])) lst16[nlong + mbcnt64(mLng[u])] = (uint16_t)e[u];
                                nlong += (uint32_t)__popcll(mLng[u]);
                            }
                            wave_sync();
                            const bool have = lane < nlong;  // nlong <= 59 (> 16-byte words of 992 bytes)
                            const uint32_t p = have ? lst16[lane] & 0x3FFu : 0u;
                            const Tables& tr = cold(t);
#ifdef MRG_NO_LREC  // (A/B variant: every long word through the start-offset list)
                            const uint64_t mR = 0;
#else
                            const uint32_t lw = p >> 4;
                            const uint32_t m0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lw << 2), (int)mA);
                            const uint32_t m1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lw + 1) << 2), (int)mA);
                            const uint32_t m2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lw + 2) << 2), (int)mA);
                            const uint64_t win = (uint64_t)(m0 & 0xFFFFu) |
                                                 ((uint64_t)(lw + 1 < 64u ? m1 & 0xFFFFu : 0xFFFFu) << 16) |
                                                 ((uint64_t)(lw + 2 < 64u ? m2 & 0xFFFFu : 0xFFFFu) << 32) |
                                                 (0xFFFFull << 48);
                            const uint32_t wl = (uint32_t)__builtin_ctzll((~win >> (p & 15u)) | (1ull << 63));
                            const uint64_t mR = tr.lrec != nullptr ? __ballot(have && wl <= 32u) : 0ull;
                            if (mR) {
                                const uint32_t rbase = __builtin_amdgcn_readfirstlane(lrec_w);
                                lrec_w = rbase + (uint32_t)__popcll(mR);
                                asm volatile("" : "+v"(lrec_w));
                                const uint32_t rcap = tr.lrec_cap;
                                const uint32_t idx = rbase + mbcnt64(mR);
                                const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
                                    (void*)(tr.lrec + (uint64_t)(blockIdx.x * kWavesPerWG + wv) * rcap * 2u), (short)0, (int)(rcap * 32u), 0x00020000);
                                const uint32_t ro = __builtin_amdgcn_inverse_ballot_w64(mR) && idx < rcap ? idx * 32u : kOutOfRange;
                                // the key's 32 bytes from the slot, zero past its length, 16 at a
                                // time; the byte masks from the length table (kmask4[len]: the first
                                // min(len, 16) bytes), not per-dword clamps (~50 VALU fewer per turn)
                                const u32x4 mk[2] = {kmask4[wl < 31u ? wl : 31u], kmask4[wl > 16u ? wl - 16u : 0u]};
        #pragma unroll
                                for (int hf = 0; hf < 2; hf++) {
                                    const lds_u32* q4 = (const lds_u32*)(uintptr_t)(bufa + (p & ~3u) + 16u * hf);
                                    uint32_t d[5], k[4];
        #pragma unroll
                                    for (int i = 0; i < 5; i++) d[i] = q4[i];
                                    const uint32_t mw[4] = {mk[hf].x, mk[hf].y, mk[hf].z, mk[hf].w};
        #pragma unroll
                                    for (int i = 0; i < 4; i++) k[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], p) & mw[i];
                                    __builtin_amdgcn_raw_buffer_store_b128((u32x4){k[0], k[1], k[2], k[3]}, rsr,
                                                                           ro == kOutOfRange ? kOutOfRange : ro + 16u * hf, 0, 0);
                                }
                                xv += 2;  // the two record stores (the next wait counts them)
                                if (rbase + (uint32_t)__popcll(mR) > rcap && lane == 0) set_status(tr.ctr, kStLrecFull);
                            }
#endif
                            const uint64_t mFall = __ballot(have) & ~mR;
                            if (mFall) {
                                const uint32_t nfall = (uint32_t)__popcll(mFall);
                                const Tables& tc = cold(t);
                                if (nfall > lleft) {  // a fresh range (rare): close the old one, one atomic, drain
                                    list_close(tc, lbase, lleft, lane);
                                    const uint32_t want = kLongReserve;
                                    unsigned long long b0 = 0;
                                    if (lane == 0) b0 = atomicAdd(&tc.ctr->nlist, (unsigned long long)want);
                                    lbase = readfirstlane64(b0);
                                    lleft = want;
                                    if (lbase + want > tc.list_cap && lane == 0) set_status(tc.ctr, kStListFull);
                                    wait_vmem_all();
                                }
                                uint64_t* lptr;
                                uint64_t lcap;
                                cold_list(t, lptr, lcap);
                                // the descriptor starts at this range's next entry, so its 32-bit
                                // offsets never limit the list's size (a base at the list start
                                // dropped entries past 2^29 without a status bit: ADVICE r03); its
                                // range check stops at the list's capacity (kStListFull is set
                                // when a range is reserved past it, and the run is repeated)
                                const uint64_t room = lbase < lcap ? lcap - lbase : 0;
                                const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(
                                    (void*)(lptr + lbase), (short)0, (int)(room < (0xFFFFFF00ull >> 3) ? room * 8u : 0xFFFFFF00ull),
                                    0x00020000);
                                const uint64_t v = cs - kBack + p;  // the word's input offset
                                __builtin_amdgcn_raw_buffer_store_b64(
                                    (u32x2){(uint32_t)v, (uint32_t)(v >> 32)}, rsl,
                                    __builtin_amdgcn_inverse_ballot_w64(mFall) ? mbcnt64(mFall) * 8u : kOutOfRange, 0, 0);
                                xv += 1;
                                lbase += nfall;
                                lleft -= nfall;
                            }
                        } else {  // several passes (> 192 words): the list slot is still needed
        #pragma unroll
                            for (int u = 0; u < kBatch; u++)
                                if (__builtin_amdgcn_inverse_ballot_w64(mLng[u])) list_append(cold(t), cs - kBack + (e[u] & 0x3FFu));
                            wait_vmem_all();
                        }
                    }
                    if constexpr ((mode & 4) != 0) {
        #pragma unroll
                        for (int u = 0; u < kBatch; u++) acc += __builtin_amdgcn_inverse_ballot_w64(mOk[u]) ? hh[u] : 0u;
                        continue;
                    }
                    bool hit[kBatch];
                    uint64_t mHit[kBatch];  // lane mask of hit[]
                    if (use_dict) {
                        u32x4 A[kBatch], B[kBatch];
                        uint32_t a1[kBatch], a2[kBatch];  // byte offsets of the two sets
        #pragma unroll
                        for (int u = 0; u < kBatch; u++) {
                            dict_set_addrs<Geo>(hh[u], __builtin_amdgcn_inverse_ballot_w64(mMid[u]), a1[u], a2[u]);
                            A[u] = *(const lds_uint4*)((const lds_u8*)dset + a1[u]);
                            B[u] = *(const lds_uint4*)((const lds_u8*)dset + a2[u]);
                        }
                        __builtin_amdgcn_sched_barrier(0);  // all 2 * kBatch set reads in flight before the compares
                        if constexpr (MRG_PRIO != 0 && (MRG_PRIO_MODE == 0 || MRG_PRIO_MODE == 3)) __builtin_amdgcn_s_setprio(0);
        #pragma unroll
                        for (int u = 0; u < kBatch; u++) {
                            // short key: any of the 4 ways of its two sets; mid key: the single
                            // 16-byte way of either set (kk = the word compared with each set's
                            // second 8 bytes)
                            const bool mid = __builtin_amdgcn_inverse_ballot_w64(mMid[u]);
                            const uint64_t kk = mid ? k1[u] : k0[u];
                            const uint64_t alo = ((uint64_t)A[u].y << 32) | A[u].x, ahi = ((uint64_t)A[u].w << 32) | A[u].z;
                            const uint64_t blo = ((uint64_t)B[u].y << 32) | B[u].x, bhi = ((uint64_t)B[u].w << 32) | B[u].z;
                            // The hit logic runs on the wave's lane masks (uniform 64-bit values,
                            // scalar ops): per-lane bool logic compiles to exec-masked branches
                            // (&&, ||) or to 0/1 VALU arithmetic.  inverse_ballot reads this
                            // lane's bit back as a condition at no cost.  The batch runs with
                            // every lane active.
                            const uint64_t mMidU = mMid[u];
                            const uint64_t mA0 = __ballot(alo == k0[u]), mA1 = __ballot(ahi == kk);
                            const uint64_t mB0 = __ballot(blo == k0[u]), mB1 = __ballot(bhi == kk);
                            const uint64_t mHa = (mA0 & mA1) | (~mMidU & (mA0 | mA1));
                            const uint64_t mHb = (mB0 & mB1) | (~mMidU & (mB0 | mB1));
                            mHit[u] = mOk[u] & (mHa | mHb);
                            hit[u] = __builtin_amdgcn_inverse_ballot_w64(mHit[u]);
                            // way within the hit set (scalar mask logic), then one select of the set
                            const uint64_t mWay = ~mMidU & ((mHa & ~mA0) | (~mHa & ~mB0));
                            const uint32_t hset = __builtin_amdgcn_inverse_ballot_w64(mHa) ? a1[u] : a2[u];
                            // counter byte offset: 4 (2 set + way) = (set offset >> 1) + 4 way
                            const uint32_t cofs = (hset >> 1) + (__builtin_amdgcn_inverse_ballot_w64(mWay) ? 4u : 0u);
                            bool cnt_lds = hit[u];
                            if constexpr ((mode & 8) != 0) cnt_lds = false;  // ablation: counters not updated
                            // only the hit lanes add (exec-masked: two scalar ops, where a
                            // per-lane dummy counter for the misses cost a select)
                            if (cnt_lds)
                                __hip_atomic_fetch_add((lds_u32*)((lds_u8*)dcnt + cofs), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        }
                        if constexpr (MRG_PRIO != 0 && MRG_PRIO_MODE == 1) __builtin_amdgcn_s_setprio(0);
                    } else {
                        if constexpr (MRG_PRIO != 0 && MRG_PRIO_MODE != 2 && MRG_PRIO_MODE != 4) __builtin_amdgcn_s_setprio(0);
        #pragma unroll
                        for (int u = 0; u < kBatch; u++) {
                            hit[u] = false;
                            mHit[u] = 0;
                        }
                    }
                    if constexpr ((mode & 16) != 0) {
        #pragma unroll
                        for (int u = 0; u < kBatch; u++) acc += hit[u];
                        continue;
                    }
                    // Misses: append to this workgroup's stream of the key's bucket.  A spill
                    // store costs per instruction (TA cycles per wave-instruction), so the
                    // pass's misses are first compacted: staged as 16-byte (k0,k1) records in
                    // the chunk's own ring slot (free once its key bytes are in registers)
                    // at their rank, then lane i appends record i — one cursor add and
                    // one 8-byte plus one 16-byte store per chunk instead of per word slot.
                    // Chunks of several passes (slot still needed) or with more than 64
                    // misses append from the word slots and drain (their VMEM count differs).
                    uint64_t mMiss[kBatch], mBig[kBatch];
                    uint32_t nmu[kBatch + 1];
                    nmu[0] = 0;
        #pragma unroll
                    for (int u = 0; u < kBatch; u++) {
                        mMiss[u] = mOk[u] & ~mHit[u];
                        mBig[u] = mMid[u];  // key of 9-16 bytes: 16-byte record
                        nmu[u + 1] = nmu[u] + (uint32_t)__popcll(mMiss[u]);
                    }
                    const uint32_t nm = nmu[kBatch];
                    if (passes == 1 && nm <= (uint32_t)kWave) {
                        if constexpr (MRG_PRIO != 0 && MRG_PRIO_MODE == 3) __builtin_amdgcn_s_setprio(MRG_PRIO);
                        lds_uint4* stage = (lds_uint4*)buf;
        #pragma unroll
                        for (int u = 0; u < kBatch; u++)
                            if (__builtin_amdgcn_inverse_ballot_w64(mMiss[u]))
                                stage[nmu[u] + mbcnt64(mMiss[u])] =
                                    (u32x4){(uint32_t)k0[u], (uint32_t)(k0[u] >> 32), (uint32_t)k1[u], (uint32_t)(k1[u] >> 32)};
                        const u32x4 r = stage[lane];  // this wave's own writes, in order
                        const bool valid = lane < nm;
                        const uint32_t b = spill_bucket<NB>(fold32(r.x, r.y, r.z, r.w));
                        const bool big = (r.z | r.w) != 0;
                        const uint32_t ci = valid ? b + (big ? (uint32_t)NB : 0u) : 2u * NB + lane;
                        const uint32_t pos = __hip_atomic_fetch_add(&curs[ci], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if constexpr (MRG_PRIO != 0 && MRG_PRIO_MODE == 3) __builtin_amdgcn_s_setprio(0);
                        if constexpr ((mode & 32) != 0) {
                            acc += pos;
                            continue;
                        }
                        // exactly two store instructions per chunk: lanes with nothing to store
                        // get an out-of-range offset, which the range check drops (the loop's
                        // VMEM count stays fixed, so its DMA waits are counted)
                        const bool fit8 = pos < sub8, fit16 = pos < sub;
                        const bool put8 = valid & !big & fit8, put16 = valid & big & fit16;
                        uint32_t o8 = put8 ? (__umul24(b, sub8) + pos) * 8u : kOutOfRange;
                        if constexpr (kS) o8 = stage_or_store(L, b, pos, ((uint64_t)r.y << 32) | r.x, o8);
                        __builtin_amdgcn_raw_buffer_store_b64((u32x2){r.x, r.y}, rs8, o8, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b128(r, rs16, put16 ? (__umul24(b, sub) + pos) * 16u : kOutOfRange,
                                                               0, 0);
                        // (lane masks, not a per-lane bool: no 0/1 VGPR round trip)
                        const uint64_t mBigS = __ballot(big), mF8 = __ballot(fit8), mF16 = __ballot(fit16);
                        const uint64_t mOver = __ballot(valid) & ((mBigS & ~mF16) | (~mBigS & ~mF8));
                        if (mOver) {  // a stream is full: count in the HBM table; the bucket then merges through it
                            if (__builtin_amdgcn_inverse_ballot_w64(mOver)) {
                                const Tables& tc = cold(t);
                                short_insert(tc, ((uint64_t)r.y << 32) | r.x, ((uint64_t)r.w << 32) | r.z, 1);
                                tc.bflag[b] = 1u;
                                ovf++;
                            }
                            wait_vmem_all();
                        }
                        continue;  // passes == 1
                    }
#ifndef MRG_NO_STAGE2
                    // More than 64 misses (high-cardinality text: most chunks of C5),
                    // one pass: the short misses staged as 8-byte keys in the chunk's
                    // slot (up to 128) and the 9-16-byte ones as 16-byte records in the
                    // list slot (free once the list entries are in registers; up to
                    // 64), then appended by type: two 8-byte and one 16-byte store
                    // instruction, every lane a record (the slot-wise appends below
                    // issue six stores, two thirds of their lanes out of range).
                    // Three stores after the DMA: the next counted wait, vmcnt(3),
                    // still leaves only them in flight.
                    uint32_t n8u[kBatch + 1], n16u[kBatch + 1];
                    n8u[0] = n16u[0] = 0;
        #pragma unroll
                    for (int u = 0; u < kBatch; u++) {
                        n8u[u + 1] = n8u[u] + (uint32_t)__popcll(mMiss[u] & ~mBig[u]);
                        n16u[u + 1] = n16u[u] + (uint32_t)__popcll(mMiss[u] & mBig[u]);
                    }
                    // (the high-cardinality layout only: in the default kernel the extra
                    // path's live state pushed the loop's scalars back into VGPR-lane spills)
                    if (NB == kSpillBucketsHi && passes == 1 && n8u[kBatch] <= 2u * kWave && n16u[kBatch] <= (uint32_t)kWave) {
                        lds_u64* st8 = (lds_u64*)buf;
                        lds_uint4* st16 = (lds_uint4*)L.ring[wv][kf];
        #pragma unroll
                        for (int u = 0; u < kBatch; u++) {
                            const uint64_t m8 = mMiss[u] & ~mBig[u], m16 = mMiss[u] & mBig[u];
                            if (__builtin_amdgcn_inverse_ballot_w64(m8)) st8[n8u[u] + mbcnt64(m8)] = k0[u];
                            if (__builtin_amdgcn_inverse_ballot_w64(m16))
                                st16[n16u[u] + mbcnt64(m16)] =
                                    (u32x4){(uint32_t)k0[u], (uint32_t)(k0[u] >> 32), (uint32_t)k1[u], (uint32_t)(k1[u] >> 32)};
                        }
                        const uint32_t n8 = n8u[kBatch], n16 = n16u[kBatch];
                        uint64_t mOverAll = 0;
        #pragma unroll
                        for (int h = 0; h < 3; h++) {  // 8-byte records lane, lane + 64; then 16-byte records
                            const bool big = h == 2;
                            const uint32_t i = lane + (h == 1 ? (uint32_t)kWave : 0u);
                            const bool valid = i < (big ? n16 : n8);
                            u32x4 r;
                            if (big) {
                                r = st16[lane];
                            } else {
                                const unsigned long long v = st8[i];
                                r = (u32x4){(uint32_t)v, (uint32_t)(v >> 32), 0u, 0u};
                            }
                            const uint32_t b = spill_bucket<NB>(big ? fold32(r.x, r.y, r.z, r.w) : fold32(r.x, r.y, 0u, 0u));
                            const uint32_t ci = valid ? b + (big ? (uint32_t)NB : 0u) : 2u * NB + lane;
                            const uint32_t pos = __hip_atomic_fetch_add(&curs[ci], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            if constexpr ((mode & 32) != 0) {
                                acc += pos;
                                continue;
                            }
                            const bool fit = pos < (big ? sub : sub8);
                            if (big)
                                __builtin_amdgcn_raw_buffer_store_b128(r, rs16, valid && fit ? (__umul24(b, sub) + pos) * 16u : kOutOfRange,
                                                                       0, 0);
                            else {
                                uint32_t o8 = valid && fit ? (__umul24(b, sub8) + pos) * 8u : kOutOfRange;
                                if constexpr (kS) o8 = stage_or_store(L, b, pos, ((uint64_t)r.y << 32) | r.x, o8);
                                __builtin_amdgcn_raw_buffer_store_b64((u32x2){r.x, r.y}, rs8, o8, 0, 0);
                            }
                            const uint64_t mOver = __ballot(valid) & ~__ballot(fit);
                            if (mOver) {  // a stream is full: count in the HBM table; the bucket then merges through it
                                if (__builtin_amdgcn_inverse_ballot_w64(mOver)) {
                                    const Tables& tc = cold(t);
                                    short_insert(tc, ((uint64_t)r.y << 32) | r.x, ((uint64_t)r.w << 32) | r.z, 1);
                                    tc.bflag[b] = 1u;
                                    ovf++;
                                }
                                mOverAll |= mOver;
                            }
                        }
                        if (mOverAll) wait_vmem_all();
                        if constexpr (NB == kSpillBucketsHi && kStage2Drain) wait_vmem_all();
                        continue;  // passes == 1
                    }
#endif
                    uint32_t pos[kBatch];
        #pragma unroll
                    for (int u = 0; u < kBatch; u++) {
                        const uint32_t b = spill_bucket<NB>(hh[u]);
                        const uint32_t ci = __builtin_amdgcn_inverse_ballot_w64(mMiss[u])
                                                ? b + (__builtin_amdgcn_inverse_ballot_w64(mBig[u]) ? (uint32_t)NB : 0u)
                                                : 2u * NB + lane;  // per-lane dummy cursor
                        pos[u] = __hip_atomic_fetch_add(&curs[ci], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    if constexpr ((mode & 32) != 0) {
        #pragma unroll
                        for (int u = 0; u < kBatch; u++) acc += pos[u];
                        continue;
                    }
        #pragma unroll
                    for (int u = 0; u < kBatch; u++) {
                        const uint32_t b = spill_bucket<NB>(hh[u]);
                        const uint64_t mFit8 = __ballot(pos[u] < sub8), mFit16 = __ballot(pos[u] < sub);
                        const uint64_t mPut8 = mMiss[u] & ~mBig[u] & mFit8, mPut16 = mMiss[u] & mBig[u] & mFit16;
                        uint32_t o8 = __builtin_amdgcn_inverse_ballot_w64(mPut8) ? (__umul24(b, sub8) + pos[u]) * 8u : kOutOfRange;
                        if constexpr (kS) o8 = stage_or_store(L, b, pos[u], k0[u], o8);
                        const uint32_t o16 = __builtin_amdgcn_inverse_ballot_w64(mPut16) ? (__umul24(b, sub) + pos[u]) * 16u : kOutOfRange;
                        __builtin_amdgcn_raw_buffer_store_b64((u32x2){(uint32_t)k0[u], (uint32_t)(k0[u] >> 32)}, rs8, o8, 0, 0);
                        __builtin_amdgcn_raw_buffer_store_b128(
                            (u32x4){(uint32_t)k0[u], (uint32_t)(k0[u] >> 32), (uint32_t)k1[u], (uint32_t)(k1[u] >> 32)},
                            rs16, o16, 0, 0);
                        const uint64_t mOver = mMiss[u] & ((mBig[u] & ~mFit16) | (~mBig[u] & ~mFit8));
                        if (mOver) {  // rare: HBM-table inserts, then drain (the counted wait assumes stores only)
                            if (__builtin_amdgcn_inverse_ballot_w64(mOver)) {
                                const Tables& tc = cold(t);
                                short_insert(tc, k0[u], k1[u], 1);
                                tc.bflag[b] = 1u;
                                ovf++;
                            }
                            wait_vmem_all();
                        }
                    }
                    // one pass (<= kBatchWords words, > 64 misses: high-cardinality text):
                    // exactly kVmemWide stores, counted by the next iteration's wait (a
                    // drain here would also wait for the DMA issued one chunk ahead);
                    // several passes: a different count, drain
                    // (2048 buckets: drained — the 4096 streams per workgroup then leave
                    // L2 less fragmented: C5 map 39.8 ms counted vs 35.5 drained)
                    if (passes == 1 && NB != kSpillBucketsHi) xv += (uint32_t)kVmemWide - 2u;
                    else wait_vmem_all();
                }
            }
        }
        if constexpr (kS && (mode & 0x20000) == 0) if (kFlushEvery == 1 || trip % kFlushEvery == kFlushEvery - 1) {
            // Write-combining round: after a barrier every stream whose LDS group
            // holds 4 records writes them as one 32-byte store (a full sector; the
            // 2048-bucket layout's 4096 streams per workgroup otherwise leave the
            // XCD's L2 half-written lines: 3.3x write amplification on C5), then
            // the group restarts at the stream's cursor (records past the group
            // were stored directly).  2 streams per thread, 4 store instructions
            // per wave (out-of-range offsets for the rest): a fixed VMEM count.
            __syncthreads();
            bool rare = false;
#pragma unroll
            for (uint32_t q = 0; q < (uint32_t)NB / kT; q++) {
                const uint32_t b = tid + q * kT;
                const uint32_t cc = curs[b];
                const uint32_t f = cc - ((cc - (uint32_t)L.fl[b]) & 0xFFFFu);
                const bool grp = cc - f >= 4u;
                const bool whole = grp && f + 4u <= sub8;
                const bool put = whole && (mode & 0x10000) == 0;  // (ablation 0x10000: the round without its stores)
                const u32x4 lo = *(const lds_uint4*)&L.stage8[b][0], hi = *(const lds_uint4*)&L.stage8[b][2];
                const uint32_t o = (__umul24(b, sub8) + f) * 8u;
                __builtin_amdgcn_raw_buffer_store_b128(lo, rs8, put ? o : kOutOfRange, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b128(hi, rs8, put ? o + 16u : kOutOfRange, 0, 0);
                if (grp && !whole) {  // the group reaches past the stream's capacity: its records below it
                    for (uint32_t j = 0; j < 4u; j++)
                        if (f + j < sub8) t.sp.pool8[((uint64_t)blockIdx.x * NB + b) * sub8 + f + j] = L.stage8[b][j];
                    rare = true;
                }
                if (grp) L.fl[b] = (uint16_t)cc;
            }
            if (__ballot(rare)) wait_vmem_all();  // (other VMEM operations: the counted wait no longer holds)
            __syncthreads();  // the groups and fl are reused by the next round's appends
            if constexpr (kFlushEvery > 1) xv += 2;  // (the next wait: vmcnt(5), as with a round every trip)
        }
        if constexpr (MRG_PRIO != 0 && MRG_PRIO_MODE == 4) __builtin_amdgcn_s_setprio(0);
        wave_sync();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every LDS read of slot kf (the list) has returned
        ds.issue<dma_policy(mode)>(lane, ring0 + kf * kSlotStride);
        ds.voff += cstep32;
        if (ds.voff >= (3u << 30)) {  // rare: the window moved 2 GiB past the base
            const uint8_t* cin;
            uint64_t cn;
            cold_input(cin, cn);
            ds.set(cin, cn, cs + 3 * cstep);
        }
    }
    list_close(t, lbase, lleft, lane);
    wait_vmem_all();  // the ring's last DMAs land before the workgroup's LDS is reused

    __syncthreads();
    if constexpr (kS) {  // the streams' last partial groups
        for (uint32_t b = tid; b < (uint32_t)NB; b += kT) {
            const uint32_t cc = curs[b];
            const uint32_t f = cc - ((cc - (uint32_t)L.fl[b]) & 0xFFFFu);
            for (uint32_t j = 0; f + j < cc && j < 4u; j++)  // (kFlushEvery > 1: a full group, the rest stored directly)
                if (f + j < sub8) t.sp.pool8[((uint64_t)blockIdx.x * NB + b) * sub8 + f + j] = L.stage8[b][j];
        }
    }
    if (lane == 0 && t.lrec) t.lrec_cnt[blockIdx.x * kWavesPerWG + wv] = lrec_w;
    unsigned long long spilled = 0, hits = 0, sp16 = 0;
    for (uint32_t b = tid; b < (uint32_t)NB; b += kT) {  // (this launch's share: minus the resumed values)
        const uint32_t k8 = min((uint32_t)curs[b], sub8), k = min((uint32_t)curs[NB + b], sub);
        uint32_t* p16 = &t.sp.counts[(uint64_t)b * t.sp.nwg + blockIdx.x];
        uint32_t* p8 = &t.sp.counts8[(uint64_t)b * t.sp.nwg + blockIdx.x];
        spilled += k + k8 - (resume ? *p16 + *p8 : 0u);
        sp16 += k - (resume ? *p16 : 0u);
        *p16 = k;
        *p8 = k8;
    }
    if (use_dict)
        for (uint32_t i = tid; i < (uint32_t)Geo::kSlots; i += kT) {
            const uint32_t v = dcnt[i];
            uint32_t* pd = &t.dict_cnt[(uint64_t)blockIdx.x * Geo::kSlots + i];
            hits += v - (resume ? *pd : 0u);
            *pd = v;
        }
    if (acc == 0x5eed5eedull) atomicAdd(&t.ctr->lds_miss, 1ull);  // keeps ablation builds honest (no DCE)
    block_add4<NW>(&t.ctr->spilled, &t.ctr->dict_hits, &t.ctr->spill_ovf, &t.ctr->chunks_utf8, spilled, hits,
                            ovf, lane == 0 ? utf8_chunks : 0, (unsigned long long*)&L.ring[0][0][0]);
    block_add4<NW>(&t.ctr->spilled16, nullptr, nullptr, nullptr, sp16, 0, 0, 0, (unsigned long long*)&L.ring[0][0][0]);
    if (t.dbg && tid == 0) t.dbg[2 * (NB + blockIdx.x) + 1] = __builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------------ bucket aggregator tables
// Two LDS tables per bucket, both 4-way set-associative with two-choice sets:
//   short keys (<= 8 bytes, k1 == 0): the 4 keys of a set are 32 contiguous
//     bytes (two ds_read_b128); a way is claimed by CAS 0 -> key, which also
//     publishes it, so a lookup is one LDS round trip;
//   mid keys (9-16 bytes): a way is 16 bytes (k0, k1), a set 64 bytes (four
//     ds_read_b128, one round trip); a way is claimed by CAS on k0, then k1 is
//     published (kUnwritten until then; 0xFF bytes never occur in UTF-8).
// Ways are never freed, so once a key's first set is full a key absent from it
// can never appear there later: lookups and claims agree on the key's set.
// Two table sizes: round 0 uses 512-thread workgroups, two per CU (1024 short
// sets = 4096 short keys + 1024 mid keys: a C2 bucket holds ~2 K distinct
// keys); later rounds of high-cardinality splits use one 1024-thread workgroup
// per CU with twice the keys, so a bucket settles in fewer rounds.
// (SW: ways per short set, 4 or 2 — A/B option MRG_AGG_WAYS: a 2-way set is one
// 16-byte read instead of two, with twice the sets for the same keys)
#ifndef MRG_AGG_WAYS
#define MRG_AGG_WAYS 4
#endif
template <int NS, int NM, int NW, int SW = 4>
struct alignas(16) AggLdsT {
    static constexpr int kShortSets = NS, kMidSets = NM, kShortWays = SW;
    static_assert(SW == 4 || SW == 2, "short set ways");
    static constexpr uint32_t kWaves = NW;
    static constexpr uint32_t kParts = NW / kAggSegs;  // waves per miss segment
    unsigned long long sk[NS * SW];
    unsigned long long mk[NM * 4 * 2];  // way w of set s: mk[2(4s+w)] = k0, mk[2(4s+w)+1] = k1
    uint32_t sc[NS * SW + kWave];       // counts (+ per-lane dummies for branch-free adds)
    uint32_t mc[NM * 4 + kWave];
    unsigned long long red[4 * NW + 4];  // block_add4 / block_alloc scratch
    uint32_t ncur8[kAggSegs], ncur16[kAggSegs];  // misses appended to each segment
};
using AggLds = AggLdsT<1024 * 4 / MRG_AGG_WAYS, 256, kAggThreads / kWave, MRG_AGG_WAYS>;
using AggLdsBig = AggLdsT<2048 * 4 / MRG_AGG_WAYS, 512, 2 * kAggThreads / kWave, MRG_AGG_WAYS>;
static_assert(AggLds::kWaves == kAggSegs && AggLdsBig::kWaves == 2 * kAggSegs, "waves per miss segment");
static_assert(2 * sizeof(AggLds) <= 160 * 1024, "two aggregator workgroups per CU");
static_assert(sizeof(AggLdsBig) <= 160 * 1024, "one big aggregator workgroup per CU");

// Claim attempts before a key is deferred to the next round (a lost race re-reads
// and retries: the winner, often the same key, published its way with its CAS).
constexpr int kClaimAttempts = 4;
__device__ __forceinline__ uint32_t second_hash(uint32_t h) { return __builtin_amdgcn_alignbit(h, h, 16) * 0xC2B2AE3Du; }
template <int NSETS, int WAYS = 4>
__device__ __forceinline__ uint32_t set_base(uint32_t h) { return __umulhi(h, NSETS) * WAYS; }
// the first way of a short key's set (first or second choice)
template <class AL>
__device__ __forceinline__ uint32_t sbase(uint32_t h) { return set_base<AL::kShortSets, AL::kShortWays>(h); }

// way masks (4 or 2 bits) of a short set holding k / holding 0
template <class AL>
__device__ __forceinline__ void short_set_masks(const AL& A, uint32_t base, uint64_t k, uint32_t& m, uint32_t& z) {
    const u64x2 a = *(const lds_u64x2*)(&A.sk[base]);
    if constexpr (AL::kShortWays == 2) {
        m = (a.x == k ? 1u : 0u) | (a.y == k ? 2u : 0u);
        z = (a.x == 0 ? 1u : 0u) | (a.y == 0 ? 2u : 0u);
    } else {
        const u64x2 b = *(const lds_u64x2*)(&A.sk[base + 2]);
        m = (a.x == k ? 1u : 0u) | (a.y == k ? 2u : 0u) | (b.x == k ? 4u : 0u) | (b.y == k ? 8u : 0u);
        z = (a.x == 0 ? 1u : 0u) | (a.y == 0 ? 2u : 0u) | (b.x == 0 ? 4u : 0u) | (b.y == 0 ? 8u : 0u);
    }
}

// Slow path of a short key absent from the first read of its first set:
// claim in the first set, else find/claim in the second.  A lost claim is
// retried once (the winner, often the same key, published it with its CAS).
// Returns false (a miss: the caller defers the key, where it is still counted
// exactly) when both sets are full without the key or claims keep racing.
// (Measured: passing the caller's "first set full" to start at the second set
// made C5's aggregation 51 -> 79 ms, a code-generation effect; not done.)
template <class AL>
__device__ bool short_insert_slow(AL& A, uint64_t k, uint32_t h, uint32_t add) {
    for (int attempt = 0; attempt < kClaimAttempts; attempt++) {
        bool raced = false;
        for (int c = 0; c < 2 && !raced; c++) {
            const uint32_t base = sbase<AL>(c == 0 ? h : second_hash(h));
            uint32_t m, z;
            short_set_masks(A, base, k, m, z);
            if (m) {
                atomicAdd(&A.sc[base + __builtin_ctz(m)], add);
                return true;
            }
            if (z) {
                const uint32_t w = base + __builtin_ctz(z);
                const unsigned long long old = atomicCAS(&A.sk[w], 0ull, (unsigned long long)k);
                if (old == 0ull || old == k) {
                    atomicAdd(&A.sc[w], add);
                    return true;
                }
                raced = true;  // lost the way to another key: re-read from the first set
            }
            // set full without the key: the second set (after the first)
        }
        if (!raced) return false;  // both sets full without the key: a retry reads the same
    }
    return false;
}

// Mid keys: way masks of a set (64 bytes, four b128 reads)
template <class AL>
__device__ __forceinline__ void mid_set_masks(const AL& A, uint32_t base, uint64_t k0, uint64_t k1, uint32_t& m,
                                              uint32_t& z, uint32_t& pend) {
    m = z = pend = 0;
#pragma unroll
    for (uint32_t w = 0; w < 4; w++) {
        const u64x2 e = *(const lds_u64x2*)(&A.mk[2 * (base + w)]);
        m |= (e.x == k0 && e.y == k1) ? 1u << w : 0u;
        z |= e.x == 0 ? 1u << w : 0u;
        pend |= (e.x == k0 && e.y == kUnwritten) ? 1u << w : 0u;  // claimed by this key's k0, k1 not yet visible
    }
}

template <class AL>
__device__ bool mid_insert(AL& A, uint64_t k0, uint64_t k1, uint32_t h, uint32_t add) {
    for (int attempt = 0; attempt < kClaimAttempts; attempt++) {
        bool raced = false;
        for (int c = 0; c < 2 && !raced; c++) {
            const uint32_t base = set_base<AL::kMidSets>(c == 0 ? h : second_hash(h));
            uint32_t m, z, pend;
            mid_set_masks(A, base, k0, k1, m, z, pend);
            if (m) {
                atomicAdd(&A.mc[base + __builtin_ctz(m)], add);
                return true;
            }
            if (pend) {  // a way of this k0 is being published: retry (or defer)
                raced = true;
                continue;
            }
            if (z) {
                const uint32_t w = base + __builtin_ctz(z);
                if (atomicCAS(&A.mk[2 * w], 0ull, (unsigned long long)k0) == 0ull) {
                    __hip_atomic_store(&A.mk[2 * w + 1], (unsigned long long)k1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    atomicAdd(&A.mc[w], add);
                    return true;
                }
                raced = true;
            }
        }
        if (!raced) return false;  // both sets full without the key
    }
    return false;
}

// Exact lookups in tables no lane is claiming in any more; -1 if absent.
template <class AL>
__device__ __forceinline__ int short_find_exact(const AL& A, uint64_t k, uint32_t h) {
    for (int c = 0; c < 2; c++) {
        const uint32_t base = sbase<AL>(c == 0 ? h : second_hash(h));
        for (uint32_t w = 0; w < (uint32_t)AL::kShortWays; w++)
            if (A.sk[base + w] == k) return (int)(base + w);
    }
    return -1;
}
template <class AL>
__device__ __forceinline__ int mid_find_exact(const AL& A, uint64_t k0, uint64_t k1, uint32_t h) {
    for (int c = 0; c < 2; c++) {
        const uint32_t base = set_base<AL::kMidSets>(c == 0 ? h : second_hash(h));
        for (uint32_t w = 0; w < 4; w++)
            if (A.mk[2 * (base + w)] == k0 && A.mk[2 * (base + w) + 1] == k1) return (int)(base + w);
    }
    return -1;
}

// Write record o (distinct short key with its total) of t.out.
__device__ __forceinline__ void put_short(const Tables& t, unsigned long long o, uint64_t k0, uint64_t k1, uint64_t cnt,
                                          bool strict) {
    if (o >= t.out_cap) {
        if (strict) set_status(t.ctr, kStRecFull);
        return;
    }
    const uint32_t len = key_len_short(k0, k1);
    t.out.k0[o] = k0;
    t.out.k1[o] = k1;
    t.out.len[o] = len;
    t.out.cnt[o] = cnt;
    t.out.part[o] = short_partition(k0, k1, len, t.nreduce);
    t.out.koff[o] = ~0ull;
}

// ------------------------------------------------------------ bucket aggregation
// Wave w walks streams w, w + kAggWaves, ... of the bucket (one stream per map
// workgroup), each contiguously: blocks of kAggUnroll * 64 records (8 per lane
// for 8-byte records, 4 for 16-byte ones), the next
// block's loads in flight while the current one is counted.  Every record of a
// block is looked up in one LDS round trip (all the block's set reads issued
// together); hits add (a per-lane dummy counter for lanes without one), and
// only first occurrences and collisions take the claim path.

// A key the tables could not take: appended to the wave's own miss segment
// (LDS cursor, no HBM round trip in the loop).  It never exceeds the segment:
// a wave's misses are at most the records it reads.
template <class AL>
__device__ __forceinline__ void defer_miss(AL& A, const Tables& t, uint64_t k0, uint64_t k1, bool keep_miss,
                                           uint32_t wv, uint64_t& miss) {
    if (keep_miss) {
        const uint32_t sg = wv % kAggSegs;  // the wave's segment (kParts waves share one)
        const uint64_t seg = (uint64_t)blockIdx.x * kAggSegs + sg;
        // (the buffers are sized from an earlier split's layout unless the host
        // read this one's: a miss past them flags the run, which is repeated)
        if (k1 == 0) {
            const uint32_t pos = atomicAdd(&A.ncur8[sg], 1u);
            const uint64_t at = t.sp.seg_off8[seg] + pos;
            if (at < t.sp.seg8_cap) t.sp.seg8_out[at] = k0;
            else set_status(t.ctr, kStSegFull);
        } else {
            const uint32_t pos = atomicAdd(&A.ncur16[sg], 1u);
            const uint64_t at = t.sp.seg_off16[seg] + pos;
            if (at < t.sp.seg16_cap)
                t.sp.seg16_out[at] = make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32));
            else set_status(t.ctr, kStSegFull);
        }
    }
    miss++;
}

template <uint32_t amode, bool kMid, uint32_t kAggUnroll, bool kRound0, class AL>
__device__ __forceinline__ void agg_pool(AL& A, const Tables& t, const void* pool_b, const uint32_t* gcounts,
                                         uint64_t gstride, uint32_t nwg, const uint64_t* gbase, bool keep_miss,
                                         uint64_t& miss) {
    // Streams s < nwg.  Map streams (gbase null): gcounts[s] records at
    // pool_b[s * gstride].  Miss segments (gbase set, nwg = kAggSegs * kParts):
    // stream s is part s / kAggSegs of segment s % kAggSegs (gcounts[seg]
    // records at gbase[seg]), split evenly between the segment's waves.
    constexpr uint32_t kAggWaves = AL::kWaves;
    constexpr uint32_t kAggBlock = kAggUnroll * kWave;
    static_assert(kMaxMapWGs <= kAggWaves * kWave, "a wave's stream counts fit one VGPR");
    auto part_range = [&](uint32_t sid, uint32_t& begin) -> uint32_t {
        const uint32_t nseg = gcounts[sid % kAggSegs], pt = sid / kAggSegs;
        begin = (uint32_t)((uint64_t)nseg * pt / AL::kParts);
        return (uint32_t)((uint64_t)nseg * (pt + 1) / AL::kParts) - begin;
    };
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint4 cur[kAggUnroll], nxt[kAggUnroll];
    // (the block body appears in both loaders: as a lambda it changed the register
    // allocation, 102 -> 128 VGPRs + scratch)
    // first-set variant: the streams as one virtual sequence (see below)
    // (measured: for C2's main aggregation, ~2.7 K-record 8-byte streams, the
    // per-record search cost more than the idle lanes it saves, 1.28 -> 1.71 ms;
    // for the dictionary sample's few-record streams the whole dictionary step
    // went 0.30 -> 0.21 ms)
    constexpr bool kVirtual = (amode & 256) != 0;
    static_assert(kMid || kAggUnroll % 2 == 0, "8-byte records load in pairs");
    if constexpr (kVirtual) {
        // The wave's streams are wv + kAggWaves * j, j < js, read as ONE virtual
        // sequence of records, so a block spans stream ends instead of idling lanes
        // past them (a C2 bucket's 16-byte map streams hold ~340 records, the
        // dictionary sample's a few).  Lane j holds stream j's record count, start
        // and exclusive prefix; record g of the sequence lies in the last stream j
        // with prefix <= g (binary search over the lanes).  Round 0's 8-byte streams
        // count as even lengths, so records 2i and 2i+1 share one aligned 16-byte
        // load (a map stream starts 16-byte aligned; the padding record reads as
        // zero; 8-byte loads run at ~0.6x the 16-byte rate, MI355X_MICROARCH.md).
        const uint32_t js = nwg > wv ? (nwg - wv + kAggWaves - 1) / kAggWaves : 0u;
        uint32_t vcnt = 0;
        uint64_t vrow = 0;
        if (lane < js) {
            const uint32_t sid = wv + kAggWaves * lane;
            if constexpr (!kRound0) {
                uint32_t b0;
                vcnt = part_range(sid, b0);
                vrow = gbase[sid % kAggSegs] + b0;
            } else {
                vcnt = gcounts[sid];
                vrow = (uint64_t)sid * gstride;
            }
        }
        constexpr bool pairs = !kMid && kRound0;
        const uint32_t vlen = pairs ? (vcnt + 1u) & ~1u : vcnt;
        uint32_t incl = vlen;
    #pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= (uint32_t)o) incl += y;
        }
        const uint32_t ex = incl - vlen;
        const uint32_t T = __builtin_amdgcn_readlane(incl, 63);
        // record g: its element index in pool_b and the records of its stream from g on
        auto locate = [&](uint32_t g, uint64_t& at, uint32_t& left) {
            uint32_t jl = 0;
    #pragma unroll
            for (uint32_t st = 32; st >= 1; st >>= 1) {
                // every lane takes part in the shuffle (a bpermute from a lane that
                // is not active returns nothing), then the condition applies
                const uint32_t c = jl + st;  // <= 63
                const uint32_t e = (uint32_t)__shfl((int)ex, (int)c);
                if (c < js && e <= g) jl = c;
            }
            const uint32_t o = g - (uint32_t)__shfl((int)ex, (int)jl);
            at = (uint64_t)__shfl((unsigned long long)vrow, (int)jl) + o;
            left = (uint32_t)__shfl((int)vcnt, (int)jl) - o;
        };
        auto load = [&](uint32_t g0, uint4* r) {
            if constexpr (pairs) {
    #pragma unroll
                for (uint32_t u = 0; u < kAggUnroll / 2; u++) {
                    const uint32_t g = g0 + 2 * (u * kWave + lane);
                    uint64_t at;
                    uint32_t left;
                    locate(g, at, left);
                    uint4 v = make_uint4(0, 0, 0, 0);
                    if (g < T) v = *(const uint4*)((const uint64_t*)pool_b + at);
                    if (g >= T || left < 2) v.z = v.w = 0;  // the padding record of an odd stream
                    r[2 * u] = make_uint4(v.x, v.y, 0, 0);
                    r[2 * u + 1] = make_uint4(v.z, v.w, 0, 0);
                }
                return;
            }
    #pragma unroll
            for (uint32_t u = 0; u < kAggUnroll; u++) {
                const uint32_t g = g0 + u * kWave + lane;
                uint64_t at;
                uint32_t left;
                locate(g, at, left);
                if (g >= T) {
                    r[u] = make_uint4(0, 0, 0, 0);
                } else if constexpr (kMid) {
                    r[u] = ((const uint4*)pool_b)[at];
                } else {
                    const uint64_t k = ((const uint64_t*)pool_b)[at];
                    r[u] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), 0, 0);
                }
            }
        };
        if (T == 0) return;
        load(0, cur);
        for (uint32_t g0 = 0; g0 < T; g0 += kAggBlock) {
            load(g0 + kAggBlock, nxt);  // the next block in flight while this one is counted
            uint32_t h[kAggUnroll];
#pragma unroll
            for (uint32_t u = 0; u < kAggUnroll; u++) h[u] = fold32(cur[u].x, cur[u].y, cur[u].z, cur[u].w);
            if constexpr ((amode & 128) != 0) {
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) miss += h[u];
            } else if constexpr (!kMid && (amode & 64) != 0) {
                // first-set lookups only, each miss its own slow path (sparse tables)
                uint32_t m[kAggUnroll], z[kAggUnroll], base[kAggUnroll];
                if constexpr (MRG_AGG_PRIO != 0) __builtin_amdgcn_s_setprio(MRG_AGG_PRIO);
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    base[u] = sbase<AL>(h[u]);
                    short_set_masks(A, base[u], ((uint64_t)cur[u].y << 32) | cur[u].x, m[u], z[u]);
                }
                bool slow[kAggUnroll];
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    const bool valid = (cur[u].x | cur[u].y) != 0;  // keys have k0 != 0
                    const bool hit = valid && m[u] != 0;
                    slow[u] = valid && m[u] == 0;
                    const uint32_t ci = hit ? base[u] + __builtin_ctz(m[u]) : (uint32_t)(AL::kShortSets * AL::kShortWays) + lane;
                    if constexpr ((amode & 1024) != 0) miss += ci;  // ablation: no count adds
                    else __hip_atomic_fetch_add(&A.sc[ci], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                if constexpr (MRG_AGG_PRIO != 0) __builtin_amdgcn_s_setprio(0);
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    if (slow[u]) {
                        const uint64_t k = ((uint64_t)cur[u].y << 32) | cur[u].x;
                        if (!short_insert_slow(A, k, h[u], 1)) defer_miss(A, t, k, 0, keep_miss, wv, miss);
                    }
                }
            } else if constexpr (!kMid) {
                // Both sets of a key are looked up before anything diverges: a key
                // sits in its second set only if its first was full when it was
                // claimed (ways are never freed), so a first set with a free way and
                // without the key settles it as new.  Only new keys (and lost claims)
                // take the slow path, all of a lane's in one loop, so a wave runs it
                // about once per block instead of once per record slot.
                // mz[u]: first-set hit ways (bits 0-3), free ways (4-7), second-set hit ways (8-11)
                uint32_t mz[kAggUnroll];
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    uint32_t m, z;
                    short_set_masks(A, sbase<AL>(h[u]), ((uint64_t)cur[u].y << 32) | cur[u].x, m, z);
                    mz[u] = m | z << 4;
                }
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    if ((cur[u].x | cur[u].y) != 0 && mz[u] == 0) {
                        uint32_t m2, z2;
                        short_set_masks(A, sbase<AL>(second_hash(h[u])), ((uint64_t)cur[u].y << 32) | cur[u].x,
                                        m2, z2);
                        mz[u] = m2 << 8 | z2 << 12 | 1u << 16;  // bit 16: second set read
                    }
                }
                uint32_t slow = 0, full = 0;
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    const bool valid = (cur[u].x | cur[u].y) != 0;  // keys have k0 != 0
                    const uint32_t m = mz[u] & 15u, m2 = (mz[u] >> 8) & 15u;
                    // both sets read, full, without the key: final for this round (ways are
                    // never freed), so the key is deferred without the claim path
                    if (valid && (mz[u] >> 8) == (1u << 8)) full |= 1u << u;
                    const uint32_t ci = !valid   ? (uint32_t)(AL::kShortSets * AL::kShortWays) + lane
                                        : m != 0  ? sbase<AL>(h[u]) + __builtin_ctz(m)
                                        : m2 != 0 ? sbase<AL>(second_hash(h[u])) + __builtin_ctz(m2)
                                                  : (uint32_t)(AL::kShortSets * AL::kShortWays) + lane;
                    if (valid && (m | m2) == 0 && !((full >> u) & 1u)) slow |= 1u << u;
                    if constexpr ((amode & 1024) != 0) miss += ci;  // ablation: no count adds
                    else __hip_atomic_fetch_add(&A.sc[ci], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++)
                    if ((full >> u) & 1u) defer_miss(A, t, ((uint64_t)cur[u].y << 32) | cur[u].x, 0, keep_miss, wv, miss);
                if constexpr ((amode & 2048) != 0) slow = 0;  // ablation: no claims
            while (slow) {  // this lane's new keys, one per trip (register arrays read by selects, not indexing)
                    const uint32_t us = __builtin_ctz(slow);
                    slow &= slow - 1;
                    uint64_t k = 0;
                    uint32_t hk = 0;
#pragma unroll
                    for (uint32_t u = 0; u < kAggUnroll; u++)
                        if (us == u) {
                            k = ((uint64_t)cur[u].y << 32) | cur[u].x;
                            hk = h[u];
                        }
                    if (!short_insert_slow(A, k, hk, 1)) defer_miss(A, t, k, 0, keep_miss, wv, miss);
                }
            } else if constexpr ((amode & 64) != 0) {
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    if ((cur[u].x | cur[u].y) != 0) {
                        const uint64_t k0 = ((uint64_t)cur[u].y << 32) | cur[u].x, k1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
                        if (!mid_insert(A, k0, k1, h[u], 1)) defer_miss(A, t, k0, k1, keep_miss, wv, miss);
                    }
                }
            } else {
                // mid keys: the same two-set lookup first (a way pending publication
                // sends the record to the slow path, which retries or defers it)
                uint32_t mm[kAggUnroll], slow = 0, full = 0;  // mm[u]: first-set hit ways (bits 0-3), second-set (4-7)
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    uint32_t m, z, pend;
                    const uint64_t k0 = ((uint64_t)cur[u].y << 32) | cur[u].x, k1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
                    mid_set_masks(A, set_base<AL::kMidSets>(h[u]), k0, k1, m, z, pend);
                    mm[u] = m;
                    if ((cur[u].x | cur[u].y) != 0 && m == 0 && (z | pend) != 0) slow |= 1u << u;  // new key / pending
                }
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    if ((cur[u].x | cur[u].y) != 0 && mm[u] == 0 && !((slow >> u) & 1u)) {
                        uint32_t m2, z2, p2;
                        const uint64_t k0 = ((uint64_t)cur[u].y << 32) | cur[u].x, k1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
                        mid_set_masks(A, set_base<AL::kMidSets>(second_hash(h[u])), k0, k1, m2, z2, p2);
                        mm[u] = m2 << 4;
                        // both sets full without the key (none pending): deferred directly
                        if (m2 == 0 && (z2 | p2) == 0) full |= 1u << u;
                        else if (m2 == 0) slow |= 1u << u;
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    const bool valid = (cur[u].x | cur[u].y) != 0;
                    const uint32_t m = mm[u] & 15u, m2 = mm[u] >> 4;
                    const uint32_t ci = !valid   ? (uint32_t)AL::kMidSets * 4 + lane
                                        : m != 0  ? set_base<AL::kMidSets>(h[u]) + __builtin_ctz(m)
                                        : m2 != 0 ? set_base<AL::kMidSets>(second_hash(h[u])) + __builtin_ctz(m2)
                                                  : (uint32_t)AL::kMidSets * 4 + lane;
                    __hip_atomic_fetch_add(&A.mc[ci], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++)
                    if ((full >> u) & 1u)
                        defer_miss(A, t, ((uint64_t)cur[u].y << 32) | cur[u].x, ((uint64_t)cur[u].w << 32) | cur[u].z,
                                   keep_miss, wv, miss);
                while (slow) {
                    const uint32_t us = __builtin_ctz(slow);
                    slow &= slow - 1;
                    uint64_t k0 = 0, k1 = 0;
                    uint32_t hk = 0;
#pragma unroll
                    for (uint32_t u = 0; u < kAggUnroll; u++)
                        if (us == u) {
                            k0 = ((uint64_t)cur[u].y << 32) | cur[u].x;
                            k1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
                            hk = h[u];
                        }
                    if (!mid_insert(A, k0, k1, hk, 1)) defer_miss(A, t, k0, k1, keep_miss, wv, miss);
                }
            }
    #pragma unroll
            for (uint32_t u = 0; u < kAggUnroll; u++) cur[u] = nxt[u];
        }

    } else {
        // The wave's streams are wv + kAggWaves * j, j < js, walked one after the
        // other; lane j holds stream j's record count, so moving to the next stream
        // is a readlane, not a load.  (The two-set variant keeps this loader: the
        // virtual one's per-record search raises its registers past 128.)
        const uint32_t js = nwg > wv ? (nwg - wv + kAggWaves - 1) / kAggWaves : 0u;
        uint32_t vcnt = 0;
        if (lane < js) {
            uint32_t b0;
            vcnt = !kRound0 ? part_range(wv + kAggWaves * lane, b0) : gcounts[wv + kAggWaves * lane];
        }
        // wave-uniform cursor: stream j, record offset off within it (cnt records)
        uint32_t j = 0, off = 0, cnt = __builtin_amdgcn_readlane(vcnt, 0);
        while (j < js && off >= cnt) {
            j++;
            cnt = j < js ? __builtin_amdgcn_readlane(vcnt, j) : 0u;
        }
        auto load = [&](uint32_t jj, uint32_t o, uint32_t c, uint4* r) {
            const uint32_t sid = wv + kAggWaves * jj;
            uint64_t row = (uint64_t)sid * gstride;
            if constexpr (!kRound0) {
                uint32_t b0 = 0;
                if (jj < js) part_range(sid, b0);
                row = jj < js ? gbase[sid % kAggSegs] + b0 : 0ull;
            }
            if constexpr (!kMid && kRound0) {
                // round 0's 8-byte records: two per 16-byte load (a map stream starts
                // 16-byte aligned and a block at a multiple of kAggBlock records)
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll / 2; u++) {
                    const uint32_t i = o + 2 * (u * kWave + lane);
                    uint4 v = make_uint4(0, 0, 0, 0);
                    if (jj < js && i < c) v = ((const uint4*)((const uint64_t*)pool_b + row + o))[u * kWave + lane];
                    if (i + 1 >= c) v.z = v.w = 0;  // the odd record past the stream's end
                    r[2 * u] = make_uint4(v.x, v.y, 0, 0);
                    r[2 * u + 1] = make_uint4(v.z, v.w, 0, 0);
                }
                return;
            }
#pragma unroll
            for (uint32_t u = 0; u < kAggUnroll; u++) {
                const uint32_t i = o + u * kWave + lane;
                if (jj < js && i < c) {
                    if constexpr (kMid) {
                        r[u] = ((const uint4*)pool_b)[row + i];
                    } else {
                        const uint64_t k = ((const uint64_t*)pool_b)[row + i];
                        r[u] = make_uint4((uint32_t)k, (uint32_t)(k >> 32), 0, 0);
                    }
                } else {
                    r[u] = make_uint4(0, 0, 0, 0);
                }
            }
        };
        load(j, off, cnt, cur);
        while (j < js) {
            // next block's position and loads
            uint32_t j2 = j, off2 = off + kAggBlock, cnt2 = cnt;
            while (j2 < js && off2 >= cnt2) {
                j2++;
                off2 = 0;
                cnt2 = j2 < js ? __builtin_amdgcn_readlane(vcnt, j2) : 0u;
            }
            load(j2, off2, cnt2, nxt);
            uint32_t h[kAggUnroll];
#pragma unroll
            for (uint32_t u = 0; u < kAggUnroll; u++) h[u] = fold32(cur[u].x, cur[u].y, cur[u].z, cur[u].w);
            if constexpr ((amode & 128) != 0) {
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) miss += h[u];
            } else if constexpr (!kMid && (amode & 64) != 0) {
                // first-set lookups only, each miss its own slow path (sparse tables)
                uint32_t m[kAggUnroll], z[kAggUnroll], base[kAggUnroll];
                if constexpr (MRG_AGG_PRIO != 0) __builtin_amdgcn_s_setprio(MRG_AGG_PRIO);
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    base[u] = sbase<AL>(h[u]);
                    short_set_masks(A, base[u], ((uint64_t)cur[u].y << 32) | cur[u].x, m[u], z[u]);
                }
                bool slow[kAggUnroll];
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    const bool valid = (cur[u].x | cur[u].y) != 0;  // keys have k0 != 0
                    const bool hit = valid && m[u] != 0;
                    slow[u] = valid && m[u] == 0;
                    const uint32_t ci = hit ? base[u] + __builtin_ctz(m[u]) : (uint32_t)(AL::kShortSets * AL::kShortWays) + lane;
                    if constexpr ((amode & 1024) != 0) miss += ci;  // ablation: no count adds
                    else __hip_atomic_fetch_add(&A.sc[ci], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                if constexpr (MRG_AGG_PRIO != 0) __builtin_amdgcn_s_setprio(0);
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    if (slow[u]) {
                        const uint64_t k = ((uint64_t)cur[u].y << 32) | cur[u].x;
                        if (!short_insert_slow(A, k, h[u], 1)) defer_miss(A, t, k, 0, keep_miss, wv, miss);
                    }
                }
            } else if constexpr (!kMid) {
                // Both sets of a key are looked up before anything diverges: a key
                // sits in its second set only if its first was full when it was
                // claimed (ways are never freed), so a first set with a free way and
                // without the key settles it as new.  Only new keys (and lost claims)
                // take the slow path, all of a lane's in one loop, so a wave runs it
                // about once per block instead of once per record slot.
                // mz[u]: first-set hit ways (bits 0-3), free ways (4-7), second-set hit ways (8-11)
                uint32_t mz[kAggUnroll];
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    uint32_t m, z;
                    short_set_masks(A, sbase<AL>(h[u]), ((uint64_t)cur[u].y << 32) | cur[u].x, m, z);
                    mz[u] = m | z << 4;
                }
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    if ((cur[u].x | cur[u].y) != 0 && mz[u] == 0) {
                        uint32_t m2, z2;
                        short_set_masks(A, sbase<AL>(second_hash(h[u])), ((uint64_t)cur[u].y << 32) | cur[u].x,
                                        m2, z2);
                        mz[u] = m2 << 8 | z2 << 12 | 1u << 16;  // bit 16: second set read
                    }
                }
                uint32_t slow = 0, full = 0;
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    const bool valid = (cur[u].x | cur[u].y) != 0;  // keys have k0 != 0
                    const uint32_t m = mz[u] & 15u, m2 = (mz[u] >> 8) & 15u;
                    // both sets read, full, without the key: final for this round (ways are
                    // never freed), so the key is deferred without the claim path
                    if (valid && (mz[u] >> 8) == (1u << 8)) full |= 1u << u;
                    const uint32_t ci = !valid   ? (uint32_t)(AL::kShortSets * AL::kShortWays) + lane
                                        : m != 0  ? sbase<AL>(h[u]) + __builtin_ctz(m)
                                        : m2 != 0 ? sbase<AL>(second_hash(h[u])) + __builtin_ctz(m2)
                                                  : (uint32_t)(AL::kShortSets * AL::kShortWays) + lane;
                    if (valid && (m | m2) == 0 && !((full >> u) & 1u)) slow |= 1u << u;
                    if constexpr ((amode & 1024) != 0) miss += ci;  // ablation: no count adds
                    else __hip_atomic_fetch_add(&A.sc[ci], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++)
                    if ((full >> u) & 1u) defer_miss(A, t, ((uint64_t)cur[u].y << 32) | cur[u].x, 0, keep_miss, wv, miss);
                if constexpr ((amode & 2048) != 0) slow = 0;  // ablation: no claims
            while (slow) {  // this lane's new keys, one per trip (register arrays read by selects, not indexing)
                    const uint32_t us = __builtin_ctz(slow);
                    slow &= slow - 1;
                    uint64_t k = 0;
                    uint32_t hk = 0;
#pragma unroll
                    for (uint32_t u = 0; u < kAggUnroll; u++)
                        if (us == u) {
                            k = ((uint64_t)cur[u].y << 32) | cur[u].x;
                            hk = h[u];
                        }
                    if (!short_insert_slow(A, k, hk, 1)) defer_miss(A, t, k, 0, keep_miss, wv, miss);
                }
            } else if constexpr ((amode & 64) != 0) {
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    if ((cur[u].x | cur[u].y) != 0) {
                        const uint64_t k0 = ((uint64_t)cur[u].y << 32) | cur[u].x, k1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
                        if (!mid_insert(A, k0, k1, h[u], 1)) defer_miss(A, t, k0, k1, keep_miss, wv, miss);
                    }
                }
            } else {
                // mid keys: the same two-set lookup first (a way pending publication
                // sends the record to the slow path, which retries or defers it)
                uint32_t mm[kAggUnroll], slow = 0, full = 0;  // mm[u]: first-set hit ways (bits 0-3), second-set (4-7)
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    uint32_t m, z, pend;
                    const uint64_t k0 = ((uint64_t)cur[u].y << 32) | cur[u].x, k1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
                    mid_set_masks(A, set_base<AL::kMidSets>(h[u]), k0, k1, m, z, pend);
                    mm[u] = m;
                    if ((cur[u].x | cur[u].y) != 0 && m == 0 && (z | pend) != 0) slow |= 1u << u;  // new key / pending
                }
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    if ((cur[u].x | cur[u].y) != 0 && mm[u] == 0 && !((slow >> u) & 1u)) {
                        uint32_t m2, z2, p2;
                        const uint64_t k0 = ((uint64_t)cur[u].y << 32) | cur[u].x, k1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
                        mid_set_masks(A, set_base<AL::kMidSets>(second_hash(h[u])), k0, k1, m2, z2, p2);
                        mm[u] = m2 << 4;
                        // both sets full without the key (none pending): deferred directly
                        if (m2 == 0 && (z2 | p2) == 0) full |= 1u << u;
                        else if (m2 == 0) slow |= 1u << u;
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++) {
                    const bool valid = (cur[u].x | cur[u].y) != 0;
                    const uint32_t m = mm[u] & 15u, m2 = mm[u] >> 4;
                    const uint32_t ci = !valid   ? (uint32_t)AL::kMidSets * 4 + lane
                                        : m != 0  ? set_base<AL::kMidSets>(h[u]) + __builtin_ctz(m)
                                        : m2 != 0 ? set_base<AL::kMidSets>(second_hash(h[u])) + __builtin_ctz(m2)
                                                  : (uint32_t)AL::kMidSets * 4 + lane;
                    __hip_atomic_fetch_add(&A.mc[ci], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
#pragma unroll
                for (uint32_t u = 0; u < kAggUnroll; u++)
                    if ((full >> u) & 1u)
                        defer_miss(A, t, ((uint64_t)cur[u].y << 32) | cur[u].x, ((uint64_t)cur[u].w << 32) | cur[u].z,
                                   keep_miss, wv, miss);
                while (slow) {
                    const uint32_t us = __builtin_ctz(slow);
                    slow &= slow - 1;
                    uint64_t k0 = 0, k1 = 0;
                    uint32_t hk = 0;
#pragma unroll
                    for (uint32_t u = 0; u < kAggUnroll; u++)
                        if (us == u) {
                            k0 = ((uint64_t)cur[u].y << 32) | cur[u].x;
                            k1 = ((uint64_t)cur[u].w << 32) | cur[u].z;
                            hk = h[u];
                        }
                    if (!mid_insert(A, k0, k1, hk, 1)) defer_miss(A, t, k0, k1, keep_miss, wv, miss);
                }
            }
#pragma unroll
            for (uint32_t u = 0; u < kAggUnroll; u++) cur[u] = nxt[u];
            j = j2;
            off = off2;
            cnt = cnt2;
        }
    }
}

// amode (compile-time): 0 = two-set lookups, 64 = first-set lookups (both
// exact; launch_wc_agg picks by layout); 256 = the wave's streams read as one
// virtual sequence (the dictionary sample); 128 = benchmark ablation, read +
// hash the records only (wrong results).  emit: see launch_wc_agg.
template <uint32_t amode, class AL>
__global__ void __launch_bounds__(AL::kWaves * 64) wc_agg_kernel(Tables t, int emit) {
    __shared__ AL A;
    constexpr uint32_t kAggWaves = AL::kWaves, kNT = kAggWaves * kWave;
    constexpr uint32_t kAggShortSets = AL::kShortSets, kAggMidSets = AL::kMidSets;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t b = blockIdx.x;
    const uint32_t E = t.sp.nb * kAggSegs;
    const bool later = t.sp.round != 0;
    if (later) {  // a later round: buckets with nothing carried over have nothing to do
        uint32_t tot = 0;
        for (uint32_t i = 0; i < kAggSegs; i++) tot += t.sp.seg_n_in[b * kAggSegs + i] + t.sp.seg_n_in[E + b * kAggSegs + i];
        if (tot == 0) {
            if (tid < kAggSegs) t.sp.seg_n_out[b * kAggSegs + tid] = t.sp.seg_n_out[E + b * kAggSegs + tid] = 0;
            return;
        }
    }
    if (t.dbg && tid == 0) t.dbg[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    for (uint32_t i = tid; i < (uint32_t)(kAggShortSets * AL::kShortWays) + kWave; i += kNT) A.sc[i] = 0;
    for (uint32_t i = tid; i < (uint32_t)(kAggShortSets * AL::kShortWays); i += kNT) A.sk[i] = 0;
    for (uint32_t i = tid; i < (uint32_t)kAggMidSets * 4; i += kNT) {
        A.mk[2 * i] = 0;
        A.mk[2 * i + 1] = kUnwritten;
        A.mc[i] = 0;
    }
    if (tid < kAggSegs) A.ncur8[tid] = A.ncur16[tid] = 0;
    if (tid == 0 && emit == 1) atomicOr(&t.ctr->round_mask, 1ull << (t.sp.round & 63));
    __syncthreads();
    const bool keep_miss = emit != 2;
    uint64_t miss = 0, carried = 0;
    if (!later) {
        // round 0: bucket b's stream of map workgroup g is pool[(g * nb + b) * sub]
        agg_pool<amode, false, 8, true>(A, t, t.sp.pool8 + b * t.sp.sub8, t.sp.counts8 + b * t.sp.nwg,
                                  (uint64_t)t.sp.nb * t.sp.sub8, t.sp.nwg, nullptr, keep_miss, miss);
        agg_pool<amode, true, 4, true>(A, t, t.sp.pool + b * t.sp.sub_keys, t.sp.counts + b * t.sp.nwg,
                                 (uint64_t)t.sp.nb * t.sp.sub_keys, t.sp.nwg, nullptr, keep_miss, miss);
    } else {
        // later rounds: wave w re-reads its own segment of the previous round's misses
        agg_pool<amode, false, 8, false>(A, t, t.sp.seg8_in, t.sp.seg_n_in + b * kAggSegs, 0, kAggWaves,
                                  t.sp.seg_off8 + b * kAggSegs, keep_miss, miss);
        agg_pool<amode, true, 4, false>(A, t, t.sp.seg16_in, t.sp.seg_n_in + E + b * kAggSegs, 0, kAggWaves,
                                 t.sp.seg_off16 + b * kAggSegs, keep_miss, miss);
    }
    __syncthreads();
    // this wave's miss segments (written in the loop above by the kParts waves
    // sharing them; each walks its own interleaved share below)
    const uint32_t sg = wv % kAggSegs, i0 = lane + kWave * (wv / kAggSegs);
    constexpr uint32_t kStep = kWave * AL::kParts;
    const uint64_t seg = b * kAggSegs + sg;
    // (misses past the segment buffers' capacity were dropped and flagged: only
    // the stored ones are read; the flagged run is repeated)
    uint32_t n8 = keep_miss ? A.ncur8[sg] : 0u, n16 = keep_miss ? A.ncur16[sg] : 0u;
    if (keep_miss) {
        const uint64_t o8 = t.sp.seg_off8[seg], o16 = t.sp.seg_off16[seg];
        const uint64_t room8 = o8 < t.sp.seg8_cap ? t.sp.seg8_cap - o8 : 0, room16 = o16 < t.sp.seg16_cap ? t.sp.seg16_cap - o16 : 0;
        if (n8 > room8) n8 = (uint32_t)room8;
        if (n16 > room16) n16 = (uint32_t)room16;
    }
    uint64_t* s8 = keep_miss ? t.sp.seg8_out + t.sp.seg_off8[seg] : nullptr;
    uint4* s16 = keep_miss ? t.sp.seg16_out + t.sp.seg_off16[seg] : nullptr;
    // merge: a key of this bucket went to the HBM table from the map kernel
    // (stream overflow), so the same key may be on both sides: merge the whole
    // bucket (tables and misses) through the HBM table.
    const bool merge = emit == 0 || (emit == 1 && t.bflag[b] != 0);
    if (merge) {
        for (uint32_t i = tid; i < (uint32_t)(kAggShortSets * AL::kShortWays); i += kNT) {
            const uint64_t k0 = A.sk[i];
            if (k0 != 0) short_insert(t, k0, 0, A.sc[i]);
        }
        for (uint32_t i = tid; i < (uint32_t)kAggMidSets * 4; i += kNT) {
            const uint64_t k0 = A.mk[2 * i];
            if (k0 != 0) short_insert(t, k0, A.mk[2 * i + 1], A.mc[i]);
        }
        for (uint32_t i = i0; i < n8; i += kStep) {  // misses, all lanes in flight
            const uint64_t k0 = s8[i];
            if (k0 != 0) short_insert(t, k0, 0, 1);
        }
        for (uint32_t i = i0; i < n16; i += kStep) {
            const uint4 k = s16[i];
            const uint64_t k0 = ((uint64_t)k.y << 32) | k.x;
            if (k0 != 0) short_insert(t, k0, ((uint64_t)k.w << 32) | k.z, 1);
        }
        if (t.sp.seg_n_out && i0 == 0) t.sp.seg_n_out[seg] = t.sp.seg_n_out[E + seg] = 0;
        if (tid == 0) atomicAdd(&t.ctr->bflush, 1ull);
    } else {
        // Settle the misses against the (now stable) tables: a key that is there
        // is counted there and its record cleared; the others are carried to the
        // next round (or, in the last round, counted in the HBM table).  So the
        // keys of every round's tables and of the HBM table are disjoint, and the
        // tables are emitted as they are.
        if (emit == 1) {
            // A bucket with fewer misses than carry_min (option; 0 = never)
            // settles them in the HBM table now instead of carrying them.
            uint32_t left = 0;
            for (uint32_t w = 0; w < kAggSegs; w++) left += A.ncur8[w] + A.ncur16[w];
            const bool last = t.sp.last != 0 || left < t.sp.carry_min;
            for (uint32_t i = i0; i < n8; i += kStep) {
                const uint64_t k0 = s8[i];
                if (k0 == 0) continue;
                const int slot = short_find_exact(A, k0, fold32((uint32_t)k0, (uint32_t)(k0 >> 32), 0, 0));
                if (slot >= 0 || last) {
                    if (slot >= 0) atomicAdd(&A.sc[slot], 1u);
                    else short_insert(t, k0, 0, 1);
                    s8[i] = 0;
                } else {
                    carried++;
                }
            }
            for (uint32_t i = i0; i < n16; i += kStep) {
                const uint4 k = s16[i];
                const uint64_t k0 = ((uint64_t)k.y << 32) | k.x, k1 = ((uint64_t)k.w << 32) | k.z;
                if (k0 == 0) continue;
                const int slot = mid_find_exact(A, k0, k1, fold32(k.x, k.y, k.z, k.w));
                if (slot >= 0 || last) {
                    if (slot >= 0) atomicAdd(&A.mc[slot], 1u);
                    else short_insert(t, k0, k1, 1);
                    s16[i] = make_uint4(0, 0, 0, 0);
                } else {
                    carried++;
                }
            }
            if (t.sp.seg_n_out && i0 == 0) {
                t.sp.seg_n_out[seg] = last ? 0u : n8;
                t.sp.seg_n_out[E + seg] = last ? 0u : n16;
            }
        }
        __syncthreads();
        // one cursor allocation per workgroup, then each thread writes its keys
        uint32_t mine = 0;
        for (uint32_t i = tid; i < (uint32_t)(kAggShortSets * AL::kShortWays); i += kNT) mine += A.sk[i] != 0;
        for (uint32_t i = tid; i < (uint32_t)kAggMidSets * 4; i += kNT) mine += A.mk[2 * i] != 0;
        unsigned long long o = block_alloc<kAggWaves>(&t.ctr->nrec, mine, A.red);
        for (uint32_t i = tid; i < (uint32_t)(kAggShortSets * AL::kShortWays); i += kNT) {
            const uint64_t k0 = A.sk[i];
            if (k0 != 0) put_short(t, o++, k0, 0, A.sc[i], emit == 1);
        }
        for (uint32_t i = tid; i < (uint32_t)kAggMidSets * 4; i += kNT) {
            const uint64_t k0 = A.mk[2 * i];
            if (k0 != 0) put_short(t, o++, k0, A.mk[2 * i + 1], A.mc[i], emit == 1);
        }
    }
    if ((amode & (128 | 1024)) != 0 && miss == 0x5eed5eedull) atomicAdd(&t.ctr->lds_miss, 1ull);  // no DCE in ablation builds
    block_add4<kAggWaves>(&t.ctr->agg_miss, &t.ctr->carried, nullptr, nullptr, (amode & 128) == 0 ? miss : 0, carried, 0, 0,
                          A.red);
    if (t.dbg && tid == 0) t.dbg[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
}

// Multi-round layout, step 1: records of bucket b's streams per aggregator wave
// (wave w reads streams w, w + kAggWaves, ...), clamped like the aggregator's reads.
__global__ void __launch_bounds__(kMaxMapWGs) seg_count_kernel(Spill sp, uint32_t* tmp) {
    __shared__ uint32_t sum[2 * kAggSegs];
    const uint32_t b = blockIdx.x, g = threadIdx.x;
    if (g < 2 * kAggSegs) sum[g] = 0;
    __syncthreads();
    if (g < sp.nwg) {
        atomicAdd(&sum[g % kAggSegs], sp.counts8[(uint64_t)b * sp.nwg + g]);
        atomicAdd(&sum[kAggSegs + g % kAggSegs], sp.counts[(uint64_t)b * sp.nwg + g]);
    }
    __syncthreads();
    const uint32_t E = sp.nb * kAggSegs;
    if (g < kAggSegs) {
        tmp[b * kAggSegs + g] = sum[g];
        tmp[E + b * kAggSegs + g] = sum[kAggSegs + g];
    }
}

// Step 2: exclusive scans (one workgroup; E / 1024 entries per thread), totals at [E].
__global__ void __launch_bounds__(1024) seg_scan_kernel(const uint32_t* tmp, uint64_t* off8, uint64_t* off16,
                                                        uint32_t E) {
    const uint32_t PER = E / 1024;  // E = nb * kAggSegs, a multiple of 1024
    __shared__ unsigned long long part[2][1024];
    const uint32_t tid = threadIdx.x;
    uint64_t a = 0, c = 0;
    for (uint32_t q = 0; q < PER; q++) {
        a += tmp[tid * PER + q];
        c += tmp[E + tid * PER + q];
    }
    part[0][tid] = a;
    part[1][tid] = c;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan of the thread totals
        const unsigned long long x = tid >= d ? part[0][tid - d] : 0ull, y = tid >= d ? part[1][tid - d] : 0ull;
        __syncthreads();
        part[0][tid] += x;
        part[1][tid] += y;
        __syncthreads();
    }
    uint64_t o8 = part[0][tid] - a, o16 = part[1][tid] - c;
    for (uint32_t q = 0; q < PER; q++) {
        off8[tid * PER + q] = o8;
        off16[tid * PER + q] = o16;
        o8 += tmp[tid * PER + q];
        o16 += tmp[E + tid * PER + q];
    }
    if (tid == 1023) {
        off8[E] = o8;
        off16[E] = o16;
    }
}

// ------------------------------------------------------------ dictionary
// Records of the dictionary keys: per slot, the sum over map workgroups.  A
// block owns 64 slots; its 16 waves each sum every 16th workgroup's row
// (coalesced 256 B per wave), then the partial sums meet in LDS.
constexpr int kEmitSlots = 64;
template <class G>
__global__ void __launch_bounds__(1024) dict_emit_kernel(Tables t, uint32_t nwg) {
    __shared__ unsigned long long part[16][kEmitSlots];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * kEmitSlots + lane;
    unsigned long long sum = 0;
    if (i < (uint32_t)G::kSlots)
        for (uint32_t g = wv; g < nwg; g += 16) sum += t.dict_cnt[(uint64_t)g * G::kSlots + i];
    part[wv][lane] = sum;
    __syncthreads();
    if (wv != 0) return;
    sum = 0;
    for (int w = 0; w < 16; w++) sum += part[w][lane];
    uint64_t k0 = 0, k1 = 0;
    if (i < (uint32_t)G::kSlots) {
        const uint32_t set = i >> 1, way = i & 1;
        const uint4 sv = t.dict[set];
        if (set >= (uint32_t)G::kShort) {
            k0 = way ? 0 : ((uint64_t)sv.y << 32) | sv.x;
            k1 = ((uint64_t)sv.w << 32) | sv.z;
        } else {
            k0 = way ? (((uint64_t)sv.w << 32) | sv.z) : (((uint64_t)sv.y << 32) | sv.x);
        }
    }
    const bool valid = k0 != 0 && sum != 0;
    const unsigned long long o = wave_alloc(&t.ctr->nrec, valid);  // one wave per block
    if (valid) put_short(t, o, k0, k1, sum, true);
}

// Copy sample windows: window w = in[w*stride, w*stride + win) -> dst[w*(win+16)],
// followed by 16 '\n' bytes (a separator, so no word spans two windows).
__global__ void sample_gather_kernel(const uint8_t* __restrict__ in, uint64_t win, uint64_t stride, uint32_t nwin,
                                     uint8_t* __restrict__ dst) {
    const uint64_t per = win / 16 + 1;  // uint4 units per window incl. the separator
    const uint64_t total = per * nwin;
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gs) {
        const uint64_t w = i / per, k = i - w * per;
        uint4 v;
        if (k + 1 == per) v = make_uint4(0x0A0A0A0Au, 0x0A0A0A0Au, 0x0A0A0A0Au, 0x0A0A0A0Au);
        else v = reinterpret_cast<const uint4*>(in + w * stride)[k];
        reinterpret_cast<uint4*>(dst)[i] = v;
    }
}

__global__ void dict_keys_kernel(Recs r, uint32_t* keys, uint32_t* idx) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.n; i += gs) {
        const uint64_t c = r.cnt[i];
        // 16-bit key, ascending = descending count (counts >= 65535 tie: the few
        // hottest keys, placed first in any order); a 16-bit sort is 2 passes
        keys[i] = 0xFFFFu - (uint32_t)(c > 0xFFFFull ? 0xFFFFull : c);
        idx[i] = (uint32_t)i;
    }
}

// Candidates in descending-count order, gathered densely (the placement below is
// one workgroup; here every gather is in flight at once): {k0, k1}, or zeros for
// keys the dictionary cannot hold (long keys).
constexpr uint64_t kDictCands = 4ull * kDictSlots;
__global__ void dict_cands_kernel(Recs r, const uint32_t* order, uint64_t lim, uint4* cand) {
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += gs) {
        const uint32_t j = order[i];
        const uint64_t k0 = r.k0[j], k1 = r.k1[j];
        cand[i] = r.koff[j] == ~0ull ? make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32))
                                     : make_uint4(0, 0, 0, 0);
    }
}

// One workgroup places the candidates in order, 1024 at a time, each into the
// first of its two sets with a free way; a key whose two sets are full stays out
// (it is then counted through the spill path).  Within a batch the 1024
// placements race, so which keys lose out varied from run to run; when one of the
// few thousand hottest lost (~3e5 words of C2), its bucket's aggregator workgroup
// ended last and the whole aggregation took ~1.25 instead of ~1.02 ms in that
// process (the kept dictionary made it last for the process).  So the kDictHot
// hottest candidates get a fix-up pass in rank order: one that lost takes the
// way of the coldest key in its two sets when that key is colder.
constexpr uint32_t kDictHot = 4096;
template <class G>
__global__ void __launch_bounds__(1024) dict_build_kernel(const uint4* cand, uint64_t lim, uint4* dict) {
    __shared__ uint4 S[G::kSets];
    __shared__ uint32_t fill[G::kSets];
    __shared__ uint32_t rk[G::kSets][2];    // candidate index (rank) of the key in each way, ~0u = empty
    __shared__ uint32_t hot[kDictHot / 32];  // placed bits of the kDictHot hottest candidates
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < (uint32_t)G::kSets; i += 1024) {
        S[i] = make_uint4(0, 0, 0, 0);
        fill[i] = 0;
        rk[i][0] = rk[i][1] = ~0u;
    }
    if (tid < kDictHot / 32) hot[tid] = 0;
    __syncthreads();
    uint4 nx = tid < lim ? cand[tid] : make_uint4(0, 0, 0, 0);
    for (uint64_t base = 0; base < lim; base += 1024) {
        const uint4 c = nx;
        const uint64_t i2 = base + 1024 + tid;  // next round's candidate, in flight during this one
        nx = i2 < lim ? cand[i2] : make_uint4(0, 0, 0, 0);
        const uint64_t k0 = ((uint64_t)c.y << 32) | c.x, k1 = ((uint64_t)c.w << 32) | c.z;
        if (k0 != 0) {
            const bool mid = k1 != 0;
            uint32_t s1, s2;
            dict_sets<G>(fold32(c.x, c.y, c.z, c.w), mid, s1, s2);
            const uint32_t ways = mid ? 1u : 2u;
            uint32_t s = s1, w = atomicAdd(&fill[s1], 1u);
            if (w >= ways) { s = s2; w = atomicAdd(&fill[s2], 1u); }
            if (w < ways) {
                if (mid) S[s] = c;
                else if (w == 0) { S[s].x = c.x; S[s].y = c.y; }
                else { S[s].z = c.x; S[s].w = c.y; }
                const uint32_t i = (uint32_t)(base + tid);
                rk[s][w] = i;
                if (i < kDictHot) atomicOr(&hot[i >> 5], 1u << (i & 31));
            }
        }
        __syncthreads();
    }
    // Fix-up, wave 0, lowest rank first (an evicted key is colder than its evictor,
    // so it is met again later in this pass if it is one of the kDictHot).
    // Only as many candidates as the dictionary holds keys: past that, nearly
    // every candidate has lost and takes a serial turn for nothing (the 1088-key
    // mini dictionary spent ~0.9 ms on ~3000 such turns: 962 us per build in
    // round 4's C5 profile, against ~105 us for the full one).
    constexpr uint32_t kFixMax = kDictHot < 2u * G::kShort + G::kMid ? kDictHot : 2u * G::kShort + G::kMid;
    if (tid < kWave) {
        const uint32_t nh = (uint32_t)(lim < kFixMax ? lim : kFixMax);
        for (uint32_t g = 0; g < nh; g += kWave) {
            const uint32_t i = g + tid;
            const uint4 c = i < nh ? cand[i] : make_uint4(0, 0, 0, 0);
            bool tried = false;  // this lane's candidate already had its fix-up
            for (;;) {
                const bool want = i < nh && (c.x | c.y) != 0 && !tried && !((hot[i >> 5] >> (i & 31)) & 1u);
                const uint64_t m = __ballot(want);
                if (m == 0) break;
                if (tid == (uint32_t)__builtin_ctzll(m)) {
                    tried = true;
                    const bool mid = (c.z | c.w) != 0;
                    uint32_t s1, s2;
                    dict_sets<G>(fold32(c.x, c.y, c.z, c.w), mid, s1, s2);
                    const uint32_t ways = mid ? 1u : 2u;
                    uint32_t bs = s1, bw = 0, br = rk[s1][0];  // the coldest way of the two sets
                    for (uint32_t k = 0; k < 2 * ways; k++) {
                        const uint32_t ss = k < ways ? s1 : s2, ww = k < ways ? k : k - ways;
                        const uint32_t r = rk[ss][ww];
                        if (r > br || (r == br && k == 0)) { bs = ss; bw = ww; br = r; }
                    }
                    if (br > i) {  // colder (or empty): this candidate takes the way
                        if (br < kDictHot) atomicAnd(&hot[br >> 5], ~(1u << (br & 31)));
                        if (mid) S[bs] = c;
                        else if (bw == 0) { S[bs].x = c.x; S[bs].y = c.y; }
                        else { S[bs].z = c.x; S[bs].w = c.y; }
                        rk[bs][bw] = i;
                        atomicOr(&hot[i >> 5], 1u << (i & 31));
                    }
                }
                // the next ballot reads what this lane wrote
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < (uint32_t)G::kSets; i += 1024) dict[i] = S[i];
}

// ------------------------------------------------------------ launchers
uint32_t wc_map_grid(uint64_t n, int grid) {
    const uint64_t nchunks = (n + kOwn - 1) / kOwn;
    uint64_t g = (nchunks + kWavesPerWG - 1) / kWavesPerWG;
    if (g > (uint64_t)grid) g = (uint64_t)grid;
    if (g > (uint64_t)kMaxMapWGs) g = kMaxMapWGs;
    return (uint32_t)(g ? g : 1);
}

bool launch_wc_map(const uint8_t* in, uint64_t n, const Tables& t, LetterTables lt, int grid, int mode, hipStream_t s,
                   uint64_t cbeg, uint64_t cend, bool resume) {
    const uint64_t nch = (n + kOwn - 1) / kOwn;
    if (nch == 0) return true;
    if (nch + (uint64_t)kMaxMapWGs * kWavesPerWG * 3 >= (1ull << 32)) return false;  // 32-bit chunk indices
    if (cend > nch) cend = nch;
    if (cbeg >= cend) return true;
    const uint32_t cb = (uint32_t)cbeg, ce = (uint32_t)cend;
    const int rs = resume ? 1 : 0;
    // first chunk whose window [cs - 16, cs + 1012) reaches the dword holding the
    // split's last n % 4 bytes (the range check zero-fills that partial dword)
    const uint64_t n4 = n & ~3ull, reach = kSlotBytes + kSlotTail - kBack;
    const uint32_t ctail = (n & 3) == 0 ? 0xFFFFFFFFu : n4 < reach ? 0u : (uint32_t)((n4 - reach) / kOwn + 1);
    const uint64_t g = wc_map_grid(n, grid);
#ifdef MRG_ISA_MAIN_ONLY  // (ISA inspection builds: the default map kernel only)
    wc_map_kernel<0, kWavesPerWG, kSpillBucketsLo><<<(unsigned)g, kThreads, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt);
    return true;
#endif
    if (t.sp.nb == kSpillBucketsHi) {  // high-cardinality layout (ablation modes apply to the default one only)
        if (t.hi_staged) {  // the mini dictionary: its LDS write-combines the 8-byte spill streams
            switch (mode) {  // ablation modes of the staged kernel (mapprobe --opt spill_buckets=2048)
#ifndef MRG_NO_STAGED_MODES
#define MRG_MAP_MODE(M)                                                                                           \
    case M:                                                                                                       \
        wc_map_kernel<M, kWavesPerWG, kSpillBucketsHi, true><<<(unsigned)g, kThreads, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt); \
        break;
                // 0x10000: the write-combining round without its stores; 0x20000:
                // no round (no barriers; the 8-byte records stored one by one)
                MRG_MAP_MODE(2) MRG_MAP_MODE(16) MRG_MAP_MODE(32) MRG_MAP_MODE(32 | 0x10000) MRG_MAP_MODE(32 | 0x20000)
                MRG_MAP_MODE(0x10000) MRG_MAP_MODE(0x20000)
#undef MRG_MAP_MODE
#endif
                default: wc_map_kernel<0, kWavesPerWG, kSpillBucketsHi, true><<<(unsigned)g, kThreads, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt);
            }
        } else
            wc_map_kernel<0, 12, kSpillBucketsHi><<<(unsigned)g, 12 * kWave, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt);
        return true;
    }
    if (t.sp.nb == kSpillBucketsLo) {  // the default layout (ablation modes: mapprobe.py)
        if (t.lean && mode == 0) {  // splits after an all-ASCII one: fewer scalars spilled in the loop
            wc_map_kernel<0, kWavesPerWG, kSpillBucketsLo, false, true><<<(unsigned)g, kThreads, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt);
            return true;
        }
        switch (mode) {
#define MRG_MAP_MODE(M) \
    case M: wc_map_kernel<M, kWavesPerWG, kSpillBucketsLo><<<(unsigned)g, kThreads, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt); break;
            MRG_MAP_MODE(1) MRG_MAP_MODE(2) MRG_MAP_MODE(4) MRG_MAP_MODE(8) MRG_MAP_MODE(16) MRG_MAP_MODE(32)
            MRG_MAP_MODE(64) MRG_MAP_MODE(64 | 2) MRG_MAP_MODE(0x100)
#undef MRG_MAP_MODE
            default: wc_map_kernel<0, kWavesPerWG, kSpillBucketsLo><<<(unsigned)g, kThreads, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt);
        }
        return true;
    }
    switch (mode) {
#define MRG_MAP_MODE(M) \
    case M: wc_map_kernel<M><<<(unsigned)g, kThreads, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt); break;
        MRG_MAP_MODE(1) MRG_MAP_MODE(2) MRG_MAP_MODE(4) MRG_MAP_MODE(8) MRG_MAP_MODE(16) MRG_MAP_MODE(32)
        MRG_MAP_MODE(0x100) MRG_MAP_MODE(0x4000) MRG_MAP_MODE(0x8000)
#undef MRG_MAP_MODE
        // occupancy benchmark: 8 or 12 waves per workgroup (results stay exact)
        case 0x1000: wc_map_kernel<0, 8><<<(unsigned)g, 8 * kWave, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt); break;
        case 0x2000: wc_map_kernel<0, 12><<<(unsigned)g, 12 * kWave, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt); break;
        default: wc_map_kernel<0><<<(unsigned)g, kThreads, 0, s>>>(in, n, cb, ce, ctail, rs, t, lt); break;
    }
    return true;
}

void launch_wc_agg(const Tables& t, int mode, int emit, bool big, hipStream_t s) {
    // mode 512 (diagnostic only, wrong results): a read-only pass first, so the
    // timed pass runs with warm caches and address translations
    const uint32_t nb = t.sp.nb;
    if (mode & 512) wc_agg_kernel<128, AggLds><<<nb, AggLds::kWaves * kWave, 0, s>>>(t, emit);
    // Lookup strategy (both exact): first-set lookups, or with mode 64 (A/B) the
    // two-set variant.  The two-set lookup paid off for C5 only while its 2048
    // buckets shared a hash bit with the table's set index (13.4 vs 16.7 ms);
    // with disjoint bits the first-set path is faster there too (11.6 vs 12.5
    // ms) and on C2 (1.29 vs 1.50 ms).
    const bool two_set = (mode & 64) != 0;
    if (big) {
        if (mode & 128) wc_agg_kernel<128, AggLdsBig><<<nb, AggLdsBig::kWaves * kWave, 0, s>>>(t, emit);
        else if (mode & 1024) wc_agg_kernel<1024, AggLdsBig><<<nb, AggLdsBig::kWaves * kWave, 0, s>>>(t, emit);
        else if (mode & 2048) wc_agg_kernel<2048, AggLdsBig><<<nb, AggLdsBig::kWaves * kWave, 0, s>>>(t, emit);
        else if (two_set) wc_agg_kernel<0, AggLdsBig><<<nb, AggLdsBig::kWaves * kWave, 0, s>>>(t, emit);
        else wc_agg_kernel<64, AggLdsBig><<<nb, AggLdsBig::kWaves * kWave, 0, s>>>(t, emit);
    } else {
        if (mode & 128) wc_agg_kernel<128, AggLds><<<nb, AggLds::kWaves * kWave, 0, s>>>(t, emit);
        else if (emit == 2) wc_agg_kernel<64 | 256, AggLds><<<nb, AggLds::kWaves * kWave, 0, s>>>(t, emit);
        else if (two_set) wc_agg_kernel<0, AggLds><<<nb, AggLds::kWaves * kWave, 0, s>>>(t, emit);
        else wc_agg_kernel<64, AggLds><<<nb, AggLds::kWaves * kWave, 0, s>>>(t, emit);
    }
}

void launch_seg_layout(const Tables& t, uint32_t* tmp, uint64_t* off8, uint64_t* off16, hipStream_t s) {
    static_assert(kSpillBuckets * kAggSegs % 1024 == 0 && kSpillBucketsHi * kAggSegs % 1024 == 0, "scan layout");
    seg_count_kernel<<<t.sp.nb, kMaxMapWGs, 0, s>>>(t.sp, tmp);
    seg_scan_kernel<<<1, 1024, 0, s>>>(tmp, off8, off16, t.sp.nb * kAggSegs);
}

void launch_dict_emit(const Tables& t, uint32_t nwg, hipStream_t s) {
    if (t.hi_staged) dict_emit_kernel<DictMini><<<(DictMini::kSlots + kEmitSlots - 1) / kEmitSlots, 1024, 0, s>>>(t, nwg);
    else dict_emit_kernel<DictFull><<<(DictFull::kSlots + kEmitSlots - 1) / kEmitSlots, 1024, 0, s>>>(t, nwg);
}

void launch_sample_gather(const uint8_t* in, uint64_t /*n*/, uint64_t win, uint64_t stride, uint32_t nwin, uint8_t* dst,
                          hipStream_t s) {
    sample_gather_kernel<<<1024, 256, 0, s>>>(in, win, stride, nwin, dst);
}

void launch_dict_keys(const Recs& r, uint32_t* keys, uint32_t* idx, hipStream_t s) {
    if (r.n) dict_keys_kernel<<<512, 256, 0, s>>>(r, keys, idx);
}

// cand: scratch for kDictCands uint4
void launch_dict_build(const Recs& r, const uint32_t* order, uint64_t n, uint4* cand, uint4* dict, bool mini, hipStream_t s) {
    const uint64_t lim = n < kDictCands ? n : kDictCands;
    if (lim) dict_cands_kernel<<<(unsigned)((lim + 255) / 256), 256, 0, s>>>(r, order, lim, cand);
    if (mini) dict_build_kernel<DictMini><<<1, 1024, 0, s>>>(cand, lim, dict);
    else dict_build_kernel<DictFull><<<1, 1024, 0, s>>>(cand, lim, dict);
}

}  // namespace mrg
