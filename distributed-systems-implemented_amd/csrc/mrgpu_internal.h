// mrgpu_internal.h — device data layout and internal launch interfaces.
//
// HBM layout (one context = one GPU):
//   input      raw split bytes (caller's device buffer, or the context's staging copy)
//   ShortTable open-addressing table of distinct keys <= 16 bytes, 32 B slots
//              {k0, k1, count, 0}: k0/k1 = key bytes 0-7 / 8-15 little-endian,
//              zero padded (letters are never 0x00, so padding is unambiguous).
//              Empty slot: k0 == 0; claimed but not yet published: k1 == kUnwritten
//              (0xFF bytes never occur in UTF-8, so no key has that k1).
//   LongTable  distinct keys > 16 bytes (wc) and every grep line: 32 B slots
//              {hash64|1, rep pointer, count, len}; bytes compared against rep.
//   Recs       compacted distinct keys: SoA k0,k1,len,cnt,part,koff + byte arena
//              for long keys (the "parts" handed between map, exchange, reduce).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace mrg {

constexpr uint64_t kUnwritten = ~0ull;
constexpr uint64_t kListHole = ~0ull;  // an unused entry of the long-word list
constexpr int kWave = 64;

// status word bits (device -> host)
enum : uint32_t {
    kStShortFull = 1u << 0,
    kStLongFull = 1u << 1,
    kStListFull = 1u << 2,
    kStSpin = 1u << 3,
    kStRecFull = 1u << 4,   // the record output buffer was too small
    kStSegFull = 1u << 5,   // an aggregation miss segment buffer was too small (sized without a host read)
    kStLrecFull = 1u << 6,  // a map workgroup's region of 32-byte long-word records was too small
};

struct ShortSlot {
    uint64_t k0, k1, count, pad;
};
struct LongSlot {
    uint64_t hash;        // fnv1a64 | 1; 0 = empty
    const uint8_t* rep;   // representative bytes; nullptr = not yet published
    uint64_t count;
    uint64_t len;
};

struct Counters {
    uint32_t status;
    uint32_t pad0;
    unsigned long long nlist;      // long-word starts / grep matches appended
    unsigned long long short_used; // distinct keys claimed in ShortTable
    unsigned long long long_used;  // distinct keys claimed in LongTable
    unsigned long long lds_miss;   // occurrences that went to HBM tables
    unsigned long long nrec;       // collect: records written
    unsigned long long arena;      // collect: arena bytes used
    unsigned long long nlong_rec;  // collect: long records
    unsigned long long chunks_utf8;// chunks that took the UTF-8 decode path
    unsigned long long long_bytes; // total bytes of distinct long keys (arena size)
    unsigned long long spilled;    // keys written to the spill pool
    unsigned long long spill_ovf;  // keys that found their bucket region full (went to the HBM table)
    unsigned long long agg_miss;   // spill keys that missed the bucket aggregator's LDS table
    unsigned long long bflush;     // spill buckets merged through the HBM table (overflow somewhere)
    unsigned long long dict_hits;  // occurrences counted by the hot-key dictionary
    unsigned long long carried;    // aggregator misses carried to the next round
    unsigned long long round_mask; // bit r: aggregation round r had input
    unsigned long long nlines;     // grep: matching line occurrences resolved (one per line, not per hit)
    unsigned long long ndefer;     // grep: hits whose line bounds lie beyond a lane's scan window
    unsigned long long nrec_base;  // ctr->nrec before the collect (a collect-only retry restores it)
    unsigned long long spilled16;  // of `spilled`: 16-byte records (keys of 9-16 bytes)
    unsigned long long line_bytes; // grep: bytes of the resolved line occurrences (the records' arena bound)
};

// Spill of dictionary misses, hash-partitioned into nb buckets (kSpillBuckets,
// or kSpillBucketsHi for high-cardinality splits whose distinct keys would not
// fit a bucket's LDS table in one aggregation round).
// Every (map workgroup g, bucket b) pair owns a fixed stream of `sub_keys`
// 16-B keys {k0,k1} at pool[(g*nb + b)*sub_keys] (a workgroup's
// streams are contiguous: its scattered appends touch few TLB pages); the
// workgroup appends with an LDS cursor (no HBM atomics, no barriers) and
// records the stream length in counts[b*nwg + g].  Keys beyond sub_keys go to
// the HBM table instead.
constexpr int kSpillBuckets = 512;
constexpr int kSpillBucketsHi = 2048;
constexpr int kSpillBucketsLo = 256;  // the default layout: fewer, longer streams; 1024-thread aggregator tables
constexpr int kMaxMapWGs = 512;   // map workgroups (spill streams per bucket) at most
constexpr int kAggSegs = 8;       // aggregator waves per bucket = miss segments per bucket
// Keys of at most 8 bytes (k1 == 0) are spilled as 8-byte records into pool8,
// longer ones as 16-byte records into pool: the combiner's misses are mostly
// tail words, and most words are short, so this roughly halves spill traffic.
struct Spill {
    uint4* pool;                     // [nwg][nb][sub_keys] 16-byte records (k0, k1)
    uint64_t* pool8;                 // [nwg][nb][sub8] 8-byte records (k0; k1 == 0)
    uint64_t sub_keys, sub8;         // stream capacities (records)
    uint32_t* counts;                // [nb * nwg] records in each 16-byte stream
    uint32_t* counts8;               // [nb * nwg] records in each 8-byte stream
    uint32_t nwg;
    uint32_t nb;                     // buckets: kSpillBuckets or kSpillBucketsHi
    // Multi-round bucket aggregation (high-cardinality buckets): the keys a round
    // could not hold in LDS are the next round's input.  Misses are appended to
    // per-(bucket, aggregator wave) segments; a segment's capacity is the records
    // that wave read in round 0 (a wave only ever re-reads its own segment), so the
    // offsets seg_off* are fixed over the rounds and the buffers ping-pong.
    const uint64_t* seg_off8;        // [nb * kAggSegs + 1] 8-byte segment offsets (records)
    const uint64_t* seg_off16;       // [nb * kAggSegs + 1] 16-byte segment offsets
    const uint32_t* seg_n_in;        // [2][nb * kAggSegs] records in each input segment (8-B, 16-B)
    uint32_t* seg_n_out;             // same layout: records appended this round
    const uint64_t* seg8_in;
    uint64_t* seg8_out;
    const uint4* seg16_in;
    uint4* seg16_out;
    uint64_t seg8_cap, seg16_cap;    // records the seg*_out buffers hold (a miss past them sets kStSegFull)
    uint32_t round;                  // 0: the input is the map's spill streams; > 0: seg*_in
    uint32_t last;                   // nonzero: unsettled misses go to the HBM table (final round)
    uint32_t carry_min;              // a bucket with fewer misses than this settles them in the HBM table
};

// Hot-key dictionary (wc): a static table of the most frequent keys of a
// sample of the split, built once per map and copied into every map
// workgroup's LDS.  Keys of 1-8 bytes live in 2-way sets of 8-byte keys, keys of
// 9-16 bytes in 1-way sets of 16-byte keys; a key may sit in either of two sets
// (two-choice), so a lookup is two aligned 16-byte LDS reads.  Count slot of
// (set s, way w) = 2*s + w.  Zero = empty (letters are never 0x00).
constexpr int kDictShortSets = 4096;
constexpr int kDictMidSets = 256;
constexpr int kDictSets = kDictShortSets + kDictMidSets;
constexpr int kDictSlots = 2 * kDictSets;
// Dictionary geometry: DictFull above; DictMini (1024 short + 64 mid keys) for
// the write-combined 2048-bucket map, whose LDS holds the spill groups instead.
// The mini table takes the hottest keys only: enough to lift the few hot words
// of a high-cardinality split off their buckets' streams.
template <int SS, int MS>
struct DictGeo {
    static constexpr int kShort = SS, kMid = MS, kSets = SS + MS, kSlots = 2 * (SS + MS);
    static_assert((SS & (SS - 1)) == 0 && (MS & (MS - 1)) == 0 && SS <= 4096 && MS <= 4096, "set index = hash bits");
};
using DictFull = DictGeo<kDictShortSets, kDictMidSets>;
using DictMini = DictGeo<512, 64>;

struct Recs {
    uint64_t* k0;
    uint64_t* k1;
    uint32_t* len;
    uint64_t* cnt;
    uint32_t* part;
    uint64_t* koff;      // arena offset (len > 16), else ~0
    uint8_t* arena;
    uint64_t n;
    uint64_t arena_n;
};

struct Tables {
    ShortSlot* sh;
    uint64_t sh_mask;
    uint32_t* sh_list;   // [sh_mask + 1] indices of the claimed ShortTable slots, in claim order (ctr->short_used)
    LongSlot* lo;
    uint64_t lo_mask;
    uint64_t* list;      // u64 offsets (long-word starts / grep match positions)
    uint64_t list_cap;
    // grep line resolution: hits sorted by position; resolved lines as (start,
    // end) pairs; hits handed to the workgroup-wide scan (indices into hits)
    const uint64_t* hits;
    uint64_t* lines;
    uint64_t* defer;
    Counters* ctr;
    Spill sp;
    // wc record output: dict_emit / wc_agg (direct) / collect append at ctr->nrec
    Recs out;
    uint64_t out_cap;
    uint32_t nreduce;
    uint32_t* bflag;        // [nb] nonzero: a key of the bucket went to the HBM table
    const uint4* dict;      // dictionary image [kDictSets] (nullptr: no dictionary)
    uint32_t* dict_cnt;     // [nwg][kDictSlots] per-map-workgroup dictionary counts
    unsigned long long* dbg;  // diagnostics (MRG_DEBUG_TIMES): per-workgroup s_memrealtime stamps, or nullptr
    // wc words of 17-32 bytes that end inside their map window: the key bytes as
    // 32-byte zero-padded records (two uint4), one region of lrec_cap records per
    // map wave ([workgroup][kWavesPerWG]); lrec_cnt[r] = records region r holds
    // (past lrec_cap: kStLrecFull).
    // nullptr: every long word goes to the start-offset list (wc_long_kernel).
    uint4* lrec;
    uint32_t* lrec_cnt;
    uint32_t lrec_cap;
    // 2048-bucket layout without a dictionary: the map kernel variant that
    // write-combines its 8-byte spill streams in LDS (mrgpu_wc.hip, kS)
    uint32_t hi_staged;
    uint32_t lean;          // wc map: the all-ASCII variant (the previous split had no UTF-8 chunk)
    // (last: fields the map kernel never reads keep the others' kernarg offsets)
    uint32_t* lrec_off;  // [256 x nwg + 1] bucket-major offsets of the records by hash bucket (wc_lrec passes)
    uint32_t* lrec_idx;  // [records] record indices in bucket order
    struct LrecPart* lrec_part;  // [kLrecGrid][kLrecSlots] per-range distinct keys with counts
    uint32_t* lrec_pcnt;         // [kLrecGrid] partials per range
    uint8_t* lrec_bkt;           // [region][lrec_cap] each record's hash bucket (lrec_hist_kernel -> lrec_scatter_kernel)
};
// A distinct long-word record of one wc_lrec range: its representative record,
// FNV-1a-64, length, count and hash bucket.
struct LrecPart {
    unsigned long long rep;
    uint64_t h;
    uint32_t len, cnt, bucket, pad;
};

struct LetterTables {
    const uint8_t* l1;
    const uint32_t* l2;
    const uint32_t* b2;  // letters among code points < U+0800: 2048 bits (from l1 / l2, built at mrg_open)
};
// The map kernels' LDS copy of the letter tables (letter_table.inc): l1 of the
// first kLetterLdsPages 256-code-point pages (no letter lies above them in
// Unicode 13.0.0; the generator asserts it) and every distinct l2 page.
constexpr int kLetterLdsPages = 788;
constexpr int kLetterUnique = 111;

// ---- launchers (mrgpu_map.hip) ----
void clear_tables(const Tables& t, bool short_table, hipStream_t s);
// Count the map's 32-byte long-word records (one workgroup per map workgroup's
// region) into the LongTable (mrgpu_map.hip).
void launch_wc_lrec(const Tables& t, uint32_t nwg, hipStream_t s);
// bytes of the bucket offsets ahead of the record indices in the lrec aux buffer
constexpr uint64_t kLrecAuxOff = (256ull * kMaxMapWGs + 64) * 4;
// the per-range partials of the long-word records (after the indices)
constexpr uint64_t kLrecPartBytes = 512ull * 4096 * sizeof(LrecPart) + 1024 * 4 + 256;  // partials, then <= 1024 range counts
// ---- wc pipeline (mrgpu_wc.hip) ----
uint32_t wc_map_grid(uint64_t n, int grid);
// Chunks [cbeg, cend) of the split (kOwn = 992 input bytes each; default: all);
// resume: a previous launch of this map already ran over chunks < cbeg.
bool launch_wc_map(const uint8_t* in, uint64_t n, const Tables& t, LetterTables lt, int grid, int mode,
                   hipStream_t s, uint64_t cbeg = 0, uint64_t cend = ~0ull, bool resume = false);
constexpr uint64_t kWcChunkBytes = 992;   // input bytes a wc map chunk owns
constexpr uint64_t kGrepChunkBytes = 960; // input bytes a grep map chunk owns
// emit: 0 = flush every bucket table into the HBM table (legacy),
//       1 = emit records directly unless the bucket overflowed (then merge through HBM),
//       2 = sample mode: emit table keys, drop misses (approximate counts for the dictionary)
// big: 1024-thread workgroups with twice the LDS table (later rounds)
void launch_wc_agg(const Tables& t, int mode, int emit, bool big, hipStream_t s);
// Segment layout of the multi-round aggregation (Spill::seg_off*) from the map's
// stream counts; off8[E] / off16[E] (E = nb * kAggSegs) are the totals.
// tmp: 2 * E u32 of scratch.
void launch_seg_layout(const Tables& t, uint32_t* tmp, uint64_t* off8, uint64_t* off16, hipStream_t s);
void launch_dict_emit(const Tables& t, uint32_t nwg, hipStream_t s);  // geometry: DictMini iff t.hi_staged
// Gather `nwin` windows of `win` bytes (stride `stride`) of in[0,n) into dst, each followed by '\n'.
void launch_sample_gather(const uint8_t* in, uint64_t n, uint64_t win, uint64_t stride, uint32_t nwin, uint8_t* dst,
                          hipStream_t s);
// Build the dictionary image from sample records ordered by descending count.
void launch_dict_build(const Recs& r, const uint32_t* order, uint64_t n, uint4* cand, uint4* dict, bool mini, hipStream_t s);
// Sort keys for the dictionary build: ~count (u32) of each record.
void launch_dict_keys(const Recs& r, uint32_t* keys, uint32_t* idx, hipStream_t s);
// nlist = ~0: the list length is read on the device (ctr->nlist; nothing to do if 0)
void launch_wc_long(const uint8_t* in, uint64_t n, const Tables& t, LetterTables lt, uint64_t nlist, hipStream_t s);
void launch_grep_map(const uint8_t* in, uint64_t n, const uint8_t* d_pat, uint32_t plen, const Tables& t, int grid,
                     hipStream_t s, uint64_t cbeg = 0, uint64_t cend = ~0ull);
// grep line resolution, linear in the input (mrgpu_map.hip): t.hits (sorted,
// or in the map kernel's order) -> one (start, end) pair per matching line
// occurrence in t.lines (ctr->nlines), hits in lines longer than a lane's scan
// window to t.defer (ctr->ndefer).  dev_count: nhits is the list's capacity
// and the kernels read the hit / deferred-hit counts on the device, so no host
// round trip sits between the map kernel and the line resolution.
void launch_grep_resolve(const uint8_t* in, uint64_t n, const uint8_t* d_pat, uint32_t plen, const Tables& t,
                         uint64_t nhits, bool dev_count, bool sorted, hipStream_t s);
void launch_grep_resolve_long(const uint8_t* in, uint64_t n, const uint8_t* d_pat, uint32_t plen, const Tables& t,
                              uint64_t ndefer, uint64_t nhits, bool dev_count, bool sorted, hipStream_t s);
// t.lines -> the LongTable (one distinct line = one slot).
// emit: each line that claims its slot also writes its record (t.out: key
// prefix, length, partition, its bytes copied to the arena at ctr->arena) —
// no collect pass over the table afterwards.  dev_count: nlines is a bound and
// the kernel reads the resolved line count on the device.
void launch_grep_insert(const uint8_t* in, const Tables& t, uint64_t nlines, bool dev_count, bool emit, hipStream_t s);
// Clear the LongTable and its fill counters, and the record / arena cursors (a
// re-run of launch_grep_insert after growth).
void clear_long_table(const Tables& t, hipStream_t s);
void launch_grep_all_lines(const uint8_t* in, uint64_t n, const Tables& t, int grid, hipStream_t s);
struct ReduceWs;
// Append the HBM tables' keys to t.out: the ShortTable's `short_used` keys at
// records [base, base + short_used) (ctr->nrec must equal base), then the
// LongTable's at ctr->nrec (arena offsets from ctr->arena).  Returns 0 or a hipError_t.
// Append the HBM tables' keys to t.out at ctr->nrec, every count read on the
// device (no host round trip): the ShortTable's claimed slots from its claim
// list, then (long_table) the LongTable's keys with their arena bytes.
// Capacity overflows set kStRecFull.  Returns 0 or a hipError_t.
int launch_collect(const Tables& t, bool long_table, hipStream_t s);
// Undo a collect whose arena was too small (records and arena bytes from
// ctr->nrec_base, kStRecFull cleared), so it can run again with a bigger arena.
void launch_collect_undo(const Tables& t, hipStream_t s);
void launch_insert_recs(const Recs& src, const Tables& t, hipStream_t s);
int map_grid_size(int device);

// ---- stable LSD radix sort (mrgpu_sort.hip) ----
struct RadixWs;
RadixWs* radix_ws_new();
void radix_ws_free(RadixWs*);
// Stable sort by the low `bits` key bits (8- or 10-bit digits, one launch per
// pass); k_in / v_in are not modified.  Returns 0 or a hipError_t.
// digit bits: 10, or 8 (0 = 8).
void radix_ws_set_digit_bits(RadixWs*, int bits);
int radix_sort_pairs_u32(RadixWs*, const uint32_t* k_in, uint32_t* k_out, const uint32_t* v_in, uint32_t* v_out,
                         uint64_t n, unsigned bits, hipStream_t s);
int radix_sort_pairs_u64(RadixWs*, const uint64_t* k_in, uint64_t* k_out, const uint32_t* v_in, uint32_t* v_out,
                         uint64_t n, unsigned bits, hipStream_t s);
int radix_sort_keys_u64(RadixWs*, const uint64_t* k_in, uint64_t* k_out, uint64_t n, unsigned bits, hipStream_t s);

// ---- reduce (mrgpu_reduce.hip) ----
struct ReduceWs;  // opaque workspace
ReduceWs* reduce_ws_new();
void reduce_ws_free(ReduceWs*);
// Sort tuning: radix digit bits of the 64-bit passes (8 or 10; others ignored),
// fold the partition into the first key pass (1 / 0; -1 keeps it), grep radix
// passes over 16 key bytes (1) or 8 (0; -1 keeps it).
void reduce_ws_set(ReduceWs*, int digit_bits, int fold_part, int grep_k1);
// Tied runs merge-sorted on compact key copies (default) or on the records.
void reduce_ws_set_compact_ties(ReduceWs*, bool on);
// The single-key wc sort pass by the hand-written bucketed sort (option) or the radix passes (default).
void reduce_ws_set_bin_sort(ReduceWs*, bool on);
// The wc single-key pass on the key's top 32 bits (default) or the whole 60/64-bit key.
void reduce_ws_set_prefix32(ReduceWs*, bool on);
// (compatibility: the radix passes are always the hand-written sort)
void reduce_ws_set_own_sort(ReduceWs*, bool on);
// grep's tied runs ranked per run (default) or all merge-sorted together.
void reduce_ws_set_tie_rank(ReduceWs*, bool on);
void reduce_ws_set_grep_bins(ReduceWs*, int v);
// Sort recs (optionally only partition `only_part`), format "key value\n" lines.
// Returns 0 or a hipError_t; output in device buffer *d_out (workspace-owned), sizes on host.
// ascii_keys: every key byte is < 0x80 (the sort key then packs 7 bits per byte).
int reduce_format(ReduceWs* ws, const Recs& r, int app, uint32_t nreduce, uint32_t only_part, uint8_t** d_out,
                  uint64_t* out_n, uint64_t* h_offsets, hipStream_t s, bool ascii_keys, uint8_t* hout = nullptr,
                  uint64_t hout_cap = 0);
// Bytes reduce_format's output can take at most (its buffer, or a host buffer
// given as hout: the lines are then written straight into pinned host memory).
uint64_t reduce_out_bound(const Recs& r, int app);
// Radix sort of u64 keys (the low `bits` bits); result in k_out.
int sort_u64_keys(ReduceWs* ws, uint64_t* k_in, uint64_t* k_out, uint64_t n, unsigned bits, hipStream_t s);
// In-place stable sort of device keys (key_bytes 4 or 8, low `bits` bits) with
// optional u32 values (nullptr: 8-byte keys only); waits for the stream.
int sort_in_place(ReduceWs* ws, int key_bytes, void* keys, uint32_t* vals, uint64_t n, unsigned bits, hipStream_t s);
// Stable radix sort of (u32 key, u32 value) pairs; result in k_out / v_out.
int sort_u32_pairs(ReduceWs* ws, uint32_t* k_in, uint32_t* k_out, uint32_t* v_in, uint32_t* v_out, uint64_t n,
                   unsigned bits, hipStream_t s);
// ---- reference JSON-lines intermediate format (mrgpu_json.hip) ----
// Per record: L = escaped {"Key":..,"Value":..}\n line bytes, T = L * count,
// P = 4 KiB output pieces; loff / toff / poff their exclusive scans.  grow(gctx, n)
// returns >= n bytes of device scratch.  Returns 0 or -1.
int json_lengths(const Recs& r, int app, uint64_t* L, uint64_t* T, uint64_t* P, uint64_t* loff, uint64_t* toff,
                 uint64_t* poff, void* (*grow)(void*, size_t), void* gctx, hipStream_t s);
// Escaped lines into `lines` (at loff), then the output (total bytes) with each
// record's line repeated count times.
int json_write(const Recs& r, int app, const uint64_t* L, const uint64_t* loff, const uint64_t* toff,
               const uint64_t* poff, uint64_t npieces, uint64_t total, uint8_t* lines, uint8_t* out, hipStream_t s);
// Compact recs with part == p (or owner rank) into dst (device), returns count on host.
int select_recs(ReduceWs* ws, const Recs& src, uint32_t mod, uint32_t want, Recs* dst_host_desc, hipStream_t s);

__host__ __device__ inline uint32_t fnv1a32_step(uint32_t h, uint32_t byte) {
    return (h ^ byte) * 16777619u;
}

}  // namespace mrg
