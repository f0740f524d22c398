// mrgpu_api.hip — the C ABI (include/mrgpu.h): contexts, map/reduce
// orchestration, intermediate export/import and the RCCL shuffle.
//
// Call flow of mrg_map for wc (replaces mr/worker.go:58-92 + mrapps/wc.go):
//   [H2D copy of the split if host-resident] -> hot-key dictionary from a
//   sample (mrgpu_wc.hip stage 0) -> wc_map_kernel -> wc_agg_kernel (direct
//   records) + dict_emit_kernel -> wc_long_kernel -> collect of whatever went
//   through the HBM tables -> records (partition = ihash % nReduce).
// grep: grep_map_kernel -> grep_lines_kernel (LongTable) -> collect.
// If a table, list or the record buffer overflowed (the status word says
// which), the capacity grows and the map is re-run, so results never depend on
// the initial sizing.
#include <rccl/rccl.h>

#include <algorithm>
#include <functional>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/mrgpu.h"
#include "letter_table.inc"
#include "mrgpu_device.h"
#include "mrgpu_exch.h"

using namespace mrg;
static_assert(MRG_LETTER_LDS_PAGES == kLetterLdsPages && MRG_LETTER_NUNIQUE == kLetterUnique,
              "regenerate letter_table.inc and update kLetterLdsPages / kLetterUnique");

namespace {

// Freed device blocks kept for reuse (parts record arrays and arenas): a map
// task's parts adopt the context's record buffer instead of copying it, and the
// next task takes a cached block instead of hipMalloc — hipFree would also
// synchronize the device.  Process-wide (contexts may live on several threads).
namespace {
struct CachedBlock {
    int dev;
    void* p;
    size_t bytes;
};
std::mutex g_cache_mu;
std::vector<CachedBlock> g_cache;
constexpr size_t kCacheBlocks = 8;
}  // namespace

// A cached block of `dev` with at least `bytes` (the smallest such), or nullptr.
static void* cache_take(int dev, size_t bytes, size_t* got) {
    std::lock_guard<std::mutex> g(g_cache_mu);
    size_t best = g_cache.size();
    for (size_t i = 0; i < g_cache.size(); i++)
        if (g_cache[i].dev == dev && g_cache[i].bytes >= bytes && (best == g_cache.size() || g_cache[i].bytes < g_cache[best].bytes))
            best = i;
    if (best == g_cache.size()) return nullptr;
    void* p = g_cache[best].p;
    *got = g_cache[best].bytes;
    g_cache.erase(g_cache.begin() + best);
    return p;
}

static void cache_put(int dev, void* p, size_t bytes) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> g(g_cache_mu);
        if (g_cache.size() < kCacheBlocks) {
            g_cache.push_back({dev, p, bytes});
            return;
        }
    }
    hipFree(p);
}

// Cached block or a fresh allocation (the caller has bound `dev`).
static hipError_t block_alloc(int dev, size_t bytes, void** p, size_t* got) {
    if ((*p = cache_take(dev, bytes, got))) return hipSuccess;
    *got = bytes;
    return hipMalloc(p, bytes);
}

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    // Like ensure(), but a missing buffer comes from the block cache (buffers
    // that are handed over to parts objects: recbuf, recarena).
    hipError_t ensure_cached(size_t n, int dev) {
        if (n <= cap) return hipSuccess;
        if (p) cache_put(dev, p, cap);
        p = nullptr;
        cap = 0;
        size_t got = 0;
        hipError_t e = block_alloc(dev, n < 4096 ? 4096 : n, &p, &got);
        if (e == hipSuccess) cap = got;
        else p = nullptr;
        return e;
    }
    // The buffer changes owner (a parts object): this one is empty afterwards.
    void* adopt(size_t* bytes) {
        void* q = p;
        *bytes = cap;
        p = nullptr;
        cap = 0;
        return q;
    }
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        size_t c = n < 4096 ? 4096 : n;
        hipError_t e = hipMalloc(&p, c);
        if (e == hipSuccess) cap = c;
        return e;
    }
    // Like ensure(), but a growing buffer gets 25 % headroom: sizes that vary a
    // little from call to call (spill totals) must not hipFree + hipMalloc
    // gigabytes every step (measured: +1.3 ms per C2 step, seconds at C5).
    hipError_t ensure_grow(size_t n) {
        if (n <= cap) return hipSuccess;
        return ensure(n + n / 4);
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
};

constexpr uint64_t kHostMagic = 0x4D524748424F5354ull;  // "MRGHBOST"

}  // namespace

struct ExchSide;
static void exch_free(ExchSide* x);

// Deadline of the collective phases (communicator setup, the shuffle).  A rank
// that never joins leaves the others blocked inside RCCL or a stream sync with
// no error to return; the watchdog thread then names the phase on stderr and
// ends the process with status 124, so a launcher sees a failed rank instead of
// a hang.  One thread per context, idle (on a condition variable) outside the
// guarded phases.
struct Watchdog {
    std::mutex mu;
    std::condition_variable cv;
    const char* phase = nullptr;
    std::chrono::steady_clock::time_point deadline;
    int64_t limit_ms = 0;
    bool stop = false;
    int rank = 0, nranks = 1;
    std::thread th;
    void run() {
        std::unique_lock<std::mutex> lk(mu);
        while (!stop) {
            if (!phase) {
                cv.wait(lk);
                continue;
            }
            cv.wait_until(lk, deadline);
            if (!stop && phase && std::chrono::steady_clock::now() >= deadline) {
                fprintf(stderr, "mrgpu: rank %d of %d: collective phase '%s' did not finish within %lld ms; exiting\n",
                        rank, nranks, phase, (long long)limit_ms);
                fflush(stderr);
                _exit(124);
            }
        }
    }
    // Start guarding (the deadline runs from here); nested phases keep it.
    void enter(const char* p, int64_t ms, int r, int n) {
        std::lock_guard<std::mutex> g(mu);
        if (!th.joinable()) th = std::thread([this] { run(); });
        phase = p;
        limit_ms = ms;
        rank = r;
        nranks = n;
        deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(ms);
        cv.notify_one();
    }
    void set(const char* p) {
        std::lock_guard<std::mutex> g(mu);
        phase = p;
    }
    void leave() {
        std::lock_guard<std::mutex> g(mu);
        phase = nullptr;
        cv.notify_one();
    }
    ~Watchdog() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
            cv.notify_one();
        }
        if (th.joinable()) th.join();
    }
};

struct mrg_ctx {
    ExchSide* exch = nullptr;  // RCCL shuffle buffers, kept across calls (no hipMalloc / hipFree per step)
    int device = 0;
    hipStream_t s = nullptr;
    hipEvent_t ev[14] = {};  // 0-3, 8-10: map phases; 4-5 reduce; 6-7 exchange / d2h; 12 exchange end; 13 unpack start
    std::string err;
    uint8_t* d_l1 = nullptr;
    uint32_t* d_l2 = nullptr;
    uint32_t* d_b2 = nullptr;  // letters among code points < U+0800 (2048 bits)
    DevBuf sh, lo, list, ctr, staging, pat, spool, spmeta;
    DevBuf shl;  // the ShortTable's claim list
    DevBuf spool_alt;     // diagnostic option spill_alt_pools: a second spill pool, the two alternate per split
    int spill_alt = 0;
    DevBuf bflag, dict, dict_cnt, sample, recbuf, recarena, sortbuf, dbg;
    DevBuf segmeta, seg8[2], seg16[2];  // multi-round aggregation: layout + ping-pong miss segments
    bool seg_sync = true;               // size the miss segments from this split's totals (host read)
    bool out_direct = true;             // mrg_run_job: output lines written straight into pinned host memory
    bool out_direct_grep = true;        // ... for grep too (out_direct = 1: wc only)
    bool grep_sort_hits = false;        // grep: hits sorted by position before line resolution (option grep_sort_hits)
    bool grep_emit = true;              // grep: records written by the table insert (option grep_emit; 0: collect pass)
    uint64_t grep_hint_lines = 0, grep_hint_bytes = 0;  // grep: the previous split's resolved lines and their bytes
    bool grep_literal = false;          // grep: regexp metacharacters taken literally (QuoteMeta) instead of refused
    DevBuf lrec, lrec_cnt;              // wc: 32-byte long-word records [map wave][lrec_cap], their counts
    DevBuf lrec_aux;                    // wc: their bucket offsets and bucket-ordered indices (launch_wc_lrec)
    uint32_t lrec_cap = 1024;           // records per map wave's region (grows on kStLrecFull)
    bool lrec_on = true;                // option long_records (-1: every long word through the offset list)
    // 2048-bucket (high-cardinality) splits: the mini dictionary (DictMini), the
    // map kernel write-combines its 8-byte spill streams in the LDS the full one
    // would take (option hi_stage)
    bool hi_stage = true;
    uint64_t arena_hint = 0;            // wc: long-key bytes expected in a split (the previous one's + 25 %)
    DevBuf jmeta, jtmp, jlines, jout;    // JSON-lines export (reference intermediate format)
    DevBuf ghits, glines, gdefer;        // grep: sorted hits, resolved (start, end) lines, deferred hits
    int agg_rounds = 8;                 // bucket aggregation rounds at most (the last sends leftovers to HBM)
    // Misses per bucket below which a round settles them in the HBM table instead
    // of carrying them (C2: ~5 per bucket, so no second round).  Kept small:
    // measured on C5, 4096 made the aggregation 59 ms -> 2.8 s (HBM inserts of
    // hot leftover keys serialize).
    uint32_t agg_carry_min = 64;
    // 1024-thread aggregator workgroups with twice the LDS table (one per CU)
    // instead of 512-thread ones (two per CU), in round 0 / later rounds.
    // Round 0: 0 = by layout (agg_big0), 1 = big, -1 = small.  Measured: the
    // 2048-bucket layout's ~4.9 K keys per bucket need the big table; at 512
    // buckets (C2, ~2 K keys) two small workgroups per CU are faster, their
    // few overflowing keys settling in round 1 (1.20 -> 1.13 ms).  Later
    // rounds: big (C5 at 512 buckets, 4 rounds instead of 6).
    int agg_big0 = 0;
    bool agg_big_later = true;
    double spill_scale = 1.0;           // spill stream capacity factor (from the dictionary sample's miss rate)
    double words_per_byte = 0.0;        // words per input byte of the previous wc split (staged spill sizing)
    double spilled_per_byte = 0.0;      // spill records per input byte of the previous wc split
    bool prev_staged = false;           // the previous wc split ran the staged map
    bool prev_ascii = false;            // the previous wc split had no UTF-8 chunk (its map: the lean variant)
    bool lean_on = true;                // option map_lean (-1: never the lean variant)
    uint64_t async_direct_max = 64ull << 20;  // option async_direct_max: larger async wc outputs copy on the output stream
    bool debug_times = getenv("MRG_DEBUG_TIMES") != nullptr;
    uint64_t rec_cap = 1u << 21;       // record output buffer capacity (grows on overflow)
    bool sh_clean = false;             // ShortTable known to be empty (skip its clear)
    int dict_mode = 0;                 // <0: never build the hot-key dictionary
    bool dict_warm = true;             // level-1 dictionary = the previous map task's (see build_dict)
    bool dict_valid = false;           // c->dict holds a dictionary built by an earlier call
    bool dict_mini = false;            // c->dict's geometry: DictMini (staged 2048-bucket map) or DictFull
    // Dictionary reuse: the previous split's dictionary is kept (no rebuild) when
    // it hits this split's sample at >= dict_keep x the fraction it hit on the
    // split it was built for (dict_frac_built, measured on that split's map).
    double dict_keep = 0.97;
    double dict_frac_built = 0;
    bool dict_fresh = false;           // the current split built its own dictionary
    uint64_t dict_min_bytes = 32ull << 20;
    uint64_t dict_sample_bytes = 16ull << 20;  // C2: 16 vs 64 MB loses 0.13% of dictionary hits, halves the build
    uint64_t spill_sub_keys = 0, spill_sub8 = 0;
    uint32_t spill_nwg = 1;
    // Spill buckets of the current layout and of the next wc split.  2048 when
    // the previous split's aggregated keys would not fit 256 buckets' LDS tables
    // (the 1024-thread ones) in one round (C5-like splits: 1e7 keys), else 256;
    // option spill_buckets fixes it (0 = this feedback rule; 512 = the previous
    // default, small round-0 tables).
    uint32_t spill_nb = kSpillBucketsLo, next_nb = kSpillBucketsLo;
    int spill_buckets_opt = 0;
    uint64_t spill_hi_keys = 6000ull * kSpillBuckets;  // aggregated keys above which the next split uses 2048
    int64_t spill_force_sub = 0;
    int spill_mid_div = 2;  // 16-byte streams hold sub8 / spill_mid_div records (option spill_mid_div)
    int map_mode = 0;  // benchmark ablation of wc_map_kernel phases (0 = normal)
    // mrg_run_job without the shuffle even with a communicator (bench.py's
    // same-process T(1) for the weak-scaling efficiency: the rank's own split,
    // every partition reduced locally)
    bool skip_exchange = false;
    // (tests) mrg_exchange runs its RCCL collectives on a one-rank communicator
    // too, instead of keeping every key locally: the calls, the count and
    // displacement arrays and the unpack, on one GPU (RCCL refuses two ranks on one)
    bool exch_force_rccl = false;
    // Host-input splits of at least ingest_min bytes are copied in pieces of
    // ~ingest_piece bytes on a second stream, each piece mapped as soon as it and
    // the next one (look-ahead) are resident.
    uint64_t ingest_piece = 256ull << 20, ingest_min = 64ull << 20;
    hipStream_t cs = nullptr;            // copy stream (created on first use)
    std::vector<hipEvent_t> piece_ev;    // one per piece, reused
    uint8_t* h_sample = nullptr;         // pinned: dictionary sample gathered from host input
    size_t h_sample_cap = 0;
    int sh_log2 = 20, lo_log2 = 14;  // HBM tables (grow on overflow); the wc short table holds only the spill path's leftovers
    // LongTable size of the current call: wc maps start from lo_log2 (words > 16
    // bytes; sticky, grows on overflow), grep maps size it per job from their
    // resolved line count, merges / imports from their record count.  Only
    // 2^lo_log2_cur slots are cleared and collected.
    int lo_log2_cur = 14;
    uint64_t list_cap = 1u << 20;
    int grid = 256;
    ReduceWs* rws = nullptr;
    mrg_stats stats{};
    Counters* h_ctr = nullptr;     // pinned
    uint64_t* h_scr = nullptr;     // pinned scratch for small device -> host reads (8 words)
    uint8_t* h_out = nullptr;      // pinned result buffer for mrg_run_job
    size_t h_out_cap = 0;
    // mrg_run_job_async: up to two jobs whose output bytes are still crossing PCIe
    // (on the output stream os, into their own pinned buffers) while the caller
    // queues the next job; aj[aj_head] is the oldest
    struct AsyncJob {
        uint8_t* host = nullptr;
        size_t cap = 0;
        uint64_t n = 0;
        std::vector<uint64_t> offsets;
        hipEvent_t start = nullptr, done = nullptr;
        mrg_stats stats{};
    } aj[2];
    int aj_head = 0, aj_count = 0;
    hipStream_t os = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    // collective deadline (option exchange_timeout_ms; comm init gets 4x)
    int64_t exch_timeout_ms = 120000;
    Watchdog wd;
};

struct mrg_parts {
    int app = 0;
    uint32_t nreduce = 1;
    int device = 0;
    bool ascii = false;  // every key byte < 0x80 (the map saw no byte >= 0x80): the reduce packs its sort key
    Recs r{};
    void* block = nullptr;  // record arrays
    uint8_t* arena = nullptr;
    size_t block_bytes = 0, arena_bytes = 0;  // returned to the block cache on free
};

static int fail(mrg_ctx* c, int code, const char* fmt, ...) {
    char b[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof b, fmt, ap);
    va_end(ap);
    if (c) c->err = b;
    return code;
}

#define HCHK(c, x)                                                                                       \
    do {                                                                                                 \
        hipError_t _e = (x);                                                                             \
        if (_e != hipSuccess)                                                                            \
            return fail((c), _e == hipErrorOutOfMemory ? MRG_ENOMEM : MRG_EDEVICE, "%s failed: %s (%s:%d)", #x, \
                        hipGetErrorString(_e), __FILE__, __LINE__);                                      \
    } while (0)

#define NCHK(c, x)                                                                                  \
    do {                                                                                            \
        ncclResult_t _r = (x);                                                                      \
        if (_r != ncclSuccess) return fail((c), MRG_ECOMM, "%s failed: %s", #x, ncclGetErrorString(_r)); \
    } while (0)

static int bind(mrg_ctx* c) {
    HCHK(c, hipSetDevice(c->device));
    return MRG_OK;
}

static Tables make_tables(mrg_ctx* c) {
    Tables t;
    t.sh = (ShortSlot*)c->sh.p;
    t.sh_mask = (1ull << c->sh_log2) - 1;
    t.lo = (LongSlot*)c->lo.p;
    t.lo_mask = (1ull << c->lo_log2_cur) - 1;
    t.hits = (const uint64_t*)c->ghits.p;
    t.lines = (uint64_t*)c->glines.p;
    t.defer = (uint64_t*)c->gdefer.p;
    t.sh_list = (uint32_t*)c->shl.p;
    t.list = (uint64_t*)c->list.p;
    t.list_cap = c->list_cap;
    t.ctr = (Counters*)c->ctr.p;
    t.sp.pool = (uint4*)c->spool.p;
    t.sp.sub_keys = c->spill_sub_keys;
    t.sp.sub8 = c->spill_sub8;
    t.sp.pool8 = c->spool.p ? (uint64_t*)((uint4*)c->spool.p + c->spill_sub_keys * c->spill_nb * c->spill_nwg)
                            : nullptr;
    t.sp.nwg = c->spill_nwg;
    t.sp.nb = c->spill_nb;
    t.sp.counts = (uint32_t*)c->spmeta.p;
    t.sp.counts8 = c->spmeta.p ? t.sp.counts + (size_t)c->spill_nb * c->spill_nwg : nullptr;
    t.sp.seg_off8 = t.sp.seg_off16 = nullptr;
    t.sp.seg_n_in = nullptr;
    t.sp.seg_n_out = nullptr;
    t.sp.seg8_in = nullptr;
    t.sp.seg8_out = nullptr;
    t.sp.seg16_in = nullptr;
    t.sp.seg16_out = nullptr;
    t.sp.seg8_cap = t.sp.seg16_cap = 0;
    t.sp.round = 0;
    t.sp.last = 1;
    t.sp.carry_min = c->agg_carry_min;
    t.out = Recs{};
    t.out_cap = 0;
    t.nreduce = 1;
    t.bflag = (uint32_t*)c->bflag.p;
    t.dict = nullptr;
    t.dict_cnt = (uint32_t*)c->dict_cnt.p;
    t.dbg = c->debug_times && c->dbg.ensure(2 * (kSpillBucketsHi + kMaxMapWGs) * 8) == hipSuccess ? (unsigned long long*)c->dbg.p : nullptr;
    t.hi_staged = 0;
    t.lean = 0;
    t.lrec = nullptr;  // set by wc_map for the split's map (sample maps and grep use the offset list)
    t.lrec_cnt = nullptr;
    t.lrec_cap = 0;
    t.lrec_off = t.lrec_idx = nullptr;
    t.lrec_part = nullptr;
    t.lrec_pcnt = nullptr;
    t.lrec_bkt = nullptr;
    return t;
}

// SoA view of the context's record output buffer (capacity rec_cap).
static Recs rec_view(mrg_ctx* c) {
    Recs r{};
    const uint64_t cap = c->rec_cap;
    char* b = (char*)c->recbuf.p;
    r.k0 = (uint64_t*)b; b += cap * 8;
    r.k1 = (uint64_t*)b; b += cap * 8;
    r.cnt = (uint64_t*)b; b += cap * 8;
    r.koff = (uint64_t*)b; b += cap * 8;
    r.len = (uint32_t*)b; b += cap * 4;
    r.part = (uint32_t*)b;
    r.arena = (uint8_t*)c->recarena.p;
    r.arena_n = c->recarena.cap;
    r.n = 0;
    return r;
}

// Spill pool for dictionary misses: 1.5 bytes of pool per input byte (C2
// spills ~0.5 bytes of records per input byte), split into spill_nb x nwg
// streams of 16-byte records (0.75 B/B) and as many of 8-byte records (0.75 B/B),
// times c->spill_scale when the dictionary sample shows a higher miss rate.
// A stream that fills up sends the rest of its keys to the HBM table, so the
// size only affects speed, never results.
static int ensure_spill(mrg_ctx* c, uint64_t n) {
    const uint32_t nwg = wc_map_grid(n, c->grid);
    const uint64_t nb = c->spill_nb;
    uint64_t sub8 = 2 * ((uint64_t)((double)((n - n / 4) / 16 / (nb * nwg)) * c->spill_scale) + 64);
    sub8 = (sub8 + 63) & ~63ull;
    uint64_t sub = (sub8 / (uint64_t)std::max(1, c->spill_mid_div) + 63) & ~63ull;
    // test knob: tiny streams (even: the aggregator reads 8-byte records in pairs)
    if (c->spill_force_sub > 0) sub = sub8 = ((uint64_t)c->spill_force_sub + 1) & ~1ull;
    // a workgroup's streams are addressed by 32-bit byte offsets in the map kernel
    // ((b * sub + pos) * 16 < 2^32): 2^32 bytes of 16-byte and as many of 8-byte
    // streams per workgroup is a ~1 TB split at scale 1 with 512 workgroups
    if (nb * std::max(sub * 16, sub8 * 8) >= (1ull << 32))
        return fail(c, MRG_EINVAL, "split too large for the spill layout (%llu bytes)", (unsigned long long)n);
    c->spill_nwg = nwg;
    c->spill_sub_keys = sub;
    c->spill_sub8 = sub8;
    const size_t pool = (sub * sizeof(uint4) + sub8 * sizeof(uint64_t)) * nb * nwg;
    if (c->debug_times && pool > c->spool.cap)
        fprintf(stderr, "[mrg spill] pool %.2f -> %.2f GB (scale %.3f, %llu buckets)\n", c->spool.cap / 1e9,
                (pool + pool / 4) / 1e9, c->spill_scale, (unsigned long long)nb);
    HCHK(c, c->spool.ensure_grow(pool));
    HCHK(c, c->spmeta.ensure((size_t)2 * nb * nwg * sizeof(uint32_t)));
    return MRG_OK;
}

static int ensure_tables(mrg_ctx* c) {
    const void* old = c->sh.p;
    HCHK(c, c->sh.ensure(sizeof(ShortSlot) << c->sh_log2));
    HCHK(c, c->shl.ensure(sizeof(uint32_t) << c->sh_log2));
    if (c->sh.p != old) c->sh_clean = false;  // fresh memory is not zeroed
    HCHK(c, c->bflag.ensure(kSpillBucketsHi * sizeof(uint32_t)));
    const size_t lo_bytes = sizeof(LongSlot) << c->lo_log2_cur;
    if (c->lo.cap > 4 * lo_bytes && c->lo.cap > (256u << 20)) c->lo.release();  // a past grep job's big table
    HCHK(c, c->lo.ensure(lo_bytes));
    HCHK(c, c->list.ensure(c->list_cap * sizeof(uint64_t)));
    HCHK(c, c->ctr.ensure(sizeof(Counters)));
    return MRG_OK;
}

static int read_counters(mrg_ctx* c) {
    HCHK(c, hipMemcpyAsync(c->h_ctr, c->ctr.p, sizeof(Counters), hipMemcpyDeviceToHost, c->s));
    HCHK(c, hipStreamSynchronize(c->s));
    if (c->h_ctr->short_used) c->sh_clean = false;
    return MRG_OK;
}

// Reset the counters (and the ShortTable unless it is known to be empty).
static void clear_for_run(mrg_ctx* c, const Tables& t) {
    clear_tables(t, !c->sh_clean, c->s);
    c->sh_clean = true;
}

static float ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 0.f;
    return ms;
}

// ---------------------------------------------------------------- parts
static int parts_alloc(mrg_ctx* c, uint64_t n, uint64_t arena_n, int app, uint32_t nreduce, mrg_parts** out) {
    mrg_parts* p = new mrg_parts();
    p->app = app;
    p->nreduce = nreduce;
    p->device = c->device;
    uint64_t cap = n ? n : 1;
    size_t bytes = cap * (8 + 8 + 4 + 8 + 4 + 8) + 256;
    hipError_t e = block_alloc(c->device, bytes, &p->block, &p->block_bytes);
    if (e != hipSuccess) { delete p; return fail(c, MRG_ENOMEM, "hipMalloc(%zu) for parts failed", bytes); }
    e = block_alloc(c->device, arena_n ? arena_n : 16, (void**)&p->arena, &p->arena_bytes);
    if (e != hipSuccess) {
        cache_put(c->device, p->block, p->block_bytes);
        delete p;
        return fail(c, MRG_ENOMEM, "hipMalloc arena failed");
    }
    char* b = (char*)p->block;
    p->r.k0 = (uint64_t*)b; b += cap * 8;
    p->r.k1 = (uint64_t*)b; b += cap * 8;
    p->r.cnt = (uint64_t*)b; b += cap * 8;
    p->r.koff = (uint64_t*)b; b += cap * 8;
    p->r.len = (uint32_t*)b; b += cap * 4;
    p->r.part = (uint32_t*)b;
    p->r.arena = p->arena;
    p->r.n = n;
    p->r.arena_n = arena_n;
    *out = p;
    return MRG_OK;
}

// Collect the current HBM tables into a fresh parts object.
static int collect_parts(mrg_ctx* c, int app, uint32_t nreduce, mrg_parts** out) {
    int rc = read_counters(c);
    if (rc) return rc;
    Counters& h = *c->h_ctr;
    uint64_t n = h.short_used + h.long_used;
    uint64_t arena = h.long_bytes;
    mrg_parts* p = nullptr;
    if ((rc = parts_alloc(c, n, arena, app, nreduce, &p))) return rc;
    Tables t = make_tables(c);
    t.out = p->r;
    t.out_cap = n;
    t.nreduce = nreduce;
    const bool sh_used = h.short_used != 0, lo_used = h.long_used != 0;
    HCHK(c, hipMemsetAsync(&t.ctr->nrec, 0, 3 * sizeof(unsigned long long), c->s));
    (void)sh_used;
    if (launch_collect(t, lo_used, c->s))
        return fail(c, MRG_EDEVICE, "collect failed");
    rc = read_counters(c);
    if (rc) { mrg_parts_free(p); return rc; }
    if (h.nrec != n || h.arena != arena || (h.status & kStRecFull)) {
        mrg_parts_free(p);
        return fail(c, MRG_EDEVICE, "collect mismatch: %llu/%llu records, %llu/%llu arena bytes", h.nrec,
                    (unsigned long long)n, h.arena, (unsigned long long)arena);
    }
    c->stats.distinct_keys = n;
    c->stats.long_keys = h.nlong_rec;
    *out = p;
    return MRG_OK;
}

// Grow whatever overflowed; returns 1 if a re-run is needed.
static int grow_on_overflow(mrg_ctx* c, uint32_t st) {
    int again = 0;
    if (st & kStShortFull) { c->sh_log2 += 2; again = 1; }
    if (st & kStLongFull) { c->lo_log2_cur += 2; again = 1; }
    if (st & kStListFull) { c->list_cap = std::max<uint64_t>(c->list_cap * 4, c->h_ctr->nlist + 1024); again = 1; }
    if (st & kStRecFull) { c->rec_cap = std::max<uint64_t>(c->rec_cap * 2, c->h_ctr->nrec + 4096); again = 1; }
    if (st & kStSegFull) { c->seg_sync = true; again = 1; }
    return again;
}

static int ensure_recbuf(mrg_ctx* c) {
    HCHK(c, c->recbuf.ensure_cached(c->rec_cap * 40, c->device));
    HCHK(c, c->recarena.ensure_cached(16, c->device));
    return MRG_OK;
}

// Diagnostics: grep_insert_kernel's per-workgroup phase stamps (ins_stamp), as
// percentiles of each phase's end relative to the earliest start, in us.  (The
// stamps of a workgroup's last grid-stride step.)
static void print_insert_stamps(mrg_ctx* c) {
    constexpr uint32_t kMaxWg = 1024;
    std::vector<unsigned long long> h(4 * kMaxWg);
    hipStreamSynchronize(c->s);
    hipMemcpy(h.data(), c->dbg.p, h.size() * 8, hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull;
    uint32_t nb = 0;
    for (uint32_t b = 0; b < kMaxWg; b++)
        if (h[4 * b + 3] > h[4 * b] && h[4 * b]) { t0 = std::min(t0, h[4 * b]); nb++; }
    if (!nb) return;
    fprintf(stderr, "[mrg stamps] grep insert, %u workgroups:", nb);
    for (int k = 0; k < 4; k++) {
        std::vector<double> v;
        for (uint32_t b = 0; b < kMaxWg; b++)
            if (h[4 * b + 3] > h[4 * b] && h[4 * b]) v.push_back((h[4 * b + k] - t0) / 100.0);
        std::sort(v.begin(), v.end());
        fprintf(stderr, " phase%d p0 %.1f p50 %.1f p100 %.1f;", k, v[0], v[v.size() / 2], v.back());
    }
    fprintf(stderr, "\n");
    hipMemset(c->dbg.p, 0, h.size() * 8);
}

// Total bytes the map's long-word record regions may take: the
// split's size, at least 256 MiB.
static uint64_t lrec_bytes_cap(uint64_t len) { return std::max<uint64_t>(len, 256ull << 20); }

// Diagnostics: distribution of per-workgroup start/end stamps (100 MHz) of the
// last aggregation kernel, relative to the earliest start.
static void print_stamps(mrg_ctx* c, const char* what, uint32_t nblocks, uint32_t off = 0) {
    if (!c->debug_times || !c->dbg.p) return;
    std::vector<unsigned long long> h(2 * nblocks);
    hipStreamSynchronize(c->s);
    hipMemcpy(h.data(), (unsigned long long*)c->dbg.p + 2 * off, h.size() * 8, hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull, s_max = 0, e_min = ~0ull, e_max = 0;
    for (uint32_t b = 0; b < nblocks; b++) t0 = std::min(t0, h[2 * b]);
    std::vector<double> st, en;
    for (uint32_t b = 0; b < nblocks; b++) {
        s_max = std::max(s_max, h[2 * b] - t0);
        e_min = std::min(e_min, h[2 * b + 1] - t0);
        e_max = std::max(e_max, h[2 * b + 1] - t0);
    }
    std::vector<std::pair<unsigned long long, uint32_t>> ends;
    for (uint32_t b = 0; b < nblocks; b++) ends.push_back({h[2 * b + 1] - t0, b});
    std::sort(ends.begin(), ends.end());
    fprintf(stderr, "[mrg stamps] %s: last start %.1f us, end p0 %.1f p50 %.1f p90 %.1f p100 %.1f us; slowest:", what,
            s_max / 100.0, e_min / 100.0, ends[nblocks / 2].first / 100.0, ends[nblocks * 9 / 10].first / 100.0,
            e_max / 100.0);
    for (uint32_t k = 0; k < 5 && k < nblocks; k++) fprintf(stderr, " %u", ends[nblocks - 1 - k].second);
    fprintf(stderr, "\n");
    if (off == 0 && c->spmeta.p) {  // bucket sizes (aggregator stamps)
        const uint32_t nwg = c->spill_nwg;
        const uint32_t nb = c->spill_nb;
        std::vector<uint32_t> cnt((size_t)2 * nb * nwg);
        hipMemcpy(cnt.data(), c->spmeta.p, cnt.size() * 4, hipMemcpyDeviceToHost);
        std::vector<uint64_t> tot(nb, 0);
        for (uint32_t b = 0; b < nb; b++)
            for (uint32_t g = 0; g < nwg; g++) tot[b] += cnt[(size_t)b * nwg + g] + cnt[(size_t)(nb + b) * nwg + g];
        std::vector<uint64_t> so(tot);
        std::sort(so.begin(), so.end());
        fprintf(stderr, "[mrg stamps]   bucket records min %llu p50 %llu max %llu; slowest buckets' records:",
                (unsigned long long)so[0], (unsigned long long)so[nb / 2], (unsigned long long)so.back());
        for (uint32_t k = 0; k < 5; k++) fprintf(stderr, " %llu", (unsigned long long)tot[ends[nblocks - 1 - k].second]);
        fprintf(stderr, "\n");
    }
}

// Stage 0 of the wc pipeline (mrgpu_wc.hip): the hottest keys of an evenly
// spaced sample of the split -> the dictionary image in c->dict.  Two levels:
// a small sample mapped with no dictionary (every word spills, so the hottest
// words crowd a few buckets — cheap only because the sample is small) gives a
// first dictionary; the full sample is then mapped WITH it, so only its tail
// spills, evenly over the buckets; its dictionary hits and aggregated tail
// become the records the final dictionary is built from.  Only speed depends
// on the dictionary: every key it misses is counted exactly through the spill.
// keep_if (warm start): the map's counters are read first and *kept set when
// keep_if(hit fraction) holds; the sample's aggregation, only needed to build a
// new dictionary, is then skipped (~45 us per split).
static int sample_pass(mrg_ctx* c, const uint8_t* in, uint64_t len, uint64_t win, uint32_t nwin, LetterTables lt,
                       bool with_dict, uint64_t* nrec_out, double* spill_rate = nullptr, const uint8_t* host = nullptr,
                       double* hit_frac = nullptr, const std::function<bool(double)>* keep_if = nullptr,
                       bool* kept = nullptr) {
    const uint64_t stride = ((len - win) / nwin) & ~15ull;
    const uint64_t sn = (uint64_t)nwin * (win + 16);
    HCHK(c, c->sample.ensure(sn + 64));
    if (host) {  // host input still in flight: the same sample bytes, gathered on the host
        if (c->h_sample_cap < sn) {
            if (c->h_sample) hipHostFree(c->h_sample);
            c->h_sample = nullptr;
            c->h_sample_cap = 0;
            HCHK(c, hipHostMalloc((void**)&c->h_sample, sn, hipHostMallocDefault));
            c->h_sample_cap = sn;
        }
        for (uint32_t w = 0; w < nwin; w++) {  // window w, then 16 '\n' (sample_gather_kernel's layout)
            memcpy(c->h_sample + w * (win + 16), host + w * stride, win);
            memset(c->h_sample + w * (win + 16) + win, '\n', 16);
        }
        HCHK(c, hipMemcpyAsync(c->sample.p, c->h_sample, sn, hipMemcpyHostToDevice, c->s));
    } else {
        launch_sample_gather(in, len, win, stride, nwin, (uint8_t*)c->sample.p, c->s);
    }
    int rc;
    if ((rc = ensure_tables(c)) || (rc = ensure_recbuf(c))) return rc;
    Tables t = make_tables(c);
    t.out = rec_view(c);
    t.out_cap = c->rec_cap;
    t.dict = with_dict ? (const uint4*)c->dict.p : nullptr;
    t.hi_staged = with_dict && c->dict_mini ? 1u : 0u;  // (a mini image is built only for 2048-bucket splits)
    clear_for_run(c, t);
    // the spill layout was sized for the split's workgroup count (ensure_spill): never launch more
    const uint32_t g = wc_map_grid(sn, (int)c->spill_nwg);
    if (!launch_wc_map((const uint8_t*)c->sample.p, sn, t, lt, (int)g, 0, c->s)) return fail(c, MRG_EINVAL, "sample too large");
    if (keep_if) {  // the map's counters decide whether the aggregation is needed at all
        HCHK(c, hipGetLastError());
        if ((rc = read_counters(c))) return rc;
        const double words = (double)(c->h_ctr->dict_hits + c->h_ctr->spilled + c->h_ctr->spill_ovf);
        const double frac = words > 0 ? (double)c->h_ctr->dict_hits / words : 0.0;
        if (spill_rate) *spill_rate = (double)(c->h_ctr->spilled + c->h_ctr->spill_ovf) / (double)sn;
        if (hit_frac) *hit_frac = frac;
        *kept = (*keep_if)(frac);
        if (*kept) {
            *nrec_out = 0;
            return MRG_OK;
        }
    }
    launch_wc_agg(t, c->map_mode & 512, 2, false, c->s);
    if (with_dict) launch_dict_emit(t, g, c->s);
    HCHK(c, hipGetLastError());
    print_stamps(c, with_dict ? "sample agg (level 2)" : "sample agg (level 1)", c->spill_nb);
    if ((rc = read_counters(c))) return rc;
    *nrec_out = std::min<uint64_t>(c->h_ctr->nrec, c->rec_cap);
    if (spill_rate) *spill_rate = (double)(c->h_ctr->spilled + c->h_ctr->spill_ovf) / (double)sn;
    if (hit_frac) {
        const double words = (double)(c->h_ctr->dict_hits + c->h_ctr->spilled + c->h_ctr->spill_ovf);
        *hit_frac = words > 0 ? (double)c->h_ctr->dict_hits / words : 0.0;
    }
    return MRG_OK;
}

// Dictionary image from the nrec records in the record buffer (descending count),
// in the mini geometry (DictMini) or the full one.
static int dict_from_recs(mrg_ctx* c, uint64_t nrec, bool mini) {
    const uint64_t cand_bytes = 4ull * kDictSlots * sizeof(uint4);
    HCHK(c, c->sortbuf.ensure(nrec * 16 + cand_bytes + 64));
    uint4* cand = (uint4*)c->sortbuf.p;
    uint32_t* keys = (uint32_t*)((char*)c->sortbuf.p + cand_bytes);
    uint32_t* keys2 = keys + nrec;
    uint32_t* idx = keys2 + nrec;
    uint32_t* idx2 = idx + nrec;
    Recs r = rec_view(c);
    r.n = nrec;
    launch_dict_keys(r, keys, idx, c->s);
    if (sort_u32_pairs(c->rws, keys, keys2, idx, idx2, nrec, 16, c->s))
        return fail(c, MRG_EDEVICE, "dictionary sort failed");
    launch_dict_build(r, idx2, nrec, cand, (uint4*)c->dict.p, mini, c->s);
    HCHK(c, hipGetLastError());
    c->dict_mini = mini;
    return MRG_OK;
}

// mini: the final image in the mini geometry (the staged 2048-bucket map); the
// sample passes map with whatever geometry c->dict has (the level-1 image is
// always full).
static int build_dict(mrg_ctx* c, const uint8_t* in, uint64_t len, LetterTables lt, bool* have, bool mini,
                      const uint8_t* host = nullptr) {
    *have = false;
    uint64_t win = 256u << 10;
    if (len < 2 * win) win = (len / 2) & ~15ull;
    if (win < 4096) return MRG_OK;
    HCHK(c, c->dict.ensure(sizeof(uint4) * kDictSets));
    const uint64_t target = std::min<uint64_t>(c->dict_sample_bytes, std::max<uint64_t>(len / 64, 4u << 20));
    const uint64_t small = std::min<uint64_t>(target, 2u << 20);
    int rc;
    uint64_t nrec = 0;
    // Warm start: a context that already built a dictionary (its previous map
    // task) maps the full sample with that one instead of first building a
    // level-1 dictionary from a small sample.  The final dictionary still comes
    // from this split's own sample; only speed depends on either.
    const bool warm = c->dict_warm && c->dict_valid && target > small && c->dict_mini == mini;
    if (!warm) {
        if ((rc = sample_pass(c, in, len, win, (uint32_t)std::max<uint64_t>(1, small / win), lt, false, &nrec, nullptr,
                              host)))
            return rc;
        if (nrec == 0) return MRG_OK;
        if ((rc = dict_from_recs(c, nrec, target > small ? false : mini))) return rc;
    }
    c->dict_fresh = true;
    if (target > small) {
        double rate = 0, frac = 0;
        // a warm dictionary that still hits this split's sample about as well as it
        // hit its own split is kept: the sample's aggregation, the candidate sort
        // and the placement are skipped (or within half a point of it: the mini
        // dictionary hits ~13 % of C5's words, where 3 % relative is sample noise
        // and a rebuild costs ~1 ms)
        const bool may_keep = warm && c->dict_keep > 0 && c->dict_frac_built > 0;
        const std::function<bool(double)> keep_if = [&](double f) {
            return f >= c->dict_keep * c->dict_frac_built || f >= c->dict_frac_built - 0.005;
        };
        bool keep = false;
        if ((rc = sample_pass(c, in, len, win, (uint32_t)std::max<uint64_t>(1, target / win), lt, true, &nrec, &rate,
                              host, &frac, may_keep ? &keep_if : nullptr, &keep)))
            return rc;
        c->dict_fresh = !keep;
        if (!keep && nrec && (rc = dict_from_recs(c, nrec, mini))) return rc;
        // Spill streams hold 0.094 8-byte records per input byte at scale 1 (C2
        // spills 0.04).  A split whose sample misses its (first-level) dictionary
        // more often gets proportionally longer streams, 30 % over the estimate
        // (the final dictionary only hits more).  Never shrinks within a context.
        // (The staged map's streams are sized from the previous split's words
        // instead, wc_map: its sample rate, measured with the mini dictionary over
        // windows that may hold a file's vocabulary-first region, overestimated it
        // and regrew a ~100 GB pool mid-run: 3.5 s.)
        const double need = 1.3 * rate / (2.0 * 0.75 / 16.0);
        if (!mini && need > c->spill_scale) c->spill_scale = std::min(need, 8.0);
    }
    c->stats.dict_keys = nrec;
    c->dict_valid = true;
    *have = true;
    return MRG_OK;
}

// Bucket aggregation in rounds.  Round 0 reads the map's spill streams; the
// keys a bucket's LDS tables cannot hold go to per-(bucket, wave) miss segments,
// which are the next round's input (a fresh table per bucket and round).  The
// last round (c->agg_rounds, or the first with nothing carried) counts the rest
// in the HBM table.  Typical splits finish in round 0; 1e7-key splits need a
// few rounds, each re-reading only the keys still unsettled.
static int aggregate_rounds(mrg_ctx* c, Tables& t) {
    const uint64_t E = (uint64_t)c->spill_nb * kAggSegs;
    const size_t meta = 2 * E * 4 + 2 * (E + 1) * 8 + 2 * (2 * E * 4) + 64;
    HCHK(c, c->segmeta.ensure(meta));
    uint32_t* tmp = (uint32_t*)c->segmeta.p;
    uint64_t* off8 = (uint64_t*)(tmp + 2 * E);
    uint64_t* off16 = off8 + E + 1;
    uint32_t* cnt[2] = {(uint32_t*)(off16 + E + 1), (uint32_t*)(off16 + E + 1) + 2 * E};
    launch_seg_layout(t, tmp, off8, off16, c->s);
    // The segment buffers hold every record a round may carry (the records round
    // 0 reads).  Sized from this split's totals with a host read the first time
    // (or after a miss overflowed them: kStSegFull, the run repeats); later splits
    // reuse them unread (a worker's map tasks are alike) and the aggregator
    // checks each miss against the capacity.
    if (c->seg_sync || !c->seg8[0].p || !c->seg16[0].p) {
        uint64_t* tot = c->h_scr;  // pinned
        HCHK(c, hipMemcpyAsync(&tot[0], off8 + E, 8, hipMemcpyDeviceToHost, c->s));
        HCHK(c, hipMemcpyAsync(&tot[1], off16 + E, 8, hipMemcpyDeviceToHost, c->s));
        HCHK(c, hipStreamSynchronize(c->s));
        for (int i = 0; i < 2; i++) {
            HCHK(c, c->seg8[i].ensure_grow(tot[0] * 8 + 64));
            HCHK(c, c->seg16[i].ensure_grow(tot[1] * 16 + 64));
        }
        c->seg_sync = false;
    }
    t.sp.seg8_cap = std::min(c->seg8[0].cap, c->seg8[1].cap) / 8;
    t.sp.seg16_cap = std::min(c->seg16[0].cap, c->seg16[1].cap) / 16;
    t.sp.seg_off8 = off8;
    t.sp.seg_off16 = off16;
    const int rounds = std::max(1, c->agg_rounds);
    int r = 0;
    for (;; r++) {
        const int o = r & 1, p = o ^ 1;
        t.sp.round = (uint32_t)r;
        t.sp.last = r + 1 >= rounds;
        t.sp.seg_n_in = cnt[p];
        t.sp.seg_n_out = cnt[o];
        t.sp.seg8_in = (const uint64_t*)c->seg8[p].p;
        t.sp.seg8_out = (uint64_t*)c->seg8[o].p;
        t.sp.seg16_in = (const uint4*)c->seg16[p].p;
        t.sp.seg16_out = (uint4*)c->seg16[o].p;
        if (c->debug_times) {
            HCHK(c, hipMemsetAsync(&t.ctr->carried, 0, 8, c->s));
            HCHK(c, hipEventRecord(c->ev[11], c->s));
        }
        const bool big0 = c->agg_big0 > 0 || (c->agg_big0 == 0 && c->spill_nb != kSpillBuckets);
        launch_wc_agg(t, c->map_mode, 1, r > 0 ? c->agg_big_later : big0, c->s);
        HCHK(c, hipGetLastError());
        if (c->debug_times) {  // diagnostics: per-round time and carried misses
            HCHK(c, hipEventRecord(c->ev[5], c->s));
            HCHK(c, hipMemcpyAsync(&c->h_scr[3], &t.ctr->carried, 8, hipMemcpyDeviceToHost, c->s));
            HCHK(c, hipStreamSynchronize(c->s));
            fprintf(stderr, "[mrg rounds] round %d: %.3f ms, carried %llu\n", r, ev_ms(c->ev[11], c->ev[5]),
                    (unsigned long long)c->h_scr[3]);
        }
        // Every round is launched without a host check: a later round's
        // workgroups exit at once when their bucket carried nothing (~4 us per
        // empty round), cheaper than reading the carried count between rounds
        // (a host round trip: ~45 us in C2's step).
        if (t.sp.last) break;
    }
    t.sp.round = 0;
    t.sp.last = 1;
    return MRG_OK;
}

// ---------------------------------------------------------------- streamed ingest
// A host-input split is copied to the staging buffer in pieces by a helper
// thread (copy stream, one event per piece) while this thread launches the map
// over each piece as soon as the piece and the next one (the chunk windows'
// 64-byte look-ahead) are resident.  Pieces are multiples of both map chunk
// sizes, so the chunk grid — and every result — is that of one whole-split map.
struct Ingest {
    mrg_ctx* c = nullptr;
    std::thread th;
    std::atomic<int> recorded{0};  // events recorded so far
    std::atomic<int> err{0};
    uint64_t piece = 0;
    int npieces = 0;
    ~Ingest() {  // every early return still joins the copy thread
        if (th.joinable()) th.join();
    }
};

static int ingest_start(mrg_ctx* c, Ingest& g, const uint8_t* host, uint8_t* dev, uint64_t len) {
    constexpr uint64_t kUnit = 29760;  // lcm(kWcChunkBytes, kGrepChunkBytes)
    static_assert(kUnit % kWcChunkBytes == 0 && kUnit % kGrepChunkBytes == 0, "piece unit");
    g.c = c;
    g.piece = std::max<uint64_t>(kUnit, c->ingest_piece / kUnit * kUnit);
    g.npieces = (int)((len + g.piece - 1) / g.piece);
    if (!c->cs) HCHK(c, hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking));
    while ((int)c->piece_ev.size() < g.npieces) {
        hipEvent_t e;
        HCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->piece_ev.push_back(e);
    }
    const int dev_id = c->device;
    hipStream_t cs = c->cs;
    hipEvent_t* ev = c->piece_ev.data();
    g.th = std::thread([&g, host, dev, len, dev_id, cs, ev]() {
        if (hipSetDevice(dev_id) != hipSuccess) g.err = 1;
        for (int k = 0; k < g.npieces && !g.err; k++) {
            const uint64_t off = (uint64_t)k * g.piece, n = std::min<uint64_t>(g.piece, len - off);
            if (hipMemcpyAsync(dev + off, host + off, n, hipMemcpyHostToDevice, cs) != hipSuccess ||
                hipEventRecord(ev[k], cs) != hipSuccess)
                g.err = 1;
            g.recorded.store(k + 1);
        }
        g.recorded.store(g.npieces);
    });
    return MRG_OK;
}

// Make c->s wait until pieces [0, k] are resident; false on a copy error.
static bool ingest_wait(Ingest& g, int k) {
    while (g.recorded.load() <= k) std::this_thread::sleep_for(std::chrono::microseconds(20));
    if (g.err) return false;
    return hipStreamWaitEvent(g.c->s, g.c->piece_ev[k], 0) == hipSuccess;
}

static int ingest_finish(mrg_ctx* c, Ingest& g) {
    if (g.th.joinable()) g.th.join();
    if (g.err) return fail(c, MRG_EDEVICE, "host input copy failed");
    return MRG_OK;
}

// Map chunk range [b, e) of piece-aligned host input: launch(cb, ce, resume)
// per piece once the piece and its successor are resident.
template <class F>
static int ingest_map(mrg_ctx* c, Ingest& g, uint64_t chunk_bytes, uint64_t len, F launch) {
    const uint64_t per = g.piece / chunk_bytes;  // chunks per piece
    const uint64_t nch = (len + chunk_bytes - 1) / chunk_bytes;
    for (int k = 0; k < g.npieces; k++) {
        if (!ingest_wait(g, std::min(k + 1, g.npieces - 1))) {
            ingest_finish(c, g);
            return fail(c, MRG_EDEVICE, "host input copy failed");
        }
        const uint64_t cb = (uint64_t)k * per, ce = std::min<uint64_t>(nch, cb + per);
        if (!launch(cb, ce, k > 0)) {
            ingest_finish(c, g);
            return fail(c, MRG_EINVAL, "split too large for 32-bit chunk indices (%llu bytes)", (unsigned long long)len);
        }
    }
    return ingest_finish(c, g);
}

// wc: dictionary, map, bucket aggregation, dictionary records, long words, collect.
static int wc_map(mrg_ctx* c, const uint8_t* in, uint64_t len, uint32_t nreduce, LetterTables lt, mrg_parts** out,
                  const uint8_t* host = nullptr) {
    int rc;
    const auto t_call = std::chrono::steady_clock::now();  // (MRG_DEBUG_TIMES diagnostics)
    auto mark = [&](const char* what) {
        if (c->debug_times)
            fprintf(stderr, "[mrg wc] %s: %.3f ms since the call\n", what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count());
    };
    c->lo_log2_cur = c->lo_log2;
    c->spill_nb = c->spill_buckets_opt ? (uint32_t)c->spill_buckets_opt : c->next_nb;
    if (c->spill_alt) std::swap(c->spool.p, c->spool_alt.p), std::swap(c->spool.cap, c->spool_alt.cap);
    Ingest ing;
    if (host && (rc = ingest_start(c, ing, host, (uint8_t*)in, len))) return rc;
    const bool staged = c->spill_nb == kSpillBucketsHi && c->hi_stage;  // (its kernel has the mini dictionary)
    // The staged 2048-bucket map's streams are sized from the previous split (a
    // worker's map tasks are alike), 30 % over: its spill records per byte if it
    // ran staged too, else its words per byte (as if every word spilled: the mini
    // dictionary takes few).  Set before the pool is sized, so it grows at most
    // once; the sample's rate (measured with the level-1 dictionary) is not used.
    if (staged) {
        const double est = c->prev_staged ? c->spilled_per_byte : c->words_per_byte;
        const double need = 1.3 * est / (2.0 * 0.75 / 16.0);
        if (need > c->spill_scale) c->spill_scale = std::min(need, 8.0);
        if (c->debug_times)
            fprintf(stderr, "[mrg spill] staged sizing: %s %.4f per byte -> scale %.3f\n",
                    c->prev_staged ? "spilled" : "words", est, c->spill_scale);
    }
    if ((rc = ensure_spill(c, len))) return rc;
    const uint32_t nwg = c->spill_nwg;
    HCHK(c, c->dict_cnt.ensure((size_t)nwg * kDictSlots * sizeof(uint32_t)));
    HCHK(c, hipEventRecord(c->ev[9], c->s));
    bool have_dict = false;
    if (c->dict_mode >= 0 && len >= c->dict_min_bytes && (rc = build_dict(c, in, len, lt, &have_dict, staged, host))) {
        ingest_finish(c, ing);
        return rc;
    }
    mark("dictionary");
    // the sample may have raised spill_scale: size the streams for this split now,
    // not only from the next call on (overflowing streams merge through HBM: slow)
    if ((rc = ensure_spill(c, len))) {
        ingest_finish(c, ing);
        return rc;
    }
    HCHK(c, hipEventRecord(c->ev[10], c->s));
    mark("spill layout");
    for (int attempt = 0; attempt < 8; attempt++) {
        c->lo_log2 = std::max(c->lo_log2, c->lo_log2_cur);  // long words: the grown size sticks for later wc maps
        if ((rc = ensure_tables(c)) || (rc = ensure_recbuf(c))) {
            ingest_finish(c, ing);
            return rc;
        }
        Tables t = make_tables(c);
        t.dict = have_dict ? (const uint4*)c->dict.p : nullptr;
        t.hi_staged = staged ? 1u : 0u;
        t.lean = c->lean_on && c->prev_ascii ? 1u : 0u;
        t.nreduce = nreduce;
        t.out = rec_view(c);
        t.out_cap = c->rec_cap;
        // The 17-32-byte key records: every map wave gets a region of lrec_cap
        // records.  Their total is capped (lrec_bytes_cap: the split's size, at least
        // 256 MiB); past it, or when the allocation fails, the records are turned off
        // for the context and every long word takes the start-offset list (the same
        // counts, more work for wc_long_kernel) instead of failing the map.
        if (c->lrec_on) {
            const uint64_t want = (uint64_t)nwg * kWavesPerWG * c->lrec_cap * 32;
            if (want > lrec_bytes_cap(len) || want / 32 >= (1ull << 32) ||  // (record indices are 32-bit)
                c->lrec.ensure_grow(want) != hipSuccess ||
                c->lrec_cnt.ensure((size_t)kMaxMapWGs * kWavesPerWG * 4) != hipSuccess ||
                c->lrec_aux.ensure_grow(kLrecAuxOff + want / 8 + want / 32 + kLrecPartBytes) != hipSuccess) {
                (void)hipGetLastError();  // (a failed allocation leaves no sticky error to report later)
                c->lrec_on = false;
            }
        }
        if (c->lrec_on) {
            t.lrec = (uint4*)c->lrec.p;
            t.lrec_cnt = (uint32_t*)c->lrec_cnt.p;
            t.lrec_cap = c->lrec_cap;
            t.lrec_off = (uint32_t*)c->lrec_aux.p;
            t.lrec_idx = (uint32_t*)((char*)c->lrec_aux.p + kLrecAuxOff);
            t.lrec_bkt = (uint8_t*)(t.lrec_idx + (uint64_t)nwg * kWavesPerWG * c->lrec_cap);  // (a byte per record after the indices)
            // the partials after the indices (the buffer only grows: the current capacity's end)
            t.lrec_part = (LrecPart*)(((uintptr_t)c->lrec_aux.p + c->lrec_aux.cap - kLrecPartBytes + 255) & ~(uintptr_t)255);
            t.lrec_pcnt = (uint32_t*)(t.lrec_part + 512ull * 4096);
        }
        clear_for_run(c, t);
        mark("tables");
        HCHK(c, hipEventRecord(c->ev[0], c->s));
        if (ing.npieces && attempt == 0) {  // the first pass runs while the host input streams in
            rc = ingest_map(c, ing, kWcChunkBytes, len, [&](uint64_t cb, uint64_t ce, bool resume) {
                return launch_wc_map(in, len, t, lt, c->grid, c->map_mode, c->s, cb, ce, resume);
            });
            if (rc) return rc;
        } else if (!launch_wc_map(in, len, t, lt, c->grid, c->map_mode, c->s)) {
            ingest_finish(c, ing);
            return fail(c, MRG_EINVAL, "split too large for 32-bit chunk indices (%llu bytes)", (unsigned long long)len);
        }
        HCHK(c, hipEventRecord(c->ev[1], c->s));
        print_stamps(c, "map", nwg, c->spill_nb);
        if ((rc = aggregate_rounds(c, t))) return rc;
        print_stamps(c, "agg", c->spill_nb);
        if (have_dict) launch_dict_emit(t, nwg, c->s);
        HCHK(c, hipEventRecord(c->ev[8], c->s));
        HCHK(c, hipGetLastError());
        // Words > 16 bytes, then the HBM tables' keys (aggregator leftovers, long
        // words) appended to the records, every count read on the device; one host
        // read of the counters afterwards checks every capacity (an overflow grows
        // what filled up and repeats the attempt).
        launch_wc_long(in, len, t, lt, ~0ull, c->s);
        launch_wc_lrec(t, nwg, c->s);
        HCHK(c, hipGetLastError());
        HCHK(c, hipEventRecord(c->ev[2], c->s));
        // the arena (long keys' bytes) sized from the previous split's long keys
        // (parts adopt the context's arena, so each split starts with a fresh one)
        if (c->arena_hint + 16 > c->recarena.cap) {
            HCHK(c, c->recarena.ensure_cached(c->arena_hint + 16, c->device));
            t.out = rec_view(c);
        }
        if (launch_collect(t, c->lo_log2_cur > 0, c->s)) return fail(c, MRG_EDEVICE, "collect failed");
        mark("launched");
        if ((rc = read_counters(c))) return rc;
        Counters h = *c->h_ctr;
        if (c->debug_times)
            fprintf(stderr, "[mrg wc] attempt %d: status %#x, %.3f ms since the call; nrec %llu, spilled %llu, ovf %llu, "
                    "dict hits %llu, buckets %u, staged %d, dict %d, long records past the LDS table %llu\n", attempt, h.status,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count(),
                    (unsigned long long)h.nrec, (unsigned long long)h.spilled, (unsigned long long)h.spill_ovf,
                    (unsigned long long)h.dict_hits, c->spill_nb, (int)staged, (int)have_dict, (unsigned long long)h.lds_miss);
        if (h.status & kStSpin) return fail(c, MRG_EDEVICE, "hash table publish timed out (status %#x)", h.status);
        if ((h.status & kStRecFull) && h.long_bytes + 16 > c->recarena.cap && h.nrec <= c->rec_cap) {
            // only the arena was short: grow it and run the collect again (not the map)
            HCHK(c, c->recarena.ensure_cached(h.long_bytes + 16, c->device));
            t.out = rec_view(c);
            launch_collect_undo(t, c->s);
            if (launch_collect(t, c->lo_log2_cur > 0, c->s)) return fail(c, MRG_EDEVICE, "collect failed");
            if ((rc = read_counters(c))) return rc;
            h = *c->h_ctr;
        }
        c->arena_hint = h.long_bytes + h.long_bytes / 4;
        if (len) {
            c->words_per_byte = (double)(h.dict_hits + h.spilled + h.spill_ovf) / (double)len;
            c->spilled_per_byte = (double)(h.spilled + h.spill_ovf) / (double)len;
            c->prev_staged = staged;
            c->prev_ascii = h.chunks_utf8 == 0;
        }
        if (h.status & kStLrecFull) {  // a record region filled up: size them for this split's busiest workgroup
            std::vector<uint32_t> cnt((size_t)nwg * kWavesPerWG);
            HCHK(c, hipMemcpy(cnt.data(), c->lrec_cnt.p, cnt.size() * 4, hipMemcpyDeviceToHost));
            const uint32_t mx = *std::max_element(cnt.begin(), cnt.end());
            const uint64_t want = std::max<uint64_t>((uint64_t)mx + mx / 4 + 1024, 2ull * c->lrec_cap);
            // (every wave's region is sized for the busiest one: a split dense in
            // 17-32-byte words would need regions past lrec_bytes_cap; the offset list
            // then takes every long word, for the rest of the context)
            if (want > (1u << 20) || (uint64_t)nwg * kWavesPerWG * want * 32 > lrec_bytes_cap(len)) c->lrec_on = false;
            else c->lrec_cap = (uint32_t)want;
        }
        if (grow_on_overflow(c, h.status & (kStListFull | kStShortFull | kStLongFull | kStRecFull | kStSegFull)) ||
            (h.status & kStLrecFull))
            continue;
        {
            // Bucket count for the next split (a worker's map tasks are alike):
            // the aggregated keys (records minus the dictionary's) against what
            // 512 buckets' round-0 tables hold (AggLdsBig: ~8 K short + 2 K mid
            // keys each), with hysteresis.
            const uint64_t agg_keys = h.nrec > (uint64_t)kDictSlots ? h.nrec - kDictSlots : 0;
            if (agg_keys > c->spill_hi_keys) c->next_nb = kSpillBucketsHi;
            else if (agg_keys < c->spill_hi_keys / 3 * 2) c->next_nb = kSpillBucketsLo;
            // switching to the staged map: size its pool now (this split's words per
            // byte, as the next call would), so the next split does not pay the
            // reallocation (~2.4 s for C5's ~100 GB pool)
            if (c->next_nb == kSpillBucketsHi && c->hi_stage && !staged && !c->spill_buckets_opt && len) {
                const double need = 1.3 * c->words_per_byte / (2.0 * 0.75 / 16.0);
                if (need > c->spill_scale) c->spill_scale = std::min(need, 8.0);
                const uint32_t nb_now = c->spill_nb;
                c->spill_nb = kSpillBucketsHi;
                rc = ensure_spill(c, len);
                c->spill_nb = nb_now;
                if (rc) return rc;
            }
        }
        // the parts object takes over the record buffer and arena (no copy); the
        // next map task gets cached blocks
        mrg_parts* p = new mrg_parts();
        p->app = MRG_APP_WC;
        p->nreduce = nreduce;
        p->device = c->device;
        p->ascii = h.chunks_utf8 == 0;
        p->r = t.out;
        p->r.n = h.nrec;
        p->r.arena_n = h.long_bytes;
        p->block = c->recbuf.adopt(&p->block_bytes);
        p->arena = (uint8_t*)c->recarena.adopt(&p->arena_bytes);
        HCHK(c, hipEventRecord(c->ev[3], c->s));
        HCHK(c, hipEventSynchronize(c->ev[3]));
        c->stats.map_kernel_ms = ev_ms(c->ev[0], c->ev[1]);
        c->stats.map_total_ms = ev_ms(c->ev[9], c->ev[3]);
        c->stats.dict_ms = ev_ms(c->ev[9], c->ev[10]);
        c->stats.agg_ms = ev_ms(c->ev[1], c->ev[8]);
        c->stats.long_ms = ev_ms(c->ev[8], c->ev[2]);
        c->stats.collect_ms = ev_ms(c->ev[2], c->ev[3]);
        c->stats.lds_overflow = h.spilled + h.spill_ovf;
        c->stats.spill_ovf = h.spill_ovf;
        c->stats.spill_record_bytes = 8 * (h.spilled - h.spilled16) + 16 * h.spilled16;
        c->stats.agg_miss = h.agg_miss;
        c->stats.agg_rounds = (uint64_t)__builtin_popcountll(h.round_mask);
        c->stats.spill_buckets = c->spill_nb;
        c->stats.dict_hits = h.dict_hits;
        if (have_dict && c->dict_fresh) {  // what this split's own dictionary hit (dictionary reuse, build_dict)
            const double words = (double)(h.dict_hits + h.spilled + h.spill_ovf);
            c->dict_frac_built = words > 0 ? (double)h.dict_hits / words : 0.0;
        }
        c->stats.distinct_keys = h.nrec;
        c->stats.long_keys = h.nlong_rec;
        *out = p;
        return MRG_OK;
    }
    return fail(c, MRG_ENOMEM, "mrg_map: tables kept overflowing");
}

// Go's utf8.Valid (the acceptance ranges of SURVEY.md Appendix A.1).
static bool go_valid_utf8(const uint8_t* p, size_t n) {
    for (size_t i = 0; i < n;) {
        const uint8_t c0 = p[i];
        if (c0 < 0x80) { i++; continue; }
        size_t need;
        uint8_t lo = 0x80, hi = 0xBF;
        if (c0 >= 0xC2 && c0 <= 0xDF) need = 1;
        else if (c0 >= 0xE0 && c0 <= 0xEF) { need = 2; if (c0 == 0xE0) lo = 0xA0; else if (c0 == 0xED) hi = 0x9F; }
        else if (c0 >= 0xF0 && c0 <= 0xF4) { need = 3; if (c0 == 0xF0) lo = 0x90; else if (c0 == 0xF4) hi = 0x8F; }
        else return false;
        if (i + need >= n) return false;  // truncated sequence
        if (p[i + 1] < lo || p[i + 1] > hi) return false;
        for (size_t k = 2; k <= need; k++)
            if ((p[i + k] & 0xC0) != 0x80) return false;
        i += need + 1;
    }
    return true;
}

// grep map (mrapps/dgrep.go:18-36) with a literal pattern:
//   grep_map_kernel -> occurrence positions (one per line per chunk) ->
//   grep_resolve_kernel (+ _long) -> one (start, end) per matching line
//   occurrence -> the LongTable sized for them, whose insert writes each
//   distinct line's record (option grep_emit = 0: a collect pass instead;
//   option grep_sort_hits = 1: the hits sorted by position first).
// The pattern is a literal (regexp.QuoteMeta semantics).  dgrep.go:20-23 returns
// no lines when regexp.Compile fails, which for a quoted literal happens exactly
// when it is not valid UTF-8; a pattern holding '\n' matches no line of
// strings.Split(contents, "\n") (dgrep.go:26).
static int grep_map(mrg_ctx* c, const uint8_t* in, uint64_t len, const uint8_t* pat, size_t plen, uint32_t nreduce,
                    mrg_parts** out, const uint8_t* host = nullptr) {
    int rc;
    if (!go_valid_utf8(pat, plen) || (plen && memchr(pat, '\n', plen))) {
        if (host) HCHK(c, hipMemcpyAsync((void*)in, host, len, hipMemcpyHostToDevice, c->s));  // no map: plain copy
        HCHK(c, hipEventRecord(c->ev[0], c->s));
        if ((rc = parts_alloc(c, 0, 0, MRG_APP_GREP, nreduce, out))) return rc;
        c->stats.distinct_keys = 0;
        return MRG_OK;
    }
    HCHK(c, c->pat.ensure(plen + 16));
    if (plen) HCHK(c, hipMemcpyAsync(c->pat.p, pat, plen, hipMemcpyHostToDevice, c->s));
    c->lo_log2_cur = 14;
    // grep_map_kernel's 32-bit chunk indices (with the grid's stride on top)
    if (len / kGrepChunkBytes + 2 * (uint64_t)c->grid * 16 + 16 >= (1ull << 32))
        return fail(c, MRG_EINVAL, "split too large for 32-bit chunk indices (%llu bytes)", (unsigned long long)len);
    Ingest ing;
    if (host && plen && (rc = ingest_start(c, ing, host, (uint8_t*)in, len))) return rc;
    if (host && !plen) HCHK(c, hipMemcpyAsync((void*)in, host, len, hipMemcpyHostToDevice, c->s));
    for (int attempt = 0; attempt < 8; attempt++) {
        if ((rc = ensure_tables(c))) {
            ingest_finish(c, ing);
            return rc;
        }
        Tables t = make_tables(c);
        clear_for_run(c, t);
        HCHK(c, hipEventRecord(c->ev[0], c->s));
        if (plen && ing.npieces && attempt == 0) {  // the first pass runs while the host input streams in
            rc = ingest_map(c, ing, kGrepChunkBytes, len, [&](uint64_t cb, uint64_t ce, bool) {
                launch_grep_map(in, len, (const uint8_t*)c->pat.p, (uint32_t)plen, t, c->grid, c->s, cb, ce);
                return true;
            });
            if (rc) return rc;
        } else if (plen) {
            launch_grep_map(in, len, (const uint8_t*)c->pat.p, (uint32_t)plen, t, c->grid, c->s);
        } else {
            launch_grep_all_lines(in, len, t, c->grid, c->s);
        }
        HCHK(c, hipGetLastError());
        HCHK(c, hipEventRecord(c->ev[1], c->s));
        // Unsorted hits (default): the line resolution follows the map kernel with
        // no host read in between (it reads the hit counts on the device, over
        // buffers sized for the list's capacity); the one counter read after it
        // also tells whether the map's list overflowed (then everything repeats
        // with a larger list).  Sorted (option grep_sort_hits): the sort needs the
        // count on the host first.
        const bool sorted = c->grep_sort_hits, dev = !sorted;
        if (sorted) {
            if ((rc = read_counters(c))) return rc;
            if (grow_on_overflow(c, c->h_ctr->status & kStListFull)) continue;
        }
        const uint64_t nhits = dev ? c->list_cap : c->h_ctr->nlist;
        if (sorted) HCHK(c, c->ghits.ensure_grow(nhits * 8 + 64));
        HCHK(c, c->glines.ensure_grow(nhits * 16 + 64));
        HCHK(c, c->gdefer.ensure_grow(nhits * 8 + 64));
        t = make_tables(c);
        if (sorted) {
            unsigned bits = 1;
            while (bits < 64 && (len >> bits) != 0) bits++;
            if (nhits && sort_u64_keys(c->rws, t.list, (uint64_t*)c->ghits.p, nhits, bits, c->s))
                return fail(c, MRG_EDEVICE, "grep: hit sort failed");
        } else {
            t.hits = t.list;  // the map kernel's order (grep_resolve_kernel: unsorted)
        }
        launch_grep_resolve(in, len, (const uint8_t*)c->pat.p, (uint32_t)plen, t, nhits, dev, sorted, c->s);
        if (dev) launch_grep_resolve_long(in, len, (const uint8_t*)c->pat.p, (uint32_t)plen, t, 0, nhits, true, false, c->s);
        HCHK(c, hipGetLastError());
        // emit (default): the insert writes each distinct line's record as it
        // claims the line's slot, into parts sized for every occurrence (records
        // <= lines, arena <= the lines' bytes); option grep_emit = 0: insert,
        // then collect the table (round 4).
        const bool emit = c->grep_emit;
        // Speculative sizes (unsorted hits, emit, a previous split mapped on this
        // context): the parts (records for the list's capacity, arena for the
        // previous split's line bytes + 25 %) and the LongTable (for its lines +
        // 25 %) are set up with no host read after the resolution, whose line
        // count the insert reads on the device; the one read after the insert
        // checks every bound, and an overflow repeats with the exact sizes.
        bool spec = dev && emit && c->grep_hint_lines > 0;
        uint64_t cap_lines, cap_bytes, want_lines;
        if (spec) {
            cap_lines = nhits;  // (the list's capacity: lines <= hits)
            cap_bytes = c->grep_hint_bytes + c->grep_hint_bytes / 4 + (1u << 20);
            want_lines = c->grep_hint_lines + c->grep_hint_lines / 4;
        } else {
            if ((rc = read_counters(c))) return rc;
            if (dev && grow_on_overflow(c, c->h_ctr->status & kStListFull)) continue;
            if (sorted && c->h_ctr->ndefer) {
                launch_grep_resolve_long(in, len, (const uint8_t*)c->pat.p, (uint32_t)plen, t, c->h_ctr->ndefer, nhits, false,
                                         true, c->s);
                HCHK(c, hipGetLastError());
                if ((rc = read_counters(c))) return rc;
            }
            if (c->h_ctr->status & kStListFull) return fail(c, MRG_EDEVICE, "grep: line list overflow");
            cap_lines = want_lines = c->h_ctr->nlines;
            cap_bytes = c->h_ctr->line_bytes;
        }
        HCHK(c, hipEventRecord(c->ev[8], c->s));
        // The LongTable holds at most nlines distinct lines: size it for them
        // (capped; a table that still fills up grows, and only the inserts re-run).
        int need = 14;
        while (need < 24 && (1ull << need) * 7 < want_lines * 10) need++;
        c->lo_log2_cur = need;
        mrg_parts* p = nullptr;
        if (emit && (rc = parts_alloc(c, cap_lines, cap_bytes, MRG_APP_GREP, nreduce, &p))) return rc;
        bool ok = false, again = false;
        for (int grow = 0; grow < 8 && !ok; grow++) {
            if ((rc = ensure_tables(c))) { if (p) mrg_parts_free(p); return rc; }
            t = make_tables(c);
            if (emit) {
                t.out = p->r;
                t.out_cap = cap_lines;
                t.nreduce = nreduce;
            }
            clear_long_table(t, c->s);
            launch_grep_insert(in, t, cap_lines, spec, emit, c->s);
            if (hipGetLastError() != hipSuccess) {
                if (p) mrg_parts_free(p);
                return fail(c, MRG_EDEVICE, "grep: line table insert launch");
            }
            if (c->debug_times && t.dbg) print_insert_stamps(c);
            if ((rc = read_counters(c))) { if (p) mrg_parts_free(p); return rc; }
            const uint32_t st = c->h_ctr->status;
            if (spec && (st & kStListFull)) {  // the map's hit list overflowed: the whole attempt again
                if (p) mrg_parts_free(p);
                grow_on_overflow(c, kStListFull);
                again = true;
                break;
            }
            if (st & kStSpin) {
                if (p) mrg_parts_free(p);
                return fail(c, MRG_EDEVICE, "grep: line table insert failed (status %#x)", st);
            }
            if (st & kStRecFull) {
                if (!spec || c->h_ctr->line_bytes <= cap_bytes) {
                    if (p) mrg_parts_free(p);
                    return fail(c, MRG_EDEVICE, "grep: line records overflow (status %#x)", st);
                }
                // the speculative arena was short: parts for the exact line bytes, insert again
                mrg_parts_free(p);
                p = nullptr;
                cap_bytes = c->h_ctr->line_bytes;
                if ((rc = parts_alloc(c, cap_lines, cap_bytes, MRG_APP_GREP, nreduce, &p))) return rc;
                continue;
            }
            if (st & kStLongFull) c->lo_log2_cur += 2;
            else ok = true;
        }
        if (again) continue;
        if (!ok) { if (p) mrg_parts_free(p); return fail(c, MRG_ENOMEM, "grep: line table kept overflowing"); }
        const uint64_t nlines = c->h_ctr->nlines;
        c->grep_hint_lines = nlines;
        c->grep_hint_bytes = c->h_ctr->line_bytes;
        HCHK(c, hipEventRecord(c->ev[2], c->s));
        c->stats.map_kernel_ms = ev_ms(c->ev[0], c->ev[1]);
        if (emit) {
            const Counters& h = *c->h_ctr;
            if (h.nrec != h.long_used || h.arena != h.long_bytes || h.nrec > nlines) {
                mrg_parts_free(p);
                return fail(c, MRG_EDEVICE, "grep: emitted %llu records / %llu bytes for %llu lines / %llu bytes",
                            h.nrec, h.arena, h.long_used, h.long_bytes);
            }
            p->r.n = h.nrec;
            p->r.arena_n = h.arena;
            c->stats.distinct_keys = h.nrec;
            c->stats.long_keys = h.nrec;
        } else if ((rc = collect_parts(c, MRG_APP_GREP, nreduce, &p))) {
            return rc;
        }
        HCHK(c, hipEventRecord(c->ev[3], c->s));
        HCHK(c, hipEventSynchronize(c->ev[3]));
        c->stats.map_total_ms = ev_ms(c->ev[0], c->ev[3]);
        c->stats.agg_ms = ev_ms(c->ev[1], c->ev[8]);
        c->stats.long_ms = ev_ms(c->ev[8], c->ev[2]);
        c->stats.collect_ms = ev_ms(c->ev[2], c->ev[3]);
        *out = p;
        return MRG_OK;
    }
    return fail(c, MRG_ENOMEM, "mrg_map: tables kept overflowing");
}

// ---------------------------------------------------------------- C ABI
extern "C" {

int mrg_device_count(int* n) {
    int k = 0;
    if (hipGetDeviceCount(&k) != hipSuccess) k = 0;
    *n = k;
    return MRG_OK;
}

int mrg_open(int device, mrg_ctx** out) {
    if (!out) return MRG_EINVAL;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MRG_EDEVICE;
    if (device < 0 || device >= ndev) return MRG_EINVAL;
    mrg_ctx* c = new mrg_ctx();
    c->device = device;
    int rc;
    if ((rc = bind(c))) { delete c; return rc; }
    if (hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) != hipSuccess) { delete c; return MRG_EDEVICE; }
    for (auto& e : c->ev) hipEventCreate(&e);
    if (hipMalloc((void**)&c->d_l1, sizeof(mrg_letter_l1_init)) != hipSuccess ||
        hipMalloc((void**)&c->d_l2, sizeof(mrg_letter_l2_init)) != hipSuccess) {
        mrg_close(c);
        return MRG_ENOMEM;
    }
    hipMemcpy(c->d_l1, mrg_letter_l1_init, sizeof(mrg_letter_l1_init), hipMemcpyHostToDevice);
    hipMemcpy(c->d_l2, mrg_letter_l2_init, sizeof(mrg_letter_l2_init), hipMemcpyHostToDevice);
    {  // the 2-byte runes' letters as one 2048-bit table (the map kernels' one-read lookup)
        uint32_t b2[64] = {};
        for (uint32_t cp = 0; cp < 2048; cp++)
            if ((mrg_letter_l2_init[mrg_letter_l1_init[cp >> 8] * 8u + ((cp >> 5) & 7u)] >> (cp & 31u)) & 1u)
                b2[cp >> 5] |= 1u << (cp & 31u);
        if (hipMalloc((void**)&c->d_b2, sizeof(b2)) != hipSuccess) {
            mrg_close(c);
            return MRG_ENOMEM;
        }
        hipMemcpy(c->d_b2, b2, sizeof(b2), hipMemcpyHostToDevice);
    }
    if (hipHostMalloc((void**)&c->h_ctr, sizeof(Counters), hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&c->h_scr, 8 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess) {
        mrg_close(c);
        return MRG_ENOMEM;
    }
    c->grid = map_grid_size(device);
    c->rws = reduce_ws_new();
    *out = c;
    return MRG_OK;
}

void mrg_close(mrg_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    if (c->s) hipStreamSynchronize(c->s);
    if (c->comm) ncclCommDestroy(c->comm);
    DevBuf* bs[] = {&c->sh, &c->shl, &c->lo, &c->list, &c->ctr, &c->staging, &c->pat, &c->spool, &c->spool_alt, &c->spmeta,
                    &c->bflag, &c->dict, &c->dict_cnt, &c->sample, &c->recbuf, &c->recarena, &c->sortbuf,
                    &c->segmeta, &c->seg8[0], &c->seg8[1], &c->seg16[0], &c->seg16[1], &c->lrec, &c->lrec_cnt, &c->lrec_aux};
    for (DevBuf* b : bs) b->release();
    if (c->d_l1) hipFree(c->d_l1);
    if (c->d_l2) hipFree(c->d_l2);
    if (c->d_b2) hipFree(c->d_b2);
    if (c->h_ctr) hipHostFree(c->h_ctr);
    if (c->h_scr) hipHostFree(c->h_scr);
    if (c->h_out) hipHostFree(c->h_out);
    for (auto& j : c->aj) {
        if (j.done) hipEventSynchronize(j.done);
        if (j.host) hipHostFree(j.host);
        if (j.start) hipEventDestroy(j.start);
        if (j.done) hipEventDestroy(j.done);
    }
    if (c->os) hipStreamDestroy(c->os);
    if (c->h_sample) hipHostFree(c->h_sample);
    for (hipEvent_t e : c->piece_ev) hipEventDestroy(e);
    if (c->cs) hipStreamDestroy(c->cs);
    reduce_ws_free(c->rws);
    for (auto& e : c->ev)
        if (e) hipEventDestroy(e);
    if (c->s) hipStreamDestroy(c->s);
    exch_free(c->exch);
    delete c;
}

const char* mrg_last_error(const mrg_ctx* c) { return c ? c->err.c_str() : "null context"; }

int mrg_set_option(mrg_ctx* c, const char* name, int64_t v) {
    if (!c || !name) return MRG_EINVAL;
    if (!strcmp(name, "short_table_log2")) c->sh_log2 = v > 0 ? (int)v : 20;
    else if (!strcmp(name, "long_table_log2")) c->lo_log2 = c->lo_log2_cur = v > 0 ? (int)v : 14;
    else if (!strcmp(name, "list_cap")) c->list_cap = v > 0 ? (uint64_t)v : (1u << 20);
    else if (!strcmp(name, "map_grid")) c->grid = v > 0 ? (int)v : map_grid_size(c->device);
    else if (!strcmp(name, "map_mode")) c->map_mode = (int)v;
    else if (!strcmp(name, "spill_stream_keys")) c->spill_force_sub = v > 0 ? v : 0;
    else if (!strcmp(name, "spill_mid_div")) c->spill_mid_div = v > 0 ? (int)v : 2;
    else if (!strcmp(name, "spill_alt_pools")) c->spill_alt = v > 0;  // diagnostic: two pools, alternating per split
    else if (!strcmp(name, "agg_rounds")) c->agg_rounds = v > 0 ? (int)v : 8;
    else if (!strcmp(name, "agg_big_later")) c->agg_big_later = v >= 0;  // -1: off
    else if (!strcmp(name, "agg_big0")) c->agg_big0 = v > 0 ? 1 : v < 0 ? -1 : 0;  // 0: by layout
    else if (!strcmp(name, "agg_carry_min")) c->agg_carry_min = v > 0 ? (uint32_t)v : v < 0 ? 0u : 64u;  // -1: always carry
    else if (!strcmp(name, "dict")) c->dict_mode = (int)v;
    else if (!strcmp(name, "dict_warm")) c->dict_warm = v >= 0;  // -1: always build the level-1 dictionary
    else if (!strcmp(name, "dict_keep")) c->dict_keep = v > 0 ? (double)v / 1000.0 : v < 0 ? 0.0 : 0.97;  // permille; -1: never
    else if (!strcmp(name, "spill_buckets")) {  // 0: chosen per split (feedback), else 256, 512 or 2048
        if (v != 0 && v != kSpillBuckets && v != kSpillBucketsHi && v != kSpillBucketsLo)
            return fail(c, MRG_EINVAL, "spill_buckets: 0, 256, 512 or 2048");
        c->spill_buckets_opt = (int)v;
    } else if (!strcmp(name, "sort_digit_bits")) {  // radix passes: 8 (0) or 10 bits per digit
        reduce_ws_set(c->rws, (int)v, -1, -1);
    } else if (!strcmp(name, "sort_fold_part")) {  // partition folded into the k0 sort key (-1: off)
        reduce_ws_set(c->rws, 0, v >= 0 ? 1 : 0, -1);
    } else if (!strcmp(name, "sort_compact_ties")) {  // tied runs merge-sorted on key copies (-1: on the records)
        reduce_ws_set_compact_ties(c->rws, v >= 0);
    } else if (!strcmp(name, "grep_emit")) {  // 0: insert the lines, then collect the LongTable (round-4 path)
        c->grep_emit = v >= 0 ? v != 0 : true;
    } else if (!strcmp(name, "grep_sort_hits")) {  // 1: the position sort before line resolution (round-4 path)
        c->grep_sort_hits = v > 0;
    } else if (!strcmp(name, "out_direct")) {  // mrg_run_job: lines into pinned host memory (default), via a copy (-1), wc only (1)
        c->out_direct = v >= 0;
        c->out_direct_grep = v >= 0 && v != 1;
    } else if (!strcmp(name, "hi_stage")) {  // 2048-bucket splits: mini dictionary + LDS write-combined spill (default) or not (-1)
        c->hi_stage = v >= 0;
    } else if (!strcmp(name, "async_direct_max")) {  // bytes (0: default 64 MB; -1: every async wc output copied)
        c->async_direct_max = v > 0 ? (uint64_t)v : v < 0 ? 0ull : (64ull << 20);
    } else if (!strcmp(name, "map_lean")) {  // wc: the all-ASCII map variant after an all-ASCII split (default) or never (-1)
        c->lean_on = v >= 0;
    } else if (!strcmp(name, "long_records")) {  // wc: words of 17-32 bytes as key records (default) or offsets (-1)
        c->lrec_on = v >= 0;
    } else if (!strcmp(name, "lrec_cap")) {  // records per map workgroup region (tests of the overflow path)
        c->lrec_cap = v > 0 ? (uint32_t)std::min<int64_t>(v, 1 << 22) : 1024u;
    } else if (!strcmp(name, "grep_literal")) {  // grep: metacharacters quoted (1) instead of refused (0)
        c->grep_literal = v > 0;
    } else if (!strcmp(name, "grep_bins")) {  // grep reduce path (include/mrgpu.h)
        reduce_ws_set_grep_bins(c->rws, (int)v);
    } else if (!strcmp(name, "tie_rank")) {  // grep reduce: tied runs ranked per run (1, default) or merge-sorted (0)
        reduce_ws_set_tie_rank(c->rws, v != 0);
    } else if (!strcmp(name, "own_sort")) {  // (compatibility: every sort is the hand-written one since round 5)
        reduce_ws_set_own_sort(c->rws, v != 0);
    } else if (!strcmp(name, "sort_prefix32")) {  // wc reduce: single pass on the top 32 key bits (1, default) or all (0)
        reduce_ws_set_prefix32(c->rws, v != 0);
    } else if (!strcmp(name, "sort_bins")) {  // wc reduce: hand-written sample sort (1) or the radix passes (0, -1: default)
        reduce_ws_set_bin_sort(c->rws, v > 0);
    } else if (!strcmp(name, "grep_sort_k1")) {  // grep radix over 16 key bytes (default) or 8 (-1)
        reduce_ws_set(c->rws, 0, -1, v >= 0 ? 1 : 0);
    } else if (!strcmp(name, "spill_hi_keys")) c->spill_hi_keys = v > 0 ? (uint64_t)v : 6000ull * kSpillBuckets;
    else if (!strcmp(name, "dict_min_bytes")) c->dict_min_bytes = v > 0 ? (uint64_t)v : (32ull << 20);
    else if (!strcmp(name, "dict_sample_bytes")) c->dict_sample_bytes = v > 0 ? (uint64_t)v : (16ull << 20);
    else if (!strcmp(name, "rec_cap")) c->rec_cap = v > 0 ? (uint64_t)v : (1u << 21);
    else if (!strcmp(name, "skip_exchange")) c->skip_exchange = v > 0;
    else if (!strcmp(name, "exch_force_rccl")) c->exch_force_rccl = v > 0;
    else if (!strcmp(name, "exchange_timeout_ms")) c->exch_timeout_ms = v > 0 ? v : 120000;
    else if (!strcmp(name, "ingest_piece")) c->ingest_piece = v > 0 ? (uint64_t)v : (256ull << 20);
    else if (!strcmp(name, "ingest_min")) c->ingest_min = v > 0 ? (uint64_t)v : (64ull << 20);
    else return fail(c, MRG_EINVAL, "unknown option %s", name);
    return MRG_OK;
}

uint32_t mrg_ihash(const uint8_t* key, size_t n) {
    uint32_t h = 2166136261u;
    for (size_t i = 0; i < n; i++) h = fnv1a32_step(h, key[i]);
    return h & 0x7fffffffu;
}

void mrg_free(void* p) {
    if (!p) return;
    uint64_t* hdr = (uint64_t*)p - 2;
    if (hdr[0] == kHostMagic) {
        hdr[0] = 0;
        free(hdr);
    }
}

static void* host_result(size_t n) {
    uint64_t* hdr = (uint64_t*)malloc(n + 16);
    if (!hdr) return nullptr;
    hdr[0] = kHostMagic;
    hdr[1] = n;
    return hdr + 2;
}

int mrg_device_alloc(mrg_ctx* c, size_t n, void** d) {
    if (!c || !d) return MRG_EINVAL;
    int rc;
    if ((rc = bind(c))) return rc;
    HCHK(c, hipMalloc(d, n ? n : 16));
    return MRG_OK;
}
int mrg_device_free(mrg_ctx* c, void* d) {
    if (!c) return MRG_EINVAL;
    int rc;
    if ((rc = bind(c))) return rc;
    HCHK(c, hipFree(d));
    return MRG_OK;
}
int mrg_memcpy_h2d(mrg_ctx* c, void* dst, const void* src, size_t n) {
    int rc;
    if ((rc = bind(c))) return rc;
    HCHK(c, hipMemcpy(dst, src, n, hipMemcpyHostToDevice));
    return MRG_OK;
}
int mrg_sort_pairs(mrg_ctx* c, void* keys, void* vals, size_t n, int key_bytes, unsigned bits) {
    if (!c || (n && !keys)) return MRG_EINVAL;
    int rc;
    if ((rc = bind(c))) return rc;
    if (n > 0xFFFFFFFFull) return fail(c, MRG_EINVAL, "mrg_sort_pairs: at most 2^32 - 1 keys");
    const int e = sort_in_place(c->rws, key_bytes, keys, (uint32_t*)vals, n, bits, c->s);
    if (e == (int)hipErrorInvalidValue) return fail(c, MRG_EINVAL, "mrg_sort_pairs: key_bytes 4 or 8; 4-byte keys need values");
    if (e) return fail(c, MRG_EDEVICE, "mrg_sort_pairs: %s", hipGetErrorString((hipError_t)e));
    return MRG_OK;
}

int mrg_memcpy_d2h(mrg_ctx* c, void* dst, const void* src, size_t n) {
    int rc;
    if ((rc = bind(c))) return rc;
    HCHK(c, hipMemcpy(dst, src, n, hipMemcpyDeviceToHost));
    return MRG_OK;
}
int mrg_sync(mrg_ctx* c) {
    int rc;
    if ((rc = bind(c))) return rc;
    HCHK(c, hipStreamSynchronize(c->s));
    HCHK(c, hipDeviceSynchronize());
    return MRG_OK;
}
int mrg_get_stats(const mrg_ctx* c, mrg_stats* out) {
    if (!c || !out) return MRG_EINVAL;
    *out = c->stats;
    return MRG_OK;
}

int mrg_map(mrg_ctx* c, int app, const void* buf, size_t len, int kind, const uint8_t* pat, size_t plen,
            uint32_t nreduce, mrg_parts** out) {
    if (!c || !out || (len && !buf) || nreduce == 0 || (app != MRG_APP_WC && app != MRG_APP_GREP))
        return c ? fail(c, MRG_EINVAL, "mrg_map: bad arguments") : MRG_EINVAL;
    if (app == MRG_APP_GREP && plen && !pat) return fail(c, MRG_EINVAL, "mrg_map: null pattern");
    // dgrep.go:20 compiles the pattern as a regexp; this path matches literals
    // only.  A valid-UTF-8 pattern holding a metacharacter would silently match
    // differently, so it is refused unless the caller asks for QuoteMeta
    // semantics (option grep_literal).  Invalid UTF-8 keeps dgrep.go:20-23's
    // behaviour (regexp.Compile fails: no lines).
    if (app == MRG_APP_GREP && !c->grep_literal && go_valid_utf8(pat, plen)) {
        for (size_t i = 0; i < plen; i++)
            if (pat[i] < 0x80 && strchr("\\.+*?()|[]{}^$", (char)pat[i]) && pat[i] != 0)
                return fail(c, MRG_EINVAL,
                            "mrg_map: grep pattern holds the regexp metacharacter '%c' (dgrep.go:20 compiles a "
                            "regexp; this path matches literals: set option grep_literal=1 for QuoteMeta semantics)",
                            (char)pat[i]);
    }
    *out = nullptr;
    int rc;
    if ((rc = bind(c))) return rc;
    c->stats = mrg_stats{};
    c->stats.input_bytes = len;
    const uint8_t* in = (const uint8_t*)buf;
    const uint8_t* host = nullptr;  // host input streamed in pieces, overlapped with the map
    if (kind == MRG_INPUT_HOST || (((uintptr_t)buf) & 15)) {
        HCHK(c, c->staging.ensure(len + 64));
        if (kind == MRG_INPUT_HOST && len >= c->ingest_min) host = (const uint8_t*)buf;
        else HCHK(c, hipMemcpyAsync(c->staging.p, buf, len, kind == MRG_INPUT_HOST ? hipMemcpyHostToDevice
                                                                                 : hipMemcpyDeviceToDevice, c->s));
        in = (const uint8_t*)c->staging.p;
        c->stats.staged_bytes = len;
    }
    LetterTables lt{c->d_l1, c->d_l2, c->d_b2};
    if (app == MRG_APP_WC) return wc_map(c, in, len, nreduce, lt, out, host);
    return grep_map(c, in, len, pat, plen, nreduce, out, host);
}

void mrg_parts_free(mrg_parts* p) {
    if (!p) return;
    hipSetDevice(p->device);
    cache_put(p->device, p->block, p->block_bytes);
    cache_put(p->device, p->arena, p->arena_bytes);
    delete p;
}

int mrg_parts_info(const mrg_parts* p, uint64_t* nkeys, uint32_t* nreduce, int* app) {
    if (!p) return MRG_EINVAL;
    if (nkeys) *nkeys = p->r.n;
    if (nreduce) *nreduce = p->nreduce;
    if (app) *app = p->app;
    return MRG_OK;
}

// Aggregate several record sets into one parts object (exact, by key).
static int aggregate(mrg_ctx* c, const std::vector<Recs>& srcs, int app, uint32_t nreduce, mrg_parts** out) {
    int rc;
    uint64_t tot = 0, longs = 0;
    for (const Recs& r : srcs) { tot += r.n; longs += r.n; }
    while ((1ull << c->sh_log2) < tot * 2) c->sh_log2++;
    c->lo_log2_cur = 14;
    while ((1ull << c->lo_log2_cur) < longs / 4 + 1024 && c->lo_log2_cur < 20) c->lo_log2_cur++;
    for (int attempt = 0; attempt < 8; attempt++) {
        if ((rc = ensure_tables(c))) return rc;
        Tables t = make_tables(c);
        clear_for_run(c, t);
        for (const Recs& r : srcs) launch_insert_recs(r, t, c->s);
        HCHK(c, hipGetLastError());
        if ((rc = read_counters(c))) return rc;
        uint32_t st = c->h_ctr->status;
        if (st & kStSpin) return fail(c, MRG_EDEVICE, "hash table publish timed out");
        if (grow_on_overflow(c, st)) continue;
        return collect_parts(c, app, nreduce, out);
    }
    return fail(c, MRG_ENOMEM, "aggregate: tables kept overflowing");
}

int mrg_parts_merge(mrg_ctx* c, mrg_parts* into, const mrg_parts* from) {
    if (!c || !into || !from) return MRG_EINVAL;
    if (into->app != from->app || into->nreduce != from->nreduce) return fail(c, MRG_EINVAL, "merge: app/nreduce mismatch");
    int rc;
    if ((rc = bind(c))) return rc;
    mrg_parts* m = nullptr;
    if ((rc = aggregate(c, {into->r, from->r}, into->app, into->nreduce, &m))) return rc;
    // aggregate() has synchronized the stream: into's old blocks are idle
    cache_put(into->device, into->block, into->block_bytes);
    cache_put(into->device, into->arena, into->arena_bytes);
    into->block = m->block;
    into->block_bytes = m->block_bytes;
    into->arena = m->arena;
    into->arena_bytes = m->arena_bytes;
    into->r = m->r;
    into->ascii = into->ascii && from->ascii;
    m->block = nullptr;
    m->arena = nullptr;
    delete m;
    return MRG_OK;
}

// Intermediate format "MRGI": header {magic, app, nreduce, part, n, arena_n} then
// SoA k0[n] k1[n] cnt[n] koff[n] len[n] part[n], then arena bytes.
struct IHdr {
    uint32_t magic, app, nreduce, part;
    uint64_t n, arena_n;
};
constexpr uint32_t kIMagic = 0x4947524Du;  // "MRGI"

static int parts_to_host(mrg_ctx* c, const Recs& r, int app, uint32_t nreduce, uint32_t part, void** bytes, size_t* nb) {
    const uint64_t n = r.n;
    size_t sz = sizeof(IHdr) + n * (8 * 4 + 4 * 2) + r.arena_n;
    uint8_t* h = (uint8_t*)host_result(sz);
    if (!h) return fail(c, MRG_ENOMEM, "host alloc %zu", sz);
    IHdr hd{kIMagic, (uint32_t)app, nreduce, part, n, r.arena_n};
    memcpy(h, &hd, sizeof hd);
    uint8_t* o = h + sizeof hd;
    auto cp = [&](const void* d, size_t b) -> hipError_t {
        hipError_t e = b ? hipMemcpyAsync(o, d, b, hipMemcpyDeviceToHost, c->s) : hipSuccess;
        o += b;
        return e;
    };
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = cp(r.k0, n * 8);
    if (e == hipSuccess) e = cp(r.k1, n * 8);
    if (e == hipSuccess) e = cp(r.cnt, n * 8);
    if (e == hipSuccess) e = cp(r.koff, n * 8);
    if (e == hipSuccess) e = cp(r.len, n * 4);
    if (e == hipSuccess) e = cp(r.part, n * 4);
    if (e == hipSuccess) e = cp(r.arena, r.arena_n);
    if (e == hipSuccess) e = hipStreamSynchronize(c->s);
    if (e != hipSuccess) { mrg_free(h); return fail(c, MRG_EDEVICE, "export copy: %s", hipGetErrorString(e)); }
    *bytes = h;
    *nb = sz;
    return MRG_OK;
}

int mrg_parts_export(mrg_ctx* c, const mrg_parts* p, uint32_t r, void** bytes, size_t* nb) {
    if (!c || !p || !bytes || !nb) return MRG_EINVAL;
    int rc;
    if ((rc = bind(c))) return rc;
    if (r == 0xFFFFFFFFu) return parts_to_host(c, p->r, p->app, p->nreduce, r, bytes, nb);
    if (r >= p->nreduce) return fail(c, MRG_EINVAL, "export: partition %u >= nreduce %u", r, p->nreduce);
    mrg_parts* sel = nullptr;
    if ((rc = parts_alloc(c, p->r.n, 0, p->app, p->nreduce, &sel))) return rc;
    Recs d = sel->r;
    if ((rc = select_recs(c->rws, p->r, p->nreduce, r, &d, c->s))) { mrg_parts_free(sel); return fail(c, MRG_EDEVICE, "select failed"); }
    rc = parts_to_host(c, d, p->app, p->nreduce, r, bytes, nb);  // arena shared with p (whole arena exported)
    mrg_parts_free(sel);
    return rc;
}

// ---- reference-format intermediate files (mr/worker.go:80-92 / :100-122) ----
static void* json_grow(void* ctx, size_t n) {
    mrg_ctx* c = (mrg_ctx*)ctx;
    return c->jtmp.ensure_grow(n) == hipSuccess ? c->jtmp.p : nullptr;
}

int mrg_parts_export_json(mrg_ctx* c, const mrg_parts* p, uint32_t r, void** bytes, size_t* nb) {
    if (!c || !p || !bytes || !nb) return MRG_EINVAL;
    int rc;
    if ((rc = bind(c))) return rc;
    if (r != 0xFFFFFFFFu && r >= p->nreduce) return fail(c, MRG_EINVAL, "export_json: partition %u >= nreduce %u", r, p->nreduce);
    mrg_parts* sel = nullptr;
    Recs src = p->r;
    if (r != 0xFFFFFFFFu) {
        if ((rc = parts_alloc(c, p->r.n, 0, p->app, p->nreduce, &sel))) return rc;
        Recs d = sel->r;
        if (select_recs(c->rws, p->r, p->nreduce, r, &d, c->s)) { mrg_parts_free(sel); return fail(c, MRG_EDEVICE, "select failed"); }
        src = d;
    }
    const uint64_t n = src.n;
    uint64_t total = 0;
    uint8_t* h = nullptr;
    if (n) {
        hipError_t e = c->jmeta.ensure_grow(n * 6 * 8 + 64);
        if (e != hipSuccess) { mrg_parts_free(sel); return fail(c, MRG_ENOMEM, "export_json: scratch"); }
        uint64_t* L = (uint64_t*)c->jmeta.p;
        uint64_t *T = L + n, *P = T + n, *loff = P + n, *toff = loff + n, *poff = toff + n;
        if (json_lengths(src, p->app, L, T, P, loff, toff, poff, json_grow, c, c->s)) {
            mrg_parts_free(sel);
            return fail(c, MRG_EDEVICE, "export_json: lengths");
        }
        uint64_t* hs = c->h_scr;  // last entries of the three scans and of L, T, P
        const uint64_t* src6[6] = {loff + n - 1, L + n - 1, toff + n - 1, T + n - 1, poff + n - 1, P + n - 1};
        for (int i = 0; i < 6; i++) HCHK(c, hipMemcpyAsync(&hs[i], src6[i], 8, hipMemcpyDeviceToHost, c->s));
        HCHK(c, hipStreamSynchronize(c->s));
        const uint64_t nlines = hs[0] + hs[1];
        total = hs[2] + hs[3];
        const uint64_t npieces = hs[4] + hs[5];
        if (c->jlines.ensure_grow(nlines + 64) != hipSuccess || c->jout.ensure_grow(total + 64) != hipSuccess) {
            mrg_parts_free(sel);
            return fail(c, MRG_ENOMEM, "export_json: %llu output bytes", (unsigned long long)total);
        }
        if (json_write(src, p->app, L, loff, toff, poff, npieces, total, (uint8_t*)c->jlines.p, (uint8_t*)c->jout.p, c->s)) {
            mrg_parts_free(sel);
            return fail(c, MRG_EDEVICE, "export_json: write");
        }
    }
    h = (uint8_t*)host_result(total);
    if (!h) { mrg_parts_free(sel); return fail(c, MRG_ENOMEM, "host alloc %llu", (unsigned long long)total); }
    hipError_t e = total ? hipMemcpyAsync(h, c->jout.p, total, hipMemcpyDeviceToHost, c->s) : hipSuccess;
    if (e == hipSuccess) e = hipStreamSynchronize(c->s);
    mrg_parts_free(sel);
    if (e != hipSuccess) { mrg_free(h); return fail(c, MRG_EDEVICE, "export_json copy: %s", hipGetErrorString(e)); }
    *bytes = h;
    *nb = total;
    return MRG_OK;
}

// One JSON string at s[i] (after its opening quote) -> raw bytes, as Go's
// decoder unquotes it (encoding/json unquoteBytes): \uXXXX with UTF-16
// surrogate pairs, a lone surrogate -> U+FFFD.  Returns the index after the
// closing quote, or 0 on malformed input.
static size_t json_unquote(const uint8_t* s, size_t i, size_t n, std::string& out) {
    auto hex4 = [&](size_t at, uint32_t* v) -> bool {
        if (at + 4 > n) return false;
        uint32_t x = 0;
        for (size_t k = at; k < at + 4; k++) {
            const uint8_t ch = s[k];
            x <<= 4;
            if (ch >= '0' && ch <= '9') x |= ch - '0';
            else if (ch >= 'a' && ch <= 'f') x |= ch - 'a' + 10;
            else if (ch >= 'A' && ch <= 'F') x |= ch - 'A' + 10;
            else return false;
        }
        *v = x;
        return true;
    };
    auto put = [&](uint32_t cp) {
        if (cp < 0x80) out.push_back((char)cp);
        else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 63))); }
        else if (cp < 0x10000) {
            out.push_back((char)(0xE0 | (cp >> 12)));
            out.push_back((char)(0x80 | ((cp >> 6) & 63)));
            out.push_back((char)(0x80 | (cp & 63)));
        } else {
            out.push_back((char)(0xF0 | (cp >> 18)));
            out.push_back((char)(0x80 | ((cp >> 12) & 63)));
            out.push_back((char)(0x80 | ((cp >> 6) & 63)));
            out.push_back((char)(0x80 | (cp & 63)));
        }
    };
    while (i < n) {
        const uint8_t ch = s[i];
        if (ch == '"') return i + 1;
        if (ch != '\\') { out.push_back((char)ch); i++; continue; }
        if (i + 1 >= n) return 0;
        const uint8_t e = s[i + 1];
        i += 2;
        switch (e) {
            case '"': case '\\': case '/': out.push_back((char)e); break;
            case 'b': out.push_back('\b'); break;
            case 'f': out.push_back('\f'); break;
            case 'n': out.push_back('\n'); break;
            case 'r': out.push_back('\r'); break;
            case 't': out.push_back('\t'); break;
            case 'u': {
                uint32_t v;
                if (!hex4(i, &v)) return 0;
                i += 4;
                if (v >= 0xD800 && v < 0xDC00) {  // high surrogate: a low one must follow
                    uint32_t lo;
                    if (i + 6 <= n && s[i] == '\\' && s[i + 1] == 'u' && hex4(i + 2, &lo) && lo >= 0xDC00 && lo < 0xE000) {
                        i += 6;
                        v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
                    } else {
                        v = 0xFFFD;
                    }
                } else if (v >= 0xDC00 && v < 0xE000) {
                    v = 0xFFFD;
                }
                put(v);
                break;
            }
            default: return 0;
        }
    }
    return 0;
}

int mrg_parts_import_json(mrg_ctx* c, int app, uint32_t nreduce, const void* bytes, size_t nb, mrg_parts** out) {
    if (!c || !out || (nb && !bytes)) return MRG_EINVAL;
    if ((app != MRG_APP_WC && app != MRG_APP_GREP) || nreduce == 0) return fail(c, MRG_EINVAL, "import_json: app / nreduce");
    // Decode the lines on the host (the format is text with escapes), one record
    // per line with count 1, then count equal keys on the GPU (aggregate()).
    const uint8_t* s = (const uint8_t*)bytes;
    static const char kHead[] = "{\"Key\":\"";
    static const char kMid[] = ",\"Value\":\"";
    std::vector<uint64_t> k0, k1, koff, cnt;
    std::vector<uint32_t> len, part;
    std::string arena, key, val;
    size_t i = 0;
    while (i < nb) {
        if (nb - i < sizeof(kHead) - 1 || memcmp(s + i, kHead, sizeof(kHead) - 1)) return fail(c, MRG_EFORMAT, "import_json: line at byte %zu", i);
        key.clear();
        val.clear();
        size_t j = json_unquote(s, i + sizeof(kHead) - 1, nb, key);
        if (!j || nb - j < sizeof(kMid) - 1 || memcmp(s + j, kMid, sizeof(kMid) - 1)) return fail(c, MRG_EFORMAT, "import_json: key at byte %zu", i);
        j = json_unquote(s, j + sizeof(kMid) - 1, nb, val);
        if (!j || j + 2 > nb || s[j] != '}' || s[j + 1] != '\n') return fail(c, MRG_EFORMAT, "import_json: value at byte %zu", i);
        i = j + 2;
        if (key.size() > 0xFFFFFFFFu) return fail(c, MRG_EFORMAT, "import_json: key too long");
        uint64_t a = 0, b = 0;
        for (size_t q = 0; q < key.size() && q < 16; q++)
            (q < 8 ? a : b) |= (uint64_t)(uint8_t)key[q] << (8 * (q & 7));
        k0.push_back(a);
        k1.push_back(b);
        cnt.push_back(1);  // Reduce sees one value per line (worker.go:129-140)
        len.push_back((uint32_t)key.size());
        uint32_t h = 2166136261u;
        for (char ch : key) h = fnv1a32_step(h, (uint8_t)ch);
        part.push_back((h & 0x7fffffffu) % nreduce);
        if (key.size() > 16) {
            koff.push_back(arena.size());
            arena += key;
        } else {
            koff.push_back(~0ull);
        }
    }
    int rc;
    if ((rc = bind(c))) return rc;
    const uint64_t n = k0.size();
    mrg_parts* raw = nullptr;
    if ((rc = parts_alloc(c, n, arena.size(), app, nreduce, &raw))) return rc;
    hipError_t e = hipSuccess;
    auto cp = [&](void* d, const void* h, size_t b) {
        if (e == hipSuccess && b) e = hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, c->s);
    };
    cp(raw->r.k0, k0.data(), n * 8);
    cp(raw->r.k1, k1.data(), n * 8);
    cp(raw->r.cnt, cnt.data(), n * 8);
    cp(raw->r.koff, koff.data(), n * 8);
    cp(raw->r.len, len.data(), n * 4);
    cp(raw->r.part, part.data(), n * 4);
    cp(raw->r.arena, arena.data(), arena.size());
    if (e == hipSuccess) e = hipStreamSynchronize(c->s);  // the host vectors go out of scope
    if (e != hipSuccess) { mrg_parts_free(raw); return fail(c, MRG_EDEVICE, "import_json copy: %s", hipGetErrorString(e)); }
    rc = aggregate(c, {raw->r}, app, nreduce, out);
    mrg_parts_free(raw);
    return rc;
}

// Every record of an intermediate buffer must be one the map could have
// written: the reduce kernels index the arena and a 16-byte key buffer with
// these fields, and place records by `part`.  Returns nullptr or what is wrong.
static const char* validate_records(const IHdr& hd, const uint8_t* soa, uint64_t* bad) {
    const uint64_t n = hd.n;
    const uint8_t *pk0 = soa, *pk1 = pk0 + n * 8, *pcnt = pk1 + n * 8, *pkoff = pcnt + n * 8, *plen = pkoff + n * 8,
                  *ppart = plen + n * 4, *arena = ppart + n * 4;
    for (uint64_t i = 0; i < n; i++) {
        *bad = i;
        uint64_t k0, k1, cnt, koff;
        uint32_t len, part;
        memcpy(&k0, pk0 + 8 * i, 8);
        memcpy(&k1, pk1 + 8 * i, 8);
        memcpy(&cnt, pcnt + 8 * i, 8);
        memcpy(&koff, pkoff + 8 * i, 8);
        memcpy(&len, plen + 4 * i, 4);
        memcpy(&part, ppart + 4 * i, 4);
        if (part >= hd.nreduce) return "partition >= nreduce";
        if (cnt == 0) return "zero count";
        if (hd.app == MRG_APP_WC && len == 0) return "empty wc key";
        uint8_t inl[16];
        for (int k = 0; k < 8; k++) {
            inl[k] = (uint8_t)(k0 >> (8 * k));
            inl[8 + k] = (uint8_t)(k1 >> (8 * k));
        }
        const uint8_t* key = inl;
        if (koff == ~0ull) {
            if (len > 16) return "inline key longer than 16 bytes";
            for (uint32_t k = len; k < 16; k++)
                if (inl[k]) return "inline key bytes past its length";
        } else {
            if (koff > hd.arena_n || len > hd.arena_n - koff) return "key outside the arena";
            key = arena + koff;
            for (uint32_t k = 0; k < 16; k++)  // k0/k1 are the key's first 16 bytes, zero padded
                if (inl[k] != (k < len ? key[k] : 0)) return "prefix words differ from the arena key";
        }
        uint32_t h = 2166136261u;
        for (uint32_t k = 0; k < len; k++) h = fnv1a32_step(h, key[k]);
        if ((h & 0x7fffffffu) % hd.nreduce != part) return "partition differs from ihash(key) % nreduce";
    }
    return nullptr;
}

int mrg_parts_import(mrg_ctx* c, const void* bytes, size_t nb, mrg_parts** out) {
    if (!c || !bytes || !out || nb < sizeof(IHdr)) return c ? fail(c, MRG_EFORMAT, "import: short buffer") : MRG_EINVAL;
    IHdr hd;
    memcpy(&hd, bytes, sizeof hd);
    if (hd.magic != kIMagic || (hd.app != MRG_APP_WC && hd.app != MRG_APP_GREP) || hd.nreduce == 0)
        return fail(c, MRG_EFORMAT, "import: bad header");
    const uint64_t n = hd.n;
    if (n > (nb - sizeof(IHdr)) / 40 || hd.arena_n > nb || sizeof(IHdr) + n * 40 + hd.arena_n != nb)
        return fail(c, MRG_EFORMAT, "import: size mismatch");
    uint64_t bad = 0;
    if (const char* why = validate_records(hd, (const uint8_t*)bytes + sizeof(IHdr), &bad))
        return fail(c, MRG_EFORMAT, "import: record %llu: %s", (unsigned long long)bad, why);
    int rc;
    if ((rc = bind(c))) return rc;
    mrg_parts* p = nullptr;
    if ((rc = parts_alloc(c, n, hd.arena_n, (int)hd.app, hd.nreduce, &p))) return rc;
    const uint8_t* s = (const uint8_t*)bytes + sizeof hd;
    auto cp = [&](void* d, size_t b) -> hipError_t {
        hipError_t e = b ? hipMemcpyAsync(d, s, b, hipMemcpyHostToDevice, c->s) : hipSuccess;
        s += b;
        return e;
    };
    hipError_t e = cp(p->r.k0, n * 8);
    if (e == hipSuccess) e = cp(p->r.k1, n * 8);
    if (e == hipSuccess) e = cp(p->r.cnt, n * 8);
    if (e == hipSuccess) e = cp(p->r.koff, n * 8);
    if (e == hipSuccess) e = cp(p->r.len, n * 4);
    if (e == hipSuccess) e = cp(p->r.part, n * 4);
    if (e == hipSuccess) e = cp(p->r.arena, hd.arena_n);
    if (e == hipSuccess) e = hipStreamSynchronize(c->s);
    if (e != hipSuccess) { mrg_parts_free(p); return fail(c, MRG_EDEVICE, "import copy: %s", hipGetErrorString(e)); }
    *out = p;
    return MRG_OK;
}

// The output transfers of queued async jobs read the reduce's device buffer:
// they finish before another reduce may write (or reallocate) it.
static int drain_async(mrg_ctx* c) {
    for (int k = 0; k < c->aj_count; k++) HCHK(c, hipEventSynchronize(c->aj[(c->aj_head + k) & 1].done));
    return MRG_OK;
}

static int reduce_common(mrg_ctx* c, const mrg_parts* p, uint32_t only, uint8_t** d_out, uint64_t* n_out, uint64_t* offsets,
                         uint8_t* hout = nullptr, uint64_t hout_cap = 0) {
    int rc;
    if ((rc = bind(c)) || (rc = drain_async(c))) return rc;
    HCHK(c, hipEventRecord(c->ev[4], c->s));
    if (only == 0xFFFFFFFFu) {
        rc = reduce_format(c->rws, p->r, p->app, p->nreduce, only, d_out, n_out, offsets, c->s, p->ascii, hout, hout_cap);
        if (rc) return fail(c, MRG_EDEVICE, "reduce_format: %s", hipGetErrorString((hipError_t)rc));
    } else {
        mrg_parts* sel = nullptr;
        if ((rc = parts_alloc(c, p->r.n, 0, p->app, p->nreduce, &sel))) return rc;
        Recs d = sel->r;
        if (select_recs(c->rws, p->r, p->nreduce, only, &d, c->s)) { mrg_parts_free(sel); return fail(c, MRG_EDEVICE, "select"); }
        rc = reduce_format(c->rws, d, p->app, p->nreduce, only, d_out, n_out, offsets, c->s, p->ascii);
        HCHK(c, hipStreamSynchronize(c->s));
        mrg_parts_free(sel);
        if (rc) return fail(c, MRG_EDEVICE, "reduce_format: %s", hipGetErrorString((hipError_t)rc));
    }
    HCHK(c, hipEventRecord(c->ev[5], c->s));
    return MRG_OK;
}

int mrg_reduce(mrg_ctx* c, const mrg_parts* p, uint32_t r, void** bytes, size_t* nb) {
    if (!c || !p || !bytes || !nb) return MRG_EINVAL;
    if (r >= p->nreduce) return fail(c, MRG_EINVAL, "reduce: partition %u >= nreduce %u", r, p->nreduce);
    uint8_t* d = nullptr;
    uint64_t n = 0, offs[2];
    int rc = reduce_common(c, p, r, &d, &n, offs);
    if (rc) return rc;
    void* h = host_result(n);
    if (!h) return fail(c, MRG_ENOMEM, "host alloc");
    if (n) HCHK(c, hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
    *bytes = h;
    *nb = n;
    c->stats.output_bytes = n;
    return MRG_OK;
}

int mrg_reduce_all(mrg_ctx* c, const mrg_parts* p, void** bytes, size_t* nb, uint64_t* offsets) {
    if (!c || !p || !bytes || !nb || !offsets) return MRG_EINVAL;
    uint8_t* d = nullptr;
    uint64_t n = 0;
    int rc = reduce_common(c, p, 0xFFFFFFFFu, &d, &n, offsets);
    if (rc) return rc;
    void* h = host_result(n);
    if (!h) return fail(c, MRG_ENOMEM, "host alloc");
    if (n) HCHK(c, hipMemcpy(h, d, n, hipMemcpyDeviceToHost));
    *bytes = h;
    *nb = n;
    c->stats.output_bytes = n;
    c->stats.reduce_ms = ev_ms(c->ev[4], c->ev[5]);
    return MRG_OK;
}

// ---------------------------------------------------------------- RCCL shuffle
int mrg_comm_unique_id(uint8_t id[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return MRG_ECOMM;
    memcpy(id, &u, 128);
    return MRG_OK;
}

int mrg_comm_init(mrg_ctx* c, const uint8_t id[128], int nranks, int rank) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return MRG_EINVAL;
    int rc;
    if ((rc = bind(c))) return rc;
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    ncclUniqueId u;
    memcpy(&u, id, 128);
    c->wd.enter("ncclCommInitRank", 4 * c->exch_timeout_ms, rank, nranks);
    const ncclResult_t ir = ncclCommInitRank(&c->comm, nranks, u, rank);
    c->wd.leave();
    if (ir != ncclSuccess) return fail(c, MRG_ECOMM, "ncclCommInitRank: %s", ncclGetErrorString(ir));
    c->nranks = nranks;
    c->rank = rank;
    return MRG_OK;
}

// Wire record: the parts SoA of one destination, then its arena bytes.
// Records are routed to owner rank part % nranks.  Per-owner counts and slots
// come from LDS histograms, one device atomic per (workgroup, owner) per step:
// a same-address device atomic per record serializes at the memory side
// (~12 ns each, MI355X_MICROARCH.md fan-in row).  Arena bytes of a key are
// padded to 16 so every key starts 16-byte aligned on the wire and is copied by
// 16-byte stores.
constexpr uint32_t kExchMaxRanks = 1024;
constexpr int kExchThreads = 256;
__host__ __device__ __forceinline__ uint64_t pad16(uint64_t x) { return (x + 15) & ~15ull; }

__global__ void __launch_bounds__(kExchThreads) owner_count_kernel(Recs r, uint32_t nranks,
                                                                   unsigned long long* cnt /*[2*nranks]*/) {
    __shared__ unsigned long long h[2 * kExchMaxRanks];
    for (uint32_t i = threadIdx.x; i < 2 * nranks; i += blockDim.x) h[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.n; i += stride) {
        const uint32_t o = r.part[i] % nranks;
        atomicAdd(&h[2 * o], 1ull);
        if (r.koff[i] != ~0ull) atomicAdd(&h[2 * o + 1], (unsigned long long)pad16(r.len[i]));
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 2 * nranks; i += blockDim.x)
        if (h[i]) atomicAdd(&cnt[i], h[i]);
}

// Pack into per-destination segments: 24-byte wire records (mrgpu_exch.h) at
// rec_base[o], long keys' bytes at ar_base[o].
__global__ void __launch_bounds__(kExchThreads) pack_kernel(Recs r, uint32_t nranks, const uint64_t* rec_base,
                                                            const uint64_t* ar_base,
                                                            unsigned long long* cur /*[2*nranks]*/, WireRec* wrec,
                                                            uint8_t* war) {
    __shared__ unsigned long long h[2 * kExchMaxRanks];     // this step's records / arena bytes per owner
    __shared__ unsigned long long gbase[2 * kExchMaxRanks];  // their global slots
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 < r.n; b0 += stride) {
        for (uint32_t k = threadIdx.x; k < 2 * nranks; k += blockDim.x) h[k] = 0;
        __syncthreads();
        const uint64_t i = b0 + threadIdx.x;
        const bool valid = i < r.n;
        uint32_t o = 0;
        unsigned long long slot = 0, aoff = 0;
        uint64_t koff = ~0ull, alen = 0;
        if (valid) {
            o = r.part[i] % nranks;
            koff = r.koff[i];
            slot = atomicAdd(&h[2 * o], 1ull);
            if (koff != ~0ull) {
                alen = pad16(r.len[i]);
                aoff = atomicAdd(&h[2 * o + 1], (unsigned long long)alen);
            }
        }
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < 2 * nranks; k += blockDim.x) gbase[k] = h[k] ? atomicAdd(&cur[k], h[k]) : 0;
        __syncthreads();
        if (valid) {
            WireRec w{r.k0[i], r.k1[i], r.cnt[i]};
            if (koff != ~0ull) {
                const unsigned long long a = gbase[2 * o + 1] + aoff;  // relative to owner o's segment from this source
                uint4* dst = (uint4*)(war + ar_base[o] + a);           // 16-byte aligned (padded lengths)
                const uint8_t* src = r.arena + koff;
                const uint64_t len = r.len[i];
                for (uint64_t q = 0; q < len; q += 16) {
                    uint64_t lo, hi;
                    load16u(src + q, len - q, lo, hi);
                    dst[q >> 4] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
                }
                w = WireRec{a, len, r.cnt[i] | kWireLong};
            }
            wrec[rec_base[o] + gbase[2 * o] + slot] = w;
        }
        __syncthreads();  // h / gbase are reused by the next step
    }
}

// Unpack received wire records into the Recs the owner's aggregation reads
// (insert_recs: k0 / k1 / cnt of short keys, arena bytes / len / cnt of long
// ones; the partition is recomputed there from the key).  A long key's arena
// offset is rebased by its source's arena displacement (the source segment of
// record i by binary search over the P record offsets).
__global__ void unpack_kernel(const WireRec* wrec, uint64_t n, const uint64_t* src_rec_begin, const uint64_t* src_ar_begin,
                              uint32_t nsrc, Recs r) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const WireRec w = wrec[i];
        if (w.c & kWireLong) {
            uint32_t lo = 0, hi = nsrc - 1;  // last s with src_rec_begin[s] <= i
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) >> 1;
                if (src_rec_begin[mid] <= i) lo = mid;
                else hi = mid - 1;
            }
            r.k0[i] = 0;
            r.k1[i] = 0;
            r.cnt[i] = w.c & ~kWireLong;
            r.len[i] = (uint32_t)w.b;
            r.koff[i] = src_ar_begin[lo] + w.a;
        } else {
            r.k0[i] = w.a;
            r.k1[i] = w.b;
            r.cnt[i] = w.c;
            r.len[i] = key_len_short(w.a, w.b);
            r.koff[i] = ~0ull;
        }
        r.part[i] = 0;  // not read by the aggregation
    }
}

// Per-rank device state of one exchange.  scratch: [2P] send counts, [2P] receive
// counts, [2P] pack cursors, [2P] send bases.
struct ExchSide {
    DevBuf scratch, sbuf, sar_b, rbuf, rar_b, rmeta;
    std::vector<unsigned long long> snd, rcv;
    ExchPlan plan;
    unsigned long long* d_cnt(int) { return (unsigned long long*)scratch.p; }
    unsigned long long* d_rcv(int P) { return d_cnt(P) + 2 * P; }
    unsigned long long* d_cur(int P) { return d_cnt(P) + 4 * P; }
    uint64_t* d_base(int P) { return (uint64_t*)(d_cnt(P) + 6 * P); }
};

// Step 1: count records / arena bytes per owner rank (on the device, async).
static int exch_count(mrg_ctx* c, const Recs& r, int P, ExchSide& x) {
    size_t meta = sizeof(unsigned long long) * (8 * P + 8);
    HCHK(c, x.scratch.ensure(meta));
    HCHK(c, hipMemsetAsync(x.scratch.p, 0, meta, c->s));
    if (P > (int)kExchMaxRanks) return fail(c, MRG_EINVAL, "exchange: more than %u ranks", kExchMaxRanks);
    if (r.n) owner_count_kernel<<<1024, kExchThreads, 0, c->s>>>(r, (uint32_t)P, x.d_cnt(P));
    HCHK(c, hipGetLastError());
    return MRG_OK;
}

// Step 2 (x.snd / x.rcv known on the host): size the buffers and pack the
// per-owner segments.  Step 3 is the transport (RCCL or in-process copies).
static int exch_pack(mrg_ctx* c, const Recs& r, int P, ExchSide& x) {
    x.plan = exch_plan(P, x.snd.data(), x.rcv.data());
    HCHK(c, x.sbuf.ensure_grow(x.plan.srec * sizeof(WireRec) + 64));
    HCHK(c, x.rbuf.ensure_grow(x.plan.rrec * sizeof(WireRec) + 64));
    HCHK(c, x.sar_b.ensure_grow(x.plan.sar + 64));
    HCHK(c, x.rar_b.ensure_cached(x.plan.rar + 64, c->device));  // handed to the received parts object
    HCHK(c, hipMemcpyAsync(x.d_base(P), x.plan.hbase.data(), 16 * P, hipMemcpyHostToDevice, c->s));
    if (r.n)
        pack_kernel<<<1024, kExchThreads, 0, c->s>>>(r, (uint32_t)P, x.d_base(P), x.d_base(P) + P, x.d_cur(P),
                                             (WireRec*)x.sbuf.p, (uint8_t*)x.sar_b.p);
    HCHK(c, hipGetLastError());
    return MRG_OK;
}

// Step 4: unpack the received records into a Recs view and re-aggregate exactly.
static int exch_finish(mrg_ctx* c, const mrg_parts* local, int P, ExchSide& x, mrg_parts** owned,
                       hipEvent_t done = nullptr) {
    int rc;
    const ExchPlan& pl = x.plan;
    HCHK(c, hipEventRecord(c->ev[13], c->s));  // the owner's unpack + re-aggregation starts
    std::vector<uint64_t> hsrc(2 * P);
    for (int o = 0; o < P; o++) { hsrc[o] = pl.rd[o] / sizeof(WireRec); hsrc[P + o] = pl.ard[o]; }
    HCHK(c, x.rmeta.ensure(16 * P));
    HCHK(c, hipMemcpyAsync(x.rmeta.p, hsrc.data(), 16 * P, hipMemcpyHostToDevice, c->s));
    mrg_parts* tmp = nullptr;
    if ((rc = parts_alloc(c, pl.rrec, 0, local->app, local->nreduce, &tmp))) return rc;
    cache_put(c->device, tmp->arena, tmp->arena_bytes);  // nothing has used it yet
    tmp->arena = (uint8_t*)x.rar_b.adopt(&tmp->arena_bytes);  // adopt the received arena
    tmp->r.arena = tmp->arena;
    tmp->r.arena_n = pl.rar;
    if (pl.rrec)
        unpack_kernel<<<1024, 256, 0, c->s>>>((const WireRec*)x.rbuf.p, pl.rrec, (const uint64_t*)x.rmeta.p,
                                              (const uint64_t*)x.rmeta.p + P, (uint32_t)P, tmp->r);
    if (hipGetLastError() != hipSuccess) { mrg_parts_free(tmp); return fail(c, MRG_EDEVICE, "unpack launch"); }
    rc = aggregate(c, {tmp->r}, local->app, local->nreduce, owned);
    if (done) hipEventRecord(done, c->s);
    hipError_t e = hipStreamSynchronize(c->s);
    mrg_parts_free(tmp);
    if (rc) return rc;
    HCHK(c, e);
    return MRG_OK;
}

static void exch_free(ExchSide* x) { delete x; }

// Wire bytes to / from the OTHER ranks (the self segment is a local copy).
static void exch_bytes(const ExchPlan& pl, int P, int me, mrg_stats* st) {
    uint64_t snd = 0, rcv = 0;
    for (int o = 0; o < P; o++) {
        if (o == me) continue;
        snd += pl.sc[o] + pl.asc[o];
        rcv += pl.rc[o] + pl.arc[o];
    }
    st->shuffle_send_bytes = snd;
    st->shuffle_recv_bytes = rcv;
    st->shuffle_recv_records = pl.rrec;  // every rank's segment, this rank's own included
}

static int exchange_rccl(mrg_ctx* c, const mrg_parts* local, int P, mrg_parts** owned);

// What RCCL itself reports for this context's communicator (not what the
// caller passed to mrg_comm_init), and the HIP device the context drives.
static void comm_identity(mrg_ctx* c) {
    int n = 0, r = -1, d = -1;
    if (c->comm) {
        if (ncclCommCount(c->comm, &n) != ncclSuccess) n = -1;
        if (ncclCommUserRank(c->comm, &r) != ncclSuccess) r = -1;
        if (ncclCommCuDevice(c->comm, &d) != ncclSuccess) d = -1;
    }
    c->stats.rccl_nranks = n;
    c->stats.rccl_rank = r;
    c->stats.device = c->comm && d >= 0 ? d : c->device;
}

int mrg_exchange(mrg_ctx* c, const mrg_parts* local, mrg_parts** owned) {
    if (!c || !local || !owned) return MRG_EINVAL;
    int rc;
    if ((rc = bind(c))) return rc;
    const int P = c->nranks;
    if (!c->comm || (P == 1 && !c->exch_force_rccl)) {  // single rank: everything is owned; copy through aggregate
        return aggregate(c, {local->r}, local->app, local->nreduce, owned);
    }
    HCHK(c, hipEventRecord(c->ev[6], c->s));
    c->wd.enter("count all-to-all", c->exch_timeout_ms, c->rank, P);
    rc = exchange_rccl(c, local, P, owned);
    c->wd.leave();
    return rc;
}

// mrg_exchange's steps, under the watchdog (c->wd names the phase).
static int exchange_rccl(mrg_ctx* c, const mrg_parts* local, int P, mrg_parts** owned) {
    int rc;
    const Recs& r = local->r;
    if (!c->exch) c->exch = new ExchSide();
    ExchSide& x = *c->exch;
    if ((rc = exch_count(c, r, P, x))) return rc;
    NCHK(c, ncclAllToAll(x.d_cnt(P), x.d_rcv(P), 2, ncclUint64, c->comm, c->s));
    x.snd.assign(2 * P, 0);
    x.rcv.assign(2 * P, 0);
    HCHK(c, hipMemcpyAsync(x.snd.data(), x.d_cnt(P), 16 * P, hipMemcpyDeviceToHost, c->s));
    HCHK(c, hipMemcpyAsync(x.rcv.data(), x.d_rcv(P), 16 * P, hipMemcpyDeviceToHost, c->s));
    // ncclAllToAllv takes host counts: one round trip for the P x 2 matrix row
    c->wd.set("count sync");
    HCHK(c, hipStreamSynchronize(c->s));
    c->wd.set("pack");
    if ((rc = exch_pack(c, r, P, x))) return rc;
    const ExchPlan& pl = x.plan;
    // records and long-key bytes as ONE grouped collective (one launch, both
    // streams of every peer pair in flight together)
    c->wd.set("payload all-to-all");
    NCHK(c, ncclGroupStart());
    ncclResult_t e1 = ncclAllToAllv(x.sbuf.p, pl.sc.data(), pl.sd.data(), x.rbuf.p, pl.rc.data(), pl.rd.data(),
                                    ncclUint8, c->comm, c->s);
    ncclResult_t e2 = ncclAllToAllv(x.sar_b.p, pl.asc.data(), pl.asd.data(), x.rar_b.p, pl.arc.data(), pl.ard.data(),
                                    ncclUint8, c->comm, c->s);
    ncclResult_t e3 = ncclGroupEnd();
    if (e1 != ncclSuccess || e2 != ncclSuccess || e3 != ncclSuccess)
        return fail(c, MRG_ECOMM, "payload all-to-all: %s", ncclGetErrorString(e1 != ncclSuccess ? e1 : e2 != ncclSuccess ? e2 : e3));
    HCHK(c, hipEventRecord(c->ev[7], c->s));
    c->wd.set("unpack + aggregate");
    rc = exch_finish(c, local, P, x, owned, c->ev[12]);
    // exchange_ms: counts + payload all-to-alls + the owner's unpack and exact
    // re-aggregation; the first two alone are exchange_a2a_ms (the xGMI part)
    c->stats.exchange_a2a_ms = ev_ms(c->ev[6], c->ev[7]);
    c->stats.exchange_unpack_ms = ev_ms(c->ev[13], c->ev[12]);
    c->stats.exchange_ms = ev_ms(c->ev[6], c->ev[12]);
    exch_bytes(pl, P, c->rank, &c->stats);
    comm_identity(c);
    return rc;
}

int mrg_exchange_group(mrg_ctx* const* ctxs, int P, const mrg_parts* const* local, mrg_parts** owned) {
    if (!ctxs || !local || !owned || P < 1) return MRG_EINVAL;
    for (int i = 0; i < P; i++) {
        if (!ctxs[i] || !local[i]) return MRG_EINVAL;
        owned[i] = nullptr;
        if (local[i]->app != local[0]->app || local[i]->nreduce != local[0]->nreduce)
            return fail(ctxs[i], MRG_EINVAL, "exchange_group: parts differ in app or nreduce");
        for (int j = 0; j < i; j++)
            if (ctxs[j] == ctxs[i]) return fail(ctxs[i], MRG_EINVAL, "exchange_group: context used twice");
    }
    std::vector<ExchSide> xs(P);
    int rc;
    auto undo = [&](int code) {
        for (int i = 0; i < P; i++) {
            if (owned[i]) mrg_parts_free(owned[i]);
            owned[i] = nullptr;
        }
        for (int i = 0; i < P; i++) hipSetDevice(ctxs[i]->device), hipStreamSynchronize(ctxs[i]->s);
        return code;
    };
    for (int i = 0; i < P; i++) {
        mrg_ctx* c = ctxs[i];
        if ((rc = bind(c))) return undo(rc);
        HCHK(c, hipEventRecord(c->ev[6], c->s));
        if ((rc = exch_count(c, local[i]->r, P, xs[i]))) return undo(rc);
        xs[i].snd.assign(2 * P, 0);
        if (hipMemcpyAsync(xs[i].snd.data(), xs[i].d_cnt(P), 16 * P, hipMemcpyDeviceToHost, c->s) != hipSuccess)
            return undo(fail(c, MRG_EDEVICE, "exchange_group: count copy"));
    }
    for (int i = 0; i < P; i++) {
        hipSetDevice(ctxs[i]->device);
        if (hipStreamSynchronize(ctxs[i]->s) != hipSuccess) return undo(fail(ctxs[i], MRG_EDEVICE, "count sync"));
    }
    for (int j = 0; j < P; j++) {  // what owner j receives from source s = what s sends to j
        xs[j].rcv.assign(2 * P, 0);
        for (int s = 0; s < P; s++) {
            xs[j].rcv[2 * s] = xs[s].snd[2 * j];
            xs[j].rcv[2 * s + 1] = xs[s].snd[2 * j + 1];
        }
    }
    for (int i = 0; i < P; i++) {
        if ((rc = bind(ctxs[i]))) return undo(rc);
        if ((rc = exch_pack(ctxs[i], local[i]->r, P, xs[i]))) return undo(rc);
    }
    for (int i = 0; i < P; i++) {  // every send segment is packed before any copy reads it
        hipSetDevice(ctxs[i]->device);
        if (hipStreamSynchronize(ctxs[i]->s) != hipSuccess) return undo(fail(ctxs[i], MRG_EDEVICE, "pack sync"));
    }
    for (int j = 0; j < P; j++) {
        mrg_ctx* c = ctxs[j];
        if ((rc = bind(c))) return undo(rc);
        for (int s = 0; s < P; s++) {
            const ExchPlan& ps = xs[s].plan;
            const ExchPlan& pj = xs[j].plan;
            if (pj.rc[s])
                HCHK(c, hipMemcpyPeerAsync((uint8_t*)xs[j].rbuf.p + pj.rd[s], c->device,
                                           (const uint8_t*)xs[s].sbuf.p + ps.sd[j], ctxs[s]->device, pj.rc[s], c->s));
            if (pj.arc[s])
                HCHK(c, hipMemcpyPeerAsync((uint8_t*)xs[j].rar_b.p + pj.ard[s], c->device,
                                           (const uint8_t*)xs[s].sar_b.p + ps.asd[j], ctxs[s]->device, pj.arc[s],
                                           c->s));
        }
        HCHK(c, hipEventRecord(c->ev[7], c->s));
    }
    for (int j = 0; j < P; j++) {  // the copies of owner j read every source's buffers: drain them all first
        hipSetDevice(ctxs[j]->device);
        if (hipStreamSynchronize(ctxs[j]->s) != hipSuccess) return undo(fail(ctxs[j], MRG_EDEVICE, "copy sync"));
    }
    for (int j = 0; j < P; j++) {
        if ((rc = bind(ctxs[j]))) return undo(rc);
        if ((rc = exch_finish(ctxs[j], local[j], P, xs[j], &owned[j], ctxs[j]->ev[12]))) return undo(rc);
        ctxs[j]->stats.exchange_a2a_ms = ev_ms(ctxs[j]->ev[6], ctxs[j]->ev[7]);
        // (from the owner's own unpack start: the contexts' finishes run one after
        // another on this host thread, so ev[7] -> ev[12] would include the others')
        ctxs[j]->stats.exchange_unpack_ms = ev_ms(ctxs[j]->ev[13], ctxs[j]->ev[12]);
        ctxs[j]->stats.exchange_ms = ev_ms(ctxs[j]->ev[6], ctxs[j]->ev[12]);
        ctxs[j]->stats.rccl_nranks = 0;  // peer copies, no communicator
        ctxs[j]->stats.rccl_rank = -1;
        ctxs[j]->stats.device = ctxs[j]->device;
        exch_bytes(xs[j].plan, P, j, &ctxs[j]->stats);
    }
    return MRG_OK;
}

int mrg_run_job(mrg_ctx* c, int app, const void* buf, size_t len, int kind, const uint8_t* pat, size_t plen,
                uint32_t nreduce, void** bytes, size_t* nb, uint64_t* offsets) {
    if (!c || !bytes || !nb || !offsets) return MRG_EINVAL;
    const auto t_job = std::chrono::steady_clock::now();
    int drc;
    if ((drc = bind(c)) || (drc = drain_async(c))) return drc;  // (its pinned output buffer is separate)
    mrg_parts* p = nullptr;
    int rc = mrg_map(c, app, buf, len, kind, pat, plen, nreduce, &p);
    if (rc) return rc;
    mrg_stats keep = c->stats;
    mrg_parts* use = p;
    if (c->comm && c->nranks > 1 && !c->skip_exchange) {
        mrg_parts* o = nullptr;
        rc = mrg_exchange(c, p, &o);
        keep.exchange_ms = c->stats.exchange_ms;
        keep.exchange_a2a_ms = c->stats.exchange_a2a_ms;
        keep.exchange_unpack_ms = c->stats.exchange_unpack_ms;
        keep.rccl_nranks = c->stats.rccl_nranks;
        keep.rccl_rank = c->stats.rccl_rank;
        keep.shuffle_send_bytes = c->stats.shuffle_send_bytes;
        keep.shuffle_recv_bytes = c->stats.shuffle_recv_bytes;
        keep.shuffle_recv_records = c->stats.shuffle_recv_records;
        mrg_parts_free(p);
        if (rc) return rc;
        use = o;
    }
    // The output lines are written straight into the context's pinned host
    // buffer by the formatting kernel (sized for the output's bound up front), so
    // the transfer overlaps the formatting and the copy's host round trip goes
    // (C2: 0.56 -> 0.50 ms for reduce + transfer; C3 ~0.1 ms once grep's blocks
    // stage 128 lines, not 256, and never fall back to byte stores).  Option
    // out_direct = -1: always the copy; 1: wc only.
    const bool direct_ok = c->out_direct && (use->app == MRG_APP_WC || c->out_direct_grep);
    const uint64_t bound = reduce_out_bound(use->r, use->app) + 1;
    const uint64_t need = direct_ok ? bound : 0;
    if (need > c->h_out_cap) {
        if (c->h_out) hipHostFree(c->h_out);
        c->h_out = nullptr;
        c->h_out_cap = 0;
        size_t cap = need + need / 4 + 4096;
        if (hipHostMalloc((void**)&c->h_out, cap, hipHostMallocDefault) != hipSuccess) {
            mrg_parts_free(use);
            return fail(c, MRG_ENOMEM, "pinned output alloc");
        }
        c->h_out_cap = cap;
    }
    uint8_t* d = nullptr;
    uint64_t n = 0;
    rc = reduce_common(c, use, 0xFFFFFFFFu, &d, &n, offsets, direct_ok ? c->h_out : nullptr, c->h_out_cap);
    if (rc) { mrg_parts_free(use); return rc; }
    const bool direct = d == c->h_out;
    if (!direct && n + 1 > c->h_out_cap) {
        if (c->h_out) hipHostFree(c->h_out);
        c->h_out = nullptr;
        c->h_out_cap = 0;
        size_t cap = n + n / 4 + 4096;
        if (hipHostMalloc((void**)&c->h_out, cap, hipHostMallocDefault) != hipSuccess) {
            mrg_parts_free(use);
            return fail(c, MRG_ENOMEM, "pinned output alloc");
        }
        c->h_out_cap = cap;
    }
    HCHK(c, hipEventRecord(c->ev[6], c->s));
    if (n && !direct) HCHK(c, hipMemcpyAsync(c->h_out, d, n, hipMemcpyDeviceToHost, c->s));
    HCHK(c, hipEventRecord(c->ev[7], c->s));
    HCHK(c, hipEventSynchronize(c->ev[7]));
    if (c->debug_times)
        fprintf(stderr, "[mrg job] %.3f ms (map total %.3f, reduce %.3f, d2h %.3f ms of events)\n",
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_job).count(),
                keep.map_total_ms, ev_ms(c->ev[4], c->ev[5]), ev_ms(c->ev[6], c->ev[7]));
    keep.reduce_ms = ev_ms(c->ev[4], c->ev[5]);
    keep.d2h_ms = ev_ms(c->ev[6], c->ev[7]);
    keep.output_bytes = n;
    keep.distinct_keys = use->r.n;
    c->stats = keep;
    mrg_parts_free(use);
    *bytes = c->h_out;  // context-owned; valid until the next call on this context (do not mrg_free)
    *nb = n;
    return MRG_OK;
}

int mrg_run_job_async(mrg_ctx* c, int app, const void* buf, size_t len, int kind, const uint8_t* pat, size_t plen,
                      uint32_t nreduce) {
    if (!c) return MRG_EINVAL;
    int rc;
    if ((rc = bind(c))) return rc;
    if (c->aj_count >= 2) return fail(c, MRG_EINVAL, "run_job_async: two jobs in flight; mrg_job_wait first");
    if (!c->os) HCHK(c, hipStreamCreateWithFlags(&c->os, hipStreamNonBlocking));
    mrg_ctx::AsyncJob& J = c->aj[(c->aj_head + c->aj_count) & 1];
    if (!J.done) {
        HCHK(c, hipEventCreate(&J.start));
        HCHK(c, hipEventCreate(&J.done));
    }
    // map (+ exchange) on the context stream: it overlaps the previous job's
    // output transfer on the output stream
    mrg_parts* p = nullptr;
    if ((rc = mrg_map(c, app, buf, len, kind, pat, plen, nreduce, &p))) return rc;
    mrg_stats keep = c->stats;
    mrg_parts* use = p;
    if (c->comm && c->nranks > 1 && !c->skip_exchange) {
        mrg_parts* o = nullptr;
        rc = mrg_exchange(c, p, &o);
        keep.exchange_ms = c->stats.exchange_ms;
        keep.exchange_a2a_ms = c->stats.exchange_a2a_ms;
        keep.exchange_unpack_ms = c->stats.exchange_unpack_ms;
        keep.rccl_nranks = c->stats.rccl_nranks;
        keep.rccl_rank = c->stats.rccl_rank;
        keep.shuffle_send_bytes = c->stats.shuffle_send_bytes;
        keep.shuffle_recv_bytes = c->stats.shuffle_recv_bytes;
        keep.shuffle_recv_records = c->stats.shuffle_recv_records;
        mrg_parts_free(p);
        if (rc) return rc;
        use = o;
    }
    // (reduce_common first waits for the previous job's transfer: it writes the
    // device output buffer that transfer reads)
    J.offsets.assign((size_t)use->nreduce + 1, 0);
    uint8_t* d = nullptr;
    uint64_t n = 0;
    // wc with a small output (C2: 10 MB): the lines go straight into this job's
    // pinned buffer (as mrg_run_job's); a large one (C5: 110 MB, ~2 ms over PCIe
    // inside the formatting kernel) and grep: device buffer + the copy below,
    // which overlaps the next job's map
    const uint64_t bound = reduce_out_bound(use->r, use->app) + 1;
    const bool direct_ok = c->out_direct && use->app == MRG_APP_WC && bound <= c->async_direct_max;
    if (direct_ok) {
        if (bound > J.cap) {
            if (J.host) hipHostFree(J.host);
            J.host = nullptr;
            J.cap = 0;
            const size_t cap = bound + bound / 4 + 4096;
            if (hipHostMalloc((void**)&J.host, cap, hipHostMallocDefault) != hipSuccess) {
                mrg_parts_free(use);
                return fail(c, MRG_ENOMEM, "pinned output alloc");
            }
            J.cap = cap;
        }
    }
    rc = reduce_common(c, use, 0xFFFFFFFFu, &d, &n, J.offsets.data(), direct_ok ? (uint8_t*)J.host : nullptr,
                       direct_ok ? J.cap : 0);
    const uint64_t nkeys = use->r.n;
    mrg_parts_free(use);
    if (rc) return rc;
    if (d == (uint8_t*)J.host && d) {  // written in place (the reduce ended with a stream synchronize)
        HCHK(c, hipEventRecord(J.start, c->os));
        HCHK(c, hipEventRecord(J.done, c->os));
        keep.reduce_ms = ev_ms(c->ev[4], c->ev[5]);
        keep.output_bytes = n;
        keep.distinct_keys = nkeys;
        J.n = n;
        J.stats = keep;
        c->stats = keep;
        c->aj_count++;
        return MRG_OK;
    }
    if (n + 1 > J.cap) {
        if (J.host) hipHostFree(J.host);
        J.host = nullptr;
        J.cap = 0;
        const size_t cap = n + n / 4 + 4096;
        if (hipHostMalloc((void**)&J.host, cap, hipHostMallocDefault) != hipSuccess)
            return fail(c, MRG_ENOMEM, "pinned output alloc");
        J.cap = cap;
    }
    // the output crosses PCIe on the output stream after the reduce (the reduce
    // ends with a stream synchronize, so its bytes are complete here)
    HCHK(c, hipEventRecord(J.start, c->os));
    if (n) HCHK(c, hipMemcpyAsync(J.host, d, n, hipMemcpyDeviceToHost, c->os));
    HCHK(c, hipEventRecord(J.done, c->os));
    keep.reduce_ms = ev_ms(c->ev[4], c->ev[5]);
    keep.output_bytes = n;
    keep.distinct_keys = nkeys;
    J.n = n;
    J.stats = keep;
    c->stats = keep;
    c->aj_count++;
    return MRG_OK;
}

int mrg_job_wait(mrg_ctx* c, void** bytes, size_t* nb, uint64_t* offsets) {
    if (!c || !bytes || !nb || !offsets) return MRG_EINVAL;
    int rc;
    if ((rc = bind(c))) return rc;
    if (c->aj_count == 0) return fail(c, MRG_EINVAL, "job_wait: no job queued");
    mrg_ctx::AsyncJob& J = c->aj[c->aj_head];
    HCHK(c, hipEventSynchronize(J.done));
    J.stats.d2h_ms = ev_ms(J.start, J.done);
    c->stats = J.stats;
    for (size_t i = 0; i < J.offsets.size(); i++) offsets[i] = J.offsets[i];
    *bytes = J.host;  // context-owned; valid until the next mrg_job_wait (do not mrg_free)
    *nb = J.n;
    c->aj_head ^= 1;
    c->aj_count--;
    return MRG_OK;
}

}  // extern "C"
