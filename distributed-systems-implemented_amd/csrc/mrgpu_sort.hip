// mrgpu_sort.hip — the reduce's stable LSD radix sort, hand-written for gfx950.
//
// Reference: MapReduce/mr/worker.go:124-146 (sort.Sort(ByKey) of the reduce
// task's KeyValues) and main/mrsequential.go:68 — the order the output lines
// come in.  The reduce sorts (partition, key-prefix) keys of ~1e5-1e7 records
// (C3 ~5e5, C2 1e6, C5 1e7); at that size rocPRIM's onesweep costs ~20 us per
// pass plus two look-back-state memsets (~4 us each) and an upfront histogram
// launch: the passes are latency-bound, not HBM-bound (1e6 u32 pairs are 16 MB
// of traffic per pass, ~3 us at HBM rate).
//
// Here a sort of P passes is P + 1 launches and no memsets:
//  - radix_hist_kernel: every pass's 256-bin digit histogram in one read of the
//    keys (LDS counters, one device atomic per (workgroup, pass, non-empty bin));
//    the last workgroup to finish (ticket counter) scans them into each pass's
//    global digit starts and re-zeroes the histogram and the ticket for the
//    next sort;
//  - radix_pass_kernel, per pass: a workgroup takes the next 4096-key tile (a
//    device counter, reset by whoever takes the last tile, so tiles start in
//    order and the look-back cannot wait on a tile that never runs), ranks its
//    keys stably (16 waves; each owns 256 consecutive keys, 4 rows of 64: an
//    8-ballot match gives a lane its peers in the row, a per-wave LDS counter
//    per digit carries the rank across rows; 4 waves x 16 rows measured ~50 us
//    slower per C3 reduce, 8 x 8 and 8 x 16 in between), publishes its
//    per-digit counts (threads 0-255, one digit each), finds the
//    counts of all earlier tiles by decoupled look-back (16 tiles' words per
//    round trip), and writes its keys
//    grouped by digit through LDS (consecutive lanes, consecutive addresses).
// The look-back words carry the pass's epoch in their high half, so the state
// array is never cleared: a word from an earlier pass simply reads as "not
// ready".  (Scalar stores: none; every global write is a vector store/atomic.)
#include <hip/hip_runtime.h>

#include <algorithm>

#include "mrgpu_device.h"

#ifndef MRG_SORT_ROWS
#define MRG_SORT_ROWS 4
#endif
#ifndef MRG_SORT_WAVES
#define MRG_SORT_WAVES 16
#endif

namespace mrg {

namespace {

// Digit width RB: 8 bits (default), or 10 (option sort_digit_bits = 10: 64-bit
// keys in 7 passes instead of 8, C2's 60-bit key in 6; 1024 per-wave digit
// counters, 64 KB of LDS, 1024 look-back threads per tile).  Measured on C2 /
// C3 (`profiles/ab_r05_radix_digits.txt`): the wider passes cost what the
// saved passes save (C2 reduce 0.410 vs 0.415 ms) or more (C3 +0.05-0.1 ms).
constexpr int kRadixBitsMax = 10;
constexpr uint32_t kBinsMax = 1u << kRadixBitsMax;
template <int RB>
constexpr uint32_t bins_of() { return 1u << RB; }
template <int RB>
constexpr int max_passes() { return (64 + RB - 1) / RB; }
constexpr int kSortWaves = MRG_SORT_WAVES;  // waves per pass workgroup
constexpr int kSortThreads = 64 * kSortWaves;
constexpr int kHistThreads = 256;
constexpr int kRowsPerWave = MRG_SORT_ROWS;
constexpr uint32_t kWaveKeys = 64 * kRowsPerWave;           // 1024
constexpr uint32_t kTileKeys = kWaveKeys * kSortWaves;      // 4096
constexpr int kMaxPasses = 8;                               // 64-bit keys (8-bit digits: the most passes)
constexpr uint32_t kFlagAgg = 1, kFlagInc = 2;
constexpr int kLookWin = 16;  // look-back words loaded per round trip

// exclusive scan of one value per thread over an NW-wave block; `red` = NW
// u32 of LDS.  Every thread must call it.
template <int NW>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* red, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan_dpp(v);
    if (lane == 63) red[w] = incl;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        const uint32_t r = red[i];
        pre += (uint32_t)i < w ? r : 0u;
        tot += r;
    }
    __syncthreads();  // red reusable
    *total = tot;
    return pre + incl - v;
}

template <class K>
__device__ __forceinline__ uint32_t digit_of(K key, uint32_t shift, uint32_t mask) {
    return (uint32_t)(key >> shift) & mask;
}

// hist: npasses * 256 u32, zero on entry (left zero on exit); starts: the
// passes' exclusive digit starts; ticket: zero on entry (left zero).
template <class K, int RB>
__global__ void __launch_bounds__(kHistThreads) radix_hist_kernel(const K* __restrict__ keys, uint64_t n, uint32_t bits,
                                                                  uint32_t npasses, uint32_t* hist, uint32_t* starts,
                                                                  uint32_t* ticket) {
    constexpr uint32_t kBins = bins_of<RB>(), kPer = kBins / kHistThreads;  // digits per thread in the scan
    constexpr int kRadixBits = RB;
    __shared__ uint32_t h[max_passes<RB>() * kBins];
    __shared__ uint32_t red[kHistThreads / 64];
    __shared__ uint32_t last;
    for (uint32_t i = threadIdx.x; i < npasses * kBins; i += kHistThreads) h[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kHistThreads;
    for (uint64_t i = (uint64_t)blockIdx.x * kHistThreads + threadIdx.x; i < n; i += stride) {
        const K k = keys[i];
        for (uint32_t p = 0; p < npasses; p++) {
            const uint32_t shift = p * kRadixBits;
            const uint32_t w = bits - shift < (uint32_t)kRadixBits ? bits - shift : (uint32_t)kRadixBits;
            atomicAdd(&h[p * kBins + digit_of(k, shift, (1u << w) - 1u)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < npasses * kBins; i += kHistThreads)
        if (h[i]) atomicAdd(&hist[i], h[i]);
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(ticket, 1u) == gridDim.x - 1 ? 1u : 0u;
    __syncthreads();
    if (!last) return;
    __threadfence();
    for (uint32_t p = 0; p < npasses; p++) {
        uint32_t* hp = hist + p * kBins;
        uint32_t v[kPer], sum = 0;  // digits kPer * tid .. + kPer - 1
#pragma unroll
        for (uint32_t q = 0; q < kPer; q++) {
            v[q] = __hip_atomic_load(hp + kPer * threadIdx.x + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sum += v[q];
        }
        uint32_t tot;
        uint32_t run = block_excl_scan<kHistThreads / 64>(sum, red, &tot);
#pragma unroll
        for (uint32_t q = 0; q < kPer; q++) {
            starts[p * kBins + kPer * threadIdx.x + q] = run;
            run += v[q];
            hp[kPer * threadIdx.x + q] = 0u;
        }
    }
    if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class K, bool kVals, int RB>
struct PassLds {
    K k[kTileKeys];
    uint32_t v[kVals ? kTileKeys : 1];
    uint32_t wcnt[kSortWaves][bins_of<RB>()];  // per-wave digit counters, then the wave's exclusive offsets
    uint32_t dst[bins_of<RB>()];               // global position of the tile's digit-d run minus its tile-local start
    uint32_t red[kSortWaves];
    uint32_t tile;
};

template <class K, bool kVals, int RB>
__global__ void __launch_bounds__(kSortThreads) radix_pass_kernel(const K* __restrict__ kin, K* __restrict__ kout,
                                                                  const uint32_t* __restrict__ vin,
                                                                  uint32_t* __restrict__ vout, uint64_t n,
                                                                  uint32_t shift, uint32_t mask,
                                                                  const uint32_t* __restrict__ starts,
                                                                  unsigned long long* state, uint32_t* tile_ctr,
                                                                  uint32_t epoch, uint32_t ntiles) {
    constexpr uint32_t kBins = bins_of<RB>();
    constexpr int kRadixBits = RB;
    static_assert(kBins <= (uint32_t)kSortThreads, "one digit per thread");
    __shared__ PassLds<K, kVals, RB> L;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) {
        const uint32_t t = atomicAdd(tile_ctr, 1u);
        if (t == ntiles - 1) __hip_atomic_store(tile_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        L.tile = t;
    }
    for (uint32_t i = tid; i < kSortWaves * kBins; i += kSortThreads) (&L.wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint32_t t = L.tile;
    const uint64_t tile0 = (uint64_t)t * kTileKeys;
    const uint32_t tile_n = (uint32_t)std::min<uint64_t>(kTileKeys, n - tile0);
    const uint64_t base = tile0 + (uint64_t)w * kWaveKeys + lane;
    const uint64_t lt = (1ull << lane) - 1ull;

    K key[kRowsPerWave];
    uint32_t val[kRowsPerWave];
    uint32_t rank[kRowsPerWave];
#pragma unroll
    for (int r = 0; r < kRowsPerWave; r++) {
        const uint64_t i = base + (uint64_t)r * 64;
        const bool ok = i < n;
        key[r] = ok ? kin[i] : (K)0;
        if constexpr (kVals) val[r] = ok ? vin[i] : 0u;
    }
    // stable ranks within the wave's 1024 keys: row by row, a lane's peers
    // (same digit) by 8 ballot bit-planes
#pragma unroll
    for (int r = 0; r < kRowsPerWave; r++) {
        const uint64_t i = base + (uint64_t)r * 64;
        const bool ok = i < n;
        const uint32_t d = digit_of(key[r], shift, mask);
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < kRadixBits; b++) {
            const uint32_t bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= m ^ ((uint64_t)bit - 1ull);  // bit 0: ~m
        }
        const uint32_t before = (uint32_t)__popcll(peers & lt);
        const uint32_t old = L.wcnt[w][d];
        rank[r] = old + before;
        if (ok && before == 0) L.wcnt[w][d] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    // thread tid < 256 = digit: wave offsets, the tile's count, the tile-local start
    const bool dig = tid < kBins;
    uint32_t cnt = 0;
    if (dig) {
#pragma unroll
        for (int i = 0; i < kSortWaves; i++) {
            const uint32_t c = L.wcnt[i][tid];
            L.wcnt[i][tid] = cnt;
            cnt += c;
        }
    }
    uint32_t tot;
    const uint32_t lstart = block_excl_scan<kSortWaves>(cnt, L.red, &tot);
    if (dig) {
    // decoupled look-back for digit tid: publish this tile's count, sum the
    // earlier tiles' counts back to the first inclusive prefix
    unsigned long long* st = state + (uint64_t)t * kBins + tid;  // (the state array holds kBinsMax words per tile)
    const uint64_t hi_agg = (uint64_t)((epoch << 2) | kFlagAgg) << 32;
    const uint64_t hi_inc = (uint64_t)((epoch << 2) | kFlagInc) << 32;
    uint32_t prefix = 0;
    if (t == 0) {
        __hip_atomic_store(st, hi_inc | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        __hip_atomic_store(st, hi_agg | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // kLookWin earlier tiles' words per round trip (loads in flight
        // together): a tile deep in the grid does not walk back one L2 round
        // trip per tile while the tiles before it still hold only aggregates
        int64_t j = (int64_t)t - 1;
        for (;;) {
            uint64_t sv[kLookWin];
#pragma unroll
            for (int q = 0; q < kLookWin; q++) {
                const int64_t jj = j - q;
                sv[q] = jj >= 0 ? __hip_atomic_load(state + (uint64_t)jj * kBins + tid, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT)
                                : hi_inc;  // (not reached: tile 0 is inclusive)
            }
            bool done = false, stop = false;
            int used = 0;
#pragma unroll
            for (int q = 0; q < kLookWin; q++) {
                if (done || stop) continue;
                const uint64_t hi = sv[q] & 0xFFFFFFFF00000000ull;
                if (hi == hi_inc) {
                    prefix += (uint32_t)sv[q];
                    done = true;
                } else if (hi == hi_agg) {
                    prefix += (uint32_t)sv[q];
                    used++;
                } else {
                    stop = true;  // not published yet (an older epoch's word): poll again from here
                }
            }
            if (done) break;
            j -= used;
        }
        __hip_atomic_store(st, hi_inc | (prefix + cnt), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    L.dst[tid] = starts[tid] + prefix - lstart;
    // the tile-local start of each digit, kept in the wave-offset table
#pragma unroll
    for (int i = 0; i < kSortWaves; i++) L.wcnt[i][tid] += lstart;
    }  // dig
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRowsPerWave; r++) {
        if (base + (uint64_t)r * 64 < n) {
            const uint32_t d = digit_of(key[r], shift, mask);
            const uint32_t pos = L.wcnt[w][d] + rank[r];
            L.k[pos] = key[r];
            if constexpr (kVals) L.v[pos] = val[r];
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < tile_n; i += kSortThreads) {
        const K k = L.k[i];
        const uint32_t o = L.dst[digit_of(k, shift, mask)] + i;
        kout[o] = k;
        if constexpr (kVals) vout[o] = L.v[i];
    }
}

}  // namespace

struct RadixWs {
    uint32_t* small = nullptr;         // hist [kMaxPasses*kBinsMax] | starts [same] | ticket | tile counter
    unsigned long long* state = nullptr;
    uint64_t state_tiles = 0;
    void* buf = nullptr;               // ping-pong keys + values
    size_t buf_cap = 0;
    uint32_t epoch = 0;
    int digit_bits = 0;  // 10: 10-bit digits; 0 or 8: 8-bit
};

void radix_ws_set_digit_bits(RadixWs* w, int bits) { w->digit_bits = bits; }

RadixWs* radix_ws_new() { return new RadixWs(); }

void radix_ws_free(RadixWs* w) {
    if (!w) return;
    if (w->small) (void)hipFree(w->small);
    if (w->state) (void)hipFree(w->state);
    if (w->buf) (void)hipFree(w->buf);
    delete w;
}

#define SCHK(x)                               \
    do {                                      \
        hipError_t _e = (x);                  \
        if (_e != hipSuccess) return (int)_e; \
    } while (0)

template <class K, bool kVals, int RB>
static void radix_launch(RadixWs* w, const K* k_in, K* k_out, const uint32_t* v_in, uint32_t* v_out, uint64_t n,
                         unsigned bits, uint64_t ntiles, hipStream_t s) {
    constexpr uint32_t kBins = bins_of<RB>();
    const uint32_t npasses = (bits + RB - 1) / RB;
    uint32_t* hist = w->small;
    uint32_t* starts = hist + kMaxPasses * kBinsMax;
    uint32_t* ticket = starts + kMaxPasses * kBinsMax;
    uint32_t* tile_ctr = ticket + 16;
    K* k_tmp = (K*)w->buf;
    uint32_t* v_tmp = (uint32_t*)((char*)w->buf + ((n * sizeof(K) + 255) & ~(size_t)255));
    const unsigned hgrid = (unsigned)std::min<uint64_t>(std::max<uint64_t>((n + 8191) / 8192, 1), 512);
    radix_hist_kernel<K, RB><<<hgrid, kHistThreads, 0, s>>>(k_in, n, bits, npasses, hist, starts, ticket);
    const K* src_k = k_in;
    const uint32_t* src_v = v_in;
    for (uint32_t p = 0; p < npasses; p++) {  // ping-pong: the last pass writes k_out / v_out
        const bool to_out = ((npasses - 1 - p) & 1u) == 0;
        K* dk = to_out ? k_out : k_tmp;
        uint32_t* dv = to_out ? v_out : v_tmp;
        const uint32_t shift = p * RB;
        const uint32_t wbits = std::min<uint32_t>(RB, bits - shift);
        radix_pass_kernel<K, kVals, RB><<<(unsigned)ntiles, kSortThreads, 0, s>>>(
            src_k, dk, src_v, dv, n, shift, (1u << wbits) - 1u, starts + p * kBins, w->state, tile_ctr, ++w->epoch,
            (uint32_t)ntiles);
        src_k = dk;
        src_v = dv;
    }
}

template <class K, bool kVals>
static int radix_sort_impl(RadixWs* w, const K* k_in, K* k_out, const uint32_t* v_in, uint32_t* v_out, uint64_t n,
                           unsigned bits, hipStream_t s) {
    if (n == 0) return 0;
    if (n > 0xFFFFFFFFull) return (int)hipErrorInvalidValue;  // 32-bit counts in the look-back words
    if (bits == 0 || bits > 8 * sizeof(K)) bits = 8 * sizeof(K);
    const uint64_t ntiles = (n + kTileKeys - 1) / kTileKeys;
    // 10-bit digits only when asked for (option sort_digit_bits = 10) and they
    // save a pass
    const bool wide = w->digit_bits == 10 && (bits + 9) / 10 < (bits + 7) / 8;
    const uint32_t npasses = wide ? (bits + 9) / 10 : (bits + 7) / 8;
    const uint32_t small_words = 2 * kMaxPasses * kBinsMax + 64;
    if (!w->small) {
        SCHK(hipMalloc(&w->small, small_words * 4));
        SCHK(hipMemsetAsync(w->small, 0, small_words * 4, s));
    }
    if (ntiles > w->state_tiles || w->epoch >= (1u << 29)) {
        if (ntiles > w->state_tiles) {
            if (w->state) SCHK(hipFree(w->state));
            w->state = nullptr;
            w->state_tiles = 0;
            const uint64_t nt = ntiles + ntiles / 4 + 16;
            SCHK(hipMalloc(&w->state, nt * kBinsMax * 8));
            w->state_tiles = nt;
        }
        SCHK(hipMemsetAsync(w->state, 0, w->state_tiles * kBinsMax * 8, s));
        w->epoch = 0;
    }
    const size_t need = n * sizeof(K) + (kVals ? n * 4 : 0) + 256;
    if (npasses > 1 && need > w->buf_cap) {
        if (w->buf) SCHK(hipFree(w->buf));
        w->buf = nullptr;
        w->buf_cap = 0;
        const size_t c = need + need / 4;
        SCHK(hipMalloc(&w->buf, c));
        w->buf_cap = c;
    }
    if (wide) radix_launch<K, kVals, 10>(w, k_in, k_out, v_in, v_out, n, bits, ntiles, s);
    else radix_launch<K, kVals, 8>(w, k_in, k_out, v_in, v_out, n, bits, ntiles, s);
    return (int)hipGetLastError();
}

int radix_sort_pairs_u32(RadixWs* w, const uint32_t* k_in, uint32_t* k_out, const uint32_t* v_in, uint32_t* v_out,
                         uint64_t n, unsigned bits, hipStream_t s) {
    return radix_sort_impl<uint32_t, true>(w, k_in, k_out, v_in, v_out, n, bits, s);
}
int radix_sort_pairs_u64(RadixWs* w, const uint64_t* k_in, uint64_t* k_out, const uint32_t* v_in, uint32_t* v_out,
                         uint64_t n, unsigned bits, hipStream_t s) {
    return radix_sort_impl<uint64_t, true>(w, k_in, k_out, v_in, v_out, n, bits, s);
}
int radix_sort_keys_u64(RadixWs* w, const uint64_t* k_in, uint64_t* k_out, uint64_t n, unsigned bits, hipStream_t s) {
    return radix_sort_impl<uint64_t, false>(w, k_in, k_out, nullptr, nullptr, n, bits, s);
}

}  // namespace mrg
