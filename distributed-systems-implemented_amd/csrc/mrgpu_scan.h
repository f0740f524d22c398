// mrgpu_scan.h — single-pass tile scans with decoupled look-back, hand-written
// for the reduce's prefix sums and compactions (MapReduce/mr/worker.go:124-146:
// the output offsets of the sorted lines, the boundaries of tied runs).
//
// The protocol is the radix sort's (mrgpu_sort.hip): a workgroup takes the next
// tile from a device counter (reset by whoever takes the last tile, so tiles
// start in order and a look-back never waits on a tile that is not running),
// publishes its aggregate in a 64-bit state word, walks back over the earlier
// tiles' words (64 per round trip, one per lane of wave 0) to the first
// inclusive prefix, and publishes its own inclusive prefix.  A state word packs
// (epoch << 2 | flag) in bits 48-63 and the value in bits 0-47, so one relaxed
// 64-bit atomic carries both and the state array is never cleared between
// scans: a word of an earlier scan reads as "not published".  (Values are
// byte offsets and counts: 48 bits hold 2.8e14.)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mrg {

constexpr uint32_t kScanThreads = 256;
constexpr uint32_t kScanPer = 16;                          // consecutive elements per thread
constexpr uint32_t kScanTile = kScanThreads * kScanPer;    // 4096
constexpr uint32_t kScanFlagAgg = 1, kScanFlagInc = 2;
constexpr uint64_t kScanValMask = (1ull << 48) - 1;
constexpr uint32_t kScanEpochMax = (1u << 14) - 1;

struct ScanState {
    unsigned long long* state;  // [ntiles]
    uint32_t* ctr;              // tile counter (zero between scans)
    uint32_t epoch;             // 1 .. kScanEpochMax
    uint32_t ntiles;
};

// Host side: state sized for ntiles, a fresh epoch per scan (the array is
// cleared only when it grows or the epoch wraps).
struct ScanWs {
    unsigned long long* state = nullptr;
    uint32_t* ctr = nullptr;
    uint64_t cap = 0;
    uint32_t epoch = kScanEpochMax;
    hipError_t prepare(uint64_t ntiles, hipStream_t s, ScanState* st) {
        hipError_t e;
        if (!ctr) {
            if ((e = hipMalloc(&ctr, 64)) != hipSuccess) return e;
            if ((e = hipMemsetAsync(ctr, 0, 64, s)) != hipSuccess) return e;
        }
        if (ntiles > cap || epoch >= kScanEpochMax) {
            if (ntiles > cap) {
                if (state) (void)hipFree(state);
                state = nullptr;
                cap = 0;
                const uint64_t c = ntiles + ntiles / 4 + 64;
                if ((e = hipMalloc(&state, c * 8)) != hipSuccess) return e;
                cap = c;
            }
            if ((e = hipMemsetAsync(state, 0, cap * 8, s)) != hipSuccess) return e;
            epoch = 0;
        }
        st->state = state;
        st->ctr = ctr;
        st->epoch = ++epoch;
        st->ntiles = (uint32_t)ntiles;
        return hipSuccess;
    }
    void release() {
        if (state) (void)hipFree(state);
        if (ctr) (void)hipFree(ctr);
        state = nullptr;
        ctr = nullptr;
        cap = 0;
    }
};

// The next tile in start order (block-uniform; uses one word of LDS).
__device__ __forceinline__ uint32_t scan_take_tile(const ScanState& st, uint32_t* lds_word) {
    if (threadIdx.x == 0) {
        const uint32_t t = atomicAdd(st.ctr, 1u);
        if (t == st.ntiles - 1) __hip_atomic_store(st.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *lds_word = t;
    }
    __syncthreads();
    return *lds_word;
}

__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(v, o);
        if (lane >= (uint32_t)o) v += y;
    }
    return v;
}

// Exclusive scan of one u64 per thread over the block (kScanThreads threads);
// `red` = kScanThreads / 64 u64 of LDS.  Every thread must call it.
__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t v, unsigned long long* red, uint64_t* total) {
    constexpr uint32_t NW = kScanThreads / 64;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t incl = wave_incl_scan_u64(v);
    if (lane == 63) red[w] = incl;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t i = 0; i < NW; i++) {
        const uint64_t r = red[i];
        pre += i < w ? r : 0ull;
        tot += r;
    }
    __syncthreads();
    *total = tot;
    return pre + incl - v;
}

// Tile t's exclusive prefix: publish its aggregate, look back, publish its
// inclusive prefix.  Called by wave 0 of the block (all 64 lanes); returns the
// prefix in every lane.
__device__ __forceinline__ uint64_t scan_lookback(const ScanState& st, uint32_t t, uint64_t agg) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t tag_agg = (uint64_t)((st.epoch << 2) | kScanFlagAgg) << 48;
    const uint64_t tag_inc = (uint64_t)((st.epoch << 2) | kScanFlagInc) << 48;
    unsigned long long* me = st.state + t;
    if (t == 0) {
        if (lane == 0) __hip_atomic_store(me, tag_inc | (agg & kScanValMask), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(me, tag_agg | (agg & kScanValMask), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t prefix = 0;
    int64_t j = (int64_t)t - 1;  // next tile to read (lane q reads j - q)
    for (;;) {
        const int64_t jj = j - (int64_t)lane;
        const uint64_t v = jj >= 0 ? __hip_atomic_load(st.state + jj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : tag_inc;
        const uint64_t tag = v & ~kScanValMask;
        const uint64_t mInc = __ballot(tag == tag_inc), mRdy = __ballot(tag == tag_inc || tag == tag_agg);
        const uint64_t stop = mInc | ~mRdy;  // the first inclusive or not-yet-published word
        const uint32_t f = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;
        const bool take = lane < f || (lane == f && ((mInc >> f) & 1ull));
        uint64_t x = take ? (v & kScanValMask) : 0ull;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
        prefix += x;
        if (f < 64 && ((mInc >> f) & 1ull)) break;
        j -= f;  // re-poll from the first word not yet published (or the next 64)
    }
    if (lane == 0)
        __hip_atomic_store(me, tag_inc | ((prefix + agg) & kScanValMask), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return prefix;
}

}  // namespace mrg
