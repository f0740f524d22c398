// spill_probe2.hip — who should own a spill stream: the workgroup (LDS cursor,
// today's map kernel) or the XCD (a cursor in global memory shared by the 32
// workgroups of one XCD, so that a stream's 128-byte lines fill 32x faster and
// leave the XCD's L2 whole instead of half written)?
// 256 workgroups x 1024 threads; every thread appends `iters` 8-byte records,
// each to a random one of NS streams of its owner, while the workgroup also
// streams its share of an input buffer with non-temporal 16-byte loads (the map
// kernel's input).  Variants:
//   0 wg      per-workgroup streams, LDS cursor (today's map kernel, C5 layout)
//   1 xcd     per-XCD streams (HW_REG_XCC_ID), agent-scope returning atomicAdd on
//             the stream's cursor in global memory, then the store
//   2 xcd_wg  the same with workgroup-scope atomics (L2-executed if the hardware
//             does that for this scope; only one XCD ever touches a cursor)
//   3 grp     per-XCD streams keyed by blockIdx % 8 instead of the XCC id
//             (placement-dependent speed only: the atomics are agent scope)
// Build: hipcc -O3 --offload-arch=gfx950 spill_probe2.hip -o spill_probe2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                       \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

typedef unsigned u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned mix(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ unsigned xcc_id() {
    unsigned r;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(r));
    return r;
}

template <int NS, int V>
__global__ void __launch_bounds__(1024) spill(unsigned long long* out, unsigned cap, unsigned* gcur, unsigned iters,
                                              const uint4* in, unsigned long long in_per_wg, int read_input,
                                              unsigned* xcc_seen) {
    __shared__ unsigned curs[NS];
    if (V == 0) {
        for (unsigned i = threadIdx.x; i < NS; i += 1024) curs[i] = 0;
        __syncthreads();
    }
    const unsigned owner = V == 0 ? blockIdx.x : V == 3 ? blockIdx.x % 8 : xcc_id();
    if (threadIdx.x == 0) xcc_seen[blockIdx.x] = xcc_id();
    unsigned long long* base = out + (unsigned long long)owner * NS * cap;
    unsigned* gc = gcur + owner * NS;
    const uint4* ip = in + (unsigned long long)blockIdx.x * in_per_wg;
    unsigned acc = 0;
    for (unsigned it = 0; it < iters; it++) {
        if (read_input) {
            const unsigned long long k = ((unsigned long long)it * 1024 + threadIdx.x) % in_per_wg;
            const u4v v = __builtin_nontemporal_load((const u4v*)(ip + k));
            acc += v.x ^ v.w;
        }
        const unsigned s = mix(blockIdx.x * 0x9E3779B9u + it * 1024 + threadIdx.x) & (NS - 1);
        unsigned pos;
        if (V == 0) pos = atomicAdd(&curs[s], 1u);
        else if (V == 2) pos = __hip_atomic_fetch_add(&gc[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else pos = __hip_atomic_fetch_add(&gc[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (pos < cap) base[(unsigned long long)s * cap + pos] = 0x0101010101010101ull * (it + 1) + acc;
    }
}

// 4 wgsync: per-workgroup streams staged in LDS, 32 bytes (4 records) per
//   stream, with a workgroup barrier every `per` records per thread: between
//   barriers a record takes a slot by an LDS cursor and lands in the stream's
//   staging group if the group has room, else goes straight to memory; after
//   the barrier every complete group leaves as one 32-byte write.
template <int NS>
__global__ void __launch_bounds__(1024) spill_wgsync(unsigned long long* out, unsigned cap, unsigned iters,
                                                     const uint4* in, unsigned long long in_per_wg, int read_input,
                                                     unsigned per) {
    __shared__ unsigned curs[NS], fl[NS];
    __shared__ unsigned long long stage[NS][4];
    for (unsigned i = threadIdx.x; i < NS; i += 1024) curs[i] = fl[i] = 0;
    __syncthreads();
    unsigned long long* base = out + (unsigned long long)blockIdx.x * NS * cap;
    const uint4* ip = in + (unsigned long long)blockIdx.x * in_per_wg;
    unsigned acc = 0;
    for (unsigned it0 = 0; it0 < iters; it0 += per) {
        for (unsigned it = it0; it < it0 + per && it < iters; it++) {
            if (read_input) {
                const unsigned long long k = ((unsigned long long)it * 1024 + threadIdx.x) % in_per_wg;
                const u4v v = __builtin_nontemporal_load((const u4v*)(ip + k));
                acc += v.x ^ v.w;
            }
            const unsigned s = mix(blockIdx.x * 0x9E3779B9u + it * 1024 + threadIdx.x) & (NS - 1);
            const unsigned pos = atomicAdd(&curs[s], 1u);
            const unsigned long long rec = 0x0101010101010101ull * (it + 1) + acc;
            const unsigned f = fl[s];
            if (pos < f + 4) stage[s][pos - f] = rec;
            else if (pos < cap) base[(unsigned long long)s * cap + pos] = rec;
        }
        __syncthreads();
        for (unsigned s = threadIdx.x; s < NS; s += 1024) {
            const unsigned c = curs[s], f = fl[s];
            if (c >= f + 4) {
                if (f + 4 <= cap) {
                    uint4* dst = (uint4*)(base + (unsigned long long)s * cap + f);
                    const uint4* src = (const uint4*)&stage[s][0];
                    dst[0] = src[0];
                    dst[1] = src[1];
                }
                fl[s] = c;  // direct writes past the group: the next group starts at c
            }
        }
        __syncthreads();
    }
    for (unsigned s = threadIdx.x; s < NS; s += 1024) {
        const unsigned c = curs[s], f = fl[s];
        for (unsigned q = f; q < c && q < cap; q++) base[(unsigned long long)s * cap + q] = stage[s][q - f];
    }
}

template <int NS, int V>
double run(unsigned long long* out, unsigned cap, unsigned* gcur, unsigned iters, const uint4* in,
           unsigned long long in_per_wg, int read_input, int nwg, unsigned* xcc_seen, int nown) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
        CHK(hipMemset(gcur, 0, (size_t)nown * NS * 4));
        CHK(hipEventRecord(a));
        if constexpr (V >= 100) spill_wgsync<NS><<<nwg, 1024>>>(out, cap, iters, in, in_per_wg, read_input, V - 100);
        else spill<NS, V><<<nwg, 1024>>>(out, cap, gcur, iters, in, in_per_wg, read_input, xcc_seen);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv) {
    const int nwg = 256;
    const unsigned iters = argc > 1 ? (unsigned)atoi(argv[1]) : 1024;
    const unsigned long long recs = (unsigned long long)nwg * 1024 * iters;
    const unsigned long long in_per_wg = 1024ull * iters;  // 16 B each
    uint4* in;
    CHK(hipMalloc(&in, (size_t)nwg * in_per_wg * 16));
    CHK(hipMemset(in, 1, (size_t)nwg * in_per_wg * 16));
    constexpr int NS = 4096;
    // per-WG cap: 2x the mean stream length + slack; per-XCD streams are 32x longer
    const unsigned cap_wg = (unsigned)(2ull * 1024 * iters / NS + 64);
    const unsigned cap_x = cap_wg * 32;
    unsigned long long* out;
    const size_t out_bytes = (size_t)nwg * NS * cap_wg * 8;
    CHK(hipMalloc(&out, out_bytes));
    unsigned* gcur;
    CHK(hipMalloc(&gcur, (size_t)nwg * NS * 4));
    unsigned* xs;
    CHK(hipMalloc(&xs, nwg * 4));
    printf("{\"records\": %llu, \"record_bytes\": %llu, \"input_bytes\": %llu}\n", recs, recs * 8,
           (unsigned long long)nwg * in_per_wg * 16);
    for (int read_input = 0; read_input < 2; read_input++) {
        double ms;
        ms = run<NS, 0>(out, cap_wg, gcur, iters, in, in_per_wg, read_input, nwg, xs, nwg);
        printf("{\"variant\": \"wg\", \"input\": %d, \"ms\": %.3f, \"rec_GBps\": %.1f}\n", read_input, ms, recs * 8 / ms / 1e6);
        ms = run<NS, 1>(out, cap_x, gcur, iters, in, in_per_wg, read_input, nwg, xs, 8);
        printf("{\"variant\": \"xcd\", \"input\": %d, \"ms\": %.3f, \"rec_GBps\": %.1f}\n", read_input, ms, recs * 8 / ms / 1e6);
        ms = run<NS, 2>(out, cap_x, gcur, iters, in, in_per_wg, read_input, nwg, xs, 8);
        printf("{\"variant\": \"xcd_wg\", \"input\": %d, \"ms\": %.3f, \"rec_GBps\": %.1f}\n", read_input, ms, recs * 8 / ms / 1e6);
        ms = run<NS, 3>(out, cap_x, gcur, iters, in, in_per_wg, read_input, nwg, xs, 8);
        printf("{\"variant\": \"grp\", \"input\": %d, \"ms\": %.3f, \"rec_GBps\": %.1f}\n", read_input, ms, recs * 8 / ms / 1e6);
    }
    // LDS staging with workgroup barriers (2048 streams: what fits in LDS), vs direct
    for (int read_input = 0; read_input < 2; read_input++) {
        constexpr int NS2 = 2048;
        const unsigned cap2 = (unsigned)(2ull * 1024 * iters / NS2 + 64);
        double ms = run<NS2, 0>(out, cap2, gcur, iters, in, in_per_wg, read_input, nwg, xs, nwg);
        printf("{\"variant\": \"wg2048\", \"input\": %d, \"ms\": %.3f, \"rec_GBps\": %.1f}\n", read_input, ms, recs * 8 / ms / 1e6);
        ms = run<NS2, 101>(out, cap2, gcur, iters, in, in_per_wg, read_input, nwg, xs, nwg);
        printf("{\"variant\": \"wgsync2048_per1\", \"input\": %d, \"ms\": %.3f, \"rec_GBps\": %.1f}\n", read_input, ms, recs * 8 / ms / 1e6);
        ms = run<NS2, 102>(out, cap2, gcur, iters, in, in_per_wg, read_input, nwg, xs, nwg);
        printf("{\"variant\": \"wgsync2048_per2\", \"input\": %d, \"ms\": %.3f, \"rec_GBps\": %.1f}\n", read_input, ms, recs * 8 / ms / 1e6);
        ms = run<NS2, 104>(out, cap2, gcur, iters, in, in_per_wg, read_input, nwg, xs, nwg);
        printf("{\"variant\": \"wgsync2048_per4\", \"input\": %d, \"ms\": %.3f, \"rec_GBps\": %.1f}\n", read_input, ms, recs * 8 / ms / 1e6);
    }
    // check: the per-XCD cursors of the last run sum to the records (nothing lost)
    unsigned h[nwg];
    CHK(hipMemcpy(h, xs, nwg * 4, hipMemcpyDeviceToHost));
    int cnt[16] = {0};
    for (int i = 0; i < nwg; i++) cnt[h[i] & 15]++;
    printf("{\"xcc_histogram\": [");
    for (int i = 0; i < 8; i++) printf("%d%s", cnt[i], i < 7 ? ", " : "");
    printf("], \"block0_xcc\": %u, \"block1_xcc\": %u, \"block8_xcc\": %u}\n", h[0], h[1], h[8]);
    return 0;
}
