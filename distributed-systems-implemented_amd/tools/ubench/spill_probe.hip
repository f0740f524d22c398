// spill_probe.hip — how fast can a workgroup append 8-byte records to NS
// per-workgroup streams (the map kernel's spill pattern), as a function of NS,
// with and without a concurrent non-temporal input stream (the map's input)?
// Each wave-instruction stores 64 records to 64 random streams of its
// workgroup, positions from LDS cursors.  Also: the same records staged through
// a 32-byte-per-stream LDS sector buffer, flushed as whole sectors.
// Build: hipcc -O3 --offload-arch=gfx950 spill_probe.hip -o spill_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                  \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
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

// direct: one 8-byte store per record
template <int NS>
__global__ void __launch_bounds__(1024) spill_direct(unsigned long long* out, unsigned cap, unsigned iters,
                                                     const uint4* in, unsigned long long in_per_wg, int read_input) {
    __shared__ unsigned curs[NS];
    for (unsigned i = threadIdx.x; i < NS; i += 1024) curs[i] = 0;
    __syncthreads();
    unsigned long long* base = out + (unsigned long long)blockIdx.x * NS * cap;
    const uint4* ip = in + (unsigned long long)blockIdx.x * in_per_wg;
    unsigned acc = 0;
    for (unsigned it = 0; it < iters; it++) {
        if (read_input) {
            const unsigned long long k = ((unsigned long long)it * 1024 + threadIdx.x) % in_per_wg;
            const u4v v = __builtin_nontemporal_load((const u4v*)(ip + k));
            acc += v.x ^ v.w;
        }
        const unsigned s = mix(blockIdx.x * 0x9E3779B9u + it * 1024 + threadIdx.x) & (NS - 1);
        const unsigned pos = atomicAdd(&curs[s], 1u);
        if (pos < cap) base[(unsigned long long)s * cap + pos] = 0x0101010101010101ull * (it + 1) + acc;
    }
}

// staged: records gather in a 32-byte sector per stream (4 records); the lane
// whose record completes a sector writes the sector (two 16-byte stores by the
// same lane).  A per-stream fill counter tells which lane completes a sector;
// the sector buffer is double-buffered by sector parity so the next sector's
// records never overwrite one still being flushed.
template <int NS>
__global__ void __launch_bounds__(1024) spill_staged(unsigned long long* out, unsigned cap, unsigned iters,
                                                     const uint4* in, unsigned long long in_per_wg, int read_input) {
    __shared__ unsigned curs[NS];
    __shared__ unsigned fill[NS * 2];
    __shared__ unsigned long long sect[NS * 2][4];
    for (unsigned i = threadIdx.x; i < NS; i += 1024) curs[i] = 0;
    for (unsigned i = threadIdx.x; i < 2 * NS; i += 1024) fill[i] = 0;
    __syncthreads();
    unsigned long long* base = out + (unsigned long long)blockIdx.x * NS * cap;
    const uint4* ip = in + (unsigned long long)blockIdx.x * in_per_wg;
    unsigned acc = 0;
    for (unsigned it = 0; it < iters; it++) {
        if (read_input) {
            const unsigned long long k = ((unsigned long long)it * 1024 + threadIdx.x) % in_per_wg;
            const u4v v = __builtin_nontemporal_load((const u4v*)(ip + k));
            acc += v.x ^ v.w;
        }
        const unsigned s = mix(blockIdx.x * 0x9E3779B9u + it * 1024 + threadIdx.x) & (NS - 1);
        const unsigned pos = atomicAdd(&curs[s], 1u);
        const unsigned sec = pos >> 2, par = sec & 1;
        sect[2 * s + par][pos & 3] = 0x0101010101010101ull * (it + 1) + acc;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        const unsigned f = atomicAdd(&fill[2 * s + par], 1u);
        if ((f & 3) == 3 && pos < cap) {  // this lane completed the sector
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const uint4* src = (const uint4*)&sect[2 * s + par][0];
            uint4* dst = (uint4*)(base + (unsigned long long)s * cap + (sec << 2));
            dst[0] = src[0];
            dst[1] = src[1];
        }
    }
}

template <int NS>
double run(int staged, unsigned long long* out, unsigned cap, unsigned iters, const uint4* in,
           unsigned long long in_per_wg, int read_input, int nwg) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
        CHK(hipEventRecord(a));
        if constexpr (NS <= 2048) {
            if (staged) spill_staged<NS><<<nwg, 1024>>>(out, cap, iters, in, in_per_wg, read_input);
            else spill_direct<NS><<<nwg, 1024>>>(out, cap, iters, in, in_per_wg, read_input);
        } else {
            if (staged) return 0;
            spill_direct<NS><<<nwg, 1024>>>(out, cap, iters, in, in_per_wg, read_input);
        }
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

int main() {
    const int nwg = 256;
    const unsigned iters = 2048;                   // records per thread
    const unsigned long long recs = (unsigned long long)nwg * 1024 * iters;  // 537M records = 4.3 GB
    const unsigned long long in_per_wg = 1024ull * iters;  // 16 B each: 8.6 GB of input
    uint4* in;
    CHK(hipMalloc(&in, (size_t)nwg * in_per_wg * 16));
    CHK(hipMemset(in, 1, (size_t)nwg * in_per_wg * 16));
    unsigned long long* out;
    // per workgroup NS streams of cap = 2 * 1024 * iters / NS + 64 records: at most
    // (2 * 1024 * iters + 64 * 4096) records for the largest NS
    const size_t out_bytes = (size_t)nwg * (2ull * 1024 * iters + 64ull * 4096) * 8;
    CHK(hipMalloc(&out, out_bytes));
    printf("{\"records\": %llu, \"record_bytes\": %llu, \"input_bytes\": %llu}\n", recs, recs * 8,
           (unsigned long long)nwg * in_per_wg * 16);
    for (int read_input = 0; read_input < 2; read_input++)
        for (int staged = 0; staged < 2; staged++) {
#define ONE(NS)                                                                                               \
    {                                                                                                         \
        const unsigned cap = (unsigned)(2ull * 1024 * iters / NS + 64);                                       \
        const double ms = run<NS>(staged, out, cap, iters, in, in_per_wg, read_input, nwg);                   \
        printf("{\"NS\": %d, \"staged\": %d, \"input\": %d, \"ms\": %.3f, \"rec_GBps\": %.1f}\n", NS, staged, \
               read_input, ms, recs * 8 / ms / 1e6);                                                          \
    }
            ONE(64) ONE(256) ONE(1024) ONE(2048) ONE(4096)
        }
    return 0;
}
