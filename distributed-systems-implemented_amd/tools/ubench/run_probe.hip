// run_probe.hip — store rate of the map kernel's spill records when one
// wave-instruction writes runs of R consecutive records per stream (what a
// workgroup-level sort of a batch of misses by bucket would produce), against
// R = 1 (today: 64 records to 64 streams), with NS streams per workgroup and a
// concurrent input stream, 256 workgroups x 1024 threads.
// Build: hipcc -O3 --offload-arch=gfx950 run_probe.hip -o run_probe
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

// Each wave-instruction: 64 records = 64/R runs of R consecutive records, run j
// to a random stream s_j, appended at the stream's workgroup-wide LDS cursor
// (sequential appends shared by the 16 waves, like the map kernel's).
template <int NS, int R>
__global__ void __launch_bounds__(1024) store_runs(unsigned long long* out, unsigned cap, unsigned iters,
                                                   const uint4* in, unsigned long long in_per_wg, int read_input) {
    __shared__ unsigned cur[NS];
    for (unsigned i = threadIdx.x; i < NS; i += 1024) cur[i] = 0;
    __syncthreads();
    const unsigned lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long* base = out + (unsigned long long)blockIdx.x * NS * cap;
    const uint4* ip = in + (unsigned long long)blockIdx.x * in_per_wg;
    unsigned acc = 0;
    for (unsigned it = 0; it < iters; it++) {
        if (read_input) {
            const unsigned long long k = ((unsigned long long)it * 1024 + threadIdx.x) % in_per_wg;
            const u4v v = __builtin_nontemporal_load((const u4v*)(ip + k));
            acc += v.x ^ v.w;
        }
        const unsigned run = lane / R, r = lane % R;
        const unsigned s = mix(blockIdx.x * 0x9E3779B9u + it * 64 + wv * 7919 + run) & (NS - 1);
        unsigned p = 0;
        if (r == 0) p = atomicAdd(&cur[s], (unsigned)R);
        p = __shfl(p, (int)(run * R));
        const unsigned off = (p + r) % cap;
        base[(unsigned long long)s * cap + off] = 0x0101010101010101ull * (it + 1) + acc;
    }
}

template <int NS, int R>
double run(unsigned long long* out, unsigned cap, unsigned iters, const uint4* in, unsigned long long in_per_wg,
           int read_input, int nwg) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {
        CHK(hipEventRecord(a));
        store_runs<NS, R><<<nwg, 1024>>>(out, cap, iters, in, in_per_wg, read_input);
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
    const unsigned iters = 2048;
    const unsigned long long recs = (unsigned long long)nwg * 1024 * iters;  // 537M records = 4.3 GB
    const unsigned long long in_per_wg = 1024ull * iters;
    uint4* in;
    CHK(hipMalloc(&in, (size_t)nwg * in_per_wg * 16));
    CHK(hipMemset(in, 1, (size_t)nwg * in_per_wg * 16));
    unsigned long long* out;
    const size_t out_bytes = (size_t)nwg * (2ull * 1024 * iters + 64ull * 4096) * 8;
    CHK(hipMalloc(&out, out_bytes));
    printf("{\"records\": %llu, \"record_bytes\": %llu}\n", recs, recs * 8);
    for (int read_input = 0; read_input < 2; read_input++) {
#define ONE(NS, R)                                                                                              \
    {                                                                                                           \
        const unsigned cap = (unsigned)(2ull * 1024 * iters / NS + 64) & ~63u;                                  \
        const double ms = run<NS, R>(out, cap, iters, in, in_per_wg, read_input, nwg);                          \
        printf("{\"NS\": %d, \"R\": %d, \"input\": %d, \"ms\": %.3f, \"rec_GBps\": %.1f}\n", NS, R, read_input, \
               ms, recs * 8 / ms / 1e6);                                                                        \
        fflush(stdout);                                                                                         \
    }
        ONE(256, 1) ONE(256, 4) ONE(256, 16) ONE(256, 64)
        ONE(512, 1) ONE(512, 4) ONE(512, 16)
        ONE(2048, 1) ONE(2048, 16)
    }
    return 0;
}
