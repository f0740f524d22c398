// h2h_probe.hip — can a kernel write its output straight into pinned host
// memory as fast as hipMemcpyAsync copies it there?  (The reduce's output goes
// to the host; writing it there from the formatting kernel would overlap the
// PCIe transfer with the formatting and drop a host round trip.)
// A kernel copies a device buffer to pinned host memory with 16-byte stores
// (one 1 KiB contiguous run per wave-instruction), against hipMemcpyAsync D2H,
// for 10 MB and 78 MB (the C2 / C3 output sizes).
// Build: hipcc -O3 --offload-arch=gfx950 h2h_probe.hip -o h2h_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__global__ void copy_out(const uint4* __restrict__ src, uint4* dst, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
typedef unsigned u4v __attribute__((ext_vector_type(4)));
__global__ void copy_out_nt(const uint4* __restrict__ src, uint4* dst, size_t n16) {
    const u4v* s = (const u4v*)src;
    u4v* o = (u4v*)dst;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(s[i], o + i);
}

static void run(size_t bytes, unsigned flags, const char* fname) {
    uint4* d;
    uint4* h;
    CHK(hipMalloc(&d, bytes));
    CHK(hipMemset(d, 7, bytes));
    CHK(hipHostMalloc((void**)&h, bytes, flags));
    memset(h, 0, bytes);
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const size_t n16 = bytes / 16;
    float best_k = 1e9f, best_knt = 1e9f, best_c = 1e9f;
    for (int grid : {256, 1024, 4096}) {
        for (int rep = 0; rep < 4; rep++) {
            float ms;
            CHK(hipEventRecord(e0));
            copy_out<<<grid, 256>>>(d, h, n16);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            CHK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best_k) best_k = ms;
            CHK(hipEventRecord(e0));
            copy_out_nt<<<grid, 256>>>(d, h, n16);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            CHK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best_knt) best_knt = ms;
        }
    }
    for (int rep = 0; rep < 4; rep++) {
        float ms;
        CHK(hipEventRecord(e0));
        CHK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0));
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best_c) best_c = ms;
    }
    unsigned bad = 0;
    for (size_t i = 0; i < bytes; i += 4093) bad += ((unsigned char*)h)[i] != 7;
    printf("%-14s %6.1f MB: kernel stores %.3f ms (%.1f GB/s), nt %.3f ms (%.1f GB/s), hipMemcpyAsync %.3f ms (%.1f GB/s), bad %u\n",
           fname, bytes / 1e6, best_k, bytes / best_k / 1e6, best_knt, bytes / best_knt / 1e6, best_c, bytes / best_c / 1e6, bad);
    fflush(stdout);
    CHK(hipHostFree(h));
    CHK(hipFree(d));
}

int main() {
    for (size_t mb : {10, 78}) {
        run(mb * 1000 * 1000 / 16 * 16, hipHostMallocDefault, "default");
        run(mb * 1000 * 1000 / 16 * 16, hipHostMallocNonCoherent, "noncoherent");
    }
    return 0;
}
