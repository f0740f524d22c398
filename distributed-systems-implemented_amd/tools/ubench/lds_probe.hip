// lds_probe.hip — hardware facts the v5 map kernel relies on (gfx950):
//  1. DPP wave_shr:1 / wave_shl:1 move a value one lane across the whole wave64.
//  2. ds_read_b128 / ds_read_b64 at byte-unaligned LDS addresses return the
//     right bytes, and what they cost relative to aligned reads.
//  3. buffer_load_dwordx4 ... lds (LDS-DMA) with a range-checked descriptor:
//     what a dword that straddles num_records returns.
// Build: hipcc -O3 --offload-arch=gfx950 lds_probe.hip -o lds_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

__global__ void dpp_test(unsigned* o) {
    unsigned v = threadIdx.x + 100;
    o[threadIdx.x] = __builtin_amdgcn_update_dpp(7u, v, 0x138, 0xf, 0xf, false);        // wave_shr:1
    o[64 + threadIdx.x] = __builtin_amdgcn_update_dpp(7u, v, 0x130, 0xf, 0xf, false);   // wave_shl:1
    o[128 + threadIdx.x] = __builtin_amdgcn_update_dpp(7u, v, 0x138, 0xf, 0xf, true);   // bound_ctrl
}

__global__ void unaligned_test(const unsigned char* src, u4* o) {
    __shared__ unsigned char buf[2048];
    for (int i = threadIdx.x; i < 2048; i++) buf[i] = src[i];  // thread 0..63 each copy overlapping; fine
    __syncthreads();
    u4 v;
    __builtin_memcpy(&v, buf + threadIdx.x * 7 + 3, 16);
    o[threadIdx.x] = v;
    unsigned long long w;
    __builtin_memcpy(&w, buf + threadIdx.x * 5 + 1, 8);
    o[64 + threadIdx.x] = (u4){(unsigned)w, (unsigned)(w >> 32), 0, 0};
}

// Throughput: each wave reads `iters` times 16 B from addresses base + lane*stride + shift.
template <int MODE>
__global__ void __launch_bounds__(1024) lds_bw(unsigned* out, int iters, int shift, int stride) {
    __shared__ unsigned char buf[65536 + 64];
    for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x) ((unsigned*)buf)[i] = i * 2654435761u;
    __syncthreads();
    unsigned acc = 0;
    const unsigned lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned addr = (wv * 4096 + lane * stride + shift) & 65535;
    for (int it = 0; it < iters; it++) {
        u4 v;
        if (MODE == 0) {
            __builtin_memcpy(&v, buf + addr, 16);
        } else if (MODE == 1) {
            unsigned long long w;
            __builtin_memcpy(&w, buf + addr, 8);
            v = (u4){(unsigned)w, (unsigned)(w >> 32), 0, 0};
        } else {
            unsigned w;
            __builtin_memcpy(&w, buf + (addr & ~3u), 4);
            v = (u4){w, 0, 0, 0};
        }
        acc += v.x ^ v.y ^ v.z ^ v.w;
        addr = (addr + 1024 + (acc & 0)) & 65535;
    }
    if (acc == 0x12345) out[0] = acc;
}

__global__ void oob_test(const unsigned char* in, int nrec, unsigned* o) {
    __shared__ unsigned char buf[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) buf[i] = 0xEE;
    __syncthreads();
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, nrec, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)buf, 16, threadIdx.x * 16, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int i = threadIdx.x; i < 64; i += 64) o[i] = ((unsigned*)buf)[i];
}

int main() {
    unsigned* d;
    hipMalloc(&d, 1 << 20);
    dpp_test<<<1, 64>>>(d);
    unsigned h[192];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int ok = 1;
    for (int i = 0; i < 64; i++) {
        unsigned shr = i == 0 ? 7u : 100 + i - 1, shl = i == 63 ? 7u : 100 + i + 1, shrb = i == 0 ? 0u : 100 + i - 1;
        if (h[i] != shr || h[64 + i] != shl || h[128 + i] != shrb) { ok = 0; printf("dpp lane %d: %u %u %u\n", i, h[i], h[64 + i], h[128 + i]); }
    }
    printf("dpp wave_shr/wave_shl: %s\n", ok ? "OK" : "FAIL");

    unsigned char hs[2048];
    for (int i = 0; i < 2048; i++) hs[i] = (unsigned char)(i * 37 + 11);
    unsigned char* ds;
    hipMalloc(&ds, 2048);
    hipMemcpy(ds, hs, 2048, hipMemcpyHostToDevice);
    unaligned_test<<<1, 64>>>(ds, (u4*)d);
    unsigned hu[128 * 4];
    hipMemcpy(hu, d, sizeof(hu), hipMemcpyDeviceToHost);
    ok = 1;
    for (int i = 0; i < 64; i++) {
        if (memcmp(&hu[i * 4], hs + i * 7 + 3, 16) != 0) ok = 0;
        if (memcmp(&hu[(64 + i) * 4], hs + i * 5 + 1, 8) != 0) ok = 0;
    }
    printf("unaligned ds_read_b128/b64: %s\n", ok ? "OK" : "FAIL");

    {
        unsigned char* src;
        hipMalloc(&src, 4096);
        unsigned char hb[256];
        for (int i = 0; i < 256; i++) hb[i] = (unsigned char)(i + 1);
        hipMemcpy(src, hb, 256, hipMemcpyHostToDevice);
        for (int nrec : {5, 6, 8, 17}) {
            oob_test<<<1, 64>>>(src, nrec, d);
            unsigned ho[64];
            hipMemcpy(ho, d, sizeof(ho), hipMemcpyDeviceToHost);
            printf("buffer-lds nrec=%d: bytes 0..23 =", nrec);
            for (int i = 0; i < 24; i++) printf(" %02x", ((unsigned char*)ho)[i]);
            printf("\n");
        }
    }
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 20000;
    for (int mode = 0; mode < 3; mode++)
        for (int stride : {16, 6, 1})
            for (int shift : {0, 1, 3, 4, 8}) {
                if (mode == 2 && shift) continue;
                for (int rep = 0; rep < 2; rep++) {
                    hipEventRecord(a);
                    if (mode == 0) lds_bw<0><<<256, 1024>>>(d, iters, shift, stride);
                    else if (mode == 1) lds_bw<1><<<256, 1024>>>(d, iters, shift, stride);
                    else lds_bw<2><<<256, 1024>>>(d, iters, shift, stride);
                    hipEventRecord(b);
                    hipEventSynchronize(b);
                    float ms;
                    hipEventElapsedTime(&ms, a, b);
                    double per_cu_instr = (double)iters * 16;  // wave-instructions per CU
                    if (rep)
                        printf("mode %s stride %2d shift %d: %.3f ms, %.2f ns per wave-instr per CU\n",
                               mode == 0 ? "b128" : mode == 1 ? "b64 " : "b32 ", stride, shift, ms, ms * 1e6 / per_cu_instr);
                }
            }
    return 0;
}
