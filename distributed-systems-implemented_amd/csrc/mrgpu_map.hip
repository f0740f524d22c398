// mrgpu_map.hip — Map-side kernels other than the wc pipeline (mrgpu_wc.hip):
//
// grep (MapReduce/mrapps/dgrep.go:18-36): streaming literal search (exact
//   per-byte SWAR first-byte filter, LDS verify); each hit's line (strings.Split
//   on "\n") is resolved and inserted, deduplicated by content, into the LongTable.
// wc words longer than 16 bytes (wc_long_kernel): decoded forward from their
//   start, counted in the LongTable.
// collect: the HBM tables' distinct keys -> records with partition =
//   ihash(key) % nReduce (mr/worker.go:33-37,76), appended at ctr->nrec.
#include "mrgpu_device.h"

namespace mrg {

// Words longer than 16 bytes: decode forward from the start (one lane per word).
__global__ void wc_long_kernel(const uint8_t* __restrict__ in, uint64_t n, Tables t, LetterTables lt, uint64_t nlist) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlist) return;
    const uint64_t s = t.list[i];
    uint64_t q = s, h = kFnv64Off;
    while (q < n) {
        uint32_t c0 = in[q];
        uint32_t c1 = q + 1 < n ? in[q + 1] : 0, c2 = q + 2 < n ? in[q + 2] : 0, c3 = q + 3 < n ? in[q + 3] : 0;
        int vl = utf8_valid_len(c0, c1, c2, c3);
        if (vl == 0 || !is_letter_cp(utf8_decode(c0, c1, c2, c3, vl), lt)) break;
        for (int k = 0; k < vl; k++) h = fnv1a64_step(h, in[q + k]);
        q += vl;
    }
    long_insert(t, h, in + s, q - s, 1);
}

// ------------------------------------------------------------ grep kernels
// Pattern occurrence search.  Every occurrence start p (with p + plen <= n) is
// appended to the list; grep_lines_kernel resolves its line.
__device__ __forceinline__ uint32_t eq_mask16(uint4 v, uint32_t rep) {
    // exact per-byte equality with the broadcast byte (no borrow false positives)
    uint32_t m = 0;
    uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t x = ws[k] ^ rep;
        uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;  // 0x80 where byte == 0
        m |= (((z >> 7) * 0x10204080u) >> 28) << (4 * k);
    }
    return m;
}

__global__ void __launch_bounds__(kThreads) grep_map_kernel(const uint8_t* __restrict__ in, uint64_t n, uint64_t nchunks,
                                                            const uint8_t* __restrict__ pat, uint32_t plen, Tables t) {
    __shared__ uint4 Wl[kWavesPerWG][kBuf / 16];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63;
    lds_uint4* W4 = (lds_uint4*)Wl[tid >> 6];
    const lds_u8* Wb = (const lds_u8*)W4;
    const uint32_t p0 = pat[0];
    const uint32_t rep = p0 * 0x01010101u;
    const bool in_lds = plen <= (uint32_t)kAhead;
    const uint64_t stride = (uint64_t)gridDim.x * kWavesPerWG;
    uint64_t c = (uint64_t)blockIdx.x * kWavesPerWG + (tid >> 6);
    ChunkRegs cur, nxt;
    if (c < nchunks) load_chunk(in, n, c * kChunk, lane, cur);
    for (; c < nchunks; c += stride) {
        const uint64_t cs = c * kChunk;
        if (c + stride < nchunks) load_chunk(in, n, (c + stride) * kChunk, lane, nxt);
        stage_chunk(W4, cur, lane);
        wave_sync();
        {
            uint32_t m = eq_mask16(cur.a, rep);
            const uint32_t base = 16 * lane;
            while (m) {
                const uint32_t bit = __builtin_ctz(m);
                m &= m - 1;
                const uint64_t pos = cs + base + bit;
                if (pos + plen > n) continue;
                bool ok = true;
                if (in_lds) {
                    const lds_u8* q = Wb + kBack + base + bit;
                    for (uint32_t k = 1; k < plen; k++)
                        if (q[k] != pat[k]) { ok = false; break; }
                } else {
                    for (uint32_t k = 1; k < plen; k++)
                        if (in[pos + k] != pat[k]) { ok = false; break; }
                }
                if (ok) list_append(t, pos);
            }
        }
        wave_sync();
        cur = nxt;
    }
}

// Empty pattern: every line (strings.Split yields len(sep-count)+1 lines).
__global__ void grep_all_lines_kernel(const uint8_t* __restrict__ in, uint64_t n, Tables t) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
        if (i == 0) list_append(t, 0);
        else if (in[i - 1] == '\n') list_append(t, i);
    }
}

// Resolve the line of each hit: [last '\n' before p]+1 .. next '\n' at/after p.
// plen == 0 means the list already holds line starts.
__global__ void grep_lines_kernel(const uint8_t* __restrict__ in, uint64_t n, uint32_t plen, Tables t, uint64_t nlist) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nlist) return;
    const uint64_t p = t.list[i];
    uint64_t s = p;
    if (plen > 0)
        while (s > 0 && in[s - 1] != '\n') s--;
    uint64_t e = p;
    while (e < n && in[e] != '\n') e++;
    uint64_t h = kFnv64Off;
    for (uint64_t k = s; k < e; k++) h = fnv1a64_step(h, in[k]);
    long_insert(t, h, in + s, e - s, 1);
}

// ------------------------------------------------------------ collect
// ShortTable: the occupied slots are compacted by rocprim select first
// (select_used_short), so record i is written at base + i with no shared cursor.
__global__ void collect_short_kernel(Tables t, const uint32_t* idx, const uint32_t* d_count, uint64_t base) {
    const uint64_t n = *d_count;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t o = base + i;
        if (o >= t.out_cap) { set_status(t.ctr, kStRecFull); continue; }
        const ShortSlot s = t.sh[idx[i]];
        const uint32_t len = key_len_short(s.k0, s.k1);
        t.out.k0[o] = s.k0;
        t.out.k1[o] = s.k1;
        t.out.len[o] = len;
        t.out.cnt[o] = s.count;
        t.out.part[o] = short_partition(s.k0, s.k1, len, t.nreduce);
        t.out.koff[o] = ~0ull;
    }
}

__global__ void nrec_add_kernel(Counters* ctr, const uint32_t* d_count) { ctr->nrec += *d_count; }

// LongTable (small): one wave-aggregated cursor per wave.
__global__ void collect_long_kernel(Tables t) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n = t.lo_mask + 1;
    for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += stride) {
        const uint64_t i = i0 + threadIdx.x;
        LongSlot s{0, nullptr, 0, 0};
        if (i < n) s = t.lo[i];
        const bool valid = s.hash != 0 && s.rep != nullptr && s.len != 0;
        const unsigned long long o = wave_alloc(&t.ctr->nrec, valid);
        const uint64_t len = valid ? s.len - 1 : 0;
        // arena bytes: exclusive wave scan of the lengths, one atomic per wave
        uint64_t incl = len;
        const uint32_t lane = threadIdx.x & 63;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint64_t y = __shfl_up(incl, off);
            if (lane >= (uint32_t)off) incl += y;
        }
        unsigned long long abase = 0;
        if (lane == 63 && incl) abase = atomicAdd(&t.ctr->arena, (unsigned long long)incl);
        abase = __shfl(abase, 63);
        const uint64_t nv = __popcll(__ballot(valid));
        if (lane == 0 && nv) atomicAdd(&t.ctr->nlong_rec, (unsigned long long)nv);
        if (!valid) continue;
        const unsigned long long off = abase + incl - len;
        if (o >= t.out_cap || off + len > t.out.arena_n) { set_status(t.ctr, kStRecFull); continue; }
        uint32_t h = 2166136261u;
        uint64_t k0 = 0, k1 = 0;
        for (uint64_t k = 0; k < len; k++) {
            const uint32_t b = s.rep[k];
            t.out.arena[off + k] = (uint8_t)b;
            h = fnv1a32_step(h, b);
            if (k < 8) k0 |= (uint64_t)b << (8 * k);
            else if (k < 16) k1 |= (uint64_t)b << (8 * (k - 8));
        }
        t.out.k0[o] = k0;
        t.out.k1[o] = k1;
        t.out.len[o] = (uint32_t)len;
        t.out.cnt[o] = s.count;
        t.out.part[o] = (h & 0x7fffffffu) % t.nreduce;
        t.out.koff[o] = off;
    }
}

// Re-aggregate records (merge / import / exchange receive).
__global__ void insert_recs_kernel(Recs src, Tables t) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < src.n; i += stride) {
        const uint64_t ko = src.koff[i];
        if (ko == ~0ull) {
            short_insert(t, src.k0[i], src.k1[i], src.cnt[i]);
        } else {
            const uint8_t* p = src.arena + ko;
            const uint32_t len = src.len[i];
            uint64_t h = kFnv64Off;
            for (uint32_t k = 0; k < len; k++) h = fnv1a64_step(h, p[k]);
            long_insert(t, h, p, len, src.cnt[i]);
        }
    }
}

__global__ void clear_tables_kernel(Tables t, bool short_table) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    if (short_table)
        for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= t.sh_mask; i += stride)
            t.sh[i] = ShortSlot{0, kUnwritten, 0, 0};
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= t.lo_mask; i += stride)
        t.lo[i] = LongSlot{0, nullptr, 0, 0};
}

// ------------------------------------------------------------ launchers
int map_grid_size(int device) {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || ncu <= 0) ncu = 256;
    return ncu;  // one 1024-thread workgroup per CU (LDS-bound), persistent over chunks
}

void clear_tables(const Tables& t, bool short_table, hipStream_t s) {
    hipMemsetAsync(t.ctr, 0, sizeof(Counters), s);
    if (t.bflag) hipMemsetAsync(t.bflag, 0, kSpillBuckets * sizeof(uint32_t), s);
    // spill stream lengths: a map launch writes those of its own workgroups only
    if (t.sp.counts) hipMemsetAsync(t.sp.counts, 0, (size_t)2 * kSpillBuckets * t.sp.nwg * sizeof(uint32_t), s);
    clear_tables_kernel<<<2048, 256, 0, s>>>(t, short_table);
}

void launch_wc_long(const uint8_t* in, uint64_t n, const Tables& t, LetterTables lt, uint64_t nlist, hipStream_t s) {
    if (nlist == 0) return;
    wc_long_kernel<<<(unsigned)((nlist + 255) / 256), 256, 0, s>>>(in, n, t, lt, nlist);
}

void launch_grep_map(const uint8_t* in, uint64_t n, const uint8_t* d_pat, uint32_t plen, const Tables& t, int grid,
                     hipStream_t s) {
    const uint64_t nchunks = (n + kChunk - 1) / kChunk;
    if (nchunks == 0 || plen == 0) return;
    uint64_t g = (nchunks + kWavesPerWG - 1) / kWavesPerWG;
    const uint64_t gmax = (uint64_t)grid * 4;
    if (g > gmax) g = gmax;
    grep_map_kernel<<<(unsigned)g, kThreads, 0, s>>>(in, n, nchunks, d_pat, plen, t);
}

void launch_grep_all_lines(const uint8_t* in, uint64_t n, const Tables& t, int grid, hipStream_t s) {
    grep_all_lines_kernel<<<grid * 4, 256, 0, s>>>(in, n, t);
}

void launch_grep_lines(const uint8_t* in, uint64_t n, uint32_t plen, const Tables& t, uint64_t nlist, hipStream_t s) {
    if (nlist == 0) return;
    grep_lines_kernel<<<(unsigned)((nlist + 255) / 256), 256, 0, s>>>(in, n, plen, t, nlist);
}

int launch_collect(const Tables& t, ReduceWs* ws, uint64_t base, uint64_t short_used, bool long_table, hipStream_t s) {
    if (short_used) {
        uint32_t *idx = nullptr, *cnt = nullptr;
        const int e = select_used_short(ws, t.sh, t.sh_mask + 1, short_used, &idx, &cnt, s);
        if (e) return e;
        uint64_t g = (short_used + 255) / 256;
        if (g > 2048) g = 2048;
        collect_short_kernel<<<(unsigned)g, 256, 0, s>>>(t, idx, cnt, base);
        nrec_add_kernel<<<1, 1, 0, s>>>(t.ctr, cnt);
    }
    if (long_table) collect_long_kernel<<<256, 256, 0, s>>>(t);
    return (int)hipGetLastError();
}

void launch_insert_recs(const Recs& src, const Tables& t, hipStream_t s) {
    if (src.n == 0) return;
    uint64_t g = (src.n + 255) / 256;
    if (g > 4096) g = 4096;
    insert_recs_kernel<<<(unsigned)g, 256, 0, s>>>(src, t);
}

}  // namespace mrg
