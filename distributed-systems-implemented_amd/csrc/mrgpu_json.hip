// mrgpu_json.hip — the reference's intermediate file format on the GPU
// (SURVEY.md §8(f) rank 3): mr-X-Y files as MapReduce/mr/worker.go:80-92 writes
// them, so a GPU map worker's output can be read by an unmodified reference
// reduce worker (worker.go:100-122).
//
// worker.go:84-86 encodes every KeyValue of bucket Y with
// json.NewEncoder(f).Encode(&kv): one line {"Key":"<k>","Value":"<v>"}\n per key
// OCCURRENCE (wc: Value "1", once per word; grep: Value "", once per matching
// line).  A parts record holds a distinct key with its count, so its line is
// written count times.  String escaping restates encoding/json's
// encodeState.string with escapeHTML = true (the Encoder default) as of Go
// 1.16-1.21, the versions SURVEY.md §8c pins (Go 1.22 added the short \b, \f
// forms; before it they are \u0008, \u000c):
//   - ASCII: '"' and '\\' get a backslash; \n \r \t their short escapes; other
//     bytes < 0x20 and '<' '>' '&' become \u00XX (lowercase hex); the rest as is;
//   - UTF-8 (utf8.DecodeRuneInString): an invalid byte becomes \ufffd (it is
//     decoded as RuneError of width 1); U+2028 / U+2029 become \u2028 / \u2029;
//     any other rune is copied.
// Pipeline: per record the escaped line length L and the output bytes L*count
// -> exclusive scans -> one escaped copy of each line in a line buffer -> the
// output is filled in 4 KiB pieces, one wave per piece (a record of a hot key
// spans many pieces, so a count of 1e8 is spread over the whole GPU).
#include "mrgpu_device.h"

#include <cstring>

#include "mrgpu_scan.h"

namespace mrg {

constexpr uint32_t kJsonPiece = 4096;
constexpr uint32_t kJsonHead = 8;   // {"Key":"
constexpr uint32_t kJsonMid = 11;   // ","Value":"
constexpr uint32_t kJsonTail = 3;   // "}\n

__device__ __forceinline__ uint8_t key_byte(const Recs& r, uint32_t j, uint32_t k) {
    if (r.koff[j] != ~0ull) return r.arena[r.koff[j] + k];
    return (uint8_t)((k < 8 ? r.k0[j] : r.k1[j]) >> (8 * (k & 7)));
}

// Width of the valid UTF-8 sequence starting at byte k (Go's accept ranges,
// SURVEY.md Appendix A.1), or 0 when the byte decodes to RuneError of width 1.
__device__ uint32_t utf8_width(const Recs& r, uint32_t j, uint32_t k, uint32_t len, uint32_t* rune) {
    const uint32_t b0 = key_byte(r, j, k);
    uint32_t w, lo = 0x80, hi = 0xBF, cp;
    if (b0 >= 0xC2 && b0 <= 0xDF) { w = 2; cp = b0 & 0x1F; }
    else if (b0 >= 0xE0 && b0 <= 0xEF) {
        w = 3; cp = b0 & 0x0F;
        if (b0 == 0xE0) lo = 0xA0;
        if (b0 == 0xED) hi = 0x9F;
    } else if (b0 >= 0xF0 && b0 <= 0xF4) {
        w = 4; cp = b0 & 0x07;
        if (b0 == 0xF0) lo = 0x90;
        if (b0 == 0xF4) hi = 0x8F;
    } else {
        return 0;
    }
    if (k + w > len) return 0;
    for (uint32_t i = 1; i < w; i++) {
        const uint32_t b = key_byte(r, j, k + i);
        if (b < (i == 1 ? lo : 0x80u) || b > (i == 1 ? hi : 0xBFu)) return 0;
        cp = (cp << 6) | (b & 0x3F);
    }
    *rune = cp;
    return w;
}

// Escaped form of the key's byte run starting at k: writes it to o (if not
// null) and returns (escaped bytes, input bytes consumed) packed as hi/lo.
__device__ uint64_t json_escape_step(const Recs& r, uint32_t j, uint32_t k, uint32_t len, uint8_t* o) {
    const char* hex = "0123456789abcdef";
    const uint32_t b = key_byte(r, j, k);
    if (b < 0x80) {
        const bool safe = b >= 0x20 && b != '"' && b != '\\' && b != '<' && b != '>' && b != '&';
        if (safe) {
            if (o) o[0] = (uint8_t)b;
            return (1ull << 32) | 1;
        }
        if (b == '"' || b == '\\' || b == '\n' || b == '\r' || b == '\t') {
            if (o) {
                o[0] = '\\';
                o[1] = b == '\n' ? 'n' : b == '\r' ? 'r' : b == '\t' ? 't' : (uint8_t)b;
            }
            return (2ull << 32) | 1;
        }
        if (o) {
            o[0] = '\\'; o[1] = 'u'; o[2] = '0'; o[3] = '0';
            o[4] = (uint8_t)hex[b >> 4]; o[5] = (uint8_t)hex[b & 15];
        }
        return (6ull << 32) | 1;
    }
    uint32_t cp = 0;
    const uint32_t w = utf8_width(r, j, k, len, &cp);
    if (w == 0 || cp == 0x2028 || cp == 0x2029) {  // \ufffd, \u2028, \u2029
        if (o) {
            o[0] = '\\'; o[1] = 'u';
            const uint32_t v = w == 0 ? 0xFFFDu : cp;
            o[2] = (uint8_t)hex[(v >> 12) & 15]; o[3] = (uint8_t)hex[(v >> 8) & 15];
            o[4] = (uint8_t)hex[(v >> 4) & 15]; o[5] = (uint8_t)hex[v & 15];
        }
        return (6ull << 32) | (w == 0 ? 1u : w);
    }
    if (o)
        for (uint32_t i = 0; i < w; i++) o[i] = key_byte(r, j, k + i);
    return ((uint64_t)w << 32) | w;
}

__device__ __forceinline__ uint32_t json_value_len(int app) { return app == 1 ? 1u : 0u; }

// L[i] = line bytes, T[i] = L[i] * count, P[i] = 4 KiB pieces of T[i]
__global__ void json_len_kernel(Recs r, int app, uint64_t* L, uint64_t* T, uint64_t* P) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.n; i += stride) {
        const uint32_t j = (uint32_t)i, len = r.len[j];
        uint64_t e = 0;
        for (uint32_t k = 0; k < len;) {
            const uint64_t st = json_escape_step(r, j, k, len, nullptr);
            e += st >> 32;
            k += (uint32_t)st;
        }
        const uint64_t l = kJsonHead + e + kJsonMid + json_value_len(app) + kJsonTail;
        L[i] = l;
        T[i] = l * r.cnt[j];
        P[i] = (T[i] + kJsonPiece - 1) / kJsonPiece;
    }
}

__global__ void json_line_kernel(Recs r, int app, const uint64_t* loff, uint8_t* lines) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < r.n; i += stride) {
        const uint32_t j = (uint32_t)i, len = r.len[j];
        uint8_t* o = lines + loff[i];
        const char* head = "{\"Key\":\"";
        const char* mid = "\",\"Value\":\"";
        for (uint32_t q = 0; q < kJsonHead; q++) *o++ = (uint8_t)head[q];
        for (uint32_t k = 0; k < len;) {
            const uint64_t st = json_escape_step(r, j, k, len, o);
            o += st >> 32;
            k += (uint32_t)st;
        }
        for (uint32_t q = 0; q < kJsonMid; q++) *o++ = (uint8_t)mid[q];
        if (app == 1) *o++ = '1';
        *o++ = '"';
        *o++ = '}';
        *o++ = '\n';
    }
}

// One wave per 4 KiB piece: piece q belongs to the record i with
// poff[i] <= q < poff[i] + P[i]; output byte p of record i is byte
// (p - toff[i]) % L[i] of its line.
__global__ void json_fill_kernel(const uint64_t* L, const uint64_t* loff, const uint64_t* toff, const uint64_t* poff,
                                 uint64_t n, uint64_t npieces, uint64_t total, const uint8_t* lines, uint8_t* out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x / 64);
    for (uint64_t q = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); q < npieces; q += nw) {
        uint64_t lo = 0, hi = n;  // last record with poff <= q
        while (hi - lo > 1) {
            const uint64_t m = (lo + hi) >> 1;
            if (poff[m] <= q) lo = m; else hi = m;
        }
        const uint64_t i = lo, l = L[i];
        const uint64_t rec_end = i + 1 < n ? toff[i + 1] : total;
        const uint64_t p0 = toff[i] + (q - poff[i]) * kJsonPiece;
        const uint64_t p1 = p0 + kJsonPiece < rec_end ? p0 + kJsonPiece : rec_end;
        const uint8_t* line = lines + loff[i];
        uint64_t x = (p0 - toff[i] + lane) % l;  // position in the line, advanced by 64 per step
        const uint64_t adv = 64 % l;
        for (uint64_t p = p0 + lane; p < p1; p += 64) {
            out[p] = line[x];
            x += adv;
            if (x >= l) x -= l;
        }
    }
}

// Exclusive scan of n u64 values with the tiles chained by decoupled look-back
// (mrgpu_scan.h); the look-back state lives in `scratch` (cleared per scan: the
// JSON export is not a hot path).
__global__ void __launch_bounds__(kScanThreads) scan_u64_kernel(const uint64_t* __restrict__ in,
                                                                uint64_t* __restrict__ out, uint64_t n, ScanState st) {
    __shared__ unsigned long long red[kScanThreads / 64];
    __shared__ unsigned long long pre;
    __shared__ uint32_t tile_w;
    const uint32_t t = scan_take_tile(st, &tile_w);
    const uint64_t i0 = (uint64_t)t * kScanTile + (uint64_t)threadIdx.x * kScanPer;
    uint64_t v[kScanPer];
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++) {
        v[k] = i0 + k < n ? in[i0 + k] : 0ull;
        sum += v[k];
    }
    uint64_t tot;
    const uint64_t ex = block_excl_scan_u64(sum, red, &tot);
    if (threadIdx.x < 64) {
        const uint64_t p = scan_lookback(st, t, tot);
        if (threadIdx.x == 0) pre = p;
    }
    __syncthreads();
    uint64_t o = pre + ex;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; k++) {
        if (i0 + k < n) out[i0 + k] = o;
        o += v[k];
    }
}

static int excl_scan(void*& tmp, size_t& tmp_bytes, const uint64_t* in, uint64_t* out, uint64_t n, hipStream_t s,
                     void* (*grow)(void* ctx, size_t), void* gctx) {
    const uint64_t ntiles = (n + kScanTile - 1) / kScanTile;
    const size_t need = ntiles * 8 + 64;
    if (need > tmp_bytes) {
        tmp = grow(gctx, need);
        if (!tmp) return -1;
        tmp_bytes = need;
    }
    if (hipMemsetAsync(tmp, 0, need, s) != hipSuccess) return -1;
    ScanState st{(unsigned long long*)((char*)tmp + 64), (uint32_t*)tmp, 1u, (uint32_t)ntiles};
    scan_u64_kernel<<<(unsigned)ntiles, kScanThreads, 0, s>>>(in, out, n, st);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int json_lengths(const Recs& r, int app, uint64_t* L, uint64_t* T, uint64_t* P, uint64_t* loff, uint64_t* toff,
                 uint64_t* poff, void* (*grow)(void*, size_t), void* gctx, hipStream_t s) {
    if (r.n == 0) return 0;
    const unsigned g = (unsigned)((r.n + 255) / 256 < 4096 ? (r.n + 255) / 256 : 4096);
    json_len_kernel<<<g, 256, 0, s>>>(r, app, L, T, P);
    void* tmp = nullptr;
    size_t tb = 0;
    if (excl_scan(tmp, tb, L, loff, r.n, s, grow, gctx) || excl_scan(tmp, tb, T, toff, r.n, s, grow, gctx) ||
        excl_scan(tmp, tb, P, poff, r.n, s, grow, gctx))
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int json_write(const Recs& r, int app, const uint64_t* L, const uint64_t* loff, const uint64_t* toff,
               const uint64_t* poff, uint64_t npieces, uint64_t total, uint8_t* lines, uint8_t* out, hipStream_t s) {
    if (r.n == 0) return 0;
    const unsigned g = (unsigned)((r.n + 255) / 256 < 4096 ? (r.n + 255) / 256 : 4096);
    json_line_kernel<<<g, 256, 0, s>>>(r, app, loff, lines);
    if (npieces) {
        const uint64_t blocks = (npieces + 3) / 4;
        json_fill_kernel<<<(unsigned)(blocks < 8192 ? blocks : 8192), 256, 0, s>>>(L, loff, toff, poff, r.n, npieces,
                                                                                  total, lines, out);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace mrg
