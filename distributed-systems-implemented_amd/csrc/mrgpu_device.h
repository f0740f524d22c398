// mrgpu_device.h — device-side building blocks shared by the map-side kernels
// (mrgpu_map.hip: grep / long words / collect; mrgpu_wc.hip: the wc pipeline).
//
// Reference semantics reproduced here (paths under /root/reference/MapReduce):
//   * UTF-8 decoding of Go's `for i, r := range s` inside strings.FieldsFunc
//     (mrapps/wc.go:26): utf8.DecodeRune acceptance ranges, an invalid byte is
//     U+FFFD of width 1;
//   * unicode.IsLetter (mrapps/wc.go:23), Unicode 13.0.0, via a two-level bitmap;
//   * ihash = FNV-1a-32 & 0x7fffffff (mr/worker.go:33-37).
#pragma once
#include "mrgpu_internal.h"

namespace mrg {

constexpr int kChunk = 1024;                      // bytes per wave-chunk (16 B per lane)
constexpr int kBack = 16;                         // look-back halo (UTF-8 rune starts, word starts)
constexpr int kAhead = 64;                        // look-ahead halo (word lengths, UTF-8 tails)
constexpr int kBuf = kBack + kChunk + kAhead;     // 1104, multiple of 16
constexpr int kWavesPerWG = 16;
constexpr int kThreads = kWavesPerWG * kWave;
constexpr int kListCap = kChunk / 2;              // max word starts in a chunk
constexpr int kGlobalProbes = 4096;

// Explicit LDS address-space views.  Through a generic pointer hipcc emits
// flat_load ... + s_waitcnt vmcnt(0) lgkmcnt(0), i.e. every LDS access would also
// wait for the wave's outstanding HBM loads and stores.
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) unsigned long long lds_u64;
typedef __attribute__((address_space(3))) u64x2 lds_u64x2;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) u32x4 lds_uint4;  // 16-byte LDS unit (HIP's uint4 has no addrspace operator=)
__device__ __forceinline__ u32x4 to_v4(uint4 a) { return (u32x4){a.x, a.y, a.z, a.w}; }
__device__ __forceinline__ uint4 from_v4(u32x4 a) { return make_uint4(a.x, a.y, a.z, a.w); }

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ const uint8_t* ld_agent_ptr(const uint8_t* const* p) {
    return __hip_atomic_load(const_cast<const uint8_t**>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void set_status(Counters* c, uint32_t bits) { atomicOr(&c->status, bits); }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A 64-bit value of lane j (uniform j).  The readlane builtins return int: each
// half goes through uint32_t, or a low word with bit 31 set sign-extends over the
// high one.
__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t j) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)j);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)j);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readfirstlane64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Exclusive prefix sum over the wave of c (0 <= c < 2^BITS) by ballot bit-planes.
template <int BITS>
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t c, uint32_t* total) {
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < BITS; k++) {
        const uint64_t b = __ballot((c >> k) & 1u);
        base += mbcnt64(b) << k;
        tot += (uint32_t)__popcll(b) << k;
    }
    *total = tot;
    return base;
}

// Inclusive prefix sum over the wave by DPP (gfx9 row_shr 1/2/4/8 within 16-lane
// rows, then row_bcast 15 / 31 across rows): 6 adds, against ballot bit-planes'
// 2 VALU + 2 mbcnt per bit.  Lanes whose DPP source is outside the row read the
// old value 0.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t v) {
    v += __builtin_amdgcn_mov_dpp(v, 0x111, 0xF, 0xF, true);  // row_shr:1 (BOUND_CTRL: 0 from outside the row)
    v += __builtin_amdgcn_mov_dpp(v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += __builtin_amdgcn_mov_dpp(v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += __builtin_amdgcn_mov_dpp(v, 0x118, 0xF, 0xF, true);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// One wave-wide atomicAdd for the lanes with `want` set; returns each such
// lane's slot (base + rank among the wanting lanes).  Replaces one same-address
// atomic per lane (which serialises at the memory side) by one per wave.
__device__ __forceinline__ unsigned long long wave_alloc(unsigned long long* ctr, bool want) {
    const uint64_t m = __ballot(want);
    if (m == 0) return 0;
    const uint32_t leader = __builtin_ctzll(m);
    unsigned long long base = 0;
    if (lane_id() == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(m));
    base = __shfl(base, (int)leader);
    return base + mbcnt64(m);
}

// Sum over the wave (every lane gets it).
__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Add each thread's v0..v3 to ctr[0..3] with ONE atomic per workgroup per
// counter.  Same-address device atomics serialise at the memory side (~12 ns
// each, MI355X_MICROARCH.md fan-in row): a per-thread atomic from every thread
// of a 256-workgroup grid costs milliseconds.  Call from every thread of the
// block (it synchronises); scratch = 4 * (waves per block) u64 of LDS.
template <int NWAVES>
__device__ __forceinline__ void block_add4(unsigned long long* c0, unsigned long long* c1, unsigned long long* c2,
                                           unsigned long long* c3, uint64_t v0, uint64_t v1, uint64_t v2, uint64_t v3,
                                           unsigned long long* scratch) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    v0 = wave_sum(v0); v1 = wave_sum(v1); v2 = wave_sum(v2); v3 = wave_sum(v3);
    if (lane == 0) {
        scratch[4 * wv + 0] = v0; scratch[4 * wv + 1] = v1; scratch[4 * wv + 2] = v2; scratch[4 * wv + 3] = v3;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        uint64_t s = 0;
        for (int w = 0; w < NWAVES; w++) s += scratch[4 * w + threadIdx.x];
        unsigned long long* c = threadIdx.x == 0 ? c0 : threadIdx.x == 1 ? c1 : threadIdx.x == 2 ? c2 : c3;
        if (s && c) atomicAdd(c, (unsigned long long)s);
    }
    __syncthreads();
}

// Block-wide slot allocation: each thread wants `mine` consecutive slots of a
// shared cursor; returns the first of them.  One atomic per workgroup.
// scratch = NWAVES + 1 u64 of LDS.  Call from every thread of the block.
template <int NWAVES>
__device__ __forceinline__ unsigned long long block_alloc(unsigned long long* ctr, uint32_t mine,
                                                          unsigned long long* scratch) {
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t incl = mine;  // inclusive wave scan
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off);
        if (lane >= (uint32_t)off) incl += y;
    }
    if (lane == 63) scratch[wv] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long run = 0;
        for (int w = 0; w < NWAVES; w++) {
            const unsigned long long x = scratch[w];
            scratch[w] = run;
            run += x;
        }
        scratch[NWAVES] = run ? atomicAdd(ctr, run) : 0ull;
    }
    __syncthreads();
    const unsigned long long base = scratch[NWAVES] + scratch[wv] + (incl - mine);
    __syncthreads();
    return base;
}

// DPP whole-wave lane shifts (gfx9 wave_shr:1 / wave_shl:1; lanes shifted in
// from outside the wave read `fill`).
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v, uint32_t fill) {
    return __builtin_amdgcn_update_dpp(fill, v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v, uint32_t fill) {
    return __builtin_amdgcn_update_dpp(fill, v, 0x130, 0xf, 0xf, false);
}
// The same with 0 shifted in, by BOUND_CTRL (no copy of a fill value first).
__device__ __forceinline__ uint32_t wave_shr1_z(uint32_t v) { return __builtin_amdgcn_mov_dpp(v, 0x138, 0xf, 0xf, true); }
__device__ __forceinline__ uint32_t wave_shl1_z(uint32_t v) { return __builtin_amdgcn_mov_dpp(v, 0x130, 0xf, 0xf, true); }

// 4 ASCII bytes -> 4-bit letter mask ([A-Za-z]); requires every byte < 0x80.
__device__ __forceinline__ uint32_t ascii_letters4(uint32_t x) {
    const uint32_t y = x | 0x20202020u;
    const uint32_t t = (y + 0x1F1F1F1Fu) & ~(y + 0x05050505u) & 0x80808080u;
    return ((t >> 7) * 0x10204080u) >> 28;
}
// 0x80 in each [A-Za-z] byte of 4 ASCII bytes, else 0 (the SWAR test above, the
// three-input and as one v_bitop3_b32: a & ~b & c = truth table 0x20).
__device__ __forceinline__ uint32_t ascii_flags4(uint32_t x) {
    const uint32_t y = x | 0x20202020u;
    return __builtin_amdgcn_bitop3_b32(y + 0x1F1F1F1Fu, y + 0x05050505u, 0x80808080u, 0x20);
}
// 16 ASCII bytes -> 16-bit letter mask.  The flag bytes are gathered by byte dot
// products (v_dot4_u32_u8) with weights 1,2,4,8 / 16,32,64,128: the 8-bit masks
// of two dwords, times 0x80, in one accumulate chain; no 32-bit multiplies.
__device__ __forceinline__ uint32_t ascii_mask16(uint4 v) {
    const uint32_t lo = __builtin_amdgcn_udot4(ascii_flags4(v.y), 0x80402010u,
                                               __builtin_amdgcn_udot4(ascii_flags4(v.x), 0x08040201u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(ascii_flags4(v.w), 0x80402010u,
                                               __builtin_amdgcn_udot4(ascii_flags4(v.z), 0x08040201u, 0u, false), false);
    return (lo | (hi << 8)) >> 7;
}

__device__ __forceinline__ bool is_letter_cp(uint32_t cp, LetterTables lt) {
    if (cp < 0x80) return ((cp | 0x20u) - 0x61u) < 26u;
    const uint32_t idx = lt.l1[cp >> 8];
    return (lt.l2[idx * 8 + ((cp >> 5) & 7)] >> (cp & 31)) & 1u;
}

// Go utf8 acceptance: length of the valid sequence starting with bytes c0..c3, or 0.
__device__ __forceinline__ int utf8_valid_len(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    if (c0 < 0x80) return 1;
    if (c0 < 0xC2 || c0 > 0xF4) return 0;
    uint32_t lo = 0x80, hi = 0xBF;
    if (c0 == 0xE0) lo = 0xA0;
    else if (c0 == 0xED) hi = 0x9F;
    else if (c0 == 0xF0) lo = 0x90;
    else if (c0 == 0xF4) hi = 0x8F;
    if (c1 < lo || c1 > hi) return 0;
    if (c0 < 0xE0) return 2;
    if ((c2 & 0xC0) != 0x80) return 0;
    if (c0 < 0xF0) return 3;
    if ((c3 & 0xC0) != 0x80) return 0;
    return 4;
}

__device__ __forceinline__ uint32_t utf8_decode(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, int n) {
    if (n == 1) return c0;
    if (n == 2) return ((c0 & 0x1F) << 6) | (c1 & 0x3F);
    if (n == 3) return ((c0 & 0x0F) << 12) | ((c1 & 0x3F) << 6) | (c2 & 0x3F);
    return ((c0 & 0x07) << 18) | ((c1 & 0x3F) << 12) | ((c2 & 0x3F) << 6) | (c3 & 0x3F);
}

// Letter mask of the W bytes at b[q0 .. q0+W) with Go decoding semantics.
// Needs b[q0-6 .. q0+W+3) addressable (zeros outside the input act as
// non-continuation terminators, matching Go's truncated-sequence rule).
// Rune starts use the local rule: byte q starts a rune unless a valid sequence
// of length > k starts at q-k, k in {1,2,3}.
template <int W, typename P>
__device__ uint32_t utf8_letter_mask(P b, int q0, LetterTables lt) {
    uint32_t mask = 0;
    int vl1 = 0, vl2 = 0, vl3 = 0;  // valid lengths at q-1, q-2, q-3
    for (int q = q0 - 6; q < q0 + W; q++) {
        const uint32_t c0 = b[q], c1 = b[q + 1], c2 = b[q + 2], c3 = b[q + 3];
        const int vl = utf8_valid_len(c0, c1, c2, c3);
        if (q >= q0 - 3) {
            const bool start = !(vl1 >= 2 || vl2 >= 3 || vl3 >= 4);
            if (start) {
                const bool let = vl > 0 && is_letter_cp(utf8_decode(c0, c1, c2, c3, vl), lt);
                if (let) {
                    for (int k = 0; k < vl; k++) {
                        const int pos = q + k - q0;
                        if (pos >= 0 && pos < W) mask |= 1u << pos;
                    }
                }
            }
        }
        vl3 = vl2; vl2 = vl1; vl1 = vl;
    }
    return mask;
}

// ---------------------------------------------------------------- UTF-8 letter mask (LDS tables)
typedef __attribute__((address_space(3))) uint32_t lds_u32_unaligned __attribute__((aligned(1)));
struct LdsLetters {
    const lds_u8* l1;   // [kLetterLdsPages]
    const lds_u32* l2;  // [kLetterUnique * 8]
    const lds_u32* b2;  // letters among code points < U+0800 (every 2-byte rune): 2048 bits, one read
                        // per rune instead of l1 + l2 (nullptr: l1 / l2 only)
};
__device__ __forceinline__ bool is_letter_lds(uint32_t cp, LdsLetters L) {
    if (cp >= ((uint32_t)kLetterLdsPages << 8)) return false;
    const uint32_t idx = L.l1[cp >> 8];
    return (L.l2[idx * 8 + ((cp >> 5) & 7)] >> (cp & 31)) & 1u;
}

// 0x80 in each byte of x that is an ASCII letter [A-Za-z] (any byte values)
__device__ __forceinline__ uint32_t ascii_flags4_any(uint32_t x) { return ascii_flags4(x & 0x7F7F7F7Fu) & ~x; }
// 0x80 in each byte >= 0xC0 (a UTF-8 lead byte or an invalid one; validated later)
__device__ __forceinline__ uint32_t lead_flags4(uint32_t x) { return x & (x << 1) & 0x80808080u; }
// four flag dwords (0x80 per flagged byte) -> 16-bit mask, byte k of dword d -> bit 4d + k
__device__ __forceinline__ uint32_t flags_to_bits16(uint32_t f0, uint32_t f1, uint32_t f2, uint32_t f3) {
    const uint32_t lo = __builtin_amdgcn_udot4(f1, 0x80402010u, __builtin_amdgcn_udot4(f0, 0x08040201u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(f3, 0x80402010u, __builtin_amdgcn_udot4(f2, 0x08040201u, 0u, false), false);
    return (lo | (hi << 8)) >> 7;
}

// One lead byte's rune (Go's acceptance ranges):
// lead_decode gives the code point, its continuation count and validity from the
// rune's 4 bytes w; lead_word the table word holding its letter bit.
struct LeadRune {
    uint32_t cp, need;
    bool valid;
};
__device__ __forceinline__ LeadRune lead_decode(uint32_t w) {
    const uint32_t c0 = w & 0xFFu, c1 = (w >> 8) & 0xFFu, c2 = (w >> 16) & 0xFFu, c3 = w >> 24;
    const uint32_t need = c0 >= 0xF0u ? 3u : c0 >= 0xE0u ? 2u : 1u;  // continuation bytes
    const uint32_t lo = c0 == 0xE0u ? 0xA0u : c0 == 0xF0u ? 0x90u : 0x80u;
    const uint32_t hi = c0 == 0xEDu ? 0x9Fu : c0 == 0xF4u ? 0x8Fu : 0xBFu;
    const bool valid = c0 >= 0xC2u && c0 <= 0xF4u && c1 >= lo && c1 <= hi && (need < 2u || (c2 & 0xC0u) == 0x80u) &&
                       (need < 3u || (c3 & 0xC0u) == 0x80u);
    const uint32_t cp = need == 1u ? ((c0 & 0x1Fu) << 6) | (c1 & 0x3Fu)
                      : need == 2u ? ((c0 & 0x0Fu) << 12) | ((c1 & 0x3Fu) << 6) | (c2 & 0x3Fu)
                                   : ((c0 & 0x07u) << 18) | ((c1 & 0x3Fu) << 12) | ((c2 & 0x3Fu) << 6) | (c3 & 0x3Fu);
    return LeadRune{cp, need, valid};
}
// the table word of cp's letter bit (bit cp & 31): a 2-byte rune by one read of
// the 2048-bit table, a longer one by the two-level l1 / l2 tables
__device__ __forceinline__ uint32_t lead_word(const LeadRune& r, LdsLetters L) {
    if (r.need == 1u && L.b2) return L.b2[r.cp >> 5];
    if (r.cp >= ((uint32_t)kLetterLdsPages << 8)) return 0u;
    return L.l2[L.l1[r.cp >> 8] * 8u + ((r.cp >> 5) & 7u)];
}

// Letter mask of the 16 slot bytes [q0, q0 + 16) with Go's decoding semantics
// (strings.FieldsFunc's range loop + unicode.IsLetter, mrapps/wc.go:23,26;
// SURVEY.md Appendix A.1), for a slot in LDS whose bytes [q0 - 4, q0 + 19) are
// readable:
//   - ASCII letters by SWAR;
//   - every lead byte (>= 0xC0) in [q0 - 3, q0 + 16) starts a rune: a lead is
//     never a continuation byte, so no valid sequence can cover it (the local
//     rune-start rule always holds); its sequence is checked with Go's
//     acceptance ranges and, if valid and a letter, marks all its bytes;
//   - continuation bytes outside a valid sequence and invalid leads are
//     U+FFFD, not letters (nothing to do).
// Work is one loop turn per lead byte of the lane (a two-leads-per-turn version
// measured slower: C2u map 23.0 vs 18.3 ms).  first: the look-back lane (q0 =
// 0), whose bytes before the slot read as 0 (only its bit 15 is used, which
// depends on bytes >= 9).
__device__ __forceinline__ uint32_t utf8_mask16(const lds_u8* slot, uint32_t q0, bool first, LdsLetters L) {
    const lds_u32* s4 = (const lds_u32*)(slot + q0);
    const uint32_t w0 = first ? 0u : s4[-1], w1 = s4[0], w2 = s4[1], w3 = s4[2], w4 = s4[3];
    uint32_t m = flags_to_bits16(ascii_flags4_any(w1), ascii_flags4_any(w2), ascii_flags4_any(w3), ascii_flags4_any(w4));
    // lead bytes at positions q0 - 3 + i, i = 0..18 (bits 0-2: bytes 1-3 of w0)
    uint32_t leads = (flags_to_bits16(lead_flags4(w0), lead_flags4(w1), lead_flags4(w2), lead_flags4(w3)) >> 1) |
                     (flags_to_bits16(lead_flags4(w4), 0u, 0u, 0u) << 15);
    while (leads) {
        const uint32_t i = __builtin_ctz(leads);
        leads &= leads - 1;
        const LeadRune r = lead_decode(*(const lds_u32_unaligned*)(slot + q0 + i - 3));
        const uint32_t tw = lead_word(r, L);
        if (r.valid && ((tw >> (r.cp & 31u)) & 1u)) m |= ((((2u << r.need) - 1u) << i) >> 3) & 0xFFFFu;
    }
    return m;
}

// Wave-compacted utf8_mask16 for the whole 1 KiB window (lane l: slot bytes
// [16 l, 16 l + 16)).  The serial loop above runs as many turns as the lane
// with the most leads (a lane of Greek or Cyrillic text has 8), the others
// idle; here every lead of the window is listed once, by the lane holding it
// (prefix scan of the lanes' counts), and the list is decoded one lead per lane
// per pass; a letter rune ORs its bits into its lane's mask word in LDS, and
// into the next lane's when it runs past the lane's 16 bytes.  scratch: 1 KiB
// of LDS free during the call (leads as u16 at [0, 768), the 64 masks at
// [768, 1024)); more than 384 leads: the serial loop.  Wave-uniform call.
constexpr uint32_t kWaveLeads = 384;
__device__ __forceinline__ uint32_t utf8_mask16_wave(const lds_u8* slot, uint32_t lane, lds_u8* scratch, LdsLetters L) {
    const uint32_t q0 = 16 * lane;
    const lds_u32* s4 = (const lds_u32*)(slot + q0);
    const uint32_t w1 = s4[0], w2 = s4[1], w3 = s4[2], w4 = s4[3];
    const uint32_t m = flags_to_bits16(ascii_flags4_any(w1), ascii_flags4_any(w2), ascii_flags4_any(w3), ascii_flags4_any(w4));
    uint32_t own = flags_to_bits16(lead_flags4(w1), lead_flags4(w2), lead_flags4(w3), lead_flags4(w4));
    const uint32_t nown = __popc(own);
    const uint32_t incl = wave_incl_scan_dpp(nown);
    const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
    if (total > kWaveLeads) return utf8_mask16(slot, q0, lane == 0, L);
    lds_u16* lst = (lds_u16*)scratch;
    lds_u32* M = (lds_u32*)(scratch + 2 * kWaveLeads);
    M[lane] = 0u;
    uint32_t j = incl - nown;
    while (own) {  // two leads per turn
        const uint32_t b1 = __builtin_ctz(own);
        own &= own - 1;
        lst[j] = (uint16_t)(q0 + b1);
        if (own) lst[j + 1] = (uint16_t)(q0 + __builtin_ctz(own));
        own &= own - 1;
        j += 2;
    }
    wave_sync();
    auto mark = [&](uint32_t e, const LeadRune& r, uint32_t tw) {
        if (r.valid && ((tw >> (r.cp & 31u)) & 1u)) {
            const uint32_t bits = ((2u << r.need) - 1u) << (e & 15u);  // up to bit 18
            const uint32_t ow = e >> 4;
            __hip_atomic_fetch_or(&M[ow], bits & 0xFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if ((bits >> 16) != 0u && ow < 63u)
                __hip_atomic_fetch_or(&M[ow + 1], bits >> 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    for (uint32_t p = 0; p < total; p += 64) {
        if (p + lane < total) {
            const uint32_t e = lst[p + lane];
            const LeadRune r = lead_decode(*(const lds_u32_unaligned*)(slot + e));
            mark(e, r, lead_word(r, L));
        }
    }
    wave_sync();
    return m | M[lane];
}

// 32-bit mix of a <= 16-byte key given as four little-endian words.
__device__ __forceinline__ uint32_t fold32(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    // (three-input xor as one v_bitop3_b32, truth table 0x96; same value as the plain xors)
    const uint32_t x = __builtin_amdgcn_bitop3_b32(w0, __builtin_rotateleft32(w1, 7), __builtin_rotateleft32(w2, 13), 0x96) ^
                       __builtin_rotateleft32(w3, 21);
    return x * 0x9E3779B1u;
}

__device__ __forceinline__ uint64_t short_hash64(uint64_t k0, uint64_t k1) {
    const uint64_t h = (k0 ^ (k1 * 0x9E3779B97F4A7C15ull)) * 0xD6E8FEB86659FD93ull;
    return h ^ (h >> 32);
}

__device__ __forceinline__ uint64_t fnv1a64_step(uint64_t h, uint32_t b) { return (h ^ b) * 1099511628211ull; }
constexpr uint64_t kFnv64Off = 14695981039346656037ull;

// Byte length of a zero-padded key of at most 16 bytes (letters are never 0x00).
__device__ __forceinline__ uint32_t key_len_short(uint64_t k0, uint64_t k1) {
    if (k1) return 8 + (uint32_t)((71 - __builtin_clzll(k1)) >> 3);
    return (uint32_t)((71 - __builtin_clzll(k0)) >> 3);
}

// ihash (mr/worker.go:33-37) of a zero-padded short key, % nreduce (worker.go:76).
__device__ __forceinline__ uint32_t short_partition(uint64_t k0, uint64_t k1, uint32_t len, uint32_t nreduce) {
    uint32_t h = 2166136261u;
    for (uint32_t k = 0; k < len; k++) {
        const uint64_t w = k < 8 ? k0 : k1;
        h = fnv1a32_step(h, (uint32_t)(w >> (8 * (k & 7))) & 0xFFu);
    }
    return (h & 0x7fffffffu) % nreduce;
}

// 16 bytes starting at p as two little-endian words; only the bytes before
// p + avail are meaningful.  Reads the aligned 16-byte block holding p and the
// next one only if bytes before p + avail lie in it (an aligned block never
// crosses a page, so nothing past the buffer's last page is touched).
__device__ __forceinline__ void load16u(const uint8_t* p, uint64_t avail, uint64_t& r0, uint64_t& r1) {
    const uintptr_t a = (uintptr_t)p, ab = a & ~(uintptr_t)15;
    uint32_t sh = (uint32_t)(a - ab);
    const uint4 lo = *(const uint4*)ab;
    uint4 hi = make_uint4(0, 0, 0, 0);
    if (sh != 0 && avail > 16 - sh) hi = *(const uint4*)(ab + 16);
    uint64_t q0 = ((uint64_t)lo.y << 32) | lo.x, q1 = ((uint64_t)lo.w << 32) | lo.z;
    uint64_t q2 = ((uint64_t)hi.y << 32) | hi.x;
    const uint64_t q3 = ((uint64_t)hi.w << 32) | hi.z;
    if (sh >= 8) { q0 = q1; q1 = q2; q2 = q3; sh -= 8; }
    if (sh) {
        const uint32_t b = 8 * sh;
        r0 = (q0 >> b) | (q1 << (64 - b));
        r1 = (q1 >> b) | (q2 << (64 - b));
    } else {
        r0 = q0;
        r1 = q1;
    }
}

// len bytes at a == len bytes at b, 64 bytes per step: four independent
// 16-byte pieces per side in flight at once (long keys, grep lines: a chain of
// byte loads, or of one 16-byte load per step, costs a memory round trip each).
__device__ inline bool bytes_equal(const uint8_t* a, const uint8_t* b, uint64_t len) {
    for (uint64_t k0 = 0; k0 < len; k0 += 64) {
        uint64_t a0[4], a1[4], b0[4], b1[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t k = k0 + 16 * i;
            a0[i] = a1[i] = b0[i] = b1[i] = 0;
            if (k < len) {
                load16u(a + k, len - k, a0[i], a1[i]);
                load16u(b + k, len - k, b0[i], b1[i]);
            }
        }
        bool eq = true;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t k = k0 + 16 * i;
            if (k >= len) break;
            const uint64_t left = len - k;
            uint64_t m0 = ~0ull, m1 = ~0ull;
            if (left < 16) {
                m0 = left >= 8 ? ~0ull : (1ull << (8 * left)) - 1;
                m1 = left <= 8 ? 0ull : (1ull << (8 * (left - 8))) - 1;
            }
            eq &= ((a0[i] ^ b0[i]) & m0) == 0 && ((a1[i] ^ b1[i]) & m1) == 0;
        }
        if (!eq) return false;
    }
    return true;
}

// ------------------------------------------------------- HBM table inserts
// Lock-free insert of a short key.  Claim = CAS on k0 (0 -> key); the claimer
// then publishes k1.  A prober that matches k0 before k1 is visible never waits
// inside the probe loop: the compiler may place the claimer's publish on the
// loop's exit path, after every other lane of its wave left the loop, so an
// in-loop wait can stall a whole wave (measured: ~100 ms per 10 GB).  Instead
// *_try returns kRetry and *_insert re-runs it from a wave-uniform outer loop,
// which only iterates after the claimer's stores have executed.  All shared
// words use agent-scope atomics (coherent across the 8 XCD L2s).
enum : int { kDone = 0, kRetry = 1, kFull = 2, kClaimed = 3 };
constexpr uint32_t kMaxRetries = 1u << 20;

__device__ inline int short_try(const Tables& t, uint64_t k0, uint64_t k1, uint64_t cnt, uint64_t& slot) {
    uint64_t i = short_hash64(k0, k1) & t.sh_mask;
    for (uint32_t probes = 0; probes <= (uint32_t)kGlobalProbes; probes++) {
        ShortSlot* s = &t.sh[i];
        uint64_t cur = ld_agent(&s->k0);
        if (cur == 0) {
            const uint64_t prev = atomicCAS((unsigned long long*)&s->k0, 0ull, (unsigned long long)k0);
            if (prev == 0) {
                st_agent(&s->k1, k1);
                atomicAdd((unsigned long long*)&s->count, (unsigned long long)cnt);
                slot = i;
                return kClaimed;
            }
            cur = prev;
        }
        if (cur == k0) {
            const uint64_t v = ld_agent(&s->k1);
            if (v == kUnwritten) return kRetry;
            if (v == k1) {
                atomicAdd((unsigned long long*)&s->count, (unsigned long long)cnt);
                return kDone;
            }
        }
        i = (i + 1) & t.sh_mask;
    }
    return kFull;
}

// One atomic per wave for the claim counter (see block_add4); the fill check
// uses the wave's post-increment total.
__device__ __forceinline__ void count_claims(unsigned long long* used_ctr, uint64_t cap, bool claimed, Counters* ctr,
                                             uint32_t full_bit) {
    const uint64_t m = __ballot(claimed);
    if (m == 0) return;
    if (lane_id() == (uint32_t)__builtin_ctzll(m)) {
        const unsigned long long k = (unsigned long long)__popcll(m);
        const unsigned long long used = atomicAdd(used_ctr, k) + k;
        if (used * 10 > cap * 7) set_status(ctr, full_bit);
    }
}

// A claim also records its slot in the claim list (the collect reads the list
// instead of scanning the whole table).
__device__ inline void short_insert(const Tables& t, uint64_t k0, uint64_t k1, uint64_t cnt) {
    bool pending = true;
    uint32_t tries = 0;
    while (__ballot(pending)) {  // wave-uniform: reconverges between attempts
        bool claimed = false;
        uint64_t slot = 0;
        if (pending) {
            const int r = short_try(t, k0, k1, cnt, slot);
            if (r == kFull) set_status(t.ctr, kStShortFull);
            claimed = r == kClaimed;
            pending = r == kRetry;
            if (pending && ++tries > kMaxRetries) { set_status(t.ctr, kStSpin); pending = false; }
        }
        const uint64_t m = __ballot(claimed);
        if (m == 0) continue;
        const uint32_t leader = (uint32_t)__builtin_ctzll(m);
        unsigned long long base = 0;
        if (lane_id() == leader) {  // one atomic per wave; the fill check on the wave's post-increment total
            const unsigned long long k = (unsigned long long)__popcll(m);
            base = atomicAdd(&t.ctr->short_used, k);
            if ((base + k) * 10 > (t.sh_mask + 1) * 7) set_status(t.ctr, kStShortFull);
        }
        base = __shfl(base, (int)leader);
        const uint64_t at = base + mbcnt64(m);
        if (claimed && at <= t.sh_mask) t.sh_list[at] = (uint32_t)slot;
    }
}

// Long keys: claim = CAS on hash; publish len+1 and rep separately; a prober
// that needs them before both are visible retries from the outer loop.
__device__ inline int long_try(const Tables& t, uint64_t h, const uint8_t* rep, uint64_t len, uint64_t cnt,
                               uint64_t* claimed_slot = nullptr) {
    uint64_t i = (h * 0x9E3779B97F4A7C15ull >> 17) & t.lo_mask;
    for (uint32_t probes = 0; probes <= (uint32_t)kGlobalProbes; probes++) {
        LongSlot* s = &t.lo[i];
        uint64_t cur = ld_agent(&s->hash);
        if (cur == 0) {
            const uint64_t prev = atomicCAS((unsigned long long*)&s->hash, 0ull, (unsigned long long)h);
            if (prev == 0) {
                st_agent(&s->len, len + 1);
                __hip_atomic_store(const_cast<const uint8_t**>(&s->rep), rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicAdd((unsigned long long*)&s->count, (unsigned long long)cnt);
                if (claimed_slot) *claimed_slot = i;
                return kClaimed;
            }
            cur = prev;
        }
        if (cur == h) {
            const uint8_t* r = ld_agent_ptr(&s->rep);
            const uint64_t lp1 = ld_agent(&s->len);
            if (r == nullptr || lp1 == 0) return kRetry;
            if (lp1 == len + 1) {
                if (bytes_equal(r, rep, len)) {
                    atomicAdd((unsigned long long*)&s->count, (unsigned long long)cnt);
                    return kDone;
                }
            }
        }
        i = (i + 1) & t.lo_mask;
    }
    return kFull;
}

__device__ inline void long_insert(const Tables& t, uint64_t h, const uint8_t* rep, uint64_t len, uint64_t cnt) {
    h |= 1ull;
    bool pending = true;
    uint32_t tries = 0;
    while (__ballot(pending)) {
        bool claimed = false;
        if (pending) {
            const int r = long_try(t, h, rep, len, cnt);
            if (r == kFull) set_status(t.ctr, kStLongFull);
            claimed = r == kClaimed;
            pending = r == kRetry;
            if (pending && ++tries > kMaxRetries) { set_status(t.ctr, kStSpin); pending = false; }
        }
        if (claimed) atomicAdd(&t.ctr->long_bytes, (unsigned long long)len);  // distinct long keys only
        count_claims(&t.ctr->long_used, t.lo_mask + 1, claimed, t.ctr, kStLongFull);
    }
}

// Append v to the list (one atomic per wave: see wave_alloc).
__device__ __forceinline__ void list_append(const Tables& t, uint64_t v) {
    const unsigned long long idx = wave_alloc(&t.ctr->nlist, true);
    if (idx < t.list_cap) t.list[idx] = v;
    else set_status(t.ctr, kStListFull);
}

// ------------------------------------------------------------ chunk loading
struct ChunkRegs {
    uint4 a, h;  // a: chunk bytes [16l, 16l+16); h: halo piece (lanes 0-3 look-ahead, lane 4 look-back)
};

__device__ __forceinline__ uint4 load16_bounded(const uint8_t* in, uint64_t n, int64_t off) {
    uint32_t w[4] = {0, 0, 0, 0};
    for (int k = 0; k < 16; k++) {
        const int64_t o = off + k;
        if (o >= 0 && (uint64_t)o < n) w[k >> 2] |= (uint32_t)in[o] << (8 * (k & 3));
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ void load_chunk(const uint8_t* __restrict__ in, uint64_t n, uint64_t cs, uint32_t lane,
                                           ChunkRegs& r) {
    if (cs + kChunk + kAhead <= n && cs >= (uint64_t)kBack) {
        const uint4* p = reinterpret_cast<const uint4*>(in + cs);
        r.a = p[lane];
        if (lane < 4) r.h = p[64 + lane];
        else if (lane == 4) r.h = p[-1];
        else r.h = make_uint4(0, 0, 0, 0);
    } else {
        r.a = load16_bounded(in, n, (int64_t)cs + 16 * lane);
        if (lane < 4) r.h = load16_bounded(in, n, (int64_t)cs + kChunk + 16 * lane);
        else if (lane == 4) r.h = load16_bounded(in, n, (int64_t)cs - 16);
        else r.h = make_uint4(0, 0, 0, 0);
    }
}

// Stage a chunk into a wave's LDS buffer: [0,16) look-back, [16,1040) chunk, [1040,1104) look-ahead.
__device__ __forceinline__ void stage_chunk(lds_uint4* b4, const ChunkRegs& r, uint32_t lane) {
    b4[1 + lane] = to_v4(r.a);
    if (lane < 4) b4[65 + lane] = to_v4(r.h);
    else if (lane == 4) b4[0] = to_v4(r.h);
}

}  // namespace mrg
