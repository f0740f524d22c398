// mrgpu_exch.h — host-side layout of the shuffle (mr/worker.go:80-122 replaced
// by one all-to-all): wire record format and the per-rank send / receive plan.
// Plain C++ (no HIP): tests/test_exch_plan.py compiles it with g++ and checks the
// displacements of every rank of a simulated P-rank all-to-all.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace mrg {

// 24-byte wire record ([key][len][count]; the partition is not
// sent — the owner's aggregation recomputes ihash % nReduce from the key):
//   key of <= 16 bytes: {k0, k1, cnt}            (len = the zero-padded key's length)
//   longer key:         {arena offset, len, cnt | kWireLong}  (bytes in the arena segment)
struct WireRec {
    uint64_t a, b, c;
};
static_assert(sizeof(WireRec) == 24, "wire record size");
constexpr uint64_t kWireLong = 1ull << 63;

// One rank's exchange: byte counts / displacements of its send segments (per
// owner rank) and receive segments (per source rank), for the record stream and
// the arena stream; what ncclAllToAllv takes.
struct ExchPlan {
    std::vector<size_t> sc, sd, rc, rd, asc, asd, arc, ard;  // records (bytes) and arena bytes
    std::vector<uint64_t> hbase;                             // [P] record base, [P] arena base (send side)
    size_t srec = 0, sar = 0, rrec = 0, rar = 0;
};

// snd[2*o] / snd[2*o+1]: records / arena bytes this rank sends to owner o;
// rcv[2*s] / rcv[2*s+1]: what it receives from source s.  Segments are laid out
// in rank order on both sides, so the all-to-all's segment from source s lands
// at rd[s] / ard[s], and a received record's source is the last s with
// rd[s] <= its byte offset (the unpack's binary search).
inline ExchPlan exch_plan(int P, const unsigned long long* snd, const unsigned long long* rcv) {
    ExchPlan x;
    for (auto* v : {&x.sc, &x.sd, &x.rc, &x.rd, &x.asc, &x.asd, &x.arc, &x.ard}) v->assign(P, 0);
    x.hbase.assign(2 * P, 0);
    for (int o = 0; o < P; o++) {
        x.hbase[o] = x.srec;
        x.hbase[P + o] = x.sar;
        x.sc[o] = snd[2 * o] * sizeof(WireRec);
        x.sd[o] = x.srec * sizeof(WireRec);
        x.srec += snd[2 * o];
        x.asc[o] = snd[2 * o + 1];
        x.asd[o] = x.sar;
        x.sar += snd[2 * o + 1];
        x.rc[o] = rcv[2 * o] * sizeof(WireRec);
        x.rd[o] = x.rrec * sizeof(WireRec);
        x.rrec += rcv[2 * o];
        x.arc[o] = rcv[2 * o + 1];
        x.ard[o] = x.rar;
        x.rar += rcv[2 * o + 1];
    }
    return x;
}

}  // namespace mrg
