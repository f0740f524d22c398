// Simulated P-rank all-to-all over the shuffle plan of csrc/mrgpu_exch.h
// (the layout mrg_exchange hands to ncclAllToAllv).  Built and run by
// tests/test_exch_plan.py on the CPU.
//
// Every rank s sends n[s][o] records and a[s][o] arena bytes to owner o (zeros
// included: empty segments, empty ranks, a rank that sends nothing at all).
// Each record carries (source, owner, index); the arena bytes are a pattern of
// (source, owner, offset).  The simulation copies segment o of rank s's send
// buffers to rank o's receive buffers exactly as ncclAllToAllv's
// (sendcounts, sdispls, recvcounts, rdispls) say, then checks on every owner:
//   - every record from every source arrived once, in the source's order;
//   - the unpack's binary search (last s with rd[s] / 24 <= i) names its source;
//   - the arena bytes of source s sit at ard[s] (the long-key offset rebase).
// Prints "ok <P> <records> <bytes>" or the first failure, exit status 1.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../distributed-systems-implemented_amd/csrc/mrgpu_exch.h"

using namespace mrg;

static int fails = 0;
#define CHECK(c, ...)                         \
    do {                                      \
        if (!(c)) {                           \
            if (fails++ < 5) {                \
                fprintf(stderr, __VA_ARGS__); \
                fputc('\n', stderr);          \
            }                                 \
        }                                     \
    } while (0)

int main(int argc, char** argv) {
    const int P = argc > 1 ? atoi(argv[1]) : 8;
    const unsigned seed = argc > 2 ? (unsigned)atoi(argv[2]) : 1;
    std::mt19937_64 rng(seed);
    // n[s][o] records, a[s][o] arena bytes (multiples of 16, as the pack pads them)
    std::vector<std::vector<unsigned long long>> n(P, std::vector<unsigned long long>(P)),
        a(P, std::vector<unsigned long long>(P));
    for (int s = 0; s < P; s++)
        for (int o = 0; o < P; o++) {
            const unsigned r = (unsigned)(rng() % 10);
            n[s][o] = r < 3 ? 0 : rng() % 200;          // 30 % empty segments
            a[s][o] = (r < 6 ? 0 : rng() % 40) * 16;    // most segments carry no long keys
        }
    if (P > 2) {
        for (int o = 0; o < P; o++) n[1][o] = a[1][o] = 0;  // a rank that sends nothing
        for (int s = 0; s < P; s++) n[s][2] = a[s][2] = 0;  // a rank that receives nothing
    }
    std::vector<ExchPlan> pl(P);
    for (int r = 0; r < P; r++) {
        std::vector<unsigned long long> snd(2 * P), rcv(2 * P);
        for (int o = 0; o < P; o++) {
            snd[2 * o] = n[r][o];
            snd[2 * o + 1] = a[r][o];
            rcv[2 * o] = n[o][r];
            rcv[2 * o + 1] = a[o][r];
        }
        pl[r] = exch_plan(P, snd.data(), rcv.data());
    }
    // send buffers as the pack kernel fills them: records of owner o at hbase[o]
    std::vector<std::vector<WireRec>> sbuf(P);
    std::vector<std::vector<unsigned char>> sar(P);
    for (int s = 0; s < P; s++) {
        sbuf[s].resize(pl[s].srec);
        sar[s].resize(pl[s].sar);
        for (int o = 0; o < P; o++) {
            CHECK(pl[s].sd[o] == pl[s].hbase[o] * sizeof(WireRec), "rank %d: sd[%d] != hbase", s, o);
            CHECK(pl[s].asd[o] == pl[s].hbase[P + o], "rank %d: asd[%d] != arena base", s, o);
            for (unsigned long long i = 0; i < n[s][o]; i++)
                sbuf[s][pl[s].hbase[o] + i] = WireRec{(uint64_t)s, (uint64_t)o, i};
            for (unsigned long long b = 0; b < a[s][o]; b++)
                sar[s][pl[s].hbase[P + o] + b] = (unsigned char)(s * 31 + o * 7 + b);
        }
    }
    // the all-to-all: segment o of source s -> owner o at rd[s] / ard[s]
    std::vector<std::vector<unsigned char>> rbuf(P), rar(P);
    for (int o = 0; o < P; o++) {
        rbuf[o].assign(pl[o].rrec * sizeof(WireRec), 0xEE);
        rar[o].assign(pl[o].rar, 0xEE);
    }
    for (int s = 0; s < P; s++)
        for (int o = 0; o < P; o++) {
            CHECK(pl[s].sc[o] == pl[o].rc[s], "send count %d->%d != receive count", s, o);
            CHECK(pl[s].asc[o] == pl[o].arc[s], "arena count %d->%d differs", s, o);
            CHECK(pl[o].rd[s] + pl[o].rc[s] <= rbuf[o].size(), "receive segment %d at %d out of range", s, o);
            CHECK(pl[s].sd[o] + pl[s].sc[o] <= sbuf[s].size() * sizeof(WireRec), "rank %d: send segment %d out of range", s, o);
            if (fails) continue;
            memcpy(rbuf[o].data() + pl[o].rd[s], (const unsigned char*)sbuf[s].data() + pl[s].sd[o], pl[s].sc[o]);
            if (pl[s].asc[o]) memcpy(rar[o].data() + pl[o].ard[s], sar[s].data() + pl[s].asd[o], pl[s].asc[o]);
        }
    unsigned long long recs = 0, bytes = 0;
    for (int o = 0; o < P && !fails; o++) {
        const WireRec* w = (const WireRec*)rbuf[o].data();
        std::vector<unsigned long long> seen(P, 0);
        for (unsigned long long i = 0; i < pl[o].rrec; i++) {
            // the unpack kernel's search: last s with rd[s] / 24 <= i
            int lo = 0, hi = P - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (pl[o].rd[mid] / sizeof(WireRec) <= i) lo = mid;
                else hi = mid - 1;
            }
            CHECK((int)w[i].a == lo, "owner %d record %llu: source %llu, search says %d", o, i,
                  (unsigned long long)w[i].a, lo);
            CHECK((int)w[i].b == o, "owner %d got a record for owner %llu", o, (unsigned long long)w[i].b);
            CHECK(w[i].a < (uint64_t)P && w[i].c == seen[w[i].a], "owner %d: source %llu out of order", o,
                  (unsigned long long)w[i].a);
            if (w[i].a < (uint64_t)P) seen[w[i].a]++;
            recs++;
        }
        for (int s = 0; s < P; s++) {
            CHECK(seen[s] == n[s][o], "owner %d: %llu of %llu records from %d", o, seen[s], n[s][o], s);
            for (unsigned long long b = 0; b < a[s][o]; b++)
                CHECK(rar[o][pl[o].ard[s] + b] == (unsigned char)(s * 31 + o * 7 + b), "owner %d arena from %d", o, s);
            bytes += a[s][o];
        }
    }
    if (fails) return 1;
    printf("ok %d %llu %llu\n", P, recs, bytes);
    return 0;
}
