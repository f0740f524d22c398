/*
 * mrcount.c — multi-threaded C restatement of the reference's wc / grep job for
 * full-size (multi-GB) inputs.
 *
 * TEST INFRASTRUCTURE ONLY (the checker).  Only tests/, __graft_entry__.smoke()
 * and bench.py's oracle check (outside the timed region) may load it; the
 * product library never links it.  Parity status: as mroracle.c (parity
 * unpinned against reference-run outputs; pinned to the FNV KATs, the UCD and
 * the Python restatement — tests/test_oracle.py checks this file against
 * mroracle.c's oracle_mr_partitioned on every golden case).
 *
 * Same semantics as mroracle.c's oracle_mr_partitioned over one split, restated
 * for size: wc.Map (mrapps/wc.go:21-34) emits one KeyValue{w, "1"} per word and
 * wc.Reduce (wc.go:41-44) returns len(values), so the mr-out-r line of a key is
 * "key count"; the group step (mr/worker.go:129-146, main/mrsequential.go:59-84)
 * is restated as a hash-table count per thread, merged, then every partition's
 * distinct keys sorted by ByKey.Less (worker.go:27: Go string '<', unsigned
 * bytewise, shorter prefix first) and printed with Fprintf("%v %v\n").
 * grep (mrapps/dgrep.go:18-46): strings.Split(contents, "\n") lines holding the
 * literal pattern; grepReduce returns the key, so each distinct line appears once
 * as "line line".
 *
 * Threads split the input at '\n' bytes: '\n' is ASCII, so it always starts a
 * rune in Go's decoding, is never a letter, and is the line separator — a cut
 * after it changes neither the word list nor the line list.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define APP_WC 1
#define APP_GREP 2

int oracle_is_letter(uint32_t cp);
size_t oracle_decode_rune(const uint8_t* s, size_t n, size_t i, uint32_t* cp);
uint32_t oracle_ihash(const uint8_t* p, size_t n);

typedef struct {
    uint64_t h;     /* 64-bit hash; 0 = empty slot */
    uint64_t k[2];  /* the key's first 16 bytes, zero padded (compared without
                       touching the input: a tail word's first occurrence is
                       usually far away in a multi-GB split) */
    const uint8_t* p;
    uint64_t n;     /* key length */
    uint64_t cnt;   /* occurrences (wc); 1 for grep */
} cslot;

static void key_prefix(const uint8_t* p, uint64_t n, uint64_t k[2]) {
    k[0] = k[1] = 0;
    memcpy(k, p, n < 16 ? n : 16);
}

typedef struct {
    cslot* s;
    uint64_t mask, used;
} ctable;

static uint64_t key_hash(const uint8_t* p, uint64_t n) {
    uint64_t h = 1469598103934665603ull;  /* FNV-1a 64, then a finalizer */
    for (uint64_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
    h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ull; h ^= h >> 32;
    return h | 1ull;
}

static int ct_init(ctable* t, uint64_t cap) {
    uint64_t c = 1024;
    while (c < cap * 2) c <<= 1;
    t->s = (cslot*)calloc(c, sizeof(cslot));
    t->mask = c - 1;
    t->used = 0;
    return t->s ? 0 : -1;
}

static int ct_grow(ctable* t);

static int ct_add(ctable* t, const uint8_t* p, uint64_t n, uint64_t h, uint64_t cnt) {
    uint64_t i = h & t->mask;
    uint64_t k[2];
    key_prefix(p, n, k);
    for (;;) {
        cslot* s = &t->s[i];
        if (s->h == 0) {
            s->h = h; s->k[0] = k[0]; s->k[1] = k[1]; s->p = p; s->n = n; s->cnt = cnt;
            if (++t->used * 10 > (t->mask + 1) * 6) return ct_grow(t);
            return 0;
        }
        if (s->h == h && s->n == n && s->k[0] == k[0] && s->k[1] == k[1] &&
            (n <= 16 || memcmp(s->p + 16, p + 16, n - 16) == 0)) {
            s->cnt += cnt;
            return 0;
        }
        i = (i + 1) & t->mask;
    }
}

static int ct_grow(ctable* t) {
    ctable u;
    if (ct_init(&u, (t->mask + 1)) != 0) return -1;
    for (uint64_t i = 0; i <= t->mask; i++)
        if (t->s[i].h) {
            cslot* s = &t->s[i];
            uint64_t j = s->h & u.mask;
            while (u.s[j].h) j = (j + 1) & u.mask;
            u.s[j] = *s;
            u.used++;
        }
    free(t->s);
    *t = u;
    return 0;
}

typedef struct {
    int app;
    const uint8_t* s;    /* the whole split (for Go's decoder bounds) */
    uint64_t n;
    uint64_t a, b;       /* this thread's byte range [a, b) */
    int last;            /* the range ends the split (grep: the final line) */
    const uint8_t* pat;
    uint64_t pn;
    ctable t;
    int err;
} cjob;

/* strings.FieldsFunc(contents, !unicode.IsLetter) over [a, b) (wc.go:21-34) */
static void wc_range(cjob* j) {
    const uint8_t* s = j->s;
    uint64_t i = j->a, start = 0;
    int in = 0;
    while (i < j->b) {
        uint32_t cp;
        size_t w;
        uint8_t c = s[i];
        int let;
        if (c < 0x80) { w = 1; let = (uint8_t)((c | 0x20) - 'a') < 26; }
        else { w = oracle_decode_rune(s, j->n, i, &cp); let = oracle_is_letter(cp); }
        if (let) {
            if (!in) { in = 1; start = i; }
        } else if (in) {
            in = 0;
            if (ct_add(&j->t, s + start, i - start, key_hash(s + start, i - start), 1)) { j->err = 1; return; }
        }
        i += w;
    }
    if (in && ct_add(&j->t, s + start, j->b - start, key_hash(s + start, j->b - start), 1)) j->err = 1;
}

static int contains(const uint8_t* h, uint64_t hn, const uint8_t* pat, uint64_t pn) {
    if (pn == 0) return 1;
    if (pn > hn) return 0;
    const uint8_t* e = h + hn - pn;
    for (const uint8_t* q = h; q <= e; q++) {
        q = (const uint8_t*)memchr(q, pat[0], (size_t)(e - q) + 1);
        if (!q) return 0;
        if (memcmp(q, pat, pn) == 0) return 1;
    }
    return 0;
}

/* grepMap (dgrep.go:26-36) over the lines of [a, b): every line of the range
 * ends with '\n', except the split's final line (strings.Split's last element,
 * "" when the split ends with '\n') */
static void grep_range(cjob* j) {
    const uint8_t* s = j->s;
    uint64_t ls = j->a;
    for (;;) {
        const uint8_t* nl = ls < j->b ? (const uint8_t*)memchr(s + ls, '\n', j->b - ls) : NULL;
        uint64_t le = nl ? (uint64_t)(nl - s) : j->b;
        if (!nl && !j->last) break;
        if (contains(s + ls, le - ls, j->pat, j->pn))
            if (ct_add(&j->t, s + ls, le - ls, key_hash(s + ls, le - ls), 1)) { j->err = 1; return; }
        if (!nl) break;
        ls = le + 1;
    }
}

static void* run_job(void* arg) {
    cjob* j = (cjob*)arg;
    if (ct_init(&j->t, 1 << 16)) { j->err = 1; return NULL; }
    if (j->app == APP_WC) wc_range(j);
    else grep_range(j);
    return NULL;
}

static int valid_utf8(const uint8_t* s, size_t n) {
    for (size_t i = 0; i < n;) {
        uint32_t cp;
        if (s[i] < 0x80) { i++; continue; }
        size_t w = oracle_decode_rune(s, n, i, &cp);
        if (w == 1) return 0;
        i += w;
    }
    return 1;
}

typedef struct { const uint8_t* p; uint64_t n, cnt; } ckey;

static int ckey_cmp(const void* a, const void* b) {
    const ckey* x = (const ckey*)a;
    const ckey* y = (const ckey*)b;
    uint64_t m = x->n < y->n ? x->n : y->n;
    int c = memcmp(x->p, y->p, m);
    if (c) return c;
    return (x->n > y->n) - (x->n < y->n);
}

/*
 * The whole job over one split s[0, n): mr-out-r for r < nreduce, concatenated
 * into *out (malloc'd; free with oracle_free), offsets[nreduce + 1].
 * Returns 0, or -1 on allocation failure.
 */
int oracle_count_mt(int app, const uint8_t* pat, size_t pn, const uint8_t* s, size_t n, int nthreads,
                    uint32_t nreduce, uint8_t** out, size_t* out_n, uint64_t* offsets) {
    if (nthreads < 1) nthreads = 1;
    if (app == APP_GREP && !valid_utf8(pat, pn)) {  /* dgrep.go:20-23: no lines */
        for (uint32_t r = 0; r <= nreduce; r++) offsets[r] = 0;
        *out = (uint8_t*)malloc(1); *out_n = 0;
        return 0;
    }
    cjob* jobs = (cjob*)calloc((size_t)nthreads, sizeof(cjob));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    uint64_t a = 0;
    int ended = 0;  /* a range already reached the split's end */
    for (int k = 0; k < nthreads; k++) {
        uint64_t b = k == nthreads - 1 ? n : (uint64_t)((unsigned __int128)n * (k + 1) / nthreads);
        if (b < a) b = a;
        if (k < nthreads - 1) {  /* end the range just after a '\n' */
            const uint8_t* nl = b < n ? (const uint8_t*)memchr(s + b, '\n', n - b) : NULL;
            b = nl ? (uint64_t)(nl - s) + 1 : n;
        }
        /* the range holding the split's final line (after its last '\n') is "last";
           ranges after it are empty */
        const int last = !ended && b == n;
        jobs[k] = (cjob){app, s, n, a, b, last, pat, pn, {0}, 0};
        if (b == n) ended = 1;
        a = b;
    }
    for (int k = 0; k < nthreads; k++) pthread_create(&th[k], NULL, run_job, &jobs[k]);
    for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
    int err = 0;
    uint64_t total = 0;
    for (int k = 0; k < nthreads; k++) { err |= jobs[k].err; total += jobs[k].t.used; }
    ctable g = {0};
    if (!err && ct_init(&g, total ? total : 1)) err = 1;
    for (int k = 0; k < nthreads; k++) {
        ctable* t = &jobs[k].t;
        for (uint64_t i = 0; !err && t->s && i <= t->mask; i++)
            if (t->s[i].h && ct_add(&g, t->s[i].p, t->s[i].n, t->s[i].h, t->s[i].cnt)) err = 1;
        free(t->s);
    }
    free(jobs); free(th);
    if (err) { free(g.s); return -1; }

    /* partition (worker.go:74-78), sort (ByKey), print (worker.go:129-146) */
    uint64_t* pc = (uint64_t*)calloc(nreduce + 1, sizeof(uint64_t));
    uint32_t* part = (uint32_t*)malloc((g.used ? g.used : 1) * sizeof(uint32_t));
    ckey* keys = (ckey*)malloc((g.used ? g.used : 1) * sizeof(ckey));
    uint64_t m = 0, bytes = 0;
    for (uint64_t i = 0; i <= g.mask; i++)
        if (g.s[i].h) {
            cslot* c = &g.s[i];
            part[m] = oracle_ihash(c->p, c->n) % nreduce;
            keys[m] = (ckey){c->p, c->n, c->cnt};
            pc[part[m] + 1]++;
            bytes += app == APP_WC ? c->n + 22 : 2 * c->n + 2;
            m++;
        }
    free(g.s);
    for (uint32_t r = 0; r < nreduce; r++) pc[r + 1] += pc[r];
    ckey* sorted = (ckey*)malloc((m ? m : 1) * sizeof(ckey));
    uint64_t* fill = (uint64_t*)malloc((nreduce + 1) * sizeof(uint64_t));
    memcpy(fill, pc, (nreduce + 1) * sizeof(uint64_t));
    for (uint64_t i = 0; i < m; i++) sorted[fill[part[i]]++] = keys[i];
    free(keys); free(part); free(fill);
    uint8_t* o = (uint8_t*)malloc(bytes ? bytes : 1);
    uint64_t on = 0;
    for (uint32_t r = 0; r < nreduce; r++) {
        if (pc[r + 1] - pc[r] > 1) qsort(sorted + pc[r], pc[r + 1] - pc[r], sizeof(ckey), ckey_cmp);
        offsets[r] = on;
        for (uint64_t i = pc[r]; i < pc[r + 1]; i++) {
            const ckey* k = &sorted[i];
            memcpy(o + on, k->p, k->n); on += k->n;
            o[on++] = ' ';
            if (app == APP_WC) on += (uint64_t)sprintf((char*)o + on, "%llu", (unsigned long long)k->cnt);
            else { memcpy(o + on, k->p, k->n); on += k->n; }
            o[on++] = '\n';
        }
    }
    offsets[nreduce] = on;
    free(sorted); free(pc);
    *out = o; *out_n = on;
    return 0;
}

/*
 * Merge R-partitioned wc outputs of several splits (lines "key count\n", each
 * partition sorted by ByKey): the reduce of worker.go:123-146 over the union of
 * the splits' intermediate files, with equal keys' counts summed.  ins[i] is
 * input i's concatenation, in_offs[i * (nreduce + 1) + r] its partition offsets;
 * the result as in oracle_count_mt.  grep (app 2): lines "L L\n", deduplicated.
 */
int oracle_merge_parts(int app, uint32_t nins, const uint8_t* const* ins, const uint64_t* in_offs, uint32_t nreduce,
                       uint8_t** out, size_t* out_n, uint64_t* offsets) {
    uint64_t cap = 1;
    for (uint32_t i = 0; i < nins; i++) cap += in_offs[i * (nreduce + 1) + nreduce];
    uint8_t* o = (uint8_t*)malloc(cap);
    uint64_t on = 0;
    uint64_t* pos = (uint64_t*)malloc((nins ? nins : 1) * sizeof(uint64_t));
    for (uint32_t r = 0; r < nreduce; r++) {
        offsets[r] = on;
        for (uint32_t i = 0; i < nins; i++) pos[i] = in_offs[i * (nreduce + 1) + r];
        for (;;) {
            /* the smallest key at the inputs' cursors */
            const uint8_t* best = NULL;
            uint64_t bn = 0;
            for (uint32_t i = 0; i < nins; i++) {
                uint64_t end = in_offs[i * (nreduce + 1) + r + 1];
                if (pos[i] >= end) continue;
                const uint8_t* l = ins[i] + pos[i];
                const uint8_t* nl = (const uint8_t*)memchr(l, '\n', end - pos[i]);
                if (!nl) { free(o); free(pos); return -1; }
                uint64_t ln = (uint64_t)(nl - l);
                uint64_t kn = app == APP_WC ? (uint64_t)((const uint8_t*)memrchr(l, ' ', ln) - l) : (ln - 1) / 2;
                ckey a = {l, kn, 0}, b = {best, bn, 0};
                if (!best || ckey_cmp(&a, &b) < 0) { best = l; bn = kn; }
            }
            if (!best) break;
            uint64_t sum = 0;
            for (uint32_t i = 0; i < nins; i++) {
                uint64_t end = in_offs[i * (nreduce + 1) + r + 1];
                if (pos[i] >= end) continue;
                const uint8_t* l = ins[i] + pos[i];
                const uint8_t* nl = (const uint8_t*)memchr(l, '\n', end - pos[i]);
                uint64_t ln = (uint64_t)(nl - l);
                uint64_t kn = app == APP_WC ? (uint64_t)((const uint8_t*)memrchr(l, ' ', ln) - l) : (ln - 1) / 2;
                if (kn == bn && memcmp(l, best, bn) == 0) {
                    if (app == APP_WC) sum += strtoull((const char*)l + kn + 1, NULL, 10);
                    pos[i] += ln + 1;
                }
            }
            memcpy(o + on, best, bn); on += bn;
            o[on++] = ' ';
            if (app == APP_WC) {
                char num[24];
                int k = sprintf(num, "%llu", (unsigned long long)sum);
                memcpy(o + on, num, (size_t)k); on += (uint64_t)k;
            } else {
                memcpy(o + on, best, bn); on += bn;
            }
            o[on++] = '\n';
        }
    }
    offsets[nreduce] = on;
    free(pos);
    *out = o; *out_n = on;
    return 0;
}
