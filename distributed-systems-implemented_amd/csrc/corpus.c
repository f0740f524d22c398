/*
 * corpus.c — deterministic synthetic corpora for the MapReduce wc/grep path.
 *
 * The reference's inputs (pg-*.txt, MapReduce/main/test-mr.sh:30) are not
 * bundled (.gitignore:36), so every BASELINE config runs on synthetic text
 * (SURVEY.md §8d): Zipf-distributed words over a fixed vocabulary, ASCII or
 * mixed UTF-8, separators mixing space / newline / punctuation / digits, and
 * for grep, lines with a literal pattern planted in a fraction of them.
 *
 * Properties relied on by tests and bench.py:
 *   - Pure function of (vocab params, file seed, size): identical bytes on any
 *     host built from this source.  Files are independent, so they are
 *     generated in parallel (one thread per file).
 *   - Every vocabulary word is distinct: rank k is written as its base-B digits
 *     (B = script alphabet size) padded to a length L >= digits(k); equal L and
 *     distinct k give distinct strings, different scripts have disjoint
 *     alphabets.
 *   - Every letter code point used is category L* in Unicode 13.0.0 and every
 *     separator is not (checked by tests/test_corpus.py against unicodedata).
 *   - Each file ends with '\n', so concatenating files never joins words,
 *     UTF-8 sequences or lines (SURVEY.md §8b file-boundary rule).
 * Host-only C; no GPU code.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MRC_KIND_ASCII 0
#define MRC_KIND_UTF8 1

#define MRC_MODE_WC 0
#define MRC_MODE_GREP 1

typedef struct {
    int mode;               /* MRC_MODE_WC | MRC_MODE_GREP */
    double invalid_rate;    /* probability per separator slot of emitting an invalid UTF-8 byte run */
    const char* pattern;    /* grep: literal planted into lines */
    double match_rate;      /* grep: fraction of lines carrying the pattern */
    double dup_rate;        /* grep: fraction of matching lines that repeat an earlier matching line */
    int line_min, line_max; /* grep: target line length range in bytes */
    uint64_t vocab_lo, vocab_hi; /* emit ranks [lo,hi) once, in order, before sampling */
} mrc_params;

typedef struct {
    int kind;
    double s;
    uint64_t V;
    uint64_t seed;
    uint32_t* prob;   /* alias method thresholds (2^32 scale) */
    uint32_t* alias;
    /* cache of the first ncache words */
    uint64_t ncache;
    uint32_t* coff;
    uint8_t* clen;
    uint8_t* cpool;
} mrc_vocab;

static inline uint64_t splitmix64(uint64_t* x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t mix64(uint64_t a) {
    uint64_t x = a;
    return splitmix64(&x);
}

/* English-like word length distribution over 1..15 (mean ~5.1) in 1/1000 units. */
static const uint16_t kLenCdf[15] = {30, 180, 380, 550, 670, 760, 840, 900, 940, 965, 980, 990, 995, 998, 1000};

static int draw_len(uint64_t h) {
    uint32_t r = (uint32_t)(h % 1000u);
    for (int i = 0; i < 15; i++)
        if (r < kLenCdf[i]) return i + 1;
    return 15;
}

/* Script alphabets (all category L* in Unicode 13.0.0). */
enum { SC_ASCII = 0, SC_GREEK, SC_CYRILLIC, SC_CJK, SC_DESERET, SC_CJKB, SC_N };

static uint32_t script_base(int sc) {
    switch (sc) {
        case SC_ASCII: return 52;       /* a-z A-Z */
        case SC_GREEK: return 25;       /* U+03B1..U+03C9 */
        case SC_CYRILLIC: return 64;    /* U+0410..U+044F */
        case SC_CJK: return 20902;      /* U+4E00..U+9FA5 */
        case SC_DESERET: return 80;     /* U+10400..U+1044F */
        default: return 42711;          /* U+20000..U+2A6D6 */
    }
}

static uint32_t script_cp(int sc, uint32_t d) {
    switch (sc) {
        case SC_ASCII: return d < 26 ? 'a' + d : 'A' + (d - 26);
        case SC_GREEK: return 0x3B1 + d;
        case SC_CYRILLIC: return 0x410 + d;
        case SC_CJK: return 0x4E00 + d;
        case SC_DESERET: return 0x10400 + d;
        default: return 0x20000 + d;
    }
}

static int put_utf8(uint8_t* o, uint32_t cp) {
    if (cp < 0x80) { o[0] = (uint8_t)cp; return 1; }
    if (cp < 0x800) { o[0] = 0xC0 | (cp >> 6); o[1] = 0x80 | (cp & 0x3F); return 2; }
    if (cp < 0x10000) {
        o[0] = 0xE0 | (cp >> 12); o[1] = 0x80 | ((cp >> 6) & 0x3F); o[2] = 0x80 | (cp & 0x3F); return 3;
    }
    o[0] = 0xF0 | (cp >> 18); o[1] = 0x80 | ((cp >> 12) & 0x3F);
    o[2] = 0x80 | ((cp >> 6) & 0x3F); o[3] = 0x80 | (cp & 0x3F);
    return 4;
}

/* Write vocabulary word k into o (at most 64 bytes); returns its byte length. */
static int make_word(const mrc_vocab* v, uint64_t k, uint8_t* o) {
    uint64_t h = mix64(v->seed * 0x9E3779B97F4A7C15ull ^ (k + 1));
    int sc = SC_ASCII;
    if (v->kind == MRC_KIND_UTF8) {
        uint32_t r = (uint32_t)(h >> 40) % 100u;
        sc = r < 70 ? SC_ASCII : r < 80 ? SC_GREEK : r < 88 ? SC_CYRILLIC : r < 95 ? SC_CJK
           : r < 98 ? SC_DESERET : SC_CJKB;
    }
    uint64_t B = script_base(sc);
    int digits = 1;
    for (uint64_t t = k / B; t; t /= B) digits++;
    int L = draw_len(h);
    if (sc == SC_CJK || sc == SC_CJKB) L = 1 + (int)((h >> 20) % 3u);
    if (L < digits) L = digits;
    int n = 0;
    uint64_t rem = k;
    for (int i = 0; i < L; i++) {
        uint64_t d = rem % B;
        rem /= B;
        uint64_t off = mix64(v->seed ^ (uint64_t)(sc * 7919 + i * 131 + L)) % B; /* k-independent => bijective */
        n += put_utf8(o + n, script_cp(sc, (uint32_t)((d + off) % B)));
    }
    return n;
}

void mrc_vocab_free(mrc_vocab* v);

mrc_vocab* mrc_vocab_new(int kind, double s, uint64_t V, uint64_t seed) {
    if (V == 0 || V > (1ull << 31)) return NULL;
    mrc_vocab* v = (mrc_vocab*)calloc(1, sizeof(mrc_vocab));
    v->kind = kind; v->s = s; v->V = V; v->seed = seed;
    v->prob = (uint32_t*)malloc(V * sizeof(uint32_t));
    v->alias = (uint32_t*)malloc(V * sizeof(uint32_t));
    double* p = (double*)malloc(V * sizeof(double));
    uint32_t* small = (uint32_t*)malloc(V * sizeof(uint32_t));
    uint32_t* large = (uint32_t*)malloc(V * sizeof(uint32_t));
    double sum = 0.0;
    for (uint64_t i = 0; i < V; i++) { p[i] = pow((double)(i + 1), -s); sum += p[i]; }
    uint64_t ns = 0, nl = 0;
    for (uint64_t i = 0; i < V; i++) {
        p[i] = p[i] * (double)V / sum;
        if (p[i] < 1.0) small[ns++] = (uint32_t)i; else large[nl++] = (uint32_t)i;
    }
    while (ns && nl) { /* Vose's alias method */
        uint32_t a = small[--ns], g = large[--nl];
        v->prob[a] = (uint32_t)fmin(4294967295.0, p[a] * 4294967296.0);
        v->alias[a] = g;
        p[g] = (p[g] + p[a]) - 1.0;
        if (p[g] < 1.0) small[ns++] = g; else large[nl++] = g;
    }
    while (nl) { uint32_t g = large[--nl]; v->prob[g] = 0xFFFFFFFFu; v->alias[g] = g; }
    while (ns) { uint32_t a = small[--ns]; v->prob[a] = 0xFFFFFFFFu; v->alias[a] = a; }
    free(p); free(small); free(large);
    v->ncache = V < (1ull << 18) ? V : (1ull << 18);
    v->coff = (uint32_t*)malloc(v->ncache * sizeof(uint32_t));
    v->clen = (uint8_t*)malloc(v->ncache);
    v->cpool = (uint8_t*)malloc(v->ncache * 64);
    uint32_t pos = 0;
    for (uint64_t k = 0; k < v->ncache; k++) {
        int n = make_word(v, k, v->cpool + pos);
        v->coff[k] = pos; v->clen[k] = (uint8_t)n; pos += (uint32_t)n;
    }
    return v;
}

void mrc_vocab_free(mrc_vocab* v) {
    if (!v) return;
    free(v->prob); free(v->alias); free(v->coff); free(v->clen); free(v->cpool); free(v);
}

/* Word bytes of rank k (for tests). */
int mrc_word(const mrc_vocab* v, uint64_t k, uint8_t* out64) { return make_word(v, k, out64); }

static inline uint64_t sample_rank(const mrc_vocab* v, uint64_t* rng) {
    uint64_t u = splitmix64(rng);
    uint64_t i = ((u >> 32) * v->V) >> 32;
    return ((uint32_t)u < v->prob[i]) ? i : v->alias[i];
}

static inline int emit_word(const mrc_vocab* v, uint64_t k, uint8_t* o) {
    if (k < v->ncache) { memcpy(o, v->cpool + v->coff[k], v->clen[k]); return v->clen[k]; }
    return make_word(v, k, o);
}

static const char kPunct[] = ",.;:!?-'\"()0123456789";

/* Separator: ASCII space 80%, newline 10%, punctuation/digits 10%; UTF-8 kind
 * also draws non-letter multibyte runes (NBSP, em dash, ideographic comma,
 * emoji, combining acute, Arabic-Indic zero). */
static int emit_sep(const mrc_vocab* v, uint64_t r, uint8_t* o) {
    uint32_t x = (uint32_t)(r % 1000u);
    if (x < 800) { o[0] = ' '; return 1; }
    if (x < 900) { o[0] = '\n'; return 1; }
    if (v->kind == MRC_KIND_UTF8 && x < 960) {
        static const uint32_t seps[6] = {0x00A0, 0x2014, 0x3001, 0x1F600, 0x0301, 0x0660};
        int n = 0;
        if (seps[(r >> 12) % 6u] == 0x0301) o[n++] = ' '; /* combining mark after a space */
        return n + put_utf8(o + n, seps[(r >> 12) % 6u]);
    }
    o[0] = (uint8_t)kPunct[(r >> 12) % (sizeof(kPunct) - 1)];
    return 1;
}

/* Invalid UTF-8 runs (Go decodes each offending byte as U+FFFD, width 1). */
static int emit_invalid(uint64_t r, uint8_t* o) {
    switch ((r >> 20) % 7u) {
        case 0: o[0] = 0xFF; return 1;
        case 1: o[0] = 0xC0; o[1] = 0xAF; return 2;                   /* overlong */
        case 2: o[0] = 0x80; return 1;                                /* stray continuation */
        case 3: o[0] = 0xE2; o[1] = 0x82; return 2;                   /* truncated 3-byte */
        case 4: o[0] = 0xED; o[1] = 0xA0; o[2] = 0x80; return 3;      /* surrogate */
        case 5: o[0] = 0xF4; o[1] = 0x90; o[2] = 0x80; o[3] = 0x80; return 4; /* > U+10FFFF */
        default: o[0] = 0xC3; return 1;                               /* lone lead */
    }
}

static size_t fill_wc(const mrc_vocab* v, uint64_t fseed, uint8_t* buf, size_t n, const mrc_params* pp) {
    uint64_t rng = mix64(fseed ^ 0xA5A5A5A5ull);
    size_t pos = 0;
    uint64_t vk = pp ? pp->vocab_lo : 0, vhi = pp ? pp->vocab_hi : 0;
    double inv = pp ? pp->invalid_rate : 0.0;
    uint32_t inv_thr = (uint32_t)(inv * 4294967296.0);
    while (pos + 160 < n) {
        uint64_t k = (vk < vhi) ? vk++ : sample_rank(v, &rng);
        pos += (size_t)emit_word(v, k, buf + pos);
        uint64_t r = splitmix64(&rng);
        if (inv_thr && (uint32_t)(r >> 32) < inv_thr) pos += (size_t)emit_invalid(r, buf + pos);
        pos += (size_t)emit_sep(v, r, buf + pos);
    }
    while (pos + 1 < n) buf[pos++] = ' ';
    if (pos < n) buf[pos++] = '\n';
    return pos;
}

static size_t fill_grep(const mrc_vocab* v, uint64_t fseed, uint8_t* buf, size_t n, const mrc_params* pp) {
    uint64_t rng = mix64(fseed ^ 0x5A5A5A5Aull);
    const char* pat = pp->pattern ? pp->pattern : "";
    size_t plen = strlen(pat);
    uint32_t match_thr = (uint32_t)(pp->match_rate * 4294967296.0);
    uint32_t dup_thr = (uint32_t)(pp->dup_rate * 4294967296.0);
    int lmin = pp->line_min > 0 ? pp->line_min : 40, lmax = pp->line_max > lmin ? pp->line_max : lmin + 1;
    /* ring of recent matching lines (offsets into buf) for duplicates */
    size_t ring_off[16], ring_len[16];
    int nring = 0, ring_head = 0;
    size_t pos = 0;
    while (pos + (size_t)lmax + plen + 200 < n) {
        uint64_t r = splitmix64(&rng);
        int is_match = plen > 0 && (uint32_t)r < match_thr;
        if (is_match && nring > 0 && (uint32_t)(r >> 32) < dup_thr) {
            int idx = (int)((r >> 8) % (uint64_t)nring);
            memmove(buf + pos, buf + ring_off[idx], ring_len[idx]);
            pos += ring_len[idx];
            buf[pos++] = '\n';
            continue;
        }
        size_t target = (size_t)lmin + (size_t)((r >> 16) % (uint64_t)(lmax - lmin));
        size_t ls = pos;
        int planted = !is_match;
        size_t plant_at = ls + (size_t)((r >> 24) % (target > 8 ? target - 8 : 1));
        while (pos - ls < target) {
            if (!planted && pos >= plant_at) {
                memcpy(buf + pos, pat, plen); pos += plen; planted = 1;
            } else {
                pos += (size_t)emit_word(v, sample_rank(v, &rng), buf + pos);
            }
            uint64_t s = splitmix64(&rng);
            uint32_t x = (uint32_t)(s % 100u);
            if (x < 85) buf[pos++] = ' ';
            else if (v->kind == MRC_KIND_UTF8 && x < 92) pos += (size_t)put_utf8(buf + pos, (s >> 8) & 1 ? 0x2014 : 0x3001);
            else buf[pos++] = (uint8_t)kPunct[(s >> 12) % 10u];
        }
        if (is_match) {
            ring_off[ring_head] = ls; ring_len[ring_head] = pos - ls;
            ring_head = (ring_head + 1) & 15; if (nring < 16) nring++;
        }
        buf[pos++] = '\n';
    }
    while (pos + 1 < n) buf[pos++] = ' ';
    if (pos < n) buf[pos++] = '\n';
    return pos;
}

/* Fill exactly n bytes of file text; returns n.  buf must hold n bytes. */
size_t mrc_fill(const mrc_vocab* v, uint64_t file_seed, uint8_t* buf, size_t n, const mrc_params* pp) {
    if (n == 0) return 0;
    if (pp && pp->mode == MRC_MODE_GREP) return fill_grep(v, file_seed, buf, n, pp);
    return fill_wc(v, file_seed, buf, n, pp);
}

typedef struct {
    const mrc_vocab* v;
    const uint64_t* seeds;
    uint8_t* const* bufs;
    const size_t* sizes;
    const mrc_params* pp;
    size_t nfiles;
    size_t next;
    pthread_mutex_t mu;
} fill_job;

static void* fill_worker(void* arg) {
    fill_job* j = (fill_job*)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        size_t f = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (f >= j->nfiles) return NULL;
        mrc_fill(j->v, j->seeds[f], j->bufs[f], j->sizes[f], j->pp);
    }
}

/* Generate nfiles files in parallel on up to nthreads host threads. */
int mrc_fill_files(const mrc_vocab* v, const uint64_t* seeds, uint8_t* const* bufs, const size_t* sizes,
                   size_t nfiles, const mrc_params* pp, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > nfiles) nthreads = (int)nfiles;
    fill_job j = {v, seeds, bufs, sizes, pp, nfiles, 0, PTHREAD_MUTEX_INITIALIZER};
    pthread_t th[256];
    if (nthreads > 256) nthreads = 256;
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, fill_worker, &j);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    return 0;
}
