/*
 * mrcpu.c — CPU restatement of the reference's *distributed* MapReduce job
 * (coordinator + N worker processes, JSON-lines M x R shuffle files).
 *
 * TEST INFRASTRUCTURE ONLY: used as bench.py's cpu_baseline ("kind": "port")
 * and by tests as a second checker.  Not part of the product.
 *
 * Mirrors (paths under /root/reference/MapReduce):
 *   coordinator: mr/coordinator.go:43-114 — map tasks first (one per input file),
 *                reduce tasks only after every map task completed, then done.
 *                Here the task table lives in MAP_SHARED memory and workers take
 *                tasks with atomic fetch-adds instead of net/rpc calls (rpc.go).
 *   worker map:  mr/worker.go:55-97 — read file, Map, ihash(key) % nReduce buckets,
 *                one JSON line {"Key":k,"Value":v} per KV into mr-X-Y (temp + rename).
 *   worker red.: mr/worker.go:99-161 — decode mr-i-Y for i < nMap (missing files
 *                skipped), sort by key, group, Reduce, "%v %v\n" into mr-out-Y.
 * Writes: one write(2) per KV line and per output line, the reference's cost
 * structure (--buffered: stdio batching instead).  Difference (documented in
 * DESIGN.md): no 10 s re-issue watchdog (tasks are sized to finish well within it).
 *
 * usage: mrcpu [--app wc|grep] [--pattern P] [--nreduce R] [--workers N] [--buffered] --dir D file...
 * prints: {"seconds": t, "bytes": n, "workers": N, "nmap": M, "nreduce": R}
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#define ORACLE_APP_WC 1
#define ORACLE_APP_GREP 2

size_t oracle_wc_words(const uint8_t* s, size_t n, uint64_t* offs, uint32_t* lens, size_t cap);
size_t oracle_grep_lines(const uint8_t* s, size_t n, const uint8_t* pat, size_t pn, uint64_t* offs,
                         uint32_t* lens, size_t cap);
uint32_t oracle_ihash(const uint8_t* p, size_t n);
size_t oracle_decode_rune(const uint8_t* s, size_t n, size_t i, uint32_t* cp);

typedef struct {
    volatile long next_map, maps_done, next_reduce, reduces_done;
} shared_state;

static int g_app = ORACLE_APP_WC;
static const char* g_pat = "";
static int g_nreduce = 10;
static const char* g_dir = ".";

static uint8_t* read_file(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", path); exit(1); }  /* worker.go:60 log.Fatalf */
    fseek(f, 0, SEEK_END); long sz = ftell(f); fseek(f, 0, SEEK_SET);
    uint8_t* b = (uint8_t*)malloc((size_t)sz + 1);
    if (sz && fread(b, 1, (size_t)sz, f) != (size_t)sz) { fprintf(stderr, "cannot read %s\n", path); exit(1); }
    fclose(f); *n = (size_t)sz; return b;
}

/* A growable byte buffer: one encoded KV line (or one output line) at a time. */
typedef struct { char* b; size_t n, cap; } sbuf;
static void sb_put(sbuf* o, const void* p, size_t n) {
    if (o->n + n > o->cap) {
        size_t c = o->cap ? o->cap : 256;
        while (c < o->n + n) c *= 2;
        o->b = (char*)realloc(o->b, c);
        o->cap = c;
    }
    memcpy(o->b + o->n, p, n);
    o->n += n;
}
static void sb_putc(sbuf* o, char c) { sb_put(o, &c, 1); }
static void sb_puts(sbuf* o, const char* s) { sb_put(o, s, strlen(s)); }

/* Each line leaves as ONE write(2), as the reference's unbuffered *os.File
 * does: json.Encoder.Encode writes the encoded KV in one Write call
 * (worker.go:84-89) and fmt.Fprintf one write per key (worker.go:144,
 * mrsequential.go:81).  --buffered batches them through stdio instead. */
static int g_buffered = 0;
static void emit_line(FILE* f, sbuf* line) {
    if (g_buffered) fwrite(line->b, 1, line->n, f);
    else if (line->n && write(fileno(f), line->b, line->n) != (ssize_t)line->n) { perror("write"); exit(1); }
    line->n = 0;
}

/* encoding/json string encoding (HTML-escaping encoder, the json.NewEncoder default). */
static void json_str(sbuf* o, const uint8_t* s, size_t n) {
    static const char hex[] = "0123456789abcdef";
    sb_putc(o, '"');
    size_t i = 0;
    while (i < n) {
        uint8_t c = s[i];
        if (c < 0x80) {
            if (c == '"' || c == '\\') { sb_putc(o, '\\'); sb_putc(o, (char)c); }
            else if (c == '\n') sb_puts(o, "\\n");
            else if (c == '\r') sb_puts(o, "\\r");
            else if (c == '\t') sb_puts(o, "\\t");
            else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
                char u[6] = {'\\', 'u', '0', '0', hex[c >> 4], hex[c & 15]};
                sb_put(o, u, 6);
            } else sb_putc(o, (char)c);
            i++;
            continue;
        }
        uint32_t cp; size_t w = oracle_decode_rune(s, n, i, &cp);
        if (cp == 0xFFFD && w == 1) sb_puts(o, "\\ufffd");
        else if (cp == 0x2028 || cp == 0x2029) { char u[8]; snprintf(u, sizeof u, "\\u%04x", cp); sb_puts(o, u); }
        else sb_put(o, s + i, w);
        i += w;
    }
    sb_putc(o, '"');
}

static void do_map(const char* path, int x) {
    size_t n; uint8_t* b = read_file(path, &n);
    size_t cap = n / 2 + 16;
    uint64_t* offs = (uint64_t*)malloc(cap * sizeof(uint64_t));
    uint32_t* lens = (uint32_t*)malloc(cap * sizeof(uint32_t));
    size_t nk = g_app == ORACLE_APP_WC ? oracle_wc_words(b, n, offs, lens, cap)
                                      : oracle_grep_lines(b, n, (const uint8_t*)g_pat, strlen(g_pat), offs, lens, cap);
    if (nk > cap) { /* more lines than n/2 only for grep on pathological input */
        free(offs); free(lens); cap = nk;
        offs = (uint64_t*)malloc(cap * sizeof(uint64_t)); lens = (uint32_t*)malloc(cap * sizeof(uint32_t));
        oracle_grep_lines(b, n, (const uint8_t*)g_pat, strlen(g_pat), offs, lens, cap);
    }
    FILE** fs = (FILE**)calloc((size_t)g_nreduce, sizeof(FILE*));
    char tmp[4096], fin[4096];
    for (int r = 0; r < g_nreduce; r++) {
        snprintf(tmp, sizeof tmp, "%s/.tmp-mr-%d-%d-%d", g_dir, x, r, (int)getpid());
        fs[r] = fopen(tmp, "wb");
        setvbuf(fs[r], NULL, _IOFBF, 1 << 16);
    }
    sbuf line = {0};
    for (size_t i = 0; i < nk; i++) {       /* worker.go:74-78 then :84-89 */
        int r = (int)(oracle_ihash(b + offs[i], lens[i]) % (uint32_t)g_nreduce);
        sb_puts(&line, "{\"Key\":");
        json_str(&line, b + offs[i], lens[i]);
        sb_puts(&line, g_app == ORACLE_APP_WC ? ",\"Value\":\"1\"}\n" : ",\"Value\":\"\"}\n");
        emit_line(fs[r], &line);
    }
    free(line.b);
    for (int r = 0; r < g_nreduce; r++) {
        fclose(fs[r]);
        snprintf(tmp, sizeof tmp, "%s/.tmp-mr-%d-%d-%d", g_dir, x, r, (int)getpid());
        snprintf(fin, sizeof fin, "%s/mr-%d-%d", g_dir, x, r);
        rename(tmp, fin);                   /* worker.go:91 */
    }
    free(fs); free(offs); free(lens); free(b);
}

typedef struct { uint8_t* p; uint32_t n; uint32_t vn; } kv_t;

static int kv_cmp(const void* a, const void* b) {
    const kv_t* x = (const kv_t*)a; const kv_t* y = (const kv_t*)b;
    uint32_t m = x->n < y->n ? x->n : y->n;
    int c = memcmp(x->p, y->p, m);
    return c ? c : (x->n > y->n) - (x->n < y->n);
}

static int hexv(int c) { return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10; }

/* decode a JSON string starting after the opening quote; writes bytes to o; returns ptr after closing quote */
static const char* json_unstr(const char* s, uint8_t* o, uint32_t* on) {
    uint32_t n = 0;
    while (*s != '"') {
        if (*s == '\\') {
            s++;
            switch (*s) {
                case 'n': o[n++] = '\n'; s++; break;
                case 'r': o[n++] = '\r'; s++; break;
                case 't': o[n++] = '\t'; s++; break;
                case 'b': o[n++] = '\b'; s++; break;
                case 'f': o[n++] = '\f'; s++; break;
                case 'u': {
                    uint32_t cp = (uint32_t)(hexv(s[1]) << 12 | hexv(s[2]) << 8 | hexv(s[3]) << 4 | hexv(s[4]));
                    s += 5;
                    if (cp < 0x80) o[n++] = (uint8_t)cp;
                    else if (cp < 0x800) { o[n++] = 0xC0 | (cp >> 6); o[n++] = 0x80 | (cp & 0x3F); }
                    else { o[n++] = 0xE0 | (cp >> 12); o[n++] = 0x80 | ((cp >> 6) & 0x3F); o[n++] = 0x80 | (cp & 0x3F); }
                    break;
                }
                default: o[n++] = (uint8_t)*s++; break;
            }
        } else o[n++] = (uint8_t)*s++;
    }
    *on = n;
    return s + 1;
}

static void do_reduce(int y, int nmap) {
    kv_t* kv = NULL; size_t nkv = 0, cap = 0;
    uint8_t** bufs = (uint8_t**)calloc((size_t)nmap, sizeof(uint8_t*));
    char path[4096];
    for (int i = 0; i < nmap; i++) {
        snprintf(path, sizeof path, "%s/mr-%d-%d", g_dir, i, y);
        struct stat st;
        if (stat(path, &st) != 0) continue;  /* worker.go:105-108 skip missing */
        size_t n; uint8_t* b = read_file(path, &n);
        bufs[i] = b;
        uint8_t* w = b;                         /* decode in place: decoded <= encoded */
        const char* s = (const char*)b;
        const char* end = (const char*)b + n;
        while (s < end && *s == '{') {
            s += 8;                              /* {"Key":" */
            uint32_t kn; s = json_unstr(s, w, &kn);
            uint8_t* kp = w; w += kn;
            s += 10;                             /* ,"Value":" */
            uint32_t vn; uint8_t vtmp[8]; (void)vtmp;
            const char* vs = s; while (*s != '"') s++; vn = (uint32_t)(s - vs); s += 3; /* "}\n */
            if (nkv == cap) { cap = cap ? cap * 2 : 4096; kv = (kv_t*)realloc(kv, cap * sizeof(kv_t)); }
            kv[nkv].p = kp; kv[nkv].n = kn; kv[nkv].vn = vn; nkv++;
        }
    }
    qsort(kv, nkv, sizeof(kv_t), kv_cmp);      /* worker.go:124 */
    char tmp[4096], fin[4096];
    snprintf(tmp, sizeof tmp, "%s/.tmp-mr-out-%d-%d", g_dir, y, (int)getpid());
    FILE* o = fopen(tmp, "wb");
    setvbuf(o, NULL, _IOFBF, 1 << 16);
    size_t i = 0;
    sbuf line = {0};
    char num[32];
    while (i < nkv) {                           /* worker.go:129-146 */
        size_t j = i + 1;
        while (j < nkv && kv[j].n == kv[i].n && memcmp(kv[j].p, kv[i].p, kv[i].n) == 0) j++;
        sb_put(&line, kv[i].p, kv[i].n);
        sb_putc(&line, ' ');
        if (g_app == ORACLE_APP_WC) { int k = snprintf(num, sizeof num, "%zu", j - i); sb_put(&line, num, (size_t)k); }
        else sb_put(&line, kv[i].p, kv[i].n);
        sb_putc(&line, '\n');
        emit_line(o, &line);
        i = j;
    }
    free(line.b);
    fclose(o);
    snprintf(fin, sizeof fin, "%s/mr-out-%d", g_dir, y);
    rename(tmp, fin);
    for (int k = 0; k < nmap; k++) {           /* worker.go:151-154 */
        snprintf(path, sizeof path, "%s/mr-%d-%d", g_dir, k, y);
        unlink(path);
        free(bufs[k]);
    }
    free(bufs); free(kv);
}

static void worker_loop(shared_state* st, char** files, int nmap) {
    for (;;) {                                  /* worker.go:46-54 RequestTask loop */
        long m = __atomic_load_n(&st->next_map, __ATOMIC_SEQ_CST);
        if (m < nmap) {
            m = __atomic_fetch_add(&st->next_map, 1, __ATOMIC_SEQ_CST);
            if (m < nmap) {
                do_map(files[m], (int)m);
                __atomic_fetch_add(&st->maps_done, 1, __ATOMIC_SEQ_CST);
            }
            continue;
        }
        if (__atomic_load_n(&st->maps_done, __ATOMIC_SEQ_CST) < nmap) { usleep(200); continue; } /* status 2 */
        long r = __atomic_fetch_add(&st->next_reduce, 1, __ATOMIC_SEQ_CST);
        if (r >= g_nreduce) return;             /* status 3 */
        do_reduce((int)r, nmap);
        __atomic_fetch_add(&st->reduces_done, 1, __ATOMIC_SEQ_CST);
    }
}

int main(int argc, char** argv) {
    int workers = 8;
    int i = 1;
    for (; i < argc; i++) {
        if (!strcmp(argv[i], "--app")) { const char* a = argv[++i]; g_app = !strcmp(a, "wc") ? ORACLE_APP_WC : ORACLE_APP_GREP; }
        else if (!strcmp(argv[i], "--pattern")) g_pat = argv[++i];
        else if (!strcmp(argv[i], "--nreduce")) g_nreduce = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--workers")) workers = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--dir")) g_dir = argv[++i];
        else if (!strcmp(argv[i], "--buffered")) g_buffered = 1;
        else break;
    }
    char** files = argv + i;
    int nmap = argc - i;
    if (nmap <= 0) { fprintf(stderr, "usage: mrcpu [opts] --dir D files...\n"); return 1; }
    size_t total = 0;
    for (int f = 0; f < nmap; f++) { struct stat st; if (stat(files[f], &st) == 0) total += (size_t)st.st_size; }
    shared_state* st = (shared_state*)mmap(NULL, sizeof(shared_state), PROT_READ | PROT_WRITE,
                                           MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    memset((void*)st, 0, sizeof *st);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int w = 0; w < workers; w++) {
        pid_t p = fork();
        if (p == 0) { worker_loop(st, files, nmap); _exit(0); }
    }
    int status, ok = 1;
    for (int w = 0; w < workers; w++) { wait(&status); if (!WIFEXITED(status) || WEXITSTATUS(status)) ok = 0; }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double sec = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    printf("{\"seconds\": %.6f, \"bytes\": %zu, \"workers\": %d, \"nmap\": %d, \"nreduce\": %d, \"buffered\": %s, "
           "\"ok\": %s}\n",
           sec, total, workers, nmap, g_nreduce, g_buffered ? "true" : "false", ok ? "true" : "false");
    return ok ? 0 : 1;
}
