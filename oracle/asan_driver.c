/*
 * asan_driver.c — TEST INFRASTRUCTURE: runs the oracle's restatements on the
 * files named on the command line under AddressSanitizer / UBSan (the host-code
 * analogue of `go build -race` in SURVEY.md §5): oracle_mr_partitioned vs
 * oracle_count_mt with 1 and 3 threads, and oracle_merge_parts over the files'
 * separate outputs, for wc and for grep:<pattern>.  Exit 0 iff all agree.
 *   asan_driver PATTERN NREDUCE file...
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_mr_partitioned(int app, const uint8_t* pat, size_t pn, const uint8_t* const* files, const size_t* sizes,
                          size_t nfiles, uint32_t nreduce, uint8_t** out, size_t* out_n, uint64_t* offsets);
int oracle_count_mt(int app, const uint8_t* pat, size_t pn, const uint8_t* s, size_t n, int nthreads, uint32_t nreduce,
                    uint8_t** out, size_t* out_n, uint64_t* offsets);
int oracle_merge_parts(int app, uint32_t nins, const uint8_t* const* ins, const uint64_t* in_offs, uint32_t nreduce,
                       uint8_t** out, size_t* out_n, uint64_t* offsets);

static uint8_t* slurp(const char* p, size_t* n) {
    FILE* f = fopen(p, "rb");
    if (!f) { perror(p); exit(2); }
    fseek(f, 0, SEEK_END);
    long m = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* b = (uint8_t*)malloc((size_t)m + 1);
    if (m && fread(b, 1, (size_t)m, f) != (size_t)m) { perror(p); exit(2); }
    fclose(f);
    *n = (size_t)m;
    return b;
}

int main(int argc, char** argv) {
    if (argc < 4) { fprintf(stderr, "usage: asan_driver PATTERN NREDUCE file...\n"); return 2; }
    const uint8_t* pat = (const uint8_t*)argv[1];
    const size_t pn = strlen(argv[1]);
    const uint32_t R = (uint32_t)atoi(argv[2]);
    const int nf = argc - 3;
    uint8_t** files = calloc((size_t)nf, sizeof(uint8_t*));
    size_t* sizes = calloc((size_t)nf, sizeof(size_t));
    for (int i = 0; i < nf; i++) files[i] = slurp(argv[3 + i], &sizes[i]);
    int bad = 0;
    for (int app = 1; app <= 2; app++) {
        for (int i = 0; i < nf; i++) {  /* one split: the partitioned oracle vs the threaded count */
            uint8_t *a, *b;
            size_t an, bn;
            uint64_t* oa = calloc(R + 1, 8);
            uint64_t* ob = calloc(R + 1, 8);
            oracle_mr_partitioned(app, pat, pn, (const uint8_t* const*)&files[i], &sizes[i], 1, R, &a, &an, oa);
            for (int th = 1; th <= 3; th += 2) {
                oracle_count_mt(app, pat, pn, files[i], sizes[i], th, R, &b, &bn, ob);
                if (an != bn || memcmp(a, b, an) || memcmp(oa, ob, (R + 1) * 8)) { fprintf(stderr, "mismatch app %d file %d th %d\n", app, i, th); bad = 1; }
                free(b);
            }
            free(a); free(oa); free(ob);
        }
        /* all files: the partitioned oracle vs the merge of per-file outputs */
        uint8_t* all;
        size_t alln;
        uint64_t* oall = calloc(R + 1, 8);
        oracle_mr_partitioned(app, pat, pn, (const uint8_t* const*)files, sizes, (size_t)nf, R, &all, &alln, oall);
        uint8_t** outs = calloc((size_t)nf, sizeof(uint8_t*));
        uint64_t* offs = calloc((size_t)nf * (R + 1), 8);
        for (int i = 0; i < nf; i++) {
            size_t on;
            oracle_count_mt(app, pat, pn, files[i], sizes[i], 2, R, &outs[i], &on, offs + (size_t)i * (R + 1));
        }
        uint8_t* m;
        size_t mn;
        uint64_t* om = calloc(R + 1, 8);
        oracle_merge_parts(app, (uint32_t)nf, (const uint8_t* const*)outs, offs, R, &m, &mn, om);
        if (mn != alln || memcmp(m, all, alln) || memcmp(om, oall, (R + 1) * 8)) { fprintf(stderr, "merge mismatch app %d\n", app); bad = 1; }
        for (int i = 0; i < nf; i++) free(outs[i]);
        free(outs); free(offs); free(m); free(om); free(all); free(oall);
    }
    for (int i = 0; i < nf; i++) free(files[i]);
    free(files); free(sizes);
    if (!bad) printf("ok\n");
    return bad;
}
