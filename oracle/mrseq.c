/*
 * mrseq.c — single-process CPU restatement of main/mrsequential.go:25-87.
 *
 * TEST INFRASTRUCTURE ONLY: bench.py's single-thread cpu_baseline variant
 * ("kind": "port") and a checker for the C1 plumbing config.  Not part of the
 * product.
 *
 * Mirrors (paths under /root/reference/MapReduce):
 *   read every input file and Map it            main/mrsequential.go:39-51
 *   sort.Sort(ByKey(intermediate)) over all KVs  main/mrsequential.go:59
 *   group equal keys, Reduce, Fprintf "%v %v\n"  main/mrsequential.go:61-84
 * The map / sort / group / Reduce are oracle_mrsequential (mroracle.c); the
 * output leaves as one write(2) per key like the reference's unbuffered
 * fmt.Fprintf on *os.File (--buffered: one write for everything).
 *
 * usage: mrseq [--app wc|grep] [--pattern P] [--buffered] [--out mr-out-0] file...
 * prints: {"seconds": t, "bytes": n, "keys": k}
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

int oracle_mrsequential(int app, const uint8_t* pat, size_t pn, const uint8_t* const* files, const size_t* sizes,
                        size_t nfiles, uint8_t** out, size_t* out_n);
void oracle_free(void* p);

static uint8_t* read_file(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) { fprintf(stderr, "cannot open %s\n", path); exit(1); }  /* mrsequential.go:42 */
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* b = (uint8_t*)malloc((size_t)sz + 1);
    if (sz && fread(b, 1, (size_t)sz, f) != (size_t)sz) { fprintf(stderr, "cannot read %s\n", path); exit(1); }
    fclose(f);
    *n = (size_t)sz;
    return b;
}

int main(int argc, char** argv) {
    int app = 1, buffered = 0;
    const char* pat = "";
    const char* outp = "mr-out-0";
    int i = 1;
    for (; i < argc; i++) {
        if (!strcmp(argv[i], "--app")) app = !strcmp(argv[++i], "wc") ? 1 : 2;
        else if (!strcmp(argv[i], "--pattern")) pat = argv[++i];
        else if (!strcmp(argv[i], "--buffered")) buffered = 1;
        else if (!strcmp(argv[i], "--out")) outp = argv[++i];
        else break;
    }
    const int nfiles = argc - i;
    if (nfiles <= 0) { fprintf(stderr, "usage: mrseq [--app wc|grep] [--pattern P] [--buffered] file...\n"); return 1; }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    const uint8_t** bufs = (const uint8_t**)calloc((size_t)nfiles, sizeof(uint8_t*));
    size_t* sizes = (size_t*)calloc((size_t)nfiles, sizeof(size_t));
    size_t total = 0;
    for (int f = 0; f < nfiles; f++) {
        bufs[f] = read_file(argv[i + f], &sizes[f]);
        total += sizes[f];
    }
    uint8_t* out = NULL;
    size_t on = 0;
    oracle_mrsequential(app, (const uint8_t*)pat, strlen(pat), bufs, sizes, (size_t)nfiles, &out, &on);
    int fd = open(outp, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) { perror(outp); return 1; }
    size_t keys = 0;
    if (buffered) {
        if (on && write(fd, out, on) != (ssize_t)on) { perror("write"); return 1; }
        for (size_t k = 0; k < on; k++) keys += out[k] == '\n';
    } else {
        size_t s = 0;
        for (size_t k = 0; k < on; k++) {
            if (out[k] != '\n') continue;
            if (write(fd, out + s, k + 1 - s) != (ssize_t)(k + 1 - s)) { perror("write"); return 1; }
            s = k + 1;
            keys++;
        }
    }
    close(fd);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double sec = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    printf("{\"seconds\": %.6f, \"bytes\": %zu, \"keys\": %zu, \"buffered\": %s}\n", sec, total, keys,
           buffered ? "true" : "false");
    oracle_free(out);
    for (int f = 0; f < nfiles; f++) free((void*)bufs[f]);
    free(bufs);
    free(sizes);
    return 0;
}
