// mrhost.cpp — C++ host side over the C ABI (the reference's Go host is not
// buildable here: no Go toolchain; INTEGRATION.md shows the cgo binding).
//
//   mrseq_gpu APP file...            main/mrsequential.go:25-87 — read every input
//                                    file, Map it, sort/group/Reduce everything into
//                                    ./mr-out-0.
//   mrjob_gpu [-n R] APP file...     the worker flow of mr/worker.go:55-161 without
//                                    the RPC coordinator: map task X per file writes
//                                    intermediates mr-X-r (r < R); then reduce task r
//                                    reads mr-i-r for every i (missing files skipped,
//                                    worker.go:105-108), writes mr-out-r, removes its
//                                    inputs (worker.go:151-154).
// APP is "wc" or "grep:<literal>".  Errors: message on stderr, exit 1 — the
// log.Fatalf behaviour of worker.go:60-64 / mrsequential.go:42-46.
#include "mrhost_util.h"

namespace {

using namespace mrhost;

int main_seq(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "Usage: mrseq_gpu wc|grep:<literal> inputfiles...\n");
        return 1;
    }
    App app = parse_app(argv[1]);
    mrg_ctx* c = nullptr;
    if (mrg_open(0, &c) != MRG_OK) fatalf("%s: no GPU context", "mrg_open");
    mrg_parts* all = nullptr;
    for (int i = 2; i < argc; i++) {  // mrsequential.go:39-51
        std::vector<uint8_t> data = read_file(argv[i]);
        mrg_parts* p = map_split(c, app, data, 1);
        if (!all) all = p;
        else {
            check(c, mrg_parts_merge(c, all, p), "mrg_parts_merge");
            mrg_parts_free(p);
        }
    }
    void* out = nullptr;
    size_t n = 0;
    uint64_t offs[2];
    check(c, mrg_reduce_all(c, all, &out, &n, offs), "mrg_reduce_all");  // mrsequential.go:59-84
    write_file_atomic("mr-out-0", out, n);
    mrg_free(out);
    mrg_parts_free(all);
    mrg_close(c);
    return 0;
}

int main_job(int argc, char** argv) {
    uint32_t nreduce = 10;  // mrcoordinator.go:23
    int i = 1;
    if (i + 1 < argc && !strcmp(argv[i], "-n")) {
        nreduce = (uint32_t)atoi(argv[i + 1]);
        i += 2;
    }
    if (argc - i < 2 || nreduce == 0) {
        fprintf(stderr, "Usage: mrjob_gpu [-n nreduce] wc|grep:<literal> inputfiles...\n");
        return 1;
    }
    App app = parse_app(argv[i++]);
    const int nmap = argc - i;
    mrg_ctx* c = nullptr;
    if (mrg_open(0, &c) != MRG_OK) fatalf("%s: no GPU context", "mrg_open");
    char name[4096];
    for (int x = 0; x < nmap; x++) {  // map task x (worker.go:55-97)
        std::vector<uint8_t> data = read_file(argv[i + x]);
        mrg_parts* p = map_split(c, app, data, nreduce);
        for (uint32_t r = 0; r < nreduce; r++) {
            void* b = nullptr;
            size_t nb = 0;
            check(c, mrg_parts_export(c, p, r, &b, &nb), "mrg_parts_export");
            snprintf(name, sizeof name, "mr-%d-%u", x, r);
            write_file_atomic(name, b, nb);
            mrg_free(b);
        }
        mrg_parts_free(p);
    }
    for (uint32_t r = 0; r < nreduce; r++) {  // reduce task r (worker.go:99-161)
        mrg_parts* acc = nullptr;
        for (int x = 0; x < nmap; x++) {
            snprintf(name, sizeof name, "mr-%d-%u", x, r);
            std::vector<uint8_t> b;
            if (!read_file_opt(name, &b)) continue;  // worker.go:105-108
            mrg_parts* q = nullptr;
            check(c, mrg_parts_import(c, b.data(), b.size(), &q), "mrg_parts_import");
            if (!acc) acc = q;
            else {
                check(c, mrg_parts_merge(c, acc, q), "mrg_parts_merge");
                mrg_parts_free(q);
            }
        }
        void* out = nullptr;
        size_t n = 0;
        if (acc) {
            check(c, mrg_reduce(c, acc, r, &out, &n), "mrg_reduce");
            mrg_parts_free(acc);
        }
        snprintf(name, sizeof name, "mr-out-%u", r);
        write_file_atomic(name, out, n);  // an empty partition still gets its file (worker.go:126-148)
        mrg_free(out);
        for (int x = 0; x < nmap; x++) {
            snprintf(name, sizeof name, "mr-%d-%u", x, r);
            remove(name);
        }
    }
    mrg_close(c);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
#if defined(MRHOST_MAIN_SEQ)
    return main_seq(argc, argv);
#else
    return main_job(argc, argv);
#endif
}
