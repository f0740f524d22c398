// mrhost_util.h — shared helpers of the C++ hosts over the C ABI (mrhost.cpp,
// mrcoord.cpp): file I/O with the reference's error behaviour (log.Fatalf ->
// message + exit 1, worker.go:60-64), temp + rename outputs (worker.go:83,91),
// and the APP argument ("wc" | "grep:<literal>"), the plugin choice of
// main/mrworker.go:34-51.
#pragma once
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mrgpu.h"

namespace mrhost {

[[noreturn]] inline void fatalf(const char* fmt, const char* a, const char* b = "") {
    fprintf(stderr, fmt, a, b);
    fputc('\n', stderr);
    exit(1);
}

inline std::vector<uint8_t> read_file(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) fatalf("cannot open %s", path);
    std::vector<uint8_t> b;
    uint8_t tmp[1 << 16];
    size_t n;
    while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) b.insert(b.end(), tmp, tmp + n);
    if (ferror(f)) fatalf("cannot read %s", path);
    fclose(f);
    return b;
}

inline bool read_file_opt(const std::string& path, std::vector<uint8_t>* out) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fclose(f);
    *out = read_file(path.c_str());
    return true;
}

// All of a file, or false if it does not exist (a reduce input that an accepted
// duplicate of the task removed meanwhile: the caller abandons the task).  Any
// other failure (EACCES, EMFILE, EIO, a read error) is fatal: abandoning the task
// would make the coordinator re-issue it forever instead of failing the job.
inline bool read_file_try(const std::string& path, std::vector<uint8_t>* out) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) {
        if (errno == ENOENT) return false;
        fatalf("cannot open %s: %s", path.c_str(), strerror(errno));
    }
    out->clear();
    uint8_t tmp[1 << 16];
    size_t n;
    while ((n = fread(tmp, 1, sizeof tmp, f)) > 0) out->insert(out->end(), tmp, tmp + n);
    if (ferror(f)) fatalf("cannot read %s", path.c_str());  // an unlinked file stays readable: a real I/O error
    fclose(f);
    return true;
}

// Temp + rename, as worker.go:83,91 (ioutil.TempFile + os.Rename): the temp file
// gets a unique name in the output's directory (mkstemp), so a re-issued task
// and the slow worker it replaced never write one inode or rename each other's
// file away; the data is flushed to disk before the rename publishes it.
inline void write_file_atomic(const std::string& name, const void* p, size_t n) {
    std::string tmpl = name + ".tmp-XXXXXX";
    std::vector<char> path(tmpl.begin(), tmpl.end());
    path.push_back('\0');
    const int fd = mkstemp(path.data());
    if (fd < 0) fatalf("cannot create %s", tmpl.c_str());
    const char* b = (const char*)p;
    size_t left = n;
    while (left) {
        const ssize_t k = write(fd, b, left);
        if (k <= 0) {
            unlink(path.data());
            fatalf("cannot write into %s", name.c_str());
        }
        b += k;
        left -= (size_t)k;
    }
    if (fsync(fd) != 0 || close(fd) != 0) {
        unlink(path.data());
        fatalf("cannot write into %s", name.c_str());
    }
    if (rename(path.data(), name.c_str()) != 0) {
        unlink(path.data());
        fatalf("cannot rename %s", path.data());
    }
}

struct App {
    int id;
    std::string pat;
};

inline App parse_app(const char* a) {
    if (!strcmp(a, "wc")) return {MRG_APP_WC, ""};
    if (!strncmp(a, "grep:", 5)) return {MRG_APP_GREP, std::string(a + 5)};
    fatalf("unknown app %s (want wc or grep:<literal>)", a);
}

inline void check(mrg_ctx* c, int rc, const char* what) {
    if (rc != MRG_OK) fatalf("%s failed: %s", what, mrg_last_error(c));
}

inline mrg_parts* map_split(mrg_ctx* c, const App& app, const std::vector<uint8_t>& data, uint32_t nreduce) {
    mrg_parts* p = nullptr;
    check(c, mrg_map(c, app.id, data.data(), data.size(), MRG_INPUT_HOST, (const uint8_t*)app.pat.data(),
                     app.pat.size(), nreduce, &p),
          "mrg_map");
    return p;
}

}  // namespace mrhost
