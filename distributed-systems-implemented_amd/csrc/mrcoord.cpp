// mrcoord.cpp — coordinator-driven multi-process GPU mode.
//
//   mrcoord_gpu [-n R] [-w P] [--json] [--sock PATH] [--task-timeout S] APP file...
//       mr/coordinator.go + main/mrcoordinator.go: serves the task protocol on a
//       unix socket and (-w P > 0) forks P worker processes, worker k on GPU
//       k % ndev.  Exits when every reduce task is done (Done(), coordinator.go:138-142).
//   mrworker_gpu [--json] [--sock PATH] [--device D] APP
//       mr/worker.go Worker() + main/mrworker.go: one process per GPU, pulling tasks.
//
// Protocol (mr/rpc.go): every call dials the socket, sends one request
// {method, TaskNumber} and reads one WorkerReply {TaskStatus 0 map | 1 reduce |
// 2 wait | 3 done, NMap, CMap, NReduce, CReduce, Filename} — the fields of
// rpc.go:18-33, carried as a fixed binary frame instead of Go's net/rpc gob
// (the RPC layer itself is out of scope).
//
// Coordinator (coordinator.go:43-114): a map task is handed out while any is
// untouched; reduce tasks only after every map task COMPLETED; status 2 while
// everything is in progress; 3 when all reduce tasks are done.  A task still in
// progress after the re-issue timeout (10 s, coordinator.go:70-77,99-106) is
// handed out again.  Deliberate fixes of the hazards SURVEY.md §5 lists:
// a completion counts once per task (the reference increments cMap / cReduce
// for every completion RPC, so a re-issued task finishing twice could start the
// reduce phase early or never end, coordinator.go:30,38), and a waiting worker
// sleeps instead of re-dialing in a tight loop (worker.go:46-54).
//
// Worker (worker.go:55-161) over the C ABI: map task X = mrg_map of the whole
// file, then one intermediate file mr-X-r per partition (temp + rename,
// worker.go:80-92) — MRGI partials (mrg_parts_export), or with --json the
// reference's JSON lines (mrg_parts_export_json), which unmodified reference
// reduce workers can read.  Reduce task r reads mr-i-r for every i (missing
// files skipped, worker.go:102-108), merges, formats mr-out-r (temp + rename)
// and removes its inputs (worker.go:150-154).  The GPU is initialised only in
// the worker processes (the coordinator never touches it, so forking is safe).
//
// Duplicate tasks (a slow worker and its re-issued replacement) are safe here,
// unlike in the reference: temp files are unique (mkstemp); every map task
// writes all nReduce mr-X-r, so a reduce task that finds one missing (or sees
// it vanish mid-read) abandons the task without writing mr-out-r; and a reduce
// worker removes its inputs only when the coordinator accepted its completion
// as the first (the reply's CReduce field is 1), so a late duplicate never reads
// a half-deleted input set.  A duplicate that read every input writes the same
// mr-out-r bytes, so its rename is harmless.
#include <errno.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <thread>

#include "mrhost_util.h"

namespace {

using namespace mrhost;

enum Method : uint32_t { kRequestTask = 1, kMapComplete = 2, kReduceComplete = 3 };
enum Status : int32_t { kMap = 0, kReduce = 1, kWait = 2, kDone = 3 };
constexpr uint32_t kMagic = 0x4D52434Fu;  // "MRCO"

struct Request {
    uint32_t magic, method;
    int64_t task;  // WorkerArgs.TaskNumber (rpc.go:18-20)
};
struct ReplyHdr {  // WorkerReply (rpc.go:22-33)
    uint32_t magic;
    int32_t status, nmap, cmap, nreduce, creduce;
    uint32_t fname_len;
};

std::string default_sock() { return "/var/tmp/824-mr-" + std::to_string(getuid()); }  // rpc.go:37-41

bool write_all(int fd, const void* p, size_t n) {
    const char* b = (const char*)p;
    while (n) {
        ssize_t k = write(fd, b, n);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        b += k;
        n -= (size_t)k;
    }
    return true;
}
bool read_all(int fd, void* p, size_t n) {
    char* b = (char*)p;
    while (n) {
        ssize_t k = read(fd, b, n);
        if (k < 0 && errno == EINTR) continue;
        if (k <= 0) return false;
        b += k;
        n -= (size_t)k;
    }
    return true;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ------------------------------------------------------------ coordinator
struct Coordinator {
    std::vector<std::string> files;
    int nmap = 0, nreduce = 10;
    int cmap = 0, creduce = 0;
    std::vector<int> map_log, reduce_log;        // 0 untouched, 1 in progress, 2 completed
    std::vector<double> map_since, reduce_since;  // when the in-progress task was handed out
    double timeout = 10.0;                         // coordinator.go:71,100
    uint64_t reissued = 0;

    // coordinator.go:70-77 / :99-106 — checked on every loop turn instead of a goroutine per task
    void expire() {
        const double t = now_s();
        for (int i = 0; i < nmap; i++)
            if (map_log[i] == 1 && t - map_since[i] >= timeout) { map_log[i] = 0; reissued++; }
        for (int i = 0; i < nreduce; i++)
            if (reduce_log[i] == 1 && t - reduce_since[i] >= timeout) { reduce_log[i] = 0; reissued++; }
    }

    // coordinator.go:43-114
    ReplyHdr request_task(std::string* fname) {
        ReplyHdr r{kMagic, kWait, nmap, 0, nreduce, 0, 0};
        if (cmap < nmap) {
            for (int i = 0; i < nmap; i++)
                if (map_log[i] == 0) {
                    map_log[i] = 1;
                    map_since[i] = now_s();
                    r.status = kMap;
                    r.cmap = i;
                    *fname = files[i];
                    break;
                }
        } else if (creduce < nreduce) {
            for (int i = 0; i < nreduce; i++)
                if (reduce_log[i] == 0) {
                    reduce_log[i] = 1;
                    reduce_since[i] = now_s();
                    r.status = kReduce;
                    r.creduce = i;
                    break;
                }
        } else {
            r.status = kDone;
        }
        r.fname_len = (uint32_t)fname->size();
        return r;
    }
    // coordinator.go:27-41, counted once per task; true if this completion is
    // the first (accepted)
    bool map_complete(int64_t x) {
        if (x < 0 || x >= nmap || map_log[x] == 2) return false;
        map_log[x] = 2;
        cmap++;
        return true;
    }
    bool reduce_complete(int64_t x) {
        if (x < 0 || x >= nreduce || reduce_log[x] == 2) return false;
        reduce_log[x] = 2;
        creduce++;
        return true;
    }
    bool done() const { return creduce == nreduce; }  // coordinator.go:138-142
};

int listen_sock(const std::string& path) {
    unlink(path.c_str());  // coordinator.go:126
    int fd = socket(AF_UNIX, SOCK_STREAM, 0);
    if (fd < 0) fatalf("socket: %s", strerror(errno));
    sockaddr_un a{};
    a.sun_family = AF_UNIX;
    if (path.size() >= sizeof a.sun_path) fatalf("socket path too long: %s", path.c_str());
    strcpy(a.sun_path, path.c_str());
    if (bind(fd, (sockaddr*)&a, sizeof a) != 0 || listen(fd, 128) != 0)
        fatalf("listen error: %s (%s)", strerror(errno), path.c_str());  // coordinator.go:128-130
    return fd;
}

void serve_one(Coordinator& co, int lfd) {
    int fd = accept(lfd, nullptr, nullptr);
    if (fd < 0) return;
    // a client that connects and never sends must not stall the loop (and with
    // it expire() and every other worker): bounded reads and writes
    timeval tv{0, 500000};  // a worker sends its request right after connecting
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    Request q{};
    if (read_all(fd, &q, sizeof q) && q.magic == kMagic) {
        std::string fname;
        ReplyHdr r{kMagic, kWait, co.nmap, 0, co.nreduce, 0, 0};
        // completion replies: CMap / CReduce = 1 if this completion was accepted
        if (q.method == kRequestTask) r = co.request_task(&fname);
        else if (q.method == kMapComplete) r.cmap = co.map_complete(q.task) ? 1 : 0;
        else if (q.method == kReduceComplete) r.creduce = co.reduce_complete(q.task) ? 1 : 0;
        if (write_all(fd, &r, sizeof r)) write_all(fd, fname.data(), fname.size());
    }
    close(fd);
}

// ------------------------------------------------------------ worker
struct WorkerOpts {
    std::string sock;
    bool json = false;
    int device = -1;  // -1: worker index % device count
    int index = 0;
};

// worker.go:172-188: dial per call; false when the coordinator is gone
bool call(const std::string& sock, uint32_t method, int64_t task, ReplyHdr* r, std::string* fname) {
    int fd = socket(AF_UNIX, SOCK_STREAM, 0);
    if (fd < 0) return false;
    sockaddr_un a{};
    a.sun_family = AF_UNIX;
    strncpy(a.sun_path, sock.c_str(), sizeof a.sun_path - 1);
    if (connect(fd, (sockaddr*)&a, sizeof a) != 0) {
        close(fd);
        return false;
    }
    Request q{kMagic, method, task};
    bool ok = write_all(fd, &q, sizeof q) && read_all(fd, r, sizeof *r) && r->magic == kMagic;
    if (ok && r->fname_len) {
        fname->resize(r->fname_len);
        ok = read_all(fd, &(*fname)[0], r->fname_len);
    } else if (ok) {
        fname->clear();
    }
    close(fd);
    return ok;
}

void do_map(mrg_ctx* c, const App& app, const WorkerOpts& o, const ReplyHdr& r, const std::string& fname) {
    std::vector<uint8_t> data = read_file(fname.c_str());  // worker.go:58-66
    mrg_parts* p = map_split(c, app, data, (uint32_t)r.nreduce);
    char name[64];
    for (int k = 0; k < r.nreduce; k++) {  // worker.go:81-92
        void* b = nullptr;
        size_t nb = 0;
        if (o.json) check(c, mrg_parts_export_json(c, p, (uint32_t)k, &b, &nb), "mrg_parts_export_json");
        else check(c, mrg_parts_export(c, p, (uint32_t)k, &b, &nb), "mrg_parts_export");
        snprintf(name, sizeof name, "mr-%d-%d", r.cmap, k);
        write_file_atomic(name, b, nb);
        mrg_free(b);
    }
    mrg_parts_free(p);
}

// false: an input is missing (a duplicate of this task finished and removed
// them): the task is abandoned, nothing is written
bool do_reduce(mrg_ctx* c, const App& app, const WorkerOpts& o, const ReplyHdr& r) {
    mrg_parts* acc = nullptr;
    char name[64];
    for (int i = 0; i < r.nmap; i++) {  // worker.go:102-122
        snprintf(name, sizeof name, "mr-%d-%d", i, r.creduce);
        std::vector<uint8_t> b;
        // every map task writes all nReduce files (do_map), so in the reduce
        // phase a missing one was removed by an accepted duplicate of this task
        // (the reference skips it, worker.go:105-108, and writes a short mr-out)
        if (!read_file_try(name, &b)) {
            if (acc) mrg_parts_free(acc);
            return false;
        }
        mrg_parts* q = nullptr;
        if (o.json) check(c, mrg_parts_import_json(c, app.id, (uint32_t)r.nreduce, b.data(), b.size(), &q), "import_json");
        else check(c, mrg_parts_import(c, b.data(), b.size(), &q), "mrg_parts_import");
        if (!acc) acc = q;
        else {
            check(c, mrg_parts_merge(c, acc, q), "mrg_parts_merge");
            mrg_parts_free(q);
        }
    }
    void* out = nullptr;
    size_t n = 0;
    if (acc) {
        check(c, mrg_reduce(c, acc, (uint32_t)r.creduce, &out, &n), "mrg_reduce");  // worker.go:124-146
        mrg_parts_free(acc);
    }
    snprintf(name, sizeof name, "mr-out-%d", r.creduce);
    write_file_atomic(name, out, n);  // an empty partition still gets its file (worker.go:126-148)
    mrg_free(out);
    return true;
}

// worker.go:150-154, once the coordinator accepted this task's completion
void remove_reduce_inputs(int nmap, int part) {
    char name[64];
    for (int i = 0; i < nmap; i++) {
        snprintf(name, sizeof name, "mr-%d-%d", i, part);
        remove(name);
    }
}

int worker_main(const App& app, WorkerOpts o) {
    int ndev = 0;
    mrg_device_count(&ndev);
    if (ndev <= 0) fatalf("%s: no GPU visible", "mrworker_gpu");
    const int dev = o.device >= 0 ? o.device : o.index % ndev;
    mrg_ctx* c = nullptr;
    if (mrg_open(dev, &c) != MRG_OK) fatalf("%s: cannot open a GPU context", "mrworker_gpu");
    // test hook: die (no completion RPC) after receiving this many tasks, so the
    // coordinator's re-issue path runs (coordinator.go:70-77)
    // (MRG_WORKER_CRASH_INDEX: only the forked worker with that index, -w mode)
    const char* crash = getenv("MRG_WORKER_CRASH_AFTER");
    const char* crash_idx = getenv("MRG_WORKER_CRASH_INDEX");
    long crash_after = crash && (!crash_idx || atoi(crash_idx) == o.index) ? atol(crash) : -1;
    long tasks = 0;
    for (;;) {  // worker.go:46-54
        ReplyHdr r{};
        std::string fname;
        if (!call(o.sock, kRequestTask, 0, &r, &fname) || r.status == kDone) break;
        if (r.status == kWait) {
            std::this_thread::sleep_for(std::chrono::milliseconds(20));
            continue;
        }
        if (crash_after >= 0 && tasks++ >= crash_after) _exit(3);
        if (r.status == kMap) {
            do_map(c, app, o, r, fname);
            call(o.sock, kMapComplete, r.cmap, &r, &fname);  // worker.go:93-97
        } else if (r.status == kReduce) {
            const int x = r.creduce, nmap = r.nmap;
            if (!do_reduce(c, app, o, r)) continue;  // abandoned (a duplicate already finished it)
            ReplyHdr a{};
            if (call(o.sock, kReduceComplete, x, &a, &fname) && a.creduce == 1)  // worker.go:157-161
                remove_reduce_inputs(nmap, x);
        }
    }
    mrg_close(c);
    return 0;
}

int main_coord(int argc, char** argv) {
    Coordinator co;
    int nworkers = 0;
    WorkerOpts wo;
    wo.sock = default_sock();
    int i = 1;
    for (; i < argc; i++) {
        if (!strcmp(argv[i], "-n") && i + 1 < argc) co.nreduce = atoi(argv[++i]);
        else if (!strcmp(argv[i], "-w") && i + 1 < argc) nworkers = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--json")) wo.json = true;
        else if (!strcmp(argv[i], "--sock") && i + 1 < argc) wo.sock = argv[++i];
        else if (!strcmp(argv[i], "--task-timeout") && i + 1 < argc) co.timeout = atof(argv[++i]);
        else break;
    }
    if (argc - i < 2 || co.nreduce <= 0) {
        fprintf(stderr, "Usage: mrcoord_gpu [-n nreduce] [-w workers] [--json] [--sock path] [--task-timeout s] "
                        "wc|grep:<literal> inputfiles...\n");
        return 1;
    }
    const App app = parse_app(argv[i++]);
    for (; i < argc; i++) co.files.push_back(argv[i]);
    co.nmap = (int)co.files.size();  // MakeCoordinator (coordinator.go:149-160)
    co.map_log.assign(co.nmap, 0);
    co.map_since.assign(co.nmap, 0.0);
    co.reduce_log.assign(co.nreduce, 0);
    co.reduce_since.assign(co.nreduce, 0.0);
    const int lfd = listen_sock(wo.sock);
    std::vector<pid_t> kids;
    for (int k = 0; k < nworkers; k++) {  // no HIP call has happened in this process: forking is safe
        pid_t p = fork();
        if (p == 0) {
            close(lfd);
            WorkerOpts w = wo;
            w.index = k;
            _exit(worker_main(app, w));
        }
        kids.push_back(p);
    }
    std::vector<int> kid_status(kids.size(), -1);  // -1: not reaped yet
    double done_at = -1;
    for (;;) {  // main/mrcoordinator.go:24-28: until Done(), then a grace period
        co.expire();
        pollfd pf{lfd, POLLIN, 0};
        if (poll(&pf, 1, 50) > 0) serve_one(co, lfd);
        if (co.done() && done_at < 0) done_at = now_s();
        if (done_at >= 0 && now_s() - done_at > 1.0) break;  // workers have seen status 3 (or will fail to dial)
        if (nworkers > 0) {  // every forked worker gone before Done(): nothing can finish the job
            bool alive = false;
            for (size_t k = 0; k < kids.size(); k++) {
                if (kid_status[k] == -1 && waitpid(kids[k], &kid_status[k], WNOHANG) != kids[k]) kid_status[k] = -1;
                alive |= kid_status[k] == -1;
            }
            if (!alive && !co.done()) {
                fprintf(stderr, "mrcoord_gpu: all workers exited before the job finished\n");
                close(lfd);
                unlink(wo.sock.c_str());
                return 1;
            }
        }
    }
    close(lfd);
    unlink(wo.sock.c_str());
    // the job's status is Done() (every reduce task completed); a worker that
    // crashed and whose tasks were re-issued and finished by others is the
    // fault tolerance working, reported but not a failure
    int bad = 0;
    for (size_t k = 0; k < kids.size(); k++) {
        int st = kid_status[k];
        if (st == -1 && waitpid(kids[k], &st, 0) != kids[k]) st = 1 << 8;
        if (!(WIFEXITED(st) && WEXITSTATUS(st) == 0)) bad++;
    }
    printf("{\"nmap\": %d, \"nreduce\": %d, \"workers\": %d, \"reissued\": %llu, \"workers_failed\": %d, "
           "\"done\": %s}\n", co.nmap, co.nreduce, nworkers, (unsigned long long)co.reissued, bad,
           co.done() ? "true" : "false");
    return co.done() ? 0 : 1;
}

int main_worker(int argc, char** argv) {
    WorkerOpts wo;
    wo.sock = default_sock();
    int i = 1;
    for (; i < argc; i++) {
        if (!strcmp(argv[i], "--json")) wo.json = true;
        else if (!strcmp(argv[i], "--sock") && i + 1 < argc) wo.sock = argv[++i];
        else if (!strcmp(argv[i], "--device") && i + 1 < argc) wo.device = atoi(argv[++i]);
        else break;
    }
    if (argc - i != 1) {
        fprintf(stderr, "Usage: mrworker_gpu [--json] [--sock path] [--device d] wc|grep:<literal>\n");
        return 1;
    }
    return worker_main(parse_app(argv[i]), wo);
}

}  // namespace

int main(int argc, char** argv) {
    signal(SIGPIPE, SIG_IGN);
#if defined(MRCOORD_MAIN_WORKER)
    return main_worker(argc, argv);
#else
    return main_coord(argc, argv);
#endif
}
