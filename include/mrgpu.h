/*
 * mrgpu.h — C ABI of the MI355X-native MapReduce hot path (wc / grep).
 *
 * This is the drop-in boundary of BASELINE.json's north_star: mr/worker.go hands
 * whole input splits to these entry points (through cgo)
 * instead of running the plugin's Map + ihash partition loop and the
 * sort/group/Reduce loop on the CPU.  Plain C types only; no torch types.
 *
 * Reference interfaces replaced (paths under MapReduce/ of the reference):
 *   mrg_map            mrapps/wc.go:21-34 (Map) or mrapps/dgrep.go:18-36 (grepMap)
 *                      + mr/worker.go:69-78 (mapf call, ihash(key) % NReduce bucketing)
 *   mrg_parts_export   mr/worker.go:80-92  (write bucket r of map task X -> intermediate mr-X-r)
 *   mrg_parts_import   mr/worker.go:100-122 (read mr-i-Y back for reduce task Y)
 *   mrg_parts_merge    mr/worker.go:120 / mrsequential.go:50 (append intermediate KVs)
 *   mrg_reduce         mr/worker.go:123-146 (sort.Sort(ByKey), group, reducef, Fprintf "%v %v\n")
 *                      + mrapps/wc.go:41-44 (Reduce) or mrapps/dgrep.go:44-46 (grepReduce)
 *   mrg_reduce_all     every partition at once; with nreduce = 1 it is
 *                      main/mrsequential.go:59-84 (single mr-out-0)
 *   mrg_exchange       the M x R intermediate-file shuffle (mr/worker.go:80-122) across GPUs,
 *                      as an RCCL all-to-all over xGMI keyed by ihash(key) % nReduce
 *   mrg_ihash          mr/worker.go:33-37 (host helper, same FNV-1a-32 & 0x7fffffff)
 *
 * Semantics are bit-exact with the reference: words are maximal runs of runes
 * with unicode.IsLetter (Unicode 13.0.0), invalid UTF-8 bytes decode to U+FFFD
 * (a separator); partition = (fnv1a32(key) & 0x7fffffff) % nreduce; output lines
 * are sorted by unsigned bytewise key order; wc prints the decimal count, grep
 * prints the line twice ("L L\n").  Every partition yields its (possibly empty)
 * output, as worker.go:126-148 always writes mr-out-r.
 *
 * Errors: every int-returning call returns MRG_OK (0) or a negative MRG_E* code
 * and leaves a message in mrg_last_error(ctx) (the Go shim maps a nonzero code to
 * log.Fatalf as worker.go:60-64 does).  The library never aborts the process, with
 * ONE exception: a collective phase of mrg_comm_init / mrg_exchange that does not
 * finish within the option exchange_timeout_ms (default 120 s; 4x for
 * mrg_comm_init) — a peer rank died or hangs — makes the context's watchdog thread
 * print the stuck phase and end the process with _exit(124), because a rank
 * blocked inside RCCL cannot return an error code; a launcher then sees a failed
 * rank instead of a hang.
 *
 * Threading: a context is bound to one device and is not re-entrant; every entry
 * point re-binds its device (cgo calls may migrate OS threads).  Several contexts
 * per process are allowed (one per GPU thread).
 *
 * Ownership: input buffers are borrowed for the duration of the call only (cgo
 * pointer rules); outputs are library-owned and released with mrg_free /
 * mrg_parts_free.
 */
#ifndef MRGPU_H
#define MRGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MRG_OK 0
#define MRG_EINVAL (-1)   /* bad argument */
#define MRG_EDEVICE (-2)  /* HIP runtime / kernel error */
#define MRG_ENOMEM (-3)   /* device or host allocation failed */
#define MRG_ECOMM (-4)    /* RCCL error */
#define MRG_EFORMAT (-5)  /* malformed intermediate bytes */

#define MRG_APP_WC 1      /* mrapps/wc.go */
#define MRG_APP_GREP 2    /* mrapps/dgrep.go, fixed literal pattern */

#define MRG_INPUT_HOST 0  /* buf is a host pointer (copied to HBM by the call) */
#define MRG_INPUT_DEVICE 1/* buf is a device pointer already resident in HBM */

typedef struct mrg_ctx mrg_ctx;
typedef struct mrg_parts mrg_parts;

/* Per-call timing of the last mrg_map / mrg_reduce_all / mrg_run_job, from HIP
 * events on the context's stream (milliseconds). */
typedef struct {
    double map_kernel_ms;     /* the tokenizer/aggregation kernel alone (dominant kernel) */
    double map_total_ms;      /* map: every kernel from first launch to last */
    double exchange_ms;       /* the whole shuffle: count + payload all-to-alls (exchange_a2a_ms) and the
                                 owner's unpack + exact re-aggregation (exchange_unpack_ms); 0 when single-GPU */
    double reduce_ms;         /* collect + sort + format */
    double d2h_ms;            /* output bytes to host */
    uint64_t input_bytes;     /* bytes mapped */
    uint64_t distinct_keys;   /* distinct keys after aggregation */
    uint64_t output_bytes;    /* total mr-out bytes */
    uint64_t long_keys;       /* keys > 16 bytes (slow path) */
    uint64_t lds_overflow;    /* occurrences that missed the map-side LDS combiner (spilled) */
    uint64_t spill_ovf;       /* spilled occurrences that found their bucket region full */
    uint64_t agg_miss;        /* spilled occurrences that missed the bucket aggregator's LDS table */
    double agg_ms;            /* wc: per-bucket aggregation kernel */
    double long_ms;           /* long-word / grep-line resolution, incl. its host round trip */
    double collect_ms;        /* distinct keys -> records (partition = ihash % nReduce) */
    double dict_ms;           /* wc: sample + hot-key dictionary build */
    uint64_t dict_keys;       /* wc: sample keys offered to the dictionary */
    uint64_t dict_hits;       /* wc: occurrences counted by the dictionary in LDS */
    uint64_t agg_rounds;      /* wc: bucket aggregation rounds run (high-cardinality splits need > 1) */
    uint64_t shuffle_send_bytes; /* exchange: wire bytes this rank sent to OTHER ranks (records + arena) */
    uint64_t shuffle_recv_bytes; /* exchange: wire bytes this rank received from other ranks */
    uint64_t staged_bytes;    /* map: bytes copied into the context's staging buffer first (host input,
                                 or a device pointer not 16-byte aligned) */
    uint64_t spill_buckets;   /* wc: hash buckets of the map's spill (256 by default; 2048 for high-cardinality splits; 512 by option) */
    double exchange_a2a_ms;   /* exchange: the count and payload all-to-alls alone (exchange_ms also holds the
                                 owner's unpack + exact re-aggregation) */
    double exchange_unpack_ms;/* exchange: unpack of the received records + re-aggregation on the owner, from
                                 the owner's own unpack start (mrg_exchange_group: its finish step alone) */
    int64_t rccl_nranks;      /* exchange: ranks of the communicator as RCCL reports them (ncclCommCount);
                                 0 for mrg_exchange_group (peer copies) or no exchange */
    int64_t rccl_rank;        /* exchange: this context's rank per ncclCommUserRank (-1: none) */
    int64_t device;           /* the HIP device this context drives (ncclCommCuDevice when attached) */
    uint64_t spill_record_bytes; /* wc map: bytes of spill records written (8 per short key, 16 per 9-16-byte key) */
    uint64_t shuffle_recv_records; /* exchange: wire records this rank received as owner, from every rank
                                      (its own segment included), before re-aggregation */
} mrg_stats;

int mrg_open(int device, mrg_ctx** out);
void mrg_close(mrg_ctx* ctx);
const char* mrg_last_error(const mrg_ctx* ctx);
int mrg_device_count(int* n);

/* Map one input split (one file = one map task).  app = MRG_APP_WC or MRG_APP_GREP
 * (pat/plen = the literal; ignored for wc).  Output: device-resident partial
 * aggregates (distinct key, count, partition) for all nreduce partitions.
 * grep: the pattern is matched as a literal.  dgrep.go:20 compiles it as a regexp,
 * so a valid-UTF-8 pattern holding any of the metacharacters \ . + * ? ( ) | [ ] { } ^ $
 * is refused with MRG_EINVAL unless option grep_literal = 1 asks for
 * regexp.QuoteMeta semantics (the caller quoted it).  dgrep.go:20-23 returns no
 * lines when regexp.Compile fails, which for a literal happens exactly when it
 * is not valid UTF-8: such a pattern maps to no lines, as does one holding '\n'
 * (no line of strings.Split(contents, "\n") contains it). */
int mrg_map(mrg_ctx* ctx, int app, const void* buf, size_t len, int input_kind, const uint8_t* pat,
            size_t plen, uint32_t nreduce, mrg_parts** out);
/* Combine `from` into `into` (both on ctx's device, same app and nreduce). */
int mrg_parts_merge(mrg_ctx* ctx, mrg_parts* into, const mrg_parts* from);
/* Number of distinct keys held. */
int mrg_parts_info(const mrg_parts* p, uint64_t* nkeys, uint32_t* nreduce, int* app);
/* Serialize partition r (r = UINT32_MAX: all) to library-owned host bytes. */
int mrg_parts_export(mrg_ctx* ctx, const mrg_parts* p, uint32_t r, void** bytes, size_t* n);
/* Deserialize an mrg_parts_export buffer.  Every record is checked on the host
 * before it reaches the device (partition < nreduce and = ihash(key) % nreduce,
 * inline keys <= 16 bytes, arena keys inside the arena, prefix words equal to
 * the key's first bytes, counts >= 1): anything else is MRG_EFORMAT. */
int mrg_parts_import(mrg_ctx* ctx, const void* bytes, size_t n, mrg_parts** out);
void mrg_parts_free(mrg_parts* p);
/* The reference's own intermediate format, for mixed clusters of GPU and
 * reference workers.  export_json: partition r (UINT32_MAX: all) as the exact
 * bytes mr/worker.go:80-92 writes to mr-X-r — one json.Encoder line
 * {"Key":k,"Value":"1"} (wc) / {"Key":k,"Value":""} (grep) per occurrence, so a
 * record of count c is c lines (Go 1.16-1.21 escaping); library-owned host bytes.
 * import_json: mr-X-Y bytes written by reference workers (worker.go:100-122
 * reads them) -> parts with equal keys counted (one value per line). */
int mrg_parts_export_json(mrg_ctx* ctx, const mrg_parts* p, uint32_t r, void** bytes, size_t* n);
int mrg_parts_import_json(mrg_ctx* ctx, int app, uint32_t nreduce, const void* bytes, size_t n, mrg_parts** out);

/* Reduce partition r: exact mr-out-r bytes (library-owned host buffer). */
int mrg_reduce(mrg_ctx* ctx, const mrg_parts* p, uint32_t r, void** bytes, size_t* n);
/* Reduce every partition: bytes of mr-out-0..R-1 back to back; offsets[R+1]. */
int mrg_reduce_all(mrg_ctx* ctx, const mrg_parts* p, void** bytes, size_t* n, uint64_t* offsets);

/* Whole job on one device: map + (exchange) + reduce_all.  With a communicator
 * attached (mrg_comm_init), every rank maps its own split and receives the
 * partitions it owns (r % nranks == rank); offsets[] then index all R partitions
 * and non-owned ones are empty. */
int mrg_run_job(mrg_ctx* ctx, int app, const void* buf, size_t len, int input_kind, const uint8_t* pat,
                size_t plen, uint32_t nreduce, void** bytes, size_t* n, uint64_t* offsets);

/* Pipelined jobs (a worker's stream of map tasks, mr/worker.go:46-161): as
 * mrg_run_job, but returns once the job's output transfer is queued; its bytes
 * cross PCIe on a second stream into a context-owned pinned buffer while the
 * caller queues the next job, whose map overlaps that transfer.  At most two
 * jobs are queued (a third call returns MRG_EINVAL); mrg_job_wait returns the
 * oldest queued job's output (bytes valid until the next mrg_run_job_async or
 * mrg_job_wait on this context; offsets[nreduce + 1] as mrg_run_job) and its
 * stats (d2h_ms = its transfer; wc jobs write their lines straight into the
 * pinned buffer, as mrg_run_job does, and have none).  Any other reduce on the
 * context first waits for queued transfers. */
int mrg_run_job_async(mrg_ctx* ctx, int app, const void* buf, size_t len, int input_kind, const uint8_t* pat,
                      size_t plen, uint32_t nreduce);
int mrg_job_wait(mrg_ctx* ctx, void** bytes, size_t* n, uint64_t* offsets);

/* Multi-GPU (one process or thread per GPU).  The 128-byte unique id is made by
 * one rank and shared out of band (the coordinator RPC stays unchanged). */
int mrg_comm_unique_id(uint8_t id[128]);
int mrg_comm_init(mrg_ctx* ctx, const uint8_t id[128], int nranks, int rank);
/* Send every key to the owner of its partition; returns the owned partials. */
int mrg_exchange(mrg_ctx* ctx, const mrg_parts* local, mrg_parts** owned);
/* The same shuffle for P contexts driven by one host thread (one context per
 * GPU of a single-process driver, or several on one device): owned[i] receives
 * the partitions r with r % P == i from every local[j].  The all-to-all is peer
 * copies instead of RCCL; packing, ownership and re-aggregation are shared with
 * mrg_exchange.  Replaces the same mr/worker.go:80-122 file shuffle. */
int mrg_exchange_group(mrg_ctx* const* ctxs, int nctx, const mrg_parts* const* local, mrg_parts** owned);

/* Device memory helpers so callers can keep inputs resident in HBM. */
int mrg_device_alloc(mrg_ctx* ctx, size_t n, void** dptr);
int mrg_device_free(mrg_ctx* ctx, void* dptr);
int mrg_memcpy_h2d(mrg_ctx* ctx, void* dst, const void* src, size_t n);
int mrg_memcpy_d2h(mrg_ctx* ctx, void* dst, const void* src, size_t n);
/* Test hook for the reduce's radix sort (no reference counterpart): stable
 * in-place sort of n device keys (key_bytes 4 or 8, by their low `bits` bits;
 * 0 = all) carrying u32 device values (NULL: 8-byte keys only), through the
 * same dispatch as the reduce (option own_sort).  Waits for completion. */
int mrg_sort_pairs(mrg_ctx* ctx, void* keys, void* vals, size_t n, int key_bytes, unsigned bits);
int mrg_sync(mrg_ctx* ctx);
int mrg_get_stats(const mrg_ctx* ctx, mrg_stats* out);

/* Tuning knobs (0 = default); for benchmarks and tests of the overflow paths.
 * Results never depend on them (every path is exact), except skip_exchange, which
 * changes what mrg_run_job computes (benchmark timing only); unknown names -> MRG_EINVAL.
 *   short_table_log2, long_table_log2, list_cap, rec_cap   HBM table / buffer sizes
 *   map_grid, map_mode                   map workgroups; ablation modes (benchmarks)
 *   spill_stream_keys                    force tiny spill streams (overflow tests)
 *   spill_buckets (0, 256, 512, 2048)    spill buckets; 0 = chosen per split from the
 *                                        previous split's aggregated keys (256 default,
 *                                        2048 high-cardinality; 512 the earlier default)
 *   spill_hi_keys                        aggregated keys above which 2048 are chosen
 *   hi_stage (-1: off)                   2048-bucket splits: a 1088-key mini dictionary and
 *                                        8-byte spill records write-combined in LDS (32-byte
 *                                        stores; default) instead of the full dictionary
 *   long_records (-1: off)               wc words of 17-32 bytes leave the map as 32-byte key
 *                                        records (default) instead of the start-offset list
 *   agg_rounds, agg_carry_min, agg_big0 (0: by layout, 1 big, -1 small tables),
 *                                        agg_big_later   bucket aggregation rounds
 *   dict (-1: off), dict_warm (-1: off), dict_keep (permille; -1: always rebuild),
 *                                        dict_min_bytes, dict_sample_bytes
 *   ingest_piece, ingest_min             host input streamed in pieces of this size
 *   skip_exchange                        CHANGES RESULTS: mrg_run_job with nranks > 1 skips
 *                                        the shuffle and reduces only this rank's own split
 *                                        (bench.py's same-process T(1); never for real jobs)
 *   exch_force_rccl (1: on)              mrg_exchange runs its RCCL collectives on a
 *                                        one-rank communicator too (tests: the collective
 *                                        calls on one GPU); same results
 *   exchange_timeout_ms                  deadline of a collective phase (mrg_exchange;
 *                                        mrg_comm_init gets 4x; default 120000): past it the
 *                                        process prints the phase and exits with status 124
 *   sort_digit_bits (10: 10-bit radix digits; default 8), sort_fold_part (-1: off),
 *                                        grep_sort_k1 (-1: 8-byte prefix passes only),
 *                                        sort_compact_ties (-1: off), sort_bins (1: sample
 *                                        sort), sort_prefix32 (0: the wc key pass over all
 *                                        60/64 bits instead of the top 32), own_sort (kept
 *                                        for compatibility: every value runs the hand-written
 *                                        LSD passes), tie_rank (0: grep's tied runs
 *                                        merge-sorted together instead of ranked per run),
 *                                        grep_bins (grep reduce: 1 = default, bins sorted in
 *                                        LDS and written out by the same workgroups when the
 *                                        lines go to pinned host memory, else the radix
 *                                        passes; 0 = radix passes + tie ranking + line
 *                                        writer always; 2 / 3 = bins for any output, sorted
 *                                        order then the line writer / fused; -1 = the
 *                                        default without reusing the previous reduce's
 *                                        splitters)
 *                                        reduce sort variants
 *   grep_literal (1: on)                 grep patterns with regexp metacharacters matched as
 *                                        literals (QuoteMeta) instead of refused with MRG_EINVAL
 *   async_direct_max (bytes; -1: none)   mrg_run_job_async: wc outputs up to this bound (default
 *                                        64 MB) are written straight into the pinned buffer,
 *                                        larger ones copied on the output stream
 *   map_lean (-1: off)                   wc: the all-ASCII map variant after an all-ASCII split
 *   out_direct (-1: off, 1: wc only)     mrg_run_job writes the output lines straight into its
 *                                        pinned host buffer (default: wc and grep) instead of
 *                                        a device buffer + copy
 *   grep_sort_hits (1: on)               grep: the hits sorted by position before the line
 *                                        resolution (default: the map kernel's order, counts
 *                                        read on the device, sizes speculated from the
 *                                        previous split and checked once after the insert;
 *                                        either way a line occurrence is resolved once, so a
 *                                        record's count = the line's occurrences)
 *   grep_emit (0: off)                   grep: each distinct line's record written by the
 *                                        LongTable insert that claims it (default) instead
 *                                        of a collect pass over the table */
int mrg_set_option(mrg_ctx* ctx, const char* name, int64_t value);

uint32_t mrg_ihash(const uint8_t* key, size_t n);
void mrg_free(void* p);

#ifdef __cplusplus
}
#endif
#endif /* MRGPU_H */
