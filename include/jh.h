/*
 * jh.h -- C ABI of libjh.so, the MI355X-native Jepsen history checker.
 *
 * This is the drop-in boundary for the verification phase of Jepsen
 * (reference: jepsen "0.1.14-SNAPSHOT", /root/reference/jepsen/project.clj:1).
 * Each entry point replaces one `jepsen.checker/Checker` reify on the JVM
 * side; a JNA shim encodes the history once into the
 * columnar layout below and calls:
 *
 *   jh_check_cas_independent  <- (independent/checker (checker/linearizable
 *                                   {:model (model/cas-register v0)}))
 *                                 jepsen/src/jepsen/independent.clj:247-298
 *                                 jepsen/src/jepsen/checker.clj:127-158
 *   jh_check_cas              <- (checker/linearizable {:model (model/cas-register)})
 *                                 jepsen/src/jepsen/checker.clj:127-158
 *   jh_check_counter          <- (checker/counter)  jepsen/src/jepsen/checker.clj:679-734
 *   jh_check_set              <- (checker/set)      jepsen/src/jepsen/checker.clj:182-233
 *   jh_check_set_full         <- (checker/set-full {:linearizable? b})
 *                                                   jepsen/src/jepsen/checker.clj:236-534
 *   jh_check_total_queue      <- (checker/total-queue) jepsen/src/jepsen/checker.clj:536-628
 *   jh_check_queue            <- (checker/queue (model/unordered-queue))
 *                                                   jepsen/src/jepsen/checker.clj:160-180
 *
 * Plain pointers and sizes only. The caller owns every buffer; the library
 * never retains a caller pointer after returning. All entry points are
 * reentrant: one jh_ctx serialises its device work with a mutex.
 *
 * History encoding (one row per history map, in history order; the row
 * number IS knossos' :index, jepsen/src/jepsen/core.clj:441):
 *   process  >= 0 for an integer client process; < 0 for anything else
 *            (:nemesis is -1, other non-integers are interned to -2, -3, ...)
 *   type     JH_TYPE_INVOKE / OK / FAIL / INFO
 *   f        JH_F_READ / WRITE / CAS / ADD, anything else interned >= 16
 *   key      (key v) when :value is an independent tuple (a MapEntry,
 *            jepsen/src/jepsen/independent.clj:21-29), interned to
 *            [0, n_keys); -1 when :value is not a tuple.  May be NULL (= all -1).
 *   value    scalar :value (after unwrapping a tuple); for :cas the `cur`
 *            element of [cur new]; JH_NIL for nil / absent :value.
 *            For a set :read, the offset of its elements in `aux`.
 *   value2   for :cas the `new` element; for a set :read the element count;
 *            JH_NIL otherwise.
 */
#ifndef JH_H
#define JH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JH_ABI_VERSION 7

/* Return codes. Anything non-zero also writes a NUL-terminated message into
 * the caller's err buffer; the JNA shim throws ex-info and check-safe turns
 * it into {:valid? :unknown :error ...} (jepsen/src/jepsen/checker.clj:77-88). */
#define JH_OK            0
#define JH_EINVAL        1   /* malformed arguments or history */
#define JH_EUNSUPPORTED  2   /* input the device path does not handle: shim falls back */
#define JH_EDEVICE       3   /* HIP error, or no device */
#define JH_ENOMEM        4   /* device allocation failed */

/* :type */
#define JH_TYPE_INVOKE 0
#define JH_TYPE_OK     1
#define JH_TYPE_FAIL   2
#define JH_TYPE_INFO   3

/* :f */
#define JH_F_READ  0
#define JH_F_WRITE 1
#define JH_F_CAS   2
#define JH_F_ADD   3
#define JH_F_ENQUEUE 4
#define JH_F_DEQUEUE 5
#define JH_F_DRAIN   6  /* an :ok :drain's :value collection is a CSR range in aux, like a set read */

#define JH_NIL INT64_MIN

/* Verdict codes, ordered like jepsen.checker/valid-priorities
 * (jepsen/src/jepsen/checker.clj:26-31): true 0 < :unknown 0.5 < false 1. */
#define JH_VALID    0
#define JH_UNKNOWN  1
#define JH_INVALID  2

/* Per-key causes. */
#define JH_CAUSE_NONE         0
#define JH_CAUSE_BUDGET       1  /* memo-insert budget exhausted -> :unknown */
#define JH_CAUSE_WINDOW       2  /* more than JH_MAX_WINDOW concurrent ops   */
#define JH_CAUSE_DOUBLE_INVOKE 3 /* knossos.history/complete would throw     */
#define JH_CAUSE_ORPHAN       4  /* :ok/:fail with no open invocation        */
#define JH_CAUSE_BAD_F        5  /* op :f the cas-register model does not know */
#define JH_CAUSE_NIL_VALUE    6  /* nil where the checker does arithmetic     */
#define JH_CAUSE_OVERFLOW     7  /* long overflow (Clojure + throws)          */
#define JH_CAUSE_STATES       8  /* more than 65532 distinct values in one key */
#define JH_CAUSE_DEFERRED     9  /* JH_LIN_PHASE1_ONLY: past the quick budget, not searched further;
                                    explored = the key's rank for the heavy-key pass, heaviest first:
                                    2^31 - 1 - its estimated inserts (the quick search's inserts over
                                    its progress, deepest layer / layers; round 5) */

#define JH_MAX_WINDOW 256

typedef struct jh_history {
    int64_t n;                 /* entries */
    const int64_t *process;
    const int64_t *type;
    const int64_t *f;
    const int64_t *key;        /* may be NULL */
    const int64_t *value;
    const int64_t *value2;
    int64_t n_keys;            /* keys are 0..n_keys-1 */
    const int64_t *aux;        /* set-read elements, CSR via value/value2; may be NULL */
    int64_t n_aux;
    int32_t on_device;         /* 1: every pointer above is a device (HBM) pointer */
    int32_t reserved;
} jh_history;

/* :algorithm of (checker/linearizable {:model m :algorithm a}), checker.clj:141-145.
 * Every algorithm decides the same :valid? (all are complete decision
 * procedures); the choice selects which analysis is reported (:analyzer) and,
 * for an invalid key, which search's frontier :configs come from. */
#define JH_ALGO_COMPETITION 0       /* knossos.competition (the default): :wgl and :linear race */
#define JH_ALGO_WGL         1       /* knossos.wgl */
#define JH_ALGO_LINEAR      2       /* knossos.linear (JIT-linearization configuration sets) */

/* jh_lin_opts.flags: test hooks, 0 in production */
#define JH_LIN_BFS_ONLY        1    /* heavy keys: the reachable-set BFS alone (no DFS race) */
#define JH_LIN_GEN_JUMP        2    /* start at the top of the memo generation range (wrap test) */
#define JH_LIN_INTERN_PER_KEY  4    /* intern values per key even when one global range fits */
#define JH_LIN_NO_HELPERS      8    /* no late helper workgroups in phase 2 */
#define JH_LIN_HELPERS_NOW    16    /* late helpers take a key at once (helper_late_us = 0) */
/* Two-stage checking for rebalancing heavy keys across devices (jh_multi,
 * jepsen_amd/shard.py): stage 1 settles every key it can under the quick
 * budget and returns the others as JH_UNKNOWN / JH_CAUSE_DEFERRED; stage 2
 * sends every key that needs a search straight to the heavy-key engines. */
#define JH_LIN_PHASE1_ONLY    32
#define JH_LIN_SKIP_PHASE1    64
/* Phase 1 keeps every key it started until the quick budget (no hand-over of
 * long searches to the heavy-key pass once its queue is empty). */
#define JH_LIN_NO_HANDOVER   128
/* The streaming heavy-key pass: its engines consume phase 1's deferrals as
 * they are made instead of starting after phase 1. Same verdicts; measured
 * slower on C3 (the heavy keys' searches share CUs with phase
 * 1 and start without helpers), so it is off by default. */
#define JH_LIN_STREAM        256
/* Round 5: phase 1 saves each deferred search (stack + memo) and the heavy-key
 * pass continues it; this flag restarts deferred keys from scratch instead
 * (round 4's behaviour; same verdicts and counts, for A/B and the tests). */
#define JH_LIN_NO_RESUME     512
/* Round 5: WGL's exact cache size for every key. Without it, a valid key the
 * reachable-set engine settles (a terminal configuration reachable and at
 * most `budget` configurations reachable: WGL's cache is a subset of them,
 * so WGL could not have run out) is emitted at once with explored =
 * JH_EXPLORED_UNCOUNTED instead of after the count pass -- the reference's
 * map has no :explored (doc/tutorial/04-checker.md:126-138); the parity
 * tests set this flag. */
#define JH_LIN_EXACT_COUNT  1024
#define JH_EXPLORED_UNCOUNTED (-3)
/* Round 6: late helpers with no key of their own enumerate dead-subtree
 * candidates posted by the helpers that run a key's exact search, which merge
 * the dead ones (same verdicts and counts); this flag turns that off (A/B and
 * the tests). */
#define JH_LIN_NO_SPEC      2048
/* Round 6: late helpers serve posted spec jobs before taking keys of their
 * own (scheduling only: same verdicts and counts). */
#define JH_LIN_SPEC_FIRST   4096
/* Round 6: late helpers pick the keys whose sequential search has gone
 * longest without reaching a deeper layer (stuck in a big dead subtree)
 * instead of the ones running longest (scheduling only). */
#define JH_LIN_HELP_STALL   8192
/* Round 6, the takeover (opt-in): a late helper that takes a key phase 2's
 * sequential search is running continues that search's saved state instead
 * of restarting it (JH_LIN_TAKEOVER); JH_LIN_NO_TAKEOVER forces it off. */
#define JH_LIN_NO_TAKEOVER  16384
#define JH_LIN_TAKEOVER     32768

typedef struct jh_lin_opts {
    int64_t init_value;        /* (model/cas-register init); JH_NIL = (cas-register) */
    int64_t budget;            /* max memo inserts per key before :unknown; <=0: default */
    int64_t stream;            /* hipStream_t to run on (0 = the ctx stream) */
    int32_t algorithm;         /* JH_ALGO_*; 0 = competition, the reference's default */
    int32_t flags;             /* JH_LIN_* test hooks */
    int64_t quick_budget;      /* phase-1 inserts before a key is deferred; <=0: 8192 */
    int64_t phase2_budget;     /* phase-2 inserts before a key restarts in phase 3; <=0: 65536 */
    /* scheduling of the heavy-key pass (every value decides the same verdicts;
     * the parity tests run the less common paths through these): */
    int32_t helpers;           /* phase-2 late helper workgroups; <=0: 64 (a quarter of the CUs), at most half the CUs (JH_LIN_NO_HELPERS: none) */
    int32_t helper_late_us;    /* run time before a helper takes a key; <=0: 250 (JH_LIN_HELPERS_NOW: 0) */
    int32_t xw_waves;          /* waves of the 65-256-member search; <=0: one per key, up to 4 per CU */
    int32_t p2_waves_per_cu;   /* 1: phase 2 at one wave per CU with the 128 KB LDS memo; else 4,
                                  or 3 with the 16 KB Bloom filter when LEAN keys run alone
                                  (round 5) */
    int32_t lean_waves;        /* at most this many phase-2 waves for LEAN keys; <=0: no cap */
    int32_t wide_waves;        /* at most this many waves for WIDE keys; <=0: no cap */
    int32_t handover_min;      /* phase 1: once its queue is empty, searches past this many
                                  inserts go to the heavy-key pass (checked every 1024
                                  inserts: 1024 hands over at 2047); 0: default (1024 when
                                  the deferred searches resume, round 5; else off), <0: never */
    int32_t p1_waves_per_cu;   /* phase-1 waves per CU (<= 26, the LDS limit); <=0: 26 */
    int32_t bfs_wgs;           /* ABI 7: phase-2 reachable-set BFS workgroups (one per CU); <=0: default */
    int32_t reserved2;
} jh_lin_opts;

#define JH_DEFAULT_BUDGET (1 << 20)

typedef struct jh_key_verdict {
    int32_t valid;             /* JH_VALID / JH_UNKNOWN / JH_INVALID */
    int32_t cause;             /* JH_CAUSE_* */
    int64_t fail_entry;        /* invalid: history row of the ok completion of the
                                  first op no linearization can get past; else -1 */
    int64_t explored;          /* memo inserts (WGL cache size) for this key, the same
                                  on every run; -1 for a key in no tuple */
    /* invalid keys, from the search frontier (knossos' :previous-ok / :last-op;
     * knossos is not vendored, so these definitions are this library's and
     * PARITY-UNPINNED against knossos: oracle and device agree with each other):
     * last_op     = history row of the :ok completion of the last op the
     *               furthest configuration got past (RET[tmax-1]), -1 if none;
     * previous_ok = history row of the last client :ok in the key's
     *               subhistory before fail_entry, -1 if none.
     * Both -1 for keys that are not invalid. */
    int64_t previous_ok;
    int64_t last_op;
    /* ABI 4: the analysis that decided the key (knossos' :analyzer):
     * JH_ANALYZER_WGL (explored = WGL's cache size) or JH_ANALYZER_LINEAR
     * (explored = configurations the JIT-linearization analysis visited) */
    int32_t analyzer;
    int32_t reserved;
} jh_key_verdict;

#define JH_ANALYZER_WGL    0
#define JH_ANALYZER_LINEAR 1

typedef struct jh_summary {
    int64_t valid;             /* merge-valid over keys (checker.clj:33-47) */
    int64_t n_invalid;         /* == (count :failures) (independent.clj:289-295) */
    int64_t n_unknown;
    int64_t first_fail_entry;  /* min fail_entry over invalid keys, or -1 */
    int64_t n_keys;            /* keys checked (keys present in the history) */
    int64_t explored;          /* sum of memo inserts */
    int64_t memo_probes;       /* memo slots read by the phase-1 search kernel k_lin_dfs (roofline bytes) */
    double  device_ms;         /* device time of the check (HIP events) */
    double  dfs_ms;            /* of which the phase-1 search kernel k_lin_dfs (all keys, quick budget) */
    /* phase 2 (keys over the quick budget), for the roofline of its kernels */
    double  seq_ms;            /* the sequential search of the deferred keys (k_lin_seq / k_lin_wg) */
    double  bfs_ms;            /* the reachable-set BFS racing it (k_lin_bfs; 0 if not run) */
    int64_t n_deferred;        /* keys the phase-1 search handed on */
    int64_t deferred_entries;  /* history entries of those keys */
    int64_t seq_probes;        /* HBM memo probes of the phase-2 sequential search (LEAN keys) */
    /* ABI 4: per-phase accounting. Each search kernel has its own probe counter
     * and its own HIP events (on the stream it runs on), so each phase's
     * roofline is (56 B x its keys' entries + 16 B x its probes) / its time. */
    double  p3_ms;             /* phase 3, LEAN keys (restarted past phase2_budget) */
    double  wide_ms;           /* WIDE keys (window 41-64 or >= 256 states), phases 2 + 3 */
    double  xw_ms;             /* windows of 65-256 members (k_lin_xw) */
    int64_t p3_probes;
    int64_t wide_probes;
    int64_t xw_probes;
    int64_t helper_probes;     /* phase-2 late helper workgroups */
    int64_t n_deferred_wide;   /* WIDE keys among n_deferred */
    int64_t n_phase3;          /* LEAN keys restarted in phase 3 */
    int64_t n_phase3_wide;     /* WIDE keys restarted in phase 3 */
    int64_t n_xw;              /* keys searched by k_lin_xw */
    int64_t lean_entries;      /* entries of the deferred LEAN keys */
    int64_t wide_entries;      /* entries of the deferred WIDE keys */
    int64_t xw_entries;        /* entries of the k_lin_xw keys */
    int64_t waves[4];          /* launched waves: phase-2 LEAN, WIDE, phase-3 LEAN, xw */
    /* ABI 5 (round 4): the streaming heavy-key pass (JH_LIN_STREAM turns it
     * on). When streamed, seq_ms / bfs_ms / xw_ms are the engines' own spans
     * (first key taken to last wave end), p3_ms runs from the end of phase 2. */
    int64_t streamed;          /* 1: heavy keys started while phase 1 still ran */
    int64_t p3_entries;        /* entries of the LEAN keys restarted in phase 3 */
    double  p2_start_ms;       /* heavy-key pass start (streamed: its first key taken), ms after phase 1 began (-1: none) */
    double  p1_span_ms;        /* phase 1's first wave to its last wave's end (streamed) */
    /* ABI 6 (round 5): deferred searches phase 1 saved and the heavy-key pass
     * continued (JH_LIN_NO_RESUME: 0), and the bytes of their records */
    int64_t resumed;
    int64_t resume_bytes;
    /* ABI 7 (round 6): speculative dead-subtree enumerations by idle late
     * helpers (JH_LIN_NO_SPEC: 0): jobs run, of which dead, dead results the
     * searches merged and the nodes those merges added to their counts */
    int64_t spec_jobs;
    int64_t spec_dead;
    int64_t spec_merges;
    int64_t spec_nodes;
    /* round 6: keys a late helper took over from the sequential search with
     * its saved state (the takeover; JH_LIN_NO_TAKEOVER: 0) */
    int64_t takeovers;
} jh_summary;

typedef struct jh_ctx jh_ctx;

int  jh_version(void);
/* Opens a context on HIP device `device`. */
int  jh_open(int device, jh_ctx **out);
/* Opens one context over devices 0..n_gpus-1 (n_gpus <= 0: every visible
 * device; SURVEY 8(b) "jh_open(n_gpus)"). jh_check_cas_independent on it
 * splits the keys over the devices by the jh_key_costs estimate (heaviest
 * first to the least-loaded device), checks every part concurrently, one host
 * thread per device, and merges the verdicts and the summary on the host:
 * same result as one device, bit for bit. The other checkers run on device 0.
 * Host columns only (on_device = 0). jh_close closes every device. */
int  jh_open_multi(int n_gpus, jh_ctx **out);
/* The same over an explicit device list; a device may appear more than once
 * (several contexts share it, each with its own streams and workspace). */
int  jh_open_devices(const int32_t *devices, int n, jh_ctx **out);
int  jh_n_devices(const jh_ctx *ctx);
void jh_close(jh_ctx *ctx);

/* Per-key search-cost estimate used to split keys between devices: the key's
 * entries plus its window sum (for every client op, the :ok returns inside its
 * window; a crashed op's window runs to the end). Host columns; no device. */
int  jh_key_costs(const jh_history *h, int64_t *cost /*[n_keys]*/, char *err, size_t errlen);

/* (independent/checker (checker/linearizable {:model (model/cas-register init)})).
 * out[k] receives the verdict of key k for k in [0, h->n_keys); keys that
 * occur in no tuple get valid = JH_VALID, explored = -1 (they have no
 * :results entry, independent.clj:222-232). */
int jh_check_cas_independent(jh_ctx *ctx, const jh_history *h,
                             const jh_lin_opts *opts,
                             jh_key_verdict *out, jh_summary *sum,
                             char *err, size_t errlen);

/* The per-key row index of an independent history, from the device's stable
 * key partition: rows[key_off[k] .. key_off[k+1]) are key k's rows in history
 * order, and rows[key_off[n_keys] .. n) the rows in no tuple (nemesis ops).
 * Key k's subhistory (independent.clj:234-245) is the merge of its rows with
 * the un-keyed rows, so the shim writes every key's history.edn
 * (independent.clj:277-284) in one O(N) pass. Only the key column is read.
 * key_off: n_keys+1 entries; rows: n entries (host buffers). */
int jh_key_index(jh_ctx *ctx, const jh_history *h, int64_t *key_off, int64_t *rows,
                 char *err, size_t errlen);

/* Round 6: the columns of a host history exactly as the device sees them
 * after staging (the packed host-buffer path for >= 2 M rows, plain copies
 * below): process, type, f, key, value, value2 -- n int64 each, in that
 * order, into out (6 * n; the key block is left as is without a key column).
 * Checks nothing: a maintainer's (and the tests') view of the staging. */
int jh_stage_history(jh_ctx *ctx, const jh_history *h, int64_t *out, char *err, size_t errlen);

/* knossos' :configs (checker.clj:146-158 passes the analysis through and
 * keeps (take 10 ...) of them), from the JIT-linearization analysis
 * (:algorithm :linear; doc/tutorial/04-checker.md:126-138 prints one).
 *  - An invalid key: its frontier -- the configurations of the last layer
 *    its search reaches, the ways of linearizing the ops before the failing
 *    :ok op from which that op cannot be.
 *  - A valid key (ABI 6): its final configurations -- the configurations the
 *    analysis holds after the key's last :ok completion: every way the
 *    crashed ops may stand once every :ok op is linearized (the register
 *    value, and which crashed ops were linearized).
 * For each requested key, up to per_key (<= 16) configurations in a
 * canonical order: register value (nil first, then ascending), then the
 * linearized members as a bit mask in call order (a JH_MAX_WINDOW-bit
 * number). n_out[i] = the count for keys[i], or -1 (no search was needed, a
 * window over JH_MAX_WINDOW members, more than budget configurations
 * reachable, or a valid key the reachable-set engine cannot hold: WGL
 * decides those, and a WGL analysis carries no configurations).
 * Windows up to 32 members with < 4096 states come from the reachable-set
 * engine, wider invalid ones (round 4) from the 65-256-member search's table.
 * out[i * per_key + j] describes configuration j of keys[i]; its rows are
 * rows_out[rows_off .. rows_off + n_linearized + n_pending): the invocation
 * rows of the linearized ops, then of the pending ones (knossos' :pending),
 * each in call order -- for a frontier the members of the window, for final
 * configurations the crashed ops (their :info completion or none) the search
 * keeps; rows_cap >= n_keys_q * per_key * JH_MAX_WINDOW. Round 6: the reads
 * the search drops (crashed reads, :ok reads of nil -- they constrain
 * nothing) are listed too: each configuration is the one knossos holds in
 * which such a read is linearized exactly when its own completion forces it,
 * so a read invoked before the configuration's point and not completed there
 * is pending (call order, at most JH_MAX_WINDOW rows in all). last_row (ABI 6)
 * is the configuration's :last-op as knossos' analysis prints it: the row of
 * the key's last client :ok completion before the configurations' point (the
 * failing op's completion for a frontier, the end of the history for final
 * configurations; a read of nil completing later than a final
 * configuration's own last op is its :last-op), -1 if there is none.
 * knossos is not vendored: this order,
 * the cut and the layer are this library's definitions (parity unpinned; the
 * oracle restates them). */
typedef struct jh_lin_config {
    int64_t key;
    int64_t model_value;       /* the register's value in this configuration (JH_NIL: nil) */
    int32_t n_linearized;
    int32_t n_pending;
    int64_t rows_off;
    int64_t last_row;          /* ABI 6: the :ok completion that is this configuration's :last-op, or -1 */
} jh_lin_config;

int jh_lin_configs(jh_ctx *ctx, const jh_history *h, const jh_lin_opts *opts,
                   const int64_t *keys, int64_t n_keys_q, int32_t per_key,
                   jh_lin_config *out, int32_t *n_out, int64_t *rows_out, int64_t rows_cap,
                   char *err, size_t errlen);

/* (checker/linearizable {:model (model/cas-register init)}) on a history
 * whose values are not tuples (key column ignored). */
int jh_check_cas(jh_ctx *ctx, const jh_history *h, const jh_lin_opts *opts,
                 jh_key_verdict *out, char *err, size_t errlen);

/* Device-resident variant for benchmarking and for callers that keep the
 * encoded history in HBM: h->on_device must be 1; out_dev is a device array
 * of n_keys verdicts; sum is host. Runs on opts->stream, synchronises it. */
int jh_check_cas_independent_device(jh_ctx *ctx, const jh_history *h,
                                    const jh_lin_opts *opts,
                                    jh_key_verdict *out_dev, jh_summary *sum,
                                    char *err, size_t errlen);

/* (checker/counter). reads_out receives 3*n_reads int64 [lower value upper]
 * triples in history order (the :reads vector); at most reads_cap triples
 * are written, *n_reads is always the full count. *valid is JH_VALID /
 * JH_INVALID / JH_UNKNOWN (cause in *cause). *first_err_entry = history row
 * of the :ok read behind (first errors), or -1. */
int jh_check_counter(jh_ctx *ctx, const jh_history *h,
                     int64_t *reads_out, int64_t reads_cap,
                     int64_t *n_reads, int64_t *n_errors,
                     int64_t *first_err_entry, int32_t *valid, int32_t *cause,
                     char *err, size_t errlen);

typedef struct jh_set_result {
    int32_t valid;             /* JH_VALID / JH_INVALID / JH_UNKNOWN ("Set was never read") */
    int32_t cause;
    int64_t attempt_count, acknowledged_count, ok_count,
            lost_count, recovered_count, unexpected_count;
    int64_t first_fail_entry;  /* min row of an :ok :add whose element is lost;
                                  else the final read's row if unexpected; else -1 */
    int64_t final_read_entry;
    /* Run-length form of the four result sets (util.clj:536-575): run r of
     * set s is [runs[s][2r], runs[s][2r+1]] inclusive. Sets: 0 ok, 1 lost,
     * 2 unexpected, 3 recovered. Caller provides runs_cap pairs per set. */
    int64_t n_runs[4];
} jh_set_result;

int jh_check_set(jh_ctx *ctx, const jh_history *h, jh_set_result *res,
                 int64_t *runs_ok, int64_t *runs_lost, int64_t *runs_unexpected,
                 int64_t *runs_recovered, int64_t runs_cap,
                 char *err, size_t errlen);

/* (checker/set) with the four result sets as bitmaps instead of runs: bit i
 * of word w of a set is element *base + 32 w + i, for w < *n_words (at most
 * words_cap words are written per set; *n_words is always the full count).
 * Same counts, first_fail_entry and n_runs as jh_check_set. The D2H is 4
 * bytes per 32 elements of span, whatever the run structure; the shim
 * formats integer-interval-set-str (util.clj:536-575) from the bits. */
int jh_check_set_bitmaps(jh_ctx *ctx, const jh_history *h, jh_set_result *res,
                         uint32_t *ok, uint32_t *lost, uint32_t *unexpected, uint32_t *recovered,
                         int64_t words_cap, int64_t *base, int64_t *n_words,
                         char *err, size_t errlen);

/* Page-locked host memory for result buffers a caller keeps across calls
 * (jh_check_counter's triples, jh_check_set_bitmaps' bitmaps): their D2H then
 * runs at PCIe speed instead of through the runtime's pageable staging
 * copies. Not in the reference's interface (a JVM has no such thing): the
 * JNA shim allocates one per checker instance and reuses it. */
int jh_host_alloc(size_t bytes, void **out, char *err, size_t errlen);
int jh_host_free(void *p);

/* (checker/set-full {:linearizable? linearizable}), checker.clj:236-534.
 * Elements are the :value of every :invoke :add by an integer process; a
 * set :read's :value is its CSR range in aux (value = offset, value2 =
 * count; a nil :value reads as the empty set). `time` is the :time column
 * (nanoseconds), indexed by row like the others (host or device pointer
 * following h->on_device). Per element (set-full-element-results,
 * checker.clj:289-345): known = the first :ok :add or :ok :read containing
 * it, last-present / last-absent = the read INVOCATION of greatest index
 * whose :ok read did / did not contain it; all counted from the element's
 * last :invoke :add on (a re-invoke resets its state, checker.clj:483-487).
 * The lost / never-read / stale element lists come back sorted, at most
 * list_cap each (the counts are always complete); worst_stale holds the
 * (take 8 (reverse (sort-by :stable-latency stale))) entries. */
#define JH_SF_QUANTILES 5          /* points [0 0.5 0.95 0.99 1], checker.clj:412 */
#define JH_SF_WORST 8

typedef struct jh_set_full_elem {
    int64_t element;
    int64_t stable_latency;        /* ms */
    int64_t known_entry;           /* row of the :known op */
    int64_t last_absent_entry;     /* row of the :last-absent read invocation, or -1 */
} jh_set_full_elem;

typedef struct jh_set_full_result {
    int32_t valid;                 /* JH_VALID / JH_INVALID / JH_UNKNOWN (no stable element) */
    int32_t cause;
    int64_t attempt_count, stable_count, lost_count, never_read_count, stale_count;
    int32_t has_stable_latencies, has_lost_latencies;
    int64_t stable_latencies[JH_SF_QUANTILES];   /* ms at the points above */
    int64_t lost_latencies[JH_SF_QUANTILES];
    int64_t n_worst;
    jh_set_full_elem worst_stale[JH_SF_WORST];
    int64_t n_reads;               /* :ok :reads by integer processes */
    int64_t read_elements;         /* sum of their element counts (aux entries scanned) */
    double  device_ms;             /* device time of the check (HIP events) */
} jh_set_full_result;

int jh_check_set_full(jh_ctx *ctx, const jh_history *h, const int64_t *time,
                      int32_t linearizable, jh_set_full_result *res,
                      int64_t *lost, int64_t *never_read, int64_t *stale, int64_t list_cap,
                      char *err, size_t errlen);

/* jh_check_set_full with options (zero-initialise; the call above is this
 * with only `linearizable` set). */
typedef struct jh_set_full_opts {
    int32_t linearizable;      /* {:linearizable? true}: stale elements make the result invalid */
    int32_t pad;
    int64_t read_batch;        /* :ok reads per bitmap batch, 0 = automatic (<= 2 GiB of bitmap,
                                  <= 65535 reads); tests use 1 and 3 to cross batch edges */
    int64_t reserved[4];
} jh_set_full_opts;
int jh_check_set_full_opts(jh_ctx *ctx, const jh_history *h, const int64_t *time,
                           const jh_set_full_opts *opts, jh_set_full_result *res,
                           int64_t *lost, int64_t *never_read, int64_t *stale, int64_t list_cap,
                           char *err, size_t errlen);

/* Queues. Values are the :value of :enqueue / :dequeue ops and the elements
 * of :ok :drain ops (integers, or ids the shim interned; JH_NIL = nil).
 * Multisets come back as (value, multiplicity) int64 pairs sorted by value,
 * at most pairs_cap pairs per multiset (n_pairs is always complete). */
typedef struct jh_queue_result {
    int32_t valid;             /* JH_VALID / JH_INVALID */
    int32_t cause;
    int64_t attempt_count, acknowledged_count, ok_count, unexpected_count,
            duplicated_count, lost_count, recovered_count;
    int64_t n_pairs[4];        /* total-queue: lost, unexpected, duplicated, recovered;
                                  queue: [0] = the final queue */
    int64_t fail_entry;        /* queue: row of the first :ok :dequeue the model cannot
                                  supply ("can't dequeue v"), else -1 */
    int64_t fail_value;
    double  device_ms;
} jh_queue_result;

/* (checker/total-queue), checker.clj:570-628, after expand-queue-drain-ops
 * (:536-568; a crashed :drain is JH_EINVAL, as the reference throws). */
int jh_check_total_queue(jh_ctx *ctx, const jh_history *h, jh_queue_result *res,
                         int64_t *lost, int64_t *unexpected, int64_t *duplicated,
                         int64_t *recovered, int64_t pairs_cap, char *err, size_t errlen);

/* (checker/queue (model/unordered-queue)), checker.clj:160-180: the model
 * reduced over :invoke :enqueue and :ok :dequeue ops in history order.
 * final_queue receives the remaining multiset when valid. */
int jh_check_queue(jh_ctx *ctx, const jh_history *h, jh_queue_result *res,
                   int64_t *final_queue, int64_t pairs_cap, char *err, size_t errlen);

#ifdef __cplusplus
}
#endif
#endif /* JH_H */
