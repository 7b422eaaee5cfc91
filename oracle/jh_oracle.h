/*
 * jh_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference verification path, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
 * The product (libjh.so) never links or calls anything here.
 *
 * Parity status: the linearizability algorithm lives in knossos 0.3.4
 * (jepsen/project.clj:13), which is NOT vendored in /root/reference and
 * cannot be fetched or run here (no JVM, no network). This restatement is
 * pinned by the reference's own known answers (tests/golden/, see
 * tests/test_oracle_golden.py): perf_test.clj:13-137 (valid cas history),
 * checker_test.clj:90-166 (six exact counter maps), independent_test.clj:78-97
 * (independent result shape), util_test.clj:14-31 (interval strings).
 * Invalid-history, :info-heavy and checker/set verdicts are cross-checked
 * between three independent CPU formulations (canonical WGL, knossos-style
 * linked-list WGL, brute-force linearization search) and are otherwise
 * "parity unpinned" against knossos itself.
 */
#ifndef JH_ORACLE_H
#define JH_ORACLE_H
#include <stdint.h>
#include <stddef.h>
#include "../include/jh.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One operation of a prepared (completed, filtered) cas-register key. */
typedef struct orc_op {
    int64_t call;      /* history row of the invocation */
    int64_t ret;       /* history row of the :ok completion; INT64_MAX if crashed */
    int32_t f;         /* JH_F_READ / WRITE / CAS */
    int32_t rr;        /* return rank among ok ops, -1 if crashed */
    int64_t v1, v2;    /* completed value(s) */
} orc_op;

typedef struct orc_key {
    int32_t status;    /* JH_CAUSE_NONE, or the cause that makes the key :unknown */
    int32_t n_ops;
    orc_op *ops;       /* in call order */
    int32_t n_ok;
    int32_t *ret_op;   /* ret_op[t] = op index of the t-th ok return */
    int32_t *w_off;    /* windows: W(t) = w_ops[w_off[t] .. w_off[t+1]) */
    int32_t *w_ops;
    int32_t max_window;
    int32_t *pred;     /* crashed-op symmetry (orc_reduce_crashed): the previous crashed op
                          of the same (f, value, value2) in call order, or -1 */
    int32_t n_noop;    /* round 6: the reads the search drops (crashed reads, :ok reads of
                          nil), kept for knossos' :pending (configs_one), in call order */
    int64_t *noop_call, *noop_ret;   /* invocation row; :ok completion row or INT64_MAX */
} orc_key;

/* Round 5: pending crashed ops of one (f, value, value2) class are
 * interchangeable -- both invoked, neither bounded by a return, the same
 * step -- so only the earliest-invoked unlinearized member of a class is a
 * candidate (a sound symmetry reduction: every configuration reachable
 * without it has an equivalent one, same register value and the same ops
 * still to linearize up to renaming, reachable with it). Changes explored
 * counts, never a verdict. Set by the caller (libjh.so's default). */
extern int orc_reduce_crashed;

/* Prepare key from the rows `sel[0..m)` (increasing history rows). */
int  orc_key_prepare(const jh_history *h, const int64_t *sel, int64_t m, orc_key *k);
void orc_key_free(orc_key *k);

/* Canonical-configuration WGL search (the semantics libjh.so implements). */
int  orc_wgl_canonical(const orc_key *k, int64_t init, int64_t budget,
                       int64_t *explored, int64_t *fail_entry);
/* knossos-style WGL: linked list of call/return entries, bitset of
 * linearized ops, cache of (bitset, state). Must agree with the canonical
 * search on verdict AND explored count. */
int  orc_wgl_list(const orc_key *k, int64_t init, int64_t budget,
                  int64_t *explored);
/* Brute-force linearization search, no memo, for tiny keys (<= 12 ops). */
int  orc_lin_bruteforce(const orc_key *k, int64_t init);

/* knossos.linear (JIT linearization) in canonical coordinates: the reachable
 * configuration set, layer by layer (jh_oracle.c). */
struct cvec;
/* history-wide: every interned state id < 4096 (set by the caller, as the
 * device computes it; the reachable-set engine packs states in 12 bits) */
extern int orc_linear_states_ok;

/* The frontier configurations of invalid keys (restates jh_lin_configs;
 * rows of configuration j of keys[q] at rows[(q * per_key + j) * 64 ...]). */
int orc_lin_configs(const jh_history *h, int64_t init, int64_t budget, const int64_t *keys, int64_t nq,
                    int32_t per_key, int32_t per_key_values, jh_lin_config *out, int32_t *n_out, int64_t *rows);

/* Whole-history linearizable check (non-independent). */
int  orc_check_cas(const jh_history *h, int64_t init, int64_t budget,
                   jh_key_verdict *out);
/* Independent checker. mode bit 0: the reference's O(K*N) per-key subhistory
 * scan (independent.clj:234-245), else one O(N) bucketed split; bit 1: the
 * knossos-style list WGL instead of the canonical one; bit 2: :algorithm
 * :linear (JIT linearization where it applies, see jh_oracle.c). */
int  orc_check_cas_independent(const jh_history *h, int64_t init, int64_t budget,
                               int mode, int threads, jh_key_verdict *out,
                               jh_summary *sum);
/* Same, restricted to keys [k0, k1) (for the bench's bounded CPU sample). */
int  orc_check_cas_independent_range(const jh_history *h, int64_t init,
                                     int64_t budget, int mode, int threads,
                                     int64_t k0, int64_t k1,
                                     jh_key_verdict *out);

int  orc_check_counter(const jh_history *h, int64_t *reads_out, int64_t reads_cap,
                       int64_t *n_reads, int64_t *n_errors, int64_t *first_err_entry,
                       int32_t *valid, int32_t *cause);

int  orc_check_set(const jh_history *h, jh_set_result *res,
                   int64_t *runs_ok, int64_t *runs_lost, int64_t *runs_unexpected,
                   int64_t *runs_recovered, int64_t runs_cap);

/* util/integer-interval-set-str over a sorted, de-duplicated array. */
int64_t orc_interval_str(const int64_t *sorted, int64_t n, char *buf, int64_t cap);
int orc_lin_selftest_key(const jh_history *h, int64_t init, int64_t budget, int64_t *res);

#ifdef __cplusplus
}
#endif
#endif
