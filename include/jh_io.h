/*
 * jh_io.h -- history ingest of libjh.so: a stored Jepsen
 * history straight into the columnar layout of jh.h, in native code.
 *
 * The reference stores a run two ways and reads it back for re-analysis:
 *   history.edn    one prn-printed op map per line
 *                  (jepsen/src/jepsen/store.clj:346-357 write-history!,
 *                   jepsen/src/jepsen/util.clj:191-213 pwrite-history!)
 *   test.fressian  the whole test map, :history among its keys
 *                  (jepsen/src/jepsen/store.clj:359-366 write-fressian!,
 *                   :177-183 load, with the handlers of :28-123)
 * The JVM shim would otherwise walk a 10^8-op history op map by op map to
 * encode it; these entry points replace (store/load ...) + the shim's encode
 * loop when the checker is run on a stored test.
 *
 * Encoding: exactly jepsen_amd/history.py `encode` (which the tests hold it
 * to, column by column): client processes >= 0, :nemesis -1, other processes
 * -2, -3, ... by first appearance; :f read/write/cas/add/enqueue/dequeue/drain
 * to the JH_F_* codes, others interned from 16 by first appearance; with
 * `independent`, the :value [k v] of an integer process is a tuple (key
 * interned by first appearance, value v); :cas [cur new] to value/value2; a
 * collection :value of a :read / :drain to an aux CSR range (sets sorted);
 * integer values as themselves, unless some value is not an integer, in
 * which case every value is interned in first-appearance order (the value
 * table). Rows keep history order: the row number is knossos' :index.
 */
#ifndef JH_IO_H
#define JH_IO_H

#include <stddef.h>
#include <stdint.h>

#include "jh.h"

#ifdef __cplusplus
extern "C" {
#endif

#define JH_FMT_AUTO     0   /* fressian if the bytes do not start like EDN text */
#define JH_FMT_EDN      1
#define JH_FMT_FRESSIAN 2

#define JH_TBL_KEYS   0     /* key id -> the key (EDN text) */
#define JH_TBL_F      1     /* interned :f id - 16 -> the :f (EDN text) */
#define JH_TBL_VALUES 2     /* value id -> the value (EDN text), when values are interned */

typedef struct jh_ingest jh_ingest;

/* Options of the _opts entry points (zero-initialise; the plain entry points
 * below are these with only `threads` set). */
typedef struct jh_ingest_opts {
    int32_t threads;      /* EDN host threads, 0 = all cores */
    int32_t debug;        /* nonzero: per-chunk parse timings on stderr */
    int64_t min_chunk;    /* smallest EDN chunk in bytes, 0 = 1 MiB (tests split small texts) */
    int64_t reserved[4];
} jh_ingest_opts;

/* Parses a history file (EDN: `threads` host threads, 0 = all cores, split at
 * line starts and verified; fressian: one pass, its caches are sequential). */
int jh_ingest_file(const char *path, int format, int independent, int threads,
                   jh_ingest **out, char *err, size_t errlen);
/* The same over bytes in memory (not retained). */
int jh_ingest_buffer(const char *buf, size_t len, int format, int independent, int threads,
                     jh_ingest **out, char *err, size_t errlen);
int jh_ingest_file_opts(const char *path, int format, int independent, const jh_ingest_opts *opts,
                        jh_ingest **out, char *err, size_t errlen);
int jh_ingest_buffer_opts(const char *buf, size_t len, int format, int independent, const jh_ingest_opts *opts,
                          jh_ingest **out, char *err, size_t errlen);
/* Host columns owned by the handle (valid until jh_ingest_free), on_device 0. */
void jh_ingest_history(const jh_ingest *g, jh_history *h);
/* The :time column (JH_NIL where absent), for jh_check_set_full. */
const int64_t *jh_ingest_time(const jh_ingest *g);
/* 1 when every value was interned (some value is not an integer). */
int jh_ingest_values_interned(const jh_ingest *g);
int64_t jh_ingest_table_size(const jh_ingest *g, int table);
/* Entry i of a table as EDN text, NUL-terminated into buf (cap bytes);
 * returns the text's length (call again with a larger buf if >= cap), -1 if
 * i or table is out of range. */
int64_t jh_ingest_table_entry(const jh_ingest *g, int table, int64_t i, char *buf, size_t cap);
void jh_ingest_free(jh_ingest *g);

#ifdef __cplusplus
}
#endif
#endif /* JH_IO_H */
