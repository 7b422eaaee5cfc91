/* A plain-C caller of libjh.so: what a JNA/JNI/cgo binding does, without
 * Python or torch in the process. Built and driven by
 * tests/test_c_harness.py.
 *
 *   jh_harness version
 *   jh_harness open                          -> prints jh_open(0)'s return code
 *   jh_harness costs <hist.bin> <out.bin>    -> jh_key_costs (host only)
 *   jh_harness check <hist.bin> <out.bin> [dev,dev,...]
 *        jh_check_cas_independent on jh_open(0), or on jh_open_devices(list);
 *        writes n_keys jh_key_verdict records, prints the summary
 *
 * hist.bin: int64 n, int64 n_keys, then the columns process, type, f, key,
 * value, value2 (n int64 each), as include/jh.h lays them out.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "jh.h"

typedef struct { int64_t n, n_keys; int64_t *col[6]; } hist_t;

static int load(const char *path, hist_t *h) {
    FILE *fp = fopen(path, "rb");
    if (!fp) return -1;
    if (fread(&h->n, 8, 1, fp) != 1 || fread(&h->n_keys, 8, 1, fp) != 1) { fclose(fp); return -1; }
    for (int c = 0; c < 6; ++c) {
        h->col[c] = (int64_t *)malloc(sizeof(int64_t) * (size_t)(h->n > 0 ? h->n : 1));
        if ((int64_t)fread(h->col[c], 8, (size_t)h->n, fp) != h->n) { fclose(fp); return -1; }
    }
    fclose(fp);
    return 0;
}

static jh_history view(const hist_t *h) {
    jh_history v;
    memset(&v, 0, sizeof v);
    v.n = h->n;
    v.process = h->col[0]; v.type = h->col[1]; v.f = h->col[2];
    v.key = h->col[3]; v.value = h->col[4]; v.value2 = h->col[5];
    v.n_keys = h->n_keys;
    return v;
}

int main(int argc, char **argv) {
    char err[512] = "";
    if (argc < 2) return 64;
    if (!strcmp(argv[1], "version")) { printf("%d\n", jh_version()); return 0; }
    if (!strcmp(argv[1], "open")) {
        jh_ctx *ctx = NULL;
        int rc = jh_open(0, &ctx);
        printf("%d\n", rc);
        if (ctx) jh_close(ctx);
        return 0;
    }
    if (argc < 4) return 64;
    hist_t h;
    if (load(argv[2], &h)) { fprintf(stderr, "cannot read %s\n", argv[2]); return 65; }
    jh_history v = view(&h);
    FILE *out = fopen(argv[3], "wb");
    if (!out) return 66;
    if (!strcmp(argv[1], "costs")) {
        int64_t *cost = (int64_t *)malloc(sizeof(int64_t) * (size_t)(h.n_keys > 0 ? h.n_keys : 1));
        int rc = jh_key_costs(&v, cost, err, sizeof err);
        if (rc) { fprintf(stderr, "jh_key_costs: %d %s\n", rc, err); return rc; }
        fwrite(cost, 8, (size_t)h.n_keys, out);
        fclose(out);
        return 0;
    }
    if (!strcmp(argv[1], "check")) {
        jh_ctx *ctx = NULL;
        int rc;
        if (argc > 4) {
            int32_t devs[64];
            int n = 0;
            for (char *s = strtok(argv[4], ","); s && n < 64; s = strtok(NULL, ",")) devs[n++] = atoi(s);
            rc = jh_open_devices(devs, n, &ctx);
        } else {
            rc = jh_open(0, &ctx);
        }
        if (rc) { fprintf(stderr, "open: %d\n", rc); return rc; }
        printf("devices=%d\n", jh_n_devices(ctx));
        jh_key_verdict *vd = (jh_key_verdict *)calloc((size_t)(h.n_keys > 0 ? h.n_keys : 1), sizeof *vd);
        jh_summary s;
        jh_lin_opts o = {JH_NIL, 0, 0};
        o.flags = JH_LIN_EXACT_COUNT;                       /* every field is compared with the oracle */
        if (argc > 5) o.quick_budget = atoll(argv[5]);       /* a small one: many keys reach stage 2 */
        rc = jh_check_cas_independent(ctx, &v, &o, vd, &s, err, sizeof err);
        if (rc) { fprintf(stderr, "check: %d %s\n", rc, err); jh_close(ctx); return rc; }
        fwrite(vd, sizeof *vd, (size_t)h.n_keys, out);
        fclose(out);
        printf("valid=%lld n_invalid=%lld n_unknown=%lld first_fail_entry=%lld n_keys=%lld explored=%lld n_deferred=%lld\n",
               (long long)s.valid, (long long)s.n_invalid, (long long)s.n_unknown,
               (long long)s.first_fail_entry, (long long)s.n_keys, (long long)s.explored,
               (long long)s.n_deferred);
        jh_close(ctx);
        return 0;
    }
    return 64;
}
