/*
 * openssl_bench.c — host-core CPU baseline with OpenSSL libcrypto
 * ECDSA_do_verify (P-256, ecp_nistz256 assembly), one pthread per core over an
 * atomic index; keys and signatures pre-built outside the timed region.
 * Labelled "fallback: OpenSSL, not Go" (BASELINE.md 2): Go is absent on the box.
 * Usage: openssl_bench <tuples.bin> <nthreads> <min_seconds> [runs]
 * SURVEY.md 8(d)'s method: one untimed warm-up run, then `runs` (default 1) timed runs of at
 * least min_seconds each; verifies_per_s is the median run, runs_per_s every run.
 * Prints one JSON object: {"verifies_per_s":..., "threads":..., "n":..., "accepted":...}
 */
#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/ecdsa.h>
#include <openssl/obj_mac.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static EC_KEY** keys;
static ECDSA_SIG** sigs;
static unsigned char* recs;
static size_t n;
static atomic_size_t next_idx;
static atomic_size_t accepted;
static size_t total_target;

static atomic_int stop_flag;  /* timed runs: the workers stop at the deadline */

static void* worker(void* arg) {
    (void)arg;
    size_t acc = 0;
    for (;;) {
        if (atomic_load_explicit(&stop_flag, memory_order_relaxed)) break;
        size_t i = atomic_fetch_add(&next_idx, 1);
        if (i >= total_target) break;
        size_t j = i % n;
        if (keys[j] && ECDSA_do_verify(recs + 160 * j, 32, sigs[j], keys[j]) == 1) ++acc;
    }
    atomic_fetch_add(&accepted, acc);
    return NULL;
}

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 3;
    int nt = atoi(argv[2]);
    double min_s = atof(argv[3]);
    fseek(f, 0, SEEK_END);
    n = (size_t)ftell(f) / 160;
    fseek(f, 0, SEEK_SET);
    recs = malloc(n * 160);
    if (fread(recs, 160, n, f) != n) return 4;
    fclose(f);
    EC_GROUP* grp = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
    keys = calloc(n, sizeof *keys);
    sigs = calloc(n, sizeof *sigs);
    for (size_t i = 0; i < n; ++i) {
        unsigned char* rec = recs + 160 * i;
        unsigned char oct[65];
        oct[0] = 4;
        memcpy(oct + 1, rec + 96, 64);
        EC_KEY* k = EC_KEY_new();
        EC_KEY_set_group(k, grp);
        if (EC_KEY_oct2key(k, oct, 65, NULL) == 1) keys[i] = k;
        else EC_KEY_free(k);
        sigs[i] = ECDSA_SIG_new();
        ECDSA_SIG_set0(sigs[i], BN_bin2bn(rec + 32, 32, NULL), BN_bin2bn(rec + 64, 32, NULL));
    }
    /* warm-up pass on one thread, then size the timed run to >= min_s */
    double t0 = now();
    size_t probe = n < 2000 ? n : 2000;
    for (size_t i = 0; i < probe; ++i)
        if (keys[i]) ECDSA_do_verify(recs + 160 * i, 32, sigs[i], keys[i]);
    double per = (now() - t0) / (double)probe;
    (void)per;
    const int runs = argc > 4 ? atoi(argv[4]) : 1;
    pthread_t* th = malloc(sizeof(pthread_t) * nt);
    double rates[64];
    double secs = 0;
    int done = 0;
    size_t count = 0;
    for (int r = -1; r < runs && r < 63; ++r) {  /* r = -1: the untimed warm-up run */
        atomic_store(&next_idx, 0);
        atomic_store(&accepted, 0);
        atomic_store(&stop_flag, 0);
        total_target = (size_t)-1;  /* every run lasts min_s: the workers stop at the deadline */
        t0 = now();
        for (int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, worker, NULL);
        const struct timespec nap = {(time_t)min_s, (long)((min_s - (double)(time_t)min_s) * 1e9)};
        nanosleep(&nap, NULL);
        atomic_store(&stop_flag, 1);
        for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
        const double dt = now() - t0;
        /* a worker takes an index only before the deadline and verifies every index it took */
        const size_t taken = atomic_load(&next_idx);
        count = taken;
        if (r < 0) continue;
        rates[done++] = (double)count / dt;
        secs = dt;
    }
    total_target = count;
    double sorted[64];
    memcpy(sorted, rates, sizeof(double) * done);
    for (int i = 1; i < done; ++i)
        for (int j = i; j > 0 && sorted[j] < sorted[j - 1]; --j) {
            const double x = sorted[j];
            sorted[j] = sorted[j - 1];
            sorted[j - 1] = x;
        }
    const double med = done % 2 ? sorted[done / 2] : 0.5 * (sorted[done / 2 - 1] + sorted[done / 2]);
    printf("{\"verifies_per_s\": %.1f, \"threads\": %d, \"n\": %zu, \"accepted\": %zu, \"seconds\": %.3f, "
           "\"runs\": %d, \"runs_per_s\": [",
           med, nt, total_target, (size_t)atomic_load(&accepted), secs, done);
    for (int i = 0; i < done; ++i) printf("%s%.1f", i ? ", " : "", rates[i]);
    printf("]}\n");
    return 0;
}
