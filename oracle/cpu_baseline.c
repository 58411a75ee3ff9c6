/*
 * cpu_baseline.c — TEST/BENCH INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The timed CPU baseline of bench.py: decode_batch_slice_with(Verify)
 * (core/binary_protocol/src/batch.rs:391-506) restated as in codec_ref.c, but
 * with the AVX2 XXH3 accumulate (twox-hash 2.x also dispatches to AVX2) and
 * built -O3 -march=native, matching the reference perf suite's
 * RUSTFLAGS="-C target-cpu=native". One thread walks one batch serially — the
 * reference's execution model (one shard thread per batch); `threads` threads
 * decode independent copies concurrently.
 */
#include "oracle.h"
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static inline uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

/* Returns computed batch checksum, or 0 with *ok = 0 on any error. layout_only:
 * validate_batch_layout (batch.rs:508-527) instead of the Verify hash walk
 * (batch.rs:474-506): the same frame walk and tiling check, no checksum. */
static uint64_t decode_walk_fast(const uint8_t *body, uint64_t len, uint8_t *scratch, int layout_only,
                                 int *ok) {
    iggy_batch_header h;
    iggy_wire_error e;
    *ok = 0;
    if (oracle_batch_header_decode(body, len, &h, &e)) return 0;
    if (len < h.batch_length) return 0;
    const uint8_t *blob = body + 256;
    uint64_t blob_len = h.batch_length - 256, pos = 0, n = 0;
    memcpy(scratch + 0, body + 0, 40);         /* 5 u64 fields in header order */
    memcpy(scratch + 40, body + 48, 4);        /* message_count */
    while (pos < blob_len) {
        if (blob_len - pos < 48 || rd64(blob + pos + 40) != 0) break;
        uint64_t end = pos + 48 + (uint64_t)rd32(blob + pos + 36) + rd32(blob + pos + 32);
        if (end > blob_len) break;
        if (!layout_only) {
            uint64_t stored = rd64(blob + pos);
            if (oracle_xxh3_64_fast(blob + pos + 8, end - pos - 8) != stored) return 0;
            memcpy(scratch + 44 + 8 * n, blob + pos, 8);
        }
        n++;
        pos = end;
    }
    if (n != h.message_count || pos != blob_len) return 0;
    if (layout_only) {
        *ok = 1;
        return 0;
    }
    uint64_t c = oracle_xxh3_64_fast(scratch, 44 + 8 * n);
    if (c != h.batch_checksum) return 0;
    *ok = 1;
    return c;
}

typedef struct {
    const uint8_t *body;
    uint64_t len;
    int reps, layout_only;
    uint64_t checksum;
    int ok;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    uint8_t *scratch = (uint8_t *)malloc(44 + 8 * (j->len / 48 + 1));
    j->ok = 1;
    for (int r = 0; r < j->reps; r++) {
        int ok;
        j->checksum = decode_walk_fast(j->body, j->len, scratch, j->layout_only, &ok);
        j->ok &= ok;
    }
    free(scratch);
    return NULL;
}

double oracle_cpu_decode_bench(const uint8_t *body, uint64_t len, int threads, int reps,
                               uint64_t *checksum_out) {
    return oracle_cpu_decode_bench_integrity(body, len, threads, reps, 0, checksum_out);
}

/* The same with integrity 0 = Verify, 1 = LayoutOnly (IGGY_INTEGRITY_*): the CPU leg
 * of a crossover timed with the same integrity as its GPU leg. */
double oracle_cpu_decode_bench_integrity(const uint8_t *body, uint64_t len, int threads, int reps,
                                         int integrity, uint64_t *checksum_out) {
    if (threads < 1) threads = 1;
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    job_t *jobs = (job_t *)calloc(threads, sizeof(job_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t].body = body;
        jobs[t].len = len;
        jobs[t].reps = reps;
        jobs[t].layout_only = integrity == 1;
        pthread_create(&tid[t], NULL, worker, &jobs[t]);
    }
    int ok = 1;
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        ok &= jobs[t].ok;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (checksum_out) *checksum_out = ok ? jobs[0].checksum : 0;
    free(tid);
    free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* SendMessagesEncoder::encode (send_messages.rs:89-181) restated in codec_ref.c,
 * timed the same way: `threads` threads each encode the same SoA input into a
 * buffer of their own, `reps` times. Returns seconds; *bytes_out = batch bytes
 * of one encode (0 on any error). */
typedef struct {
    const iggy_raw_messages *m;
    uint64_t partition_id, need, bytes;
    int reps, ok;
} enc_job_t;

static void *enc_worker(void *arg) {
    enc_job_t *j = (enc_job_t *)arg;
    uint8_t *out = (uint8_t *)malloc(j->need + 16);
    j->ok = out != NULL;
    for (int r = 0; r < j->reps && j->ok; r++) {
        uint64_t n = 0;
        iggy_wire_error e;
        j->ok &= oracle_encode_batch(j->m, j->partition_id, out, j->need, &n, &e) == 0;
        j->bytes = n;
    }
    free(out);
    return NULL;
}

double oracle_cpu_encode_bench(const iggy_raw_messages *m, uint64_t partition_id, int threads, int reps,
                               uint64_t *bytes_out) {
    if (threads < 1) threads = 1;
    const uint64_t need = oracle_encoded_batch_size(m);
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    enc_job_t *jobs = (enc_job_t *)calloc(threads, sizeof(enc_job_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t].m = m;
        jobs[t].partition_id = partition_id;
        jobs[t].need = need;
        jobs[t].reps = reps;
        pthread_create(&tid[t], NULL, enc_worker, &jobs[t]);
    }
    int ok = 1;
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        ok &= jobs[t].ok;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (bytes_out) *bytes_out = ok ? jobs[0].bytes : 0;
    free(tid);
    free(jobs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---------------------------------------------------------------------------
 * CPU baseline of the at-rest encryption re-encode's crypto: AES-256-GCM seal of
 * nsec sections of secsize bytes per thread through the system OpenSSL
 * (libcrypto EVP_aes_256_gcm, AES-NI / PCLMULQDQ when the CPU has them) -- the
 * same algorithm the reference's `aes-gcm` crate runs per section
 * (crypto.rs:70-78). libcrypto is opened at run time (no link dependency);
 * returns seconds, or -1 when it is unavailable. */
#include <dlfcn.h>
typedef struct {
    void *(*ctx_new)(void);
    void (*ctx_free)(void *);
    const void *(*cipher)(void);
    int (*init)(void *, const void *, void *, const unsigned char *, const unsigned char *);
    int (*update)(void *, unsigned char *, int *, const unsigned char *, int);
    int (*final)(void *, unsigned char *, int *);
    int (*ctrl)(void *, int, int, void *);
    /* OpenSSL 3: a cipher fetched per worker (EVP_CIPHER_fetch), so the workers share
     * no reference-counted cipher object; NULL -> the legacy EVP_aes_256_gcm() */
    void *(*fetch)(void *, const char *, const char *);
    void (*cipher_free)(void *);
} evp_t;
typedef struct {
    const evp_t *e;
    int nsec, secsize, ok;
    /* timed form: every worker starts at the barrier and seals until the shared
     * deadline; done = sections sealed */
    pthread_barrier_t *start;
    const struct timespec *deadline;
    long long done;
} gcm_job_t;
static int past(const struct timespec *d) {
    struct timespec now;
    clock_gettime(CLOCK_MONOTONIC, &now);
    return now.tv_sec > d->tv_sec || (now.tv_sec == d->tv_sec && now.tv_nsec >= d->tv_nsec);
}
static void *gcm_worker(void *arg) {
    gcm_job_t *j = (gcm_job_t *)arg;
    unsigned char key[32], iv[12], tag[16];
    for (int i = 0; i < 32; ++i) key[i] = (unsigned char)(i * 7 + 1);
    memset(iv, 3, 12);
    unsigned char *in = (unsigned char *)malloc(j->secsize + 16), *out = (unsigned char *)malloc(j->secsize + 32);
    memset(in, 0x5a, j->secsize);
    void *c = j->e->ctx_new();
    j->ok = c != NULL;
    /* The key schedule once per thread (as a long-lived Aes256GcmEncryptor), a fresh
     * nonce per section. The nonce comes from the context's own IV generator
     * (EVP_CTRL_GCM_SET_IV_FIXED over the whole 12 bytes, then EVP_CTRL_GCM_IV_GEN per
     * section: the counter advances and the GCM state is re-keyed with it in place).
     * Re-initialising the context with each nonce (EVP_EncryptInit_ex(ctx, NULL, ...,
     * iv)) takes and drops references on the provider's shared cipher object on every
     * section: threads then contend on one cache line (1 -> 16 threads measured 1.8x
     * on the GPU box; 1 -> 2 threads 1.0x here), which says nothing about AES-GCM. */
    void *own = j->e->fetch ? j->e->fetch(NULL, "AES-256-GCM", NULL) : NULL;
    if (j->ok) j->ok &= j->e->init(c, own ? own : j->e->cipher(), NULL, key, iv) == 1;
    if (j->ok) j->ok &= j->e->ctrl(c, 0x12 /* EVP_CTRL_GCM_SET_IV_FIXED */, -1, iv) == 1;
    if (j->start) pthread_barrier_wait(j->start);
    for (long long s = 0; j->ok; ++s) {
        if (j->deadline ? ((s & 63) == 0 && past(j->deadline)) : s >= j->nsec) break;
        j->done = s + 1;
        int ol = 0, fl = 0;
        unsigned char nonce[12];
        j->ok &= j->e->ctrl(c, 0x13 /* EVP_CTRL_GCM_IV_GEN */, 12, nonce) == 1;
        j->ok &= j->e->update(c, out, &ol, in, j->secsize) == 1;
        j->ok &= j->e->final(c, out + ol, &fl) == 1;
        j->ok &= j->e->ctrl(c, 0x10 /* EVP_CTRL_GCM_GET_TAG */, 16, tag) == 1;
    }
    if (c) j->e->ctx_free(c);
    if (own && j->e->cipher_free) j->e->cipher_free(own);
    free(in);
    free(out);
    return NULL;
}
static evp_t gcm_evp;
static int gcm_load(void) {
    static int loaded = 0;
    evp_t *e = &gcm_evp;
    if (!loaded) {
        void *h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
        if (!h) return 0;
        e->ctx_new = (void *(*)(void))dlsym(h, "EVP_CIPHER_CTX_new");
        e->ctx_free = (void (*)(void *))dlsym(h, "EVP_CIPHER_CTX_free");
        e->cipher = (const void *(*)(void))dlsym(h, "EVP_aes_256_gcm");
        e->init = (int (*)(void *, const void *, void *, const unsigned char *, const unsigned char *))dlsym(
            h, "EVP_EncryptInit_ex");
        e->update = (int (*)(void *, unsigned char *, int *, const unsigned char *, int))dlsym(h, "EVP_EncryptUpdate");
        e->final = (int (*)(void *, unsigned char *, int *))dlsym(h, "EVP_EncryptFinal_ex");
        e->ctrl = (int (*)(void *, int, int, void *))dlsym(h, "EVP_CIPHER_CTX_ctrl");
        e->fetch = (void *(*)(void *, const char *, const char *))dlsym(h, "EVP_CIPHER_fetch");
        e->cipher_free = (void (*)(void *))dlsym(h, "EVP_CIPHER_free");
        if (!e->ctx_new || !e->ctx_free || !e->cipher || !e->init || !e->update || !e->final || !e->ctrl) return 0;
        loaded = 1;
    }
    return 1;
}

/* threads x nsec seals; returns seconds (spawn included), -1 when unavailable */
double oracle_cpu_gcm_bench(int threads, int nsec, int secsize) {
    if (!gcm_load()) return -1.0;
    if (threads < 1) threads = 1;
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    gcm_job_t *jobs = (gcm_job_t *)calloc(threads, sizeof(gcm_job_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t].e = &gcm_evp;
        jobs[t].nsec = nsec;
        jobs[t].secsize = secsize;
        pthread_create(&tid[t], NULL, gcm_worker, &jobs[t]);
    }
    int ok = 1;
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        ok &= jobs[t].ok;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(tid);
    free(jobs);
    if (!ok) return -1.0;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* Timed form: `threads` workers released together by a barrier seal secsize-byte
 * sections until a shared deadline `seconds` later; returns the sections sealed
 * (throughput = sections x secsize / seconds), -1 when unavailable. Thread start-up is
 * outside the timed window, so T threads measure T cores, not spawn latency. */
double oracle_cpu_gcm_bench_timed(int threads, double seconds, int secsize) {
    if (!gcm_load()) return -1.0;
    if (threads < 1) threads = 1;
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    gcm_job_t *jobs = (gcm_job_t *)calloc(threads, sizeof(gcm_job_t));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)threads + 1);
    struct timespec dl;
    for (int t = 0; t < threads; t++) {
        jobs[t].e = &gcm_evp;
        jobs[t].secsize = secsize;
        jobs[t].start = &bar;
        jobs[t].deadline = &dl;
        pthread_create(&tid[t], NULL, gcm_worker, &jobs[t]);
    }
    clock_gettime(CLOCK_MONOTONIC, &dl);  /* set before the release: workers read it after the barrier */
    const long long ns = (long long)(seconds * 1e9);
    dl.tv_sec += ns / 1000000000LL;
    dl.tv_nsec += ns % 1000000000LL;
    if (dl.tv_nsec >= 1000000000L) { dl.tv_sec += 1; dl.tv_nsec -= 1000000000L; }
    pthread_barrier_wait(&bar);
    int ok = 1;
    long long total = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        ok &= jobs[t].ok;
        total += jobs[t].done;
    }
    pthread_barrier_destroy(&bar);
    free(tid);
    free(jobs);
    return ok ? (double)total : -1.0;
}
