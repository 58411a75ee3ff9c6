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

/* Returns computed batch checksum, or 0 with *ok = 0 on any error. */
static uint64_t decode_verify_fast(const uint8_t *body, uint64_t len, uint8_t *scratch,
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
        uint64_t stored = rd64(blob + pos);
        if (oracle_xxh3_64_fast(blob + pos + 8, end - pos - 8) != stored) return 0;
        memcpy(scratch + 44 + 8 * n, blob + pos, 8);
        n++;
        pos = end;
    }
    if (n != h.message_count || pos != blob_len) return 0;
    uint64_t c = oracle_xxh3_64_fast(scratch, 44 + 8 * n);
    if (c != h.batch_checksum) return 0;
    *ok = 1;
    return c;
}

typedef struct {
    const uint8_t *body;
    uint64_t len;
    int reps;
    uint64_t checksum;
    int ok;
} job_t;

static void *worker(void *arg) {
    job_t *j = (job_t *)arg;
    uint8_t *scratch = (uint8_t *)malloc(44 + 8 * (j->len / 48 + 1));
    j->ok = 1;
    for (int r = 0; r < j->reps; r++) {
        int ok;
        j->checksum = decode_verify_fast(j->body, j->len, scratch, &ok);
        j->ok &= ok;
    }
    free(scratch);
    return NULL;
}

double oracle_cpu_decode_bench(const uint8_t *body, uint64_t len, int threads, int reps,
                               uint64_t *checksum_out) {
    if (threads < 1) threads = 1;
    pthread_t *tid = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    job_t *jobs = (job_t *)calloc(threads, sizeof(job_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < threads; t++) {
        jobs[t].body = body;
        jobs[t].len = len;
        jobs[t].reps = reps;
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
