/* Measurement helper for bench.py (not part of the codec): times synchronous
 * iggy_codec_decode_batch calls from C, the way a native caller (the Rust shim of
 * INTEGRATION.md) makes them, without the Python/ctypes cost of building arguments
 * per call. The function is passed in by address, so this library links nothing.
 * build: gcc -O2 -shared -fPIC -o scripts/_c_loop.so scripts/c_loop.c */
#include <stdint.h>
#include <time.h>

#include "../include/iggy_codec.h"

typedef int (*decode_fn)(iggy_codec_ctx *ctx, const uint8_t *body, uint64_t len, int integrity, iggy_batch_header *hdr,
                         uint64_t *frame_pos, uint64_t cap, uint64_t *nframes, iggy_wire_error *err);

/* reps passes over the nrec records; returns the mean ns per call, or -rc of the first
 * failing call (a call that decodes fewer than expect[i] frames fails with -1000) */
double c_loop_decode(void *fn, void *ctx, const uint8_t **recs, const uint64_t *lens, uint64_t **poss,
                     const uint64_t *caps, const uint64_t *expect, int nrec, int integrity, int reps) {
    decode_fn f = (decode_fn)fn;
    iggy_batch_header h;
    iggy_wire_error e;
    uint64_t n = 0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; ++r)
        for (int i = 0; i < nrec; ++i) {
            const int rc = f((iggy_codec_ctx *)ctx, recs[i], lens[i], integrity, &h, poss[i], caps[i], &n, &e);
            if (rc) return -(double)rc;
            if (n != expect[i]) return -1000.0;
        }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double ns = (double)(t1.tv_sec - t0.tv_sec) * 1e9 + (double)(t1.tv_nsec - t0.tv_nsec);
    return ns / ((double)reps * nrec);
}
