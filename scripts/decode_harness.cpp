// Diagnostic (not product): time iggy_codec_decode_batch_device from plain C++
// (no Python/torch in the process) on a C2 record file (argv[1]), to separate
// the kernel's own rate from anything the Python benchmark environment adds.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <chrono>
#include "../include/iggy_codec.h"
#include <string.h>
extern "C" int iggy_codec_debug_read(iggy_codec_ctx *, void *, uint64_t);
extern "C" int iggy_codec_debug_clear(iggy_codec_ctx *);

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: %s record.bin [reps]\n", argv[0]); return 2; }
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    FILE *f = fopen(argv[1], "rb");
    if (!f) { perror("open"); return 1; }
    fseek(f, 0, SEEK_END);
    const long L = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<unsigned char> h(L);
    if (fread(h.data(), 1, L, f) != (size_t)L) { fprintf(stderr, "short read\n"); return 1; }
    fclose(f);
    iggy_codec_ctx *cx = nullptr;
    if (iggy_codec_create(0, &cx)) { fprintf(stderr, "create failed\n"); return 1; }
    iggy_codec_reserve(cx, L, 0);
    unsigned char *d = nullptr;
    uint64_t *pos = nullptr;
    iggy_decode_result *res = nullptr;
    const uint64_t n = (uint64_t)L / 48;
    if (hipMalloc(&d, L) || hipMalloc(&pos, n * 8) || hipMalloc(&res, sizeof(*res))) return 1;
    if (hipMemcpy(d, h.data(), L, hipMemcpyHostToDevice)) return 1;
    void *s = iggy_codec_stream(cx);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) iggy_codec_decode_batch_device(cx, d, L, 0, pos, n, res, s);
    (void)hipStreamSynchronize((hipStream_t)s);
    (void)hipEventRecord(e0, (hipStream_t)s);
    for (int r = 0; r < reps; ++r) iggy_codec_decode_batch_device(cx, d, L, 0, pos, n, res, s);
    (void)hipEventRecord(e1, (hipStream_t)s);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    iggy_decode_result hr;
    (void)hipMemcpy(&hr, res, sizeof(hr), hipMemcpyDeviceToHost);
    printf("decode Verify: %.4f ms/decode  %.1f GB/s  err=%u frames=%lu path=%u\n", ms / reps,
           L / (ms / reps * 1e-3) / 1e9, hr.error.kind, (unsigned long)hr.frame_count, hr.path);
    if (getenv("HARNESS_STREAMS")) {  // decodes alternated over S contexts/streams (pipelined batches)
        const int ns = atoi(getenv("HARNESS_STREAMS"));
        std::vector<iggy_codec_ctx *> cs(ns, nullptr);
        std::vector<unsigned char *> recs(ns, nullptr);
        std::vector<iggy_decode_result *> rs(ns, nullptr);
        std::vector<uint64_t *> ps(ns, nullptr);
        for (int i = 0; i < ns; ++i) {
            if (iggy_codec_create(0, &cs[i])) return 1;
            iggy_codec_reserve(cs[i], L, 0);
            if (hipMalloc(&recs[i], L) || hipMalloc(&ps[i], n * 8) || hipMalloc(&rs[i], sizeof(iggy_decode_result)))
                return 1;
            (void)hipMemcpy(recs[i], d, L, hipMemcpyDeviceToDevice);
        }
        for (int w = 0; w < 2 * ns; ++w)
            iggy_codec_decode_batch_device(cs[w % ns], recs[w % ns], L, 0, ps[w % ns], n, rs[w % ns], nullptr);
        (void)hipDeviceSynchronize();
        auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < reps; ++r)
            iggy_codec_decode_batch_device(cs[r % ns], recs[r % ns], L, 0, ps[r % ns], n, rs[r % ns], nullptr);
        (void)hipDeviceSynchronize();
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        int bad = 0;
        for (int i = 0; i < ns; ++i) {
            iggy_decode_result x;
            (void)hipMemcpy(&x, rs[i], sizeof(x), hipMemcpyDeviceToHost);
            bad += x.error.kind != 0 || x.frame_count != 1048576;
        }
        printf("%d streams: %.4f ms/decode  %.1f GB/s  results_bad=%d\n", ns, sec * 1e3 / reps, L * reps / sec / 1e9,
               bad);
    }
    if (getenv("IGGY_CODEC_DBG") && (strtoul(getenv("IGGY_CODEC_DBG"), nullptr, 0) & 512)) {
        // one more decode with fresh stamps (us since consumer start, 100 MHz ticks)
        iggy_codec_debug_clear(cx);
        iggy_codec_decode_batch_device(cx, d, L, 0, pos, n, res, s);
        uint64_t t[64];
        iggy_codec_debug_read(cx, t, 512);
        const uint64_t *ts = t + 32;  // small + 256
        printf("stamps (us from consumer start):");
        for (int i = 0; i < 23; ++i)
            if (ts[i]) printf(" [%d]=%.1f", i, (double)(ts[i] - ts[0]) / 100.0);
        printf("\n");
    }
    iggy_codec_destroy(cx);
    return 0;
}
