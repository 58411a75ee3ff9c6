// host_ctx.hpp -- the codec context and its scratch: device / mapped-host buffers, the
// asynchronous slots, the context struct, scratch sizing and the stream order
//
// Part of the unity build of libiggy_codec.so: included by codec_api.hip, after the
// kernel translation units and the units before it (see codec_api.hip for the order).
#pragma once

namespace {

// Host-memory history: every registration, mapped / pinned allocation and their
// release, so a later fault can be checked against ranges the codec pinned or mapped
// (VERDICT r05 item 5). IGGY_CODEC_DEBUG: on stderr; IGGY_CODEC_HOSTMEM_LOG=<path>:
// appended to that file, one line per event with a monotonic timestamp (the test suite
// sets it and attaches the tail to a failing test's report, tests/conftest.py).
FILE *hostmem_file() {
    static FILE *f = [] {
        const char *p = getenv("IGGY_CODEC_HOSTMEM_LOG");
        FILE *h = p && *p ? fopen(p, "a") : nullptr;
        if (h) setvbuf(h, nullptr, _IOLBF, 0);
        return h;
    }();
    return f;
}
bool hostmem_log_on() {
    static const bool on = getenv("IGGY_CODEC_DEBUG") != nullptr || hostmem_file() != nullptr;
    return on;
}
void hostmem_log(const char *what, const void *p, uint64_t n) {
    if (!hostmem_log_on()) return;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    char line[256];
    snprintf(line, sizeof line, "%.6f iggy_codec hostmem: %s [%p, %p) %llu B\n", t, what, p,
             (const void *)((const uint8_t *)p + n), (unsigned long long)n);
    if (getenv("IGGY_CODEC_DEBUG")) fputs(line, stderr);
    if (FILE *f = hostmem_file()) fputs(line, f);
}

// process-wide allocation counters (iggy_codec_host_stats)
std::atomic<uint64_t> g_dev_allocs{0}, g_pin_allocs{0};

// one device allocation that grows on demand (never inside an enqueue path
// whose caller asked for graph-safety: grow happens in reserve / sync APIs)
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t n) {
        if (n <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(n, 256);
        if (hipMalloc(&p, want) != hipSuccess) return IGGY_ERR_DEVICE;
        g_dev_allocs.fetch_add(1, std::memory_order_relaxed);
        cap = want;
        return 0;
    }
    template <class T> T *as(size_t off = 0) { return (T *)((uint8_t *)p + off); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Mapped, coherent pinned host memory that kernels read and write directly (small
// tables in, results / positions / flags out): no copy operation on the stream.
constexpr size_t kHostMapKeep = 8ull << 20;  // pinned bytes a context keeps between calls
struct HostMap {
    void *h = nullptr;
    uint8_t *d = nullptr;  // the device's address of the same bytes
    size_t cap = 0;
    int ensure(size_t n) {
        // grown past kHostMapKeep by one large call (a poll of many small frames, a
        // 16 MiB decode with positions): given back at the next ordinary-sized call
        // instead of staying pinned for the context's life
        if (n <= cap && !(cap > kHostMapKeep && n <= kHostMapKeep)) return 0;
        release();
        const size_t want = std::max<size_t>(n, 64 << 10);
        if (hipHostMalloc(&h, want, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
            h = nullptr;
            return IGGY_ERR_DEVICE;
        }
        if (hipHostGetDevicePointer((void **)&d, h, 0) != hipSuccess) {
            release();
            return IGGY_ERR_DEVICE;
        }
        cap = want;
        g_pin_allocs.fetch_add(1, std::memory_order_relaxed);
        hostmem_log("mapped alloc", h, want);
        // the completion flag lives in the first word: pinned memory handed back by the
        // allocator may still hold another context's flag values, one of which this
        // context's sequence could reach before its kernel writes it
        memset(h, 0, 256);
        return 0;
    }
    template <class T> T *hp(size_t off = 0) { return (T *)((uint8_t *)h + off); }
    template <class T> T *dp(size_t off = 0) { return (T *)(d + off); }
    void release() {
        if (h) {
            hostmem_log("mapped free", h, cap);
            (void)hipHostFree(h);
        }
        h = nullptr;
        d = nullptr;
        cap = 0;
    }
};

}  // namespace

// an asynchronous encode's own scratch (enqueue_encode's per-batch arrays)
struct EncOwn {
    DevBuf epl, euh, etile, ecs, emisc, bsums;
    void release() {
        for (DevBuf *b : {&epl, &euh, &etile, &ecs, &emisc, &bsums}) b->release();
    }
};

// one asynchronous host-buffer operation in flight (iggy_codec_*_submit / iggy_codec_poll)
constexpr int kSlots = 8;
struct Slot {
    bool busy = false;
    uint64_t ticket = 0;
    uint32_t op = 0;
    uint64_t cap = 0, out_len = 0;
    // a single-stride decode submitted on the fast path (one records launch): what
    // iggy_codec_poll needs to run the general walk when its stride breaks mid-record
    bool fast = false, g_pending = false;
    const uint8_t *g_in = nullptr;
    uint64_t g_len = 0, g_pcap = 0;
    uint64_t *g_pos = nullptr;  // device-visible positions destination of the launch
    int g_integ = 0;
    bool g_pos_copy = false;    // positions go through `pos` and a D2H copy
    uint64_t *frame_pos = nullptr;               // host destination of the decode's positions
    DevBuf in, pos, out, res;                    // device input / positions / encode output / result
    DevBuf ids, ots, pay, plen, uhb, uhl;        // encode SoA inputs
    HostMap tab;                                 // k_decode_records task table of an in-flight decode
    // a pageable input of the fast path, copied here at submit: the kernel reads it in
    // place (<= kZeroCopyBytes) or one DMA copies it, and the slot keeps it until it is
    // done, so submit never waits on the stream for the caller's bytes
    HostMap zin;
    // the fast path's own stream and k_decode_records scratch: fast-path decodes of
    // different slots run side by side (a small record's launch is bound by its reads'
    // round trips over the host link, not by the chip)
    hipStream_t st = nullptr;
    DevBuf rstate, rbsums, rcount;
    EncOwn eown;  // (small encodes in place: the same, for enqueue_encode)
    hipEvent_t ev_in = nullptr, ev_k = nullptr, ev_done = nullptr;
    // a pageable caller output is never a DMA target: the copy-out stream lands it in
    // this pinned bounce and iggy_codec_poll copies it to the caller (hout_dst, hout_len)
    void *hout = nullptr;
    size_t hout_cap = 0;
    uint8_t *hout_dst = nullptr;
    uint64_t hout_len = 0;
    int hout_ensure(size_t n) {
        if (n <= hout_cap && !(hout_cap > (8ull << 20) && n <= (8ull << 20))) return 0;
        if (hout) {
            hostmem_log("bounce free", hout, hout_cap);
            (void)hipHostFree(hout);
        }
        hout = nullptr;
        hout_cap = 0;
        const size_t want = std::max<size_t>(n, 64 << 10);
        if (hipHostMalloc(&hout, want, hipHostMallocDefault) != hipSuccess) {
            hout = nullptr;
            return IGGY_ERR_DEVICE;
        }
        hout_cap = want;
        g_pin_allocs.fetch_add(1, std::memory_order_relaxed);
        hostmem_log("bounce alloc", hout, want);
        return 0;
    }
    void release() {
        DevBuf *b[] = {&in, &pos, &out, &res, &ids, &ots, &pay, &plen, &uhb, &uhl, &rstate, &rbsums, &rcount};
        for (DevBuf *x : b) x->release();
        tab.release();
        zin.release();
        eown.release();
        if (st) (void)hipStreamDestroy(st), st = nullptr;
        for (hipEvent_t *e : {&ev_in, &ev_k, &ev_done})
            if (*e) (void)hipEventDestroy(*e), *e = nullptr;
        if (hout) {
            hostmem_log("bounce free", hout, hout_cap);
            (void)hipHostFree(hout);
        }
        hout = nullptr;
        hout_cap = 0;
    }
};

constexpr size_t kCrTabBytesHost = (size_t)kGhPowers * 32 * 8;  // GHASH tables (= kCrTabBytes below)
constexpr int kEncSegs = 4;                   // encode segments (checksum chain overlap); bounds below
constexpr uint64_t kEncSegMinFrames = 1 << 18;  // below this one segment

struct iggy_codec_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    int ncu = 256;
    // uniform decode grid: one WG per CU but one. A pipelined decode's consumer WG
    // (the previous batch's chain tail) then never holds back one of the next
    // decode's producer WGs. IGGY_CODEC_UNIFORM_GRID overrides it in the diagnostic
    // build only.
    int ugrid = 255;
    uint32_t epoch = 0;
    int allow_unaligned = 0;
    uint32_t dbg = 0;  // IGGY_CODEC_DBG ablation bits: read only by the diagnostic build (kDiagMask)
    // one stream order per context (its scratch is shared by every enqueue): the
    // stream of the latest enqueue, and the event a switch to another stream waits on
    hipStream_t last = nullptr;
    hipEvent_t order_ev = nullptr;
    // decode scratch
    uint64_t dec_cap_len = 0;
    DevBuf dsync;    // exited | first_bad | spec_fail | bar[4] | misc[16] | small[512] | bar2 (128-B stride)
    DevBuf dsums, derr;
    DevBuf gtiles_s, gtiles_x, gtiles_cnt, gtiles_pre, gtiles_list, gtiles_e, gtiles_base, ggrp, gfpos, gcs, gvrec, gtiles_lcs, gbsums;
    int gen_grid = 0;  // WGs of k_decode_general (the ones that get a CU join its barriers)
    // encode: the batch-checksum chain of earlier frame segments runs on `side`
    // while later segments are encoded on the call's stream
    hipStream_t side = nullptr;
    hipEvent_t seg_ev[kEncSegs + 2] = {};  // segment ends, side-stream end, fork ([kEncSegs + 1])
    DevBuf dresult;  // iggy_decode_result + iggy_encode_result + u64 scratch
    // sync-API staging
    DevBuf din, dpos, dout;
    // encode scratch
    DevBuf epl, euh, etile, ecs, emisc;
    DevBuf eids, eots, epay, eplen, euhb, euhl;
    DevBuf erec, esink;  // k_enc_ring's frame records and store sink
    // big one-shot hash
    DevBuf hbsums;
    // poll
    DevBuf ppos, pmsgs, pres;
    DevBuf cwk;  // disk-chunk walk: state, gates, per-batch slice results, fragments
    // multi-record decode (decode_records.hip): tasks | states | wg map, block sums,
    // results, and the pinned staging of the task table (uploaded in one copy)
    DevBuf rtab, rbsums, rres, clinks, rstate, rcount;
    HostMap rmap;  // task table + workgroup map (read by the kernel in place when small)
    HostMap cmap;  // chunk-walk candidates (read in place)
    HostMap omap;  // [0, 64): completion flag; then results / positions / chunk-walk outputs
    // a pageable record of <= kZeroCopyBytes for the synchronous fast path (or a small
    // synchronous encode's SoA input), copied here and read by the kernels in place
    HostMap zin;
    HostMap zout;  // a small synchronous encode's wire bytes when the caller's `out` is not mapped
    uint32_t hseq = 0;  // completion flag values
    uint32_t chunk_epoch = 0;  // k_chunk_walk link tags
    // segment writer: pinned staging halves and their copy events
    void *wstage = nullptr;
    hipEvent_t wev[2] = {nullptr, nullptr};
    // slice / device stamp: [0,512) control words + header + small, then tile counts
    DevBuf sl, slres;
    // at-rest encryption: [0,64) misc, [64,192) output header, [192] n, [200] checksum,
    // [256,384) decode result, [1024, +16 KiB) GHASH tables, then sizes / positions / tile sums
    DevBuf cr;
    void *cr_pinned = nullptr;   // host staging of the GHASH tables
    // poll reply body: per-record decrypt verdicts, and the pinned host staging of the
    // concatenated records / decrypted output (one H2D, one D2H per body)
    DevBuf pbres;
    void *pb_pinned = nullptr;
    size_t pb_cap = 0;
    // fingerprint of the key whose tables are on the device: E_K(0) || E_K(1), never the
    // key itself (the reference keeps the key only inside its Aes256Gcm cipher object)
    uint8_t cr_fp[32] = {};
    bool cr_key_set = false;
    // pinned host mirror of results
    void *h_pinned = nullptr;
    // caller host memory (put_host / get_host): the two pinned chunks pageable bytes are
    // staged through, their last copies' events, and the event after a call's last H2D
    void *xst = nullptr;
    hipEvent_t xev[2] = {nullptr, nullptr};
    bool xlive[2] = {false, false};
    uint32_t xnext = 0;
    hipEvent_t xin_ev = nullptr;
    bool xin_live = false;
    iggy_host_stats hs = {};  // iggy_codec_host_stats (the allocation counts are process-wide)
    // resident decode service (iggy_codec_service_start, k_decode_service): its mailbox
    // (host-mapped), control block, record state and block sums, its stream, the last
    // post's sequence number, and whether the context uses it
    struct {
        HostMap mb;
        DevBuf ctl, st, bsums;
        hipStream_t s = nullptr;
        bool enabled = false, launched = false;
        uint32_t seq = 0;
        uint64_t posts = 0, launches = 0;
        uint64_t dev_ticks[8] = {};  // (diagnostic build: summed device time of the posts)
    } svc;
    // asynchronous host-buffer operations: copy-in stream -> the context's stream -> copy-out
    // stream, so one operation's H2D, another's kernels and a third's D2H overlap
    hipStream_t h2d = nullptr, d2h = nullptr;
    Slot slots[kSlots];
    void *slot_pinned = nullptr;  // kSlots x 256 B: completion records
    uint8_t *slot_pinned_d = nullptr;  // its device-mapped address (kernels write decode verdicts there)
    uint64_t seq = 0;
    // profiling
    int profile = 0;
    hipEvent_t ev0[2] = {nullptr, nullptr}, ev1[2] = {nullptr, nullptr};
    uint64_t prof_n[2] = {0, 0};
    double prof_ms[2] = {0, 0};
    bool ev_pending[2] = {false, false};
};

namespace {

constexpr size_t kSyncExited = 0, kSyncFirstBad = 8, kSyncSpecFail = 16, kSyncBar = 32,
                 kSyncMisc = 64, kSyncSmall = 256, kSyncBar2 = 1024,  // + kBar2Words u32 at 128-B stride
                 kSyncSink = kSyncBar2 + kBar2Words * 128,            // 64 x u64 (DecodeScratch::sink)
                 kSyncBytes = kSyncSink + 512;

int ensure_decode_scratch(iggy_codec_ctx *c, uint64_t len) {
    if (len <= c->dec_cap_len && c->dsync.p) return 0;
    const uint64_t L = std::max<uint64_t>(len, 1 << 20);
    const uint64_t max_frames = L / 48 + 2;
    const uint64_t max_chunks = (max_frames + 6) / 256 + 2;
    const uint64_t ntiles = L / kTileMin + 2;
    const uint64_t ngroups = ntiles / kGrpTiles + 2;
    const uint64_t max_blocks = (44 + 8 * max_frames) / 1024 + 2;
    int r = 0;
    if (!c->dsync.p) {
        r |= c->dsync.ensure(kSyncBytes);
        if (r) return r;
        HIP_OK(hipMemset(c->dsync.p, 0, kSyncBytes));
    }
    // one 128-B block record per 128 frames (2 per chunk, decode_uniform.hip); zeroed
    // so no stale tag can match a live epoch
    r |= c->dsums.ensure(max_chunks * kChunkSumWords * 8 + 64);
    if (!r && c->dsums.p) HIP_OK(hipMemset(c->dsums.p, 0, c->dsums.cap));
    r |= c->derr.ensure(max_chunks * 32 * 16);  // (stored, computed) per 8-frame group
    r |= c->gtiles_s.ensure(ntiles * 8);
    r |= c->gtiles_x.ensure(ntiles * 8);
    r |= c->gtiles_cnt.ensure(ntiles * 4);
    r |= c->gtiles_e.ensure(ntiles * 8);
    r |= c->gtiles_pre.ensure(ntiles * 4);
    r |= c->gtiles_list.ensure(tile_list_words(L) * 4);
    r |= c->ggrp.ensure(ngroups * kGrpWords * 8);
    r |= c->gtiles_base.ensure(ntiles * 8);
    r |= c->gfpos.ensure(max_frames * 8);
    r |= c->gcs.ensure(max_frames * 8 + 16);       // verify_frames_dma reads aligned pairs
    r |= c->gvrec.ensure((max_frames + 1) * 16);   // walk-order frame records + "none"
    r |= c->gtiles_lcs.ensure(tile_list_words(L) * 8);
    r |= c->gbsums.ensure(max_blocks * 64);
    if (r) return IGGY_ERR_DEVICE;
    c->dec_cap_len = L;
    return 0;
}

DecodeScratch dscratch(iggy_codec_ctx *c) {
    DecodeScratch s;
    s.exited = c->dsync.as<uint32_t>(kSyncExited);
    s.first_bad = c->dsync.as<uint64_t>(kSyncFirstBad);
    s.spec_fail = c->dsync.as<uint64_t>(kSyncSpecFail);
    s.sums = c->dsums.as<uint64_t>();
    s.errslot = c->derr.as<uint64_t>();
    s.small = c->dsync.as<uint8_t>(kSyncSmall);
    s.sink = c->dsync.as<uint64_t>(kSyncSink);
    s.gbar = c->dsync.as<uint32_t>(kSyncBar);
    s.gbar2 = c->dsync.as<uint32_t>(kSyncBar2);
    s.gmisc = c->dsync.as<uint64_t>(kSyncMisc);
    s.max_chunks = (c->dsums.cap - 64) / (kChunkSumWords * 8);
    return s;
}

// diagnostic ablation bits, zero in the product build
inline uint32_t diag_bits(const iggy_codec_ctx *c) { return c->dbg & kDiagMask; }

GeneralScratch gscratch(iggy_codec_ctx *c) {
    GeneralScratch g;
    g.tile_s = c->gtiles_s.as<uint64_t>();
    g.tile_x = c->gtiles_x.as<uint64_t>();
    g.tile_cnt = c->gtiles_cnt.as<uint32_t>();
    g.tile_e = c->gtiles_e.as<uint64_t>();
    g.tile_pre = c->gtiles_pre.as<uint32_t>();
    g.tile_list = c->gtiles_list.as<uint32_t>();
    g.grp = c->ggrp.as<uint64_t>();
    g.tile_base = c->gtiles_base.as<uint64_t>();
    g.fpos = c->gfpos.as<uint64_t>();
    g.cs = c->gcs.as<uint64_t>();
    g.vrec = c->gvrec.as<uint64_t>();
    g.tile_lcs = c->gtiles_lcs.as<uint64_t>();
    g.bsums = c->gbsums.as<uint64_t>();
    g.misc = c->dsync.as<uint64_t>(kSyncMisc);
    g.bar = c->dsync.as<uint32_t>(kSyncBar);
    g.bar2 = c->dsync.as<uint32_t>(kSyncBar2);
    g.u_exited = c->dsync.as<uint32_t>(kSyncExited);
    g.u_first_bad = c->dsync.as<uint64_t>(kSyncFirstBad);
    g.u_spec_fail = c->dsync.as<uint64_t>(kSyncSpecFail);
    g.small = c->dsync.as<uint8_t>(kSyncSmall);
    g.ntiles = c->gtiles_s.cap / 8;
    g.max_frames = c->gfpos.cap / 8;
    g.max_blocks = c->gbsums.cap / 64;
    g.dbg = diag_bits(c);
    return g;
}

// Every enqueue of a context runs in ONE stream order: the scratch it uses (sync
// words, unit sums, walk tables, result staging) belongs to the context. An
// enqueue on another stream than the previous one first makes that stream wait
// for everything enqueued before (an event recorded on the previous stream, which
// must therefore still exist). Enqueues on one stream pay nothing.
hipStream_t bind(iggy_codec_ctx *c, void *stream) {
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    if (s != c->last) {
        if (c->last && c->order_ev && hipEventRecord(c->order_ev, c->last) == hipSuccess)
            (void)hipStreamWaitEvent(s, c->order_ev, 0);
        c->last = s;
    }
    return s;
}

// The context's device is current for the duration of an entry point; the
// caller's current device is restored on return (multi-GPU processes keep
// one context per GPU on arbitrary threads).
struct DevGuard {
    int prev = -1, dev;
    explicit DevGuard(int d) : dev(d) {
        int cur = -1;
        if (hipGetDevice(&cur) == hipSuccess && cur != d && hipSetDevice(d) == hipSuccess) prev = cur;
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace
