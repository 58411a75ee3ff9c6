// host_decode.hpp -- decode enqueue and the host-buffer decode entry points: single-record
// decode (uniform + general walk), multi-record launches, the synchronous decode /
// checksum / stamp / admission entries and the device-resident decode APIs
//
// Part of the unity build of libiggy_codec.so: included by codec_api.hip, after the
// kernel translation units and the units before it (see codec_api.hip for the order).
#pragma once

namespace {



void prof_begin(iggy_codec_ctx *c, int which, hipStream_t s) {
    if (!c->profile) return;
    if (c->ev_pending[which]) {
        float ms = 0;
        if (hipEventSynchronize(c->ev1[which]) == hipSuccess &&
            hipEventElapsedTime(&ms, c->ev0[which], c->ev1[which]) == hipSuccess) {
            c->prof_ms[which] += ms;
            c->prof_n[which] += 1;
        }
        c->ev_pending[which] = false;
    }
    (void)hipEventRecord(c->ev0[which], s);
}
void prof_end(iggy_codec_ctx *c, int which, hipStream_t s) {
    if (!c->profile) return;
    (void)hipEventRecord(c->ev1[which], s);
    c->ev_pending[which] = true;
}

// launch the whole decode (uniform kernel + guarded general kernel)
// k_bsum_blocks grid: one wave per 1024-B block of the checksum input (44 + 8 N
// bytes, N <= max_frames), at most 4 WGs per CU; small inputs launch a small grid
static uint32_t bsum_grid(const iggy_codec_ctx *c, uint64_t max_frames) {
    const uint64_t blocks = (44 + 8 * max_frames) / 1024 + 1;
    return (uint32_t)std::min<uint64_t>((uint64_t)c->ncu * 4, (blocks + 3) / 4);
}

// k_decode_general after a first-pass kernel on stream s: it returns at once unless that
// kernel left d_res->status == kStatusNeedGeneral (ensure_decode_scratch done by the caller)
void launch_general(iggy_codec_ctx *c, const uint8_t *d_body, uint64_t len, int integrity, uint64_t *d_pos,
                    uint64_t cap, iggy_decode_result *d_res, hipStream_t s) {
    GeneralScratch gs = gscratch(c);
    const uint32_t ggrid = (uint32_t)std::min<uint64_t>((uint64_t)c->gen_grid, len / (64 << 10) + 2);
    if (integrity == IGGY_INTEGRITY_VERIFY)
        hipLaunchKernelGGL(k_decode_general<true>, dim3(ggrid), dim3(kGenThreads), kGenLds, s, d_body, len, d_pos,
                           cap, d_res, gs);
    else
        hipLaunchKernelGGL(k_decode_general<false>, dim3(ggrid), dim3(kGenThreads), 0, s, d_body, len, d_pos, cap,
                           d_res, gs);
}

int enqueue_decode(iggy_codec_ctx *c, const uint8_t *d_body, uint64_t len, int integrity,
                   uint64_t *d_pos, uint64_t cap, iggy_decode_result *d_res, hipStream_t s) {
    int r = ensure_decode_scratch(c, len);
    if (r) return r;
    if (++c->epoch > kEpochMask) {  // 24-bit tags: re-zero the block records before reusing one
        c->epoch = 1;
        HIP_OK(hipMemsetAsync(c->dsums.p, 0, c->dsums.cap, s));
    }
    const bool verify = integrity == IGGY_INTEGRITY_VERIFY;
    DecodeScratch ds = dscratch(c);
    // one persistent grid: one WG per CU, block 0 the consumer (chain) WG. Small
    // records get grids sized to their work (at most one producer WG per 128-frame
    // block of 48-B frames; one general WG per 64 KiB): dispatching two full
    // persistent grids dominated a 300-KB decode. Both kernels split their work
    // over whatever grid they get.
    const uint64_t ub_blocks = len / (48 * 128) + 2;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((uint64_t)c->ugrid, ub_blocks + 1);
    const uint32_t au = (uint32_t)c->allow_unaligned;
    prof_begin(c, 0, s);
    if (verify)
        hipLaunchKernelGGL(k_decode_uniform<true>, dim3(grid), dim3(kUniformThreads), kUniformLds, s, d_body, len, d_pos,
                           cap, d_res, ds, c->epoch, au, diag_bits(c));
    else
        hipLaunchKernelGGL(k_decode_uniform<false>, dim3(grid), dim3(kUniformThreads), kUniformLds, s, d_body, len, d_pos,
                           cap, d_res, ds, c->epoch, au, diag_bits(c));
    HIP_OK(hipGetLastError());
    launch_general(c, d_body, len, integrity, d_pos, cap, d_res, s);
    // the profiled interval is the whole decode: both kernels (the general one writes a
    // lane-group decode's frame positions, decode_uniform.hip kPosEpilogue)
    prof_end(c, 0, s);
    HIP_OK(hipGetLastError());
    return 0;
}

void fill_err(iggy_wire_error *err, const iggy_wire_error &e) {
    if (err) *err = e;
}
void set_err(iggy_wire_error *err, uint32_t kind, uint32_t reason = 0, uint64_t a = 0,
             uint64_t b = 0, uint64_t cc = 0) {
    if (!err) return;
    err->kind = kind;
    err->reason = reason;
    err->a = a;
    err->b = b;
    err->c = cc;
}

int reset_after_timeout(iggy_codec_ctx *c) {
    HIP_OK(hipStreamSynchronize(c->stream));
    HIP_OK(hipMemset(c->dsync.p, 0, kSyncBytes));
    return 0;
}

// synchronous decode of a host buffer; also used by stamp / checksum helpers
constexpr uint64_t kHostFastBytes = 16ull << 20;
#ifndef IGGY_ZERO_COPY_BYTES
#define IGGY_ZERO_COPY_BYTES (4ull << 20)  // (build knob for same-box A/B: 1 MiB measured slower)
#endif
constexpr uint64_t kZeroCopyBytes = IGGY_ZERO_COPY_BYTES;  // host inputs up to this size are read in place
#ifndef IGGY_POLL_IN_PLACE
#define IGGY_POLL_IN_PLACE 1  // (build knob for same-box A/B: poll bodies read in place)
#endif
int decode_host_fast(iggy_codec_ctx *c, const uint8_t *body, uint64_t len, int integrity,
                     iggy_decode_result *res_out, uint64_t *frame_pos, uint64_t cap, bool *done);
int decode_host(iggy_codec_ctx *c, const uint8_t *body, uint64_t len, int integrity,
                iggy_decode_result *res_out, uint64_t *frame_pos, uint64_t cap, bool keep_on_device) {
    bool done = false;
    int r = decode_host_fast(c, body, len, integrity, res_out, frame_pos, cap, &done);
    if (r || done) return r;
    r |= c->din.ensure(len + 16);
    const uint64_t pcap = frame_pos ? std::min<uint64_t>(cap, len / 48 + 1) : 0;
    r |= c->dpos.ensure((pcap + 1) * 8);
    if (r) return IGGY_ERR_DEVICE;
    r = put_host(c, c->din.p, body, len, c->stream);
    if (r) return r;
    iggy_decode_result *d_res = c->dresult.as<iggy_decode_result>();
    r = enqueue_decode(c, c->din.as<uint8_t>(), len, integrity, pcap ? c->dpos.as<uint64_t>() : nullptr,
                       pcap, d_res, c->stream);
    if (r) return r;
    iggy_decode_result *h_res = (iggy_decode_result *)c->h_pinned;
    HIP_OK(hipMemcpyAsync(h_res, d_res, sizeof(*h_res), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    *res_out = *h_res;
    if (res_out->error.kind == IGGY_ERR_TIMEOUT) reset_after_timeout(c);
    if (frame_pos && pcap && res_out->error.kind == IGGY_OK) {
        const uint64_t n = std::min<uint64_t>(res_out->frame_count, pcap);
        if (n) return get_host(c, frame_pos, c->dpos.p, n * 8, c->stream);
    }
    (void)keep_on_device;
    return 0;
}


// ------------------------------------------------------- multi-record decode
// The walks over a sequence of batches (disk chunk, segment recovery, transferred
// segment, poll body) decode every record in ONE launch of k_decode_records
// (decode_records.hip). The host plans the launch from its own copy of the bytes
// with the same stride speculation as make_plan: each single-stride record gets one
// workgroup per 128-frame checksum block; a record that is not single-stride (or
// is large enough to fill the chip on its own) takes the single-record path.
struct RecIn {
    uint64_t off, len;           // record start in the buffer, bytes available from there
    uint64_t pos_base, pos_cap;  // frame positions (device buffer passed to enqueue_records)
    uint64_t msg_base;           // polled messages (idem)
};
constexpr uint64_t kRecSingleBytes = 64ull << 20;  // larger records: the persistent single-record decode

// -> workgroups of record [h, h + len) in k_decode_records (>= 1), 0 = single-record path
uint64_t rec_plan(const uint8_t *h, uint64_t len, uint64_t *n_frames) {
    *n_frames = 0;
    if (len < kHdr) return 1;  // UnexpectedEof: resolved by the kernel from the header alone
    uint64_t bl;
    memcpy(&bl, h + 32, 8);
    if (bl < kHdr) return 1;
    for (uint32_t i = 52; i < kHdr; ++i)
        if (h[i]) return 1;
    if (len < bl) return 1;
    const uint64_t blob = bl - kHdr;
    if (blob == 0) return 1;
    uint64_t resv;
    if (blob < kFrameHdr) return 1;
    memcpy(&resv, h + kHdr + 40, 8);
    if (resv) return 1;
    uint32_t uh, pl;
    memcpy(&uh, h + kHdr + 32, 4);
    memcpy(&pl, h + kHdr + 36, 4);
    const uint64_t S = kFrameHdr + (uint64_t)uh + pl;
    if (S > blob) return 1;
    if (blob % S != 0 || S > (1u << 20) || bl > kRecSingleBytes) return 0;
    *n_frames = blob / S;
    return rec_blocks(blob / S);
}

// Enqueue the decode of K records of the device buffer d_base (h_base: the host
// copy of the same bytes) on the context's stream: one k_decode_records launch for
// every planned record, then the single-record decode of the others (appended to
// *single). d_res[k] receives record k's verdict (device or host-mapped memory when
// no record takes the single path); a record left with status kStatusNeedGeneral
// (its stride breaks mid-record) is re-decoded by redo_general. host_flag (device
// address of host-mapped memory, nullable): raised to flag_value when the launch is
// complete. n_frames[k] (nullable) = the planned frame count (0 for single-path
// records).
constexpr uint64_t kRecZeroCopyWgs = 4096;  // larger launches upload their tables (H2D)

int enqueue_records(iggy_codec_ctx *c, const uint8_t *d_base, const uint8_t *h_base, const RecIn *recs, size_t K,
                    int integrity, uint64_t *d_pos, iggy_polled_message *d_msgs, iggy_decode_result *d_res,
                    std::vector<size_t> *single, std::vector<uint64_t> *n_frames = nullptr,
                    uint32_t *host_flag = nullptr, uint32_t flag_value = 0, HostMap *tab = nullptr,
                    GenRearm rearm = GenRearm{nullptr, nullptr, nullptr}, Slot *own = nullptr) {
    // tab (nullable): host-mapped memory for the launch's task table that stays the
    // caller's until the launch completes (asynchronous submits); else the context's.
    // own (nullable): a fast-path slot whose stream and scratch the launch uses (no
    // context scratch: every record must plan, so nothing takes the single path)
    hipStream_t s = own ? own->st : c->stream;
    HostMap &rm = tab ? *tab : c->rmap;
    DevBuf &rbsums = own ? own->rbsums : c->rbsums;
    DevBuf &rstate = own ? own->rstate : c->rstate;
    DevBuf &rcount = own ? own->rcount : c->rcount;
    std::vector<RecTask> tasks(K);
    std::vector<uint32_t> wgmap;
    uint64_t nbs = 0, maxlen = 0;
    if (n_frames) n_frames->assign(K, 0);
    for (size_t k = 0; k < K; ++k) {
        uint64_t nf = 0;
        const uint64_t nw = rec_plan(h_base + recs[k].off, recs[k].len, &nf);
        RecTask &t = tasks[k];
        t.off = recs[k].off;
        t.len = recs[k].len;
        t.pos_base = recs[k].pos_base;
        t.pos_cap = d_pos ? recs[k].pos_cap : 0;
        t.msg_base = recs[k].msg_base;
        t.bsum_base = nbs;
        t.wg0 = (uint32_t)wgmap.size();
        t.nwg = (uint32_t)nw;
        if (!nw) {
            single->push_back(k);
            maxlen = std::max(maxlen, recs[k].len);
            continue;
        }
        if (n_frames) (*n_frames)[k] = nf;
        nbs += nw;
        wgmap.insert(wgmap.end(), nw, (uint32_t)k);
    }
    const uint64_t W = wgmap.size();
    if (W) {
        const size_t tb = K * sizeof(RecTask), wb = W * 4;
        int r = rm.ensure(tb + wb);
        r |= rbsums.ensure(nbs * 64 + 64);
        const size_t st_before = rstate.cap;
        r |= rstate.ensure(K * sizeof(RecState));
        if (!rcount.p) {
            r |= rcount.ensure(64);
            if (!r) HIP_OK(hipMemsetAsync(rcount.p, 0, rcount.cap, s));
        }
        if (r) return IGGY_ERR_DEVICE;
        if (rstate.cap != st_before)  // fresh state: zero (the resolvers keep it zero after)
            HIP_OK(hipMemsetAsync(rstate.p, 0, rstate.cap, s));
        memcpy(rm.hp<uint8_t>(), tasks.data(), tb);
        memcpy(rm.hp<uint8_t>(tb), wgmap.data(), wb);
        const RecTask *dt = rm.dp<RecTask>();
        const uint32_t *dw = rm.dp<uint32_t>(tb);
        const RecTask inl = tasks[0];
        if (K == 1) {  // one record: the task rides in the kernel arguments
            dt = nullptr;
            dw = nullptr;
        } else if (W > kRecZeroCopyWgs && !tab) {  // a big launch: every workgroup would read its task over PCIe
            r = c->rtab.ensure(tb + wb);
            if (r) return IGGY_ERR_DEVICE;
            HIP_OK(hipMemcpyAsync(c->rtab.p, rm.h, tb + wb, hipMemcpyHostToDevice, s));
            dt = c->rtab.as<RecTask>();
            dw = c->rtab.as<uint32_t>(tb);
        }
        RecState *ds = rstate.as<RecState>();
        uint32_t *flag = single->empty() ? host_flag : nullptr;
        if (integrity == IGGY_INTEGRITY_VERIFY)
            hipLaunchKernelGGL(k_decode_records<true>, dim3((uint32_t)W), dim3(kRecThreads), 0, s, d_base, dt, dw, ds,
                               rbsums.as<uint64_t>(), d_pos, d_msgs, d_res, rcount.as<uint32_t>(), flag,
                               flag_value, rearm, inl);
        else
            hipLaunchKernelGGL(k_decode_records<false>, dim3((uint32_t)W), dim3(kRecThreads), 0, s, d_base, dt, dw,
                               ds, rbsums.as<uint64_t>(), d_pos, d_msgs, d_res, rcount.as<uint32_t>(), flag,
                               flag_value, rearm, inl);
        HIP_OK(hipGetLastError());
    }
    if (!single->empty()) {
        if (own) return IGGY_ERR_DEVICE;  // (the caller planned every record)
        int r = ensure_decode_scratch(c, maxlen);
        if (r) return r;
        for (size_t k : *single) {
            r = enqueue_decode(c, d_base + recs[k].off, recs[k].len, integrity,
                               d_pos ? d_pos + recs[k].pos_base : nullptr, d_pos ? recs[k].pos_cap : 0, d_res + k, s);
            if (r) return r;
        }
    }
    return 0;
}

// true when every record goes to the multi-record kernel (the launch can raise the
// host flag: results straight into host-mapped memory, no copy, no stream sync)
bool records_all_planned(const uint8_t *h_base, const RecIn *recs, size_t K) {
    for (size_t k = 0; k < K; ++k) {
        uint64_t nf;
        if (!rec_plan(h_base + recs[k].off, recs[k].len, &nf)) return false;
    }
    return true;
}

// Wait for a kernel to raise the host-mapped completion flag (a spin: the host
// round trip of a stream sync or a result copy is what small host-buffer calls pay
// most for). If the stream drains without the flag, the launch failed.
// Bounded: a launch that neither raises the flag nor drains within kHostWaitLimit
// (the kernels' own spin guards are 4 s) returns IGGY_ERR_TIMEOUT to the caller's
// thread instead of holding it.
constexpr double kHostWaitLimitS = 10.0;
int wait_host_flag(iggy_codec_ctx *c, uint32_t v) {
    volatile uint32_t *flag = c->omap.hp<volatile uint32_t>();
    auto dbg = [&](const char *what, int rc) {
        if (getenv("IGGY_CODEC_DEBUG"))
            fprintf(stderr, "iggy_codec: wait_host_flag(%u): %s (flag %u)\n", v, what, *flag);
        return rc;
    };
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t i = 1;; ++i) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == v) return 0;
        if ((i & 1023) == 0) {
            const hipError_t q = hipStreamQuery(c->stream);
            if (q == hipSuccess) {
                // the stream drained: the flag store (system scope, over PCIe) may still be
                // in flight behind the completion signal for a moment; then it is final
                for (int k = 0; k < 100000; ++k) {
                    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == v) return 0;
                    __builtin_ia32_pause();
                }
                return dbg("stream drained without the flag", IGGY_ERR_DEVICE);
            }
            if (q != hipErrorNotReady) return dbg(hipGetErrorString(q), IGGY_ERR_DEVICE);
            if ((i & 0xfffff) == 0 &&
                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kHostWaitLimitS)
                return dbg("time limit", IGGY_ERR_TIMEOUT);
        }
        __builtin_ia32_pause();
    }
}
uint32_t next_flag(iggy_codec_ctx *c) {
    if (++c->hseq == 0) c->hseq = 1;
    return c->hseq;
}

// After the launch: records the multi-record kernel left with status
// kStatusNeedGeneral are decoded again by the single-record path (general walk, into
// the device results buffer) and res (host) is refreshed for them. Returns
// IGGY_ERR_TIMEOUT if a bug guard fired anywhere.
int redo_general(iggy_codec_ctx *c, const uint8_t *d_base, const RecIn *recs, size_t K, int integrity,
                 uint64_t *d_pos, iggy_decode_result *res, std::vector<size_t> *redone) {
    std::vector<size_t> redo;
    uint64_t maxlen = 0;
    for (size_t k = 0; k < K; ++k) {
        if (res[k].error.kind == IGGY_ERR_TIMEOUT) {
            reset_after_timeout(c);
            return IGGY_ERR_TIMEOUT;
        }
        if (res[k].status == kStatusNeedGeneral) {
            redo.push_back(k);
            maxlen = std::max(maxlen, recs[k].len);
        }
    }
    if (redo.empty()) return 0;
    int r = ensure_decode_scratch(c, maxlen);
    r |= c->rres.ensure(K * sizeof(iggy_decode_result));
    if (r) return r ? r : IGGY_ERR_DEVICE;
    iggy_decode_result *d_res = c->rres.as<iggy_decode_result>();
    for (size_t k : redo) {
        r = enqueue_decode(c, d_base + recs[k].off, recs[k].len, integrity, d_pos ? d_pos + recs[k].pos_base : nullptr,
                           d_pos ? recs[k].pos_cap : 0, d_res + k, c->stream);
        if (r) return r;
    }
    for (size_t k : redo) {
        r = get_host(c, res + k, d_res + k, sizeof(iggy_decode_result), c->stream);
        if (r) return r;
    }
    for (size_t k : redo)
        if (res[k].error.kind == IGGY_ERR_TIMEOUT) {
            reset_after_timeout(c);
            return IGGY_ERR_TIMEOUT;
        }
    if (redone) *redone = redo;
    return 0;
}

// Every record of the device buffer d_base decoded, the verdicts in res (host): one
// launch; when every record is planned for the multi-record kernel its results land
// in host-mapped memory and the host spins on the completion flag, otherwise device
// results, one copy and a stream sync; then the general re-walks, if any.
int decode_records_to_host(iggy_codec_ctx *c, const uint8_t *d_base, const uint8_t *h_base, const RecIn *recs,
                           size_t K, int integrity, iggy_decode_result *res) {
    std::vector<size_t> single;
    const size_t rb = K * sizeof(iggy_decode_result);
    if (records_all_planned(h_base, recs, K)) {
        if (c->omap.ensure(64 + rb)) return IGGY_ERR_DEVICE;
        const uint32_t v = next_flag(c);
        int r = enqueue_records(c, d_base, h_base, recs, K, integrity, nullptr, nullptr,
                                c->omap.dp<iggy_decode_result>(64), &single, nullptr, c->omap.dp<uint32_t>(), v);
        if (r) return r;
        r = wait_host_flag(c, v);
        if (!r) r = xfer_settle(c);
        if (r) return r;
        memcpy(res, c->omap.hp<uint8_t>(64), rb);
    } else {
        if (c->rres.ensure(rb)) return IGGY_ERR_DEVICE;
        iggy_decode_result *d_res = c->rres.as<iggy_decode_result>();
        int r = enqueue_records(c, d_base, h_base, recs, K, integrity, nullptr, nullptr, d_res, &single);
        if (!r) r = get_host(c, res, d_res, rb, c->stream);
        if (r) return r;
    }
    return redo_general(c, d_base, recs, K, integrity, nullptr, res, nullptr);
}

// ------------------------------------------------------- resident decode service
// (k_decode_service, decode_records.hip) A context with the service enabled posts a
// small single-stride record read in place (registered, or copied into the context's
// mapped staging) to the resident workgroups instead of launching a kernel per call.
SvcMailbox *svc_mb(iggy_codec_ctx *c) { return c->svc.mb.hp<SvcMailbox>(); }

// (re)launch the service kernel; start_seq: the last post it must not decode again
int svc_launch(iggy_codec_ctx *c, uint32_t start_seq) {
    auto &v = c->svc;
    if (v.launched) HIP_OK(hipStreamSynchronize(v.s));  // the previous grid has exited
    volatile SvcMailbox *mb = svc_mb(c);
    mb->stop = 0;
    mb->alive = 1;
    HIP_OK(hipMemsetAsync(v.ctl.p, 0, sizeof(SvcCtl), v.s));
    hipLaunchKernelGGL(k_decode_service, dim3(kSvcWgs), dim3(kRecThreads), 0, v.s, v.mb.dp<SvcMailbox>(), start_seq,
                       v.ctl.as<SvcCtl>(), v.st.as<RecState>(), v.bsums.as<uint64_t>());
    HIP_OK(hipGetLastError());
    v.launched = true;
    v.launches++;
    return 0;
}

int svc_enable(iggy_codec_ctx *c) {
    auto &v = c->svc;
    if (v.enabled) return 0;
    if (!v.s && hipStreamCreateWithFlags(&v.s, hipStreamNonBlocking) != hipSuccess) {
        v.s = nullptr;
        return IGGY_ERR_DEVICE;
    }
    int r = v.mb.ensure(sizeof(SvcMailbox));
    r |= v.ctl.ensure(sizeof(SvcCtl));
    const bool fresh = !v.st.p;
    r |= v.st.ensure(sizeof(RecState));
    r |= v.bsums.ensure(8 * 8 * (kSvcWgs + 1));
    if (r) return IGGY_ERR_DEVICE;
    if (fresh) HIP_OK(hipMemsetAsync(v.st.p, 0, v.st.cap, v.s));  // (the resolver keeps it zero after)
    memset(v.mb.h, 0, sizeof(SvcMailbox));
    v.seq = 0;
    v.enabled = true;
    return svc_launch(c, v.seq);
}

int svc_disable(iggy_codec_ctx *c) {
    auto &v = c->svc;
    if (!v.enabled) return 0;
    v.enabled = false;
    if (!v.launched) return 0;
    ((volatile SvcMailbox *)svc_mb(c))->stop = 1;
    v.launched = false;
    HIP_OK(hipStreamSynchronize(v.s));  // every workgroup has seen the stop word and exited
    return 0;
}

// Post one record to the service and wait for its completion flag (the same flag and
// host-mapped results as the launch path). A grid that exited idle is relaunched first;
// one that exits while the post is pending (it never relays a post it has not read) is
// relaunched to take it.
int svc_post_wait(iggy_codec_ctx *c, const uint8_t *d_base, const uint8_t *host_prefix, uint64_t len, int integrity,
                  uint32_t nwg, uint64_t pcap, uint32_t v) {
    auto &s = c->svc;
    volatile SvcMailbox *mb = svc_mb(c);
    if (!mb->alive && svc_launch(c, s.seq)) return IGGY_ERR_DEVICE;
    mb->integrity = (uint32_t)integrity;
    mb->nwg = nwg;
    mb->flag_value = v;
    mb->len = len;
    mb->pos_cap = pcap;
    mb->base = d_base;
    mb->frame_pos = pcap ? c->omap.dp<uint64_t>(192) : nullptr;  // (decode_host_fast passes 0)
    mb->result = c->omap.dp<iggy_decode_result>(64);
    mb->host_flag = c->omap.dp<uint32_t>();
    // the record's first 304 B (zero past its end), 12 B per tagged piece
    uint8_t pre[12 * kSvcPre] = {};
    memcpy(pre, host_prefix, std::min<uint64_t>(len, kHdr + kFrameHdr));
    for (uint32_t k = 0; k < kSvcPre; ++k) memcpy((void *)mb->pre[k].b, pre + 12 * k, 12);
    std::atomic_thread_fence(std::memory_order_release);
    // every chunk's tag after its words (x86 keeps stores in order): a device load round
    // that sees the new number in all 32 tagged chunks saw the whole post
    if (++s.seq == 0) ++s.seq;  // (0 is never a post: a zeroed relay unit carries it)
    const uint32_t seq = s.seq;
    for (uint32_t k = 0; k < kSvcPre; ++k) mb->pre[k].seq = seq;
    mb->seq0 = seq; mb->seq1 = seq; mb->seq2 = seq; mb->seq3 = seq; mb->seq4 = seq; mb->seq5 = seq;
    s.posts++;
    volatile uint32_t *flag = c->omap.hp<volatile uint32_t>();
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t i = 1;; ++i) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == v) {
            if (kDiagMask) {  // (diagnostic build: the device's part, 100 MHz ticks)
                s.dev_ticks[0] += mb->_r7[0];
                for (int k = 1; k < 8; ++k) s.dev_ticks[k] += mb->diag[k];
            }
            return 0;
        }
        if (!mb->alive) {
            HIP_OK(hipStreamSynchronize(s.s));  // the grid is gone; every store it made has landed
            if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) == v) return 0;
            if (svc_launch(c, s.seq - 1)) return IGGY_ERR_DEVICE;  // it sees this post as new
        }
        if ((i & 0xfffff) == 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > kHostWaitLimitS) {
            if (getenv("IGGY_CODEC_DEBUG")) fprintf(stderr, "iggy_codec: service post %u: time limit\n", s.seq);
            return IGGY_ERR_TIMEOUT;
        }
        __builtin_ia32_pause();
    }
}

// A small single-stride record from host memory (iggy_codec_decode_batch and the
// host entry points built on it): one H2D copy and ONE k_decode_records launch that
// writes the verdict and the frame positions straight into host-mapped memory, the
// host spinning on its completion flag -- two stream operations instead of the
// persistent pair's five (H2D, two kernels, two copies back, a sync). *done = false
// leaves the record to the persistent path (not single-stride, too large, or the
// stride broke mid-record).
int decode_host_fast(iggy_codec_ctx *c, const uint8_t *body, uint64_t len, int integrity,
                     iggy_decode_result *res_out, uint64_t *frame_pos, uint64_t cap, bool *done) {
    *done = false;
    uint64_t nf = 0;
    if (len > kHostFastBytes || !rec_plan(body, len, &nf)) return 0;
    // (diagnostic build, IGGY_CODEC_TIMING=N: mean stage times of the next N calls)
    static int timing = kDiagMask && getenv("IGGY_CODEC_TIMING") ? atoi(getenv("IGGY_CODEC_TIMING")) : 0;
    static double tsum[4] = {0, 0, 0, 0};
    static int tn = 0;
    using tclk = std::chrono::steady_clock;
    const auto tt0 = tclk::now();
    auto tmark = [&](int k) {
        if (timing) tsum[k] += std::chrono::duration<double, std::micro>(tclk::now() - tt0).count();
    };
    const uint64_t pcap = frame_pos ? std::min<uint64_t>(cap, len / 48 + 1) : 0;
    if (c->omap.ensure(64 + 128 + pcap * 8)) return IGGY_ERR_DEVICE;
    // a registered (page-locked, device-mapped) record of at most kZeroCopyBytes is read
    // by the kernel in place over the host link: no H2D, one launch and the flag
    const uint8_t *d_base = nullptr;
    if (len <= kZeroCopyBytes) d_base = host_device_ptr(body, len);
    int r = 0;
    if (!d_base && len <= kZeroCopyBytes && !host_pinned(body, len)) {
        // pageable: into the context's own mapped staging, read in place (the previous
        // fast call's kernel is done: every synchronous entry waits for its flag)
        if (c->zin.ensure(len + 16)) return IGGY_ERR_DEVICE;
        memcpy(c->zin.h, body, len);
        d_base = c->zin.d;
    }
    if (!d_base) {
        if (c->din.ensure(len + 16)) return IGGY_ERR_DEVICE;
        r = put_host(c, c->din.p, body, len, c->stream);
        if (r) return r;
        d_base = c->din.as<uint8_t>();
    }
    tmark(0);
    const RecIn rec{0, len, 0, pcap, 0};
    std::vector<size_t> single;
    const uint32_t v = next_flag(c);
    const uint64_t nwg = rec_blocks(nf);
    bool svc_pos = false;
    if (c->svc.enabled && nf && nwg <= kSvcWgs && len <= kZeroCopyBytes) {
        // the resident service: no launch (d_base is host memory the device reads in place)
        // No positions from the device: a record the service decodes is single-stride
        // (every frame's header was checked against the stride S), so its positions are
        // i * S, written below from the verdict -- no blocks fencing 8 KB of host-mapped
        // stores before they hand over, no copy of them back out of the mapped buffer.
        tmark(1);
        r = svc_post_wait(c, d_base, body, len, integrity, (uint32_t)nwg, 0, v);
        svc_pos = true;
    } else {
        r = enqueue_records(c, d_base, body, &rec, 1, integrity,
                            pcap ? c->omap.dp<uint64_t>(192) : nullptr, nullptr, c->omap.dp<iggy_decode_result>(64),
                            &single, nullptr, c->omap.dp<uint32_t>(), v);
        if (r) return r;
        tmark(1);
        r = wait_host_flag(c, v);
    }
    if (!r) r = xfer_settle(c);
    if (r) return r;
    tmark(2);
    const iggy_decode_result res = *c->omap.hp<iggy_decode_result>(64);
    if (res.status == kStatusNeedGeneral) return 0;
    *res_out = res;
    if (frame_pos && pcap && res.error.kind == IGGY_OK) {
        const uint64_t n = std::min<uint64_t>(res.frame_count, pcap);
        if (svc_pos) {
            const uint64_t S = res.frame_count ? (res.header.batch_length - kHdr) / res.frame_count : 0;
            for (uint64_t i = 0; i < n; ++i) frame_pos[i] = i * S;
        } else {
            memcpy(frame_pos, c->omap.hp<uint64_t>(192), n * 8);
        }
    }
    *done = true;
    tmark(3);
    if (timing && ++tn == timing) {
        fprintf(stderr, "iggy_codec timing (%d calls, us from entry): staged %.2f launched %.2f flag %.2f done %.2f"
                " service-device %.2f (block entry %.2f hashed %.2f resolver %.2f computed %.2f result %.2f"
                " followers entered (max) %.2f followers hashed (max) %.2f)\n",
                tn, tsum[0] / tn, tsum[1] / tn, tsum[2] / tn, tsum[3] / tn, c->svc.dev_ticks[0] * 0.01 / tn,
                c->svc.dev_ticks[1] * 0.01 / tn, c->svc.dev_ticks[2] * 0.01 / tn, c->svc.dev_ticks[3] * 0.01 / tn,
                c->svc.dev_ticks[4] * 0.01 / tn, c->svc.dev_ticks[5] * 0.01 / tn, c->svc.dev_ticks[6] * 0.01 / tn,
                c->svc.dev_ticks[7] * 0.01 / tn);
        for (auto &x : c->svc.dev_ticks) x = 0;
        tn = 0;
        tsum[0] = tsum[1] = tsum[2] = tsum[3] = 0;
    }
    return 0;
}

}  // namespace

extern "C" {

// ------------------------------------------------------------ synchronous
int iggy_codec_decode_batch(iggy_codec_ctx *c, const uint8_t *body, uint64_t len, int integrity,
                            iggy_batch_header *hdr, uint64_t *frame_pos, uint64_t cap,
                            uint64_t *nframes, iggy_wire_error *err) {
    if (!c || (!body && len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    iggy_decode_result res;
    int r = decode_host(c, body, len, integrity, &res, frame_pos, cap, false);
    if (r) return r;
    fill_err(err, res.error);
    if (hdr) *hdr = res.header;
    if (nframes) *nframes = res.frame_count;
    if (res.error.kind != IGGY_OK) return (int)res.error.kind;
    if (frame_pos && res.frame_count > cap) {
        set_err(err, IGGY_ERR_CAPACITY, 0, res.frame_count, cap);
        return IGGY_ERR_CAPACITY;
    }
    return 0;
}

// Stage [256-B header built from *h][blob] in the context's input buffer: two
// copies straight from the caller's memory (no host-side concatenation).
static int stage_record(iggy_codec_ctx *c, const iggy_batch_header &h, const uint8_t *blob, uint64_t blob_len) {
    if (c->din.ensure(256 + blob_len + 16)) return IGGY_ERR_DEVICE;
    uint8_t *hb = (uint8_t *)c->h_pinned + 2048;  // pinned: the copy is truly async
    iggy_batch_header_encode(&h, hb);
    HIP_OK(hipMemcpyAsync(c->din.p, hb, 256, hipMemcpyHostToDevice, c->stream));
    return put_host(c, c->din.as<uint8_t>(256), blob, blob_len, c->stream);
}

int iggy_codec_verify_and_recompute_batch_checksum(iggy_codec_ctx *c, const iggy_batch_header *hdr,
                                                   const uint8_t *blob, uint64_t blob_len,
                                                   uint64_t *out, iggy_wire_error *err) {
    if (!c || !hdr || (!blob && blob_len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    // the BatchRef's header fields as given; batch_length is the record's own
    // (256 + blob), as for every BatchRef a decode hands out (batch.rs:391-406)
    iggy_batch_header h = *hdr;
    h.batch_length = 256 + blob_len;
    int r = stage_record(c, h, blob, blob_len);
    if (r) return r;
    iggy_decode_result *d_res = c->dresult.as<iggy_decode_result>();
    r = enqueue_decode(c, c->din.as<uint8_t>(), 256 + blob_len, IGGY_INTEGRITY_VERIFY, nullptr, 0, d_res, c->stream);
    if (r) return r;
    iggy_decode_result *h_res = (iggy_decode_result *)c->h_pinned;
    HIP_OK(hipMemcpyAsync(h_res, d_res, sizeof(*h_res), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    const iggy_decode_result res = *h_res;
    if (res.error.kind == IGGY_ERR_TIMEOUT) reset_after_timeout(c);
    // the stored batch checksum is the caller's business here (batch.rs:474-506)
    if (res.error.kind == IGGY_ERR_INVALID_BATCH_CHECKSUM || res.error.kind == IGGY_OK) {
        if (out) *out = res.computed_checksum;
        set_err(err, IGGY_OK);
        return 0;
    }
    fill_err(err, res.error);
    return (int)res.error.kind;
}

static int checksum_of_walk(iggy_codec_ctx *c, const iggy_batch_header *hdr, uint64_t nframes,
                            const uint8_t *d_blob, const uint64_t *d_pos, uint64_t *d_out, hipStream_t s) {
    // header fields and frame count travel as kernel arguments (no host copy)
    iggy_batch_header *dh = c->dresult.as<iggy_batch_header>(2048);
    uint64_t *d_n = c->dresult.as<uint64_t>(3096);
    hipLaunchKernelGGL(k_put_header, dim3(1), dim3(64), 0, s, *hdr, nframes, (const uint64_t *)nullptr, dh, d_n);
    CsSource src{nullptr, d_blob, d_pos};
    hipLaunchKernelGGL(k_bsum_blocks, dim3(bsum_grid(c, nframes)), dim3(256), 0, s, dh, d_n, src,
                       c->gbsums.as<uint64_t>(), nullptr);
    hipLaunchKernelGGL(k_bsum_chain, dim3(1), dim3(128), 0, s, dh, d_n, src,
                       (const uint64_t *)c->gbsums.as<uint64_t>(), c->dsync.as<uint8_t>(kSyncSmall), d_out,
                       nullptr);
    HIP_OK(hipGetLastError());
    return 0;
}

// The frames BatchIteratorWithOffsets yields over the staged record (a LayoutOnly
// decode: its frame_count is the walk's, whatever error ends it) and the batch
// checksum over them with header fields *hdr, all in one enqueue.
static int enqueue_checksum_of_staged(iggy_codec_ctx *c, const iggy_batch_header &hdr, uint64_t blob_len,
                                      uint64_t *d_out) {
    const uint64_t cap = blob_len / 48 + 1;
    int r = c->dpos.ensure((cap + 1) * 8);
    r |= c->gbsums.ensure(((44 + 8 * cap) / 1024 + 2) * 64);
    if (r) return IGGY_ERR_DEVICE;
    iggy_decode_result *d_res = c->dresult.as<iggy_decode_result>();
    r = enqueue_decode(c, c->din.as<uint8_t>(), 256 + blob_len, IGGY_INTEGRITY_LAYOUT_ONLY, c->dpos.as<uint64_t>(),
                       cap, d_res, c->stream);
    if (r) return r;
    iggy_batch_header *dh = c->dresult.as<iggy_batch_header>(2048);
    uint64_t *d_n = c->dresult.as<uint64_t>(3096);
    hipLaunchKernelGGL(k_put_header, dim3(1), dim3(64), 0, c->stream, hdr, (uint64_t)0,
                       (const uint64_t *)&d_res->frame_count, dh, d_n);
    CsSource src{nullptr, c->din.as<uint8_t>(256), c->dpos.as<uint64_t>()};
    hipLaunchKernelGGL(k_bsum_blocks, dim3(bsum_grid(c, cap)), dim3(256), 0, c->stream, dh, d_n, src,
                       c->gbsums.as<uint64_t>(), nullptr);
    hipLaunchKernelGGL(k_bsum_chain, dim3(1), dim3(128), 0, c->stream, dh, d_n, src,
                       (const uint64_t *)c->gbsums.as<uint64_t>(), c->dsync.as<uint8_t>(kSyncSmall), d_out, nullptr);
    HIP_OK(hipGetLastError());
    return 0;
}

int iggy_codec_calculate_batch_checksum(iggy_codec_ctx *c, const iggy_batch_header *hdr,
                                        const uint8_t *blob, uint64_t blob_len, uint64_t *out) {
    if (!c || !hdr || !out || (!blob && blob_len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    // the walk sees a header of this blob's length and no message count (only the
    // frames matter); the checksum hashes the caller's header fields
    iggy_batch_header h = *hdr;
    h.batch_length = 256 + blob_len;
    h.message_count = 0;
    h.batch_checksum = 0;
    int r = stage_record(c, h, blob, blob_len);
    if (r) return r;
    uint64_t *d_out = c->dresult.as<uint64_t>(3080);
    r = enqueue_checksum_of_staged(c, *hdr, blob_len, d_out);
    if (r) return r;
    uint64_t *h_out = (uint64_t *)((uint8_t *)c->h_pinned + 1536);
    HIP_OK(hipMemcpyAsync(h_out, d_out, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    *out = *h_out;
    return 0;
}

int iggy_codec_stamp_batch(iggy_codec_ctx *c, uint8_t *batch, uint64_t len, uint64_t base_offset,
                           uint64_t base_timestamp, iggy_batch_header *out, iggy_wire_error *err) {
    if (!c || (!batch && len)) return IGGY_ERR_INVALID_ARGUMENT;
    iggy_batch_header h;
    int r = iggy_batch_header_decode(batch, len, &h, err);
    if (r) return r;
    if (len < h.batch_length) {
        set_err(err, IGGY_ERR_UNEXPECTED_EOF, 0, 0, h.batch_length, len);
        return IGGY_ERR_UNEXPECTED_EOF;
    }
    h.base_offset = base_offset;
    h.base_timestamp = base_timestamp;
    uint64_t cs = 0;
    r = iggy_codec_calculate_batch_checksum(c, &h, batch + 256, h.batch_length - 256, &cs);
    if (r) return r;
    h.batch_checksum = cs;
    uint8_t hb[256];
    iggy_batch_header_encode(&h, hb);
    memcpy(batch, hb, 256);
    if (out) *out = h;
    set_err(err, IGGY_OK);
    return 0;
}

// batch_error (server_common/src/send_messages.rs:52-66): integrity errors keep
// their payloads, every other wire error becomes InvalidCommand
static int server_error(int rc, iggy_wire_error *err) {
    if (rc == IGGY_OK || rc == IGGY_ERR_INVALID_BATCH_CHECKSUM || rc == IGGY_ERR_INVALID_MESSAGE_CHECKSUM ||
        rc >= IGGY_ERR_DEVICE)
        return rc;
    set_err(err, IGGY_ERR_INVALID_COMMAND);
    return IGGY_ERR_INVALID_COMMAND;
}

// decode_prepare_slice_inner (server_common/src/send_messages.rs:581-622): the
// structural checks on the host, the per-message + batch checksum pass on the GPU
int iggy_codec_decode_prepare(iggy_codec_ctx *c, const uint8_t *frame, uint64_t len, int validate,
                              iggy_batch_header *hdr_out, iggy_wire_error *err) {
    if (!c || (!frame && len)) return IGGY_ERR_INVALID_ARGUMENT;
    set_err(err, IGGY_OK);
    const uint64_t hs = IGGY_PREPARE_HEADER_SIZE;
    if (len < hs) return server_error(IGGY_ERR_VALIDATION, err);
    uint32_t total = 0;
    memcpy(&total, frame + IGGY_PREPARE_SIZE_OFFSET, 4);
    if (total < hs || len < total) return server_error(IGGY_ERR_VALIDATION, err);
    const uint8_t *body = frame + hs;
    const uint64_t body_len = total - hs;
    if (body_len < 256) return server_error(IGGY_ERR_VALIDATION, err);
    iggy_batch_header h;
    int r = iggy_batch_header_decode(body, 256, &h, err);
    if (r) return server_error(r, err);
    if (body_len != h.batch_length) return server_error(IGGY_ERR_VALIDATION, err);
    if (hdr_out) *hdr_out = h;
    if (!validate) return 0;
    r = iggy_codec_decode_batch(c, body, body_len, IGGY_INTEGRITY_VERIFY, nullptr, nullptr, 0, nullptr, err);
    return server_error(r, err);
}

// admit_wire_request after SendMessagesMetadata::decode
// (server_common/src/send_messages.rs:505-540)
int iggy_codec_admit_batch(iggy_codec_ctx *c, const uint8_t *batch, uint64_t len,
                           uint32_t metadata_messages_count, uint64_t partition_id, int checksum_mode,
                           uint8_t *out, uint64_t cap, iggy_batch_header *hdr_out, iggy_wire_error *err) {
    if (!c || (!batch && len) || !out) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    set_err(err, IGGY_OK);
    // one H2D copy and one Verify decode (positions kept on the device); the stamped
    // header's checksum (send_messages.rs:529-537) is computed from those positions in
    // the same enqueue, before the host has seen the verdict (discarded on failure)
    const uint64_t pcap = len / 48 + 1;
    int r = c->din.ensure(len + 16);
    r |= c->dpos.ensure((pcap + 1) * 8);
    r |= c->gbsums.ensure(((44 + 8 * pcap) / 1024 + 2) * 64);
    if (r) return IGGY_ERR_DEVICE;
    r = put_host(c, c->din.p, batch, len, c->stream);
    if (r) return r;
    iggy_decode_result *d_res = c->dresult.as<iggy_decode_result>();
    r = enqueue_decode(c, c->din.as<uint8_t>(), len, IGGY_INTEGRITY_VERIFY, c->dpos.as<uint64_t>(), pcap, d_res,
                       c->stream);
    if (r) return r;
    uint64_t *d_cs = c->dresult.as<uint64_t>(3080);
    const bool compute = checksum_mode == IGGY_CHECKSUM_COMPUTE;
    if (compute) {
        iggy_batch_header *dh = c->dresult.as<iggy_batch_header>(2048);
        uint64_t *d_n = c->dresult.as<uint64_t>(3096);
        hipLaunchKernelGGL(k_admit_header, dim3(1), dim3(64), 0, c->stream, (const iggy_decode_result *)d_res,
                           partition_id, dh, d_n);
        CsSource src{nullptr, c->din.as<uint8_t>(256), c->dpos.as<uint64_t>()};
        hipLaunchKernelGGL(k_bsum_blocks, dim3(bsum_grid(c, pcap)), dim3(256), 0, c->stream, dh, d_n, src,
                           c->gbsums.as<uint64_t>(), nullptr);
        hipLaunchKernelGGL(k_bsum_chain, dim3(1), dim3(128), 0, c->stream, dh, d_n, src,
                           (const uint64_t *)c->gbsums.as<uint64_t>(), c->dsync.as<uint8_t>(kSyncSmall), d_cs,
                           nullptr);
        HIP_OK(hipGetLastError());
    }
    iggy_decode_result *h_res = (iggy_decode_result *)c->h_pinned;
    uint64_t *h_cs = (uint64_t *)((uint8_t *)c->h_pinned + 1536);
    HIP_OK(hipMemcpyAsync(h_res, d_res, sizeof(*h_res), hipMemcpyDeviceToHost, c->stream));
    if (compute) HIP_OK(hipMemcpyAsync(h_cs, d_cs, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    const iggy_decode_result res = *h_res;
    if (res.error.kind == IGGY_ERR_TIMEOUT) reset_after_timeout(c);
    if (res.error.kind != IGGY_OK) {
        fill_err(err, res.error);
        return server_error((int)res.error.kind, err);
    }
    iggy_batch_header h = res.header;
    if (h.message_count == 0 || h.message_count != metadata_messages_count || len != h.batch_length) {
        set_err(err, IGGY_ERR_INVALID_COMMAND);
        return IGGY_ERR_INVALID_COMMAND;
    }
    if (cap < len) {
        set_err(err, IGGY_ERR_CAPACITY, 0, len);
        return IGGY_ERR_CAPACITY;
    }
    memcpy(out, batch, len);
    h.partition_id = partition_id;
    h.batch_checksum = compute ? *h_cs : 0;
    uint8_t hb[256];
    iggy_batch_header_encode(&h, hb);
    memcpy(out, hb, 256);
    if (hdr_out) *hdr_out = h;
    set_err(err, IGGY_OK);
    return 0;
}

int iggy_codec_decode_records(iggy_codec_ctx *c, const uint8_t *buf, uint64_t len, const uint64_t *offsets,
                              uint64_t nrec, int integrity, iggy_decode_result *out) {
    if (!c || (!buf && len) || (nrec && (!offsets || !out))) return IGGY_ERR_INVALID_ARGUMENT;
    if (integrity != IGGY_INTEGRITY_VERIFY && integrity != IGGY_INTEGRITY_LAYOUT_ONLY) return IGGY_ERR_INVALID_ARGUMENT;
    for (uint64_t k = 0; k < nrec; ++k)
        if (offsets[k] > len) return IGGY_ERR_INVALID_ARGUMENT;
    if (!nrec) return 0;
    DevGuard dg(c->device);
    bind(c, nullptr);
    if (c->din.ensure(len + 16)) return IGGY_ERR_DEVICE;
    int r = put_host(c, c->din.p, buf, len, c->stream);
    if (r) return r;
    std::vector<RecIn> recs(nrec);
    for (uint64_t k = 0; k < nrec; ++k) recs[k] = RecIn{offsets[k], len - offsets[k], 0, 0, 0};
    return decode_records_to_host(c, c->din.as<uint8_t>(), buf, recs.data(), nrec, integrity, out);
}


int iggy_codec_xxh3_64(iggy_codec_ctx *c, const void *data, uint64_t len, uint64_t *out) {
    if (!c || !out || (!data && len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    int r = c->din.ensure(len + 16);
    const uint64_t nb = len ? (len - 1) / 1024 + 1 : 1;
    r |= c->hbsums.ensure(nb * 64 + 64);
    if (r) return IGGY_ERR_DEVICE;
    r = put_host(c, c->din.p, data, len, c->stream);
    if (r) return r;
    uint64_t *dout = c->dresult.as<uint64_t>(3088);
    if (len > 240)
        hipLaunchKernelGGL(k_xxh3_big_blocks, dim3(c->ncu * 4), dim3(256), 0, c->stream,
                           c->din.as<uint8_t>(), len, c->hbsums.as<uint64_t>());
    hipLaunchKernelGGL(k_xxh3_big_chain, dim3(1), dim3(64), 0, c->stream, c->din.as<uint8_t>(), len,
                       (const uint64_t *)c->hbsums.as<uint64_t>(), dout);
    HIP_OK(hipGetLastError());
    return get_host(c, out, dout, 8, c->stream);
}


// ------------------------------------------------------------ device APIs
int iggy_codec_decode_batch_device(iggy_codec_ctx *c, const uint8_t *d_body, uint64_t len,
                                   int integrity, uint64_t *d_frame_pos, uint64_t cap,
                                   iggy_decode_result *d_result, void *stream) {
    if (!c || !d_result || (!d_body && len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    return enqueue_decode(c, d_body, len, integrity, d_frame_pos, d_frame_pos ? cap : 0, d_result,
                          bind(c, stream));
}

int iggy_codec_batch_checksum_device(iggy_codec_ctx *c, const iggy_batch_header *hdr,
                                     const uint8_t *d_blob, const uint64_t *d_frame_pos,
                                     uint64_t nframes, uint64_t *d_out, void *stream) {
    if (!c || !hdr || !d_out || (nframes && (!d_blob || !d_frame_pos))) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    hipStream_t s = bind(c, stream);
    int r = c->gbsums.ensure(((44 + 8 * nframes) / 1024 + 2) * 64);
    if (r) return r;
    return checksum_of_walk(c, hdr, nframes, d_blob, d_frame_pos, d_out, s);
}

int iggy_codec_xxh3_64_ranges_device(iggy_codec_ctx *c, const uint8_t *d_data, const uint64_t *d_offsets,
                                     const uint32_t *d_lengths, uint64_t n, uint64_t *d_out,
                                     void *stream) {
    if (!c || !d_out || (n && (!d_data || !d_offsets || !d_lengths))) return IGGY_ERR_INVALID_ARGUMENT;
    if (!n) return 0;
    DevGuard dg(c->device);
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, (uint64_t)c->ncu * 16);
    hipLaunchKernelGGL(k_xxh3_ranges, dim3((uint32_t)blocks), dim3(256), 0, bind(c, stream), d_data,
                       d_offsets, d_lengths, n, d_out);
    HIP_OK(hipGetLastError());
    return 0;
}

}  // extern "C"
