// host_async.hpp -- asynchronous host-buffer operations: slots, submit / poll / wait
//
// Part of the unity build of libiggy_codec.so: included by codec_api.hip, after the
// kernel translation units and the units before it (see codec_api.hip for the order).
#pragma once

extern "C" {

// ------------------------------------------------ asynchronous host buffers
// Shard threads have no blocking pool (server_common/src/executor.rs:80-88): a
// host-buffer decode/encode is submitted (async H2D into a device slot on the copy-in
// stream, the kernels on the context's stream, results and outputs back on the
// copy-out stream) and its ticket polled from the reactor. Kernels only ever read
// device memory; a caller buffer registered with iggy_codec_host_register is copied
// at link speed without a bounce.
namespace {
int async_init(iggy_codec_ctx *c) {
    if (c->h2d) return 0;
    if (hipStreamCreateWithFlags(&c->h2d, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->d2h, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc(&c->slot_pinned, kSlots * 256, hipHostMallocDefault) != hipSuccess)
        return IGGY_ERR_DEVICE;
    {
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, c->slot_pinned, 0) != hipSuccess) {
            (void)hipGetLastError();
            dp = nullptr;
        }
        c->slot_pinned_d = (uint8_t *)dp;
    }
    for (Slot &sl : c->slots)
        if (hipEventCreateWithFlags(&sl.ev_in, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&sl.ev_k, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&sl.ev_done, hipEventDisableTiming) != hipSuccess)
            return IGGY_ERR_DEVICE;
    return 0;
}
int take_slot(iggy_codec_ctx *c, uint32_t op, int *idx) {
    int r = async_init(c);
    if (r) return r;
    for (int k = 0; k < kSlots; ++k)
        if (!c->slots[k].busy) {
            Slot &sl = c->slots[k];
            sl.busy = true;
            sl.op = op;
            sl.ticket = (++c->seq << 4) | (uint64_t)k;
            *idx = k;
            return 0;
        }
    return IGGY_ERR_BUSY;
}
}  // namespace


int iggy_codec_decode_submit(iggy_codec_ctx *c, const uint8_t *body, uint64_t len, int integrity,
                             uint64_t *frame_pos, uint64_t cap, iggy_ticket *ticket) {
    if (!c || !ticket || (!body && len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    int k = 0;
    int r = take_slot(c, IGGY_OP_DECODE, &k);
    if (r) return r;
    Slot &sl = c->slots[k];
    const uint64_t pcap = frame_pos ? std::min<uint64_t>(cap, len / 48 + 1) : 0;
    r = sl.in.ensure(len + 16);
    r |= sl.pos.ensure((pcap + 1) * 8);
    r |= sl.res.ensure(256);
    if (!r) r = ensure_decode_scratch(c, len);
    if (r) {
        sl.busy = false;
        return IGGY_ERR_DEVICE;
    }
    sl.cap = cap;
    sl.frame_pos = frame_pos;
    sl.hout_dst = nullptr;
    sl.hout_len = 0;
    const bool pos_pinned = host_pinned(frame_pos, pcap * 8);
    if (pcap && !pos_pinned && sl.hout_ensure(pcap * 8)) r = IGGY_ERR_DEVICE;
    uint64_t nf = 0;
    if (!r && c->slot_pinned_d && len <= kHostFastBytes && rec_plan(body, len, &nf)) {
        // a single-stride record of <= 16 MiB, on the slot's own stream with the slot's
        // own k_decode_records scratch (so the slots' launches overlap): the input
        // (read in place when <= kZeroCopyBytes, else copied), one launch whose verdict
        // lands in the slot's host-mapped completion record, the positions back, the
        // completion event; k_decode_general, for a stride that breaks mid-record, is
        // started by iggy_codec_poll on the context's stream
        if (!sl.st && hipStreamCreateWithFlags(&sl.st, hipStreamNonBlocking) != hipSuccess) {
            sl.st = nullptr;
            sl.busy = false;
            return IGGY_ERR_DEVICE;
        }
        hipStream_t s = sl.st;
        const uint8_t *d_in = len <= kZeroCopyBytes ? host_device_ptr(body, len) : nullptr;
        if (!d_in && !host_pinned(body, len)) {
            // pageable: copied into the slot's own pinned staging now (the caller's bytes
            // are free when submit returns), then read in place or DMA'd from there; the
            // slot holds the staging until the ticket completes, so nothing here waits
            if (sl.zin.ensure(len + 16)) {
                r = IGGY_ERR_DEVICE;
            } else {
                memcpy(sl.zin.h, body, len);
                if (len <= kZeroCopyBytes) {
                    d_in = sl.zin.d;
                } else {
                    if (hipMemcpyAsync(sl.in.p, sl.zin.h, len, hipMemcpyHostToDevice, s) != hipSuccess)
                        r = IGGY_ERR_DEVICE;
                    d_in = sl.in.as<uint8_t>();
                }
            }
        }
        if (!d_in && !r) {  // pinned caller memory above kZeroCopyBytes: one DMA, no wait
            r = put_host(c, sl.in.p, body, len, s);
            d_in = sl.in.as<uint8_t>();
        }
        iggy_decode_result *d_res = (iggy_decode_result *)(c->slot_pinned_d + 256 * k);
        // positions straight into host memory the device can write: the caller's pinned
        // array, else the slot's pinned bounce (copied out in iggy_codec_poll); a device
        // buffer and a D2H copy only when neither is mapped
        uint64_t *d_pos = nullptr;
        bool pos_copy = false;
        if (pcap) {
            if (pos_pinned) d_pos = (uint64_t *)host_device_ptr(frame_pos, pcap * 8);
            if (!d_pos && !pos_pinned) {
                void *dp = nullptr;
                if (hipHostGetDevicePointer(&dp, sl.hout, 0) == hipSuccess && dp) d_pos = (uint64_t *)dp;
                else (void)hipGetLastError();
                if (d_pos) sl.hout_dst = (uint8_t *)frame_pos;
            }
            if (!d_pos) {
                d_pos = sl.pos.as<uint64_t>();
                pos_copy = true;
            }
        }
        std::vector<size_t> single;
        const RecIn rec{0, len, 0, pcap, 0};
        if (!r) {
            // a stride break mid-record is left to iggy_codec_poll (k_decode_general)
            r = enqueue_records(c, d_in, body, &rec, 1, integrity, d_pos, nullptr, d_res, &single, nullptr, nullptr,
                                0, &sl.tab, GenRearm{nullptr, nullptr, nullptr}, &sl);
        }
        if (!r && hipGetLastError() != hipSuccess) r = IGGY_ERR_DEVICE;
        if (!r && pos_copy) {
            if (!pos_pinned) sl.hout_dst = (uint8_t *)frame_pos;
            if (hipMemcpyAsync(pos_pinned ? (void *)frame_pos : sl.hout, sl.pos.p, pcap * 8, hipMemcpyDeviceToHost,
                               s) != hipSuccess)
                r = IGGY_ERR_DEVICE;
        }
        sl.fast = true;
        sl.g_pending = false;
        sl.g_in = d_in;
        sl.g_len = len;
        sl.g_pcap = pcap;
        sl.g_pos = d_pos;
        sl.g_integ = integrity;
        sl.g_pos_copy = pos_copy;
        if (!r && hipEventRecord(sl.ev_done, s) != hipSuccess) r = IGGY_ERR_DEVICE;
        if (r) {
            sl.busy = false;
            return r;
        }
        *ticket = sl.ticket;
        return 0;
    }
    sl.fast = false;
    if (!r) r = put_host(c, sl.in.p, body, len, c->h2d);
    if (r) {
        sl.busy = false;
        return r;
    }
    HIP_OK(hipEventRecord(sl.ev_in, c->h2d));
    hipStream_t s = bind(c, nullptr);
    HIP_OK(hipStreamWaitEvent(s, sl.ev_in, 0));
    iggy_decode_result *d_res = sl.res.as<iggy_decode_result>();
    r = enqueue_decode(c, sl.in.as<uint8_t>(), len, integrity, pcap ? sl.pos.as<uint64_t>() : nullptr, pcap, d_res, s);
    if (r) {
        sl.busy = false;
        return r;
    }
    HIP_OK(hipEventRecord(sl.ev_k, s));
    HIP_OK(hipStreamWaitEvent(c->d2h, sl.ev_k, 0));
    HIP_OK(hipMemcpyAsync((uint8_t *)c->slot_pinned + 256 * k, d_res, sizeof(iggy_decode_result),
                          hipMemcpyDeviceToHost, c->d2h));
    // positions: straight into pinned caller memory; a pageable array gets them from the
    // slot's pinned bounce in iggy_codec_poll (and only when the decode succeeded)
    if (pcap) {
        if (!pos_pinned) sl.hout_dst = (uint8_t *)frame_pos;
        HIP_OK(hipMemcpyAsync(pos_pinned ? (void *)frame_pos : sl.hout, sl.pos.p, pcap * 8, hipMemcpyDeviceToHost,
                              c->d2h));
    }
    HIP_OK(hipEventRecord(sl.ev_done, c->d2h));
    *ticket = sl.ticket;
    return 0;
}

int iggy_codec_encode_submit(iggy_codec_ctx *c, const iggy_raw_messages *m, uint64_t partition_id, uint8_t *out,
                             uint64_t cap, iggy_ticket *ticket) {
    if (!c || !m || !ticket) return IGGY_ERR_INVALID_ARGUMENT;
    if (m->count == 0 || m->count > 0xFFFFFFFFull || !out) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    const uint64_t n = m->count;
    uint64_t spl = 0, suh = 0;
    for (uint64_t i = 0; i < n; ++i) {
        spl += m->payload_lengths[i];
        suh += m->user_headers_lengths ? m->user_headers_lengths[i] : 0;
    }
    const uint64_t need = 256 + 48 * n + spl + suh;
    int k = 0;
    int r = take_slot(c, IGGY_OP_ENCODE, &k);
    if (r) return r;
    Slot &sl = c->slots[k];
    const bool has_uh = m->user_headers_lengths != nullptr;
    r = sl.ids.ensure(n * 16);
    r |= sl.ots.ensure(n * 8);
    r |= sl.pay.ensure(spl + 16);
    r |= sl.plen.ensure(n * 4);
    r |= sl.uhb.ensure(suh + 16);
    r |= sl.uhl.ensure(n * 4);
    r |= sl.out.ensure(need + 16);
    r |= sl.res.ensure(256);
    if (r) {
        sl.busy = false;
        return IGGY_ERR_DEVICE;
    }
    sl.cap = cap;
    sl.out_len = need;
    sl.fast = false;
    sl.frame_pos = nullptr;
    sl.hout_dst = nullptr;
    sl.hout_len = 0;
    const bool out_pinned = host_pinned(out, need);
    if (cap >= need && !out_pinned && sl.hout_ensure(need)) r = IGGY_ERR_DEVICE;
    // Small batches (SoA input of <= kZeroCopyBytes, one segment) in place: the kernels
    // read the SoA arrays over the host link (registered ones where they are, anything
    // else copied with one memcpy per array into the slot's mapped staging, so the
    // caller's bytes are free when submit returns) and write the wire bytes and the
    // verdict straight into mapped host memory (the caller's pinned `out`, else the
    // slot's bounce). No copy operation on any stream; the kernels on the slot's own
    // stream with the slot's own scratch, so the slots' encodes run side by side.
    const uint64_t in_bytes = n * 28 + spl + (has_uh ? suh + n * 4 : 0);
    if (!r && c->slot_pinned_d && cap >= need && in_bytes <= kZeroCopyBytes && n < kEncSegMinFrames) {
        iggy_raw_messages dm;
        if (stage_soa(m, n, spl, suh, sl.zin, &dm)) {
            sl.busy = false;
            return IGGY_ERR_DEVICE;
        }
        uint8_t *d_out = out_pinned ? (uint8_t *)host_device_ptr(out, need) : nullptr;
        if (!d_out) {
            void *dp = nullptr;
            if (out_pinned || !sl.hout || hipHostGetDevicePointer(&dp, sl.hout, 0) != hipSuccess || !dp) {
                (void)hipGetLastError();
                dp = nullptr;
            }
            d_out = (uint8_t *)dp;
            if (d_out) sl.hout_dst = out;
        }
        if (d_out) {
            if (!sl.st && hipStreamCreateWithFlags(&sl.st, hipStreamNonBlocking) != hipSuccess) {
                sl.st = nullptr;
                sl.busy = false;
                return IGGY_ERR_DEVICE;
            }
            iggy_encode_result *d_res = (iggy_encode_result *)(c->slot_pinned_d + 256 * k);
            r = enqueue_encode(c, &dm, partition_id, d_out, cap, d_res, sl.st, &sl.eown);
            if (!r && hipEventRecord(sl.ev_done, sl.st) != hipSuccess) r = IGGY_ERR_DEVICE;
            if (r) {
                sl.busy = false;
                return r;
            }
            *ticket = sl.ticket;
            return 0;
        }
        sl.hout_dst = nullptr;  // (no mapped destination: the copy path below)
    }
    hipStream_t h = c->h2d;
    if (!r) {
        r |= put_host(c, sl.ids.p, m->ids, n * 16, h);
        r |= put_host(c, sl.ots.p, m->origin_timestamps, n * 8, h);
        r |= put_host(c, sl.pay.p, m->payloads, spl, h);
        r |= put_host(c, sl.plen.p, m->payload_lengths, n * 4, h);
        if (has_uh) {
            r |= put_host(c, sl.uhb.p, m->user_headers, suh, h);
            r |= put_host(c, sl.uhl.p, m->user_headers_lengths, n * 4, h);
        }
    }
    if (r) {
        sl.busy = false;
        return IGGY_ERR_DEVICE;
    }
    HIP_OK(hipEventRecord(sl.ev_in, h));
    hipStream_t s = bind(c, nullptr);
    HIP_OK(hipStreamWaitEvent(s, sl.ev_in, 0));
    iggy_raw_messages dm;
    dm.count = n;
    dm.ids = sl.ids.as<uint64_t>();
    dm.origin_timestamps = sl.ots.as<uint64_t>();
    dm.payloads = sl.pay.as<uint8_t>();
    dm.payload_lengths = sl.plen.as<uint32_t>();
    dm.user_headers = has_uh ? sl.uhb.as<uint8_t>() : nullptr;
    dm.user_headers_lengths = has_uh ? sl.uhl.as<uint32_t>() : nullptr;
    iggy_encode_result *d_res = sl.res.as<iggy_encode_result>();
    // a batch that does not fit `cap` is reported by the device (nothing is written)
    r = enqueue_encode(c, &dm, partition_id, sl.out.as<uint8_t>(), cap, d_res, s);
    if (r) {
        sl.busy = false;
        return r;
    }
    HIP_OK(hipEventRecord(sl.ev_k, s));
    HIP_OK(hipStreamWaitEvent(c->d2h, sl.ev_k, 0));
    HIP_OK(hipMemcpyAsync((uint8_t *)c->slot_pinned + 256 * k, d_res, sizeof(iggy_encode_result),
                          hipMemcpyDeviceToHost, c->d2h));
    if (cap >= need) {  // (a pageable `out` from the slot's pinned bounce, in iggy_codec_poll)
        if (!out_pinned) sl.hout_dst = out;
        HIP_OK(hipMemcpyAsync(out_pinned ? (void *)out : sl.hout, sl.out.p, need, hipMemcpyDeviceToHost, c->d2h));
    }
    HIP_OK(hipEventRecord(sl.ev_done, c->d2h));
    *ticket = sl.ticket;
    return 0;
}

int iggy_codec_poll(iggy_codec_ctx *c, iggy_ticket ticket, iggy_completion *out) {
    if (!c || !out) return IGGY_ERR_INVALID_ARGUMENT;
    Slot &sl = c->slots[ticket & (kSlots - 1)];
    if (!sl.busy || sl.ticket != ticket) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    const hipError_t q = hipEventQuery(sl.ev_done);
    if (q == hipErrorNotReady) {
        (void)hipGetLastError();  // not an error: leave no sticky status for the caller's HIP code
        return IGGY_ERR_PENDING;
    }
    if (q == hipSuccess && sl.op == IGGY_OP_DECODE && sl.fast && !sl.g_pending) {
        // the records launch found a stride break the walk goes past: the general walk
        // (its barrier words re-armed first), the positions, the completion event again
        const size_t k = ticket & (kSlots - 1);
        const iggy_decode_result *rr = (const iggy_decode_result *)((const uint8_t *)c->slot_pinned + 256 * k);
        if (rr->status == kStatusNeedGeneral) {
            hipStream_t s = bind(c, nullptr);
            const DecodeScratch dsc = dscratch(c);
            iggy_decode_result *d_res = (iggy_decode_result *)(c->slot_pinned_d + 256 * k);
            // each operation checked where it is issued: the thread's last-error status is
            // cleared first, so a launch failure is this launch's and not an unrelated
            // earlier error of the caller's own HIP code
            (void)hipGetLastError();
            hipError_t e = hipSuccess;
            hipLaunchKernelGGL(k_general_rearm, dim3(1), dim3(64), 0, s, GenRearm{dsc.gbar, dsc.gbar2, dsc.gmisc});
            e = hipGetLastError();
            if (e == hipSuccess) {
                launch_general(c, sl.g_in, sl.g_len, sl.g_integ, sl.g_pos, sl.g_pcap, d_res, s);
                e = hipGetLastError();
            }
            if (e == hipSuccess && sl.g_pos_copy)
                e = hipMemcpyAsync(host_pinned(sl.frame_pos, sl.g_pcap * 8) ? (void *)sl.frame_pos : sl.hout,
                                   sl.pos.p, sl.g_pcap * 8, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipEventRecord(sl.ev_done, s);
            sl.g_pending = true;
            if (e != hipSuccess) {
                // whatever was issued may still use the slot's buffers and the caller's
                // memory: drain the stream before the slot is free again
                (void)hipGetLastError();
                (void)hipStreamSynchronize(s);
                sl.busy = false;
                return IGGY_ERR_DEVICE;
            }
            return IGGY_ERR_PENDING;
        }
    }
    sl.busy = false;
    if (q != hipSuccess) return IGGY_ERR_DEVICE;
    memset(out, 0, sizeof(*out));
    out->op = sl.op;
    const uint8_t *rec = (const uint8_t *)c->slot_pinned + 256 * (ticket & (kSlots - 1));
    if (sl.op == IGGY_OP_DECODE) {
        iggy_decode_result res;
        memcpy(&res, rec, sizeof(res));
        if (res.error.kind == IGGY_ERR_TIMEOUT) reset_after_timeout(c);
        out->header = res.header;
        out->error = res.error;
        out->frame_count = res.frame_count;
        out->computed_checksum = res.computed_checksum;
        if (res.error.kind == IGGY_OK && sl.frame_pos && res.frame_count > sl.cap) {
            out->error = iggy_wire_error{IGGY_ERR_CAPACITY, 0, res.frame_count, sl.cap, 0};
        } else if (res.error.kind == IGGY_OK && sl.hout_dst && res.frame_count) {
            memcpy(sl.hout_dst, sl.hout, std::min<uint64_t>(res.frame_count, sl.cap) * 8);
        }
    } else {
        iggy_encode_result res;
        memcpy(&res, rec, sizeof(res));
        out->header = res.header;
        out->error = res.error;
        out->bytes = res.error.kind == IGGY_OK ? res.batch_length : 0;
        if (res.error.kind == IGGY_OK && sl.hout_dst) memcpy(sl.hout_dst, sl.hout, sl.out_len);
    }
    return 0;
}

int iggy_codec_wait(iggy_codec_ctx *c, iggy_ticket ticket, iggy_completion *out) {
    if (!c || !out) return IGGY_ERR_INVALID_ARGUMENT;
    Slot &sl = c->slots[ticket & (kSlots - 1)];
    if (!sl.busy || sl.ticket != ticket) return IGGY_ERR_INVALID_ARGUMENT;
    while (true) {  // (a fast-path decode's general walk, started by poll, means one more round)
        {
            DevGuard dg(c->device);
            HIP_OK(hipEventSynchronize(sl.ev_done));
        }
        const int r = iggy_codec_poll(c, ticket, out);
        if (r != IGGY_ERR_PENDING) return r;
    }
}

}  // extern "C"
