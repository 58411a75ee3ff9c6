// host_poll.hpp -- poll-side decode: SDK poll responses and the server conversion entries
//
// Part of the unity build of libiggy_codec.so: included by codec_api.hip, after the
// kernel translation units and the units before it (see codec_api.hip for the order).
#pragma once

extern "C" {

// ------------------------------------------------------------- poll decode
int iggy_codec_poll_decode(iggy_codec_ctx *c, const uint8_t *buf, uint64_t len, int mode,
                           iggy_polled_message *out, uint64_t cap, uint64_t *n_out,
                           iggy_wire_error *err) {
    if (!c || (!buf && len)) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    set_err(err, IGGY_OK);
    if (n_out) *n_out = 0;
    // 1. the record chain from the 256-B headers (polled_messages.rs:99-106,
    //    poll_messages.rs:123-125); the header walk's own failure, if any, comes
    //    after every record before it
    struct Rec { uint64_t pos, bl, pbase; };
    std::vector<Rec> recs;
    int stop_rc = 0;
    iggy_wire_error stop_err{};
    uint64_t position = 0, pwords = 0;
    while (position < len) {
        iggy_batch_header h;
        iggy_wire_error he;
        const int hr = iggy_batch_header_decode(buf + position, len - position, &h, &he);
        if (mode == IGGY_POLL_MODE_SDK) {
            if (hr || h.batch_length > len - position) {
                set_err(err, IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH);
                return IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH;
            }
        } else if (hr) {
            stop_rc = hr;
            stop_err = he;
            break;
        }
        const uint64_t avail = std::min<uint64_t>(h.batch_length, len - position);
        recs.push_back({position, h.batch_length, pwords});
        pwords += avail / 48 + 1;
        if (h.batch_length > len - position) break;  // its decode reports the EOF
        position += h.batch_length;
    }
    // 2. every record's frame walk (LayoutOnly) in ONE multi-record launch, which also
    //    writes the message descriptors of the single-stride records; the others take
    //    the single-record decode and k_poll_fill. Descriptor slots: record k's planned
    //    frame count, consecutive, so a body of well-formed records comes back in one
    //    copy; single-path and re-walked records fill a tail area instead.
    const size_t K = recs.size();
    std::vector<RecIn> rin(K);
    std::vector<uint64_t> slot(K), tailb(K);
    uint64_t nslots = 0;
    for (size_t k = 0; k < K; ++k) {
        const uint64_t avail = std::min<uint64_t>(recs[k].bl, len - recs[k].pos);
        uint64_t nf = 0;
        const uint64_t nw = rec_plan(buf + recs[k].pos, len - recs[k].pos, &nf);
        slot[k] = nslots;
        nslots += nw ? nf : 0;
        rin[k] = RecIn{recs[k].pos, len - recs[k].pos, recs[k].pbase, avail / 48 + 1, slot[k]};
    }
    for (size_t k = 0; k < K; ++k) tailb[k] = nslots + recs[k].pbase;
    if (K && records_all_planned(buf, rin.data(), K)) {
        // every record single-stride: descriptors and verdicts straight into host-mapped
        // memory, the host spinning on the launch's completion flag (one H2D, one launch)
        const size_t rb = K * sizeof(iggy_decode_result), mo = (64 + rb + 127) & ~(size_t)127;
        if (c->din.ensure(len + 16) || c->omap.ensure(mo + (nslots + 1) * sizeof(iggy_polled_message)))
            return IGGY_ERR_DEVICE;
        // a body of <= kZeroCopyBytes is read in place (registered: where it is;
        // pageable: one memcpy into the context's mapped staging), larger ones copied
        const uint8_t *d_body = nullptr;
        if (IGGY_POLL_IN_PLACE && len <= kZeroCopyBytes) {
            d_body = host_device_ptr(buf, len);
            if (!d_body && !host_pinned(buf, len)) {
                if (c->zin.ensure(len + 16)) return IGGY_ERR_DEVICE;
                memcpy(c->zin.h, buf, len);
                d_body = c->zin.d;
            }
        }
        int r = 0;
        if (!d_body) {
            r = put_host(c, c->din.p, buf, len, c->stream);
            if (r) return r;
            d_body = c->din.as<uint8_t>();
        }
        std::vector<size_t> single;
        const uint32_t v = next_flag(c);
        r = enqueue_records(c, d_body, buf, rin.data(), K, IGGY_INTEGRITY_LAYOUT_ONLY, nullptr,
                            c->omap.dp<iggy_polled_message>(mo), c->omap.dp<iggy_decode_result>(64), &single,
                            nullptr, c->omap.dp<uint32_t>(), v);
        if (r) return r;
        r = wait_host_flag(c, v);
        if (!r) r = xfer_settle(c);
        if (r) return r;
        const iggy_decode_result *res = c->omap.hp<iggy_decode_result>(64);
        bool general = false;
        for (size_t k = 0; k < K; ++k) {
            if (res[k].error.kind == IGGY_ERR_TIMEOUT) {
                reset_after_timeout(c);
                set_err(err, IGGY_ERR_TIMEOUT);
                return IGGY_ERR_TIMEOUT;
            }
            general |= res[k].status == kStatusNeedGeneral;
        }
        if (!general) {  // (a stride that broke mid-record: the path below, from scratch)
            const iggy_polled_message *msgs = c->omap.hp<iggy_polled_message>(mo);
            uint64_t n = 0;
            int rc = 0;
            for (size_t k = 0; k < K && !rc; ++k) {
                const iggy_decode_result &rs = res[k];
                if (mode == IGGY_POLL_MODE_SDK) {
                    if (rs.covered != recs[k].bl - 256) {
                        set_err(err, IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH);
                        return IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH;
                    }
                } else if (rs.error.kind != IGGY_OK) {
                    fill_err(err, rs.error);
                    rc = (int)rs.error.kind;
                    break;
                }
                const uint64_t nf = rs.frame_count;
                if (n + nf > cap) {
                    set_err(err, IGGY_ERR_CAPACITY, 0, n + nf, cap);
                    rc = IGGY_ERR_CAPACITY;
                    break;
                }
                if (nf) memcpy(out + n, msgs + slot[k], nf * sizeof(iggy_polled_message));
                n += nf;
            }
            if (!rc && stop_rc) {
                fill_err(err, stop_err);
                rc = stop_rc;
            }
            if (n_out) *n_out = n;
            return rc;
        }
    }
    int r = c->din.ensure(len + 16);
    r |= c->ppos.ensure((pwords + 1) * 8);
    r |= c->pres.ensure((K + 1) * sizeof(iggy_decode_result));
    r |= c->pmsgs.ensure((nslots + pwords + 1) * sizeof(iggy_polled_message));
    if (r) return IGGY_ERR_DEVICE;
    r = put_host(c, c->din.p, buf, len, c->stream);
    if (r) return r;
    iggy_decode_result *d_res = c->pres.as<iggy_decode_result>();
    iggy_polled_message *d_msgs = c->pmsgs.as<iggy_polled_message>();
    std::vector<size_t> single, redone;
    r = enqueue_records(c, c->din.as<uint8_t>(), buf, rin.data(), K, IGGY_INTEGRITY_LAYOUT_ONLY, c->ppos.as<uint64_t>(),
                        d_msgs, d_res, &single);
    if (r) return r;
    std::vector<iggy_decode_result> res(K);
    r = get_host(c, res.data(), d_res, K * sizeof(iggy_decode_result), c->stream);
    if (r) return r;
    r = redo_general(c, c->din.as<uint8_t>(), rin.data(), K, IGGY_INTEGRITY_LAYOUT_ONLY, c->ppos.as<uint64_t>(),
                     res.data(), &redone);
    if (r) {
        if (r == IGGY_ERR_TIMEOUT) set_err(err, IGGY_ERR_TIMEOUT);
        return r;
    }
    std::vector<uint8_t> in_tail(K, 0);
    for (size_t k : single) in_tail[k] = 1;
    for (size_t k : redone) in_tail[k] = 1;
    // 3. verdicts in record order; descriptors of tail records expanded, one copy out
    uint64_t n = 0;
    int rc = 0;
    struct Span { uint64_t src, n; };
    std::vector<Span> spans;
    for (size_t k = 0; k < K && !rc; ++k) {
        const iggy_decode_result &rs = res[k];
        if (mode == IGGY_POLL_MODE_SDK) {
            // the SDK walk only needs the frames to tile the record (no count check)
            if (rs.covered != recs[k].bl - 256) {
                set_err(err, IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH);
                return IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH;
            }
        } else if (rs.error.kind != IGGY_OK) {  // yielded after the messages before it
            fill_err(err, rs.error);
            rc = (int)rs.error.kind;
            break;
        }
        const uint64_t nf = rs.frame_count;
        if (n + nf > cap) {
            set_err(err, IGGY_ERR_CAPACITY, 0, n + nf, cap);
            rc = IGGY_ERR_CAPACITY;
            break;
        }
        if (nf) {
            uint64_t src = slot[k];
            if (in_tail[k]) {
                src = tailb[k];
                hipLaunchKernelGGL(k_poll_fill, dim3((uint32_t)std::min<uint64_t>((nf + 255) / 256, 65535)), dim3(256),
                                   0, c->stream, c->din.as<uint8_t>(), recs[k].pos,
                                   c->ppos.as<uint64_t>(8 * recs[k].pbase), nf, d_msgs + src);
                HIP_OK(hipGetLastError());
            }
            if (!spans.empty() && spans.back().src + spans.back().n == src) spans.back().n += nf;
            else spans.push_back({src, nf});
        }
        n += nf;
    }
    if (!rc && stop_rc) {
        fill_err(err, stop_err);
        rc = stop_rc;
    }
    uint64_t o = 0;
    for (const Span &sp : spans) {
        r = get_host(c, out + o, d_msgs + sp.src, sp.n * sizeof(iggy_polled_message), c->stream);
        if (r) return r;
        o += sp.n;
    }
    HIP_OK(hipStreamSynchronize(c->stream));
    if (n_out) *n_out = n;
    return rc;
}

}  // extern "C"
