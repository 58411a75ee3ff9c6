// host_pollbody.hpp -- the poll reply body (iggy_codec_build_polled_body)
//
// Part of the unity build of libiggy_codec.so: included by codec_api.hip, after the
// kernel translation units and the units before it (see codec_api.hip for the order).
#pragma once

extern "C" {

// ----------------------------------------------- poll reply body
// build_polled_messages_body (core/server/src/responses.rs:1666-1714): the fragments
// concatenated into one stream, walked record by record (BatchHeader::decode,
// batch_end = position + total_size checked against the stream), each record copied or
// -- with an encryptor -- decrypted (decrypt_batch_record, send_messages.rs:364-415,
// on the GPU: one H2D of the stream, every record's decrypt enqueued back to back on
// the context stream, one D2H of the verdicts and the plaintext), the message count
// summed with checked_add and backpatched into [partition_id u32][current_offset u64]
// [count u32]. Errors in the reference's order: record k's header / bounds, then its
// decrypt, then the count overflow, before anything of record k + 1.
namespace {
uint32_t poll_error_kind(uint32_t kind) {
    // decrypt_batch_record's `?` on decode_batch_slice_with (LayoutOnly) goes through
    // batch_error (send_messages.rs:52-66): checksum kinds keep their identity (never
    // produced by a layout walk), everything else is InvalidCommand
    switch (kind) {
        case IGGY_OK:
        case IGGY_ERR_CANNOT_DECRYPT_DATA:
        case IGGY_ERR_INVALID_COMMAND:
        case IGGY_ERR_INVALID_BATCH_CHECKSUM:
        case IGGY_ERR_INVALID_MESSAGE_CHECKSUM:
        case IGGY_ERR_TIMEOUT:
        case IGGY_ERR_DEVICE:
            return kind;
        default:
            return IGGY_ERR_INVALID_COMMAND;
    }
}
int pb_pinned_ensure(iggy_codec_ctx *c, size_t n) {
    // grown past kHostMapKeep by one large decrypting poll: given back at the next
    // ordinary-sized one instead of staying pinned for the context's life
    if (n <= c->pb_cap && !(c->pb_cap > kHostMapKeep && n <= kHostMapKeep)) return 0;
    if (c->pb_pinned) (void)hipHostFree(c->pb_pinned);
    c->pb_pinned = nullptr;
    c->pb_cap = 0;
    const size_t want = std::max<size_t>(n, 1 << 20);
    if (hipHostMalloc(&c->pb_pinned, want, hipHostMallocDefault) != hipSuccess) {
        c->pb_pinned = nullptr;
        return IGGY_ERR_DEVICE;
    }
    c->pb_cap = want;
    return 0;
}
}  // namespace

int iggy_codec_build_polled_body(iggy_codec_ctx *c, uint32_t partition_id, uint64_t current_offset,
                                 const iggy_poll_fragment *frags, uint64_t nfrags, const uint8_t *key, uint8_t *out,
                                 uint64_t cap, uint64_t *out_len, iggy_wire_error *err) {
    if (!c || (!frags && nfrags) || !out_len || (!out && cap)) return IGGY_ERR_INVALID_ARGUMENT;
    set_err(err, IGGY_OK);
    *out_len = 0;
    uint64_t total = 0;
    for (uint64_t f = 0; f < nfrags; ++f) {
        if (!frags[f].data && frags[f].len) return IGGY_ERR_INVALID_ARGUMENT;
        total += frags[f].len;
    }
    auto fail = [&](uint32_t kind, uint64_t a = 0, uint64_t b = 0) {
        set_err(err, kind, 0, a, b);
        return (int)kind;
    };
    // 1. the concatenated stream: straight into the body when it fits and nothing is
    //    decrypted (the reply IS the stored encoding); into host memory when it does
    //    not fit (only walked, for the reference's error order, then CAPACITY); into
    //    the pinned staging (stream, then the plaintext) when records are decrypted
    uint8_t *stream;
    std::vector<uint8_t> walk_only;
    if (!key && cap >= 16 + total) {
        stream = out + 16;
    } else if (!key) {
        walk_only.resize(total + 1);
        stream = walk_only.data();
    } else {
        if (pb_pinned_ensure(c, 2 * total + 64)) return IGGY_ERR_DEVICE;
        stream = (uint8_t *)c->pb_pinned;
    }
    {
        uint64_t o = 0;
        for (uint64_t f = 0; f < nfrags; ++f) {
            if (frags[f].len) memcpy(stream + o, frags[f].data, frags[f].len);
            o += frags[f].len;
        }
    }
    // 2. the record walk (headers only)
    struct Rec { uint64_t pos, len; uint32_t count; };
    std::vector<Rec> recs;
    bool walk_failed = false;
    for (uint64_t pos = 0; pos < total;) {
        iggy_batch_header h;
        iggy_wire_error e;
        if (iggy_batch_header_decode(stream + pos, total - pos, &h, &e) != 0) {
            walk_failed = true;  // BatchHeader::decode -> InvalidCommand
            break;
        }
        const uint64_t end = pos + h.batch_length;
        if (end < pos || end > total) {  // checked_add / batch_end > stream.len()
            walk_failed = true;
            break;
        }
        recs.push_back({pos, h.batch_length, h.message_count});
        pos = end;
    }
    // 3. decrypt every walked record on the device
    std::vector<iggy_crypt_result> res;
    uint64_t dec_total = 0;
    if (key && !recs.empty()) {
        const uint64_t span = recs.back().pos + recs.back().len;
        uint64_t maxlen = 0;
        for (const Rec &r : recs) maxlen = std::max(maxlen, r.len);
        DevGuard dg(c->device);
        bind(c, nullptr);
        int r = c->din.ensure(span + 16);
        r |= c->dout.ensure(span + 16);
        r |= c->pbres.ensure(recs.size() * sizeof(iggy_crypt_result));
        if (r) return IGGY_ERR_DEVICE;
        r = crypt_reserve(c, maxlen);
        if (r) return r;
        HIP_OK(hipMemcpyAsync(c->din.p, stream, span, hipMemcpyHostToDevice, c->stream));
        iggy_crypt_result *d_res = c->pbres.as<iggy_crypt_result>();
        for (size_t k = 0; k < recs.size(); ++k) {
            r = enqueue_crypt(c, false, key, c->din.as<uint8_t>(recs[k].pos), recs[k].len, nullptr,
                              c->dout.as<uint8_t>(recs[k].pos), recs[k].len, d_res + k, c->stream);
            if (r) return r;
        }
        // verdicts and plaintext back into the staging's second half
        uint8_t *hout = stream + total + 32;
        res.resize(recs.size());
        HIP_OK(hipMemcpyAsync(hout, c->dout.p, span, hipMemcpyDeviceToHost, c->stream));
        r = get_host(c, res.data(), d_res, recs.size() * sizeof(iggy_crypt_result), c->stream);
        if (r) return r;
        for (const iggy_crypt_result &q : res)
            if (q.error.kind == IGGY_ERR_TIMEOUT) { reset_after_timeout(c); break; }
    }
    // 4. the reference's per-record order: decrypt verdict, then the count
    uint32_t count = 0;
    for (size_t k = 0; k < recs.size(); ++k) {
        if (key) {
            const iggy_crypt_result &q = res[k];
            const uint32_t kind = poll_error_kind(q.error.kind);
            if (kind != IGGY_OK) {
                if (err) {
                    *err = q.error;
                    err->kind = kind;
                    if (kind != q.error.kind) err->reason = 0, err->a = err->b = err->c = 0;
                }
                return (int)kind;
            }
            dec_total += q.out_len;
        }
        if ((uint64_t)count + recs[k].count > 0xFFFFFFFFull) return fail(IGGY_ERR_INVALID_COMMAND);
        count += recs[k].count;
    }
    if (walk_failed) return fail(IGGY_ERR_INVALID_COMMAND);
    const uint64_t body_len = 16 + (key ? dec_total : total);
    if (cap < body_len) return fail(IGGY_ERR_CAPACITY, body_len, cap);
    if (key) {
        const uint8_t *hout = stream + total + 32;
        uint64_t o = 16;
        for (size_t k = 0; k < recs.size(); ++k) {
            memcpy(out + o, hout + recs[k].pos, res[k].out_len);
            o += res[k].out_len;
        }
    } else if (stream != out + 16) {
        memcpy(out + 16, stream, total);
    }
    memcpy(out, &partition_id, 4);
    memcpy(out + 4, &current_offset, 8);
    memcpy(out + 12, &count, 4);
    *out_len = body_len;
    return 0;
}

}  // extern "C"
