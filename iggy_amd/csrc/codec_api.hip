// codec_api.hip — host side of the C ABI declared in include/iggy_codec.h.
//
// Unity build: the kernel translation units are included here so the whole
// library is one code object (libiggy_codec.so). Host code only sizes scratch,
// enqueues kernels and converts results; every byte of the hot path (frame
// walk, XXH3, batch checksum, encode) runs on the GPU. There is deliberately
// no CPU fallback: without a usable gfx950 device iggy_codec_create fails.
#include <hip/hip_runtime.h>

#include <errno.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/iggy_codec.h"

#ifndef IGGY_ENC_RING
#define IGGY_ENC_RING 1  // (build knob for same-box A/B: 0 = k_enc_lanes for segmented encodes too)
#endif
#ifndef IGGY_ENC_SPLIT
#define IGGY_ENC_SPLIT 0  // (build knob for same-box A/B: 1 = writer waves in k_enc_ring, encode.hip)
#endif
#include "batch_checksum.hip"
#include "decode_general.hip"
#include "decode_uniform.hip"
#include "decode_records.hip"
#include "encode.hip"
#include "poll.hip"
#include "slice.hip"
#include "crypt.hip"
static_assert(!IGGY_ENC_SPLIT || iggy::kErWaves == 4, "the writer-wave split is built for 4 hasher waves");

using namespace iggy;

#define HIP_OK(x)                                                              \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            if (getenv("IGGY_CODEC_DEBUG"))                                    \
                fprintf(stderr, "iggy_codec: %s failed: %s (%s:%d)\n", #x,     \
                        hipGetErrorString(e_), __FILE__, __LINE__);            \
            return IGGY_ERR_DEVICE;                                            \
        }                                                                      \
    } while (0)

// Host runtime, by concern (each unit includes nothing itself; this order is the
// dependency order):
//   host_ctx      context, scratch buffers, slots, stream order
//   host_mem      caller host memory: registry, pinned / pageable copies, history log
//   host_decode   decode enqueue, synchronous decode / checksum / admission entries
//   host_segment  segment recovery, state-transfer walk, segment writes
//   host_encode   encode enqueue and entries
//   host_poll     SDK poll decode, server conversion
//   host_crypt    at-rest encryption host setup
//   host_pollbody poll reply body
//   host_slice    poll-path slicing, disk-chunk walk, device stamp
//   host_async    asynchronous submit / poll / wait
#include "host_ctx.hpp"
#include "host_mem.hpp"
#include "host_decode.hpp"
#include "host_segment.hpp"
#include "host_encode.hpp"
#include "host_poll.hpp"
#include "host_crypt.hpp"
#include "host_pollbody.hpp"
#include "host_slice.hpp"
#include "host_async.hpp"


// ===================================================================== ABI
extern "C" {

uint32_t iggy_codec_abi_version(void) { return IGGY_CODEC_ABI_VERSION; }

int iggy_codec_create(int device, iggy_codec_ctx **out) {
    if (!out) return IGGY_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return IGGY_ERR_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return IGGY_ERR_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return IGGY_ERR_DEVICE;
    iggy_codec_ctx *c = new (std::nothrow) iggy_codec_ctx();
    if (!c) return IGGY_ERR_DEVICE;
    c->device = device;
    c->ncu = prop.multiProcessorCount;
    c->ugrid = std::max(2, c->ncu - 1);
    if (kDiagMask) {  // diagnostic build only: tuning / ablation knobs never reach the product
        if (const char *d = getenv("IGGY_CODEC_DBG")) c->dbg = (uint32_t)strtoul(d, nullptr, 0);
        if (const char *g = getenv("IGGY_CODEC_UNIFORM_GRID")) {
            const long v = strtol(g, nullptr, 0);
            if (v >= 2 && v <= c->ncu) c->ugrid = (int)v;
        }
    }
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess) {
        if (c->stream) (void)hipStreamDestroy(c->stream);
        delete c;
        return IGGY_ERR_DEVICE;
    }
    for (auto &ev : c->seg_ev)
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
    c->last = c->stream;
    int r = 0;
    if (hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming) != hipSuccess) r = IGGY_ERR_DEVICE;
    r |= c->dresult.ensure(4096);
    if (hipHostMalloc(&c->h_pinned, 4096, hipHostMallocDefault) != hipSuccess) r = IGGY_ERR_DEVICE;
    if (!r) {
        if (hipFuncSetAttribute((const void *)k_decode_uniform<true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, kUniformLds) != hipSuccess ||
            hipFuncSetAttribute((const void *)k_decode_uniform<false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, kUniformLds) != hipSuccess ||
            hipFuncSetAttribute((const void *)k_decode_general<true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, kGenLds) != hipSuccess ||
            hipFuncSetAttribute((const void *)k_enc_ring<false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, kErLds) != hipSuccess ||
            (IGGY_ENC_SPLIT && hipFuncSetAttribute((const void *)k_enc_ring<true>,
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, kEsLds) != hipSuccess))
            r = IGGY_ERR_DEVICE;
    }
    if (!r) {
        // the general decode's grid barriers need every WG co-resident
        int occ_t = 0, occ_f = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_t, k_decode_general<true>, kGenThreads, kGenLds) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_f, k_decode_general<false>, kGenThreads, 0) != hipSuccess)
            r = IGGY_ERR_DEVICE;
        c->gen_grid = c->ncu * std::max(1, std::min(2, std::min(occ_t, occ_f)));
    }
    for (int w = 0; w < 2 && !r; ++w)
        if (hipEventCreate(&c->ev0[w]) != hipSuccess || hipEventCreate(&c->ev1[w]) != hipSuccess)
            r = IGGY_ERR_DEVICE;
    if (!r) r = ensure_decode_scratch(c, 1 << 20);
    if (!r) {
        // probe: does global_load_lds_dwordx4 honour unaligned sources here?
        DevBuf pb;
        if (pb.ensure(8192) == 0) {
            // (pattern and verdict through the pinned result mirror, unused until now)
            uint8_t *pat = (uint8_t *)c->h_pinned;
            for (size_t i = 0; i < 4096; ++i) pat[i] = (uint8_t)(i * 131 + 7);
            uint32_t *flag = c->dresult.as<uint32_t>(1024);
            if (hipMemcpyAsync(pb.p, pat, 4096, hipMemcpyHostToDevice, c->stream) == hipSuccess &&
                hipMemsetAsync(flag, 0, 4, c->stream) == hipSuccess) {
                hipLaunchKernelGGL(k_probe_glds_unaligned, dim3(1), dim3(64), 16 * 64 * 4, c->stream,
                                   (const uint8_t *)pb.p, flag);
                if (hipMemcpyAsync(pat, flag, 4, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
                    hipStreamSynchronize(c->stream) == hipSuccess) {
                    uint32_t ok = 0;
                    memcpy(&ok, pat, 4);
                    c->allow_unaligned = ok == 1;
                }
            }
            pb.release();
        }
    }
    if (r) {
        iggy_codec_destroy(c);
        return IGGY_ERR_DEVICE;
    }
    *out = c;
    return 0;
}

void iggy_codec_destroy(iggy_codec_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    // every stream that may still run this context's work (the caller's last stream,
    // the side stream of segmented encodes, the copy streams of the asynchronous host
    // operations) drains before any buffer it reads or writes goes back to the allocator
    (void)svc_disable(c);  // the resident service's grid stops and drains first
    if (c->svc.s) (void)hipStreamSynchronize(c->svc.s);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->last && c->last != c->stream) (void)hipStreamSynchronize(c->last);
    if (c->side) (void)hipStreamSynchronize(c->side);
    if (c->h2d) (void)hipStreamSynchronize(c->h2d);
    if (c->d2h) (void)hipStreamSynchronize(c->d2h);
    for (Slot &sl : c->slots)  // the fast-path decodes' own streams
        if (sl.st) (void)hipStreamSynchronize(sl.st);
    {
        // ranges this context registered and the caller never unregistered: unpinned now,
        // so no registry entry outlives the context that vouches for it
        std::vector<uintptr_t> mine;
        {
            std::lock_guard<std::mutex> lk(g_reg_mu);
            for (size_t i = 0; i < g_reg.size();)
                if (g_reg[i].owner == c) {
                    mine.push_back(g_reg[i].h);
                    hostmem_log("unregister (context destroyed)", (const void *)g_reg[i].h, g_reg[i].len);
                    g_reg.erase(g_reg.begin() + (long)i);
                } else {
                    ++i;
                }
        }
        for (uintptr_t h : mine)
            if (hipHostUnregister((void *)h) != hipSuccess) (void)hipGetLastError();
    }
    DevBuf *bufs[] = {&c->dsync, &c->dsums, &c->derr, &c->gtiles_s, &c->gtiles_x,
                      &c->gtiles_cnt, &c->gtiles_pre, &c->gtiles_list, &c->gtiles_e, &c->gtiles_base, &c->ggrp, &c->gfpos, &c->gcs, &c->gvrec, &c->gtiles_lcs,
                      &c->gbsums, &c->dresult, &c->din, &c->dpos, &c->dout, &c->epl, &c->euh,
                      &c->etile, &c->ecs, &c->emisc, &c->eids, &c->eots, &c->epay, &c->eplen,
                      &c->euhb, &c->euhl, &c->erec, &c->esink, &c->hbsums, &c->ppos, &c->pmsgs, &c->pres, &c->cwk, &c->sl, &c->slres, &c->cr,
                      &c->rtab, &c->rbsums, &c->rres, &c->clinks, &c->rstate, &c->rcount, &c->pbres};
    for (DevBuf *b : bufs) b->release();
    if (c->h_pinned) (void)hipHostFree(c->h_pinned);
    if (c->pb_pinned) (void)hipHostFree(c->pb_pinned);
    if (c->xst) (void)hipHostFree(c->xst);
    for (auto &ev : c->xev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->xin_ev) (void)hipEventDestroy(c->xin_ev);
    for (int w = 0; w < 2; ++w) {
        if (c->ev0[w]) (void)hipEventDestroy(c->ev0[w]);
        if (c->ev1[w]) (void)hipEventDestroy(c->ev1[w]);
    }
    for (auto &ev : c->seg_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (c->order_ev) (void)hipEventDestroy(c->order_ev);
    if (c->wstage) (void)hipHostFree(c->wstage);
    c->rmap.release();
    c->cmap.release();
    c->omap.release();
    c->zin.release();
    c->zout.release();
    if (c->cr_pinned) {  // GHASH tables of the key: cleared before the pages go back
        volatile uint8_t *z = (volatile uint8_t *)c->cr_pinned;
        for (size_t i = 0; i < kCrTabBytesHost; ++i) z[i] = 0;
        (void)hipHostFree(c->cr_pinned);
    }
    {
        volatile uint8_t *z = c->cr_fp;
        for (int i = 0; i < 32; ++i) z[i] = 0;
    }
    for (auto &ev : c->wev)
        if (ev) (void)hipEventDestroy(ev);
    for (Slot &sl : c->slots) sl.release();
    if (c->slot_pinned) (void)hipHostFree(c->slot_pinned);
    if (c->h2d) (void)hipStreamSynchronize(c->h2d), (void)hipStreamDestroy(c->h2d);
    if (c->d2h) (void)hipStreamSynchronize(c->d2h), (void)hipStreamDestroy(c->d2h);
    if (c->side) (void)hipStreamDestroy(c->side);
    c->svc.mb.release();
    c->svc.ctl.release();
    c->svc.st.release();
    c->svc.bsums.release();
    if (c->svc.s) (void)hipStreamDestroy(c->svc.s);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int iggy_codec_reserve(iggy_codec_ctx *c, uint64_t max_batch_bytes, uint64_t max_frames) {
    if (!c) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    bind(c, nullptr);
    (void)max_frames;
    return ensure_decode_scratch(c, max_batch_bytes);
}

void *iggy_codec_stream(iggy_codec_ctx *c) { return c ? (void *)c->stream : nullptr; }

int iggy_codec_synchronize(iggy_codec_ctx *c) {
    if (!c) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    HIP_OK(hipStreamSynchronize(c->stream));
    for (Slot &sl : c->slots)  // the fast-path submits' own streams
        if (sl.st) HIP_OK(hipStreamSynchronize(sl.st));
    return 0;
}

// iggy_batch_header_decode / _encode and iggy_encoded_batch_size (host pure) live in
// sdk.cpp, which also builds alone for the host sanitizer run (tests/fuzz/).

// -------------------------------------------------------------- profiling
int iggy_codec_host_stats(iggy_codec_ctx *c, iggy_host_stats *out) {
    if (!c || !out) return IGGY_ERR_INVALID_ARGUMENT;
    *out = c->hs;
    out->device_allocs = g_dev_allocs.load(std::memory_order_relaxed);
    out->pinned_allocs = g_pin_allocs.load(std::memory_order_relaxed);
    out->service_posts = c->svc.posts;
    out->service_launches = c->svc.launches;
    return 0;
}

int iggy_codec_service_start(iggy_codec_ctx *c) {
    if (!c) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    return svc_enable(c);
}

int iggy_codec_service_stop(iggy_codec_ctx *c) {
    if (!c) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    return svc_disable(c);
}

int iggy_codec_profile_enable(iggy_codec_ctx *c, int enable) {
    if (!c) return IGGY_ERR_INVALID_ARGUMENT;
    c->profile = enable ? 1 : 0;
    for (int w = 0; w < 2; ++w) {
        c->prof_n[w] = 0;
        c->prof_ms[w] = 0;
        c->ev_pending[w] = false;
    }
    return 0;
}

int iggy_codec_profile_read(iggy_codec_ctx *c, int which, uint64_t *launches, double *total_ms) {
    if (!c || which < 0 || which > 1) return IGGY_ERR_INVALID_ARGUMENT;
    if (c->ev_pending[which]) {
        float ms = 0;
        HIP_OK(hipEventSynchronize(c->ev1[which]));
        if (hipEventElapsedTime(&ms, c->ev0[which], c->ev1[which]) == hipSuccess) {
            c->prof_ms[which] += ms;
            c->prof_n[which] += 1;
        }
        c->ev_pending[which] = false;
    }
    if (launches) *launches = c->prof_n[which];
    if (total_ms) *total_ms = c->prof_ms[which];
    c->prof_n[which] = 0;
    c->prof_ms[which] = 0;
    return 0;
}

// Diagnostics only (not part of include/iggy_codec.h): copy the context's small
// sync scratch (768 B; the decode's dbg-512 stamps live at [256..]) to host.
int iggy_codec_debug_read(iggy_codec_ctx *c, void *out, uint64_t bytes) {
    if (!c || !out) return IGGY_ERR_INVALID_ARGUMENT;
    HIP_OK(hipStreamSynchronize(c->stream));
    HIP_OK(hipDeviceSynchronize());
    return get_host(c, out, c->dsync.as<uint8_t>(kSyncSmall), std::min<uint64_t>(bytes, kSyncBytes - kSyncSmall),
                    c->stream);
}
// Diagnostics only: set the ablation bits of a context (no effect in the product
// build, where kDiagMask is zero).
int iggy_codec_debug_set(iggy_codec_ctx *c, uint32_t bits) {
    if (!c) return IGGY_ERR_INVALID_ARGUMENT;
    if (kDiagMask && (bits & 0x40000000u)) {  // completion-flag sequence 16 values before its wrap
        c->hseq = 0xFFFFFFF0u;
        bits &= ~0x40000000u;
    }
    c->dbg = bits;
    return 0;
}
int iggy_codec_debug_clear(iggy_codec_ctx *c) {
    if (!c) return IGGY_ERR_INVALID_ARGUMENT;
    HIP_OK(hipMemset(c->dsync.as<uint8_t>(kSyncSmall + 256), 0, 512));
    return 0;
}

const char *iggy_codec_error_string(uint32_t kind, uint32_t reason) {
    switch (kind) {
        case IGGY_OK: return "ok";
        case IGGY_ERR_UNEXPECTED_EOF: return "unexpected end of buffer";
        case IGGY_ERR_VALIDATION:
            switch (reason) {
                case IGGY_V_BATCH_LENGTH_SHORT: return "batch length must cover the batch header";
                case IGGY_V_BATCH_RESERVED: return "batch header reserved bytes must be zero";
                case IGGY_V_FRAMES_DO_NOT_TILE: return "batch frames do not tile message_count exactly";
                case IGGY_V_FRAME_RESERVED: return "message frame reserved bytes must be zero";
                case IGGY_V_EMPTY_BATCH: return "cannot encode an empty message batch";
                case IGGY_V_NUMERIC_ID_LENGTH: return "numeric identifier must be 4 bytes";
                case IGGY_V_STRING_ID_EMPTY: return "string identifier cannot be empty";
                case IGGY_V_BALANCED_LENGTH: return "balanced partitioning must have length 0";
                case IGGY_V_PARTITION_ID_LENGTH: return "partition_id partitioning must have length 4";
                case IGGY_V_MESSAGES_KEY_EMPTY: return "messages_key partitioning cannot have empty key";
                default: return "validation failed";
            }
        case IGGY_ERR_INVALID_BATCH_CHECKSUM: return "invalid batch checksum";
        case IGGY_ERR_INVALID_MESSAGE_CHECKSUM: return "invalid message checksum";
        case IGGY_ERR_INVALID_TIMESTAMP_DELTA: return "message timestamp delta exceeds the batch maximum";
        case IGGY_ERR_PAYLOAD_TOO_LARGE: return "payload too large";
        case IGGY_ERR_INVALID_UTF8: return "invalid utf-8";
        case IGGY_ERR_UNKNOWN_DISCRIMINANT: return "unknown discriminant";
        case IGGY_ERR_INVALID_NUMBER_ENCODING: return "invalid number encoding";
        case IGGY_ERR_INVALID_MESSAGE_PAYLOAD_LENGTH: return "invalid message payload length";
        case IGGY_ERR_DEVICE: return "device error";
        case IGGY_ERR_INVALID_ARGUMENT: return "invalid argument";
        case IGGY_ERR_CAPACITY: return "output capacity too small";
        case IGGY_ERR_TIMEOUT: return "device wait timed out";
        default: return "unknown";
    }
}

}  // extern "C"
