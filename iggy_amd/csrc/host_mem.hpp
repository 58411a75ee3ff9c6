// host_mem.hpp -- caller host memory at the boundary: the registry of registered ranges, the
// pinned / pageable classification, staged copies (put_host / get_host) and the
// host-memory history log
//
// Part of the unity build of libiggy_codec.so: included by codec_api.hip, after the
// kernel translation units and the units before it (see codec_api.hip for the order).
#pragma once

namespace {

// ------------------------------------------------------- caller host memory
// Every byte of caller host memory that crosses PCIe goes through put_host / get_host.
// The reference codec borrows `&[u8]` for the call only (batch.rs:391); the caller may
// free or reuse the memory the moment a call returns. Pinned memory (hipHostMalloc,
// hipHostRegister, iggy_codec_host_register: the server's socket and segment buffers)
// is a DMA source / target as it is. PAGEABLE memory is never handed to the runtime's
// copy engine: for such a copy ROCclr pins (locks) the caller's range and releases
// the lock only when it retires the copy command, at a later synchronisation of that
// stream, so a synchronous entry returning on a host flag could leave a lock on memory
// the caller then frees. Pageable bytes are therefore staged through the context's own
// two pinned chunks (memcpy of chunk k+1 under the DMA of chunk k), and no runtime lock
// on caller memory exists. That was round 5's explanation of the hipErrorIllegalAddress
// faults of rounds 3-4, but it does not cover the last one (round 5: torch's own
// pageable copy, no codec call since a device sync). What the round-6 history log found
// in the suite instead: registrations of neighbouring unaligned arrays
// that shared a page, 23 per run, ahead of that module -- now refused by
// iggy_codec_host_register. Neither is proven to be the faults' cause.
constexpr uint64_t kXferChunk = 4ull << 20;
// Ranges registered through iggy_codec_host_register. The registry is process-wide
// (iggy_codec_host_pinned takes no context), but each entry belongs to the context that
// registered it: iggy_codec_destroy unregisters that context's leftovers, so no entry
// outlives its registration. Entries are trusted without a HIP query on every hit: a
// range must be unregistered through the codec (iggy_codec_host_unregister), never with
// a bare hipHostUnregister, or a later lookup would DMA from / map an unpinned range.
std::mutex g_reg_mu;
struct RegRange {
    uintptr_t h;   // host address
    uint64_t len;
    uintptr_t d;   // its device-mapped address on `device` (0: not mapped)
    int device;
    const iggy_codec_ctx *owner;
};
std::vector<RegRange> g_reg;

bool host_pinned(const void *p, uint64_t n) {
    if (!p || !n) return true;
    const uintptr_t a = (uintptr_t)p;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        for (const auto &r : g_reg)
            if (a >= r.h && a - r.h <= r.len && n <= r.len - (a - r.h)) return true;
    }
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable: not an error for the caller's HIP code
        return false;
    }
    if (at.type != hipMemoryTypeHost) return false;
    void *start = nullptr;
    size_t size = 0;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) != hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    // only a range the query reports in host addresses that covers [p, p + n) counts;
    // anything else is staged (always correct, only slower)
    const uintptr_t s0 = (uintptr_t)start;
    return a >= s0 && a - s0 <= size && n <= size - (a - s0);
}

// the device-mapped address of pinned host memory [p, p + n) (nullptr: not pinned or
// not mapped); ranges registered through the codec answer from the registry
const uint8_t *host_device_ptr(const void *p, uint64_t n) {
    const uintptr_t a = (uintptr_t)p;
    int dev = -1;
    (void)hipGetDevice(&dev);  // (the calling entry's DevGuard: the context's device)
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        for (const auto &r : g_reg)
            if (a >= r.h && a - r.h <= r.len && n <= r.len - (a - r.h) && r.device == dev)
                return r.d ? (const uint8_t *)(r.d + (a - r.h)) : nullptr;
    }
    if (!host_pinned(p, n)) return nullptr;
    void *dp = nullptr;
    if (hipHostGetDevicePointer(&dp, (void *)p, 0) != hipSuccess || !dp) {
        (void)hipGetLastError();
        return nullptr;
    }
    return (const uint8_t *)dp;
}

int xfer_init(iggy_codec_ctx *c) {
    if (c->xst) return 0;
    if (hipHostMalloc(&c->xst, 2 * kXferChunk, hipHostMallocDefault) != hipSuccess) {
        c->xst = nullptr;
        return IGGY_ERR_DEVICE;
    }
    for (auto &ev : c->xev)
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return IGGY_ERR_DEVICE;
    return 0;
}

// the next staging chunk, free for the host (its previous copy has run)
int xfer_chunk(iggy_codec_ctx *c, uint8_t **chunk, int *idx) {
    const int b = (int)(c->xnext++ & 1);
    if (c->xlive[b]) {
        c->hs.host_waits++;
        HIP_OK(hipEventSynchronize(c->xev[b]));
        c->xlive[b] = false;
    }
    *chunk = (uint8_t *)c->xst + (size_t)b * kXferChunk;
    *idx = b;
    return 0;
}

// H2D of n caller bytes on stream s. Returns with the caller's bytes consumed as far
// as the caller is concerned: staged into pinned chunks (pageable), or enqueued from
// memory the caller keeps pinned (a plain DMA source: the caller keeps it alive until
// the call, or the ticket, completes; nothing of the runtime's outlives that copy).
// Only a staged copy records xin_ev, the event a synchronous entry settles before it
// returns (xfer_settle): an asynchronous submit of pinned memory issues no event and
// no wait here, so its copy overlaps everything else in flight (round 5 recorded the
// event for every copy, and its H2D / D2H no longer overlapped: C4 24.7 -> 17.6 GiB/s,
// scripts/c4_diag.py).
int put_host(iggy_codec_ctx *c, void *d_dst, const void *h_src, uint64_t n, hipStream_t s) {
    if (!n) return 0;
    if (host_pinned(h_src, n)) {
        HIP_OK(hipMemcpyAsync(d_dst, h_src, n, hipMemcpyHostToDevice, s));
        c->hs.pinned_h2d_bytes += n;
        return 0;
    }
    c->hs.staged_bytes += n;
    if (xfer_init(c)) return IGGY_ERR_DEVICE;
    for (uint64_t off = 0; off < n; off += kXferChunk) {
        const uint64_t m = std::min(kXferChunk, n - off);
        uint8_t *st;
        int b;
        int r = xfer_chunk(c, &st, &b);
        if (r) return r;
        memcpy(st, (const uint8_t *)h_src + off, m);
        HIP_OK(hipMemcpyAsync((uint8_t *)d_dst + off, st, m, hipMemcpyHostToDevice, s));
        HIP_OK(hipEventRecord(c->xev[b], s));
        c->xlive[b] = true;
    }
    if (!c->xin_ev && hipEventCreateWithFlags(&c->xin_ev, hipEventDisableTiming) != hipSuccess) {
        c->xin_ev = nullptr;
        return IGGY_ERR_DEVICE;
    }
    HIP_OK(hipEventRecord(c->xin_ev, s));
    c->hs.settle_events++;
    c->xin_live = true;
    return 0;
}

// Before a synchronous entry that saw its completion through a host-mapped flag (no
// stream sync) returns: its staged H2D copies are done. They ran before the kernel that
// raised the flag, so this costs one signal read (nothing at all after pinned copies).
int xfer_settle(iggy_codec_ctx *c) {
    if (c->xin_live) {
        c->hs.host_waits++;
        HIP_OK(hipEventSynchronize(c->xin_ev));
        c->xin_live = false;
    }
    return 0;
}

// D2H of n bytes into caller memory on stream s; synchronous (returns with the bytes
// in h_dst and nothing of the call outstanding on s).
int get_host(iggy_codec_ctx *c, void *h_dst, const void *d_src, uint64_t n, hipStream_t s) {
    if (!n) return 0;
    c->hs.host_waits++;  // (returns with the bytes in h_dst)
    if (host_pinned(h_dst, n)) {
        HIP_OK(hipMemcpyAsync(h_dst, d_src, n, hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
        return 0;
    }
    if (xfer_init(c)) return IGGY_ERR_DEVICE;
    const uint64_t nk = (n + kXferChunk - 1) / kXferChunk;
    uint8_t *st[2] = {nullptr, nullptr};
    int bi[2] = {0, 0};
    auto issue = [&](uint64_t k) -> int {
        const uint64_t off = k * kXferChunk, m = std::min(kXferChunk, n - off);
        int r = xfer_chunk(c, &st[k & 1], &bi[k & 1]);
        if (r) return r;
        HIP_OK(hipMemcpyAsync(st[k & 1], (const uint8_t *)d_src + off, m, hipMemcpyDeviceToHost, s));
        HIP_OK(hipEventRecord(c->xev[bi[k & 1]], s));
        c->xlive[bi[k & 1]] = true;
        return 0;
    };
    int r = issue(0);
    for (uint64_t k = 0; k < nk && !r; ++k) {
        HIP_OK(hipEventSynchronize(c->xev[bi[k & 1]]));
        c->xlive[bi[k & 1]] = false;
        const uint8_t *src = st[k & 1];
        if (k + 1 < nk) r = issue(k + 1);  // the next chunk's copy runs under this memcpy
        const uint64_t off = k * kXferChunk;
        memcpy((uint8_t *)h_dst + off, src, std::min(kXferChunk, n - off));
    }
    return r;
}

}  // namespace

extern "C" {


// Page-lock a caller range. The runtime pins whole pages, so a range that shares a page
// with another live registration (two unaligned numpy arrays side by side) makes two
// runtime objects over one page; unregistering either one tears down the page's GPU
// mapping under the other, and the runtime's pointer lookup can resolve a later,
// unrelated host pointer in that page to a dead object. The round-3-5 suites registered
// such neighbours 23 times per run before the module that faulted (DESIGN.md §8,
// profiles/r06_hostmem_history.txt), so the codec refuses it: a registration's page
// span [ptr & ~4095, end rounded up) must not meet a live registration's page span
// (the server registers whole 4096-aligned Owned<MESSAGE_ALIGN> buffers, iobuf.rs).
int iggy_codec_host_register(iggy_codec_ctx *c, void *ptr, uint64_t len) {
    if (!c || !ptr || !len) return IGGY_ERR_INVALID_ARGUMENT;
    constexpr uintptr_t kPage = 4096;
    const uintptr_t p0 = (uintptr_t)ptr & ~(kPage - 1), p1 = ((uintptr_t)ptr + len + kPage - 1) & ~(kPage - 1);
    std::lock_guard<std::mutex> lk(g_reg_mu);  // (held across the runtime call: no racing neighbour)
    for (const auto &r : g_reg) {
        const uintptr_t q0 = r.h & ~(kPage - 1), q1 = (r.h + r.len + kPage - 1) & ~(kPage - 1);
        if (p0 < q1 && q0 < p1) {
            hostmem_log("register refused: shares a page with", (const void *)r.h, r.len);
            return IGGY_ERR_INVALID_ARGUMENT;
        }
    }
    DevGuard dg(c->device);
    HIP_OK(hipHostRegister(ptr, len, hipHostRegisterDefault));
    void *dp = nullptr;
    if (hipHostGetDevicePointer(&dp, ptr, 0) != hipSuccess) {
        (void)hipGetLastError();
        dp = nullptr;
    }
    hostmem_log("register", ptr, len);
    g_reg.push_back(RegRange{(uintptr_t)ptr, len, (uintptr_t)dp, c->device, c});
    return 0;
}

int iggy_codec_host_unregister(iggy_codec_ctx *c, void *ptr) {
    if (!c || !ptr) return IGGY_ERR_INVALID_ARGUMENT;
    DevGuard dg(c->device);
    uint64_t len = 0;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        for (size_t i = 0; i < g_reg.size(); ++i)
            if (g_reg[i].h == (uintptr_t)ptr) {
                len = g_reg[i].len;
                g_reg.erase(g_reg.begin() + (long)i);
                break;
            }
    }
    hostmem_log("unregister", ptr, len);
    HIP_OK(hipHostUnregister(ptr));
    return 0;
}

int iggy_codec_host_pinned(const void *ptr, uint64_t len) { return host_pinned(ptr, len) ? 1 : 0; }

}  // extern "C"
