// xs_api.cpp — host side of libxspect_hip.so: bank files, device residency,
// per-handle workspace and the C ABI declared in include/xspect_hip.h.
//
// Bank file layouts (restated; COBS and rbloom are not available offline, see
// DESIGN.md "Oracle" — parity with their real files is unpinned):
//   COBS classic  "COBS:CLASSIC_INDEX" u32 version=1, u32 num_docs, u32 term_size,
//                 u8 canonicalize, u64 signature_size, u64 num_hashes,
//                 num_docs x (name '\n'), "CLASSIC_INDEX",
//                 then signature_size rows of ceil(num_docs/8) bytes
//                 (doc d = byte d>>3, bit d&7).
//   COBS compact  "COBS:COMPACT_INDEX" u32 version=1, u32 term_size, u8 canonicalize,
//                 u64 num_groups, num_groups x (u64 signature_size, u64 num_hashes),
//                 u64 page_size, u32 num_docs, names, "COMPACT_INDEX", zero pad to a
//                 multiple of page_size; then per group signature_size rows of
//                 page_size bytes (group g = docs [8*page_size*g, 8*page_size*(g+1))).
//   rbloom        u64 little-endian K, then the filter bytes (bit i = byte i>>3,
//                 bit i&7).
// On the device every row is padded to a 16, 32 or 64-byte pitch, or to a
// multiple of 128 bytes: one row of a group is whole aligned dwordx4 chunks
// (128 docs each) and never straddles a 128-byte line.
#include "../../include/xspect_hip.h"

#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "xs_internal.h"

using namespace xs;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t _e = (expr);                                                            \
        if (_e != hipSuccess)                                                              \
            return fail(XS_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                        __FILE__, __LINE__);                                               \
    } while (0)

const char kClassicMagic[] = "CLASSIC_INDEX";
const char kCompactMagic[] = "COMPACT_INDEX";
constexpr uint64_t kPad = 64;  // spare bytes after staged host reads

// Device bytes a handle's workspace holds now and has held at most at once
// (xs_bank_workspace_bytes).
struct WsAcct {
    uint64_t held = 0, peak = 0;
};

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    WsAcct* acct = nullptr;  // the owning handle's workspace tally, if any
    // Workspace buffers of a bank handle: every enqueue that touches them ends
    // with a record of the handle's ws_ev (ws_leave), so waiting for that event
    // is enough before freeing the old buffer on growth.  Buffers without a
    // guard wait for the device.
    const hipEvent_t* guard_ev = nullptr;
    const bool* guard_used = nullptr;
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return XS_OK;
        if (p) {
            // Growth only: work queued earlier on any stream (a device query on
            // the caller's stream) may still read the old buffer.
            if (guard_ev) {
                if (*guard_used) (void)hipEventSynchronize(*guard_ev);
            } else {
                (void)hipDeviceSynchronize();
            }
            (void)hipFree(p);
            if (acct) acct->held -= cap;
        }
        p = nullptr;
        cap = 0;
        size_t want = bytes < 256 ? 256 : bytes;
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess)
            return fail(XS_ERR_HIP, "hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
        cap = want;
        if (acct) acct->peak = std::max(acct->peak, acct->held += want);
        return XS_OK;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
    // give the memory back now (the caller has synchronised every stream that used it)
    void release() {
        if (p) (void)hipFree(p);
        if (acct) acct->held -= cap;
        p = nullptr;
        cap = 0;
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// Pinned host staging for large device -> pageable-host copies.
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap && p) return XS_OK;
        xs::pinned_free(p);
        p = nullptr;
        cap = 0;
        if (int rc = xs::pinned_alloc(bytes, &p)) return rc;
        cap = bytes;
        return XS_OK;
    }
    ~PinnedBuf() { xs::pinned_free(p); }
};

// memcpy on up to `threads` host threads.
void par_memcpy(void* dst, const void* src, size_t n, int threads) {
    if (n < (4u << 20) || threads <= 1) {
        memcpy(dst, src, n);
        return;
    }
    const size_t per = (n + threads - 1) / threads;
    const int T = (int)((n + per - 1) / per);
    xs::parallel_for(T, [=](int t) {
        const size_t a = per * (size_t)t;
        memcpy(static_cast<char*>(dst) + a, static_cast<const char*>(src) + a, std::min(per, n - a));
    });
}

// Ask for transparent huge pages over the page-aligned part of a pageable
// host destination the library is about to fill.  On the MI355X boxes the
// first write to fresh 4 KiB pages costs ~70 ms per 400 MB from one thread and
// ~34 ms from eight (the faults serialise); over 2 MiB pages it is ~25 ms from
// one thread and ~3.6 ms from eight (profiles/r05k_thp.json,
// tools/thp_probe.py), and the copy-out already writes from eight threads.
// Advisory only: pages already present stay as they are, and a mapping that
// cannot take the advice (file-backed, hugetlbfs) is left alone.
void advise_huge_pages(void* p, size_t bytes) {
    constexpr uintptr_t kPage = 4096;
    const uintptr_t a = (reinterpret_cast<uintptr_t>(p) + kPage - 1) & ~(kPage - 1);
    const uintptr_t e = (reinterpret_cast<uintptr_t>(p) + bytes) & ~(kPage - 1);
    if (e > a + (4u << 20)) (void)madvise(reinterpret_cast<void*>(a), e - a, MADV_HUGEPAGE);
}

}  // namespace

struct xs_bank {
    int kind = 0;
    int device = 0;
    uint32_t k = 0, h = 0, canonicalize = 1;
    uint64_t D = 0, G = 0, page = 0;
    std::vector<uint64_t> sig;
    std::vector<std::string> names;
    // device image
    uint64_t pitch = 0;  // COBS: padded bytes per row
    uint64_t dev_bytes = 0;
    uint64_t nbytes = 0;  // rbloom filter bytes
    WsAcct ws_acct;       // the workspace buffers below (not the image)
    DevBuf image;
    DevBuf groups;
    hipStream_t stream = nullptr;
    std::mutex mu;
    // workspace
    DevBuf seqs, offs, nseg, unit_ofs, unit_read, n_units, scan_tmp, nk, hits, partials, totals, tmp,
        best, narrow, ovf;
    DevBuf rows_read;               // profiling: filter words the rbloom probe loaded
    DevBuf pk_nkc, pk_kofs, pk_scan, pk_entries, pk_tbl, pk_miss, pk_aux;  // partitioned probes (rbloom, COBS)
    // rbloom path choice: member fraction of the last query whose totals have
    // landed (members, k-mers), copied back asynchronously after every query
    DevBuf bloom_tot;
    PinnedBuf bloom_tot_h;
    hipEvent_t bloom_ev = nullptr;
    bool bloom_pending = false;
    double member_frac = 1.0;
    int last_path = XS_PATH_GATHER;
    ProbeOptions opt;               // path selection (xs_bank_set_probe_options)
    PinnedBuf stage[3];             // D2H staging ring for large host outputs (d2h_pageable: 2, HitSink: 3)
    hipEvent_t stage_ev[3] = {nullptr, nullptr, nullptr};
    PinnedBuf hstage[2];            // H2D staging ring for host read batches
    PinnedBuf small_h;              // small host calls: the whole request and its results (query_small)
    PinnedBuf cut_ofs;              // device-read batches: read offsets at the chunk cuts
    PinnedBuf offs_h;               // host batches: the read offsets rebased to 0, for their H2D copy
    DevBuf small_d;
    hipEvent_t hstage_ev[2] = {nullptr, nullptr};
    hipStream_t copy_stream = nullptr, d2h_stream = nullptr;
    std::vector<hipEvent_t> chunk_ev;  // probe of batch chunk i done
    // The workspace above is shared by every query and build on the handle.  A
    // call enqueued on a different stream than the previous one waits for that
    // one's work on the device (ws_ev), so callers may mix streams freely.
    hipEvent_t ws_ev = nullptr;
    hipStream_t ws_stream = nullptr;
    bool ws_used = false;
    bool profiling = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;  // one pair per profiled probe
    size_t events_used = 0;
    std::vector<hipEvent_t> pass_ev;  // profiling: pass boundaries of the partitioned probes
    std::vector<int> pass_tag;
    size_t pass_used = 0;

    xs_bank() {
        for (DevBuf* d : {&seqs, &offs, &nseg, &unit_ofs, &unit_read, &n_units, &scan_tmp, &nk, &hits, &partials,
                          &totals, &tmp, &best, &narrow, &ovf, &rows_read, &pk_nkc, &pk_kofs, &pk_scan, &pk_entries, &pk_tbl,
                          &pk_miss, &pk_aux, &bloom_tot}) {
            d->guard_ev = &ws_ev;
            d->guard_used = &ws_used;
            d->acct = &ws_acct;
        }
        small_d.acct = &ws_acct;
    }

    uint64_t sig_total() const {
        uint64_t s = 0;
        for (auto v : sig) s += v;
        return s;
    }
    uint64_t payload_bytes() const {
        return kind == XS_BANK_RBLOOM ? nbytes : sig_total() * page;
    }
    CobsView cobs_view() const {
        CobsView v;
        v.rows = image.as<uint8_t>();
        v.groups = groups.as<GroupDesc>();
        v.G = (uint32_t)G;
        v.pitch = (uint32_t)pitch;
        v.nchunks = (uint32_t)((page + 15) / 16);  // chunks that hold doc bits
        v.h = h;
        v.page = page;
        v.D = D;
        v.sig0 = sig.empty() ? 0 : sig[0];
        v.sig_max = 0;
        for (auto x : sig) v.sig_max = x > v.sig_max ? x : v.sig_max;
        return v;
    }
    BloomView bloom_view() const {
        BloomView v;
        v.bits = image.as<uint32_t>();
        v.mbits = nbytes * 8;
        v.magic = barrett_magic(v.mbits);
        v.K = h;
        v.rows_read = profiling ? rows_read.as<uint64_t>() : nullptr;
        return v;
    }
};

namespace {

// Order the handle's next enqueue on stream s after its previous one.
int ws_enter(xs_bank* b, hipStream_t s) {
    if (b->ws_used && b->ws_stream != s) HIPCHK(hipStreamWaitEvent(s, b->ws_ev, 0));
    return XS_OK;
}
int ws_leave(xs_bank* b, hipStream_t s) {
    if (!b->ws_ev) HIPCHK(hipEventCreateWithFlags(&b->ws_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(b->ws_ev, s));
    b->ws_stream = s;
    b->ws_used = true;
    return XS_OK;
}

int validate_geometry(xs_bank* b) {
    if (b->k < 1 || b->k > kMaxK)
        return fail(XS_ERR_UNSUPPORTED, "term_size %u unsupported on the device (1..%u)", b->k, kMaxK);
    if (b->h < 1 || b->h > kMaxHashes)
        return fail(XS_ERR_UNSUPPORTED, "num_hashes %u unsupported on the device (1..%u)", b->h,
                    kMaxHashes);
    if (b->kind == XS_BANK_RBLOOM) {
        if (b->nbytes == 0) return fail(XS_ERR_FORMAT, "empty rbloom filter");
        return XS_OK;
    }
    if (b->D == 0) return fail(XS_ERR_FORMAT, "bank has no documents");
    if (b->page == 0 || b->G == 0 || b->sig.size() != b->G)
        return fail(XS_ERR_FORMAT, "bad group geometry");
    if (b->G * 8 * b->page < b->D || (b->G - 1) * 8 * b->page >= b->D)
        return fail(XS_ERR_FORMAT, "groups (%llu x %llu bytes) do not match %llu docs",
                    (unsigned long long)b->G, (unsigned long long)b->page,
                    (unsigned long long)b->D);
    for (auto s : b->sig)
        if (s == 0) return fail(XS_ERR_FORMAT, "zero signature size");
    // Device row pitch: 16, 32, 64 or a multiple of 128 bytes, so that no row
    // straddles a 128-byte line (a 48-byte pitch made 2 rows in 8 cost two
    // line fills).  The kernels load only the (page + 15) / 16 data chunks.
    const uint64_t p16 = (b->page + 15) / 16 * 16;
    b->pitch = p16 <= 64 ? (p16 <= 16 ? 16 : p16 <= 32 ? 32 : 64) : (p16 + 127) / 128 * 128;
    int wpb;
    size_t lds;
    if (probe_blocks(b->D, &wpb, &lds) != 0)
        return fail(XS_ERR_UNSUPPORTED, "%llu documents exceed the LDS counter budget",
                    (unsigned long long)b->D);
    return XS_OK;
}

// Allocate the (zeroed) device image and group table.
int alloc_image(xs_bank* b) {
    HIPCHK(hipSetDevice(b->device));
    if (!b->stream) HIPCHK(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
    if (b->kind == XS_BANK_RBLOOM) {
        b->dev_bytes = (b->nbytes + 15) / 16 * 16 + 16;
        if (int rc = b->image.ensure(b->dev_bytes)) return rc;
        HIPCHK(hipMemsetAsync(b->image.p, 0, b->dev_bytes, b->stream));
    } else {
        b->dev_bytes = b->sig_total() * b->pitch;
        if (int rc = b->image.ensure(b->dev_bytes)) return rc;
        HIPCHK(hipMemsetAsync(b->image.p, 0, b->dev_bytes, b->stream));
        std::vector<GroupDesc> gd(b->G);
        uint64_t base = 0;
        for (uint64_t g = 0; g < b->G; ++g) {
            gd[g].sig = b->sig[g];
            gd[g].magic = barrett_magic(b->sig[g]);
            gd[g].base = base;
            base += b->sig[g] * b->pitch;
        }
        if (int rc = b->groups.ensure(sizeof(GroupDesc) * b->G)) return rc;
        HIPCHK(hipMemcpyAsync(b->groups.p, gd.data(), sizeof(GroupDesc) * b->G,
                              hipMemcpyHostToDevice, b->stream));
    }
    HIPCHK(hipStreamSynchronize(b->stream));
    return XS_OK;
}

// FILE layout payload (host) -> device image.
int upload_payload(xs_bank* b, const void* host, uint64_t nbytes) {
    if (nbytes != b->payload_bytes())
        return fail(XS_ERR_ARG, "payload of %llu bytes, bank expects %llu",
                    (unsigned long long)nbytes, (unsigned long long)b->payload_bytes());
    HIPCHK(hipSetDevice(b->device));
    if (int rc = ws_enter(b, b->stream)) return rc;
    if (b->kind == XS_BANK_RBLOOM) {
        HIPCHK(hipMemcpyAsync(b->image.p, host, nbytes, hipMemcpyHostToDevice, b->stream));
    } else if (b->pitch == b->page) {
        HIPCHK(hipMemcpyAsync(b->image.p, host, nbytes, hipMemcpyHostToDevice, b->stream));
    } else {
        if (int rc = b->tmp.ensure(nbytes)) return rc;
        HIPCHK(hipMemcpyAsync(b->tmp.p, host, nbytes, hipMemcpyHostToDevice, b->stream));
        HIPCHK(launch_repack(b->tmp.as<uint8_t>(), b->page, b->image.as<uint8_t>(), b->pitch,
                             b->sig_total(), b->page, b->stream));
    }
    HIPCHK(hipStreamSynchronize(b->stream));
    return XS_OK;
}

int download_payload(xs_bank* b, void* host, uint64_t nbytes) {
    if (nbytes != b->payload_bytes())
        return fail(XS_ERR_ARG, "buffer of %llu bytes, payload is %llu",
                    (unsigned long long)nbytes, (unsigned long long)b->payload_bytes());
    HIPCHK(hipSetDevice(b->device));
    if (int rc = ws_enter(b, b->stream)) return rc;
    if (b->kind == XS_BANK_RBLOOM || b->pitch == b->page) {
        HIPCHK(hipMemcpyAsync(host, b->image.p, nbytes, hipMemcpyDeviceToHost, b->stream));
    } else {
        if (int rc = b->tmp.ensure(nbytes)) return rc;
        HIPCHK(launch_repack(b->image.as<uint8_t>(), b->pitch, b->tmp.as<uint8_t>(), b->page,
                             b->sig_total(), b->page, b->stream));
        HIPCHK(hipMemcpyAsync(host, b->tmp.p, nbytes, hipMemcpyDeviceToHost, b->stream));
    }
    HIPCHK(hipStreamSynchronize(b->stream));
    return XS_OK;
}

// ---- bank payloads straight from their files ------------------------------
// A model load (ProbabilisticFilterModel.load, probabilistic_filter_model.py:
// 351-391: cobs.Search(path) reads the whole index) moved the payload through
// a zero-filled std::vector, one ifstream read and a pageable H2D copy: 169 ms
// for config 2's 0.5 GB file (2.9 GB/s, profiles/r05q_open.json).  Here the
// file is read in pieces by up to 8 threads (pread) into a ring of pinned
// slots, each piece sent by DMA while the next is read.
constexpr uint64_t kLoadPiece = 32u << 20;
constexpr int kLoadSlots = 3;

// run(a, e, &ok) over the ranges of [0, n) of up to `threads` (<= 8) threads, at least
// 4 MiB each; false if any range failed
template <class F>
bool par_io(uint64_t n, int threads, F run) {
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)threads, 8, n / (4u << 20)}));
    const uint64_t per = (n + T - 1) / T;
    bool ok[8] = {true, true, true, true, true, true, true, true};
    xs::parallel_for(T, [&](int t) {
        const uint64_t a = per * (uint64_t)t;
        if (a < n) run(a, std::min(n, a + per), &ok[t]);
    });
    for (bool o : ok)
        if (!o) return false;
    return true;
}

// [off, off + n) of fd into dst, split over up to `threads` threads; false on a
// read error or a short file
bool pread_all(int fd, uint8_t* dst, uint64_t n, uint64_t off, int threads) {
    auto run = [=](uint64_t a, uint64_t e, bool* ok) {
        while (a < e) {
            const ssize_t got = pread(fd, dst + a, (size_t)(e - a), (off_t)(off + a));
            if (got <= 0) {
                if (got < 0 && errno == EINTR) continue;
                *ok = false;
                return;
            }
            a += (uint64_t)got;
        }
        *ok = true;
    };
    return par_io(n, threads, run);
}

// nbytes of `path` from byte `pos`, in pieces of `piece` bytes (the last one shorter) read by
// up to 8 threads into a ring of pinned slots; emit(off, m, slot) enqueues piece [off, off + m)'s
// transfer out of its slot on b->stream, which is synchronised on return
template <class Emit>
int stream_file(xs_bank* b, const char* path, uint64_t pos, uint64_t nbytes, uint64_t piece, Emit emit) {
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return fail(XS_ERR_IO, "cannot open %s", path);
    struct Closer {
        int fd;
        ~Closer() { ::close(fd); }
    } closer{fd};
    PinnedBuf ring[kLoadSlots];
    hipEvent_t ev[kLoadSlots] = {};
    // on every exit path: no DMA may still read a slot when the ring is freed
    struct Drain {
        hipStream_t s;
        hipEvent_t* ev;
        ~Drain() {
            (void)hipStreamSynchronize(s);
            for (int i = 0; i < kLoadSlots; ++i)
                if (ev[i]) (void)hipEventDestroy(ev[i]);
        }
    } drain{b->stream, ev};
    piece = std::min<uint64_t>(piece, std::max<uint64_t>(nbytes, 1));
    for (int i = 0; i < kLoadSlots; ++i) {
        if (int rc = ring[i].ensure(piece)) return rc;
        HIPCHK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    }
    const int threads = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    uint64_t i = 0;
    for (uint64_t off = 0; off < nbytes; off += piece, ++i) {
        const int s = (int)(i % kLoadSlots);
        if (i >= (uint64_t)kLoadSlots) HIPCHK(hipEventSynchronize(ev[s]));  // the slot's last DMA is done
        const uint64_t m = std::min(piece, nbytes - off);
        if (!pread_all(fd, static_cast<uint8_t*>(ring[s].p), m, pos + off, threads))
            return fail(XS_ERR_IO, "%s: short read", path);
        HIPCHK(emit(off, m, static_cast<const uint8_t*>(ring[s].p)));
        HIPCHK(hipEventRecord(ev[s], b->stream));
    }
    HIPCHK(hipStreamSynchronize(b->stream));
    return XS_OK;
}

// nbytes of `path` from byte `pos` to the device at dst, on b->stream (synchronised on return)
int stream_file_to_device(xs_bank* b, const char* path, uint64_t pos, uint64_t nbytes, uint8_t* dst) {
    return stream_file(b, path, pos, nbytes, kLoadPiece, [&](uint64_t off, uint64_t m, const uint8_t* src) {
        return hipMemcpyAsync(dst + off, src, m, hipMemcpyHostToDevice, b->stream);
    });
}

// [off, off + n) of fd from src, split over up to `threads` threads; false on a write error
bool pwrite_all(int fd, const uint8_t* src, uint64_t n, uint64_t off, int threads) {
    auto run = [=](uint64_t a, uint64_t e, bool* ok) {
        while (a < e) {
            const ssize_t put = pwrite(fd, src + a, (size_t)(e - a), (off_t)(off + a));
            if (put <= 0) {
                if (put < 0 && errno == EINTR) continue;
                *ok = false;
                return;
            }
            a += (uint64_t)put;
        }
        *ok = true;
    };
    return par_io(n, threads, run);
}

// nbytes of the device buffer src to `path` from byte `pos` (the header before it is
// already written): pieces come back by DMA into a ring of pinned slots and are written
// by up to 8 threads while the next pieces cross
int stream_device_to_file(xs_bank* b, const char* path, uint64_t pos, uint64_t nbytes, const uint8_t* src) {
    const int fd = ::open(path, O_WRONLY | O_CLOEXEC);
    if (fd < 0) return fail(XS_ERR_IO, "cannot open %s for writing", path);
    struct Closer {  // an error path's close; the success path closes (and checks) below
        int fd;
        ~Closer() {
            if (fd >= 0) ::close(fd);
        }
    } closer{fd};
    PinnedBuf ring[kLoadSlots];
    hipEvent_t ev[kLoadSlots] = {};
    struct Drain {  // on every exit path: no DMA may still write a slot when the ring is freed
        hipStream_t s;
        hipEvent_t* ev;
        ~Drain() {
            (void)hipStreamSynchronize(s);
            for (int i = 0; i < kLoadSlots; ++i)
                if (ev[i]) (void)hipEventDestroy(ev[i]);
        }
    } drain{b->stream, ev};
    const uint64_t piece = std::min<uint64_t>(kLoadPiece, std::max<uint64_t>(nbytes, 1));
    for (int i = 0; i < kLoadSlots; ++i) {
        if (int rc = ring[i].ensure(piece)) return rc;
        HIPCHK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    }
    const int threads = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    const uint64_t pieces = (nbytes + piece - 1) / piece;
    auto queue = [&](uint64_t i) -> hipError_t {
        const int s = (int)(i % kLoadSlots);
        const uint64_t off = i * piece, m = std::min(piece, nbytes - off);
        hipError_t e = hipMemcpyAsync(ring[s].p, src + off, m, hipMemcpyDeviceToHost, b->stream);
        return e == hipSuccess ? hipEventRecord(ev[s], b->stream) : e;
    };
    for (uint64_t i = 0; i < std::min<uint64_t>(pieces, kLoadSlots); ++i) HIPCHK(queue(i));
    for (uint64_t i = 0; i < pieces; ++i) {
        const int s = (int)(i % kLoadSlots);
        HIPCHK(hipEventSynchronize(ev[s]));
        const uint64_t off = i * piece, m = std::min(piece, nbytes - off);
        if (!pwrite_all(fd, static_cast<const uint8_t*>(ring[s].p), m, pos + off, threads))
            return fail(XS_ERR_IO, "write to %s failed", path);
        if (i + kLoadSlots < pieces) HIPCHK(queue(i + kLoadSlots));
    }
    closer.fd = -1;
    if (::close(fd) != 0) return fail(XS_ERR_IO, "write to %s failed: %s", path, strerror(errno));
    return XS_OK;
}

// The bank's payload in file layout to `path` from byte `pos`.
int write_file_payload(xs_bank* b, const char* path, uint64_t pos) {
    const uint64_t nbytes = b->payload_bytes();
    HIPCHK(hipSetDevice(b->device));
    if (int rc = ws_enter(b, b->stream)) return rc;
    if (b->kind == XS_BANK_RBLOOM || b->pitch == b->page)
        return stream_device_to_file(b, path, pos, nbytes, b->image.as<uint8_t>());
    if (int rc = b->tmp.ensure(nbytes)) return rc;
    HIPCHK(launch_repack(b->image.as<uint8_t>(), b->pitch, b->tmp.as<uint8_t>(), b->page, b->sig_total(), b->page,
                         b->stream));
    return stream_device_to_file(b, path, pos, nbytes, b->tmp.as<uint8_t>());
}

// The bank's payload (the file's bytes after the header, at `pos`) into its image.
int upload_file_payload(xs_bank* b, const char* path, uint64_t pos) {
    const uint64_t nbytes = b->payload_bytes();
    HIPCHK(hipSetDevice(b->device));
    if (int rc = ws_enter(b, b->stream)) return rc;
    if (b->kind == XS_BANK_RBLOOM || b->pitch == b->page)
        return stream_file_to_device(b, path, pos, nbytes, b->image.as<uint8_t>());
    if (int rc = b->tmp.ensure(nbytes)) return rc;
    if (int rc = stream_file_to_device(b, path, pos, nbytes, b->tmp.as<uint8_t>())) return rc;
    HIPCHK(launch_repack(b->tmp.as<uint8_t>(), b->page, b->image.as<uint8_t>(), b->pitch, b->sig_total(), b->page,
                         b->stream));
    HIPCHK(hipStreamSynchronize(b->stream));
    return XS_OK;
}

// ---- little binary reader -------------------------------------------------
struct Reader {
    std::ifstream f;
    bool ok = true;
    template <class T>
    T get() {
        T v{};
        f.read(reinterpret_cast<char*>(&v), sizeof(T));
        if (!f) ok = false;
        return v;
    }
    bool expect(const char* s) {
        std::string got(strlen(s), '\0');
        f.read(&got[0], (std::streamsize)got.size());
        if (!f || got != s) ok = false;
        return ok;
    }
    std::string line() {
        std::string s;
        if (!std::getline(f, s)) ok = false;
        return s;
    }
};

template <class T>
void put(std::ofstream& o, T v) {
    o.write(reinterpret_cast<const char*>(&v), sizeof(T));
}

int read_cobs_header(xs_bank* b, Reader& rd, const char* path) {
    if (!rd.expect("COBS:")) return fail(XS_ERR_FORMAT, "%s: not a COBS index", path);
    if (b->kind == XS_BANK_COBS_CLASSIC) {
        if (!rd.expect(kClassicMagic)) return fail(XS_ERR_FORMAT, "%s: not a classic index", path);
        const uint32_t ver = rd.get<uint32_t>();
        const uint32_t nd = rd.get<uint32_t>();
        b->k = rd.get<uint32_t>();
        b->canonicalize = rd.get<uint8_t>();
        const uint64_t s = rd.get<uint64_t>();
        b->h = (uint32_t)rd.get<uint64_t>();
        if (!rd.ok || ver != 1) return fail(XS_ERR_FORMAT, "%s: bad classic header", path);
        b->D = nd;
        b->G = 1;
        b->page = (nd + 7) / 8;
        b->sig.assign(1, s);
        for (uint32_t i = 0; i < nd; ++i) b->names.push_back(rd.line());
        if (!rd.expect(kClassicMagic)) return fail(XS_ERR_FORMAT, "%s: bad classic trailer", path);
    } else {
        if (!rd.expect(kCompactMagic)) return fail(XS_ERR_FORMAT, "%s: not a compact index", path);
        const uint32_t ver = rd.get<uint32_t>();
        b->k = rd.get<uint32_t>();
        b->canonicalize = rd.get<uint8_t>();
        const uint64_t G = rd.get<uint64_t>();
        if (!rd.ok || ver != 1 || G == 0 || G > (1u << 20))
            return fail(XS_ERR_FORMAT, "%s: bad compact header", path);
        b->G = G;
        for (uint64_t g = 0; g < G; ++g) {
            b->sig.push_back(rd.get<uint64_t>());
            const uint32_t hg = (uint32_t)rd.get<uint64_t>();
            if (g == 0) b->h = hg;
            else if (hg != b->h) return fail(XS_ERR_FORMAT, "%s: mixed num_hashes", path);
        }
        b->page = rd.get<uint64_t>();
        const uint32_t nd = rd.get<uint32_t>();
        b->D = nd;
        for (uint32_t i = 0; i < nd; ++i) b->names.push_back(rd.line());
        if (!rd.expect(kCompactMagic)) return fail(XS_ERR_FORMAT, "%s: bad compact trailer", path);
        if (b->page == 0) return fail(XS_ERR_FORMAT, "%s: zero page size", path);
        const uint64_t pos = (uint64_t)rd.f.tellg();
        const uint64_t pad = (b->page - pos % b->page) % b->page;
        rd.f.seekg((std::streamoff)(pos + pad));
    }
    if (!rd.ok) return fail(XS_ERR_FORMAT, "%s: truncated header", path);
    if (b->canonicalize != 1)
        return fail(XS_ERR_UNSUPPORTED, "%s: non-canonical COBS indices are not supported", path);
    return XS_OK;
}

int write_cobs_file(xs_bank* b, const char* path) {
    std::ofstream o(path, std::ios::binary | std::ios::trunc);
    if (!o) return fail(XS_ERR_IO, "cannot open %s for writing", path);
    o.write("COBS:", 5);
    if (b->kind == XS_BANK_COBS_CLASSIC) {
        o.write(kClassicMagic, (std::streamsize)strlen(kClassicMagic));
        put<uint32_t>(o, 1);
        put<uint32_t>(o, (uint32_t)b->D);
        put<uint32_t>(o, b->k);
        put<uint8_t>(o, (uint8_t)b->canonicalize);
        put<uint64_t>(o, b->sig[0]);
        put<uint64_t>(o, b->h);
        for (auto& n : b->names) o << n << '\n';
        o.write(kClassicMagic, (std::streamsize)strlen(kClassicMagic));
    } else {
        o.write(kCompactMagic, (std::streamsize)strlen(kCompactMagic));
        put<uint32_t>(o, 1);
        put<uint32_t>(o, b->k);
        put<uint8_t>(o, (uint8_t)b->canonicalize);
        put<uint64_t>(o, b->G);
        for (uint64_t g = 0; g < b->G; ++g) {
            put<uint64_t>(o, b->sig[g]);
            put<uint64_t>(o, b->h);
        }
        put<uint64_t>(o, b->page);
        put<uint32_t>(o, (uint32_t)b->D);
        for (auto& n : b->names) o << n << '\n';
        o.write(kCompactMagic, (std::streamsize)strlen(kCompactMagic));
        const uint64_t pos = (uint64_t)o.tellp();
        const uint64_t pad = (b->page - pos % b->page) % b->page;
        std::vector<char> z(pad, 0);
        o.write(z.data(), (std::streamsize)pad);
    }
    const uint64_t pos = (uint64_t)o.tellp();
    o.close();
    if (!o) return fail(XS_ERR_IO, "write to %s failed", path);
    return write_file_payload(b, path, pos);  // the payload after the header, streamed from the device
}

int write_bloom_file(xs_bank* b, const char* path) {
    std::ofstream o(path, std::ios::binary | std::ios::trunc);
    if (!o) return fail(XS_ERR_IO, "cannot open %s for writing", path);
    put<uint64_t>(o, b->h);
    o.close();
    if (!o) return fail(XS_ERR_IO, "write to %s failed", path);
    return write_file_payload(b, path, 8);
}

// ---- query / build pipeline --------------------------------------------------
struct Inputs {
    const uint8_t* seqs;
    uint64_t seq_bytes;      // readable bytes from seqs (window loads stop there)
    const uint64_t* offs;
    uint64_t n;
    uint64_t read_bytes = 0;  // bytes of these n reads (plans and bounds); 0: seq_bytes
    uint64_t plan_bytes() const { return read_bytes ? read_bytes : seq_bytes; }
};

// Unit decomposition (k-mer counts, units, unit -> read map) for n device-resident reads.
// units = false (the partitioned COBS probe, which maps k-mers to reads itself and
// zeroes the hit matrix): only the per-read k-mer counts, when the caller wants them.
int prepare_units(xs_bank* b, const Inputs& in, uint32_t step, uint64_t* d_nk, uint32_t* hits_zero,
                  uint64_t zero_cols, hipStream_t s, ReadView* rv, bool units = true) {
    if (int rc = b->nseg.ensure((in.n + 1) * 8)) return rc;
    if (int rc = b->unit_ofs.ensure((in.n + 1) * 8)) return rc;
    if (int rc = b->n_units.ensure(2 * sizeof(uint64_t))) return rc;
    const uint64_t unit_bound = in.n + in.plan_bytes() / kSegKmers + 1;
    if (int rc = b->unit_read.ensure(unit_bound * 4)) return rc;
    const size_t tb = scan_temp_bytes(in.n ? in.n : 1);
    if (int rc = b->scan_tmp.ensure(tb)) return rc;
    if (units || d_nk) HIPCHK(launch_units(in.offs, in.n, b->k, step, d_nk, b->nseg.as<uint64_t>(), s));
    if (units) {
        HIPCHK(launch_scan(b->scan_tmp.p, b->scan_tmp.cap, b->nseg.as<uint64_t>(),
                           b->unit_ofs.as<uint64_t>(), in.n, s));
        HIPCHK(launch_scatter_units(b->nseg.as<uint64_t>(), b->unit_ofs.as<uint64_t>(), in.n,
                                    b->unit_read.as<uint32_t>(), b->n_units.as<uint64_t>(), hits_zero,
                                    zero_cols, s));
    }
    rv->seq = in.seqs;
    rv->seq_bytes = in.seq_bytes;
    rv->offs = in.offs;
    rv->unit_read = b->unit_read.as<uint32_t>();
    rv->unit_ofs = b->unit_ofs.as<uint64_t>();
    rv->queue = b->n_units.as<uint64_t>();
    rv->n = in.n;
    rv->k = b->k;
    rv->step = step;
    return XS_OK;
}

int probe_grid(xs_bank* b) {
    HIPCHK(hipSetDevice(b->device));
    const int g = b->kind == XS_BANK_RBLOOM ? probe_grid_bloom() : probe_grid_cobs(b->cobs_view(), b->k);
    return g > 0 ? g : 1;
}

// Enqueue one query on device buffers.  d_totals: D+1 entries (or 2 for rbloom).
int run_query(xs_bank* b, const Inputs& in, uint32_t step, uint32_t* d_hits, uint64_t* d_nk,
              uint64_t* d_totals, hipStream_t s) {
    if (step == 0) return fail(XS_ERR_ARG, "step must be >= 1");
    if (in.n >= (1ull << 31)) return fail(XS_ERR_ARG, "at most 2^31-1 reads per call");
    const uint64_t cols = b->kind == XS_BANK_RBLOOM ? 1 : b->D;
    if (int rc = ws_enter(b, s)) return rc;
    const bool bloom = b->kind == XS_BANK_RBLOOM;
    // the COBS path is chosen first: the partitioned probe needs no unit map
    CobsPartPlan cplan;
    bool cobs_part = false;
    if (!bloom) {
        cobs_part = cobs_part_plan(b->cobs_view(), b->k, in.n, in.plan_bytes(), step, b->opt, &cplan) &&
                    !(b->pk_nkc.ensure(cplan.nkc_bytes) || b->pk_kofs.ensure(cplan.nkc_bytes) ||
                      b->pk_scan.ensure(cplan.scan_bytes) || b->pk_entries.ensure(cplan.entry_bytes) ||
                      b->pk_tbl.ensure(cplan.tbl_bytes) || b->pk_aux.ensure(cplan.aux_bytes));
        (void)hipGetLastError();  // a workspace that did not fit: the direct probe
    }
    ReadView rv;
    if (int rc = prepare_units(b, in, step, d_nk, d_hits, cols, s, &rv, !cobs_part)) return rc;
    const int blocks = probe_grid(b);
    uint64_t* partials = nullptr;
    const uint64_t pcols = b->kind == XS_BANK_RBLOOM ? 2 : b->D + 1;
    if (d_totals || bloom) {  // rbloom always: its totals steer the next query's path
        if (int rc = b->partials.ensure((size_t)blocks * pcols * 8)) return rc;
        partials = b->partials.as<uint64_t>();
    }
    if (bloom && b->bloom_pending) {
        const hipError_t q = hipEventQuery(b->bloom_ev);
        (void)hipGetLastError();  // hipErrorNotReady is not an error here
        if (q == hipSuccess) {
            const uint64_t* t = static_cast<const uint64_t*>(b->bloom_tot_h.p);
            if (t[1]) b->member_frac = (double)t[0] / (double)t[1];
            b->bloom_pending = false;
        }
    }
    // probe events: at most kPassMarksMax queries between two xs_bank_probe_stats
    const bool timed = b->profiling && b->events_used < kPassMarksMax;
    if (timed) {
        if (b->events_used == b->events.size()) {
            hipEvent_t a, c;
            HIPCHK(hipEventCreate(&a));
            HIPCHK(hipEventCreate(&c));
            b->events.emplace_back(a, c);
        }
        HIPCHK(hipEventRecord(b->events[b->events_used].first, s));
    }
    BloomPartPlan plan;
    int path = XS_PATH_GATHER;
    // The partitioned path's workspace is transient: when HBM cannot hold it,
    // the query takes the gather path instead of failing.
    auto part_ws = [&]() -> bool {
        if (b->pk_nkc.ensure(plan.nkc_bytes) || b->pk_kofs.ensure(plan.nkc_bytes) ||
            b->pk_scan.ensure(plan.scan_bytes) || b->pk_entries.ensure(plan.entry_bytes) ||
            b->pk_tbl.ensure(plan.tbl_bytes) || b->pk_miss.ensure(plan.miss_bytes) || b->pk_aux.ensure(plan.aux_bytes)) {
            (void)hipGetLastError();
            return false;
        }
        return true;
    };
    if (bloom && bloom_part_plan(b->bloom_view(), in.n, in.plan_bytes(), step, b->member_frac, b->opt, &plan) &&
        part_ws()) {
        path = XS_PATH_PARTITIONED;
        const BloomPartWs ws{b->pk_nkc.as<uint64_t>(), b->pk_kofs.as<uint64_t>(), b->pk_scan.p, b->pk_scan.cap,
                             b->pk_entries.as<uint64_t>(), b->pk_tbl.as<uint16_t>(), b->pk_miss.as<uint32_t>(),
                             b->pk_aux.as<uint32_t>()};
        PassRecorder rec{&b->pass_ev, &b->pass_tag, &b->pass_used};
        HIPCHK(launch_probe_bloom_part(rv, b->bloom_view(), plan, ws, d_hits, partials, blocks, s,
                                       b->profiling ? &rec : nullptr));
    } else if (b->kind == XS_BANK_RBLOOM) {
        HIPCHK(launch_probe_bloom(rv, b->bloom_view(), d_hits, partials, blocks, s));
    } else {
        const CobsView cv = b->cobs_view();
        if (cobs_part) {
            path = XS_PATH_PARTITIONED;
            const PartWs ws{b->pk_nkc.as<uint64_t>(), b->pk_kofs.as<uint64_t>(), b->pk_scan.p, b->pk_scan.cap,
                            b->pk_entries.p, b->pk_tbl.as<uint16_t>(), b->pk_aux.as<uint32_t>()};
            PassRecorder rec{&b->pass_ev, &b->pass_tag, &b->pass_used};
            HIPCHK(launch_probe_cobs_part(rv, cv, cplan, ws, d_hits, partials, blocks, s, b->profiling ? &rec : nullptr));
        } else {
            HIPCHK(launch_probe_cobs(rv, cv, d_hits, partials, blocks, s));
        }
    }
    b->last_path = path;
    if (timed) {
        HIPCHK(hipEventRecord(b->events[b->events_used].second, s));
        ++b->events_used;
    }
    if (d_totals) HIPCHK(launch_reduce_partials(partials, blocks, pcols, d_totals, s));
    if (bloom && !b->bloom_pending) {
        if (int rc = b->bloom_tot.ensure(2 * sizeof(uint64_t))) return rc;
        if (int rc = b->bloom_tot_h.ensure(2 * sizeof(uint64_t))) return rc;
        if (!b->bloom_ev) HIPCHK(hipEventCreateWithFlags(&b->bloom_ev, hipEventDisableTiming));
        HIPCHK(launch_reduce_partials(partials, blocks, pcols, b->bloom_tot.as<uint64_t>(), s));
        HIPCHK(hipMemcpyAsync(b->bloom_tot_h.p, b->bloom_tot.p, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
        HIPCHK(hipEventRecord(b->bloom_ev, s));
        b->bloom_pending = true;
    }
    return ws_leave(b, s);
}

// Copy host reads to the handle's device buffers (offsets rebased to 0).
int stage_host_reads(xs_bank* b, const char* seqs, const uint64_t* offsets, uint64_t n,
                     Inputs* in) {
    const uint64_t base = offsets[0];
    const uint64_t bytes = offsets[n] - base;
    for (uint64_t r = 0; r < n; ++r)
        if (offsets[r + 1] < offsets[r]) return fail(XS_ERR_ARG, "offsets must be non-decreasing");
    std::vector<uint64_t> rebased(n + 1);
    for (uint64_t r = 0; r <= n; ++r) rebased[r] = offsets[r] - base;
    if (int rc = b->seqs.ensure(bytes + kPad)) return rc;
    if (int rc = b->offs.ensure((n + 1) * 8)) return rc;
    if (bytes) HIPCHK(hipMemcpyAsync(b->seqs.p, seqs + base, bytes, hipMemcpyHostToDevice, b->stream));
    HIPCHK(hipMemcpyAsync(b->offs.p, rebased.data(), (n + 1) * 8, hipMemcpyHostToDevice, b->stream));
    HIPCHK(hipStreamSynchronize(b->stream));  // `rebased` leaves scope
    in->seqs = b->seqs.as<uint8_t>();
    in->seq_bytes = bytes;
    in->offs = b->offs.as<uint64_t>();
    in->n = n;
    return XS_OK;
}

// Device -> pageable host copy of `bytes`, ordered after the work already on
// stream `st`.  Large copies go through a pinned two-slot ring: the DMA of
// chunk i overlaps the host copy of chunk i-1 (a plain pageable D2H runs at
// about 9 GB/s on the box, a pinned one at PCIe rate).  Returns once the data
// is in `host`.
int d2h_pageable(xs_bank* b, void* host, const void* dev, size_t bytes, hipStream_t st) {
    constexpr size_t kChunk = 32u << 20;
    bool pinned = false;
    if (bytes >= 2 * kChunk) {
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, host) == hipSuccess) pinned = attr.type == hipMemoryTypeHost;
        else (void)hipGetLastError();  // pageable memory is "not a HIP pointer"
    }
    if (bytes < 2 * kChunk || pinned) {
        HIPCHK(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        return XS_OK;
    }
    for (int s = 0; s < 2; ++s) {
        if (int rc = b->stage[s].ensure(kChunk)) return rc;
        if (!b->stage_ev[s]) HIPCHK(hipEventCreateWithFlags(&b->stage_ev[s], hipEventDisableTiming));
    }
    const unsigned hw = std::thread::hardware_concurrency();
    const int threads = (int)std::max(1u, std::min(8u, hw ? hw : 1u));
    size_t prev_off = 0, prev_n = 0;
    int prev_slot = -1;
    for (size_t off = 0, i = 0; off < bytes; off += kChunk, ++i) {
        const int slot = (int)(i & 1);
        const size_t n = std::min(kChunk, bytes - off);
        HIPCHK(hipMemcpyAsync(b->stage[slot].p, static_cast<const char*>(dev) + off, n, hipMemcpyDeviceToHost,
                              st));
        HIPCHK(hipEventRecord(b->stage_ev[slot], st));
        if (prev_slot >= 0) {
            HIPCHK(hipEventSynchronize(b->stage_ev[prev_slot]));
            par_memcpy(static_cast<char*>(host) + prev_off, b->stage[prev_slot].p, prev_n, threads);
        }
        prev_off = off;
        prev_n = n;
        prev_slot = slot;
    }
    HIPCHK(hipEventSynchronize(b->stage_ev[prev_slot]));
    par_memcpy(static_cast<char*>(host) + prev_off, b->stage[prev_slot].p, prev_n, threads);
    return XS_OK;
}

// ---- host batches: staging overlapped with the probe --------------------------
// A host batch is cut at read boundaries into chunks of about kHostChunk
// sequence bytes (the first smaller, so the probe starts early).  Chunk i is
// copied into a pinned slot by host threads and sent on the copy stream while
// the bank stream probes chunk i-1.  With host hits wanted, chunk i-1's hit
// rows go back through the D2H ring on a third stream while chunk i is probed.
// Device buffers span the whole batch, so chunks never overwrite each other's
// reads or hits, and the workspace is sized for the whole batch up front (no
// reallocation, hence no implicit device sync, between chunks).
constexpr size_t kHostChunk = 32u << 20;
constexpr size_t kHostFirst = 8u << 20;

int host_threads() {
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(8u, hw ? hw : 1u));
}

// fn(t, a, e) over the ranges of [0, n) of up to `threads` threads (one below 2^18 items:
// a host batch's per-read passes run before its first copy, in the call's critical path)
template <class F>
void par_ranges(uint64_t n, int threads, F fn) {
    const int T = n < (1u << 18) ? 1 : threads;
    const uint64_t per = (n + T - 1) / T;
    if (T == 1) return fn(0, 0, n);
    xs::parallel_for(T, [&](int t) {
        const uint64_t a = per * (uint64_t)t;
        if (a < n) fn(t, a, std::min(n, a + per));
    });
}

// ---- hit rows back to a host array, behind the probe ------------------------
// A host call's hit rows go to the caller's array on a worker thread while the
// bank stream probes the next chunks (the main thread only launches): each
// chunk's rows, in the wire width (uint8 / uint16 narrowed on the device when
// every read's sampled k-mers fit, else uint32), are cut into pieces of
// kSinkPiece bytes, DMA'd on d2h_stream into a ring of three pinned slots (two
// pieces in flight while a third is copied out) and copied by host threads
// into the caller's array, widened to its element width where the wire is
// narrower.  A pinned destination of the wire width takes the DMA directly.
// xs_query's uint32 matrix of 1 M reads x 100 docs thus crosses PCIe as 100 MB
// of uint8 instead of 400 MB, and its copy-out overlaps the probe.
constexpr size_t kSinkPiece = 32u << 20;
constexpr int kSinkSlots = 3;

template <class S, class D>
void widen_rows(D* dst, const S* src, size_t n, int threads) {
    auto run = [=](size_t a, size_t e) {
        for (size_t i = a; i < e; ++i) dst[i] = (D)src[i];
    };
    if (n < (1u << 20) || threads <= 1) {
        run(0, n);
        return;
    }
    const size_t per = (n + threads - 1) / threads;
    xs::parallel_for(threads, [&](int t) {
        const size_t a = per * (size_t)t;
        if (a < n) run(a, std::min(n, a + per));
    });
}

class HitSink {
  public:
    // rows of `cols` counts: on the device at `src` (wire bytes each), to `host` (out bytes each)
    HitSink(xs_bank* b, void* host, const void* src, uint64_t cols, int wire, int out)
        : b_(b), host_(static_cast<uint8_t*>(host)), src_(static_cast<const uint8_t*>(src)), cols_(cols),
          wire_(wire), out_(out) {}
    HitSink(const HitSink&) = delete;
    HitSink& operator=(const HitSink&) = delete;
    // an early return of the caller: the copies stop, and the caller's error stays the one reported
    ~HitSink() { join(); }

    int start(uint64_t total_bytes_out) {
        if (wire_ == out_ && total_bytes_out >= 2 * kSinkPiece) {
            hipPointerAttribute_t attr;
            if (hipPointerGetAttributes(&attr, host_) == hipSuccess) direct_ = attr.type == hipMemoryTypeHost;
            else (void)hipGetLastError();  // pageable memory is "not a HIP pointer"
        } else if (wire_ == out_) {
            direct_ = true;  // small: one DMA into pageable memory is as fast as staging it
        }
        if (!direct_) {  // a pageable destination, filled by the copy-out threads
            advise_huge_pages(host_, total_bytes_out);
            for (int s = 0; s < kSinkSlots; ++s) {
                if (int rc = b_->stage[s].ensure(kSinkPiece)) return rc;
                if (!b_->stage_ev[s]) HIPCHK(hipEventCreateWithFlags(&b_->stage_ev[s], hipEventDisableTiming));
            }
        }
        th_ = std::thread([this] { run(); });
        return XS_OK;
    }
    // rows [r0, r1) are complete on the device once `ev` has fired
    void push(uint64_t r0, uint64_t r1, hipEvent_t ev) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(Job{r0, r1, ev});
        }
        cv_.notify_one();
    }
    // no more rows: wait for the copies; the worker's error, if any, becomes this thread's
    int finish() {
        join();
        return rc_ ? xs::set_error(rc_, err_.c_str()) : XS_OK;
    }

  private:
    void join() {
        if (!th_.joinable()) return;
        {
            std::lock_guard<std::mutex> g(mu_);
            closed_ = true;
        }
        cv_.notify_one();
        th_.join();
    }
    struct Job {
        uint64_t r0, r1;
        hipEvent_t ev;
    };
    struct Piece {
        int slot;
        uint64_t elem0, elems;  // first element and count
    };
    int copy_out(const Piece& p) {
        if (hipEventSynchronize(b_->stage_ev[p.slot]) != hipSuccess) return XS_ERR_HIP;
        const void* in = b_->stage[p.slot].p;
        const int t = threads_;
        if (wire_ == out_) par_memcpy(host_ + p.elem0 * out_, in, p.elems * out_, t);
        else if (wire_ == 1 && out_ == 2) widen_rows(reinterpret_cast<uint16_t*>(host_) + p.elem0, static_cast<const uint8_t*>(in), p.elems, t);
        else if (wire_ == 1) widen_rows(reinterpret_cast<uint32_t*>(host_) + p.elem0, static_cast<const uint8_t*>(in), p.elems, t);
        else widen_rows(reinterpret_cast<uint32_t*>(host_) + p.elem0, static_cast<const uint16_t*>(in), p.elems, t);
        return XS_OK;
    }
    void fail_with(int rc, const char* what) {
        if (!rc_) {
            rc_ = rc;
            err_ = what;
        }
    }
    // the worker thread's body: a C++ exception in it (a failed allocation, a copy-out
    // task) becomes the call's error instead of ending the process
    void run() {
        try {
            copy_loop();
        } catch (const std::bad_alloc&) {
            fail_with(XS_ERR_NOMEM, "host memory allocation failed in the hit copier");
        } catch (const std::exception& e) {
            fail_with(XS_ERR_INTERNAL, e.what());
        } catch (...) {
            fail_with(XS_ERR_INTERNAL, "unknown C++ exception in the hit copier");
        }
        // whatever happened above: no DMA may still be writing a staging slot when the call returns
        if (hipStreamSynchronize(b_->d2h_stream) != hipSuccess) fail_with(XS_ERR_HIP, "hit D2H failed");
    }
    void copy_loop() {
        if (hipSetDevice(b_->device) != hipSuccess) return fail_with(XS_ERR_HIP, "hipSetDevice failed in the hit copier");
        std::deque<Piece> inflight;
        int next_slot = 0;
        for (;;) {
            Job j;
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return closed_ || !q_.empty(); });
                if (q_.empty()) break;
                j = q_.front();
                q_.pop_front();
            }
            if (rc_) continue;  // drain the queue after a failure
            hipError_t e = hipStreamWaitEvent(b_->d2h_stream, j.ev, 0);
            const uint64_t e0 = j.r0 * cols_, e1 = j.r1 * cols_;
            const uint64_t per = kSinkPiece / (uint64_t)wire_;
            for (uint64_t a = e0; e == hipSuccess && a < e1; a += per) {
                const uint64_t m = std::min(per, e1 - a);
                if (direct_) {
                    e = hipMemcpyAsync(host_ + a * out_, src_ + a * wire_, m * wire_, hipMemcpyDeviceToHost,
                                       b_->d2h_stream);
                    continue;
                }
                if ((int)inflight.size() == kSinkSlots - 1) {  // the oldest piece out of its slot first
                    if (int rc = copy_out(inflight.front())) {
                        fail_with(rc, "hit copy-out failed");
                        break;
                    }
                    inflight.pop_front();
                }
                const int slot = next_slot;
                next_slot = (next_slot + 1) % kSinkSlots;
                e = hipMemcpyAsync(b_->stage[slot].p, src_ + a * wire_, m * wire_, hipMemcpyDeviceToHost, b_->d2h_stream);
                if (e == hipSuccess) e = hipEventRecord(b_->stage_ev[slot], b_->d2h_stream);
                inflight.push_back(Piece{slot, a, m});
            }
            if (e != hipSuccess) fail_with(XS_ERR_HIP, hipGetErrorString(e));
        }
        while (!inflight.empty() && !rc_) {
            if (int rc = copy_out(inflight.front())) fail_with(rc, "hit copy-out failed");
            inflight.pop_front();
        }
    }

    xs_bank* b_;
    uint8_t* host_;
    const uint8_t* src_;
    uint64_t cols_;
    int wire_, out_;
    bool direct_ = false;
    int threads_ = (int)std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    std::thread th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Job> q_;
    bool closed_ = false;
    int rc_ = XS_OK;
    std::string err_;
};

// Narrowest transport width (bytes) of hit counts up to max_count, at most `out`.
int wire_width(uint64_t max_count, int out) {
    const int w = max_count <= 0xFFu ? 1 : max_count <= 0xFFFFu ? 2 : 4;
    return std::min(w, out);
}

// Reads already in HBM (a device-mode reader's batch): query_host then only
// chunks the probe and the hit-row D2H.
struct DevReads {
    const uint8_t* seqs;
    uint64_t seq_bytes;
    const uint64_t* offs;  // n+1, offs[0] = 0
};
constexpr uint64_t kDevChunkReads = 1u << 18;

// hits_host: n x cols rows back on the host (needs d_hits), as hit_bytes-wide
// counts, crossing PCIe as wire_bytes-wide counts (0: hit_bytes; narrower
// counts are narrowed on the device into b->narrow and widened on the host,
// the caller having checked that they fit); tot_host: cols + 1 entries
// (per-doc sums, then the k-mer total).  dev: the reads are on the device
// (seqs and offsets unused); chunks are then cut by read count.
int query_host(xs_bank* b, const char* seqs, const uint64_t* offsets, uint64_t n, uint32_t step,
               uint32_t* d_hits, void* hits_host, uint64_t* d_nk, uint64_t* tot_host, int hit_bytes = 4,
               const DevReads* dev = nullptr, int wire_bytes = 0) {
    int wire = wire_bytes ? std::min(wire_bytes, hit_bytes) : hit_bytes;
    if (hits_host && wire != hit_bytes) {  // a pinned destination takes the rows by DMA as they are
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, hits_host) == hipSuccess) {
            if (attr.type == hipMemoryTypeHost) wire = hit_bytes;
        } else {
            (void)hipGetLastError();  // pageable memory is "not a HIP pointer"
        }
    }
    const uint64_t base = dev ? 0 : offsets[0];
    if (!dev) {
        // one pass, on several threads: the offsets checked and rebased to 0 into pinned memory
        // (their H2D copy then needs no staging)
        if (int rc = b->offs_h.ensure((n + 1) * 8)) return rc;
        uint64_t* rb = static_cast<uint64_t*>(b->offs_h.p);
        bool bad[8] = {};
        par_ranges(n, host_threads(), [&](int t, uint64_t a, uint64_t e) {
            bool ok = true;
            for (uint64_t r = a; r < e; ++r) {
                ok &= offsets[r + 1] >= offsets[r];
                rb[r] = offsets[r] - base;
            }
            bad[t] = !ok;
        });
        rb[n] = offsets[n] - base;
        for (bool x : bad)
            if (x) return fail(XS_ERR_ARG, "offsets must be non-decreasing");
    }
    const uint64_t bytes = dev ? dev->seq_bytes : offsets[n] - base;
    const uint64_t cols = b->kind == XS_BANK_RBLOOM ? 1 : b->D;
    const uint64_t pcols = cols + 1;
    std::vector<uint64_t> cut{0};
    std::vector<uint64_t> cut_ofs;  // device reads: offsets at the cuts (the chunks' byte counts)
    if (dev) {
        // chunks overlap the hit rows' D2H with the next chunk's probe; without
        // rows to bring back, one chunk (a partitioned probe reloads the bank's
        // partitions into L2 per chunk)
        const uint64_t per = hits_host ? std::max<uint64_t>(kDevChunkReads, (n + 3) / 4) : n;
        while (cut.back() < n) cut.push_back(std::min(n, cut.back() + per));
        if (cut.size() == 2) {
            // one chunk: its bytes are the batch's (offsets start at 0; seq_bytes bounds the
            // last offset, which is all the probe's planner needs), no round trip to the device
            cut_ofs = {0, dev->seq_bytes};
        } else {
            if (int rc = b->cut_ofs.ensure(cut.size() * 8)) return rc;
            cut_ofs.resize(cut.size());
            for (size_t j = 0; j < cut.size(); ++j)
                HIPCHK(hipMemcpyAsync(static_cast<uint64_t*>(b->cut_ofs.p) + j, dev->offs + cut[j], 8,
                                      hipMemcpyDeviceToHost, b->stream));
            HIPCHK(hipStreamSynchronize(b->stream));
            memcpy(cut_ofs.data(), b->cut_ofs.p, cut.size() * 8);
        }
    } else {
        for (size_t limit = kHostFirst; cut.back() < n; limit = kHostChunk) {
            const uint64_t r0 = cut.back();
            uint64_t e =
                (uint64_t)(std::upper_bound(offsets + r0 + 1, offsets + n + 1, offsets[r0] + limit) - offsets) - 1;
            cut.push_back(e > r0 ? e : r0 + 1);  // a read over the limit is a chunk of its own
        }
    }
    const size_t nc = cut.size() - 1;
    if (!dev) {
        if (int rc = b->seqs.ensure(bytes + kPad)) return rc;
        if (int rc = b->offs.ensure((n + 1) * 8)) return rc;
    }
    if (int rc = b->nseg.ensure((n + 1) * 8)) return rc;
    if (int rc = b->unit_ofs.ensure((n + 1) * 8)) return rc;
    if (int rc = b->n_units.ensure(2 * sizeof(uint64_t))) return rc;
    if (int rc = b->unit_read.ensure((n + bytes / kSegKmers + 1) * 4)) return rc;
    if (int rc = b->scan_tmp.ensure(scan_temp_bytes(n))) return rc;
    if (int rc = b->partials.ensure((size_t)probe_grid(b) * pcols * 8)) return rc;
    if (tot_host)
        if (int rc = b->totals.ensure(nc * pcols * 8)) return rc;
    if (!dev) {  // host reads: the H2D staging ring and its copy stream (device reads need neither)
        for (int s = 0; s < 2; ++s) {
            if (int rc = b->hstage[s].ensure(kHostChunk)) return rc;
            if (!b->hstage_ev[s]) HIPCHK(hipEventCreateWithFlags(&b->hstage_ev[s], hipEventDisableTiming));
        }
        if (!b->copy_stream) HIPCHK(hipStreamCreateWithFlags(&b->copy_stream, hipStreamNonBlocking));
    }
    if (hits_host && !b->d2h_stream) HIPCHK(hipStreamCreateWithFlags(&b->d2h_stream, hipStreamNonBlocking));
    const bool narrowing = hits_host && wire != 4;
    if (narrowing) {
        if (int rc = b->narrow.ensure(n * cols * (uint64_t)wire + 16)) return rc;
        if (int rc = b->ovf.ensure(sizeof(uint32_t))) return rc;
        HIPCHK(hipMemsetAsync(b->ovf.p, 0, sizeof(uint32_t), b->stream));
    }
    while (hits_host && b->chunk_ev.size() < nc) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        b->chunk_ev.push_back(e);
    }
    const uint8_t* d_seqs = dev ? dev->seqs : b->seqs.as<uint8_t>();
    const uint64_t* d_offs = dev ? dev->offs : b->offs.as<uint64_t>();
    // whatever way the call ends (an error return included), no H2D copy may still be
    // reading the caller's reads or the rebased offsets once it has: the copy stream drains on exit
    struct DrainOnExit {
        hipStream_t s = nullptr;
        ~DrainOnExit() {
            if (s) (void)hipStreamSynchronize(s);
        }
    } drain;
    if (!dev) {
        drain.s = b->copy_stream;
        HIPCHK(hipMemcpyAsync(b->offs.p, b->offs_h.p, (n + 1) * 8, hipMemcpyHostToDevice, b->copy_stream));
    }
    const int threads = host_threads();
    // the hit rows go back behind the probe (HitSink: its own thread, stream and pinned ring)
    std::unique_ptr<HitSink> sink;
    if (hits_host) {
        sink.reset(new HitSink(b, hits_host, narrowing ? b->narrow.p : static_cast<const void*>(d_hits), cols, wire,
                               hit_bytes));
        if (int rc = sink->start(n * cols * (uint64_t)hit_bytes)) return rc;
    }
    bool used[2] = {false, false};
    for (size_t i = 0; i < nc; ++i) {
        const uint64_t r0 = cut[i], r1 = cut[i + 1];
        if (!dev) {
            const uint64_t o0 = offsets[r0] - base, o1 = offsets[r1] - base, nb = o1 - o0;
            const int slot = (int)(i & 1);
            uint8_t* stage_dst = b->seqs.as<uint8_t>() + o0;
            if (used[slot]) HIPCHK(hipEventSynchronize(b->hstage_ev[slot]));  // the slot's last H2D is done
            if (nb && nb <= kHostChunk) {
                par_memcpy(b->hstage[slot].p, seqs + base + o0, nb, threads);
                HIPCHK(hipMemcpyAsync(stage_dst, b->hstage[slot].p, nb, hipMemcpyHostToDevice, b->copy_stream));
            } else if (nb) {  // one read larger than a slot
                HIPCHK(hipMemcpyAsync(stage_dst, seqs + base + o0, nb, hipMemcpyHostToDevice, b->copy_stream));
            }
            HIPCHK(hipEventRecord(b->hstage_ev[slot], b->copy_stream));
            used[slot] = true;
            HIPCHK(hipStreamWaitEvent(b->stream, b->hstage_ev[slot], 0));
        }
        const Inputs in{d_seqs, dev ? bytes : offsets[r1] - base, d_offs + r0, r1 - r0,
                        dev ? cut_ofs[i + 1] - cut_ofs[i] : offsets[r1] - offsets[r0]};
        if (int rc = run_query(b, in, step, d_hits ? d_hits + r0 * cols : nullptr, d_nk ? d_nk + r0 : nullptr,
                               tot_host ? b->totals.as<uint64_t>() + i * pcols : nullptr, b->stream))
            return rc;
        if (hits_host) {
            if (narrowing)
                HIPCHK(launch_narrow_hits(d_hits + r0 * cols, b->narrow.as<uint8_t>() + r0 * cols * wire,
                                          (r1 - r0) * cols, wire, b->stream, b->ovf.as<uint32_t>()));
            HIPCHK(hipEventRecord(b->chunk_ev[i], b->stream));
            sink->push(r0, r1, b->chunk_ev[i]);
        }
    }
    if (sink)
        if (int rc = sink->finish()) return rc;
    if (tot_host) {
        std::vector<uint64_t> t(nc * pcols);
        HIPCHK(hipMemcpyAsync(t.data(), b->totals.p, t.size() * 8, hipMemcpyDeviceToHost, b->stream));
        HIPCHK(hipStreamSynchronize(b->stream));
        for (uint64_t c = 0; c < pcols; ++c) {
            uint64_t v = 0;
            for (size_t i = 0; i < nc; ++i) v += t[i * pcols + c];
            tot_host[c] = v;
        }
    }
    if (!dev) HIPCHK(hipStreamSynchronize(b->copy_stream));  // offs_h is rewritten by the next call
    if (narrowing) {  // a count wider than the wire (device reads: the caller's max_len understated)
        uint32_t over = 0;
        HIPCHK(hipMemcpyAsync(&over, b->ovf.p, sizeof(over), hipMemcpyDeviceToHost, b->stream));
        HIPCHK(hipStreamSynchronize(b->stream));
        if (over) return fail(XS_ERR_ARG, "a hit count does not fit %d byte(s): max_len is below the longest read",
                              wire);
    }
    return XS_OK;
}

// ---- small host calls ------------------------------------------------------------
// A request of a few reads (a serving loop's request, the per-read drop-in
// `search` of INTEGRATION.md §2) costs its launches, copies and syncs, not its
// probe: query_host's unit pipeline (units, scan, scatter), staging ring and
// three streams take 150-200 us for one read.  Here the host builds the unit
// map and packs the whole request into one pinned buffer: one H2D copy, the
// same direct probe kernel as query_host's gather path, one D2H copy of the
// per-block partials and the hit rows, one sync.  k-mer counts are the host's
// own (the formula of units_kernel), totals the sum of the partials.
constexpr uint64_t kSmallReads = 4096;
constexpr uint64_t kSmallBytes = 1u << 20;  // sequence bytes of the request
constexpr uint64_t kSmallUnits = 8192;
constexpr uint64_t kSmallUnitsPerBlock = 4;  // 4 waves taking 1 unit per grab (ReadView::grab)

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

// *done = false: the call does not qualify (nothing was enqueued).  Hit rows
// go to hits_host as hit_bytes-wide counts (the caller checked the width).
int query_small(xs_bank* b, const char* seqs, const uint64_t* offsets, uint64_t n, uint32_t step,
                void* hits_host, int hit_bytes, uint64_t* nk_host, uint64_t* tot_host, bool* done) {
    *done = false;
    if (b->profiling || n == 0 || n > kSmallReads || !b->opt.small_calls) return XS_OK;
    const uint64_t base = offsets[0];
    for (uint64_t r = 0; r < n; ++r)
        if (offsets[r + 1] < offsets[r]) return fail(XS_ERR_ARG, "offsets must be non-decreasing");
    const uint64_t bytes = offsets[n] - base;
    if (bytes > kSmallBytes) return XS_OK;
    const bool bloom = b->kind == XS_BANK_RBLOOM;
    const uint64_t cols = bloom ? 1 : b->D;
    const uint64_t pcols = cols + 1;
    std::vector<uint64_t> nk(n), uofs(n + 1);
    uint64_t U = 0;
    bool zero_rows = false;  // rows the probe does not store whole (no k-mers, or several units)
    for (uint64_t r = 0; r < n; ++r) {
        const uint64_t len = offsets[r + 1] - offsets[r];
        nk[r] = len >= b->k ? (len - b->k) / step + 1 : 0;
        const uint64_t s = (nk[r] + kSegKmers - 1) / kSegKmers;
        zero_rows |= s != 1;
        uofs[r] = U;
        U += s;
    }
    uofs[n] = U;
    if (U > kSmallUnits) return XS_OK;
    // only where query_host would take the direct / gather probe as well (a forced
    // or member-rich partitioned path keeps its own pipeline)
    if (bloom) {
        if (b->bloom_pending && hipEventQuery(b->bloom_ev) == hipSuccess) {  // as run_query
            const uint64_t* t = static_cast<const uint64_t*>(b->bloom_tot_h.p);
            if (t[1]) b->member_frac = (double)t[0] / (double)t[1];
            b->bloom_pending = false;
        }
        (void)hipGetLastError();  // hipErrorNotReady is not an error here
        BloomPartPlan plan;
        if (bloom_part_plan(b->bloom_view(), n, bytes, step, b->member_frac, b->opt, &plan)) return XS_OK;
    } else {
        CobsPartPlan plan;
        if (cobs_part_plan(b->cobs_view(), b->k, n, bytes, step, b->opt, &plan)) return XS_OK;
    }
    const int blocks = (int)std::min<uint64_t>((uint64_t)probe_grid(b), std::max<uint64_t>(1, (U + kSmallUnitsPerBlock - 1) / kSmallUnitsPerBlock));
    // device / pinned layout: [queue | offsets | unit_ofs | unit_read | seqs] [partials | hits]
    const size_t o_off = 16, o_uofs = o_off + align16((n + 1) * 8), o_uread = o_uofs + align16((n + 1) * 8);
    const size_t o_seq = o_uread + align16(U * 4 + 4);
    const size_t in_bytes = o_seq + align16(bytes + kPad);
    const size_t o_part = in_bytes, part_bytes = align16((size_t)blocks * pcols * 8);
    const size_t o_hits = o_part + part_bytes;
    const size_t out_bytes = part_bytes + (hits_host ? n * cols * 4 : 0);
    if (int rc = b->small_h.ensure(in_bytes + out_bytes)) return rc;
    if (int rc = b->small_d.ensure(in_bytes + out_bytes)) return rc;
    char* h = static_cast<char*>(b->small_h.p);
    char* d = static_cast<char*>(b->small_d.p);
    auto* q = reinterpret_cast<uint64_t*>(h);
    q[0] = U;
    q[1] = 0;
    auto* ho = reinterpret_cast<uint64_t*>(h + o_off);
    for (uint64_t r = 0; r <= n; ++r) ho[r] = offsets[r] - base;
    memcpy(h + o_uofs, uofs.data(), (n + 1) * 8);
    auto* ur = reinterpret_cast<uint32_t*>(h + o_uread);
    for (uint64_t r = 0; r < n; ++r)
        for (uint64_t u = uofs[r]; u < uofs[r + 1]; ++u) ur[u] = (uint32_t)r;
    if (bytes) memcpy(h + o_seq, seqs + base, bytes);
    memset(h + o_seq + bytes, 0, kPad);
    const hipStream_t s = b->stream;
    HIPCHK(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, s));
    uint32_t* d_hits = hits_host ? reinterpret_cast<uint32_t*>(d + o_hits) : nullptr;
    if (d_hits && zero_rows) HIPCHK(hipMemsetAsync(d_hits, 0, n * cols * 4, s));
    ReadView rv;
    rv.seq = reinterpret_cast<const uint8_t*>(d + o_seq);
    rv.seq_bytes = bytes;
    rv.offs = reinterpret_cast<const uint64_t*>(d + o_off);
    rv.unit_read = reinterpret_cast<const uint32_t*>(d + o_uread);
    rv.unit_ofs = reinterpret_cast<const uint64_t*>(d + o_uofs);
    rv.queue = reinterpret_cast<uint64_t*>(d);
    rv.n = n;
    rv.k = b->k;
    rv.step = step;
    rv.grab = 1;
    auto* d_part = reinterpret_cast<uint64_t*>(d + o_part);
    if (bloom) HIPCHK(launch_probe_bloom(rv, b->bloom_view(), d_hits, d_part, blocks, s));
    else HIPCHK(launch_probe_cobs(rv, b->cobs_view(), d_hits, d_part, blocks, s));
    HIPCHK(hipMemcpyAsync(h + o_part, d + o_part, out_bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    b->last_path = XS_PATH_GATHER;
    const auto* part = reinterpret_cast<const uint64_t*>(h + o_part);
    std::vector<uint64_t> tot(pcols, 0);
    for (int i = 0; i < blocks; ++i)
        for (uint64_t c = 0; c < pcols; ++c) tot[c] += part[(uint64_t)i * pcols + c];
    if (bloom) {  // the next query's path choice follows this one's member fraction
        if (tot[1]) b->member_frac = (double)tot[0] / (double)tot[1];
        b->bloom_pending = false;
    }
    if (tot_host) memcpy(tot_host, tot.data(), pcols * 8);
    if (nk_host) memcpy(nk_host, nk.data(), n * 8);
    if (hits_host) {
        const auto* hr = reinterpret_cast<const uint32_t*>(h + o_hits);
        const uint64_t m = n * cols;
        if (hit_bytes == 4) memcpy(hits_host, hr, m * 4);
        else if (hit_bytes == 2)
            for (uint64_t i = 0; i < m; ++i) static_cast<uint16_t*>(hits_host)[i] = (uint16_t)hr[i];
        else
            for (uint64_t i = 0; i < m; ++i) static_cast<uint8_t*>(hits_host)[i] = (uint8_t)hr[i];
    }
    *done = true;
    return XS_OK;
}

xs_bank* new_bank(int device, int kind) {
    xs_bank* b = new xs_bank();
    b->device = device;
    b->kind = kind;
    return b;
}

}  // namespace

int xs::set_error(int code, const char* msg) {
    g_err = msg;
    return code;
}

namespace {
std::mutex g_pin_mu;
std::unordered_map<void*, size_t> g_pins;  // registered mappings: start -> length
}  // namespace

int xs::pinned_alloc(size_t bytes, void** out) {
    *out = nullptr;
    constexpr size_t kHuge = size_t(2) << 20;
    const size_t n = (std::max<size_t>(bytes, 1) + kHuge - 1) & ~(kHuge - 1);
    if (bytes >= kHuge) {
        const size_t len = n + kHuge;  // room to align the start to a 2 MiB page
        void* raw = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (raw != MAP_FAILED) {
            char* r = static_cast<char*>(raw);
            char* p = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(r) + kHuge - 1) & ~(uintptr_t)(kHuge - 1));
            if (p > r) (void)munmap(r, (size_t)(p - r));           // the unaligned head
            if (r + len > p + n) (void)munmap(p + n, (size_t)(r + len - (p + n)));  // and tail
            (void)madvise(p, n, MADV_HUGEPAGE);
            // fault every page now, from several threads (2 MiB pages fault in parallel; the
            // registration below would otherwise fault them one by one)
            const int threads = (int)std::min<size_t>(8, std::max<size_t>(1, n / (size_t(16) << 20)));
            const size_t per = (n / kHuge + threads - 1) / threads * kHuge;
            xs::parallel_for(threads, [=](int t) {
                if (per * t < n) memset(p + per * t, 0, std::min(per, n - per * t));
            });
            if (hipHostRegister(p, n, hipHostRegisterDefault) == hipSuccess) {
                std::lock_guard<std::mutex> g(g_pin_mu);
                g_pins[p] = n;
                *out = p;
                return XS_OK;
            }
            (void)hipGetLastError();
            (void)munmap(p, n);
        }
    }
    const hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
    if (e != hipSuccess) {
        *out = nullptr;
        return fail(XS_ERR_HIP, "hipHostMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    }
    return XS_OK;
}

void xs::pinned_free(void* p) {
    if (!p) return;
    size_t n = 0;
    {
        std::lock_guard<std::mutex> g(g_pin_mu);
        auto it = g_pins.find(p);
        if (it != g_pins.end()) {
            n = it->second;
            g_pins.erase(it);
        }
    }
    if (n) {
        (void)hipHostUnregister(p);
        (void)munmap(p, n);
    } else {
        (void)hipHostFree(p);
    }
}

extern "C" {

int xs_version(void) { return 100; }

const char* xs_last_error(void) { return g_err.c_str(); }

int xs_device_count(int* count) {
    return xs::guard([&]() -> int {
        if (!count) return fail(XS_ERR_ARG, "null count");
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        if (e != hipSuccess) {
            *count = 0;
            return fail(XS_ERR_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
        }
        *count = n;
        return XS_OK;
    });
}

int xs_bank_open(const char* path, int kind, int device, xs_bank** out) {
    return xs::guard([&]() -> int {
        if (!path || !out) return fail(XS_ERR_ARG, "null argument");
        *out = nullptr;
        if (kind != XS_BANK_COBS_CLASSIC && kind != XS_BANK_COBS_COMPACT && kind != XS_BANK_RBLOOM)
            return fail(XS_ERR_ARG, "unknown bank kind %d", kind);
        Reader rd;
        rd.f.open(path, std::ios::binary);
        if (!rd.f) return fail(XS_ERR_IO, "cannot open %s", path);
        rd.f.seekg(0, std::ios::end);
        const uint64_t fsize = (uint64_t)rd.f.tellg();
        rd.f.seekg(0);
        xs_bank* b = new_bank(device, kind);
        int rc = XS_OK;
        if (kind == XS_BANK_RBLOOM) {
            b->h = (uint32_t)rd.get<uint64_t>();
            if (!rd.ok || fsize <= 8) rc = fail(XS_ERR_FORMAT, "%s: truncated rbloom file", path);
            b->nbytes = fsize - 8;
            b->D = 1;
            b->names.push_back("0");
            b->k = 0;  // set by the caller's model metadata through xs_bank_create_bloom
        } else {
            rc = read_cobs_header(b, rd, path);
        }
        if (rc == XS_OK && kind == XS_BANK_RBLOOM) {
            // An rbloom file carries no k (the model JSON does); default to XspecT's
            // k = 21 (train.py:167-174) until xs_bank_set_term_size overrides it.
            b->k = 21;
        }
        if (rc == XS_OK) rc = validate_geometry(b);
        if (rc == XS_OK) {
            const uint64_t pos = (uint64_t)rd.f.tellg();
            if (fsize - pos != b->payload_bytes())
                rc = fail(XS_ERR_FORMAT, "%s: payload is %llu bytes, header implies %llu", path,
                          (unsigned long long)(fsize - pos), (unsigned long long)b->payload_bytes());
        }
        if (rc == XS_OK) rc = alloc_image(b);
        if (rc == XS_OK) rc = upload_file_payload(b, path, (uint64_t)rd.f.tellg());
        if (rc != XS_OK) {
            delete b;
            return rc;
        }
        *out = b;
        return XS_OK;
    });
}

int xs_bank_open_docs(const char* path, int device, uint64_t doc_lo, uint64_t doc_hi, xs_bank** out) {
    return xs::guard([&]() -> int {
        if (!path || !out) return fail(XS_ERR_ARG, "null argument");
        *out = nullptr;
        Reader rd;
        rd.f.open(path, std::ios::binary);
        if (!rd.f) return fail(XS_ERR_IO, "cannot open %s", path);
        rd.f.seekg(0, std::ios::end);
        const uint64_t fsize = (uint64_t)rd.f.tellg();
        rd.f.seekg(0);
        xs_bank* full = new_bank(device, XS_BANK_COBS_CLASSIC);
        std::unique_ptr<xs_bank> keep_full(full);
        if (int rc = read_cobs_header(full, rd, path)) return rc;
        const uint64_t D = full->D, R = full->page, S = full->sig[0];
        if (doc_lo % 8 || doc_lo >= doc_hi || doc_hi > D || (doc_hi % 8 && doc_hi != D))
            return fail(XS_ERR_ARG, "doc range [%llu, %llu) of %llu docs: bounds must be multiples of 8 (or the end)",
                        (unsigned long long)doc_lo, (unsigned long long)doc_hi, (unsigned long long)D);
        const uint64_t pos = (uint64_t)rd.f.tellg();
        if (fsize - pos != S * R)
            return fail(XS_ERR_FORMAT, "%s: payload is %llu bytes, header implies %llu", path,
                        (unsigned long long)(fsize - pos), (unsigned long long)(S * R));
        xs_bank* b = new_bank(device, XS_BANK_COBS_CLASSIC);
        std::unique_ptr<xs_bank> keep(b);
        b->k = full->k;
        b->h = full->h;
        b->canonicalize = full->canonicalize;
        b->D = doc_hi - doc_lo;
        b->G = 1;
        b->page = (b->D + 7) / 8;
        b->sig.assign(1, S);
        b->names.assign(full->names.begin() + (ptrdiff_t)doc_lo, full->names.begin() + (ptrdiff_t)doc_hi);
        if (int rc = validate_geometry(b)) return rc;
        if (int rc = alloc_image(b)) return rc;
        // whole rows to the device a piece at a time (about kLoadPiece bytes of whole rows), each
        // piece's byte columns [doc_lo / 8, + page) repacked into the image at its first row: the
        // device holds the slice and one piece of whole rows, never the whole bank (config 5's
        // column split exists for banks one GPU cannot hold)
        const uint64_t c0 = doc_lo / 8, P = b->page;
        const uint64_t piece = std::max<uint64_t>(1, kLoadPiece / R) * R;
        HIPCHK(hipSetDevice(b->device));
        if (int rc = ws_enter(b, b->stream)) return rc;
        if (int rc = b->tmp.ensure(std::min<uint64_t>(piece, S * R))) return rc;
        uint8_t* stage = b->tmp.as<uint8_t>();
        // one staging buffer: the stream orders each piece's copy after the previous piece's repack
        if (int rc = stream_file(b, path, pos, S * R, piece, [&](uint64_t off, uint64_t m, const uint8_t* src) {
                hipError_t e = hipMemcpyAsync(stage, src, m, hipMemcpyHostToDevice, b->stream);
                if (e != hipSuccess) return e;
                return launch_repack(stage + c0, R, b->image.as<uint8_t>() + off / R * b->pitch, b->pitch, m / R, P,
                                     b->stream);
            }))
            return rc;
        b->tmp.release();  // the staging piece is not kept beside the slice
        *out = keep.release();
        return XS_OK;
    });
}

int xs_bank_create_cobs(int device, int kind, uint32_t term_size, uint32_t num_hashes,
                        uint64_t num_docs, uint64_t page_size, uint64_t num_groups,
                        const uint64_t* sig, const char* const* doc_names, xs_bank** out) {
    return xs::guard([&]() -> int {
        if (!out || !sig) return fail(XS_ERR_ARG, "null argument");
        *out = nullptr;
        if (kind != XS_BANK_COBS_CLASSIC && kind != XS_BANK_COBS_COMPACT)
            return fail(XS_ERR_ARG, "kind must be a COBS kind");
        if (kind == XS_BANK_COBS_CLASSIC && (num_groups != 1 || page_size != (num_docs + 7) / 8))
            return fail(XS_ERR_ARG, "classic banks have one group of ceil(D/8) bytes");
        xs_bank* b = new_bank(device, kind);
        b->k = term_size;
        b->h = num_hashes;
        b->D = num_docs;
        b->G = num_groups;
        b->page = page_size;
        b->sig.assign(sig, sig + num_groups);
        for (uint64_t i = 0; i < num_docs; ++i)
            b->names.push_back(doc_names ? std::string(doc_names[i]) : std::to_string(i));
        int rc = validate_geometry(b);
        if (rc == XS_OK) rc = alloc_image(b);
        if (rc != XS_OK) {
            delete b;
            return rc;
        }
        *out = b;
        return XS_OK;
    });
}

int xs_bank_create_bloom(int device, uint32_t term_size, uint64_t nbytes, uint32_t nhash,
                         xs_bank** out) {
    return xs::guard([&]() -> int {
        if (!out) return fail(XS_ERR_ARG, "null argument");
        *out = nullptr;
        xs_bank* b = new_bank(device, XS_BANK_RBLOOM);
        b->k = term_size;
        b->h = nhash;
        b->nbytes = nbytes;
        b->D = 1;
        b->names.push_back("0");
        int rc = validate_geometry(b);
        if (rc == XS_OK) rc = alloc_image(b);
        if (rc != XS_OK) {
            delete b;
            return rc;
        }
        *out = b;
        return XS_OK;
    });
}

static int build_impl(xs_bank* b, const Inputs& in, const uint32_t* d_doc, hipStream_t s) {
    if (int rc = ws_enter(b, s)) return rc;
    ReadView rv;
    if (int rc = prepare_units(b, in, 1, nullptr, nullptr, 0, s, &rv)) return rc;
    const int blocks = probe_grid(b);
    if (b->kind == XS_BANK_RBLOOM)
        HIPCHK(launch_build_bloom(rv, b->bloom_view(), b->image.as<uint32_t>(), blocks, s));
    else
        HIPCHK(launch_build_cobs(rv, d_doc, b->cobs_view(), b->image.as<uint32_t>(), blocks, s));
    return ws_leave(b, s);
}

int xs_bank_build(xs_bank* b, const char* seqs, const uint64_t* offsets, const uint32_t* rec_doc,
                  uint64_t n_rec) {
    return xs::guard([&]() -> int {
        if (!b || (!seqs && n_rec) || !offsets) return fail(XS_ERR_ARG, "null argument");
        if (b->kind != XS_BANK_RBLOOM && n_rec && !rec_doc) return fail(XS_ERR_ARG, "rec_doc required");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        if (n_rec == 0) return XS_OK;
        if (b->kind != XS_BANK_RBLOOM)
            for (uint64_t r = 0; r < n_rec; ++r)
                if (rec_doc[r] >= b->D) return fail(XS_ERR_ARG, "rec_doc[%llu] out of range", (unsigned long long)r);
        Inputs in;
        if (int rc = stage_host_reads(b, seqs, offsets, n_rec, &in)) return rc;
        uint32_t* d_doc = nullptr;
        if (b->kind != XS_BANK_RBLOOM) {
            if (int rc = b->tmp.ensure(n_rec * 4)) return rc;
            d_doc = b->tmp.as<uint32_t>();
            HIPCHK(hipMemcpyAsync(d_doc, rec_doc, n_rec * 4, hipMemcpyHostToDevice, b->stream));
        }
        if (int rc = build_impl(b, in, d_doc, b->stream)) return rc;
        HIPCHK(hipStreamSynchronize(b->stream));
        return XS_OK;
    });
}

int xs_bank_build_device(xs_bank* b, const void* d_seqs, uint64_t seq_bytes,
                         const uint64_t* d_offsets, const uint32_t* d_rec_doc, uint64_t n_rec,
                         void* stream) {
    return xs::guard([&]() -> int {
        if (!b || !d_offsets) return fail(XS_ERR_ARG, "null argument");
        if (b->kind != XS_BANK_RBLOOM && n_rec && !d_rec_doc) return fail(XS_ERR_ARG, "rec_doc required");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        if (n_rec == 0) return XS_OK;
        Inputs in{static_cast<const uint8_t*>(d_seqs), seq_bytes, d_offsets, n_rec};
        hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null (legacy default) stream
        return build_impl(b, in, d_rec_doc, s);
    });
}

int xs_bank_save(xs_bank* b, const char* path) {
    return xs::guard([&]() -> int {
        if (!b || !path) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        HIPCHK(hipDeviceSynchronize());
        // the file is written beside its destination and renamed over it once whole: a failed
        // save leaves no short or holed file at `path`, and an existing model there intact
        struct Partial {  // removed on every way out (an exception included) but the rename
            std::string path;
            bool renamed = false;
            ~Partial() {
                if (!renamed) (void)::unlink(path.c_str());
            }
        } tmp{std::string(path) + ".xs-part-" + std::to_string((long)getpid())};
        const char* t = tmp.path.c_str();
        if (int rc = b->kind == XS_BANK_RBLOOM ? write_bloom_file(b, t) : write_cobs_file(b, t)) return rc;
        if (::rename(t, path) != 0) return fail(XS_ERR_IO, "cannot rename %s to %s: %s", t, path, strerror(errno));
        tmp.renamed = true;
        return XS_OK;
    });
}

int xs_bank_download(xs_bank* b, void* host, uint64_t nbytes) {
    return xs::guard([&]() -> int {
        if (!b || !host) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        HIPCHK(hipDeviceSynchronize());
        return download_payload(b, host, nbytes);
    });
}

int xs_bank_upload(xs_bank* b, const void* host, uint64_t nbytes) {
    return xs::guard([&]() -> int {
        if (!b || !host) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        return upload_payload(b, host, nbytes);
    });
}

int xs_bank_set_term_size(xs_bank* b, uint32_t term_size) {
    return xs::guard([&]() -> int {
        if (!b) return fail(XS_ERR_ARG, "null argument");
        if (b->kind != XS_BANK_RBLOOM)
            return fail(XS_ERR_ARG, "COBS banks carry their term size in the file header");
        if (term_size < 1 || term_size > kMaxK)
            return fail(XS_ERR_UNSUPPORTED, "term_size %u unsupported on the device (1..%u)", term_size, kMaxK);
        std::lock_guard<std::mutex> lk(b->mu);
        b->k = term_size;
        return XS_OK;
    });
}

int xs_bank_info(const xs_bank* b, xs_bank_info_t* o) {
    return xs::guard([&]() -> int {
        if (!b || !o) return fail(XS_ERR_ARG, "null argument");
        memset(o, 0, sizeof(*o));
        o->kind = b->kind;
        o->device = b->device;
        o->term_size = b->k;
        o->num_hashes = b->h;
        o->canonicalize = b->canonicalize;
        o->num_docs = b->D;
        o->num_groups = b->kind == XS_BANK_RBLOOM ? 0 : b->G;
        o->page_size = b->page;
        o->signature_rows = b->sig_total();
        o->bloom_bits = b->kind == XS_BANK_RBLOOM ? b->nbytes * 8 : 0;
        o->device_bytes = b->dev_bytes;
        o->device_row_pitch = b->pitch;
        return XS_OK;
    });
}

int xs_bank_signature_sizes(const xs_bank* b, uint64_t* out, uint64_t n) {
    return xs::guard([&]() -> int {
        if (!b || !out) return fail(XS_ERR_ARG, "null argument");
        if (b->kind == XS_BANK_RBLOOM) return fail(XS_ERR_ARG, "rbloom banks have no signature groups");
        if (n != b->sig.size()) return fail(XS_ERR_ARG, "bank has %zu groups, %llu requested", b->sig.size(),
                                            (unsigned long long)n);
        for (uint64_t g = 0; g < n; ++g) out[g] = b->sig[g];
        return XS_OK;
    });
}

const char* xs_bank_doc_name(const xs_bank* b, uint64_t i) {
    return xs::guard([&]() -> const char* {
        if (!b || i >= b->names.size()) {
            fail(XS_ERR_ARG, "doc index out of range");
            return nullptr;
        }
        return b->names[i].c_str();
    });
}

static int query_impl(xs_bank* b, const char* seqs, const uint64_t* offsets, uint64_t n, uint32_t step,
                      void* hits_out, int hit_bytes, uint64_t* num_kmers_out) {
    if (!b || !offsets || (!seqs && n)) return fail(XS_ERR_ARG, "null argument");
    if (hit_bytes != 1 && hit_bytes != 2 && hit_bytes != 4) return fail(XS_ERR_ARG, "hit_bytes must be 1, 2 or 4");
    if (step == 0) return fail(XS_ERR_ARG, "step must be >= 1");
    // a count never exceeds its read's sampled k-mers: they must fit the width, and
    // the rows cross PCIe in the narrowest width that holds the largest (wire_width)
    uint64_t max_nk = 0;
    if (hits_out) {
        const uint64_t cap = hit_bytes == 1 ? 0xFFu : hit_bytes == 2 ? 0xFFFFu : 0xFFFFFFFFu;
        uint64_t mx[8] = {}, over[8];
        for (auto& o : over) o = ~0ull;
        const uint32_t k = b->k;
        par_ranges(n, host_threads(), [&](int t, uint64_t a, uint64_t e) {
            uint64_t m = 0;
            for (uint64_t r = a; r < e; ++r) {
                const uint64_t len = offsets[r + 1] >= offsets[r] ? offsets[r + 1] - offsets[r] : 0;
                const uint64_t nk = len >= k ? (len - k) / step + 1 : 0;
                if (nk > cap && over[t] == ~0ull) over[t] = r;
                m = std::max(m, nk);
            }
            mx[t] = m;
        });
        for (int t = 0; t < 8; ++t) {
            if (over[t] != ~0ull) {
                const uint64_t r = over[t], len = offsets[r + 1] - offsets[r];
                return fail(XS_ERR_ARG, "read %llu has %llu sampled k-mers: counts may not fit %d byte(s)",
                            (unsigned long long)r, (unsigned long long)((len - k) / step + 1), hit_bytes);
            }
            max_nk = std::max(max_nk, mx[t]);
        }
    }
    std::lock_guard<std::mutex> lk(b->mu);
    HIPCHK(hipSetDevice(b->device));
    if (n == 0) return XS_OK;
    bool done = false;
    if (int rc = query_small(b, seqs, offsets, n, step, hits_out, hit_bytes, num_kmers_out, nullptr, &done)) return rc;
    if (done) return XS_OK;
    const uint64_t cols = b->kind == XS_BANK_RBLOOM ? 1 : b->D;
    uint32_t* d_hits = nullptr;
    uint64_t* d_nk = nullptr;
    if (hits_out) {
        if (int rc = b->hits.ensure(n * cols * 4)) return rc;
        d_hits = b->hits.as<uint32_t>();
    }
    if (num_kmers_out) {
        if (int rc = b->nk.ensure(n * 8)) return rc;
        d_nk = b->nk.as<uint64_t>();
    }
    if (int rc = query_host(b, seqs, offsets, n, step, d_hits, hits_out, d_nk, nullptr, hit_bytes, nullptr,
                            wire_width(max_nk, hit_bytes)))
        return rc;
    if (num_kmers_out) HIPCHK(hipMemcpyAsync(num_kmers_out, d_nk, n * 8, hipMemcpyDeviceToHost, b->stream));
    HIPCHK(hipStreamSynchronize(b->stream));
    return XS_OK;
}

int xs_query(xs_bank* b, const char* seqs, const uint64_t* offsets, uint64_t n, uint32_t step,
             uint32_t* hits_out, uint64_t* num_kmers_out) {
    return xs::guard([&]() -> int {
        return query_impl(b, seqs, offsets, n, step, hits_out, 4, num_kmers_out);
    });
}

int xs_query_hits(xs_bank* b, const char* seqs, const uint64_t* offsets, uint64_t n, uint32_t step,
                  void* hits_out, int hit_bytes, uint64_t* num_kmers_out) {
    return xs::guard([&]() -> int {
        return query_impl(b, seqs, offsets, n, step, hits_out, hit_bytes, num_kmers_out);
    });
}

int xs_query_hits_device(xs_bank* b, const void* d_seqs, uint64_t seq_bytes, const uint64_t* d_offsets, uint64_t n,
                         uint64_t max_len, uint32_t step, void* hits_out, int hit_bytes, uint64_t* num_kmers_out,
                         uint64_t* totals_out) {
    return xs::guard([&]() -> int {
        if (!b || (n && (!d_seqs || !d_offsets))) return fail(XS_ERR_ARG, "null argument");
        if (hit_bytes != 1 && hit_bytes != 2 && hit_bytes != 4) return fail(XS_ERR_ARG, "hit_bytes must be 1, 2 or 4");
        if (step == 0) return fail(XS_ERR_ARG, "step must be >= 1");
        const uint64_t max_nk = max_len >= b->k ? (max_len - b->k) / step + 1 : 0;
        if (hits_out && hit_bytes != 4) {
            const uint64_t cap = hit_bytes == 1 ? 0xFFu : 0xFFFFu;
            if (max_nk > cap)
                return fail(XS_ERR_ARG, "a read has %llu sampled k-mers: counts may not fit %d byte(s)",
                            (unsigned long long)max_nk, hit_bytes);
        }
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        const uint64_t cols = b->kind == XS_BANK_RBLOOM ? 1 : b->D;
        if (n == 0) {
            if (totals_out) memset(totals_out, 0, (cols + 1) * 8);
            return XS_OK;
        }
        uint32_t* d_hits = nullptr;
        if (hits_out) {
            if (int rc = b->hits.ensure(n * cols * 4)) return rc;
            d_hits = b->hits.as<uint32_t>();
        }
        if (num_kmers_out)
            if (int rc = b->nk.ensure(n * 8)) return rc;
        std::vector<uint64_t> tot(totals_out ? cols + 1 : 0);
        const DevReads dev{static_cast<const uint8_t*>(d_seqs), seq_bytes, d_offsets};
        if (int rc = query_host(b, nullptr, nullptr, n, step, d_hits, hits_out, num_kmers_out ? b->nk.as<uint64_t>() : nullptr,
                                totals_out ? tot.data() : nullptr, hit_bytes, &dev))
            return rc;
        if (num_kmers_out) HIPCHK(hipMemcpyAsync(num_kmers_out, b->nk.p, n * 8, hipMemcpyDeviceToHost, b->stream));
        HIPCHK(hipStreamSynchronize(b->stream));
        if (totals_out) memcpy(totals_out, tot.data(), (cols + 1) * 8);
        return XS_OK;
    });
}

int xs_memcpy_to_host(void* host, const void* dev, uint64_t bytes) {
    return xs::guard([&]() -> int {
        if (bytes && (!host || !dev)) return fail(XS_ERR_ARG, "null argument");
        if (bytes) HIPCHK(hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost));
        return XS_OK;
    });
}

int xs_memcpy_device(void* dst, const void* src, uint64_t bytes, void* stream) {
    return xs::guard([&]() -> int {
        if (bytes && (!dst || !src)) return fail(XS_ERR_ARG, "null argument");
        if (bytes) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
        return XS_OK;
    });
}

int xs_host_alloc(uint64_t bytes, void** out) {
    return xs::guard([&]() -> int {
        if (!out) return fail(XS_ERR_ARG, "null argument");
        return xs::pinned_alloc(bytes, out);
    });
}

void xs_host_free(void* p) {
    xs::guard([&] { xs::pinned_free(p); });
}

int xs_query_best(xs_bank* b, const char* seqs, const uint64_t* offsets, uint64_t n, uint32_t step,
                  uint32_t* best_doc, uint32_t* best_hits, uint64_t* num_kmers_out, uint64_t* totals_out) {
    return xs::guard([&]() -> int {
        if (!b || !offsets || ((!seqs || !best_doc) && n)) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        const uint64_t cols = b->kind == XS_BANK_RBLOOM ? 1 : b->D;
        if (n == 0) {
            if (totals_out) memset(totals_out, 0, (cols + 1) * 8);
            return XS_OK;
        }
        if (n <= kSmallReads && n * cols <= (1u << 16)) {  // a small request: the per-read call made on the host
            std::vector<uint32_t> rows(n * cols);
            std::vector<uint64_t> tot(cols + 1);
            bool done = false;
            if (int rc = query_small(b, seqs, offsets, n, step, rows.data(), 4, num_kmers_out, tot.data(), &done)) return rc;
            if (done) {
                for (uint64_t r = 0; r < n; ++r) {  // best_doc_kernel's rule: a unique maximum, else ambiguous
                    const uint32_t* row = rows.data() + r * cols;
                    uint32_t m = 0, arg = 0, cnt = 0;
                    for (uint64_t c = 0; c < cols; ++c) {
                        if (cnt == 0 || row[c] > m) {
                            m = row[c];
                            arg = (uint32_t)c;
                            cnt = 1;
                        } else if (row[c] == m) {
                            ++cnt;
                        }
                    }
                    best_doc[r] = cnt == 1 ? arg : kBestAmbiguous;
                    if (best_hits) best_hits[r] = m;
                }
                if (totals_out) memcpy(totals_out, tot.data(), (cols + 1) * 8);
                return XS_OK;
            }
        }
        if (int rc = b->hits.ensure(n * cols * 4)) return rc;
        if (int rc = b->nk.ensure(n * 8)) return rc;
        if (int rc = b->best.ensure(n * 8)) return rc;
        uint32_t* d_hits = b->hits.as<uint32_t>();
        uint32_t* d_best = b->best.as<uint32_t>();
        uint32_t* d_bhits = d_best + n;
        std::vector<uint64_t> tot(totals_out ? cols + 1 : 0);
        if (int rc = query_host(b, seqs, offsets, n, step, d_hits, nullptr, b->nk.as<uint64_t>(),
                                totals_out ? tot.data() : nullptr))
            return rc;
        HIPCHK(launch_best_doc(d_hits, n, cols, d_best, d_bhits, b->stream));
        HIPCHK(hipMemcpyAsync(best_doc, d_best, n * 4, hipMemcpyDeviceToHost, b->stream));
        if (best_hits) HIPCHK(hipMemcpyAsync(best_hits, d_bhits, n * 4, hipMemcpyDeviceToHost, b->stream));
        if (num_kmers_out)
            HIPCHK(hipMemcpyAsync(num_kmers_out, b->nk.p, n * 8, hipMemcpyDeviceToHost, b->stream));
        HIPCHK(hipStreamSynchronize(b->stream));
        if (totals_out) memcpy(totals_out, tot.data(), (cols + 1) * 8);
        return XS_OK;
    });
}

int xs_gather_reads_device(const void* d_seqs, const uint64_t* d_offsets, const uint32_t* d_index, uint64_t m,
                           void* d_out_seqs, const uint64_t* d_out_offsets, void* stream) {
    return xs::guard([&]() -> int {
        if (m && (!d_seqs || !d_offsets || !d_index || !d_out_seqs || !d_out_offsets))
            return fail(XS_ERR_ARG, "null argument");
        HIPCHK(launch_gather_reads(static_cast<const uint8_t*>(d_seqs), d_offsets, d_index, m,
                                   static_cast<uint8_t*>(d_out_seqs), d_out_offsets, static_cast<hipStream_t>(stream)));
        return XS_OK;
    });
}

int xs_best_device(const uint32_t* d_hits, uint64_t n, uint64_t num_docs, uint32_t* d_best_doc,
                   uint32_t* d_best_hits, void* stream) {
    return xs::guard([&]() -> int {
        if ((!d_hits || !d_best_doc) && n) return fail(XS_ERR_ARG, "null argument");
        if (num_docs == 0) return fail(XS_ERR_ARG, "num_docs must be >= 1");
        HIPCHK(launch_best_doc(d_hits, n, num_docs, d_best_doc, d_best_hits, static_cast<hipStream_t>(stream)));
        return XS_OK;
    });
}

int xs_query_totals(xs_bank* b, const char* seqs, const uint64_t* offsets, uint64_t n,
                    uint32_t step, uint64_t* totals_out, uint64_t* total_kmers_out) {
    return xs::guard([&]() -> int {
        if (!b || !offsets || (!seqs && n) || !totals_out) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        const uint64_t cols = b->kind == XS_BANK_RBLOOM ? 1 : b->D;
        if (n == 0) {
            memset(totals_out, 0, cols * 8);
            if (total_kmers_out) *total_kmers_out = 0;
            return XS_OK;
        }
        std::vector<uint64_t> t(cols + 1);
        bool done = false;
        if (int rc = query_small(b, seqs, offsets, n, step, nullptr, 4, nullptr, t.data(), &done)) return rc;
        if (!done)
            if (int rc = query_host(b, seqs, offsets, n, step, nullptr, nullptr, nullptr, t.data())) return rc;
        memcpy(totals_out, t.data(), cols * 8);
        if (total_kmers_out) *total_kmers_out = t[cols];
        return XS_OK;
    });
}

int xs_query_device(xs_bank* b, const void* d_seqs, uint64_t seq_bytes, const uint64_t* d_offsets,
                    uint64_t n, uint32_t step, uint32_t* d_hits, uint64_t* d_num_kmers,
                    uint64_t* d_totals, void* stream) {
    return xs::guard([&]() -> int {
        if (!b || !d_offsets || (!d_seqs && n)) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        hipStream_t s = static_cast<hipStream_t>(stream);  // NULL = the null (legacy default) stream
        if (n == 0) {
            if (d_totals) {
                const uint64_t cols = b->kind == XS_BANK_RBLOOM ? 2 : b->D + 1;
                HIPCHK(hipMemsetAsync(d_totals, 0, cols * 8, s));
            }
            return XS_OK;
        }
        Inputs in{static_cast<const uint8_t*>(d_seqs), seq_bytes, d_offsets, n};
        return run_query(b, in, step, d_hits, d_num_kmers, d_totals, s);
    });
}

int xs_mlst_sum(xs_bank* b, const uint32_t* hits, const uint32_t* seq_of_chunk, uint64_t n_chunks,
                uint64_t n_seqs, uint32_t threshold, uint64_t* scores) {
    return xs::guard([&]() -> int {
        if (!b || (!hits && n_chunks) || (!seq_of_chunk && n_chunks) || !scores)
            return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        const uint64_t D = b->D;
        for (uint64_t c = 0; c < n_chunks; ++c)
            if (seq_of_chunk[c] >= n_seqs) return fail(XS_ERR_ARG, "seq_of_chunk[%llu] out of range", (unsigned long long)c);
        if (n_seqs == 0) return XS_OK;
        if (int rc = ws_enter(b, b->stream)) return rc;
        if (int rc = b->hits.ensure(n_chunks * D * 4 + 4)) return rc;
        if (int rc = b->tmp.ensure(n_chunks * 4 + 4)) return rc;
        if (int rc = b->totals.ensure(n_seqs * D * 8)) return rc;
        if (n_chunks) {
            HIPCHK(hipMemcpyAsync(b->hits.p, hits, n_chunks * D * 4, hipMemcpyHostToDevice, b->stream));
            HIPCHK(hipMemcpyAsync(b->tmp.p, seq_of_chunk, n_chunks * 4, hipMemcpyHostToDevice, b->stream));
        }
        HIPCHK(hipMemsetAsync(b->totals.p, 0, n_seqs * D * 8, b->stream));
        HIPCHK(launch_mlst_sum(b->hits.as<uint32_t>(), b->tmp.as<uint32_t>(), n_chunks, D, threshold,
                               b->totals.as<unsigned long long>(), nullptr, nullptr, b->stream));
        HIPCHK(hipMemcpyAsync(scores, b->totals.p, n_seqs * D * 8, hipMemcpyDeviceToHost, b->stream));
        HIPCHK(hipStreamSynchronize(b->stream));
        return XS_OK;
    });
}

int xs_mlst_query(xs_bank* b, const char* seqs, const uint64_t* offsets, uint64_t n_direct, uint64_t n_chunks,
                  const uint32_t* chunk_owner, uint64_t n_owners, uint32_t step, uint32_t threshold,
                  uint32_t* direct_hits, uint64_t* owner_scores, uint32_t* owner_first,
                  uint32_t* owner_first_score) {
    return xs::guard([&]() -> int {
        const uint64_t n = n_direct + n_chunks;
        if (!b || !offsets || (!seqs && n) || (n_chunks && !chunk_owner)) return fail(XS_ERR_ARG, "null argument");
        if (b->kind == XS_BANK_RBLOOM) return fail(XS_ERR_ARG, "MLST queries need a COBS bank");
        if (owner_first_score && !owner_first) return fail(XS_ERR_ARG, "owner_first_score needs owner_first");
        for (uint64_t c = 0; c < n_chunks; ++c)
            if (chunk_owner[c] >= n_owners || (c && chunk_owner[c] < chunk_owner[c - 1]))
                return fail(XS_ERR_ARG, "chunk_owner must be non-decreasing and < n_owners (chunk %llu)",
                            (unsigned long long)c);
        if (n_chunks >= (1ull << 32) - 1) return fail(XS_ERR_ARG, "at most 2^32-2 chunks per call");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        const uint64_t D = b->D, od = n_owners * D;
        if (n_owners) {
            if (owner_scores) memset(owner_scores, 0, od * 8);
            if (owner_first) memset(owner_first, 0xFF, od * 4);
            if (owner_first_score) memset(owner_first_score, 0, od * 4);
        }
        if (n == 0) return XS_OK;
        if (int rc = ws_enter(b, b->stream)) return rc;
        if (int rc = b->hits.ensure(n * D * 4)) return rc;
        uint32_t* d_hits = b->hits.as<uint32_t>();
        // every record probed in one pass; only the direct rows cross to the host
        if (int rc = query_host(b, seqs, offsets, n, step, d_hits, nullptr, nullptr, nullptr)) return rc;
        if (n_direct && direct_hits)
            if (int rc = d2h_pageable(b, direct_hits, d_hits, n_direct * D * 4, b->stream)) return rc;
        if (n_chunks && n_owners) {
            if (int rc = ws_enter(b, b->stream)) return rc;
            if (int rc = b->tmp.ensure(n_chunks * 4)) return rc;
            if (int rc = b->totals.ensure(od * 8)) return rc;
            if (int rc = b->best.ensure(od * 8)) return rc;
            uint32_t* d_first = b->best.as<uint32_t>();
            uint32_t* d_fscore = d_first + od;
            HIPCHK(hipMemcpyAsync(b->tmp.p, chunk_owner, n_chunks * 4, hipMemcpyHostToDevice, b->stream));
            HIPCHK(hipMemsetAsync(b->totals.p, 0, od * 8, b->stream));
            HIPCHK(hipMemsetAsync(d_first, 0xFF, od * 4, b->stream));
            HIPCHK(hipMemsetAsync(d_fscore, 0, od * 4, b->stream));
            HIPCHK(launch_mlst_sum(d_hits + n_direct * D, b->tmp.as<uint32_t>(), n_chunks, D, threshold,
                                   b->totals.as<unsigned long long>(), d_first, d_fscore, b->stream));
            if (owner_scores) HIPCHK(hipMemcpyAsync(owner_scores, b->totals.p, od * 8, hipMemcpyDeviceToHost, b->stream));
            if (owner_first) HIPCHK(hipMemcpyAsync(owner_first, d_first, od * 4, hipMemcpyDeviceToHost, b->stream));
            if (owner_first_score)
                HIPCHK(hipMemcpyAsync(owner_first_score, d_fscore, od * 4, hipMemcpyDeviceToHost, b->stream));
            if (int rc = ws_leave(b, b->stream)) return rc;
        }
        HIPCHK(hipStreamSynchronize(b->stream));
        return XS_OK;
    });
}

int xs_bank_set_profiling(xs_bank* b, int on) {
    return xs::guard([&]() -> int {
        if (!b) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        if (on && !b->profiling) {
            HIPCHK(hipSetDevice(b->device));
            if (int rc = b->rows_read.ensure(sizeof(uint64_t))) return rc;
            HIPCHK(hipMemsetAsync(b->rows_read.p, 0, sizeof(uint64_t), b->stream));
            HIPCHK(hipStreamSynchronize(b->stream));
        }
        if (on != 0 && !b->profiling) {  // a fresh profiling session: no marks left from an earlier one
            b->pass_used = 0;
            b->events_used = 0;
        }
        b->profiling = on != 0;
        return XS_OK;
    });
}

int xs_bank_probe_rows(xs_bank* b, uint64_t* rows) {
    return xs::guard([&]() -> int {
        if (!b || !rows) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        *rows = 0;
        if (b->kind != XS_BANK_RBLOOM || !b->rows_read.p) return XS_OK;
        HIPCHK(hipSetDevice(b->device));
        HIPCHK(hipDeviceSynchronize());  // probes may have run on a caller's stream
        HIPCHK(hipMemcpy(rows, b->rows_read.p, sizeof(uint64_t), hipMemcpyDeviceToHost));
        HIPCHK(hipMemset(b->rows_read.p, 0, sizeof(uint64_t)));
        return XS_OK;
    });
}

int xs_bank_probe_path(const xs_bank* b, int* path) {
    return xs::guard([&]() -> int {
        if (!b || !path) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(const_cast<xs_bank*>(b)->mu);  // after any query in flight on the handle
        *path = b->last_path;
        return XS_OK;
    });
}

int xs_bank_set_probe_options(xs_bank* b, const xs_probe_options_t* o) {
    return xs::guard([&]() -> int {
        if (!b || !o) return fail(XS_ERR_ARG, "null argument");
        if (o->cobs_part < 0 || o->cobs_part > 4) return fail(XS_ERR_ARG, "cobs_part must be 0..4");
        if (o->bloom_part < 0 || o->bloom_part > 3) return fail(XS_ERR_ARG, "bloom_part must be 0..3");
        if (o->workspace_mib < 1) return fail(XS_ERR_ARG, "workspace_mib must be >= 1");
        if (o->small_calls != 0 && o->small_calls != 1) return fail(XS_ERR_ARG, "small_calls must be 0 or 1");
        std::lock_guard<std::mutex> lk(b->mu);  // after any query in flight on the handle
        b->opt.cobs_part = o->cobs_part;
        b->opt.bloom_part = o->bloom_part;
        b->opt.workspace_mib = o->workspace_mib;
        b->opt.small_calls = o->small_calls;
        return XS_OK;
    });
}

int xs_bank_workspace_bytes(const xs_bank* b, uint64_t* held, uint64_t* peak) {
    return xs::guard([&]() -> int {
        if (!b || !held || !peak) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(const_cast<xs_bank*>(b)->mu);
        *held = b->ws_acct.held;
        *peak = b->ws_acct.peak;
        return XS_OK;
    });
}

int xs_bank_get_probe_options(const xs_bank* b, xs_probe_options_t* o) {
    return xs::guard([&]() -> int {
        if (!b || !o) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(const_cast<xs_bank*>(b)->mu);
        o->cobs_part = b->opt.cobs_part;
        o->bloom_part = b->opt.bloom_part;
        o->workspace_mib = b->opt.workspace_mib;
        o->small_calls = b->opt.small_calls;
        return XS_OK;
    });
}

int xs_bank_last_probe_ms(xs_bank* b, float* ms) {
    return xs::guard([&]() -> int {
        if (!b || !ms) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        if (b->events_used == 0) return fail(XS_ERR_ARG, "no profiled query on this handle");
        HIPCHK(hipSetDevice(b->device));
        auto& ev = b->events[b->events_used - 1];
        HIPCHK(hipEventSynchronize(ev.second));
        HIPCHK(hipEventElapsedTime(ms, ev.first, ev.second));
        return XS_OK;
    });
}

int xs_bank_probe_stats(xs_bank* b, uint64_t* count, double* total_ms, float* max_ms) {
    return xs::guard([&]() -> int {
        if (!b || !count || !total_ms) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        double tot = 0.0;
        float mx = 0.0f;
        for (size_t i = 0; i < b->events_used; ++i) {
            float ms = 0.0f;
            HIPCHK(hipEventSynchronize(b->events[i].second));
            HIPCHK(hipEventElapsedTime(&ms, b->events[i].first, b->events[i].second));
            tot += ms;
            mx = ms > mx ? ms : mx;
        }
        *count = b->events_used;
        *total_ms = tot;
        if (max_ms) *max_ms = mx;
        b->events_used = 0;
        return XS_OK;
    });
}

int xs_bank_pass_stats(xs_bank* b, double* ms, uint64_t* count) {
    return xs::guard([&]() -> int {
        if (!b || !ms || !count) return fail(XS_ERR_ARG, "null argument");
        std::lock_guard<std::mutex> lk(b->mu);
        HIPCHK(hipSetDevice(b->device));
        for (int t = 0; t < kPassTags; ++t) {
            ms[t] = 0.0;
            count[t] = 0;
        }
        for (size_t i = 1; i < b->pass_used; ++i) {
            const int t = b->pass_tag[i];
            if (t < 0 || t >= kPassTags) continue;  // a query's opening mark
            float x = 0.0f;
            HIPCHK(hipEventSynchronize(b->pass_ev[i]));
            HIPCHK(hipEventElapsedTime(&x, b->pass_ev[i - 1], b->pass_ev[i]));
            ms[t] += x;
            ++count[t];
        }
        b->pass_used = 0;
        return XS_OK;
    });
}

void xs_bank_close(xs_bank* b) {
    xs::guard([&] {
        if (!b) return;
        (void)hipSetDevice(b->device);
        if (b->ws_used) (void)hipEventSynchronize(b->ws_ev);  // the last call's stream may be the caller's
        if (b->ws_ev) (void)hipEventDestroy(b->ws_ev);
        if (b->stream) (void)hipStreamSynchronize(b->stream);
        for (hipStream_t st : {b->copy_stream, b->d2h_stream})
            if (st) (void)hipStreamSynchronize(st);
        for (auto& ev : b->stage_ev)
            if (ev) (void)hipEventDestroy(ev);
        for (auto& ev : b->hstage_ev)
            if (ev) (void)hipEventDestroy(ev);
        if (b->bloom_ev) (void)hipEventDestroy(b->bloom_ev);
        for (auto& ev : b->chunk_ev) (void)hipEventDestroy(ev);
        for (auto& ev : b->events) {
            (void)hipEventDestroy(ev.first);
            (void)hipEventDestroy(ev.second);
        }
        for (auto& ev : b->pass_ev) (void)hipEventDestroy(ev);
        for (hipStream_t st : {b->stream, b->copy_stream, b->d2h_stream})
            if (st) (void)hipStreamDestroy(st);
        delete b;  // DevBuf destructors free device memory
    });
}

}  // extern "C"
