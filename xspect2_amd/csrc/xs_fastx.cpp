// xs_fastx.cpp — native FASTA/FASTQ reader that feeds the probe path
// (SURVEY.md §8 f1).  It replaces Bio.SeqIO.parse, which the reference reaches
// through get_record_iterator (src/xspect/file_io.py:47-79) for every
// predict() on a file (probabilistic_filter_model.py:316-330).
//
// Record semantics, restated from Biopython's SimpleFastaParser and
// FastqGeneralIterator (Bio is not installed offline; the pure-Python
// restatement oracle/fastx.py is the checker, tests/test_fastx.py):
//   * lines end at '\n'; every line is right-stripped of ASCII whitespace;
//   * FASTA: text before the first '>' line is skipped; title = header minus
//     '>', id = first whitespace-separated token of the title ("" if none);
//     sequence = the record's lines joined, with ' ' and '\r' removed;
//   * FASTQ: blank lines between records are skipped; a header must start
//     with '@'; sequence lines run to the first line starting with '+' (whose
//     caption, if any, must equal the title); no ' ' or '\t' in the sequence;
//     quality lines are read until they hold >= len(sequence) characters and
//     must then hold exactly len(sequence).
//
// A batch covers a window of the memory-mapped file cut at a record start.
// The window is split at record starts into one part per thread, the parts
// are parsed concurrently and copied into one packed batch (bytes + offsets,
// the layout xs_query takes).  Two batches are double-buffered so the caller
// can probe batch i while batch i+1 is parsed.  FASTQ with wrapped sequence
// or quality lines cannot be split safely; such files are parsed by one
// thread.
//
// Device mode (xs_fastx_open_device): the host only copies each window's text
// into pinned memory (parallel pread) and on to HBM, overlapped with the
// caller's work on the previous batch; the records are found on the GPU
// (xs_fastx_dev.hip).  A window the device rules do not cover is parsed here
// instead, so both modes yield the same batches.
#include "../../include/xspect_hip.h"

#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "xs_internal.h"

namespace {

inline bool is_ws(unsigned char c) {
    return c == ' ' || (c >= '\t' && c <= '\r') || (c >= 0x1c && c <= 0x1f);
}

inline const char* rstrip(const char* b, const char* e) {
    while (e > b && is_ws((unsigned char)e[-1])) --e;
    return e;
}

// Next line [b, le) of [p, end) (le excludes '\n'); advances p.
inline bool next_line(const char*& p, const char* end, const char*& b, const char*& le) {
    if (p >= end) return false;
    b = p;
    const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
    if (nl) {
        le = nl;
        p = nl + 1;
    } else {
        le = end;
        p = end;
    }
    return true;
}

struct HostBuf {
    char* p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    int ensure(size_t bytes) {  // contents are not preserved
        if (bytes <= cap && p) return XS_OK;
        release();
        size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
        if (pinned) {
            if (xs::pinned_alloc(want, reinterpret_cast<void**>(&p)) != XS_OK) {
                p = nullptr;
                return xs::set_error(XS_ERR_HIP, "pinned allocation failed for the reader's batch buffer");
            }
        } else {
            p = static_cast<char*>(malloc(want));
            if (!p) return xs::set_error(XS_ERR_ARG, "out of host memory for the reader's batch buffer");
        }
        cap = want;
        return XS_OK;
    }
    void release() {
        if (p) {
            if (pinned) xs::pinned_free(p);
            else free(p);
        }
        p = nullptr;
        cap = 0;
    }
    ~HostBuf() { release(); }
};

// One thread's records.
struct Part {
    std::string seq, ids, descs;
    std::vector<uint64_t> lens, id_lens, desc_lens;
    std::string err;
    const char* stop = nullptr;  // where parsing ended (next record start)
    void clear() {
        seq.clear();
        ids.clear();
        descs.clear();
        lens.clear();
        id_lens.clear();
        desc_lens.clear();
        err.clear();
        stop = nullptr;
    }
};

// Record title (header minus '>'/'@', right-stripped) and id (its first token).
void push_id(Part& out, const char* tb, const char* te) {
    out.descs.append(tb, (size_t)(te - tb));
    out.desc_lens.push_back((uint64_t)(te - tb));
    while (tb < te && is_ws((unsigned char)*tb)) ++tb;
    const char* t = tb;
    while (t < te && !is_ws((unsigned char)*t)) ++t;
    out.ids.append(tb, (size_t)(t - tb));
    out.id_lens.push_back((uint64_t)(t - tb));
}

// FASTA records of [p, end).  `budget`: stop at the first record that starts
// at or beyond p + budget (0: no limit).
void parse_fasta(const char* p, const char* end, size_t budget, Part& out) {
    const char* limit = budget ? p + budget : end;
    const char *b, *le;
    bool have = false;
    size_t seq0 = 0;
    const char* q = p;
    for (;;) {
        const char* line_start = q;
        if (!next_line(q, end, b, le)) break;
        if (le > b && *b == '>') {
            if (have) {
                out.lens.push_back(out.seq.size() - seq0);
                if (line_start >= limit) {
                    out.stop = line_start;
                    return;
                }
            }
            have = true;
            seq0 = out.seq.size();
            push_id(out, b + 1, rstrip(b + 1, le));
        } else if (have) {
            const char* e = rstrip(b, le);
            const char* s = b;
            while (s < e) {  // drop ' ' and '\r' inside the line
                const char* run = s;
                while (s < e && *s != ' ' && *s != '\r') ++s;
                out.seq.append(run, (size_t)(s - run));
                while (s < e && (*s == ' ' || *s == '\r')) ++s;
            }
        }
    }
    if (have) out.lens.push_back(out.seq.size() - seq0);
    out.stop = end;
}

void fastq_error(Part& out, const char* msg, const char* tb, const char* te) {
    out.err = std::string(msg) + " (record '" + std::string(tb, (size_t)std::min<ptrdiff_t>(te - tb, 200)) + "')";
}

void parse_fastq(const char* p, const char* end, size_t budget, Part& out) {
    const char* limit = budget ? p + budget : end;
    const char *b, *le;
    const char* q = p;
    for (;;) {
        // header (blank lines skipped)
        const char* rec_start = q;
        bool got = false;
        while (next_line(q, end, b, le)) {
            if (rstrip(b, le) == b) {
                rec_start = q;
                continue;
            }
            got = true;
            break;
        }
        if (!got) break;
        if (rec_start >= limit && !out.lens.empty()) {
            out.stop = rec_start;
            return;
        }
        if (*b != '@') {
            out.err = "Records in Fastq files should start with '@' character";
            return;
        }
        const char* tb = b + 1;
        const char* te = rstrip(tb, le);
        // sequence lines up to the '+' line
        const size_t seq0 = out.seq.size();
        bool plus = false;
        while (next_line(q, end, b, le)) {
            if (le > b && *b == '+') {
                plus = true;
                break;
            }
            out.seq.append(b, (size_t)(rstrip(b, le) - b));
        }
        const size_t slen = out.seq.size() - seq0;
        if (!plus) {
            fastq_error(out, slen ? "End of file without quality information." : "Unexpected end of file",
                        tb, te);
            return;
        }
        const char* ce = rstrip(b + 1, le);
        if (ce > b + 1 && ((size_t)(ce - (b + 1)) != (size_t)(te - tb) || memcmp(b + 1, tb, (size_t)(te - tb)) != 0)) {
            fastq_error(out, "Sequence and quality captions differ.", tb, te);
            return;
        }
        if (memchr(out.seq.data() + seq0, ' ', slen) || memchr(out.seq.data() + seq0, '\t', slen)) {
            fastq_error(out, "Whitespace is not allowed in the sequence.", tb, te);
            return;
        }
        size_t qlen = 0;
        while (qlen < slen && next_line(q, end, b, le)) qlen += (size_t)(rstrip(b, le) - b);
        if (qlen != slen) {
            char msg[128];
            snprintf(msg, sizeof(msg), "Lengths of sequence and quality values differs (%zu and %zu).", slen, qlen);
            fastq_error(out, msg, tb, te);
            return;
        }
        push_id(out, tb, te);
        out.lens.push_back(slen);
    }
    out.stop = end;
}

// Record start at or after `pos` in [lo, end): FASTA '>' at a line start.
const char* fasta_boundary(const char* lo, const char* pos, const char* end) {
    if (pos <= lo) return lo;
    const char* p = pos - 1;
    while (p < end) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
        if (!nl || nl + 1 >= end) return end;
        if (nl[1] == '>') return nl + 1;
        p = nl + 1;
    }
    return end;
}

// FASTQ (4-line records) record start at or after `pos`: a line "@..." whose
// third line starts with '+', whose fourth line is as long as its second, and
// which is followed by end of text or another '@' line.
const char* fastq_boundary(const char* lo, const char* pos, const char* end) {
    if (pos <= lo) return lo;
    const char* p = pos - 1;
    while (p < end) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
        if (!nl || nl + 1 >= end) return end;
        const char* cand = nl + 1;
        p = cand;
        if (*cand != '@') continue;
        const char* q = cand;
        const char *b[4], *le[4];
        int n = 0;
        while (n < 4 && next_line(q, end, b[n], le[n])) ++n;
        if (n < 4) continue;
        if (le[2] <= b[2] || *b[2] != '+') continue;
        if (rstrip(b[1], le[1]) - b[1] != rstrip(b[3], le[3]) - b[3]) continue;
        if (q < end && *q != '@') continue;
        return cand;
    }
    return end;
}

// True if some FASTQ record among the first ones of the file wraps its
// sequence or quality over several lines (then the file is not split).
bool fastq_wrapped(const char* p, const char* end) {
    const char* stop = p + std::min<size_t>((size_t)(end - p), 1 << 20);
    const char *b, *le;
    const char* q = p;
    int records = 0;
    while (q < stop && records < 1000) {
        if (!next_line(q, end, b, le)) break;
        if (rstrip(b, le) == b) continue;
        if (*b != '@') return true;  // malformed: let the sequential parser report it
        int seq_lines = 0;
        bool plus = false;
        size_t slen = 0;
        while (next_line(q, end, b, le)) {
            if (le > b && *b == '+') {
                plus = true;
                break;
            }
            slen += (size_t)(rstrip(b, le) - b);
            ++seq_lines;
        }
        if (!plus || seq_lines > 1) return true;
        if (slen) {
            if (!next_line(q, end, b, le)) return true;
            if ((size_t)(rstrip(b, le) - b) != slen) return true;
        }
        ++records;
    }
    return false;
}

// Wrapped FASTQ cannot be cut by pattern: the first record start at or after
// `pos`, found by walking the records from the start of the text (the same
// line rules as parse_fastq, nothing copied).  A malformed record ends the
// walk there; the part that holds it reports the error when parsed.
const char* fastq_boundary_sequential(const char* lo, const char* pos, const char* end) {
    const char *b, *le;
    const char* q = lo;
    for (;;) {
        const char* rec_start = q;
        bool got = false;
        while (next_line(q, end, b, le)) {
            if (rstrip(b, le) == b) {
                rec_start = q;
                continue;
            }
            got = true;
            break;
        }
        if (!got) return end;
        if (rec_start >= pos) return rec_start;
        if (*b != '@') return rec_start;
        size_t slen = 0;
        bool plus = false;
        while (next_line(q, end, b, le)) {
            if (le > b && *b == '+') {
                plus = true;
                break;
            }
            slen += (size_t)(rstrip(b, le) - b);
        }
        if (!plus) return rec_start;
        size_t qlen = 0;
        while (qlen < slen && next_line(q, end, b, le)) qlen += (size_t)(rstrip(b, le) - b);
    }
}

struct Batch {
    HostBuf seqs, offs, ids, id_offs, descs, desc_offs;
    uint64_t n = 0, seq_bytes = 0;
};

// ---- device mode -------------------------------------------------------------
bool fx_trace();
double fx_ms();
// Pinned host and device buffers outlive their reader in a process-wide pool:
// pinning host memory costs (xs::pinned_alloc) and a hipFree synchronises
// the device, so a reader per input file would otherwise pay more for its
// buffers than for its parse.  Reuse takes the smallest pooled buffer that
// fits and is at most 4x the request.
struct BufPool {
    struct Entry {
        void* p;
        size_t cap;
        int device;  // -1: pinned host memory
    };
    std::mutex mu;
    std::vector<Entry> free_list;
    size_t bytes = 0;
    static constexpr size_t kMaxBytes = size_t(6) << 30;
    static constexpr size_t kMaxEntries = 96;
    void* take(size_t want, int device, size_t* cap) {
        std::lock_guard<std::mutex> g(mu);
        size_t best = free_list.size();
        for (size_t i = 0; i < free_list.size(); ++i) {
            const Entry& e = free_list[i];
            if (e.device == device && e.cap >= want && e.cap / 4 <= want &&
                (best == free_list.size() || e.cap < free_list[best].cap))
                best = i;
        }
        if (best == free_list.size()) return nullptr;
        void* p = free_list[best].p;
        *cap = free_list[best].cap;
        bytes -= *cap;
        free_list.erase(free_list.begin() + (ptrdiff_t)best);
        return p;
    }
    bool give(void* p, size_t cap, int device) {  // false: the caller frees it
        std::lock_guard<std::mutex> g(mu);
        if (bytes + cap > kMaxBytes || free_list.size() >= kMaxEntries) return false;
        free_list.push_back({p, cap, device});
        bytes += cap;
        return true;
    }
};
BufPool g_pool;

struct PinBuf {
    char* p = nullptr;
    size_t cap = 0;
    // contents are not preserved; exact: no 1/8 headroom (a fixed-size buffer)
    int ensure(size_t bytes, bool exact = false) {
        if (bytes <= cap && p) return XS_OK;
        release();
        if ((p = static_cast<char*>(g_pool.take(bytes, -1, &cap)))) return XS_OK;
        const size_t want = std::max<size_t>(exact ? bytes : bytes + bytes / 8, 1 << 16);
        const double t0 = fx_ms();
        if (xs::pinned_alloc(want, reinterpret_cast<void**>(&p)) != XS_OK) {
            p = nullptr;
            return xs::set_error(XS_ERR_HIP, "pinned allocation failed for the device reader");
        }
        if (fx_trace()) fprintf(stderr, "[fastx-device] pinned %zu B in %.2f ms\n", want, fx_ms() - t0);
        cap = want;
        return XS_OK;
    }
    void release() {
        if (p && !g_pool.give(p, cap, -1)) {
            if (fx_trace()) fprintf(stderr, "[fastx-device] unpinned %zu B\n", cap);
            xs::pinned_free(p);
        }
        p = nullptr;
        cap = 0;
    }
    ~PinBuf() { release(); }
};

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    int device = 0;
    int ensure(size_t bytes) {  // contents are not preserved
        if (bytes <= cap && p) return XS_OK;
        release();
        if ((p = g_pool.take(bytes, device, &cap))) return XS_OK;
        const size_t want = std::max<size_t>(bytes + bytes / 8, 4096);
        if (hipMalloc(&p, want) != hipSuccess) {
            p = nullptr;
            return xs::set_error(XS_ERR_HIP, "hipMalloc failed for the device reader");
        }
        cap = want;
        return XS_OK;
    }
    void release() {
        if (p && !g_pool.give(p, cap, device)) {
            if (fx_trace()) fprintf(stderr, "[fastx-device] hipFree %zu B\n", cap);
            (void)hipFree(p);
        }
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const {
        return static_cast<T*>(p);
    }
    ~DBuf() { release(); }
};

constexpr size_t kPieceBytes = 4u << 20;  // pread + DMA unit of a window's text
constexpr size_t kRingMax = 64;            // most pinned pieces in flight (see DevSide::ring)
// XSPECT2_AMD_FX_RING: pinned ring pieces (read once; default 32 = 128 MiB;
// 0 = a pinned buffer the size of each window, per text slot)
size_t ring_pieces() {
    static const size_t r = [] {
        const char* e = getenv("XSPECT2_AMD_FX_RING");
        const long v = e ? atol(e) : 32;
        return (size_t)std::max<long>(0, std::min<long>(v, (long)kRingMax));
    }();
    return r;
}
// pread threads of a window load: 6 outrun the DMA (~50 GB/s) and leave the
// caller's threads their CPU share (profiles/r04_e2e_ring.txt)
constexpr size_t kLoadThreads = 6;
constexpr size_t kDevPad = 64;            // defined zero bytes past a batch's sequences

struct DevSide {
    int device = 0;
    hipStream_t stream = nullptr;  // parse kernels
    hipStream_t copy = nullptr;    // text DMA
    // Window text in two slots: the next window loads into one while the
    // current one is parsed from the other.
    hipEvent_t text_ev[2] = {nullptr, nullptr};
    hipEvent_t kern_ev = nullptr;                // a batch's device data complete
    hipEvent_t host_ev[2] = {nullptr, nullptr};  // slot s's host arrays complete
    // Window text goes to HBM through a ring of pinned pieces (ring_pieces()
    // x kPieceBytes): pinning cost ~0.19 ms per MiB with hipHostMalloc (~0.02
    // with xs::pinned_alloc's registered 2 MiB pages), and whole-window pinned
    // buffers (two of up to 288 MiB) are more than a window needs at once; the
    // ring is 128 MiB whatever the window.
    PinBuf ring;
    PinBuf pin[2];                     // XSPECT2_AMD_FX_RING=0: a window's whole text per slot
    hipEvent_t ring_ev[kRingMax] = {};  // the DMA out of ring piece r done (recorded on `copy`)
    bool ring_used[kRingMax] = {};
    PinBuf status;      // small D2H results
    DBuf text[2];       // a window's text, zero-padded to whole tiles
    DBuf tiles, tile_ofs, nl, temp, flag;
    DBuf hdr, hofs, line_src, line_len, line_ofs, rec_line, lens, maxlen;
    DBuf seq_src, seq_len, id_src, id_len, desc_src, desc_len, id_ofs, desc_ofs, ids_d, descs_d;
    DBuf seqs[2], offs[2];
    DBuf fq_blk, fq_blk_ofs, fq_status;  // FASTQ record blocks' sums and offsets, the window's status
    PinBuf ids[2], id_offs[2], descs[2], desc_offs[2], hoffs[2];
    int flip = 0;
    // Text of the next windows, loaded in order by `loader` while the caller
    // works: up to two ahead, window j+2 into window j's slot as soon as j is
    // parsed (the parse is the only reader of a slot's text).
    struct PfJob {
        size_t lo, hi;
        int slot;
        bool started, done;
        int rc;
        std::string err;
    };
    std::thread loader;
    std::mutex pf_mu;
    std::condition_variable pf_cv;
    std::deque<PfJob> pf_q;  // oldest first; popped by text_for once done
    bool pf_stop = false;
    int next_text = 0;  // text slot of the next window queued or loaded inline
    double load_ms[2] = {0, 0};  // each slot's last load_text: pread + DMA queueing
    void set_device(int dev) {
        device = dev;
        for (DBuf* b : {&text[0], &text[1], &tiles, &tile_ofs, &nl, &temp, &flag, &hdr, &hofs, &line_src, &line_len, &line_ofs,
                        &rec_line, &lens, &maxlen, &seq_src, &seq_len, &id_src, &id_len, &desc_src, &desc_len,
                        &id_ofs, &desc_ofs, &ids_d, &descs_d, &seqs[0], &seqs[1], &offs[0], &offs[1], &fq_blk,
                        &fq_blk_ofs, &fq_status})
            b->device = dev;
    }
    ~DevSide();
};

// The streams and events of closed device readers, kept for the next reader
// on the same device: creating them costs about a millisecond per open,
// as much as parsing the first window.
struct StreamSet {
    int device;
    hipStream_t stream, copy;
    hipEvent_t ev[5];  // text_ev[2], kern_ev, host_ev[2]
};
std::mutex g_ss_mu;
std::vector<StreamSet> g_ss;
constexpr size_t kStreamSetsKept = 16;

bool take_streams(DevSide& d) {
    std::lock_guard<std::mutex> g(g_ss_mu);
    for (size_t i = 0; i < g_ss.size(); ++i) {
        if (g_ss[i].device != d.device) continue;
        d.stream = g_ss[i].stream;
        d.copy = g_ss[i].copy;
        d.text_ev[0] = g_ss[i].ev[0];
        d.text_ev[1] = g_ss[i].ev[1];
        d.kern_ev = g_ss[i].ev[2];
        d.host_ev[0] = g_ss[i].ev[3];
        d.host_ev[1] = g_ss[i].ev[4];
        g_ss.erase(g_ss.begin() + (long)i);
        return true;
    }
    return false;
}

// Whole device sides of closed readers, kept for the next reader on the same
// device: their streams, events and buffers at the sizes the last file grew
// them to, so a process reading file after file allocates and pins nothing
// after its first (a reader's buffers otherwise went back to g_pool piece by
// piece and the next reader's ramp took them out in a different order,
// pinning and freeing afresh: 17 -> 26 ms per 313 MB file over six files,
// profiles/r04_e2e_ring.txt).  A batch's arrays are the reader's and are
// invalid after xs_fastx_close, as before.
// End the loader thread after the loads it has started (a queued load
// that has not started is dropped), and forget the queue.
void stop_loader(DevSide& d) {
    {
        std::lock_guard<std::mutex> g(d.pf_mu);
        d.pf_stop = true;
    }
    d.pf_cv.notify_all();
    if (d.loader.joinable()) d.loader.join();
    d.pf_stop = false;
    d.pf_q.clear();
}

std::mutex g_ds_mu;
std::vector<DevSide*> g_ds;
constexpr size_t kDevSidesKept = 4;

DevSide* take_devside(int device) {
    std::lock_guard<std::mutex> g(g_ds_mu);
    for (size_t i = 0; i < g_ds.size(); ++i) {
        if (g_ds[i]->device != device) continue;
        DevSide* d = g_ds[i];
        g_ds.erase(g_ds.begin() + (long)i);
        return d;
    }
    return nullptr;
}

// Quiesce a closed reader's device side and keep it (or destroy it when
// kDevSidesKept are kept already or its streams were never made).
void put_devside(DevSide* d) {
    if (!d) return;
    stop_loader(*d);
    bool ok = d->stream && d->copy && hipSetDevice(d->device) == hipSuccess &&
              hipStreamSynchronize(d->stream) == hipSuccess && hipStreamSynchronize(d->copy) == hipSuccess;
    if (ok) {
        d->flip = 0;
        d->next_text = 0;
        d->load_ms[0] = d->load_ms[1] = 0;
        std::lock_guard<std::mutex> g(g_ds_mu);
        if (g_ds.size() < kDevSidesKept) {
            g_ds.push_back(d);
            return;
        }
    }
    delete d;
}

DevSide::~DevSide() {
    stop_loader(*this);
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    if (copy) (void)hipStreamSynchronize(copy);
    for (hipEvent_t e : ring_ev)
        if (e) (void)hipEventDestroy(e);
    hipEvent_t* evs[5] = {&text_ev[0], &text_ev[1], &kern_ev, &host_ev[0], &host_ev[1]};
    bool all = stream && copy;
    for (hipEvent_t* e : evs) all = all && *e;
    if (all) {
        std::lock_guard<std::mutex> g(g_ss_mu);
        if (g_ss.size() < kStreamSetsKept) {
            g_ss.push_back(StreamSet{device, stream, copy, {text_ev[0], text_ev[1], kern_ev, host_ev[0], host_ev[1]}});
            return;
        }
    }
    for (hipEvent_t* e : evs)
        if (*e) (void)hipEventDestroy(*e);
    if (stream) (void)hipStreamDestroy(stream);
    if (copy) (void)hipStreamDestroy(copy);
}

}  // namespace

struct xs_fastx {
    int format = XS_FASTX_FASTA;
    int threads = 1;
    bool wrapped = false;
    int fd = -1;
    const char* base = nullptr;
    size_t size = 0;   // mapped bytes
    size_t stop = 0;   // end of this reader's text (the file, or its part)
    size_t cur = 0;
    uint64_t records = 0;
    uint64_t windows = 0;  // windows consumed (window_budget's ramp)
    Batch batch[2];
    int flip = 0;
    std::vector<Part> parts;
    DevSide* dev = nullptr;
    ~xs_fastx() {
        put_devside(dev);
        if (base && size) munmap(const_cast<char*>(base), size);
        if (fd >= 0) close(fd);
    }
};

namespace {

// Windows ramp up: the reader's k-th window takes at most first_window() << k
// bytes of text (for budgets of at least twice the first), so the caller's
// first probe starts after a small parse while the later, larger windows are
// read behind it.
// XSPECT2_AMD_FX_FIRST_MB sets the first window (MiB, read once; default 16:
// file -> totals of 1 M reads 16.8-16.9 ms against 17.0-17.5 at 32 MiB and
// 35-48 at 8 MiB, profiles/r04_e2e_first_window.txt).
size_t first_window() {
    static const size_t w = [] {
        const char* e = getenv("XSPECT2_AMD_FX_FIRST_MB");
        const long v = e ? atol(e) : 0;
        return v > 0 ? (size_t)v << 20 : (size_t)16 << 20;
    }();
    return w;
}
size_t window_budget(uint64_t max_text_bytes, uint64_t k) {
    const size_t b = std::max<uint64_t>(max_text_bytes, 1);
    const size_t w0 = first_window();
    if (b < 2 * w0 || k >= 16) return b;
    return std::min(b, w0 << k);
}

// End of the window that starts at lo: the first record start at or after
// lo + budget (the whole rest if that is within budget; one record at least).
const char* window_end(const xs_fastx* r, const char* lo, const char* end, size_t budget) {
    auto boundary = r->format == XS_FASTX_FASTA ? fasta_boundary : fastq_boundary;
    const char* hi = (size_t)(end - lo) <= budget ? end : boundary(lo, lo + budget, end);
    if (hi == lo) hi = boundary(lo, lo + 1, end);  // one record larger than the budget
    return hi;
}

// Parse [lo, hi) (cut at record starts) on up to r->threads threads into r->parts.
int parse_window(xs_fastx* r, const char* lo, const char* hi, int* nparts) {
    const bool fasta = r->format == XS_FASTX_FASTA;
    auto boundary = fasta ? fasta_boundary : fastq_boundary;
    const size_t span = (size_t)(hi - lo);
    const int T = (int)std::min<size_t>((size_t)r->threads, std::max<size_t>(1, span >> 20));  // >= 1 MiB per part
    std::vector<const char*> cut(T + 1);
    cut[0] = lo;
    cut[T] = hi;
    for (int i = 1; i < T; ++i) cut[i] = std::max(cut[i - 1], boundary(lo, lo + span * i / T, hi));
    auto work = [&](int i) {
        Part& pt = r->parts[i];
        pt.clear();
        if (cut[i] < cut[i + 1]) {
            if (fasta) parse_fasta(cut[i], cut[i + 1], 0, pt);
            else parse_fastq(cut[i], cut[i + 1], 0, pt);
        } else {
            pt.stop = cut[i + 1];
        }
    };
    xs::parallel_for(T, work);
    r->parts[T - 1].stop = hi;
    *nparts = T;
    for (int i = 0; i < T; ++i)
        if (!r->parts[i].err.empty()) return xs::set_error(XS_ERR_FORMAT, r->parts[i].err.c_str());
    return XS_OK;
}

// Concatenate r->parts[0 .. nparts) into bt (the layout xs_query takes).
int pack_parts(xs_fastx* r, Batch& bt, int nparts) {
    uint64_t n = 0, sbytes = 0, ibytes = 0, dbytes = 0;
    for (int i = 0; i < nparts; ++i) {
        n += r->parts[i].lens.size();
        sbytes += r->parts[i].seq.size();
        ibytes += r->parts[i].ids.size();
        dbytes += r->parts[i].descs.size();
    }
    if (int rc = bt.seqs.ensure(sbytes + 64)) return rc;
    if (int rc = bt.offs.ensure((n + 1) * 8)) return rc;
    if (int rc = bt.ids.ensure(ibytes + 1)) return rc;
    if (int rc = bt.id_offs.ensure((n + 1) * 8)) return rc;
    if (int rc = bt.descs.ensure(dbytes + 1)) return rc;
    if (int rc = bt.desc_offs.ensure((n + 1) * 8)) return rc;
    auto* offs = reinterpret_cast<uint64_t*>(bt.offs.p);
    auto* ioffs = reinterpret_cast<uint64_t*>(bt.id_offs.p);
    auto* doffs = reinterpret_cast<uint64_t*>(bt.desc_offs.p);
    std::vector<uint64_t> rec0(nparts + 1, 0), s0(nparts + 1, 0), i0(nparts + 1, 0), d0(nparts + 1, 0);
    for (int i = 0; i < nparts; ++i) {
        rec0[i + 1] = rec0[i] + r->parts[i].lens.size();
        s0[i + 1] = s0[i] + r->parts[i].seq.size();
        i0[i + 1] = i0[i] + r->parts[i].ids.size();
        d0[i + 1] = d0[i] + r->parts[i].descs.size();
    }
    auto pack = [&](int i) {
        const Part& pt = r->parts[i];
        if (!pt.seq.empty()) memcpy(bt.seqs.p + s0[i], pt.seq.data(), pt.seq.size());
        if (!pt.ids.empty()) memcpy(bt.ids.p + i0[i], pt.ids.data(), pt.ids.size());
        if (!pt.descs.empty()) memcpy(bt.descs.p + d0[i], pt.descs.data(), pt.descs.size());
        uint64_t so = s0[i], io = i0[i], dd = d0[i];
        for (size_t j = 0; j < pt.lens.size(); ++j) {
            offs[rec0[i] + j] = so;
            ioffs[rec0[i] + j] = io;
            doffs[rec0[i] + j] = dd;
            so += pt.lens[j];
            io += pt.id_lens[j];
            dd += pt.desc_lens[j];
        }
    };
    xs::parallel_for(nparts, pack);
    offs[n] = sbytes;
    ioffs[n] = ibytes;
    doffs[n] = dbytes;
    memset(bt.seqs.p + sbytes, 0, 64);  // defined bytes past the end
    bt.n = n;
    bt.seq_bytes = sbytes;
    return XS_OK;
}

void fill_host_batch(const xs_fastx* r, const Batch& bt, xs_fastx_batch* out) {
    out->n = bt.n;
    out->seqs = bt.seqs.p;
    out->seq_bytes = bt.seq_bytes;
    out->offsets = reinterpret_cast<const uint64_t*>(bt.offs.p);
    out->ids = bt.ids.p;
    out->id_offsets = reinterpret_cast<const uint64_t*>(bt.id_offs.p);
    out->text_offset = r->cur;
    out->text_bytes = r->stop;
    out->descs = bt.descs.p;
    out->desc_offsets = reinterpret_cast<const uint64_t*>(bt.desc_offs.p);
}

// XSPECT2_AMD_FASTX_TRACE set: one line per device window on stderr with the
// time of each phase (diagnostics of the device mode).
bool fx_trace() {
    static const bool on = getenv("XSPECT2_AMD_FASTX_TRACE") != nullptr;
    return on;
}
double fx_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
struct FxTimes {
    double load = 0, count = 0, records = 0, copy = 0;
};
thread_local FxTimes g_fx;

#define FXCHK(expr)                                                                                     \
    do {                                                                                                \
        hipError_t _e = (expr);                                                                         \
        if (_e != hipSuccess) return xs::set_error(XS_ERR_HIP, hipGetErrorString(_e));                 \
    } while (0)

// The text of [lo, hi) (file offsets) into d.text[ts] (zero-padded to whole
// tiles), through the pinned ring: host threads pread 4 MiB pieces into ring
// slots, the DMA of each piece is queued on d.copy as soon as it is in, and a
// ring slot is reused once its previous DMA has completed.
// d.text_ev[ts] marks the end.
int load_text(xs_fastx* r, size_t lo, size_t hi, int ts) {
    DevSide& d = *r->dev;
    const double t0 = fx_ms();
    FXCHK(hipSetDevice(d.device));
    const size_t span = hi - lo;
    const size_t tiles = std::max<size_t>(1, (span + xs::kFxTile - 1) / xs::kFxTile);
    const size_t padded = tiles * xs::kFxTile;
    DBuf& text = d.text[ts];
    const size_t R = ring_pieces();
    if (R) {
        if (int rc = d.ring.ensure(R * kPieceBytes, true)) return rc;
        for (size_t i = 0; i < R; ++i)
            if (!d.ring_ev[i]) FXCHK(hipEventCreateWithFlags(&d.ring_ev[i], hipEventDisableTiming));
    } else if (int rc = d.pin[ts].ensure(span + 1)) {
        return rc;
    }
    char* const host = R ? d.ring.p : d.pin[ts].p;
    // host buffer of piece p: its ring slot, or its place in the window's buffer
    auto at = [&](size_t p) { return host + (R ? p % R : p) * kPieceBytes; };
    if (int rc = text.ensure(padded + 16)) return rc;
    const size_t pieces = (span + kPieceBytes - 1) / kPieceBytes;
    // pread outruns the DMA (~50 GB/s) with a few threads; more only burn the
    // CPU share the caller's own threads need
    const int T = (int)std::max<size_t>(1, std::min<size_t>({(size_t)r->threads, kLoadThreads, pieces}));
    std::vector<uint8_t> done(pieces, 0);
    size_t queued = 0;  // pieces whose DMA is queued (in order)
    std::mutex mu;
    std::condition_variable cv;
    bool failed = false;
    auto work = [&](int t) {
        for (size_t p = (size_t)t; p < pieces; p += (size_t)T) {
            bool bad = false;
            if (R) {
                const size_t slot = p % R;
                {   // the ring slot's previous piece must be on its way before it is overwritten
                    std::unique_lock<std::mutex> g(mu);
                    cv.wait(g, [&] { return failed || p < R || queued > p - R; });
                    if (failed) return;
                }
                if (d.ring_used[slot] && hipEventSynchronize(d.ring_ev[slot]) != hipSuccess) bad = true;
            }
            char* dst = at(p);
            const size_t n = std::min(span, (p + 1) * kPieceBytes) - p * kPieceBytes;
            size_t o = 0;
            while (!bad && o < n) {
                const ssize_t got = pread(r->fd, dst + o, n - o, (off_t)(lo + p * kPieceBytes + o));
                if (got <= 0) {
                    bad = true;
                    break;
                }
                o += (size_t)got;
            }
            {
                std::lock_guard<std::mutex> g(mu);
                done[p] = 1;
                failed |= bad;
            }
            cv.notify_all();
        }
    };
    xs::ThreadGroup th;  // pread workers beside this thread, which queues each piece's DMA
    try {
        for (int t = 0; t < T; ++t) th.start(work, t);
    } catch (...) {  // the workers already started stop at `failed` before the group joins them
        {
            std::lock_guard<std::mutex> g(mu);
            failed = true;
        }
        cv.notify_all();
        throw;
    }
    int rc = XS_OK;
    for (size_t p = 0; p < pieces; ++p) {  // queue each piece's DMA as soon as it is in
        {
            std::unique_lock<std::mutex> g(mu);
            cv.wait(g, [&] { return done[p] != 0 || failed; });
            if (failed) break;
        }
        const size_t o = p * kPieceBytes, n = std::min(span, o + kPieceBytes) - o;
        hipError_t e = hipMemcpyAsync(text.as<char>() + o, at(p), n, hipMemcpyHostToDevice, d.copy);
        if (e == hipSuccess && R) e = hipEventRecord(d.ring_ev[p % R], d.copy);
        if (e != hipSuccess) {
            rc = xs::set_error(XS_ERR_HIP, hipGetErrorString(e));
            std::lock_guard<std::mutex> g(mu);
            failed = true;
        } else {
            std::lock_guard<std::mutex> g(mu);
            if (R) d.ring_used[p % R] = true;
            queued = p + 1;
        }
        cv.notify_all();
        if (rc) break;
    }
    th.join();
    if (rc) return rc;
    if (failed) return xs::set_error(XS_ERR_IO, "read failed while loading the window's text");
    FXCHK(hipMemsetAsync(text.as<char>() + span, 0, padded + 16 - span, d.copy));
    FXCHK(hipEventRecord(d.text_ev[ts], d.copy));
    d.load_ms[ts] = fx_ms() - t0;
    return XS_OK;
}

// The loader thread: loads queued windows in order until stopped.
void loader_main(xs_fastx* r) {
    DevSide& d = *r->dev;
    std::unique_lock<std::mutex> g(d.pf_mu);
    for (;;) {
        DevSide::PfJob* job = nullptr;
        d.pf_cv.wait(g, [&] {
            if (d.pf_stop) return true;
            for (auto& j : d.pf_q)
                if (!j.started) {
                    job = &j;  // deque references survive push_back and pop_front of others
                    return true;
                }
            return false;
        });
        if (d.pf_stop) return;
        job->started = true;
        const size_t lo = job->lo, hi = job->hi;
        const int slot = job->slot;
        g.unlock();
        const double t0 = fx_ms();
        const int rc = load_text(r, lo, hi, slot);
        std::string err = rc ? xs_last_error() : "";
        if (fx_trace()) fprintf(stderr, "[fastx-device] t=%.2f prefetch %zu+%zu done in %.2f ms\n", fx_ms(), lo, hi - lo,
                                fx_ms() - t0);
        g.lock();
        job->rc = rc;
        job->err = std::move(err);
        job->done = true;
        d.pf_cv.notify_all();
    }
}

// Queue [lo, hi) for the next text slot (in window order).
void queue_window(xs_fastx* r, size_t lo, size_t hi) {
    DevSide& d = *r->dev;
    {
        std::lock_guard<std::mutex> g(d.pf_mu);
        d.pf_q.push_back(DevSide::PfJob{lo, hi, d.next_text, false, false, XS_OK, std::string()});
        d.next_text ^= 1;
    }
    if (!d.loader.joinable()) d.loader = std::thread(loader_main, r);
    d.pf_cv.notify_all();
}

bool is_queued(DevSide& d, size_t lo) {
    std::lock_guard<std::mutex> g(d.pf_mu);
    for (const auto& j : d.pf_q)
        if (j.lo == lo) return true;
    return false;
}

// Wait for every queued load to finish and forget them.
void drain_loads(DevSide& d) {
    std::unique_lock<std::mutex> g(d.pf_mu);
    d.pf_cv.wait(g, [&] {
        for (const auto& j : d.pf_q)
            if (!j.done && (j.started || !d.pf_stop)) return false;
        return true;
    });
    d.pf_q.clear();
}

// Wait for the text of [lo, hi) to be queued for its slot (loading it now if
// it is not the oldest queued window); *ts = the slot, *prefetched = whether
// it came from the queue.
int text_for(xs_fastx* r, size_t lo, size_t hi, int* ts, bool* prefetched) {
    DevSide& d = *r->dev;
    *prefetched = false;
    {
        std::unique_lock<std::mutex> g(d.pf_mu);
        if (!d.pf_q.empty() && d.pf_q.front().lo == lo && d.pf_q.front().hi == hi) {
            d.pf_cv.wait(g, [&] { return d.pf_q.front().done; });
            DevSide::PfJob j = std::move(d.pf_q.front());
            d.pf_q.pop_front();
            *ts = j.slot;
            *prefetched = true;
            if (j.rc) return xs::set_error(j.rc, j.err.c_str());
            return XS_OK;
        }
    }
    // other windows than the queued ones (the caller changed its batch size):
    // let those loads finish, then load this one here
    drain_loads(d);
    {
        std::lock_guard<std::mutex> g(d.pf_mu);
        *ts = d.next_text;
        d.next_text ^= 1;
    }
    return load_text(r, lo, hi, *ts);
}

// Record finding on the device for the window [lo, hi) whose text is queued
// for d.text.  *ok = false: the window needs the host parser (nothing of the
// batch is kept).  On success the batch is in slot `slot` and `out` is filled.
int parse_on_device(xs_fastx* r, size_t lo, size_t hi, int slot, int ts, bool* ok, xs_fastx_dbatch* out) {
    DevSide& d = *r->dev;
    *ok = false;
    const size_t span = hi - lo;
    if (span == 0 || span >= (1ull << 31) - xs::kFxTile) {  // u32 positions, int scan sizes: host parser
        // the slot's text DMA must be done before the slot is queued for a later window
        // (whose larger buffer could otherwise take this one's back while it is written)
        FXCHK(hipEventSynchronize(d.text_ev[ts]));
        return XS_OK;
    }
    const hipStream_t s = d.stream;
    FXCHK(hipStreamWaitEvent(s, d.text_ev[ts], 0));
    const uint64_t tiles = (span + xs::kFxTile - 1) / xs::kFxTile;
    if (int rc = d.tiles.ensure((tiles + 1) * 8)) return rc;
    if (int rc = d.tile_ofs.ensure((tiles + 1) * 8)) return rc;
    if (int rc = d.status.ensure(64)) return rc;
    if (int rc = d.flag.ensure(8)) return rc;
    size_t tb = xs::fx_temp_bytes(tiles + 1);
    if (int rc = d.temp.ensure(tb)) return rc;
    auto* st = reinterpret_cast<uint64_t*>(d.status.p);
    FXCHK(xs::launch_fx_count(d.text[ts].as<uint8_t>(), tiles, d.tiles.as<uint64_t>(), s));
    FXCHK(hipMemsetAsync(d.tiles.as<uint64_t>() + tiles, 0, 8, s));
    FXCHK(xs::launch_scan(d.temp.p, tb, d.tiles.as<uint64_t>(), d.tile_ofs.as<uint64_t>(), tiles + 1, s));
    const double t0 = fx_ms();
    FXCHK(hipMemcpyAsync(st, d.tile_ofs.as<uint64_t>() + tiles, 8, hipMemcpyDeviceToHost, s));
    FXCHK(hipStreamSynchronize(s));
    const double t1 = fx_ms();
    g_fx.count = t1 - t0;
    const uint64_t newlines = st[0];
    const bool tail = r->base[hi - 1] != '\n';  // a last line without '\n' ends at hi
    const uint64_t L = newlines + (tail ? 1 : 0);
    const bool fasta = r->format == XS_FASTX_FASTA;
    if (!fasta && (L == 0 || L % 4)) return XS_OK;
    const uint64_t nmax = fasta ? L : L / 4;  // records, or an upper bound of them
    if (int rc = d.nl.ensure(L * 4 + 4)) return rc;
    tb = xs::fx_temp_bytes((fasta ? L : nmax) + 1);
    if (int rc = d.temp.ensure(tb)) return rc;
    FXCHK(xs::launch_fx_positions(d.text[ts].as<uint8_t>(), tiles, d.tile_ofs.as<uint64_t>(), d.nl.as<uint32_t>(),
                                  s));
    if (tail) FXCHK(hipMemsetD32Async(d.nl.as<uint32_t>() + newlines, (int)span, 1, s));
    FXCHK(hipMemsetAsync(d.flag.p, 0, 4, s));
    for (DBuf* b : {&d.seq_src, &d.id_src, &d.desc_src})
        if (int rc = b->ensure((nmax + 1) * 4)) return rc;
    for (DBuf* b : {&d.seq_len, &d.id_len, &d.desc_len, &d.id_ofs, &d.desc_ofs})
        if (int rc = b->ensure((nmax + 1) * 8)) return rc;
    if (int rc = d.offs[slot].ensure((nmax + 1) * 8)) return rc;
    if (int rc = d.maxlen.ensure(8)) return rc;
    const xs::FxRuns runs{d.seq_src.as<uint32_t>(), d.seq_len.as<uint64_t>(), d.id_src.as<uint32_t>(),
                          d.id_len.as<uint64_t>(), d.desc_src.as<uint32_t>(), d.desc_len.as<uint64_t>()};
    uint64_t* offs = d.offs[slot].as<uint64_t>();
    const uint8_t* text = d.text[ts].as<uint8_t>();
    const uint32_t* nl = d.nl.as<uint32_t>();
    // status: [0] bad, [1] records, [2] sequence bytes, [3] id bytes, [4] title bytes, [5] longest record
    if (fasta) {
        for (DBuf* b : {&d.hdr, &d.hofs, &d.line_len, &d.line_ofs, &d.lens})
            if (int rc = b->ensure((L + 1) * 8)) return rc;
        for (DBuf* b : {&d.line_src, &d.rec_line})
            if (int rc = b->ensure((L + 1) * 4)) return rc;
        // records past the last header keep zero-length ids and titles
        FXCHK(hipMemsetAsync(d.id_len.p, 0, (L + 1) * 8, s));
        FXCHK(hipMemsetAsync(d.desc_len.p, 0, (L + 1) * 8, s));
        FXCHK(hipMemsetAsync(d.lens.p, 0, (L + 1) * 8, s));
        FXCHK(xs::launch_fa_headers(text, nl, L, d.hdr.as<uint64_t>(), s));
        FXCHK(hipMemsetAsync(d.hdr.as<uint64_t>() + L, 0, 8, s));
        FXCHK(xs::launch_scan(d.temp.p, tb, d.hdr.as<uint64_t>(), d.hofs.as<uint64_t>(), L + 1, s));
        FXCHK(xs::launch_fa_lines(text, nl, L, d.hofs.as<uint64_t>(), d.line_src.as<uint32_t>(),
                                  d.line_len.as<uint64_t>(), d.rec_line.as<uint32_t>(), runs, d.flag.as<uint32_t>(), s));
        FXCHK(hipMemsetAsync(d.line_len.as<uint64_t>() + L, 0, 8, s));
        FXCHK(xs::launch_scan(d.temp.p, tb, d.line_len.as<uint64_t>(), d.line_ofs.as<uint64_t>(), L + 1, s));
        FXCHK(xs::launch_fa_offsets(d.rec_line.as<uint32_t>(), d.line_ofs.as<uint64_t>(), L,
                                    d.hofs.as<uint64_t>() + L, offs, d.lens.as<uint64_t>(), s));
        FXCHK(xs::launch_scan(d.temp.p, tb, d.id_len.as<uint64_t>(), d.id_ofs.as<uint64_t>(), L + 1, s));
        FXCHK(xs::launch_scan(d.temp.p, tb, d.desc_len.as<uint64_t>(), d.desc_ofs.as<uint64_t>(), L + 1, s));
        FXCHK(xs::launch_max_u64(d.temp.p, tb, d.lens.as<uint64_t>(), L, d.maxlen.as<uint64_t>(), s));
        FXCHK(hipMemcpyAsync(st + 1, d.hofs.as<uint64_t>() + L, 8, hipMemcpyDeviceToHost, s));
        FXCHK(hipMemcpyAsync(st + 2, d.line_ofs.as<uint64_t>() + L, 8, hipMemcpyDeviceToHost, s));
        FXCHK(hipMemcpyAsync(st + 3, d.id_ofs.as<uint64_t>() + L, 8, hipMemcpyDeviceToHost, s));
        FXCHK(hipMemcpyAsync(st + 4, d.desc_ofs.as<uint64_t>() + L, 8, hipMemcpyDeviceToHost, s));
    } else {
        // records, their offsets and the window's status in three kernels and one copy back
        const uint64_t n = nmax, nblk = (n + 255) / 256;
        if (int rc = d.fq_blk.ensure((nblk + 1) * sizeof(xs::FqBlockSums))) return rc;
        if (int rc = d.fq_blk_ofs.ensure((nblk + 1) * 3 * 8)) return rc;
        if (int rc = d.fq_status.ensure(6 * 8)) return rc;
        FXCHK(xs::launch_fq_records(text, nl, n, runs, d.flag.as<uint32_t>(),
                                    static_cast<xs::FqBlockSums*>(d.fq_blk.p), d.fq_blk_ofs.as<uint64_t>(), offs,
                                    d.id_ofs.as<uint64_t>(), d.desc_ofs.as<uint64_t>(), d.fq_status.as<uint64_t>(), s));
        FXCHK(hipMemcpyAsync(st, d.fq_status.p, 6 * 8, hipMemcpyDeviceToHost, s));
    }
    if (fasta) {
        st[0] = 0;
        FXCHK(hipMemcpyAsync(st, d.flag.p, 4, hipMemcpyDeviceToHost, s));
        FXCHK(hipMemcpyAsync(st + 5, d.maxlen.p, 8, hipMemcpyDeviceToHost, s));
    }
    FXCHK(hipStreamSynchronize(s));
    const double t2 = fx_ms();
    g_fx.records = t2 - t1;
    if ((uint32_t)st[0]) return XS_OK;
    const uint64_t n = st[1], sbytes = st[2], ibytes = st[3], dbytes = st[4];
    if (int rc = d.seqs[slot].ensure(sbytes + kDevPad)) return rc;
    if (int rc = d.ids_d.ensure(ibytes + 1)) return rc;
    if (int rc = d.descs_d.ensure(dbytes + 1)) return rc;
    if (int rc = d.ids[slot].ensure(ibytes + 1)) return rc;
    if (int rc = d.descs[slot].ensure(dbytes + 1)) return rc;
    if (int rc = d.id_offs[slot].ensure((n + 1) * 8)) return rc;
    if (int rc = d.desc_offs[slot].ensure((n + 1) * 8)) return rc;
    if (int rc = d.hoffs[slot].ensure((n + 1) * 8)) return rc;
    const double t2a = fx_ms();
    uint8_t* seqs = d.seqs[slot].as<uint8_t>();
    if (fasta)
        FXCHK(xs::launch_fx_copy(text, d.line_src.as<uint32_t>(), d.line_ofs.as<uint64_t>(), L, sbytes, seqs, s));
    else FXCHK(xs::launch_fx_copy(text, d.seq_src.as<uint32_t>(), offs, n, sbytes, seqs, s));
    FXCHK(hipMemsetAsync(seqs + sbytes, 0, kDevPad, s));
    FXCHK(xs::launch_fx_copy(text, d.id_src.as<uint32_t>(), d.id_ofs.as<uint64_t>(), n, ibytes, d.ids_d.as<uint8_t>(),
                             s));
    FXCHK(xs::launch_fx_copy(text, d.desc_src.as<uint32_t>(), d.desc_ofs.as<uint64_t>(), n, dbytes,
                             d.descs_d.as<uint8_t>(), s));
    FXCHK(hipEventRecord(d.kern_ev, s));  // the batch's device data: what the caller probes
    const double t2b = fx_ms();
    // the host arrays land behind the caller's probe; xs_fastx_wait_host waits for them
    if (ibytes) FXCHK(hipMemcpyAsync(d.ids[slot].p, d.ids_d.p, ibytes, hipMemcpyDeviceToHost, s));
    if (dbytes) FXCHK(hipMemcpyAsync(d.descs[slot].p, d.descs_d.p, dbytes, hipMemcpyDeviceToHost, s));
    FXCHK(hipMemcpyAsync(d.id_offs[slot].p, d.id_ofs.p, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    FXCHK(hipMemcpyAsync(d.desc_offs[slot].p, d.desc_ofs.p, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    FXCHK(hipMemcpyAsync(d.hoffs[slot].p, offs, (n + 1) * 8, hipMemcpyDeviceToHost, s));
    FXCHK(hipEventRecord(d.host_ev[slot], s));
    const double t2c = fx_ms();
    FXCHK(hipEventSynchronize(d.kern_ev));
    g_fx.copy = fx_ms() - t2;
    if (fx_trace())
        fprintf(stderr, "[fastx-device] copy phase: buffers %.2f launches %.2f D2H queue %.2f wait %.2f ms\n", t2a - t2,
                t2b - t2a, t2c - t2b, fx_ms() - t2c);
    out->host_ready = d.host_ev[slot];
    *ok = true;
    out->n = n;
    out->seq_bytes = sbytes;
    out->seqs = seqs;
    out->offsets = offs;
    out->host_offsets = reinterpret_cast<const uint64_t*>(d.hoffs[slot].p);
    out->max_len = st[5];
    out->ids = d.ids[slot].p;
    out->id_offsets = reinterpret_cast<const uint64_t*>(d.id_offs[slot].p);
    out->descs = d.descs[slot].p;
    out->desc_offsets = reinterpret_cast<const uint64_t*>(d.desc_offs[slot].p);
    out->parsed_on_device = 1;
    return XS_OK;
}

// A host batch into device slot `slot` (the host parser's result for a window
// the device rules do not cover, or a wrapped FASTQ file's batch).
int upload_host_batch(xs_fastx* r, const xs_fastx_batch& hb, int slot, xs_fastx_dbatch* out) {
    DevSide& d = *r->dev;
    if (int rc = d.seqs[slot].ensure(hb.seq_bytes + kDevPad)) return rc;
    if (int rc = d.offs[slot].ensure((hb.n + 1) * 8)) return rc;
    uint8_t* seqs = d.seqs[slot].as<uint8_t>();
    if (hb.seq_bytes) FXCHK(hipMemcpyAsync(seqs, hb.seqs, hb.seq_bytes, hipMemcpyHostToDevice, d.stream));
    FXCHK(hipMemsetAsync(seqs + hb.seq_bytes, 0, kDevPad, d.stream));
    FXCHK(hipMemcpyAsync(d.offs[slot].p, hb.offsets, (hb.n + 1) * 8, hipMemcpyHostToDevice, d.stream));
    FXCHK(hipStreamSynchronize(d.stream));
    uint64_t mx = 0;
    for (uint64_t i = 0; i < hb.n; ++i) mx = std::max(mx, hb.offsets[i + 1] - hb.offsets[i]);
    out->n = hb.n;
    out->seq_bytes = hb.seq_bytes;
    out->seqs = seqs;
    out->offsets = d.offs[slot].as<uint64_t>();
    out->host_offsets = hb.offsets;
    out->max_len = mx;
    out->ids = hb.ids;
    out->id_offsets = hb.id_offsets;
    out->descs = hb.descs;
    out->desc_offsets = hb.desc_offsets;
    out->parsed_on_device = 0;
    return XS_OK;
}

}  // namespace

extern "C" {

int xs_fastx_open(const char* path, int format, int threads, int flags, xs_fastx** out) {
    return xs::guard([&]() -> int {
        return xs_fastx_open_range(path, format, threads, flags, 0, 1, out);
    });
}

int xs_fastx_open_range(const char* path, int format, int threads, int flags, uint32_t part, uint32_t parts,
                        xs_fastx** out) {
    return xs::guard([&]() -> int {
        if (!path || !out) return xs::set_error(XS_ERR_ARG, "null argument");
        if (parts == 0 || part >= parts) return xs::set_error(XS_ERR_ARG, "part must be < parts");
        if (format != XS_FASTX_FASTA && format != XS_FASTX_FASTQ)
            return xs::set_error(XS_ERR_ARG, "format must be XS_FASTX_FASTA or XS_FASTX_FASTQ");
        *out = nullptr;
        auto* r = new xs_fastx();
        r->format = format;
        r->fd = open(path, O_RDONLY);
        if (r->fd < 0) {
            delete r;
            return xs::set_error(XS_ERR_IO, (std::string("cannot open ") + path).c_str());
        }
        struct stat st;
        if (fstat(r->fd, &st) != 0) {
            delete r;
            return xs::set_error(XS_ERR_IO, (std::string("cannot stat ") + path).c_str());
        }
        r->size = (size_t)st.st_size;
        if (r->size) {
            void* m = mmap(nullptr, r->size, PROT_READ, MAP_PRIVATE, r->fd, 0);
            if (m == MAP_FAILED) {
                delete r;
                return xs::set_error(XS_ERR_IO, (std::string("cannot map ") + path).c_str());
            }
            r->base = static_cast<const char*>(m);
            (void)madvise(m, r->size, MADV_SEQUENTIAL);
        }
        int t = threads > 0 ? threads : (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
        r->threads = std::min(t, 64);
        if (format == XS_FASTX_FASTQ && r->size) r->wrapped = fastq_wrapped(r->base, r->base + r->size);
        // Part p of P: the records whose first byte lies in [cut(p), cut(p+1)), cut(i)
        // = the first record start at or after size*i/P (cut(0) = 0, cut(P) = size).
        // Every record belongs to exactly one part, in file order.
        r->stop = r->size;
        if (parts > 1 && r->size) {
            const char* lo = r->base;
            const char* end = r->base + r->size;
            auto cut = [&](uint64_t i) -> size_t {
                if (i == 0) return 0;
                if (i >= parts) return r->size;
                const char* pos = lo + (size_t)((unsigned __int128)r->size * i / parts);
                const char* c = format == XS_FASTX_FASTA ? fasta_boundary(lo, pos, end)
                                : r->wrapped             ? fastq_boundary_sequential(lo, pos, end)
                                                         : fastq_boundary(lo, pos, end);
                return (size_t)(c - lo);
            };
            r->cur = cut(part);
            r->stop = std::max(r->cur, cut((uint64_t)part + 1));
        }
        for (auto& b : r->batch) {
            const bool pinned = (flags & XS_FASTX_PINNED) != 0;
            b.seqs.pinned = b.offs.pinned = pinned;
        }
        r->parts.resize((size_t)r->threads);
        *out = r;
        return XS_OK;
    });
}

int xs_fastx_next(xs_fastx* r, uint64_t max_text_bytes, xs_fastx_batch* out) {
    return xs::guard([&]() -> int {
        if (!r || !out) return xs::set_error(XS_ERR_ARG, "null argument");
        memset(out, 0, sizeof(*out));
        Batch& bt = r->batch[r->flip];
        r->flip ^= 1;
        bt.n = bt.seq_bytes = 0;
        const char* end = r->base + r->stop;
        int nparts = 0;
        // a window can hold no record (text before the first one): go on until
        // records are found or the file ends
        for (;;) {
            const char* lo = r->base + r->cur;
            const size_t budget = window_budget(max_text_bytes, r->windows);
            nparts = 0;
            if (lo < end) {
                ++r->windows;
                if (r->format == XS_FASTX_FASTQ && r->wrapped) {
                    // sequential: the parser itself stops at the first record past the budget
                    Part& pt = r->parts[0];
                    pt.clear();
                    parse_fastq(lo, end, budget, pt);
                    nparts = 1;
                    if (!pt.err.empty()) return xs::set_error(XS_ERR_FORMAT, pt.err.c_str());
                } else if (int rc = parse_window(r, lo, window_end(r, lo, end, budget), &nparts)) {
                    return rc;
                }
            }
            if (nparts) r->cur = (size_t)(r->parts[nparts - 1].stop - r->base);
            size_t got = 0;
            for (int i = 0; i < nparts; ++i) got += r->parts[i].lens.size();
            if (got || r->cur >= r->stop || !nparts) break;
        }
        if (int rc = pack_parts(r, bt, nparts)) return rc;
        r->records += bt.n;
        fill_host_batch(r, bt, out);
        return XS_OK;
    });
}

int xs_fastx_open_device(const char* path, int format, int threads, int device, uint32_t part, uint32_t parts,
                         xs_fastx** out) {
    return xs::guard([&]() -> int {
        if (int rc = xs_fastx_open_range(path, format, threads, 0, part, parts, out)) return rc;
        xs_fastx* r = *out;
        auto fail = [&](hipError_t e) {
            xs_fastx_close(r);
            *out = nullptr;
            return xs::set_error(XS_ERR_HIP, hipGetErrorString(e));
        };
        hipError_t e = hipSetDevice(device);
        if (e != hipSuccess) return fail(e);
        if ((r->dev = take_devside(device))) return XS_OK;
        r->dev = new DevSide();
        r->dev->set_device(device);
        if (take_streams(*r->dev)) return XS_OK;
        // The parse kernels are short and sit between the caller's probes of the
        // previous batch: a high-priority stream lets their workgroups in as soon
        // as the probe frees a slot, instead of after the whole probe.  The text
        // DMA has a stream of its own, so the next window's copy never queues
        // behind this window's parse.
        int least = 0, greatest = 0;
        if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        (void)least;
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&r->dev->stream, hipStreamNonBlocking, greatest);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&r->dev->copy, hipStreamNonBlocking);
        for (hipEvent_t* ev : {&r->dev->text_ev[0], &r->dev->text_ev[1], &r->dev->kern_ev, &r->dev->host_ev[0],
                               &r->dev->host_ev[1]})
            if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
        if (e != hipSuccess) return fail(e);
        return XS_OK;
    });
}

int xs_fastx_wait_host(const xs_fastx_dbatch* b) {
    return xs::guard([&]() -> int {
        if (!b) return xs::set_error(XS_ERR_ARG, "null argument");
        if (b->host_ready) FXCHK(hipEventSynchronize(static_cast<hipEvent_t>(b->host_ready)));
        return XS_OK;
    });
}

int xs_fastx_next_device(xs_fastx* r, uint64_t max_text_bytes, xs_fastx_dbatch* out) {
    return xs::guard([&]() -> int {
        if (!r || !out) return xs::set_error(XS_ERR_ARG, "null argument");
        if (!r->dev) return xs::set_error(XS_ERR_ARG, "reader was not opened with xs_fastx_open_device");
        memset(out, 0, sizeof(*out));
        DevSide& d = *r->dev;
        FXCHK(hipSetDevice(d.device));
        if (fx_trace()) fprintf(stderr, "[fastx-device] t=%.2f next_device\n", fx_ms());
        const int slot = d.flip;
        d.flip ^= 1;
        if (r->format == XS_FASTX_FASTQ && r->wrapped) {  // records cannot be cut by pattern: host parser
            xs_fastx_batch hb;
            if (int rc = xs_fastx_next(r, max_text_bytes, &hb)) return rc;
            if (int rc = upload_host_batch(r, hb, slot, out)) return rc;
            out->text_offset = hb.text_offset;
            out->text_bytes = hb.text_bytes;
            return XS_OK;
        }
        const char* end = r->base + r->stop;
        for (;;) {
            if (r->cur >= r->stop) {
                drain_loads(d);
                out->text_offset = r->cur;
                out->text_bytes = r->stop;
                return XS_OK;
            }
            const char* lo = r->base + r->cur;
            const char* hi = window_end(r, lo, end, window_budget(max_text_bytes, r->windows));
            const size_t flo = (size_t)(lo - r->base), fhi = (size_t)(hi - r->base);
            const double t0 = fx_ms();
            bool prefetched = false;
            int ts = 0;
            if (int rc = text_for(r, flo, fhi, &ts, &prefetched)) return rc;
            const double t1 = fx_ms();
            r->cur = fhi;
            ++r->windows;
            // The next window's text loads into the other slot while this one is
            // parsed and the caller works on the batch; the one after it goes
            // into this window's slot once this parse is done.
            size_t n1_hi = 0;  // end of the next window
            if (r->cur < r->stop)
                n1_hi = (size_t)(window_end(r, r->base + r->cur, end, window_budget(max_text_bytes, r->windows)) - r->base);
            auto queue_next = [&] {
                if (n1_hi && !is_queued(d, r->cur)) queue_window(r, r->cur, n1_hi);
            };
            queue_next();
            bool ok = false;
            g_fx = FxTimes{};
            if (int rc = parse_on_device(r, flo, fhi, slot, ts, &ok, out)) return rc;
            if (n1_hi && n1_hi < r->stop && !is_queued(d, n1_hi))  // this slot's text is free now
                queue_window(r, n1_hi,
                             (size_t)(window_end(r, r->base + n1_hi, end, window_budget(max_text_bytes, r->windows + 1)) -
                                      r->base));
            if (fx_trace())
                fprintf(stderr,
                        "[fastx-device] t=%.2f window %zu+%zu: text %s load %.2f ms, wait %.2f ms | count %.2f records %.2f "
                        "copy %.2f ms | %s\n",
                        t0, flo, fhi - flo, prefetched ? "prefetched" : "inline", d.load_ms[ts], t1 - t0, g_fx.count,
                        g_fx.records, g_fx.copy, ok ? "device" : "host parser");
            if (!ok) {  // the host parser's batch for exactly this window
                int nparts = 0;
                if (int rc = parse_window(r, lo, hi, &nparts)) return rc;
                Batch& bt = r->batch[r->flip];
                r->flip ^= 1;
                if (int rc = pack_parts(r, bt, nparts)) return rc;
                xs_fastx_batch hb;
                memset(&hb, 0, sizeof(hb));
                fill_host_batch(r, bt, &hb);
                if (int rc = upload_host_batch(r, hb, slot, out)) return rc;
            }
            if (out->n) {
                r->records += out->n;
                out->text_offset = r->cur;
                out->text_bytes = r->stop;
                if (fx_trace()) fprintf(stderr, "[fastx-device] t=%.2f return n=%llu\n", fx_ms(), (unsigned long long)out->n);
                return XS_OK;
            }
            memset(out, 0, sizeof(*out));  // no record in this window (text before the first one)
        }
    });
}

void xs_fastx_close(xs_fastx* r) { delete r; }

int xs_write_fasta(const char* path, int append, const char* seqs, const uint64_t* offsets, const char* descs,
                   const uint64_t* desc_offsets, const uint32_t* index, uint64_t n, uint32_t width) {
    return xs::guard([&]() -> int {
        if (!path || (n && (!seqs || !offsets || !desc_offsets))) return xs::set_error(XS_ERR_ARG, "null argument");
        if (width == 0) return xs::set_error(XS_ERR_ARG, "width must be >= 1");
        FILE* f = fopen(path, append ? "ab" : "wb");
        if (!f) return xs::set_error(XS_ERR_IO, (std::string("cannot open ") + path).c_str());
        const int T = (int)std::min<uint64_t>(16, std::max<uint64_t>(1, n / 4096));
        const uint64_t block = 1 << 15;
        std::vector<std::string> out((size_t)T);
        bool ok = true;
        for (uint64_t b0 = 0; b0 < n && ok; b0 += block) {
            const uint64_t b1 = std::min(n, b0 + block), per = (b1 - b0 + T - 1) / T;
            auto work = [&](int t) {
                std::string& o = out[t];
                o.clear();
                const uint64_t lo = b0 + per * t, hi = std::min(b1, lo + per);
                for (uint64_t i = lo; i < hi; ++i) {
                    const uint64_t r = index ? index[i] : i;
                    o += '>';
                    o.append(descs + desc_offsets[r], (size_t)(desc_offsets[r + 1] - desc_offsets[r]));
                    o += '\n';
                    const char* s = seqs + offsets[r];
                    const uint64_t len = offsets[r + 1] - offsets[r];
                    for (uint64_t p = 0; p < len; p += width) {
                        o.append(s + p, (size_t)std::min<uint64_t>(width, len - p));
                        o += '\n';
                    }
                }
            };
            xs::parallel_for(T, work);
            for (int t = 0; t < T && ok; ++t) ok = fwrite(out[t].data(), 1, out[t].size(), f) == out[t].size();
        }
        if (fclose(f) != 0) ok = false;
        if (!ok) return xs::set_error(XS_ERR_IO, (std::string("write failed: ") + path).c_str());
        return XS_OK;
    });
}

}  // extern "C"
