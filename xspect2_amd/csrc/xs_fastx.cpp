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
#include "../../include/xspect_hip.h"

#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
            if (hipHostMalloc(reinterpret_cast<void**>(&p), want, hipHostMallocDefault) != hipSuccess) {
                p = nullptr;
                return xs::set_error(XS_ERR_HIP, "hipHostMalloc failed for the reader's batch buffer");
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
            if (pinned) (void)hipHostFree(p);
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
    Batch batch[2];
    int flip = 0;
    std::vector<Part> parts;
    ~xs_fastx() {
        if (base && size) munmap(const_cast<char*>(base), size);
        if (fd >= 0) close(fd);
    }
};

extern "C" {

int xs_fastx_open(const char* path, int format, int threads, int flags, xs_fastx** out) {
    return xs_fastx_open_range(path, format, threads, flags, 0, 1, out);
}

int xs_fastx_open_range(const char* path, int format, int threads, int flags, uint32_t part, uint32_t parts,
                        xs_fastx** out) {
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
}

int xs_fastx_next(xs_fastx* r, uint64_t max_text_bytes, xs_fastx_batch* out) {
    if (!r || !out) return xs::set_error(XS_ERR_ARG, "null argument");
    memset(out, 0, sizeof(*out));
    Batch& bt = r->batch[r->flip];
    r->flip ^= 1;
    bt.n = bt.seq_bytes = 0;
    const char* end = r->base + r->stop;
    const size_t budget = std::max<uint64_t>(max_text_bytes, 1);
    int nparts = 0;
    // a window can hold no record (text before the first one): go on until
    // records are found or the file ends
    for (;;) {
    const char* lo = r->base + r->cur;
    nparts = 0;
    if (lo < end) {
        const bool fasta = r->format == XS_FASTX_FASTA;
        if (!fasta && r->wrapped) {
            // sequential: the parser itself stops at the first record past the budget
            Part& pt = r->parts[0];
            pt.clear();
            parse_fastq(lo, end, budget, pt);
            nparts = 1;
        } else {
            auto boundary = fasta ? fasta_boundary : fastq_boundary;
            const char* hi = (size_t)(end - lo) <= budget ? end : boundary(lo, lo + budget, end);
            if (hi == lo) hi = boundary(lo, lo + 1, end);  // one record larger than the budget
            const size_t span = (size_t)(hi - lo);
            int T = (int)std::min<size_t>((size_t)r->threads, std::max<size_t>(1, span >> 20));  // >= 1 MiB per part
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
            std::vector<std::thread> th;
            for (int i = 1; i < T; ++i) th.emplace_back(work, i);
            work(0);
            for (auto& x : th) x.join();
            r->parts[T - 1].stop = hi;
            nparts = T;
        }
        for (int i = 0; i < nparts; ++i)
            if (!r->parts[i].err.empty()) return xs::set_error(XS_ERR_FORMAT, r->parts[i].err.c_str());
    }
    if (nparts) r->cur = (size_t)(r->parts[nparts - 1].stop - r->base);
    size_t got = 0;
    for (int i = 0; i < nparts; ++i) got += r->parts[i].lens.size();
    if (got || r->cur >= r->stop || !nparts) break;
    }
    // pack the parts
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
    {
        std::vector<std::thread> th;
        for (int i = 1; i < nparts; ++i) th.emplace_back(pack, i);
        if (nparts) pack(0);
        for (auto& x : th) x.join();
    }
    offs[n] = sbytes;
    ioffs[n] = ibytes;
    doffs[n] = dbytes;
    memset(bt.seqs.p + sbytes, 0, 64);  // defined bytes past the end
    bt.n = n;
    bt.seq_bytes = sbytes;
    r->records += n;
    out->n = n;
    out->seqs = bt.seqs.p;
    out->seq_bytes = sbytes;
    out->offsets = offs;
    out->ids = bt.ids.p;
    out->id_offsets = ioffs;
    out->text_offset = r->cur;
    out->text_bytes = r->stop;
    out->descs = bt.descs.p;
    out->desc_offsets = doffs;
    return XS_OK;
}

void xs_fastx_close(xs_fastx* r) { delete r; }

int xs_write_fasta(const char* path, int append, const char* seqs, const uint64_t* offsets, const char* descs,
                   const uint64_t* desc_offsets, const uint32_t* index, uint64_t n, uint32_t width) {
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
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t) th.emplace_back(work, t);
        work(0);
        for (auto& x : th) x.join();
        for (int t = 0; t < T && ok; ++t) ok = fwrite(out[t].data(), 1, out[t].size(), f) == out[t].size();
    }
    if (fclose(f) != 0) ok = false;
    if (!ok) return xs::set_error(XS_ERR_IO, (std::string("write failed: ") + path).c_str());
    return XS_OK;
}

}  // extern "C"
