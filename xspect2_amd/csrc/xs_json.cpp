// xs_json.cpp — the per-read sections of a ModelResult JSON, written from a
// hit matrix.
//
// The reference serialises results with json.dumps(result.to_dict(), indent=4)
// (src/xspect/models/result.py:151-202): "hits" {read: {label: count}} with each
// read's labels in COBS result order (count descending; ties by doc index
// here), "scores" {read: {label: round(count/num_kmers, 2)},
// "total": {...}} and "num_kmers" {read: n}.  At 10^6 reads x 100 species that
// is ~10^8 entries, which per-read Python dicts cannot produce in reasonable
// time; here the three sections are formatted by several threads, block by
// block, straight from the matrix.  The caller writes the small leading and
// trailing fields (model_slug, sparse_sampling_step, misclassified,
// input_source, prediction) around them; the file is byte-identical to the
// reference's (tests/test_json_writer.py compares with json.dumps).
//
// Scores: Python's round(h / n, 2) rounds the exact binary value of the double
// h/n half-to-even at two decimals and repr() prints the shortest form, which
// is the two-decimal string without trailing zeros ("0.3", "1.0", "0.0").
// glibc's printf("%.2f") rounds the same exact value the same way.
#include "../../include/xspect_hip.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <functional>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "xs_internal.h"

namespace {

std::string score_text(uint64_t h, uint64_t n) {
    char buf[64];
    snprintf(buf, sizeof(buf), "%.2f", (double)h / (double)n);
    std::string s(buf);
    // "0.30" -> "0.3", "1.00" -> "1.0"
    if (s.size() >= 2 && s.back() == '0' && s[s.size() - 2] != '.') s.pop_back();
    return s;
}

struct ScoreCache {  // per thread: score strings of h = 0..n for the n of the last read
    std::unordered_map<uint64_t, std::vector<std::string>> by_n;
    uint64_t last_n = ~0ull;
    const std::vector<std::string>* last = nullptr;
    const std::string& get(uint64_t h, uint64_t n) {
        if (n != last_n) {  // reads of one batch mostly share n: one hash lookup per change
            auto& v = by_n[n];
            if (v.empty() && n <= (1u << 16)) {
                v.resize(n + 1);
                for (uint64_t i = 0; i <= n; ++i) v[i] = score_text(i, n);
            }
            last_n = n;
            last = &v;
        }
        if (h < last->size()) return (*last)[h];
        thread_local std::string tmp;
        tmp = score_text(h, n);
        return tmp;
    }
};

template <class T>
struct Ctx {
    uint64_t n, D;
    const T* hits;  // n x D counts (uint8, uint16 or uint32)
    const uint64_t* nk;
    const char* ids;
    const uint64_t* ids_off;
    const char* labels;
    const uint64_t* labels_off;
    std::vector<uint32_t> docs;       // emitted docs (doc_mask), ascending
    std::vector<std::string> entry;   // per doc: ",\n", the indented label key and ": "
    std::vector<std::string> count;   // decimal text of small counts
    size_t row_bound = 0;             // bytes one read's entries can take (ids aside)
};

// Docs of one hit row in COBS result order: count descending, ties by doc index
// (one sort of 64-bit keys (~count << 32 | doc): no allocation per row).
template <class T>
void order_of(const std::vector<uint32_t>& docs, const T* row, std::vector<uint32_t>& ord,
              std::vector<uint64_t>& keys) {
    keys.resize(docs.size());
    for (size_t j = 0; j < docs.size(); ++j) keys[j] = ((uint64_t)(~(uint32_t)row[docs[j]]) << 32) | docs[j];
    std::sort(keys.begin(), keys.end());
    ord.resize(docs.size());
    for (size_t j = 0; j < docs.size(); ++j) ord[j] = (uint32_t)keys[j];
}
template <class T>
void order_of(const std::vector<uint32_t>& docs, const T* row, std::vector<uint32_t>& ord) {
    std::vector<uint64_t> keys;
    order_of(docs, row, ord, keys);
}

// The same order by a counting sort over the counts 0..cap (a read's counts
// never exceed its k-mer count, the cap passed): bucket offsets from the top
// count down, docs placed in ascending order within a bucket.  cnt: cap + 2
// scratch entries.  False (nothing done) if some count exceeds cap.
template <class T>
bool order_counting(const std::vector<uint32_t>& docs, const T* row, uint32_t cap, std::vector<uint32_t>& ord,
                    std::vector<uint32_t>& cnt) {
    for (uint32_t d : docs)
        if ((uint32_t)row[d] > cap) return false;
    cnt.assign((size_t)cap + 2, 0);
    for (uint32_t d : docs) ++cnt[cap - (uint32_t)row[d] + 1];
    for (size_t i = 1; i < cnt.size(); ++i) cnt[i] += cnt[i - 1];
    ord.resize(docs.size());
    for (uint32_t d : docs) ord[cnt[cap - (uint32_t)row[d]]++] = d;
    return true;
}

inline void put_key(std::string& o, const char* base, const uint64_t* off, uint64_t i) {
    o.append(base + off[i], (size_t)(off[i + 1] - off[i]));
}

constexpr uint32_t kCountText = 1024;  // counts below this are formatted once

template <class T>
void prepare(Ctx<T>& c) {
    c.entry.resize(c.D);
    size_t bound = 64;
    for (uint64_t d = 0; d < c.D; ++d) {
        std::string& e = c.entry[d];
        e = ",\n            ";
        put_key(e, c.labels, c.labels_off, d);
        e += ": ";
        bound += e.size() + 32;  // + the count or score text
    }
    c.row_bound = bound;
    c.count.resize(kCountText);
    for (uint32_t v = 0; v < kCountText; ++v) c.count[v] = std::to_string(v);
}

// Appends to a byte buffer through a cursor: capacity is ensured once per
// read, then every piece is a memcpy.
struct Sink {
    std::string& s;
    size_t len;
    explicit Sink(std::string& out) : s(out), len(out.size()) {}
    void ensure(size_t more) {
        if (len + more > s.size()) s.resize(std::max(s.size() * 2, len + more));
    }
    void put(const char* p, size_t n) {
        memcpy(&s[len], p, n);
        len += n;
    }
    void put(const std::string& x) { put(x.data(), x.size()); }
    void finish() { s.resize(len); }
};

// section 0: hits, 1: scores, 2: num_kmers — entries of reads [lo, hi)
template <class T>
void format_block(const Ctx<T>& c, int section, uint64_t lo, uint64_t hi, std::string& o) {
    std::vector<uint32_t> ord, cnt;
    std::vector<uint64_t> keys;
    ScoreCache cache;
    char num[32];
    Sink k(o);
    for (uint64_t r = lo; r < hi; ++r) {
        const size_t idl = (size_t)(c.ids_off[r + 1] - c.ids_off[r]);
        k.ensure(idl + 64 + (section == 2 ? 0 : c.row_bound));
        if (r) k.put(",\n", 2);
        k.put("        ", 8);
        k.put(c.ids + c.ids_off[r], idl);
        if (section == 2) {
            int n = snprintf(num, sizeof(num), ": %llu", (unsigned long long)c.nk[r]);
            k.put(num, (size_t)n);
            continue;
        }
        if (c.docs.empty()) {
            k.put(": {}", 4);
            continue;
        }
        k.put(": {\n", 4);
        const T* row = c.hits + r * c.D;
        if (c.nk[r] >= 4096 || !order_counting(c.docs, row, (uint32_t)c.nk[r], ord, cnt))
            order_of(c.docs, row, ord, keys);
        for (size_t j = 0; j < ord.size(); ++j) {
            const std::string& e = c.entry[ord[j]];
            if (j) k.put(e);
            else k.put(e.data() + 2, e.size() - 2);  // the first entry has no ",\n"
            const uint32_t v = (uint32_t)row[ord[j]];
            if (section == 0) {
                if (v < kCountText) {
                    k.put(c.count[v]);
                } else {
                    int n = snprintf(num, sizeof(num), "%u", v);
                    k.put(num, (size_t)n);
                }
            } else {
                k.put(cache.get(v, c.nk[r]));
            }
        }
        k.put("\n        }", 10);
    }
    k.finish();
}

template <class T>
int write_sections(const char* path, const Ctx<T>& c, const uint64_t* total_hits, uint64_t total_kmers_in,
                   const uint32_t* total_order_row, int threads) {
    const uint64_t n = c.n, num_docs = c.D;
    FILE* f = fopen(path, "ab");
    if (!f) return xs::set_error(XS_ERR_IO, (std::string("cannot append to ") + path).c_str());
    const int NT = std::max(1, std::min(threads > 0 ? threads : 16, 64));
    const uint64_t block = 1 << 14;  // reads per formatting round
    // two sets of per-thread buffers: round i is formatted while round i-1 is written
    std::vector<std::string> out[2] = {std::vector<std::string>((size_t)NT), std::vector<std::string>((size_t)NT)};
    bool ok = true;
    const char* heads[3] = {"\"hits\": ", "\"scores\": ", "\"num_kmers\": "};
    for (int section = 0; section < 3 && ok; ++section) {
        // an empty section is "{}" as json.dumps writes it (a shard without reads)
        const bool empty = n == 0 && section != 1;
        ok = fputs(heads[section], f) >= 0 && fputs(empty ? "{}" : "{\n", f) >= 0;
        xs::ThreadGroup writer;  // the previous round's buffers go out while this round is formatted
        bool wok = true;
        int cur = 0;
        for (uint64_t b0 = 0; b0 < n && ok; b0 += block, cur ^= 1) {
            const uint64_t b1 = std::min(n, b0 + block);
            const uint64_t per = (b1 - b0 + NT - 1) / NT;
            xs::parallel_for(NT, [&, b0, b1, per, cur](int t) {
                out[cur][t].clear();
                const uint64_t lo = b0 + per * t, hi = std::min(b1, lo + per);
                if (lo < hi) format_block(c, section, lo, hi, out[cur][t]);
            });
            writer.join();
            ok = wok;
            if (!ok) break;
            writer.start([&, cur] {
                for (int t = 0; t < NT && wok; ++t)
                    wok = fwrite(out[cur][t].data(), 1, out[cur][t].size(), f) == out[cur][t].size();
            });
        }
        writer.join();
        ok = ok && wok;
        if (!ok) break;
        if (section == 1) {
            // "total": labels in the first read's order, round(sum hits / sum num_kmers, 2);
            // a shard of a read-sharded job passes the whole job's sums and first row
            std::vector<uint64_t> tot(num_docs, 0);
            uint64_t total_kmers = total_kmers_in;
            if (total_hits) {
                std::copy(total_hits, total_hits + num_docs, tot.begin());
            } else {
                for (uint64_t r = 0; r < n; ++r)
                    for (uint64_t d = 0; d < num_docs; ++d) tot[d] += c.hits[r * num_docs + d];
                total_kmers = std::accumulate(c.nk, c.nk + n, (uint64_t)0);
            }
            std::vector<uint32_t> ord;
            if (total_order_row) order_of(c.docs, total_order_row, ord);
            else order_of(c.docs, c.hits, ord);
            std::string o = n ? ",\n        \"total\": " : "        \"total\": ";
            if (ord.empty()) {
                o += "{}";
            } else {
                o += "{\n";
                for (size_t j = 0; j < ord.size(); ++j) {
                    if (j) o += ",\n";
                    o += "            ";
                    put_key(o, c.labels, c.labels_off, ord[j]);
                    o += ": " + score_text(tot[ord[j]], total_kmers);
                }
                o += "\n        }";
            }
            ok = fwrite(o.data(), 1, o.size(), f) == o.size();
        }
        if (ok)
            ok = fputs(empty ? (section < 2 ? ",\n    " : ",\n") : (section < 2 ? "\n    },\n    " : "\n    },\n"), f) >= 0;
    }
    if (fclose(f) != 0) ok = false;
    if (!ok) return xs::set_error(XS_ERR_IO, (std::string("write failed: ") + path).c_str());
    return XS_OK;
}

template <class T>
int write_typed(const char* path, uint64_t n, uint64_t num_docs, const void* hits, const uint64_t* num_kmers,
                const char* ids_json, const uint64_t* ids_off, const char* labels_json, const uint64_t* labels_off,
                const uint8_t* doc_mask, const uint64_t* total_hits, uint64_t total_kmers,
                const uint32_t* total_order_row, int threads) {
    Ctx<T> c{n, num_docs, static_cast<const T*>(hits), num_kmers, ids_json, ids_off, labels_json, labels_off,
             {}, {}, {}, 0};
    for (uint64_t d = 0; d < num_docs; ++d)
        if (!doc_mask || doc_mask[d]) c.docs.push_back((uint32_t)d);
    prepare(c);
    return write_sections(path, c, total_hits, total_kmers, total_order_row, threads);
}

}  // namespace

extern "C" {

int xs_write_result_sections(const char* path, uint64_t n, uint64_t num_docs, const void* hits, int hit_bytes,
                             const uint64_t* num_kmers, const char* ids_json, const uint64_t* ids_off,
                             const char* labels_json, const uint64_t* labels_off, const uint8_t* doc_mask,
                             const uint64_t* total_hits, uint64_t total_kmers, const uint32_t* total_order_row,
                             int threads) {
    return xs::guard([&]() -> int {
        if (!path || (n && (!hits || !num_kmers || !ids_json || !ids_off)) || !labels_json || !labels_off)
            return xs::set_error(XS_ERR_ARG, "null argument");
        if (hit_bytes != 1 && hit_bytes != 2 && hit_bytes != 4) return xs::set_error(XS_ERR_ARG, "hit_bytes must be 1, 2 or 4");
        if (total_hits) {
            if (!total_order_row) return xs::set_error(XS_ERR_ARG, "total_hits needs total_order_row");
            if (total_kmers == 0) return xs::set_error(XS_ERR_ARG, "total_kmers must be > 0 (scores divide by it)");
        } else if (n == 0) {
            return xs::set_error(XS_ERR_ARG, "a result needs at least one read");
        }
        for (uint64_t r = 0; r < n; ++r)
            if (num_kmers[r] == 0) return xs::set_error(XS_ERR_ARG, "a read has no k-mers (scores divide by zero)");
        auto w = hit_bytes == 1 ? write_typed<uint8_t> : hit_bytes == 2 ? write_typed<uint16_t> : write_typed<uint32_t>;
        return w(path, n, num_docs, hits, num_kmers, ids_json, ids_off, labels_json, labels_off, doc_mask, total_hits,
                 total_kmers, total_order_row, threads);
    });
}

}  // extern "C"

// ---- packed read ids ------------------------------------------------------------
// The reader hands ids over as one byte buffer + offsets; a result of 10^6..10^7
// reads keeps them that way (MatrixResult with PackedIds) instead of building
// Python strings.  Both helpers take ASCII ids only (the caller checks; other
// ids go through Python's own decoding and json.dumps).

// json.dumps(id) with ensure_ascii (Python's json encoder, py_encode_basestring_ascii):
// '"' and '\\' escaped, \n \r \t \b \f short forms, other bytes outside ' '..'~'
// (< 0x20, 0x7f) as \u00xx (lower-case hex); everything else as is.
int xs_ids_json_quote(const char* buf, const uint64_t* offs, uint64_t n, char* out, uint64_t out_cap,
                      uint64_t* out_offs) {
    return xs::guard([&]() -> int {
        if (!offs || !out_offs || (!out && n) || (!buf && n && offs[n])) return xs::set_error(XS_ERR_ARG, "null argument");
        static const char hex[] = "0123456789abcdef";
        uint64_t o = 0;
        out_offs[0] = 0;
        for (uint64_t i = 0; i < n; ++i) {
            if (offs[i + 1] < offs[i]) return xs::set_error(XS_ERR_ARG, "id offsets must be non-decreasing");
            const uint64_t len = offs[i + 1] - offs[i];
            if (o + 2 + 6 * len > out_cap) return xs::set_error(XS_ERR_ARG, "output buffer too small");
            out[o++] = '"';
            const unsigned char* s = reinterpret_cast<const unsigned char*>(buf + offs[i]);
            for (uint64_t j = 0; j < len; ++j) {
                const unsigned char c = s[j];
                if (c >= 0x80) return xs::set_error(XS_ERR_ARG, "non-ASCII id");
                if (c == '"' || c == '\\') {
                    out[o++] = '\\';
                    out[o++] = (char)c;
                } else if (c >= 0x20 && c < 0x7f) {
                    out[o++] = (char)c;
                } else if (c == '\n' || c == '\r' || c == '\t' || c == '\b' || c == '\f') {
                    out[o++] = '\\';
                    out[o++] = c == '\n' ? 'n' : c == '\r' ? 'r' : c == '\t' ? 't' : c == '\b' ? 'b' : 'f';
                } else {
                    out[o++] = '\\';
                    out[o++] = 'u';
                    out[o++] = '0';
                    out[o++] = '0';
                    out[o++] = hex[c >> 4];
                    out[o++] = hex[c & 15];
                }
            }
            out[o++] = '"';
            out_offs[i + 1] = o;
        }
        return XS_OK;
    });
}

// XXH64 (the published xxHash 64-bit algorithm), host side, for id keys.
namespace {
constexpr uint64_t kP1 = 0x9E3779B185EBCA87ull, kP2 = 0xC2B2AE3D27D4EB4Full, kP3 = 0x165667B19E3779F9ull,
                   kP4 = 0x85EBCA77C2B2AE63ull, kP5 = 0x27D4EB2F165667C5ull;
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const unsigned char* p) { uint64_t v; memcpy(&v, p, 8); return v; }
inline uint32_t rd32(const unsigned char* p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint64_t xround(uint64_t acc, uint64_t in) { return rotl64(acc + in * kP2, 31) * kP1; }
inline uint64_t xmerge(uint64_t acc, uint64_t v) { return (acc ^ xround(0, v)) * kP1 + kP4; }

uint64_t xxh64(const unsigned char* p, uint64_t len, uint64_t seed) {
    const unsigned char* const end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + kP1 + kP2, v2 = seed + kP2, v3 = seed, v4 = seed - kP1;
        for (; p + 32 <= end; p += 32) {
            v1 = xround(v1, rd64(p));
            v2 = xround(v2, rd64(p + 8));
            v3 = xround(v3, rd64(p + 16));
            v4 = xround(v4, rd64(p + 24));
        }
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xmerge(xmerge(xmerge(xmerge(h, v1), v2), v3), v4);
    } else {
        h = seed + kP5;
    }
    h += len;
    for (; p + 8 <= end; p += 8) h = rotl64(h ^ xround(0, rd64(p)), 27) * kP1 + kP4;
    if (p + 4 <= end) {
        h = rotl64(h ^ (uint64_t)rd32(p) * kP1, 23) * kP2 + kP3;
        p += 4;
    }
    for (; p < end; ++p) h = rotl64(h ^ (uint64_t)(*p) * kP5, 11) * kP1;
    h ^= h >> 33;
    h *= kP2;
    h ^= h >> 29;
    h *= kP3;
    return h ^ (h >> 32);
}
}  // namespace

// out[2i], out[2i+1] = XXH64(id i, seed 0), XXH64(id i, seed kP5): a 128-bit
// key per id, for finding ids repeated across the shards of a read-sharded
// job without moving the ids themselves.
int xs_ids_hash128(const char* buf, const uint64_t* offs, uint64_t n, uint64_t* out) {
    return xs::guard([&]() -> int {
        if (!offs || (!out && n) || (!buf && n && offs[n])) return xs::set_error(XS_ERR_ARG, "null argument");
        for (uint64_t i = 0; i < n; ++i)
            if (offs[i + 1] < offs[i]) return xs::set_error(XS_ERR_ARG, "id offsets must be non-decreasing");
        // a read-sharded job hashes every id of its shard (12.5 M at config 3): spread over threads
        auto run = [=](uint64_t a, uint64_t e) {
            for (uint64_t i = a; i < e; ++i) {
                const unsigned char* s = reinterpret_cast<const unsigned char*>(buf + offs[i]);
                const uint64_t len = offs[i + 1] - offs[i];
                out[2 * i] = xxh64(s, len, 0);
                out[2 * i + 1] = xxh64(s, len, kP5);
            }
        };
        const uint64_t T = std::min<uint64_t>(16, std::max<uint64_t>(1, n / (1u << 16)));
        const uint64_t per = (n + T - 1) / T;
        xs::parallel_for((int)T, [&](int t) {
            const uint64_t a = per * (uint64_t)t;
            if (a < n) run(a, std::min(n, a + per));
        });
        return XS_OK;
    });
}

int xs_u64_member_mask(const uint64_t* keys, uint64_t n, const uint64_t* set, uint64_t m, uint8_t* out) {
    return xs::guard([&]() -> int {
        if ((n && (!keys || !out)) || (m && !set)) return xs::set_error(XS_ERR_ARG, "null argument");
        if (!m) {
            if (n) memset(out, 0, n);
            return XS_OK;
        }
        // open addressing over 2^b >= 2m slots; a slot holds value + 1 (0 = empty) and
        // the value ~0 is checked apart
        unsigned b = 1;
        while ((1ull << b) < 2 * m) ++b;
        const uint64_t mask = (1ull << b) - 1;
        std::vector<uint64_t> slot(mask + 1, 0);
        bool has_max = false;
        auto mix = [](uint64_t x) { return (x ^ (x >> 31)) * 0x9E3779B97F4A7C15ull; };
        for (uint64_t j = 0; j < m; ++j) {
            const uint64_t v = set[j];
            if (v == ~0ull) {
                has_max = true;
                continue;
            }
            uint64_t h = mix(v) >> (64 - b);
            while (slot[h] && slot[h] != v + 1) h = (h + 1) & mask;
            slot[h] = v + 1;
        }
        auto run = [&](uint64_t a, uint64_t e) {
            for (uint64_t i = a; i < e; ++i) {
                const uint64_t v = keys[i];
                uint8_t hit = 0;
                if (v == ~0ull) {
                    hit = has_max;
                } else {
                    uint64_t h = mix(v) >> (64 - b);
                    while (slot[h]) {
                        if (slot[h] == v + 1) {
                            hit = 1;
                            break;
                        }
                        h = (h + 1) & mask;
                    }
                }
                out[i] = hit;
            }
        };
        const uint64_t T = std::min<uint64_t>(16, std::max<uint64_t>(1, n / (1u << 16)));
        const uint64_t per = (n + T - 1) / T;
        xs::parallel_for((int)T, [&](int t) {
            const uint64_t a = per * (uint64_t)t;
            if (a < n) run(a, std::min(n, a + per));
        });
        return XS_OK;
    });
}

// *has_dup = 1 when two of the n ids are equal (byte for byte).  Open addressing
// over a 64-bit FNV-1a of each id; equal hashes are compared in full.
int xs_ids_has_duplicates(const char* buf, const uint64_t* offs, uint64_t n, int* has_dup) {
    return xs::guard([&]() -> int {
        if (!offs || !has_dup || (!buf && n && offs[n])) return xs::set_error(XS_ERR_ARG, "null argument");
        *has_dup = 0;
        if (n < 2) return XS_OK;
        // every read of a file is checked (MatrixResult; 12.5 M per rank at config 3): the ids are
        // hashed by up to 16 threads, binned by hash into 256 buckets, and each bucket is searched
        // for equal ids with a small table of its own (one thread per bucket at a time)
        const int T = (int)std::min<uint64_t>(16, std::max<uint64_t>(1, n / 65536));
        constexpr int kBucketBits = 8, kBuckets = 1 << kBucketBits;
        std::vector<uint64_t> hv(n);
        std::vector<uint64_t> cnt((size_t)T * kBuckets, 0);
        const uint64_t per = (n + T - 1) / T;
        auto par = [&](const std::function<void(int)>& fn) { xs::parallel_for(T, fn); };
        par([&](int t) {
            const uint64_t a = per * t, e = std::min(n, a + per);
            uint64_t* c = &cnt[(size_t)t * kBuckets];
            for (uint64_t i = a; i < e; ++i) {
                const unsigned char* s = reinterpret_cast<const unsigned char*>(buf + offs[i]);
                uint64_t h = 1469598103934665603ull;
                for (uint64_t j = 0, len = offs[i + 1] - offs[i]; j < len; ++j) h = (h ^ s[j]) * 1099511628211ull;
                h ^= h >> 29;
                h *= 0xBF58476D1CE4E5B9ull;
                h ^= h >> 32;
                hv[i] = h;
                ++c[h >> (64 - kBucketBits)];
            }
        });
        // bucket b holds [start[b], start[b + 1]) of `order`; thread t writes from its own cursor
        std::vector<uint64_t> start(kBuckets + 1, 0), cur((size_t)T * kBuckets);
        for (int b = 0; b < kBuckets; ++b) {
            uint64_t o = start[b];
            for (int t = 0; t < T; ++t) {
                cur[(size_t)t * kBuckets + b] = o;
                o += cnt[(size_t)t * kBuckets + b];
            }
            start[b + 1] = o;
        }
        std::vector<uint64_t> order(n);
        par([&](int t) {
            const uint64_t a = per * t, e = std::min(n, a + per);
            uint64_t* c = &cur[(size_t)t * kBuckets];
            for (uint64_t i = a; i < e; ++i) order[c[hv[i] >> (64 - kBucketBits)]++] = i;
        });
        std::atomic<int> found{0};
        par([&](int t) {
            std::vector<uint64_t> slot;  // index into order + 1; 0 = empty
            for (int b = t; b < kBuckets && !found.load(std::memory_order_relaxed); b += T) {
                const uint64_t b0 = start[b], m = start[b + 1] - b0;
                if (m < 2) continue;
                uint64_t cap = 16;
                while (cap < 2 * m) cap <<= 1;
                slot.assign(cap, 0);
                for (uint64_t q = 0; q < m; ++q) {
                    const uint64_t i = order[b0 + q], h = hv[i], len = offs[i + 1] - offs[i];
                    for (uint64_t p = (h * 0x9E3779B97F4A7C15ull) >> 1 & (cap - 1);; p = (p + 1) & (cap - 1)) {
                        if (!slot[p]) {
                            slot[p] = q + 1;
                            break;
                        }
                        const uint64_t k = order[b0 + slot[p] - 1];
                        if (hv[k] == h && offs[k + 1] - offs[k] == len && memcmp(buf + offs[k], buf + offs[i], len) == 0) {
                            found.store(1, std::memory_order_relaxed);
                            return;
                        }
                    }
                }
            }
        });
        *has_dup = found.load();
        return XS_OK;
    });
}
