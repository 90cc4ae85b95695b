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
#include <cstdio>
#include <cstring>
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

struct ScoreCache {  // per thread: score strings of h = 0..n for the last n seen
    std::unordered_map<uint64_t, std::vector<std::string>> by_n;
    const std::string& get(uint64_t h, uint64_t n) {
        auto& v = by_n[n];
        if (v.empty() && n <= (1u << 16)) {
            v.resize(n + 1);
            for (uint64_t i = 0; i <= n; ++i) v[i] = score_text(i, n);
        }
        if (h < v.size()) return v[h];
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
    std::vector<uint32_t> docs;  // emitted docs (doc_mask), ascending
};

// Docs of one hit row in COBS result order: count descending, ties by doc index.
template <class T>
void order_of(const std::vector<uint32_t>& docs, const T* row, std::vector<uint32_t>& ord) {
    ord = docs;
    std::stable_sort(ord.begin(), ord.end(), [row](uint32_t a, uint32_t b) { return row[a] > row[b]; });
}

inline void put_key(std::string& o, const char* base, const uint64_t* off, uint64_t i) {
    o.append(base + off[i], (size_t)(off[i + 1] - off[i]));
}

// section 0: hits, 1: scores, 2: num_kmers — entries of reads [lo, hi)
template <class T>
void format_block(const Ctx<T>& c, int section, uint64_t lo, uint64_t hi, std::string& o) {
    std::vector<uint32_t> ord;
    ScoreCache cache;
    char num[32];
    for (uint64_t r = lo; r < hi; ++r) {
        if (r) o += ",\n";
        o += "        ";
        put_key(o, c.ids, c.ids_off, r);
        if (section == 2) {
            int k = snprintf(num, sizeof(num), ": %llu", (unsigned long long)c.nk[r]);
            o.append(num, (size_t)k);
            continue;
        }
        if (c.docs.empty()) {
            o += ": {}";
            continue;
        }
        o += ": {\n";
        const T* row = c.hits + r * c.D;
        order_of(c.docs, row, ord);
        for (size_t j = 0; j < ord.size(); ++j) {
            if (j) o += ",\n";
            o += "            ";
            put_key(o, c.labels, c.labels_off, ord[j]);
            o += ": ";
            if (section == 0) {
                int k = snprintf(num, sizeof(num), "%u", (unsigned)row[ord[j]]);
                o.append(num, (size_t)k);
            } else {
                o += cache.get(row[ord[j]], c.nk[r]);
            }
        }
        o += "\n        }";
    }
}

template <class T>
int write_sections(const char* path, const Ctx<T>& c, const uint64_t* total_hits, uint64_t total_kmers_in,
                   const uint32_t* total_order_row, int threads) {
    const uint64_t n = c.n, num_docs = c.D;
    FILE* f = fopen(path, "ab");
    if (!f) return xs::set_error(XS_ERR_IO, (std::string("cannot append to ") + path).c_str());
    const int NT = std::max(1, std::min(threads > 0 ? threads : 16, 64));
    const uint64_t block = 1 << 16;  // reads per formatting round
    std::vector<std::string> out((size_t)NT);
    bool ok = true;
    const char* heads[3] = {"\"hits\": ", "\"scores\": ", "\"num_kmers\": "};
    for (int section = 0; section < 3 && ok; ++section) {
        // an empty section is "{}" as json.dumps writes it (a shard without reads)
        const bool empty = n == 0 && section != 1;
        ok = fputs(heads[section], f) >= 0 && fputs(empty ? "{}" : "{\n", f) >= 0;
        for (uint64_t b0 = 0; b0 < n && ok; b0 += block) {
            const uint64_t b1 = std::min(n, b0 + block);
            const uint64_t per = (b1 - b0 + NT - 1) / NT;
            std::vector<std::thread> th;
            auto work = [&](int t) {
                out[t].clear();
                const uint64_t lo = b0 + per * t, hi = std::min(b1, lo + per);
                if (lo < hi) format_block(c, section, lo, hi, out[t]);
            };
            for (int t = 1; t < NT; ++t) th.emplace_back(work, t);
            work(0);
            for (auto& x : th) x.join();
            for (int t = 0; t < NT && ok; ++t) ok = fwrite(out[t].data(), 1, out[t].size(), f) == out[t].size();
        }
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
    Ctx<T> c{n, num_docs, static_cast<const T*>(hits), num_kmers, ids_json, ids_off, labels_json, labels_off, {}};
    for (uint64_t d = 0; d < num_docs; ++d)
        if (!doc_mask || doc_mask[d]) c.docs.push_back((uint32_t)d);
    return write_sections(path, c, total_hits, total_kmers, total_order_row, threads);
}

}  // namespace

extern "C" {

int xs_write_result_sections(const char* path, uint64_t n, uint64_t num_docs, const void* hits, int hit_bytes,
                             const uint64_t* num_kmers, const char* ids_json, const uint64_t* ids_off,
                             const char* labels_json, const uint64_t* labels_off, const uint8_t* doc_mask,
                             const uint64_t* total_hits, uint64_t total_kmers, const uint32_t* total_order_row,
                             int threads) {
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
}

}  // extern "C"
