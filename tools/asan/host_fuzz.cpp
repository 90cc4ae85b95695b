// Host-side sanitizer run (AddressSanitizer + UndefinedBehaviorSanitizer, host
// code only) of the FASTA/FASTQ reader and the JSON/FASTA writers of
// libxspect_hip.so: randomised well-formed and malformed inputs, every batch
// size from one byte up, 1..8 parser threads.  Functional equality with
// Biopython / json.dumps is tested in tests/test_fastx.py and
// tests/test_json_writer.py; this driver looks for memory errors only.
//   make -C tools/asan run
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/xspect_hip.h"
#include "../../xspect2_amd/csrc/xs_internal.h"

namespace xs {
int set_error(int code, const char* msg) {  // the library's version lives in xs_api.cpp (GPU side)
    (void)msg;
    return code;
}
// likewise (xs_api.cpp pins host memory; no GPU here, so plain host memory)
int pinned_alloc(size_t bytes, void** out) {
    *out = malloc(bytes ? bytes : 1);
    return *out ? 0 : -6;
}
void pinned_free(void* p) { free(p); }
}  // namespace xs
extern "C" const char* xs_last_error(void) { return ""; }  // likewise

static std::mt19937_64 rng(12345);

static std::string rand_seq(size_t n, const char* alpha) {
    std::string s;
    const size_t m = strlen(alpha);
    for (size_t i = 0; i < n; ++i) s += alpha[rng() % m];
    return s;
}

static std::string make_fasta(int recs, bool crlf, bool trailing_nl) {
    std::string out, nl = crlf ? "\r\n" : "\n";
    for (int r = 0; r < recs; ++r) {
        out += ">r" + std::to_string(r) + (rng() % 2 ? " desc words\t x" : "") + nl;
        const size_t len = rng() % 400;
        const std::string s = rand_seq(len, "ACGTNacgtRY");
        const size_t w = 1 + rng() % 90;
        for (size_t i = 0; i < s.size(); i += w) out += s.substr(i, w) + nl;
        if (rng() % 7 == 0) out += nl;  // blank line
    }
    if (!trailing_nl && !out.empty()) out.resize(out.size() - nl.size());
    return out;
}

static std::string make_fastq(int recs, bool wrapped, bool trailing_nl, bool malformed) {
    std::string out;
    for (int r = 0; r < recs; ++r) {
        const size_t len = rng() % 300;
        const std::string s = rand_seq(len, "ACGTN");
        std::string q = rand_seq(len, "@+IJ#!");  // '@' and '+' in qualities
        if (malformed && r == recs / 2) q.resize(q.size() / 2);
        out += "@r" + std::to_string(r) + " x\n";
        if (wrapped && len > 10) out += s.substr(0, len / 2) + "\n" + s.substr(len / 2) + "\n";
        else out += s + "\n";
        out += "+\n";
        if (wrapped && q.size() > 10) out += q.substr(0, q.size() / 2) + "\n" + q.substr(q.size() / 2) + "\n";
        else out += q + "\n";
    }
    if (!trailing_nl && !out.empty()) out.pop_back();
    return out;
}

static int read_all(const std::string& path, int fmt, int threads, uint64_t batch, uint64_t* recs,
                    uint32_t part = 0, uint32_t parts = 1) {
    xs_fastx* r = nullptr;
    int rc = xs_fastx_open_range(path.c_str(), fmt, threads, 0, part, parts, &r);
    if (rc) return rc;
    *recs = 0;
    xs_fastx_batch b;
    for (;;) {
        rc = xs_fastx_next(r, batch, &b);
        if (rc || b.n == 0) break;
        *recs += b.n;
        // touch everything the batch hands out
        volatile uint64_t sink = 0;
        for (uint64_t i = 0; i < b.n; ++i) {
            for (uint64_t o = b.offsets[i]; o < b.offsets[i + 1]; ++o) sink += (uint8_t)b.seqs[o];
            for (uint64_t o = b.id_offsets[i]; o < b.id_offsets[i + 1]; ++o) sink += (uint8_t)b.ids[o];
            for (uint64_t o = b.desc_offsets[i]; o < b.desc_offsets[i + 1]; ++o) sink += (uint8_t)b.descs[o];
        }
        std::vector<uint32_t> idx;
        for (uint64_t i = 0; i < b.n; i += 2) idx.push_back((uint32_t)i);
        if (xs_write_fasta("/tmp/xs_asan_out.fasta", 0, b.seqs, b.offsets, b.descs, b.desc_offsets, idx.data(),
                           idx.size(), 60))
            return -99;
    }
    xs_fastx_close(r);
    return rc;
}

static void write_file(const std::string& path, const std::string& text) {
    FILE* f = fopen(path.c_str(), "wb");
    fwrite(text.data(), 1, text.size(), f);
    fclose(f);
}

int main() {
    const std::string path = "/tmp/xs_asan_in.txt";
    int files = 0, errors = 0, unexpected = 0;
    auto sweep = [&](const std::string& text, int fmt, bool must_parse) {
        write_file(path, text);
        ++files;
        uint64_t whole = 0;
        for (uint64_t batch : {1ull, 7ull, 64ull, 1000ull, 1ull << 20})
            for (int threads : {1, 3, 8}) {
                uint64_t n = 0;
                const int rc = read_all(path, fmt, threads, batch, &n);
                if (rc) ++errors;  // malformed inputs must fail with an error code, not a crash
                if (rc && must_parse) ++unexpected;
                if (!rc) whole = n;
            }
        // byte-range parts (one rank each of a read-sharded job): well-formed
        // files split into parts whose record counts add up to the whole file's
        for (uint32_t parts : {2u, 3u, 7u}) {
            uint64_t sum = 0;
            bool failed = false;
            for (uint32_t part = 0; part < parts; ++part) {
                uint64_t n = 0;
                const int rc = read_all(path, fmt, 1 + part % 3, 64, &n, part, parts);
                if (rc) {
                    ++errors;
                    failed = true;
                }
                sum += n;
            }
            if (must_parse && (failed || sum != whole)) ++unexpected;
        }
    };
    for (int trial = 0; trial < 60; ++trial) {
        const bool fq = trial % 2;
        const int recs = (int)(rng() % 40);
        const bool bad = fq && trial % 11 == 0;
        const std::string text = fq ? make_fastq(recs, trial % 3 == 0, trial % 5 != 0, bad)
                                    : make_fasta(recs, trial % 3 == 0, trial % 5 != 0);
        sweep(text, fq ? XS_FASTX_FASTQ : XS_FASTX_FASTA, !bad);
        // the same file cut at a random byte, and with random bytes spliced in
        if (!text.empty()) {
            sweep(text.substr(0, rng() % text.size()), fq ? XS_FASTX_FASTQ : XS_FASTX_FASTA, !fq);
            std::string g = text;
            for (int i = 0; i < 8; ++i) g[rng() % g.size()] = (char)(rng() % 256);
            sweep(g, fq ? XS_FASTX_FASTQ : XS_FASTX_FASTA, false);
        }
    }
    for (const char* t : {"", ">", "@", ">\n", "@\n", "@r\n", "@r\nACGT\n+", "@r\nACGT\n+\nII", "\n\n\n", ">a\r\n\r\n",
                          "ACGT\n>x\nAC"})
        for (int fmt : {XS_FASTX_FASTA, XS_FASTX_FASTQ}) sweep(t, fmt, false);
    // JSON result sections: random hit matrices, masks, long ids
    for (int trial = 0; trial < 20; ++trial) {
        const uint64_t n = 1 + rng() % 300, D = 1 + rng() % 40;
        std::vector<uint32_t> hits(n * D);
        std::vector<uint64_t> nk(n);
        for (auto& h : hits) h = rng() % 200;
        for (auto& k : nk) k = 1 + rng() % 200;
        std::string ids, labels;
        std::vector<uint64_t> io{0}, lo{0};
        for (uint64_t i = 0; i < n; ++i) {
            ids += "\"read_" + std::to_string(i) + std::string(rng() % 30, 'x') + "\"";
            io.push_back(ids.size());
        }
        for (uint64_t d = 0; d < D; ++d) {
            labels += "\"" + std::to_string(470 + d) + "\"";
            lo.push_back(labels.size());
        }
        std::vector<uint8_t> mask(D);
        for (auto& m : mask) m = rng() % 3 != 0;
        FILE* f = fopen("/tmp/xs_asan_out.json", "wb");
        fclose(f);
        if (xs_write_result_sections("/tmp/xs_asan_out.json", n, D, hits.data(), 4, nk.data(), ids.c_str(), io.data(),
                                     labels.c_str(), lo.data(), trial % 2 ? mask.data() : nullptr, nullptr, 0,
                                     nullptr, 1 + trial % 8))
            ++errors;
    }
    // 128-bit id keys (xs_ids_hash128): ids of every length 0..200 packed back
    // to back in an exactly sized buffer, so a read past an id's end is caught
    for (int trial = 0; trial < 20; ++trial) {
        std::vector<uint64_t> off{0};
        std::string buf;
        for (int i = 0; i <= 200; ++i) {
            buf += rand_seq((size_t)((i + trial) % 201), "ACGT_:0123456789");
            off.push_back(buf.size());
        }
        std::vector<char> exact(buf.begin(), buf.end());
        std::vector<uint64_t> key(2 * (off.size() - 1));
        if (xs_ids_hash128(exact.data(), off.data(), off.size() - 1, key.data())) ++unexpected;
    }
    // a large batch takes the threaded path (n / 2^16 threads): keys equal the per-id ones;
    // a null offsets argument with ids is refused, not dereferenced
    {
        const uint64_t n = 300000;
        std::vector<uint64_t> off{0};
        std::string buf;
        for (uint64_t i = 0; i < n; ++i) {
            buf += "read_" + std::to_string(i);
            off.push_back(buf.size());
        }
        std::vector<char> exact(buf.begin(), buf.end());
        std::vector<uint64_t> key(2 * n), one(2);
        if (xs_ids_hash128(exact.data(), off.data(), n, key.data())) ++unexpected;
        for (uint64_t i = 0; i < n; i += 997) {
            const uint64_t o2[2] = {0, off[i + 1] - off[i]};
            if (xs_ids_hash128(exact.data() + off[i], o2, 1, one.data()) || one[0] != key[2 * i] ||
                one[1] != key[2 * i + 1])
                ++unexpected;
        }
        if (xs_ids_hash128(nullptr, nullptr, 5, key.data()) == 0) ++unexpected;
        else ++errors;
    }
    // member mask (xs_u64_member_mask): threaded pass over 400 k keys against sets with repeats,
    // 0 and 2^64-1, checked against std::set
    for (int trial = 0; trial < 6; ++trial) {
        const uint64_t n = 400000, m = trial == 0 ? 0 : 1000u * (uint64_t)trial;
        std::vector<uint64_t> keys(n), set;
        for (auto& k : keys) k = ((uint64_t)rng() << 32) ^ rng();
        keys[0] = 0;
        keys[1] = ~0ull;
        for (uint64_t j = 0; j < m; ++j) set.push_back(j % 2 ? keys[rng() % n] : ((uint64_t)rng() << 32) ^ rng());
        if (m) {
            set.push_back(0);
            set.push_back(~0ull);
            set.push_back(set[0]);
        }
        std::vector<uint8_t> out(n, 7);
        if (xs_u64_member_mask(keys.data(), n, set.empty() ? nullptr : set.data(), set.size(), out.data())) ++unexpected;
        std::set<uint64_t> ref(set.begin(), set.end());
        for (uint64_t i = 0; i < n; ++i)
            if (out[i] != (ref.count(keys[i]) ? 1 : 0)) ++unexpected;
    }
    // the persistent host workers (xs::parallel_for): 6 caller threads at once, each running jobs of
    // 1..20 tasks, some nested (a task starting its own job) and some throwing: every task runs
    // exactly once, a throwing task's exception reaches its caller after the others have finished
    {
        std::vector<std::thread> callers;
        std::atomic<int> bad{0};
        for (int c = 0; c < 6; ++c)
            callers.emplace_back([c, &bad] {
                std::mt19937_64 r(c);
                for (int job = 0; job < 300; ++job) {
                    const int n = 1 + (int)(r() % 20);
                    std::vector<std::atomic<int>> ran(n);
                    for (auto& x : ran) x = 0;
                    const int thrower = job % 7 == 0 ? (int)(r() % n) : -1;
                    bool caught = false;
                    try {
                        xs::parallel_for(n, [&](int t) {
                            ran[t]++;
                            if (job % 5 == 0) xs::parallel_for(3, [](int) {});  // nested
                            if (t == thrower) throw std::runtime_error("task failed");
                        });
                    } catch (const std::runtime_error&) {
                        caught = true;
                    }
                    if (caught != (thrower >= 0)) ++bad;
                    for (auto& x : ran)
                        if (x != 1) ++bad;
                }
            });
        for (auto& t : callers) t.join();
        unexpected += bad.load();
    }
    // repeated ids (xs_ids_has_duplicates): threaded passes over 300 k ids of 0..12 bytes, distinct
    // and with one repeat at random places, checked against std::set
    for (int trial = 0; trial < 6; ++trial) {
        const uint64_t n = 300000;
        std::vector<std::string> ids;
        std::set<std::string> seen;
        while (ids.size() < n) {
            std::string s = std::to_string(ids.size()) + rand_seq(rng() % 6, "ab:_");
            if (seen.insert(s).second) ids.push_back(s);
        }
        if (trial % 2) ids[rng() % n] = ids[rng() % n];
        std::string buf;
        std::vector<uint64_t> off{0};
        for (auto& s : ids) {
            buf += s;
            off.push_back(buf.size());
        }
        int dup = -1;
        if (xs_ids_has_duplicates(buf.data(), off.data(), n, &dup)) ++unexpected;
        const bool want = std::set<std::string>(ids.begin(), ids.end()).size() != n;
        if (dup != (want ? 1 : 0)) ++unexpected;
    }
    printf("host sanitizer run: %d input files x 15 reader configurations + 12 byte-range parts, 20 JSON matrices, "
           "20 id-key batches + a threaded one, 6 member masks, 6 threaded repeat checks, 1800 worker-pool jobs from 6 threads (nested, throwing); %d clean error returns, "
           "%d unexpected results\n",
           files, errors, unexpected);
    return unexpected ? 1 : 0;
}
