/*
 * xs_oracle.c — CPU ORACLE (test infrastructure only).
 *
 * This file is the plain-C restatement of the k-mer extract + probabilistic
 * filter lookup that XspecT delegates to its native dependencies.  It is the
 * CHECKER for the HIP product path in xspect2_amd/csrc; nothing in the product
 * links, loads or calls it.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may use it.
 *
 * What it restates (reference call sites, /root/reference relative):
 *   - species model search: cobs_index.Search.search(query, step)
 *       src/xspect/models/probabilistic_filter_model.py:227 (calculate_hits),
 *       k-mer count formula :462 (_count_kmers)
 *   - species model construction: cobs.classic_construct_list
 *       src/xspect/models/probabilistic_filter_model.py:186-192
 *   - MLST model search/construction on COBS compact indices
 *       src/xspect/models/probabilistic_filter_mlst_model.py:132-142,242,274
 *   - genus model: rbloom.Bloom.__contains__/add with hash_func=xxh3_64_intdigest
 *       src/xspect/models/probabilistic_single_filter_model.py:88-91,122-124,
 *       k-mer generator :161-180 (min(kmer, revcomp) on case-preserved bytes)
 *
 * The arithmetic lives in third-party libraries that are NOT in /root/reference
 * and are unpinned in its pyproject.toml:16-18 (cobs-reloaded, rbloom, xxhash).
 * Their published algorithms are restated here:
 *   - XXH64 and XXH3-64 (xxHash spec, libxxhash 0.8.x): PINNED against
 *     python-xxhash 3.8.1 golden vectors in tests/golden/xxh_vectors.json.
 *   - COBS: canonical k-mer, row_j = XXH64(canonical, k, seed=j) mod S for
 *     j < num_hashes, AND of the h rows, doc d = byte d>>3 bit d&7, score =
 *     number of sampled positions whose AND has bit d.  PARITY UNPINNED
 *     against the real cobs-reloaded (absent offline).
 *   - rbloom: 128-bit LCG index generator seeded by the XXH3-64 hash.
 *     PARITY UNPINNED against the real rbloom (absent offline).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ */
/* xxHash primitives                                                   */
/* ------------------------------------------------------------------ */
#define P64_1 0x9E3779B185EBCA87ULL
#define P64_2 0xC2B2AE3D27D4EB4FULL
#define P64_3 0x165667B19E3779F9ULL
#define P64_4 0x85EBCA77C2B2AE63ULL
#define P64_5 0x27D4EB2F165667C5ULL
#define P32_1 0x9E3779B1U
#define P32_2 0x85EBCA77U
#define P32_3 0xC2B2AE3DU

static const uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};

static inline uint64_t rd64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}
static inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }
static inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

static inline uint64_t xxh64_round(uint64_t acc, uint64_t in) {
    acc += in * P64_2;
    acc = rotl64(acc, 31);
    return acc * P64_1;
}
static inline uint64_t xxh64_merge(uint64_t acc, uint64_t v) {
    acc ^= xxh64_round(0, v);
    return acc * P64_1 + P64_4;
}
static inline uint64_t xxh64_avalanche(uint64_t h) {
    h ^= h >> 33; h *= P64_2;
    h ^= h >> 29; h *= P64_3;
    h ^= h >> 32;
    return h;
}

uint64_t xo_xxh64(const void* data, uint64_t len, uint64_t seed) {
    const uint8_t* p = (const uint8_t*)data;
    const uint8_t* end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P64_1 + P64_2, v2 = seed + P64_2, v3 = seed, v4 = seed - P64_1;
        const uint8_t* limit = end - 32;
        do {
            v1 = xxh64_round(v1, rd64(p));
            v2 = xxh64_round(v2, rd64(p + 8));
            v3 = xxh64_round(v3, rd64(p + 16));
            v4 = xxh64_round(v4, rd64(p + 24));
            p += 32;
        } while (p <= limit);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xxh64_merge(h, v1); h = xxh64_merge(h, v2);
        h = xxh64_merge(h, v3); h = xxh64_merge(h, v4);
    } else {
        h = seed + P64_5;
    }
    h += len;
    while (p + 8 <= end) {
        h ^= xxh64_round(0, rd64(p));
        h = rotl64(h, 27) * P64_1 + P64_4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)rd32(p) * P64_1;
        h = rotl64(h, 23) * P64_2 + P64_3;
        p += 4;
    }
    while (p < end) {
        h ^= (uint64_t)(*p) * P64_5;
        h = rotl64(h, 11) * P64_1;
        ++p;
    }
    return xxh64_avalanche(h);
}

static inline uint64_t mul128_fold64(uint64_t a, uint64_t b) {
    __uint128_t r = (__uint128_t)a * b;
    return (uint64_t)r ^ (uint64_t)(r >> 64);
}
static inline uint64_t xxh3_avalanche(uint64_t h) {
    h ^= h >> 37;
    h *= 0x165667919E3779F9ULL;
    h ^= h >> 32;
    return h;
}
static inline uint64_t xxh3_rrmxmx(uint64_t h, uint64_t len) {
    h ^= rotl64(h, 49) ^ rotl64(h, 24);
    h *= 0x9FB21C651E98DF25ULL;
    h ^= (h >> 35) + len;
    h *= 0x9FB21C651E98DF25ULL;
    return h ^ (h >> 28);
}
static inline uint64_t xxh3_mix16(const uint8_t* in, const uint8_t* sec, uint64_t seed) {
    return mul128_fold64(rd64(in) ^ (rd64(sec) + seed), rd64(in + 8) ^ (rd64(sec + 8) - seed));
}

/* XXH3-64 with the default secret and seed 0 (xxh3_64_intdigest(b)),
 * lengths 0..240.  Returns 0 and sets *ok=0 for longer inputs. */
uint64_t xo_xxh3_64(const void* data, uint64_t len, int* ok) {
    const uint8_t* in = (const uint8_t*)data;
    const uint8_t* s = kSecret;
    const uint64_t seed = 0;
    if (ok) *ok = 1;
    if (len == 0) return xxh64_avalanche(seed ^ (rd64(s + 56) ^ rd64(s + 64)));
    if (len <= 3) {
        uint32_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
        uint32_t comb = (c1 << 16) | (c2 << 24) | c3 | ((uint32_t)len << 8);
        uint64_t flip = (uint64_t)(rd32(s) ^ rd32(s + 4)) + seed;
        return xxh64_avalanche((uint64_t)comb ^ flip);
    }
    if (len <= 8) {
        uint64_t sd = seed ^ ((uint64_t)bswap32((uint32_t)seed) << 32);
        uint32_t i1 = rd32(in), i2 = rd32(in + len - 4);
        uint64_t flip = (rd64(s + 8) ^ rd64(s + 16)) - sd;
        uint64_t i64 = (uint64_t)i2 + ((uint64_t)i1 << 32);
        return xxh3_rrmxmx(i64 ^ flip, len);
    }
    if (len <= 16) {
        uint64_t f1 = (rd64(s + 24) ^ rd64(s + 32)) + seed;
        uint64_t f2 = (rd64(s + 40) ^ rd64(s + 48)) - seed;
        uint64_t lo = rd64(in) ^ f1;
        uint64_t hi = rd64(in + len - 8) ^ f2;
        uint64_t acc = len + bswap64(lo) + hi + mul128_fold64(lo, hi);
        return xxh3_avalanche(acc);
    }
    if (len <= 128) {
        uint64_t acc = len * P64_1;
        if (len > 32) {
            if (len > 64) {
                if (len > 96) {
                    acc += xxh3_mix16(in + 48, s + 96, seed);
                    acc += xxh3_mix16(in + len - 64, s + 112, seed);
                }
                acc += xxh3_mix16(in + 32, s + 64, seed);
                acc += xxh3_mix16(in + len - 48, s + 80, seed);
            }
            acc += xxh3_mix16(in + 16, s + 32, seed);
            acc += xxh3_mix16(in + len - 32, s + 48, seed);
        }
        acc += xxh3_mix16(in, s, seed);
        acc += xxh3_mix16(in + len - 16, s + 16, seed);
        return xxh3_avalanche(acc);
    }
    if (len <= 240) {
        uint64_t acc = len * P64_1;
        int rounds = (int)(len / 16);
        for (int i = 0; i < 8; ++i) acc += xxh3_mix16(in + 16 * i, s + 16 * i, seed);
        acc = xxh3_avalanche(acc);
        for (int i = 8; i < rounds; ++i) acc += xxh3_mix16(in + 16 * i, s + 16 * (i - 8) + 3, seed);
        acc += xxh3_mix16(in + len - 16, s + 136 - 17, seed);
        return xxh3_avalanche(acc);
    }
    if (ok) *ok = 0;
    return 0;
}

/* ------------------------------------------------------------------ */
/* Canonical k-mers                                                    */
/* ------------------------------------------------------------------ */
/* COBS spec (restated, UNVERIFIED): bases are normalised (ACGT kept,
 * acgt upper-cased, any other byte -> 'N'), then the canonical k-mer is the
 * byte-lexicographic min of the normalised forward strand and its reverse
 * complement (A<->T, C<->G, N<->N). */
static uint8_t cobs_norm[256], cobs_comp[256], bio_comp[256];
static int tables_ready = 0;

static void init_tables(void) {
    if (tables_ready) return;
    for (int i = 0; i < 256; ++i) { cobs_norm[i] = 'N'; cobs_comp[i] = 'N'; bio_comp[i] = (uint8_t)i; }
    const char* up = "ACGT"; const char* lo = "acgt";
    for (int i = 0; i < 4; ++i) { cobs_norm[(uint8_t)up[i]] = up[i]; cobs_norm[(uint8_t)lo[i]] = up[i]; }
    cobs_comp['A'] = 'T'; cobs_comp['T'] = 'A'; cobs_comp['C'] = 'G'; cobs_comp['G'] = 'C';
    /* Biopython ambiguous_dna_complement (both cases); unmapped bytes unchanged. */
    const char* pairs = "ATTACGGCMKKMRYYRWWSSVBBVHDDHXXNN";
    for (int i = 0; pairs[i]; i += 2) {
        uint8_t a = (uint8_t)pairs[i], b = (uint8_t)pairs[i + 1];
        bio_comp[a] = b;
        bio_comp[a + 32] = (uint8_t)(b + 32);
    }
    tables_ready = 1;
}

void xo_canonical_cobs(const uint8_t* in, int k, uint8_t* out) {
    init_tables();
    uint8_t fwd[256], rc[256];
    for (int i = 0; i < k; ++i) fwd[i] = cobs_norm[in[i]];
    for (int i = 0; i < k; ++i) rc[i] = cobs_comp[fwd[k - 1 - i]];
    memcpy(out, memcmp(rc, fwd, (size_t)k) < 0 ? rc : fwd, (size_t)k);
}

/* Genus spec: min(kmer, str(kmer.reverse_complement())) on raw bytes
 * (probabilistic_single_filter_model.py:179); case preserved. */
void xo_canonical_bio(const uint8_t* in, int k, uint8_t* out) {
    init_tables();
    uint8_t rc[256];
    for (int i = 0; i < k; ++i) rc[i] = bio_comp[in[k - 1 - i]];
    memcpy(out, memcmp(rc, in, (size_t)k) < 0 ? rc : in, (size_t)k);
}

/* COBS calc_signature_size (restated): ceil(-h*n / ln(1 - fpr^(1/h))). */
uint64_t xo_cobs_signature_size(uint64_t n, uint64_t h, double fpr) {
    double s = ceil(-(double)h * (double)n / log(1.0 - pow(fpr, 1.0 / (double)h)));
    return (uint64_t)s;
}

/* Sampled k-mer positions of a record: i*step for i < ceil((L-k+1)/step)
 * (probabilistic_filter_model.py:462; single_filter_model.py:175-178). */
uint64_t xo_num_kmers(uint64_t len, int k, uint32_t step) {
    if (len < (uint64_t)k || step == 0) return 0;
    uint64_t n = len - (uint64_t)k + 1;
    return (n + step - 1) / step;
}

/* ------------------------------------------------------------------ */
/* COBS classic/compact bank: a list of doc groups.  Group g covers docs */
/* [g*8*P, min((g+1)*8*P, D)), has S_g rows of P bytes, and its rows start */
/* at byte base_g of one contiguous array.  Classic = one group, P = R.   */
/* ------------------------------------------------------------------ */
typedef struct {
    const uint8_t* rows;
    const uint64_t* sig;   /* [G] rows per group */
    uint64_t G, P, D;
    uint32_t h;
    int k;
} xo_bank;

static void bank_kmer_mask(const xo_bank* b, const uint8_t* canon, uint8_t* mask, uint64_t* hashes) {
    for (uint32_t j = 0; j < b->h; ++j) hashes[j] = xo_xxh64(canon, (uint64_t)b->k, j);
    uint64_t base = 0;
    for (uint64_t g = 0; g < b->G; ++g) {
        uint8_t* m = mask + g * b->P;
        for (uint32_t j = 0; j < b->h; ++j) {
            const uint8_t* row = b->rows + base + (hashes[j] % b->sig[g]) * b->P;
            if (j == 0) memcpy(m, row, b->P);
            else for (uint64_t x = 0; x < b->P; ++x) m[x] &= row[x];
        }
        base += b->sig[g] * b->P;
    }
}

/* hits[r*D + d] = number of sampled positions of read r whose canonical
 * k-mer has doc d set in all h rows; nk[r] = number of sampled positions. */
int xo_cobs_query(const uint8_t* rows, const uint64_t* sig, uint64_t G, uint64_t P, uint64_t D,
                  uint32_t h, int k, const uint8_t* seqs, const uint64_t* offsets, uint64_t n,
                  uint32_t step, uint32_t* hits, uint64_t* nk, int nthreads) {
    if (k < 1 || k > 255 || h < 1 || h > 64 || step < 1) return -1;
    xo_bank b = {rows, sig, G, P, D, h, k};
    init_tables();
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        uint8_t canon[256];
        uint64_t hashes[64];
        uint8_t* mask = (uint8_t*)malloc(G * P);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
        for (int64_t r = 0; r < (int64_t)n; ++r) {
            const uint8_t* s = seqs + offsets[r];
            uint64_t len = offsets[r + 1] - offsets[r];
            uint64_t cnt = xo_num_kmers(len, k, step);
            uint32_t* out = hits + (uint64_t)r * D;
            memset(out, 0, D * sizeof(uint32_t));
            nk[r] = cnt;
            for (uint64_t i = 0; i < cnt; ++i) {
                xo_canonical_cobs(s + i * step, k, canon);
                bank_kmer_mask(&b, canon, mask, hashes);
                for (uint64_t d = 0; d < D; ++d) {
                    uint64_t g = d / (8 * P), bit = d % (8 * P);
                    out[d] += (mask[g * P + (bit >> 3)] >> (bit & 7)) & 1;
                }
            }
        }
        free(mask);
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* The same query, batched for the CPU baseline (bench.py cpu_baseline): */
/* identical hits and counts (tests/test_oracle.py checks them against   */
/* xo_cobs_query bit for bit), computed the way a tuned CPU port would:  */
/*  - XXH64 of a k < 32 byte key: the seed enters only through the start */
/*    value, so each 8/4/1-byte term is computed once per k-mer and the  */
/*    h seeds run the short chain (xo_xxh64 is the pinned reference);    */
/*  - the row addresses of every sampled k-mer of a read are computed    */
/*    first and the rows prefetched kLook k-mers ahead (memory-level     */
/*    parallelism instead of one dependent miss after another);          */
/*  - counts are added 4 docs at a time: one table lookup per mask       */
/*    nibble into 16-bit lanes, flushed to the uint32 output every 65535 */
/*    k-mers.                                                            */
/* ------------------------------------------------------------------ */
typedef struct {
    uint64_t t8[4];  /* xxh64_round(0, chunk) of each 8-byte chunk */
    uint64_t t4;     /* 4-byte chunk * P1 */
    uint64_t t1[4];  /* trailing bytes * P5 */
    int n8, has4, n1;
    uint64_t len;
} xo_xxh64_terms;

static inline void xxh64_terms(const uint8_t* p, uint64_t len, xo_xxh64_terms* t) {
    const uint8_t* end = p + len;
    t->len = len;
    t->n8 = 0;
    while (p + 8 <= end) { t->t8[t->n8++] = xxh64_round(0, rd64(p)); p += 8; }
    t->has4 = p + 4 <= end;
    if (t->has4) { t->t4 = (uint64_t)rd32(p) * P64_1; p += 4; }
    t->n1 = 0;
    while (p < end) t->t1[t->n1++] = (uint64_t)(*p++) * P64_5;
}

static inline uint64_t xxh64_seeded(const xo_xxh64_terms* t, uint64_t seed) {
    uint64_t h = seed + P64_5 + t->len;
    for (int i = 0; i < t->n8; ++i) { h ^= t->t8[i]; h = rotl64(h, 27) * P64_1 + P64_4; }
    if (t->has4) { h ^= t->t4; h = rotl64(h, 23) * P64_2 + P64_3; }
    for (int i = 0; i < t->n1; ++i) { h ^= t->t1[i]; h = rotl64(h, 11) * P64_1; }
    return xxh64_avalanche(h);
}

/* xo_xxh64 through the batched form: the tests compare the two for every
 * length 0..31 and many seeds (the batched query relies on it) */
uint64_t xo_xxh64_terms_check(const void* data, uint64_t len, uint64_t seed) {
    if (len >= 32) return xo_xxh64(data, len, seed);
    xo_xxh64_terms t;
    xxh64_terms((const uint8_t*)data, len, &t);
    return xxh64_seeded(&t, seed);
}

static uint64_t nibble_lanes[16];  /* bit i of a nibble -> 16-bit lane i */

/* a % d without a division: q = mulhi(a, floor((2^64-1)/d)) undershoots the
 * quotient by at most 2, so at most two corrections follow */
static inline uint64_t mod_barrett(uint64_t a, uint64_t d, uint64_t magic) {
    const uint64_t q = (uint64_t)(((__uint128_t)a * magic) >> 64);
    uint64_t r = a - q * d;
    while (r >= d) r -= d;
    return r;
}

/* dst[0..P) &= src[0..P) in 8-byte words (the last word overlapping when P
 * is not a multiple of 8; AND is idempotent, so the overlap is harmless) */
static inline void and_row(uint8_t* dst, const uint8_t* src, uint64_t P) {
    if (P < 8) {
        for (uint64_t x = 0; x < P; ++x) dst[x] &= src[x];
        return;
    }
    uint64_t x = 0, a, b;
    for (; x + 8 <= P; x += 8) {
        memcpy(&a, dst + x, 8);
        memcpy(&b, src + x, 8);
        a &= b;
        memcpy(dst + x, &a, 8);
    }
    if (x < P) {
        memcpy(&a, dst + P - 8, 8);
        memcpy(&b, src + P - 8, 8);
        a &= b;
        memcpy(dst + P - 8, &a, 8);
    }
}

int xo_cobs_query_batched(const uint8_t* rows, const uint64_t* sig, uint64_t G, uint64_t P, uint64_t D,
                          uint32_t h, int k, const uint8_t* seqs, const uint64_t* offsets, uint64_t n,
                          uint32_t step, uint32_t* hits, uint64_t* nk, int nthreads) {
    if (k < 1 || k > 255 || h < 1 || h > 64 || step < 1) return -1;
    if (k >= 32) return xo_cobs_query(rows, sig, G, P, D, h, k, seqs, offsets, n, step, hits, nk, nthreads);
    init_tables();
    for (int x = 0; x < 16; ++x) {
        uint64_t v = 0;
        for (int i = 0; i < 4; ++i)
            if (x >> i & 1) v |= 1ull << (16 * i);
        nibble_lanes[x] = v;
    }
    uint64_t* base = (uint64_t*)malloc((G + 1) * sizeof(uint64_t));
    uint64_t* magic = (uint64_t*)malloc(G * sizeof(uint64_t));
    base[0] = 0;
    for (uint64_t g = 0; g < G; ++g) {
        base[g + 1] = base[g] + sig[g] * P;
        magic[g] = sig[g] ? ~0ull / sig[g] : 0;
    }
#ifndef XO_LOOK
#define XO_LOOK 12
#endif
    enum { kLook = XO_LOOK, kFlush = 65535 };
    const uint64_t lanes = 2 * G * P;  /* 4 docs per uint64 of counters */
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        uint8_t canon[256];
        uint8_t* mask = (uint8_t*)malloc(G * P);
        uint64_t* cnt = (uint64_t*)calloc(lanes, sizeof(uint64_t));
        uint64_t cap = 0;
        const uint8_t** rp = NULL;  /* [k-mer][group][hash] row pointers of one read */
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
        for (int64_t r = 0; r < (int64_t)n; ++r) {
            const uint8_t* s = seqs + offsets[r];
            const uint64_t len = offsets[r + 1] - offsets[r];
            const uint64_t m = xo_num_kmers(len, k, step);
            uint32_t* out = hits + (uint64_t)r * D;
            memset(out, 0, D * sizeof(uint32_t));
            nk[r] = m;
            const uint64_t per = G * h;
            if (m * per > cap) {
                cap = m * per;
                rp = (const uint8_t**)realloc(rp, cap * sizeof(*rp));
            }
            for (uint64_t i = 0; i < m; ++i) {
                xo_canonical_cobs(s + i * step, k, canon);
                xo_xxh64_terms t;
                xxh64_terms(canon, (uint64_t)k, &t);
                for (uint32_t j = 0; j < h; ++j) {
                    const uint64_t hv = xxh64_seeded(&t, j);
                    for (uint64_t g = 0; g < G; ++g)
                        rp[i * per + g * h + j] = rows + base[g] + mod_barrett(hv, sig[g], magic[g]) * P;
                }
            }
            for (uint64_t i = 0; i < m && i < kLook; ++i)
                for (uint64_t q = 0; q < per; ++q) __builtin_prefetch(rp[i * per + q]);
            uint64_t since = 0;
            for (uint64_t i = 0; i < m; ++i) {
                if (i + kLook < m)
                    for (uint64_t q = 0; q < per; ++q) __builtin_prefetch(rp[(i + kLook) * per + q]);
                const uint8_t* const* kr = rp + i * per;
                for (uint64_t g = 0; g < G; ++g) {
                    uint8_t* mg = mask + g * P;
                    memcpy(mg, kr[g * h], P);
                    for (uint32_t j = 1; j < h; ++j) and_row(mg, kr[g * h + j], P);
                }
                for (uint64_t x = 0; x < G * P; ++x) {
                    const uint8_t v = mask[x];
                    if (!v) continue;
                    cnt[2 * x] += nibble_lanes[v & 15];
                    cnt[2 * x + 1] += nibble_lanes[v >> 4];
                }
                if (++since == kFlush || i + 1 == m) {  /* 16-bit lanes: flush before they can wrap */
                    for (uint64_t q = 0; q < lanes; ++q) {
                        const uint64_t c = cnt[q];
                        if (!c) continue;
                        for (int l = 0; l < 4; ++l) {
                            const uint64_t d = 4 * q + (uint64_t)l;  /* group-major doc order = doc index */
                            if (d < D) out[d] += (uint32_t)(c >> (16 * l) & 0xFFFF);
                        }
                        cnt[q] = 0;
                    }
                    since = 0;
                }
            }
        }
        free(rp);
        free(cnt);
        free(mask);
    }
    free(magic);
    free(base);
    return 0;
}

/* Construction: every position (step 1) of every record of doc rec_doc[r]
 * sets bit (doc - group start) of its h rows in the doc's group. */
int xo_cobs_build(uint8_t* rows, const uint64_t* sig, uint64_t G, uint64_t P, uint64_t D,
                  uint32_t h, int k, const uint8_t* seqs, const uint64_t* offsets,
                  const uint32_t* rec_doc, uint64_t n_rec) {
    if (k < 1 || k > 255 || h < 1 || h > 64) return -1;
    init_tables();
    uint64_t* base = (uint64_t*)malloc((G + 1) * sizeof(uint64_t));
    base[0] = 0;
    for (uint64_t g = 0; g < G; ++g) base[g + 1] = base[g] + sig[g] * P;
    uint8_t canon[256];
    for (uint64_t r = 0; r < n_rec; ++r) {
        uint64_t d = rec_doc[r];
        if (d >= D) { free(base); return -2; }
        uint64_t g = d / (8 * P), bit = d % (8 * P);
        const uint8_t* s = seqs + offsets[r];
        uint64_t len = offsets[r + 1] - offsets[r];
        uint64_t cnt = xo_num_kmers(len, k, 1);
        for (uint64_t i = 0; i < cnt; ++i) {
            xo_canonical_cobs(s + i, k, canon);
            for (uint32_t j = 0; j < h; ++j) {
                uint64_t row = xo_xxh64(canon, (uint64_t)k, j) % sig[g];
                rows[base[g] + row * P + (bit >> 3)] |= (uint8_t)(1u << (bit & 7));
            }
        }
    }
    free(base);
    return 0;
}

/* ------------------------------------------------------------------ */
/* rbloom restatement (UNVERIFIED index generator)                      */
/* ------------------------------------------------------------------ */
/* state_{i+1} = state_i * M + C (mod 2^128), index_i = (state_{i+1} >> 64) % m,
 * state_0 = xxh3_64(canonical bytes).  M, C = the 128-bit PCG LCG constants. */
static const __uint128_t LCG_M = ((__uint128_t)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL;
static const __uint128_t LCG_C = ((__uint128_t)0x5851F42D4C957F2DULL << 64) | 0x14057B7EF767814FULL;

void xo_bloom_indexes(uint64_t hash, uint64_t nhash, uint64_t mbits, uint64_t* out) {
    __uint128_t st = hash;
    for (uint64_t i = 0; i < nhash; ++i) {
        st = st * LCG_M + LCG_C;
        out[i] = (uint64_t)(st >> 64) % mbits;
    }
}

int xo_bloom_build(uint8_t* bits, uint64_t nbytes, uint64_t nhash, int k, const uint8_t* seqs,
                   const uint64_t* offsets, uint64_t n_rec) {
    if (k < 1 || k > 240 || nhash < 1 || nhash > 64) return -1;
    uint8_t canon[256];
    uint64_t idx[64];
    for (uint64_t r = 0; r < n_rec; ++r) {
        const uint8_t* s = seqs + offsets[r];
        uint64_t cnt = xo_num_kmers(offsets[r + 1] - offsets[r], k, 1);
        for (uint64_t i = 0; i < cnt; ++i) {
            xo_canonical_bio(s + i, k, canon);
            xo_bloom_indexes(xo_xxh3_64(canon, (uint64_t)k, 0), nhash, nbytes * 8, idx);
            for (uint64_t j = 0; j < nhash; ++j) bits[idx[j] >> 3] |= (uint8_t)(1u << (idx[j] & 7));
        }
    }
    return 0;
}

int xo_bloom_query(const uint8_t* bits, uint64_t nbytes, uint64_t nhash, int k, const uint8_t* seqs,
                   const uint64_t* offsets, uint64_t n, uint32_t step, uint32_t* hits, uint64_t* nk,
                   int nthreads) {
    if (k < 1 || k > 240 || nhash < 1 || nhash > 64 || step < 1) return -1;
    init_tables();
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        uint8_t canon[256];
        uint64_t idx[64];
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
        for (int64_t r = 0; r < (int64_t)n; ++r) {
            const uint8_t* s = seqs + offsets[r];
            uint64_t cnt = xo_num_kmers(offsets[r + 1] - offsets[r], k, step);
            uint32_t c = 0;
            for (uint64_t i = 0; i < cnt; ++i) {
                xo_canonical_bio(s + i * step, k, canon);
                xo_bloom_indexes(xo_xxh3_64(canon, (uint64_t)k, 0), nhash, nbytes * 8, idx);
                int in = 1;
                for (uint64_t j = 0; j < nhash && in; ++j) in = (bits[idx[j] >> 3] >> (idx[j] & 7)) & 1;
                c += (uint32_t)in;
            }
            hits[r] = c;
            nk[r] = cnt;
        }
    }
    return 0;
}

/* The same query batched for the CPU baseline (bit-identical, tests/test_oracle.py):
 * every sampled k-mer's K bit indices first (Barrett remainders instead of
 * divisions), their bytes prefetched kLook k-mers ahead, then the test with
 * rbloom's stop at the first zero bit. */
int xo_bloom_query_batched(const uint8_t* bits, uint64_t nbytes, uint64_t nhash, int k, const uint8_t* seqs,
                           const uint64_t* offsets, uint64_t n, uint32_t step, uint32_t* hits, uint64_t* nk,
                           int nthreads) {
    if (k < 1 || k > 240 || nhash < 1 || nhash > 64 || step < 1 || nbytes == 0) return -1;
    init_tables();
    const uint64_t mbits = nbytes * 8, magic = ~0ull / mbits;
    int failed = 0;
    enum { kLook = 12 };
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        uint8_t canon[256];
        uint64_t cap = 0;
        uint64_t* idx = NULL;  /* [k-mer][hash] bit indices of one read */
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
        for (int64_t r = 0; r < (int64_t)n; ++r) {
            const uint8_t* s = seqs + offsets[r];
            const uint64_t cnt = xo_num_kmers(offsets[r + 1] - offsets[r], k, step);
            if (cnt * nhash > cap) {
                uint64_t* grown = (uint64_t*)realloc(idx, cnt * nhash * sizeof(*idx));
                if (!grown) {
#ifdef _OPENMP
#pragma omp atomic write
#endif
                    failed = 1;
                    continue;
                }
                idx = grown;
                cap = cnt * nhash;
            }
            for (uint64_t i = 0; i < cnt; ++i) {
                xo_canonical_bio(s + i * step, k, canon);
                __uint128_t st = xo_xxh3_64(canon, (uint64_t)k, 0);
                for (uint64_t j = 0; j < nhash; ++j) {
                    st = st * LCG_M + LCG_C;
                    idx[i * nhash + j] = mod_barrett((uint64_t)(st >> 64), mbits, magic);
                }
            }
            for (uint64_t i = 0; i < cnt && i < kLook; ++i)
                for (uint64_t j = 0; j < nhash; ++j) __builtin_prefetch(bits + (idx[i * nhash + j] >> 3));
            uint32_t c = 0;
            for (uint64_t i = 0; i < cnt; ++i) {
                if (i + kLook < cnt)
                    for (uint64_t j = 0; j < nhash; ++j) __builtin_prefetch(bits + (idx[(i + kLook) * nhash + j] >> 3));
                const uint64_t* x = idx + i * nhash;
                int in = 1;
                for (uint64_t j = 0; j < nhash && in; ++j) in = (bits[x[j] >> 3] >> (x[j] & 7)) & 1;
                c += (uint32_t)in;
            }
            hits[r] = c;
            nk[r] = cnt;
        }
        free(idx);
    }
    return failed ? -2 : 0;
}

int xo_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
