// xs_kernels.hip — gfx950 (MI355X, CDNA4) kernels of the k-mer x filter probe path.
//
// Pipeline of one query call (reads already in HBM):
//   strands  : normalised forward strand + reverse-complement strand of every
//              read, written once (byte tables in LDS)          [HBM stream]
//   units    : per-read sampled k-mer count and #units (segments of kSegKmers)
//   scan     : exclusive scan of #units (hipCUB)
//   scatter  : unit -> read map; zero hit rows of split reads
//   probe    : one wavefront per unit, one lane per k-mer: canonical k-mer
//              from the two strand windows, h x XXH64 (or XXH3-64 + LCG for
//              rbloom), h random 16-byte row gathers from the bank, AND, and
//              per-doc ballot/popcount counting into per-wave LDS counters
//                                                   [HBM random-read bound]
//   reduce   : per-block partial totals -> per-doc totals (u64)
//
// Reference semantics restated (see oracle/xs_oracle.c for the CPU version):
//   cobs_index.Search.search(query, step)  probabilistic_filter_model.py:227
//   rbloom `kmer in bf`                    probabilistic_single_filter_model.py:122-124
#include <hipcub/hipcub.hpp>

#include "xs_internal.h"

// v_writelane_b32: this clang exposes only readlane as a builtin; bind the
// LLVM intrinsic directly.
extern "C" __device__ int xs_writelane_i32(int value, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

namespace xs {

// ------------------------------------------------------------------ hashing
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull;
constexpr uint64_t P64_2 = 0xC2B2AE3D27D4EB4Full;
constexpr uint64_t P64_3 = 0x165667B19E3779F9ull;
constexpr uint64_t P64_4 = 0x85EBCA77C2B2AE63ull;
constexpr uint64_t P64_5 = 0x27D4EB2F165667C5ull;

// First 64 bytes of the XXH3 default secret, as little-endian words.
constexpr uint64_t kS64[8] = {
    0xbe4ba423396cfeb8ull, 0x1cad21f72c81017cull, 0xdb979083e96dd4deull, 0x1f67b3b7a4a44072ull,
    0x78e5c0cc4ee679cbull, 0x2172ffcc7dd05a82ull, 0x8e2443f7744608b8ull, 0x4c263a81e69035e0ull,
};
constexpr uint32_t kS32_0 = 0x396cfeb8u, kS32_1 = 0xbe4ba423u;

// 128-bit LCG of the rbloom restatement (oracle/xs_oracle.c: xo_bloom_indexes).
constexpr uint64_t kLcgMh = 0x2360ED051FC65DA4ull, kLcgMl = 0x4385DF649FCCF645ull;
constexpr uint64_t kLcgCh = 0x5851F42D4C957F2Dull, kLcgCl = 0x14057B7EF767814Full;

__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

__device__ __forceinline__ uint64_t xxh64_round0(uint64_t in) {
    return rotl64(in * P64_2, 31) * P64_1;
}
__device__ __forceinline__ uint64_t xxh64_round(uint64_t acc, uint64_t in) {
    return rotl64(acc + in * P64_2, 31) * P64_1;
}
__device__ __forceinline__ uint64_t xxh64_avalanche(uint64_t h) {
    h ^= h >> 33; h *= P64_2;
    h ^= h >> 29; h *= P64_3;
    return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t xxh3_avalanche(uint64_t h) {
    h ^= h >> 37; h *= 0x165667919E3779F9ull;
    return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t fold64(uint64_t a, uint64_t b) {
    return (a * b) ^ __umul64hi(a, b);
}
// x mod d with m = floor((2^64-1)/d): q <= x/d < q + 3.
__device__ __forceinline__ uint64_t fastmod(uint64_t x, uint64_t d, uint64_t m) {
    uint64_t r = x - __umul64hi(x, m) * d;
    r = r >= d ? r - d : r;
    return r >= d ? r - d : r;
}

// Canonical k-mer, held as 8 little-endian dwords (bytes >= k are zero) + a
// zero guard word.
struct Kmer {
    uint32_t w[9];
};

__device__ __forceinline__ uint64_t kmer_u64(const Kmer& c, uint32_t off) {
    // 8 bytes at byte offset `off` (compile-time constant on the fast paths).
    const uint32_t i = off >> 2, sh = off & 3;
    const uint32_t lo = __builtin_amdgcn_alignbyte(c.w[i + 1], c.w[i], sh);
    const uint32_t hi = __builtin_amdgcn_alignbyte(c.w[i + 2], c.w[i + 1], sh);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ uint32_t kmer_u32(const Kmer& c, uint32_t off) {
    const uint32_t i = off >> 2, sh = off & 3;
    return __builtin_amdgcn_alignbyte(c.w[i + 1], c.w[i], sh);
}
__device__ __forceinline__ uint32_t kmer_u8(const Kmer& c, uint32_t off) {
    return (c.w[off >> 2] >> ((off & 3) * 8)) & 0xFF;
}

// Window of k bytes at byte offset `off` of `base`, as dwords (tail zeroed).
template <int KT>
__device__ __forceinline__ void load_window(const uint8_t* base, uint64_t off, uint32_t k,
                                            uint32_t (&w)[8]) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(base + (off & ~3ull));
    const uint32_t sh = (uint32_t)(off & 3);
    const uint32_t nw = KT ? (KT + 3) / 4 : (k + 3) / 4;
    uint32_t raw[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) raw[i] = (i <= (int)nw) ? p[i] : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t v = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh);
        const int kk = KT ? KT : (int)k;
        const int valid = kk - 4 * i;  // bytes of word i that belong to the k-mer
        v = valid >= 4 ? v : (valid <= 0 ? 0u : (v & ((1u << (8 * valid)) - 1u)));
        w[i] = v;
    }
}

// Byte-lexicographic min of the forward and reverse-complement windows.
__device__ __forceinline__ void canonical_select(const uint32_t (&f)[8], const uint32_t (&r)[8],
                                                 Kmer& c) {
    bool decided = false, rc_less = false;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t a = __builtin_bswap32(f[i]), b = __builtin_bswap32(r[i]);
        const bool diff = a != b;
        rc_less = (!decided && diff) ? (b < a) : rc_less;
        decided = decided || diff;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) c.w[i] = rc_less ? r[i] : f[i];
    c.w[8] = 0;
}

// Seed-independent part of XXH64 over a short (< 32 byte) input.
struct Xxh64Pre {
    uint64_t r8[4];
    uint64_t r4;
    uint64_t rb[3];
};

template <int KT>
__device__ __forceinline__ void xxh64_pre(const Kmer& c, uint32_t k, Xxh64Pre& p) {
    const uint32_t kk = KT ? KT : k;
    const uint32_t n8 = kk >> 3;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i)
        p.r8[i] = i < n8 ? xxh64_round0((uint64_t)c.w[2 * i] | ((uint64_t)c.w[2 * i + 1] << 32)) : 0;
    const uint32_t o4 = n8 * 8;
    p.r4 = (kk & 4) ? (uint64_t)c.w[o4 >> 2] * P64_1 : 0;
    const uint32_t ob = o4 + (kk & 4);
#pragma unroll
    for (uint32_t i = 0; i < 3; ++i) p.rb[i] = i < (kk & 3) ? (uint64_t)kmer_u8(c, ob + i) * P64_5 : 0;
}

template <int KT>
__device__ __forceinline__ uint64_t xxh64_seed(const Kmer& c, const Xxh64Pre& p, uint32_t k,
                                               uint64_t seed) {
    const uint32_t kk = KT ? KT : k;
    if (kk >= 32) {  // one 32-byte stripe (k == 32)
        uint64_t v1 = xxh64_round(seed + P64_1 + P64_2, (uint64_t)c.w[0] | ((uint64_t)c.w[1] << 32));
        uint64_t v2 = xxh64_round(seed + P64_2, (uint64_t)c.w[2] | ((uint64_t)c.w[3] << 32));
        uint64_t v3 = xxh64_round(seed, (uint64_t)c.w[4] | ((uint64_t)c.w[5] << 32));
        uint64_t v4 = xxh64_round(seed - P64_1, (uint64_t)c.w[6] | ((uint64_t)c.w[7] << 32));
        uint64_t h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = (h ^ xxh64_round0(v1)) * P64_1 + P64_4;
        h = (h ^ xxh64_round0(v2)) * P64_1 + P64_4;
        h = (h ^ xxh64_round0(v3)) * P64_1 + P64_4;
        h = (h ^ xxh64_round0(v4)) * P64_1 + P64_4;
        h += 32;
        return xxh64_avalanche(h);
    }
    uint64_t h = seed + P64_5 + kk;
    const uint32_t n8 = kk >> 3;
#pragma unroll
    for (uint32_t i = 0; i < 3; ++i)
        if (i < n8) h = rotl64(h ^ p.r8[i], 27) * P64_1 + P64_4;
    if (kk & 4) h = rotl64(h ^ p.r4, 23) * P64_2 + P64_3;
#pragma unroll
    for (uint32_t i = 0; i < 3; ++i)
        if (i < (kk & 3)) h = rotl64(h ^ p.rb[i], 11) * P64_1;
    return xxh64_avalanche(h);
}

// XXH3-64, default secret, seed 0, for 1 <= len <= 32.
template <int KT>
__device__ __forceinline__ uint64_t xxh3_kmer(const Kmer& c, uint32_t k) {
    const uint32_t len = KT ? KT : k;
    if (len > 16) {
        uint64_t acc = len * P64_1;
        acc += fold64(kmer_u64(c, 0) ^ kS64[0], kmer_u64(c, 8) ^ kS64[1]);
        acc += fold64(kmer_u64(c, len - 16) ^ kS64[2], kmer_u64(c, len - 8) ^ kS64[3]);
        return xxh3_avalanche(acc);
    }
    if (len > 8) {
        const uint64_t lo = kmer_u64(c, 0) ^ (kS64[3] ^ kS64[4]);
        const uint64_t hi = kmer_u64(c, len - 8) ^ (kS64[5] ^ kS64[6]);
        return xxh3_avalanche(len + __builtin_bswap64(lo) + hi + fold64(lo, hi));
    }
    if (len >= 4) {
        const uint64_t in64 = (uint64_t)kmer_u32(c, len - 4) + ((uint64_t)kmer_u32(c, 0) << 32);
        uint64_t x = in64 ^ (kS64[1] ^ kS64[2]);
        x ^= rotl64(x, 49) ^ rotl64(x, 24);
        x *= 0x9FB21C651E98DF25ull;
        x ^= (x >> 35) + len;
        x *= 0x9FB21C651E98DF25ull;
        return x ^ (x >> 28);
    }
    const uint32_t comb = (kmer_u8(c, 0) << 16) | (kmer_u8(c, len >> 1) << 24) |
                          kmer_u8(c, len - 1) | (len << 8);
    return xxh64_avalanche((uint64_t)comb ^ (uint64_t)(kS32_0 ^ kS32_1));
}

// ------------------------------------------------------------------ strands
__device__ __forceinline__ void strand_tables(int mode, uint8_t* tf, uint8_t* tr) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        uint8_t f = (uint8_t)i, r = (uint8_t)i;
        if (mode == kStrandCobs) {
            const uint8_t u = (uint8_t)(i & 0xDF);
            const bool base = (i >= 'A' && i <= 'Z') || (i >= 'a' && i <= 'z');
            f = (base && (u == 'A' || u == 'C' || u == 'G' || u == 'T')) ? u : (uint8_t)'N';
            r = f == 'A' ? 'T' : f == 'T' ? 'A' : f == 'C' ? 'G' : f == 'G' ? 'C' : 'N';
        } else {
            // Biopython ambiguous_dna_complement, both cases; others unchanged.
            const bool lower = i >= 'a' && i <= 'z';
            const uint8_t u = lower ? (uint8_t)(i - 32) : (uint8_t)i;
            uint8_t m = 0;
            switch (u) {
                case 'A': m = 'T'; break; case 'T': m = 'A'; break;
                case 'C': m = 'G'; break; case 'G': m = 'C'; break;
                case 'M': m = 'K'; break; case 'K': m = 'M'; break;
                case 'R': m = 'Y'; break; case 'Y': m = 'R'; break;
                case 'W': m = 'W'; break; case 'S': m = 'S'; break;
                case 'V': m = 'B'; break; case 'B': m = 'V'; break;
                case 'H': m = 'D'; break; case 'D': m = 'H'; break;
                case 'X': m = 'X'; break; case 'N': m = 'N'; break;
                default: break;
            }
            if (m) r = lower ? (uint8_t)(m + 32) : m;
        }
        tf[i] = f;
        tr[i] = r;
    }
}

constexpr uint64_t kStrandChunk = 4096;

__global__ void __launch_bounds__(256) strands_kernel(const uint8_t* __restrict__ seqs,
                                                      const uint64_t* __restrict__ offs,
                                                      uint64_t n, int mode,
                                                      uint8_t* __restrict__ fwd,
                                                      uint8_t* __restrict__ rc) {
    __shared__ uint8_t tf[256], tr[256];
    __shared__ uint64_t s_r0;
    strand_tables(mode, tf, tr);
    const uint64_t lo = offs[0], hi = offs[n];
    const uint64_t nchunks = (hi - lo + kStrandChunk - 1) / kStrandChunk;
    for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
        const uint64_t start = lo + ch * kStrandChunk;
        const uint64_t end = min(start + kStrandChunk, hi);
        __syncthreads();
        if (threadIdx.x == 0) {  // last read r with offs[r] <= start
            uint64_t a = 0, b = n;  // offs[a] <= start < offs[b]
            while (b - a > 1) {
                const uint64_t m = (a + b) >> 1;
                if (offs[m] <= start) a = m; else b = m;
            }
            s_r0 = a;
        }
        __syncthreads();
        uint64_t r = s_r0;
        uint64_t re = offs[r + 1];
        for (uint64_t i = start + threadIdx.x; i < end; i += blockDim.x) {
            while (re <= i) { ++r; re = offs[r + 1]; }
            const uint8_t x = seqs[i];
            if (fwd) fwd[i] = tf[x];
            rc[offs[r] + re - 1 - i] = tr[x];
        }
    }
}

// ------------------------------------------------------------------ units
__device__ __forceinline__ uint64_t num_kmers(uint64_t len, uint32_t k, uint32_t step) {
    return len >= k ? (len - k + step) / step : 0;  // ceil((len-k+1)/step)
}

__global__ void units_kernel(const uint64_t* __restrict__ offs, uint64_t n, uint32_t k,
                             uint32_t step, uint64_t* __restrict__ nk_out,
                             uint64_t* __restrict__ nseg) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t nk = num_kmers(offs[r + 1] - offs[r], k, step);
        if (nk_out) nk_out[r] = nk;
        nseg[r] = (nk + kSegKmers - 1) / kSegKmers;
    }
}

__global__ void scatter_units_kernel(const uint64_t* __restrict__ nseg,
                                     const uint64_t* __restrict__ unit_ofs, uint64_t n,
                                     uint32_t* __restrict__ unit_read, uint64_t* n_units,
                                     uint32_t* __restrict__ hits_zero, uint64_t D) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = nseg[r], b = unit_ofs[r];
        for (uint64_t u = 0; u < s; ++u) unit_read[b + u] = (uint32_t)r;
        // rows the probe does not store whole: no k-mers (never visited) or
        // several units (accumulated atomically)
        if (s != 1 && hits_zero)
            for (uint64_t d = 0; d < D; ++d) hits_zero[r * D + d] = 0;
        if (r == n - 1) *n_units = b + s;
    }
}

// ------------------------------------------------------------------ counting
// Adds the per-doc bit counts of this tile's 64 masks (one per lane) for docs
// [cd0, cd0 + nd) (nd <= 128) to the wave's LDS counters.  Doc cd0+32q+b is
// bit b of mask word q.  A ballot per doc transposes the 64 masks; its
// popcount is that doc's count for the tile.
__device__ __forceinline__ void count_chunk(const uint4& m, uint32_t nd, int lane, uint32_t* acc) {
    uint32_t tv0 = 0, tv1 = 0;
    const uint32_t w[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if ((uint32_t)(q * 32) >= nd) break;
#pragma unroll
        for (int b = 0; b < 32; ++b) {
            const uint32_t bi = q * 32 + b;
            if (bi >= nd) break;
            const int pc = __popcll(__ballot((w[q] >> b) & 1u));
            if (bi < 64) tv0 = xs_writelane_i32(pc, bi, tv0);
            else tv1 = xs_writelane_i32(pc, bi - 64, tv1);
        }
    }
    if ((uint32_t)lane < nd) acc[lane] += tv0;
    if ((uint32_t)lane + 64 < nd) acc[64 + lane] += tv1;
}

__device__ __forceinline__ uint4 and4(uint4 a, uint4 b) {
    return make_uint4(a.x & b.x, a.y & b.y, a.z & b.z, a.w & b.w);
}

// ------------------------------------------------------------------ COBS probe
// One wavefront per unit (<= kSegKmers k-mers of one read), one lane per k-mer.
template <int KT, int HT>
__global__ void __launch_bounds__(kProbeThreads) probe_cobs_kernel(ReadView rv, CobsView bv,
                                                                   uint32_t* __restrict__ hits,
                                                                   uint64_t* __restrict__ partials,
                                                                   uint32_t dpad) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int wpb = blockDim.x >> 6;
    uint32_t* acc = smem + (size_t)wid * 2 * dpad;
    uint32_t* tot = acc + dpad;
    __shared__ uint64_t s_kmers[kProbeThreads / kWave];
    for (uint32_t d = lane; d < 2 * dpad; d += 64) acc[d] = 0;

    const uint32_t k = KT ? KT : rv.k;
    const uint32_t h = HT ? HT : bv.h;
    const uint32_t step = rv.step;
    const uint64_t D = bv.D;
    const uint64_t U = *rv.n_units;
    uint64_t kmer_total = 0;

    for (uint64_t u = (uint64_t)blockIdx.x * wpb + wid; u < U; u += (uint64_t)gridDim.x * wpb) {
        const uint32_t r = rv.unit_read[u];
        const uint64_t seg = u - rv.unit_ofs[r];
        const uint64_t o0 = rv.offs[r];
        const uint64_t len = rv.offs[r + 1] - o0;
        const uint64_t nk = num_kmers(len, k, step);
        const uint64_t t0 = seg * kSegKmers;
        const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
        const bool whole = nk <= kSegKmers;
        kmer_total += cnt;

        for (uint32_t tb = 0; tb < cnt; tb += 64) {
            const bool act = tb + lane < cnt;
            uint64_t hv[HT ? HT : kMaxHashes];
            if (act) {
                const uint64_t p = (t0 + tb + lane) * step;  // k-mer start within the read
                uint32_t f[8], q[8];
                load_window<KT>(rv.fwd, o0 + p, k, f);
                load_window<KT>(rv.rc, o0 + (len - p - k), k, q);
                Kmer c;
                canonical_select(f, q, c);
                Xxh64Pre pre;
                xxh64_pre<KT>(c, k, pre);
#pragma unroll
                for (uint32_t j = 0; j < (HT ? HT : kMaxHashes); ++j)
                    if (j < h) hv[j] = xxh64_seed<KT>(c, pre, k, j);
            }
            for (uint32_t g = 0; g < bv.G; ++g) {
                const GroupDesc gd = bv.groups[g];
                const uint64_t doc0 = (uint64_t)g * 8 * bv.page;
                const uint64_t dlim = min(D, doc0 + 8 * bv.page);
                uint64_t ro[HT ? HT : kMaxHashes];
#pragma unroll
                for (uint32_t j = 0; j < (HT ? HT : kMaxHashes); ++j)
                    if (j < h) ro[j] = act ? gd.base + fastmod(hv[j], gd.sig, gd.magic) * bv.pitch : 0;
                for (uint32_t cc = 0; cc < bv.nchunks; ++cc) {
                    const uint64_t cd0 = doc0 + (uint64_t)cc * 128;
                    if (cd0 >= dlim) break;
                    uint4 m = make_uint4(0u, 0u, 0u, 0u);
                    if (act) {
                        m = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
                        for (uint32_t j = 0; j < (HT ? HT : kMaxHashes); ++j)
                            if (j < h)
                                m = and4(m, *reinterpret_cast<const uint4*>(bv.rows + ro[j] + cc * 16));
                    }
                    count_chunk(m, (uint32_t)min((uint64_t)128, dlim - cd0), lane, acc + cd0);
                }
            }
        }
        // unit done: move counters to the hit matrix and the wave totals
        for (uint64_t d = lane; d < D; d += 64) {
            const uint32_t v = acc[d];
            acc[d] = 0;
            tot[d] += v;
            if (hits) {
                if (whole) hits[(uint64_t)r * D + d] = v;
                else if (v) atomicAdd(&hits[(uint64_t)r * D + d], v);
            }
        }
    }
    if (partials) {
        if (lane == 0) s_kmers[wid] = kmer_total;
        __syncthreads();
        uint64_t* out = partials + (uint64_t)blockIdx.x * (D + 1);
        for (uint64_t d = threadIdx.x; d < D; d += blockDim.x) {
            uint64_t s = 0;
            for (int w = 0; w < wpb; ++w) s += smem[(size_t)w * 2 * dpad + dpad + d];
            out[d] = s;
        }
        if (threadIdx.x == 0) {
            uint64_t s = 0;
            for (int w = 0; w < wpb; ++w) s += s_kmers[w];
            out[D] = s;
        }
    }
}

// ------------------------------------------------------------------ rbloom probe
template <int KT>
__device__ __forceinline__ bool bloom_member(const Kmer& c, uint32_t k, const BloomView& bv) {
    const uint64_t hsh = xxh3_kmer<KT>(c, k);
    uint64_t sl = hsh, sh = 0;
    bool in = true;
    for (uint32_t j = 0; j < bv.K; ++j) {
        const uint64_t p = sl * kLcgMl;
        const uint64_t nl = p + kLcgCl;
        const uint64_t carry = nl < p;
        const uint64_t nh = sh * kLcgMl + sl * kLcgMh + __umul64hi(sl, kLcgMl) + kLcgCh + carry;
        sl = nl;
        sh = nh;
        const uint64_t idx = fastmod(nh, bv.mbits, bv.magic);
        in = in && ((bv.bits[idx >> 5] >> (idx & 31)) & 1u);
    }
    return in;
}

template <int KT>
__global__ void __launch_bounds__(kProbeThreads) probe_bloom_kernel(ReadView rv, BloomView bv,
                                                                    uint32_t* __restrict__ hits,
                                                                    uint64_t* __restrict__ partials) {
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int wpb = blockDim.x >> 6;
    __shared__ uint64_t s_hits[kProbeThreads / kWave], s_kmers[kProbeThreads / kWave];
    const uint32_t k = KT ? KT : rv.k;
    const uint32_t step = rv.step;
    const uint64_t U = *rv.n_units;
    uint64_t hit_total = 0, kmer_total = 0;

    for (uint64_t u = (uint64_t)blockIdx.x * wpb + wid; u < U; u += (uint64_t)gridDim.x * wpb) {
        const uint32_t r = rv.unit_read[u];
        const uint64_t seg = u - rv.unit_ofs[r];
        const uint64_t o0 = rv.offs[r];
        const uint64_t len = rv.offs[r + 1] - o0;
        const uint64_t nk = num_kmers(len, k, step);
        const uint64_t t0 = seg * kSegKmers;
        const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
        uint32_t c_unit = 0;
        for (uint32_t tb = 0; tb < cnt; tb += 64) {
            bool in = false;
            if (tb + lane < cnt) {
                const uint64_t p = (t0 + tb + lane) * step;
                uint32_t f[8], q[8];
                load_window<KT>(rv.fwd, o0 + p, k, f);
                load_window<KT>(rv.rc, o0 + (len - p - k), k, q);
                Kmer c;
                canonical_select(f, q, c);
                in = bloom_member<KT>(c, k, bv);
            }
            c_unit += (uint32_t)__popcll(__ballot(in));
        }
        kmer_total += cnt;
        hit_total += c_unit;
        if (hits && lane == 0) {
            if (nk <= kSegKmers) hits[r] = c_unit;
            else if (c_unit) atomicAdd(&hits[r], c_unit);
        }
    }
    if (partials) {
        if (lane == 0) { s_hits[wid] = hit_total; s_kmers[wid] = kmer_total; }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t a = 0, b = 0;
            for (int w = 0; w < wpb; ++w) { a += s_hits[w]; b += s_kmers[w]; }
            partials[blockIdx.x * 2ull] = a;
            partials[blockIdx.x * 2ull + 1] = b;
        }
    }
}

// ------------------------------------------------------------------ builders
// Sets bit (doc - group start) of the h rows of every k-mer (step 1) of every
// record: cobs classic_construct_list / compact_construct_list restated.
template <int KT, int HT>
__global__ void __launch_bounds__(kProbeThreads) build_cobs_kernel(ReadView rv,
                                                                   const uint32_t* __restrict__ rec_doc,
                                                                   CobsView bv, uint32_t* rows) {
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int wpb = blockDim.x >> 6;
    const uint32_t k = KT ? KT : rv.k;
    const uint32_t h = HT ? HT : bv.h;
    const uint64_t U = *rv.n_units;
    for (uint64_t u = (uint64_t)blockIdx.x * wpb + wid; u < U; u += (uint64_t)gridDim.x * wpb) {
        const uint32_t r = rv.unit_read[u];
        const uint64_t seg = u - rv.unit_ofs[r];
        const uint64_t o0 = rv.offs[r];
        const uint64_t len = rv.offs[r + 1] - o0;
        const uint64_t nk = num_kmers(len, k, 1);
        const uint64_t t0 = seg * kSegKmers;
        const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
        const uint64_t doc = rec_doc[r];
        const uint64_t g = doc / (8 * bv.page), bit = doc % (8 * bv.page);
        if (doc >= bv.D) continue;
        const GroupDesc gd = bv.groups[g];
        for (uint32_t tb = 0; tb < cnt; tb += 64) {
            if (tb + lane >= cnt) continue;
            const uint64_t p = t0 + tb + lane;
            uint32_t f[8], q[8];
            load_window<KT>(rv.fwd, o0 + p, k, f);
            load_window<KT>(rv.rc, o0 + (len - p - k), k, q);
            Kmer c;
            canonical_select(f, q, c);
            Xxh64Pre pre;
            xxh64_pre<KT>(c, k, pre);
            for (uint32_t j = 0; j < h; ++j) {
                const uint64_t row = fastmod(xxh64_seed<KT>(c, pre, k, j), gd.sig, gd.magic);
                const uint64_t byte = gd.base + row * bv.pitch + (bit >> 3);
                atomicOr(&rows[byte >> 2], 1u << (bit & 31));
            }
        }
    }
}

template <int KT>
__global__ void __launch_bounds__(kProbeThreads) build_bloom_kernel(ReadView rv, BloomView bv,
                                                                    uint32_t* bits) {
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int wpb = blockDim.x >> 6;
    const uint32_t k = KT ? KT : rv.k;
    const uint64_t U = *rv.n_units;
    for (uint64_t u = (uint64_t)blockIdx.x * wpb + wid; u < U; u += (uint64_t)gridDim.x * wpb) {
        const uint32_t r = rv.unit_read[u];
        const uint64_t seg = u - rv.unit_ofs[r];
        const uint64_t o0 = rv.offs[r];
        const uint64_t len = rv.offs[r + 1] - o0;
        const uint64_t nk = num_kmers(len, k, 1);
        const uint64_t t0 = seg * kSegKmers;
        const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
        for (uint32_t tb = 0; tb < cnt; tb += 64) {
            if (tb + lane >= cnt) continue;
            const uint64_t p = t0 + tb + lane;
            uint32_t f[8], q[8];
            load_window<KT>(rv.fwd, o0 + p, k, f);
            load_window<KT>(rv.rc, o0 + (len - p - k), k, q);
            Kmer c;
            canonical_select(f, q, c);
            uint64_t sl = xxh3_kmer<KT>(c, k), sh = 0;
            for (uint32_t j = 0; j < bv.K; ++j) {
                const uint64_t pm = sl * kLcgMl;
                const uint64_t nl = pm + kLcgCl;
                const uint64_t carry = nl < pm;
                sh = sh * kLcgMl + sl * kLcgMh + __umul64hi(sl, kLcgMl) + kLcgCh + carry;
                sl = nl;
                const uint64_t idx = fastmod(sh, bv.mbits, bv.magic);
                atomicOr(&bits[idx >> 5], 1u << (idx & 31));
            }
        }
    }
}

// ------------------------------------------------------------------ misc
__global__ void reduce_partials_kernel(const uint64_t* __restrict__ partials, int blocks,
                                       uint64_t cols, uint64_t* __restrict__ totals) {
    for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < cols;
         c += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t s = 0;
        for (int b = 0; b < blocks; ++b) s += partials[(uint64_t)b * cols + c];
        totals[c] = s;
    }
}

__global__ void repack_kernel(const uint8_t* __restrict__ src, uint64_t src_pitch,
                              uint8_t* __restrict__ dst, uint64_t dst_pitch, uint64_t rows,
                              uint64_t copy_bytes) {
    for (uint64_t row = blockIdx.x * (uint64_t)blockDim.y + threadIdx.y; row < rows;
         row += (uint64_t)gridDim.x * blockDim.y) {
        for (uint64_t b = threadIdx.x; b < dst_pitch; b += blockDim.x)
            dst[row * dst_pitch + b] = b < copy_bytes ? src[row * src_pitch + b] : 0;
    }
}

__global__ void mlst_sum_kernel(const uint32_t* __restrict__ hits,
                                const uint32_t* __restrict__ seq_of_chunk, uint64_t n_chunks,
                                uint64_t D, uint32_t threshold, unsigned long long* scores) {
    const uint64_t total = n_chunks * D;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = hits[i];
        if (v > threshold) {
            const uint64_t c = i / D, d = i - c * D;
            atomicAdd(&scores[(uint64_t)seq_of_chunk[c] * D + d], (unsigned long long)v);
        }
    }
}

// ------------------------------------------------------------------ launchers
static inline int grid_for(uint64_t work, int per_block, int cap) {
    uint64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > (uint64_t)cap) g = cap;
    return (int)g;
}

hipError_t launch_strands(const uint8_t* seqs, const uint64_t* offs, uint64_t n, uint64_t nbytes,
                          int mode, uint8_t* fwd_out, uint8_t* rc_out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int grid = grid_for(nbytes / kStrandChunk + 1, 1, 4096);
    strands_kernel<<<grid, 256, 0, s>>>(seqs, offs, n, mode, fwd_out, rc_out);
    return hipGetLastError();
}

hipError_t launch_units(const uint64_t* offs, uint64_t n, uint32_t k, uint32_t step,
                        uint64_t* nk_out, uint64_t* nseg, hipStream_t s) {
    if (n == 0) return hipSuccess;
    units_kernel<<<grid_for(n, 256, 4096), 256, 0, s>>>(offs, n, k, step, nk_out, nseg);
    return hipGetLastError();
}

size_t scan_temp_bytes(uint64_t n) {
    size_t bytes = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (int)n);
    return bytes;
}

hipError_t launch_scan(void* temp, size_t temp_bytes, const uint64_t* in, uint64_t* out,
                       uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)n, s);
}

hipError_t launch_scatter_units(const uint64_t* nseg, const uint64_t* unit_ofs, uint64_t n,
                                uint32_t* unit_read, uint64_t* n_units, uint32_t* hits_zero,
                                uint64_t D, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(n_units, 0, sizeof(uint64_t), s);
    scatter_units_kernel<<<grid_for(n, 256, 4096), 256, 0, s>>>(nseg, unit_ofs, n, unit_read,
                                                               n_units, hits_zero, D);
    return hipGetLastError();
}

int probe_blocks(uint64_t D, int* waves_per_block, size_t* lds_bytes) {
    const uint64_t dpad = (D + 127) / 128 * 128;
    int wpb = kProbeThreads / kWave;
    while (wpb > 1 && (uint64_t)wpb * 2 * dpad * 4 > kLdsBudget) wpb >>= 1;
    if ((uint64_t)wpb * 2 * dpad * 4 > kLdsBudget) return -1;
    *waves_per_block = wpb;
    *lds_bytes = (size_t)wpb * 2 * dpad * 4;
    return 0;
}

// 256 CUs x 8 blocks of 4 waves keep 32 waves per CU in flight.
constexpr int kProbeGridCap = 256 * 8;

template <int KT, int HT>
static hipError_t launch_cobs_t(const ReadView& rv, const CobsView& bv, uint32_t* hits,
                                uint64_t* partials, int blocks, int wpb, size_t lds,
                                uint32_t dpad, hipStream_t s) {
    probe_cobs_kernel<KT, HT><<<blocks, wpb * kWave, lds, s>>>(rv, bv, hits, partials, dpad);
    return hipGetLastError();
}

hipError_t launch_probe_cobs(const ReadView& rv, const CobsView& bv, uint32_t* hits,
                             uint64_t* partials, int blocks, hipStream_t s) {
    int wpb;
    size_t lds;
    if (probe_blocks(bv.D, &wpb, &lds) != 0) return hipErrorInvalidValue;
    const uint32_t dpad = (uint32_t)((bv.D + 127) / 128 * 128);
    if (rv.k == 21 && bv.h == 7) return launch_cobs_t<21, 7>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
    if (rv.k == 31 && bv.h == 1) return launch_cobs_t<31, 1>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
    if (rv.k == 21 && bv.h == 1) return launch_cobs_t<21, 1>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
    if (rv.k == 31 && bv.h == 7) return launch_cobs_t<31, 7>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
    return launch_cobs_t<0, 0>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
}

hipError_t launch_probe_bloom(const ReadView& rv, const BloomView& bv, uint32_t* hits,
                              uint64_t* partials, int blocks, hipStream_t s) {
    if (rv.k == 21) probe_bloom_kernel<21><<<blocks, kProbeThreads, 0, s>>>(rv, bv, hits, partials);
    else probe_bloom_kernel<0><<<blocks, kProbeThreads, 0, s>>>(rv, bv, hits, partials);
    return hipGetLastError();
}

hipError_t launch_reduce_partials(const uint64_t* partials, int blocks, uint64_t cols,
                                  uint64_t* totals, hipStream_t s) {
    reduce_partials_kernel<<<grid_for(cols, 256, 1024), 256, 0, s>>>(partials, blocks, cols, totals);
    return hipGetLastError();
}

hipError_t launch_build_cobs(const ReadView& rv, const uint32_t* rec_doc, const CobsView& bv,
                             uint32_t* rows_mut, int blocks, hipStream_t s) {
    if (rv.k == 21 && bv.h == 7)
        build_cobs_kernel<21, 7><<<blocks, kProbeThreads, 0, s>>>(rv, rec_doc, bv, rows_mut);
    else
        build_cobs_kernel<0, 0><<<blocks, kProbeThreads, 0, s>>>(rv, rec_doc, bv, rows_mut);
    return hipGetLastError();
}

hipError_t launch_build_bloom(const ReadView& rv, const BloomView& bv, uint32_t* bits_mut,
                              int blocks, hipStream_t s) {
    if (rv.k == 21) build_bloom_kernel<21><<<blocks, kProbeThreads, 0, s>>>(rv, bv, bits_mut);
    else build_bloom_kernel<0><<<blocks, kProbeThreads, 0, s>>>(rv, bv, bits_mut);
    return hipGetLastError();
}

hipError_t launch_repack(const uint8_t* src, uint64_t src_pitch, uint8_t* dst, uint64_t dst_pitch,
                         uint64_t rows, uint64_t copy_bytes, hipStream_t s) {
    if (rows == 0) return hipSuccess;
    dim3 block(64, 4);
    repack_kernel<<<grid_for(rows, 4, 16384), block, 0, s>>>(src, src_pitch, dst, dst_pitch, rows,
                                                            copy_bytes);
    return hipGetLastError();
}

hipError_t launch_mlst_sum(const uint32_t* hits, const uint32_t* seq_of_chunk, uint64_t n_chunks,
                           uint64_t D, uint32_t threshold, unsigned long long* scores,
                           hipStream_t s) {
    if (n_chunks == 0 || D == 0) return hipSuccess;
    mlst_sum_kernel<<<grid_for(n_chunks * D, 256, 4096), 256, 0, s>>>(hits, seq_of_chunk, n_chunks,
                                                                      D, threshold, scores);
    return hipGetLastError();
}

}  // namespace xs
