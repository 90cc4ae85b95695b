// xs_kernels.hip — gfx950 (MI355X, CDNA4) kernels of the k-mer x filter probe path.
//
// Pipeline of one query call (reads already in HBM):
//   units    : per-read sampled k-mer count and #units (segments of kSegKmers)
//   scan     : exclusive scan of #units (hipCUB)
//   scatter  : unit -> read map; zero hit rows of split reads
//   probe    : one wavefront per unit, one lane per k-mer: canonical k-mer
//              built in registers from one read window, h x XXH64 (or XXH3-64 + LCG for
//              rbloom), h random 16-byte row gathers from the bank, AND, and
//              per-doc ballot/popcount counting into per-wave LDS counters
//                                                   [HBM random-read bound]
//   reduce   : per-block partial totals -> per-doc totals (u64)
//
// Reference semantics restated (see oracle/xs_oracle.c for the CPU version):
//   cobs_index.Search.search(query, step)  probabilistic_filter_model.py:227
//   rbloom `kmer in bf`                    probabilistic_single_filter_model.py:122-124
#include <hipcub/hipcub.hpp>

#include <atomic>
#include <cstdlib>

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

// ------------------------------------------------------------------ k-mer assembly
// A k-mer is built in registers straight from the read bytes: one unaligned
// k-byte window load, byte normalisation (COBS) and the reverse complement by
// a byte-table permute, then the byte-lexicographic min of the two strands.
//
// COBS (species, MLST): ACGT/acgt -> ACGT, any other byte -> N (restated
// canonicalisation; oracle/xs_oracle.c xo_canonical_cobs).
// rbloom (genus): bytes kept as they are, complement = Biopython's
// ambiguous_dna_complement in both cases, other bytes unchanged
// (probabilistic_single_filter_model.py:161-180; xo_canonical_bio).

// 0x80 in every byte of v that is zero (exact, no carries between bytes).
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {
    return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);
}
__device__ __forceinline__ uint32_t bytes_equal(uint32_t x, uint32_t c) { return zero_bytes(x ^ (c * 0x01010101u)); }

// COBS normalisation of 4 bytes.  (b & 0xDF) is one of A/C/G/T only for
// A/C/G/T/a/c/g/t, so the upper-cased test is exact.
__device__ __forceinline__ uint32_t cobs_norm4(uint32_t x) {
    const uint32_t u = x & 0xDFDFDFDFu;
    const uint32_t ok = bytes_equal(u, 'A') | bytes_equal(u, 'C') | bytes_equal(u, 'G') | bytes_equal(u, 'T');
    const uint32_t m = (ok >> 7) * 0xFFu;
    return (u & m) | (0x4E4E4E4Eu & ~m);
}

// Complement of bytes in {A, C, G, T, N, 0}: b & 7 is 1, 3, 7, 4, 6, 0 for
// them, and v_perm_b32 looks the complement up in an 8-byte table
// {0, 'T', -, 'G', 'A', -, 'N', 'C'} (0 stays 0: padding).
__device__ __forceinline__ uint32_t comp4(uint32_t f) {
    return __builtin_amdgcn_perm(0x434E0041u, 0x47005400u, f & 0x07070707u);
}

// Biopython ambiguous_dna_complement of one byte, both cases; other bytes unchanged.
__device__ __forceinline__ uint32_t bio_comp_byte(uint32_t b) {
    const uint32_t lower = (b >= 'a' && b <= 'z') ? 32u : 0u;
    const uint32_t u = b - lower;
    uint32_t m = 0;
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
    return m ? m + lower : b;
}

// Bytes of dword i that belong to a k-mer of length k.
__device__ __forceinline__ uint32_t tail_mask(int i, int k) {
    const int valid = k - 4 * i;
    return valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : ((1u << (8 * valid)) - 1u));
}

// k bytes of the read buffer at byte offset `off`, as 8 dwords, unmasked.
// Dwords that start at or past the end of the buffer are not loaded (device
// buffers handed over by the caller carry no padding).
template <int KT>
__device__ __forceinline__ void load_window(const uint8_t* seq, uint64_t seq_bytes, uint64_t off,
                                            uint32_t k, uint32_t (&w)[8]) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(seq) + off;
    const uint32_t* p = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uintptr_t lim = reinterpret_cast<uintptr_t>(seq) + seq_bytes;
    const uint32_t nw = KT ? (KT + 3) / 4 : (k + 3) / 4;
    uint32_t raw[9];
#pragma unroll
    for (int i = 0; i < 9; ++i)
        raw[i] = (i <= (int)nw && reinterpret_cast<uintptr_t>(p + i) < lim) ? p[i] : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = __builtin_amdgcn_alignbyte(raw[i + 1], raw[i], sh);
}

// Reverse complement of the k-byte window f (tail zero) when every byte is in
// {A, C, G, T, N}: complement + byte-reverse the nw dwords, then drop the
// 4*nw - k leading pad bytes.
template <int NW>
__device__ __forceinline__ void rc_perm_nw(const uint32_t (&f)[8], uint32_t sh, uint32_t (&r)[8]) {
    uint32_t R[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) R[j] = j < NW ? __builtin_bswap32(comp4(f[NW - 1 - j])) : 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = __builtin_amdgcn_alignbyte(R[i + 1], R[i], sh);
}

template <int KT>
__device__ __forceinline__ void rc_perm(const uint32_t (&f)[8], uint32_t k, uint32_t (&r)[8]) {
    if constexpr (KT != 0) {
        rc_perm_nw<(KT + 3) / 4>(f, (uint32_t)(4 * ((KT + 3) / 4) - KT), r);
    } else {
        const uint32_t nw = (k + 3) / 4, sh = 4 * nw - k;
        switch (nw) {
            case 1: rc_perm_nw<1>(f, sh, r); break;
            case 2: rc_perm_nw<2>(f, sh, r); break;
            case 3: rc_perm_nw<3>(f, sh, r); break;
            case 4: rc_perm_nw<4>(f, sh, r); break;
            case 5: rc_perm_nw<5>(f, sh, r); break;
            case 6: rc_perm_nw<6>(f, sh, r); break;
            case 7: rc_perm_nw<7>(f, sh, r); break;
            default: rc_perm_nw<8>(f, sh, r); break;
        }
    }
}

// ------------------------------------------------------------------ units
__device__ __forceinline__ uint64_t num_kmers(uint64_t len, uint32_t k, uint32_t step) {
    return len >= k ? (len - k + step) / step : 0;  // ceil((len-k+1)/step)
}

// Per read: sampled k-mer count and #units.
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

// queue[0] = number of units, queue[1] = next unit to hand out (zeroed here,
// before the probe kernel of the same stream starts).
__global__ void scatter_units_kernel(const uint64_t* __restrict__ nseg,
                                     const uint64_t* __restrict__ unit_ofs, uint64_t n,
                                     uint32_t* __restrict__ unit_read, uint64_t* queue,
                                     uint32_t* __restrict__ hits_zero, uint64_t D) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = nseg[r], b = unit_ofs[r];
        for (uint64_t u = 0; u < s; ++u) unit_read[b + u] = (uint32_t)r;
        // rows the probe does not store whole: no k-mers (never visited) or
        // several units (accumulated atomically)
        if (s != 1 && hits_zero)
            for (uint64_t d = 0; d < D; ++d) hits_zero[r * D + d] = 0;
        if (r == n - 1) {
            queue[0] = b + s;
            queue[1] = 0;
        }
    }
}

// Hand out kGrab units per atomic to balance ragged reads across waves.
constexpr uint32_t kGrab = 4;

__device__ __forceinline__ uint64_t grab_units(uint64_t* queue, int lane) {
    uint64_t base = 0;
    if (lane == 0) base = atomicAdd(reinterpret_cast<unsigned long long*>(queue + 1), (unsigned long long)kGrab);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// ------------------------------------------------------------------ counting
// Column popcount of a 32x32 bit matrix held one row per lane of each 32-lane
// half: five exchange stages (lane ^ 16, 8, 4, 2, 1) transpose the matrix, so
// lane c then holds column c (bit r = row r's bit c), whose popcount is the
// number of rows (k-mers) with bit c (doc) set.  Stage s swaps the s-wide bit
// blocks between partner lanes: 1 shuffle + 1 rotate + 1 bit-select.
struct Xpose {
    uint32_t msk[5];  // bfi select: keep own bits (m_s, or ~m_s on the upper lane of a pair)
    uint32_t rot[4];  // rotate-right that aligns the partner's block (stages 8..1)
};

__device__ __forceinline__ void xpose_init(int lane, Xpose& X) {
    const uint32_t ss[5] = {16, 8, 4, 2, 1};
    const uint32_t mm[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const bool upper = (lane & ss[i]) != 0;
        X.msk[i] = upper ? ~mm[i] : mm[i];
        if (i > 0) X.rot[i - 1] = upper ? ss[i] : 32 - ss[i];
    }
}

__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

// The 32x32 transpose itself: bit r of lane c's result is row r's bit c.
__device__ __forceinline__ uint32_t xpose32(uint32_t x, const Xpose& X) {
    uint32_t y;
    y = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x401F);                 // lane ^ 16
    x = bsel(X.msk[0], x, __builtin_amdgcn_alignbit(y, y, 16));
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xF, 0xF, false);  // row_ror:8 = lane ^ 8
    x = bsel(X.msk[1], x, __builtin_amdgcn_alignbit(y, y, X.rot[0]));
    y = (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, 0x101F);                 // lane ^ 4
    x = bsel(X.msk[2], x, __builtin_amdgcn_alignbit(y, y, X.rot[1]));
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);   // quad_perm 2301 = lane ^ 2
    x = bsel(X.msk[3], x, __builtin_amdgcn_alignbit(y, y, X.rot[2]));
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);   // quad_perm 1032 = lane ^ 1
    x = bsel(X.msk[4], x, __builtin_amdgcn_alignbit(y, y, X.rot[3]));
    return x;
}

__device__ __forceinline__ uint32_t column_popc32(uint32_t x, const Xpose& X) {
    return (uint32_t)__popc(xpose32(x, X));
}

// Sum of lane l and lane l ^ 32 (the two halves' counts of the same doc).
__device__ __forceinline__ uint32_t fold_halves(uint32_t v) {
    return v + (uint32_t)__shfl_xor((int)v, 32, 64);
}

__device__ __forceinline__ uint4 and4(uint4 a, uint4 b) {
    return make_uint4(a.x & b.x, a.y & b.y, a.z & b.z, a.w & b.w);
}

// Canonical k-mer of read position p (byte offset o0 of a read of length len).
template <int KT, int MODE>
__device__ __forceinline__ void kmer_at(const ReadView& rv, uint64_t o0, uint64_t len, uint64_t p,
                                        uint32_t k, Kmer& c) {
    (void)len;
    const int kk = KT ? KT : (int)k;
    uint32_t f[8], r[8];
    load_window<KT>(rv.seq, rv.seq_bytes, o0 + p, k, f);
    if constexpr (MODE == kKmerCobs) {
#pragma unroll
        for (int i = 0; i < 8; ++i) f[i] = cobs_norm4(f[i]) & tail_mask(i, kk);
        rc_perm<KT>(f, k, r);
    } else {
        bool fast = true;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t m = tail_mask(i, kk);
            f[i] &= m;
            const uint32_t ok = bytes_equal(f[i], 'A') | bytes_equal(f[i], 'C') | bytes_equal(f[i], 'G') |
                                bytes_equal(f[i], 'T') | bytes_equal(f[i], 'N');
            fast = fast && ((ok | ~m) & 0x80808080u) == 0x80808080u;
        }
        if (fast) {
            rc_perm<KT>(f, k, r);
        } else {  // IUPAC / lower case: per-byte table, bytes re-read from the read
            const uint8_t* s = rv.seq + o0 + p;
#pragma unroll
            for (int i = 0; i < 8; ++i) r[i] = 0;
#pragma unroll
            for (int i = 0; i < (int)kMaxK; ++i)
                if (i < kk) r[i >> 2] |= bio_comp_byte(s[kk - 1 - i]) << (8 * (i & 3));
        }
    }
    canonical_select(f, r, c);
}

// ------------------------------------------------------------------ COBS probe (fast)
// Classic bank with D <= 128 docs: one 16-byte row per hash, counters in
// registers.  One wavefront per unit (<= kSegKmers k-mers of one read), one
// lane per k-mer; units are handed out kGrab at a time.
struct FastBank {
    const uint8_t* rows;
    uint64_t sig, magic;
    uint32_t D, nwords;  // nwords = ceil(D/32)
    uint32_t image_bytes;
};

// Row gather policies (XSPECT2_AMD_LOADPOL): 0 global_load_dwordx4; buffer_load
// with cache-policy aux 1: none, 2: nt, 3: sc1, 4: sc0 sc1 (L1 bypass forms).
template <int POL>
__device__ __forceinline__ uint4 load_row(const FastBank& fb, uint32_t off) {
    if constexpr (POL == 0) {
        return *reinterpret_cast<const uint4*>(fb.rows + off);
    } else {
        constexpr int aux = POL == 1 ? 0 : POL == 2 ? 2 : POL == 3 ? 16 : 17;
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(fb.rows), (short)0,
                                                            (int)fb.image_bytes, 0x00020000);
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)off, 0, aux);
        return make_uint4(v[0], v[1], v[2], v[3]);
    }
}

template <int KT, int HT, int POL>
__global__ void __launch_bounds__(kProbeThreads, 2) probe_cobs_fast(ReadView rv, FastBank fb,
                                                                    uint32_t* __restrict__ hits,
                                                                    uint64_t* __restrict__ partials) {
    __shared__ uint64_t s_tot[kProbeThreads / kWave][128];
    __shared__ uint64_t s_kmers[kProbeThreads / kWave];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    s_tot[wid][lane] = 0;
    s_tot[wid][lane + 64] = 0;
    Xpose X;
    xpose_init(lane, X);
    const uint32_t k = KT ? KT : rv.k;
    const uint32_t step = rv.step;
    const uint32_t D = fb.D, nwords = fb.nwords;
    const uint64_t U = rv.queue[0];
    uint64_t kmer_total = 0;

    for (;;) {
        const uint64_t base = grab_units(rv.queue, lane);
        if (base >= U) break;
        const uint64_t uend = min(base + kGrab, U);
        for (uint64_t u = base; u < uend; ++u) {
            const uint32_t r = rv.unit_read[u];
            const uint64_t seg = u - rv.unit_ofs[r];
            const uint64_t o0 = rv.offs[r];
            const uint64_t len = rv.offs[r + 1] - o0;
            const uint64_t nk = num_kmers(len, k, step);
            const uint64_t t0 = seg * kSegKmers;
            const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
            kmer_total += cnt;
            uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
            for (uint32_t tb = 0; tb < cnt; tb += 64) {
                uint4 m = make_uint4(0u, 0u, 0u, 0u);
                if (tb + lane < cnt) {
                    Kmer c;
                    kmer_at<KT, kKmerCobs>(rv, o0, len, (t0 + tb + lane) * step, k, c);
                    Xxh64Pre pre;
                    xxh64_pre<KT>(c, k, pre);
                    uint32_t off[HT];
#pragma unroll
                    for (int j = 0; j < HT; ++j)
                        off[j] = (uint32_t)fastmod(xxh64_seed<KT>(c, pre, k, (uint64_t)j), fb.sig, fb.magic) * 16u;
                    m = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
                    for (int j = 0; j < HT; ++j)
                        m = and4(m, load_row<POL>(fb, off[j]));
                }
                a0 += column_popc32(m.x, X);
                if (nwords > 1) a1 += column_popc32(m.y, X);
                if (nwords > 2) a2 += column_popc32(m.z, X);
                if (nwords > 3) a3 += column_popc32(m.w, X);
            }
            // lane c < 32 holds doc 32q + c of word q after folding the halves
            const bool whole = nk <= kSegKmers;
            const uint32_t acc[4] = {a0, a1, a2, a3};
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                if (q >= nwords) break;
                const uint32_t v = fold_halves(acc[q]);
                const uint32_t d = q * 32 + (uint32_t)lane;
                if (lane < 32 && d < D) {
                    s_tot[wid][d] += v;
                    if (hits) {
                        if (whole) hits[(uint64_t)r * D + d] = v;
                        else if (v) atomicAdd(&hits[(uint64_t)r * D + d], v);
                    }
                }
            }
        }
    }
    if (partials) {
        if (lane == 0) s_kmers[wid] = kmer_total;
        __syncthreads();
        const int wpb = blockDim.x >> 6;
        uint64_t* out = partials + (uint64_t)blockIdx.x * (D + 1);
        for (uint32_t d = threadIdx.x; d < D; d += blockDim.x) {
            uint64_t s = 0;
            for (int w = 0; w < wpb; ++w) s += s_tot[w][d];
            out[d] = s;
        }
        if (threadIdx.x == 0) {
            uint64_t s = 0;
            for (int w = 0; w < wpb; ++w) s += s_kmers[w];
            out[D] = s;
        }
    }
}

// ------------------------------------------------------------------ COBS probe (general)
// Any D the LDS counters hold, compact doc groups, any row width (chunks in batches of kMaxChunks 16-byte
// row.  Same unit scheme and column-popcount counting as the fast kernel.
template <int KT, int HT>
__global__ void __launch_bounds__(kProbeThreads) probe_cobs_kernel(ReadView rv, CobsView bv,
                                                                   uint32_t* __restrict__ hits,
                                                                   uint64_t* __restrict__ partials,
                                                                   uint32_t dpad) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    __shared__ uint64_t s_kmers[kProbeThreads / kWave];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int wpb = blockDim.x >> 6;
    uint32_t* acc = smem + (size_t)wid * 2 * dpad;  // per unit
    uint32_t* tot = acc + dpad;                     // per wave
    for (uint32_t d = lane; d < 2 * dpad; d += 64) acc[d] = 0;
    Xpose X;
    xpose_init(lane, X);

    const uint32_t k = KT ? KT : rv.k;
    const uint32_t h = HT ? HT : bv.h;
    const uint32_t step = rv.step;
    const uint64_t D = bv.D;
    const uint64_t U = rv.queue[0];
    uint64_t kmer_total = 0;

    for (;;) {
        const uint64_t base = grab_units(rv.queue, lane);
        if (base >= U) break;
        const uint64_t uend = min(base + kGrab, U);
        for (uint64_t u = base; u < uend; ++u) {
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
                    Kmer c;
                    kmer_at<KT, kKmerCobs>(rv, o0, len, (t0 + tb + lane) * step, k, c);
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
                        if (j < h) ro[j] = gd.base + fastmod(act ? hv[j] : 0, gd.sig, gd.magic) * bv.pitch;
                    // kMaxChunks chunk loads of the group's h rows in flight, then count
                    const uint32_t nch_all = (uint32_t)min((uint64_t)bv.nchunks, (dlim - doc0 + 127) / 128);
                    for (uint32_t cb = 0; cb < nch_all; cb += kMaxChunks) {
                    const uint32_t nch = min(kMaxChunks, nch_all - cb);
                    // unconditional loads (chunk 0 past the batch, row 0 without a
                    // k-mer), masked afterwards, so they all stay in flight
                    uint4 mk[kMaxChunks];
#pragma unroll
                    for (uint32_t cc = 0; cc < kMaxChunks; ++cc) {
                        const uint32_t co = cc < nch ? (cb + cc) * 16 : 0;
                        uint4 m = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
                        for (uint32_t j = 0; j < (HT ? HT : kMaxHashes); ++j)
                            if (j < h) m = and4(m, *reinterpret_cast<const uint4*>(bv.rows + ro[j] + co));
                        mk[cc] = (cc < nch && act) ? m : make_uint4(0u, 0u, 0u, 0u);
                    }
#pragma unroll
                    for (uint32_t cc = 0; cc < kMaxChunks; ++cc) {
                        if (cc >= nch) break;
                        const uint64_t cd0 = doc0 + (uint64_t)(cb + cc) * 128;
                        const uint32_t nd = (uint32_t)min((uint64_t)128, dlim - cd0);
                        const uint32_t w[4] = {mk[cc].x, mk[cc].y, mk[cc].z, mk[cc].w};
#pragma unroll
                        for (uint32_t q = 0; q < 4; ++q) {
                            if (q * 32 >= nd) break;
                            if (__ballot(w[q] != 0u) == 0ull) continue;  // no k-mer of the tile hits these docs
                            const uint32_t v = fold_halves(column_popc32(w[q], X));
                            // return-free ds_add: no read-modify-write latency chain
                            if (lane < 32 && q * 32 + lane < nd && v) atomicAdd(&acc[cd0 + q * 32 + lane], v);
                        }
                    }
                    }  // chunk batch
                }
            }
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

// ------------------------------------------------------------------ COBS probe (wide classic rows)
// Classic banks of 129..2048 docs: a row is C 16-byte chunks (C = 2, 4, 8 or
// 16, the next power of two of its data chunks; the pitch is padded so a row
// is one 128-byte line, or two aligned lines at C = 16).  Hashing stays one lane per k-mer, but the
// gathers run C lanes per k-mer: in sub-tile s, lane l loads chunk l % C of
// k-mer s * (64 / C) + l / C.  One load instruction then reads 64 / C whole
// rows, so the vector L1 sees each row line once instead of once per chunk.
// Counting: after the 32x32 transpose of a 32-lane half, bit r of lane t is
// lane r's bit t, and lanes r = c (mod C) hold chunk c: one masked popcount
// per chunk.
template <int C>
struct ChunkLanes {  // bits r of a 32-row column with r % C == 0
    static constexpr uint32_t m0 = C == 2 ? 0x55555555u : C == 4 ? 0x11111111u : C == 8 ? 0x01010101u : 0x00010001u;
};

template <int KT, int HT, int C, int P>
__global__ void __launch_bounds__(kProbeThreads, 2) probe_cobs_wide(ReadView rv, CobsView bv,
                                                                    uint32_t* __restrict__ hits,
                                                                    uint64_t* __restrict__ partials,
                                                                    uint32_t dpad) {
    constexpr int K = 64 / C;  // k-mers per sub-tile
    constexpr uint32_t M0 = ChunkLanes<C>::m0;
    static_assert(C % P == 0, "sub-tiles in flight must divide the sub-tile count");
    extern __shared__ __attribute__((aligned(16))) uint64_t s_tot[];  // [dpad] per block
    __shared__ uint64_t s_kmers[kProbeThreads / kWave];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    for (uint32_t d = threadIdx.x; d < dpad; d += blockDim.x) s_tot[d] = 0;
    __syncthreads();
    Xpose X;
    xpose_init(lane, X);

    constexpr int NH = HT ? HT : (int)kMaxHashes;
    const uint32_t k = KT ? KT : rv.k;
    const uint32_t h = HT ? HT : bv.h;
    const uint32_t step = rv.step;
    const uint64_t D = bv.D;
    const uint32_t cpg = bv.nchunks;  // data chunks, <= C (host-checked)
    const GroupDesc gd = bv.groups[0];  // sig < 2^32 (host-checked): 32-bit row indices
    const uint8_t* rows = bv.rows + gd.base;
    const uint32_t pitch = bv.pitch;
    const int my_c = lane % C, my_slot = lane / C;
    const bool my_chunk_on = (uint32_t)my_c < cpg;
    const uint32_t my_c_ofs = my_chunk_on ? (uint32_t)my_c * 16 : 0;
    const uint64_t U = rv.queue[0];
    uint64_t kmer_total = 0;

    for (;;) {
        const uint64_t base = grab_units(rv.queue, lane);
        if (base >= U) break;
        const uint64_t uend = min(base + kGrab, U);
        for (uint64_t u = base; u < uend; ++u) {
            const uint32_t r = rv.unit_read[u];
            const uint64_t seg = u - rv.unit_ofs[r];
            const uint64_t o0 = rv.offs[r];
            const uint64_t len = rv.offs[r + 1] - o0;
            const uint64_t nk = num_kmers(len, k, step);
            const uint64_t t0 = seg * kSegKmers;
            const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
            kmer_total += cnt;
            uint32_t acc[2 * C];  // chunk cc, words q: 16-bit counters, reg 2*cc + (q >> 1)
#pragma unroll
            for (int i = 0; i < 2 * C; ++i) acc[i] = 0;

            for (uint32_t tb = 0; tb < cnt; tb += 64) {
                const bool act = tb + lane < cnt;
                uint32_t ri[NH];  // row index of hash j
#pragma unroll
                for (int j = 0; j < NH; ++j) ri[j] = 0;
                if (act) {
                    Kmer c;
                    kmer_at<KT, kKmerCobs>(rv, o0, len, (t0 + tb + lane) * step, k, c);
                    Xxh64Pre pre;
                    xxh64_pre<KT>(c, k, pre);
#pragma unroll
                    for (int j = 0; j < NH; ++j)
                        if ((uint32_t)j < h)
                            ri[j] = (uint32_t)fastmod(xxh64_seed<KT>(c, pre, k, (uint64_t)j), gd.sig, gd.magic);
                }
                const uint32_t tile = min(64u, cnt - tb);
#pragma unroll
                for (int s0 = 0; s0 < C; s0 += P) {
                    if ((uint32_t)(s0 * K) >= tile) continue;  // uniform
                    // P sub-tiles' row chunks in flight before any counting.  The
                    // loads are unconditional (a lane without a k-mer has row 0,
                    // a lane past the data chunks reads chunk 0) and masked
                    // afterwards: a load under a divergent branch would be
                    // waited for before the branch joins, one row at a time.
                    uint4 mm[P];
#pragma unroll
                    for (int p = 0; p < P; ++p) {
                        const int src = (s0 + p) * K + my_slot;
                        const bool on = (uint32_t)src < tile && my_chunk_on;
                        uint4 v[NH];
#pragma unroll
                        for (int j = 0; j < NH; ++j) {
                            if ((uint32_t)j >= h) continue;
                            const uint32_t rj = (uint32_t)__shfl((int)ri[j], src, 64);
                            v[j] = *reinterpret_cast<const uint4*>(rows + (uint64_t)rj * pitch + my_c_ofs);
                        }
                        uint4 m = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
                        for (int j = 0; j < NH; ++j)
                            if ((uint32_t)j < h) m = and4(m, v[j]);
                        mm[p] = on ? m : make_uint4(0u, 0u, 0u, 0u);
                    }
#pragma unroll
                    for (int p = 0; p < P; ++p) {
                        const uint32_t w[4] = {mm[p].x, mm[p].y, mm[p].z, mm[p].w};
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            if (__ballot(w[q] != 0u) == 0ull) continue;
                            const uint32_t x = xpose32(w[q], X);
#pragma unroll
                            for (int cc = 0; cc < C; ++cc)
                                acc[2 * cc + (q >> 1)] += (uint32_t)__popc(x & (M0 << cc)) << (16 * (q & 1));
                        }
                    }
                }
            }
            // lane t < 32 holds doc 128 cc + 32 q + t after folding the halves
            const bool whole = nk <= kSegKmers;
#pragma unroll
            for (int cc = 0; cc < C; ++cc) {
                if ((uint32_t)cc >= cpg) continue;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint64_t d0 = (uint64_t)cc * 128 + q * 32;
                    if (d0 >= D) continue;
                    const uint32_t v = fold_halves((acc[2 * cc + (q >> 1)] >> (16 * (q & 1))) & 0xFFFFu);
                    const uint64_t d = d0 + (uint64_t)lane;
                    if (lane < 32 && d < D) {
                        if (v) atomicAdd(reinterpret_cast<unsigned long long*>(&s_tot[d]), (unsigned long long)v);
                        if (hits) {
                            if (whole) hits[(uint64_t)r * D + d] = v;
                            else if (v) atomicAdd(&hits[(uint64_t)r * D + d], v);
                        }
                    }
                }
            }
        }
    }
    if (lane == 0) s_kmers[wid] = kmer_total;
    __syncthreads();
    if (partials) {
        const int wpb = blockDim.x >> 6;
        uint64_t* out = partials + (uint64_t)blockIdx.x * (D + 1);
        for (uint64_t d = threadIdx.x; d < D; d += blockDim.x) out[d] = s_tot[d];
        if (threadIdx.x == 0) {
            uint64_t s = 0;
            for (int w = 0; w < wpb; ++w) s += s_kmers[w];
            out[D] = s;
        }
    }
}

// ------------------------------------------------------------------ COBS probe (slots)
// Banks whose rows span at most GM groups x CM 16-byte chunks (classic
// rows the fast and wide kernels do not take, as GM = 1; compact schemes such
// as an MLST locus: 3 groups x 4 chunks).  The layout is compile-time, so every slot's group and chunk is a
// constant; runtime guards only switch slots off.  Every chunk of every
// group's h rows is in flight before any counting; per-doc counts of the unit
// live in registers, two 16-bit counters per VGPR (a unit has <= 256 k-mers,
// so one lane-half count is <= 128); block totals go to LDS with return-free
// ds_add.
template <int KT, int HT, int GM, int CM>
__global__ void __launch_bounds__(kProbeThreads, 2) probe_cobs_slots(ReadView rv, CobsView bv,
                                                                     uint32_t* __restrict__ hits,
                                                                     uint64_t* __restrict__ partials,
                                                                     uint32_t dpad) {
    constexpr int NS = GM * CM;
    extern __shared__ __attribute__((aligned(16))) uint64_t s_tot[];  // [dpad] per block
    __shared__ uint64_t s_kmers[kProbeThreads / kWave];
    // group descriptors staged once in LDS (slots past G alias group 0): their
    // reads wait on lgkmcnt, never behind the row loads' vmcnt
    __shared__ GroupDesc s_gd[GM];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    for (uint32_t d = threadIdx.x; d < dpad; d += blockDim.x) s_tot[d] = 0;
    if (threadIdx.x < GM) s_gd[threadIdx.x] = bv.groups[threadIdx.x < bv.G ? threadIdx.x : 0];
    __syncthreads();
    Xpose X;
    xpose_init(lane, X);

    constexpr int NH = HT ? HT : (int)kMaxHashes;
    const uint32_t k = KT ? KT : rv.k;
    const uint32_t h = HT ? HT : bv.h;
    const uint32_t step = rv.step;
    const uint64_t D = bv.D;
    const uint32_t G = bv.G;               // <= GM (host-checked)
    const uint32_t cpg = bv.nchunks;       // <= CM (host-checked)
    const uint64_t gdocs = 8 * bv.page;    // docs per group
    uint32_t cofs[CM];                     // byte offset of chunk cc (0 past the data chunks)
#pragma unroll
    for (int cc = 0; cc < CM; ++cc) cofs[cc] = (uint32_t)cc < cpg ? cc * 16 : 0;
    const uint64_t U = rv.queue[0];
    uint64_t kmer_total = 0;

    for (;;) {
        const uint64_t base = grab_units(rv.queue, lane);
        if (base >= U) break;
        const uint64_t uend = min(base + kGrab, U);
        for (uint64_t u = base; u < uend; ++u) {
            const uint32_t r = rv.unit_read[u];
            const uint64_t seg = u - rv.unit_ofs[r];
            const uint64_t o0 = rv.offs[r];
            const uint64_t len = rv.offs[r + 1] - o0;
            const uint64_t nk = num_kmers(len, k, step);
            const uint64_t t0 = seg * kSegKmers;
            const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
            kmer_total += cnt;
            uint32_t acc[2 * NS];
#pragma unroll
            for (int i = 0; i < 2 * NS; ++i) acc[i] = 0;

            for (uint32_t tb = 0; tb < cnt; tb += 64) {
                const bool act = tb + lane < cnt;
                uint64_t hv[NH];
#pragma unroll
                for (int j = 0; j < NH; ++j) hv[j] = 0;
                if (act) {
                    Kmer c;
                    kmer_at<KT, kKmerCobs>(rv, o0, len, (t0 + tb + lane) * step, k, c);
                    Xxh64Pre pre;
                    xxh64_pre<KT>(c, k, pre);
#pragma unroll
                    for (int j = 0; j < NH; ++j)
                        if ((uint32_t)j < h) hv[j] = xxh64_seed<KT>(c, pre, k, (uint64_t)j);
                }
                // Every row load is unconditional: a lane without a k-mer has
                // hash 0 (a valid row), a chunk past the data reads chunk 0, a
                // group past G reads group 0; results are masked afterwards.  A
                // load under a divergent branch would be waited for at the join.
                uint4 mk[NS];
#pragma unroll
                for (int g = 0; g < GM; ++g) {
                    const GroupDesc gd = s_gd[g];
                    uint64_t ro[NH];
#pragma unroll
                    for (int j = 0; j < NH; ++j)
                        ro[j] = (uint32_t)j < h ? gd.base + fastmod(hv[j], gd.sig, gd.magic) * bv.pitch : 0;
                    // row-major issue order: the chunks of one row leave back to back,
                    // so the vector L1 sees one row line in consecutive requests
#pragma unroll
                    for (int cc = 0; cc < CM; ++cc) mk[g * CM + cc] = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
                    for (int j = 0; j < NH; ++j) {
                        if ((uint32_t)j >= h) continue;
#pragma unroll
                        for (int cc = 0; cc < CM; ++cc)
                            mk[g * CM + cc] = and4(mk[g * CM + cc],
                                                   *reinterpret_cast<const uint4*>(bv.rows + ro[j] + cofs[cc]));
                    }
                    const bool on = (uint32_t)g < G && act;
#pragma unroll
                    for (int cc = 0; cc < CM; ++cc)
                        if (!(on && (uint32_t)cc < cpg)) mk[g * CM + cc] = make_uint4(0u, 0u, 0u, 0u);
                }
#pragma unroll
                for (int g = 0; g < GM; ++g) {
#pragma unroll
                    for (int cc = 0; cc < CM; ++cc) {
                        if ((uint32_t)g < G && (uint32_t)cc < cpg) {
                            const int i = g * CM + cc;
                            const uint32_t w[4] = {mk[i].x, mk[i].y, mk[i].z, mk[i].w};
#pragma unroll
                            for (int q = 0; q < 4; ++q)
                                if (__ballot(w[q] != 0u) != 0ull)  // some k-mer of the tile hits these docs
                                    acc[2 * i + (q >> 1)] += column_popc32(w[q], X) << (16 * (q & 1));
                        }
                    }
                }
            }
            // lane c < 32 holds doc 32q + c of chunk (g, cc) after folding the halves
            const bool whole = nk <= kSegKmers;
#pragma unroll
            for (int g = 0; g < GM; ++g) {
                if ((uint32_t)g >= G) continue;
                const uint64_t glim = min(D, (uint64_t)g * gdocs + gdocs);
#pragma unroll
                for (int cc = 0; cc < CM; ++cc) {
                    if ((uint32_t)cc >= cpg) continue;
                    const int i = g * CM + cc;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint64_t d0 = (uint64_t)g * gdocs + cc * 128 + q * 32;
                        if (d0 >= glim) continue;
                        const uint32_t v = fold_halves((acc[2 * i + (q >> 1)] >> (16 * (q & 1))) & 0xFFFFu);
                        const uint64_t d = d0 + (uint64_t)lane;
                        if (lane < 32 && d < glim) {
                            if (v) atomicAdd(reinterpret_cast<unsigned long long*>(&s_tot[d]), (unsigned long long)v);
                            if (hits) {
                                if (whole) hits[(uint64_t)r * D + d] = v;
                                else if (v) atomicAdd(&hits[(uint64_t)r * D + d], v);
                            }
                        }
                    }
                }
            }
        }
    }
    if (lane == 0) s_kmers[wid] = kmer_total;
    __syncthreads();
    if (partials) {
        const int wpb = blockDim.x >> 6;
        uint64_t* out = partials + (uint64_t)blockIdx.x * (D + 1);
        for (uint64_t d = threadIdx.x; d < D; d += blockDim.x) out[d] = s_tot[d];
        if (threadIdx.x == 0) {
            uint64_t s = 0;
            for (int w = 0; w < wpb; ++w) s += s_kmers[w];
            out[D] = s;
        }
    }
}

// ------------------------------------------------------------------ rbloom probe
// Filter bits tested before the rest: 2 measured fastest for member-heavy
// and foreign-heavy reads alike (tools/gpu_bloom_ab.sh).
constexpr int kBloomSplitDefault = 2;
// All K bit indices first, then all K dword loads in flight at once (the
// reference stops at the first zero bit; the answer is the same).
// Returns bit 0: member; bit 1: the second load phase ran.
template <int KT, int KB, int SPLIT>
__device__ __forceinline__ uint32_t bloom_member(const Kmer& c, uint32_t k, const BloomView& bv) {
    constexpr int NK = KB ? KB : (int)kMaxHashes;
    const uint32_t K = KB ? KB : bv.K;
    uint64_t sl = xxh3_kmer<KT>(c, k), sh = 0;
    uint64_t idx[NK];
#pragma unroll
    for (int j = 0; j < NK; ++j) {
        if ((uint32_t)j < K) {
            const uint64_t p = sl * kLcgMl;
            const uint64_t nl = p + kLcgCl;
            const uint64_t carry = nl < p;
            sh = sh * kLcgMl + sl * kLcgMh + __umul64hi(sl, kLcgMl) + kLcgCh + carry;
            sl = nl;
            idx[j] = fastmod(sh, bv.mbits, bv.magic);
        }
    }
    // The first SPLIT bits decide most non-members (rbloom stops at the
    // first zero bit); the other loads go out only for lanes still in.
    // SPLIT = 0: all K loads at once.
    uint32_t all = 1;
#pragma unroll
    for (int j = 0; j < NK; ++j)
        if ((uint32_t)j < K && (SPLIT == 0 || j < SPLIT)) all &= bv.bits[idx[j] >> 5] >> (idx[j] & 31);
    uint32_t phase2 = 0;
    if (SPLIT != 0 && (all & 1u) && (uint32_t)SPLIT < K) {
        phase2 = 2u;
#pragma unroll
        for (int j = SPLIT; j < NK; ++j)
            if ((uint32_t)j < K) all &= bv.bits[idx[j] >> 5] >> (idx[j] & 31);
    }
    return (all & 1u) | phase2;
}

template <int KT, int KB, int SPLIT>
__global__ void __launch_bounds__(kProbeThreads) probe_bloom_kernel(ReadView rv, BloomView bv,
                                                                    uint32_t* __restrict__ hits,
                                                                    uint64_t* __restrict__ partials) {
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int wpb = blockDim.x >> 6;
    __shared__ uint64_t s_hits[kProbeThreads / kWave], s_kmers[kProbeThreads / kWave];
    const uint32_t k = KT ? KT : rv.k;
    const uint32_t step = rv.step;
    const uint64_t U = rv.queue[0];
    uint64_t hit_total = 0, kmer_total = 0, rows_total = 0;

    for (;;) {
        const uint64_t base = grab_units(rv.queue, lane);
        if (base >= U) break;
        const uint64_t uend = min(base + kGrab, U);
        for (uint64_t u = base; u < uend; ++u) {
            const uint32_t r = rv.unit_read[u];
            const uint64_t seg = u - rv.unit_ofs[r];
            const uint64_t o0 = rv.offs[r];
            const uint64_t len = rv.offs[r + 1] - o0;
            const uint64_t nk = num_kmers(len, k, step);
            const uint64_t t0 = seg * kSegKmers;
            const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
            uint32_t c_unit = 0;
            for (uint32_t tb = 0; tb < cnt; tb += 64) {
                bool in = false, again = false;
                if (tb + lane < cnt) {
                    Kmer c;
                    kmer_at<KT, kKmerBio>(rv, o0, len, (t0 + tb + lane) * step, k, c);
                    const uint32_t res = bloom_member<KT, KB, SPLIT>(c, k, bv);
                    in = res & 1u;
                    again = (res & 2u) != 0;
                }
                c_unit += (uint32_t)__popcll(__ballot(in));
                if (bv.rows_read) {
                    const uint32_t K = KB ? KB : bv.K;
                    const uint32_t first = SPLIT == 0 || (uint32_t)SPLIT >= K ? K : (uint32_t)SPLIT;
                    rows_total += (uint64_t)__popcll(__ballot(tb + lane < cnt)) * first +
                                  (uint64_t)__popcll(__ballot(again)) * (K - first);
                }
            }
            kmer_total += cnt;
            hit_total += c_unit;
            if (hits && lane == 0) {
                if (nk <= kSegKmers) hits[r] = c_unit;
                else if (c_unit) atomicAdd(&hits[r], c_unit);
            }
        }
    }
    if (bv.rows_read && lane == 0 && rows_total)
        atomicAdd(reinterpret_cast<unsigned long long*>(bv.rows_read), (unsigned long long)rows_total);
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
    const uint32_t k = KT ? KT : rv.k;
    const uint32_t h = HT ? HT : bv.h;
    const uint64_t U = rv.queue[0];
    for (;;) {
        const uint64_t base = grab_units(rv.queue, lane);
        if (base >= U) break;
        const uint64_t uend = min(base + kGrab, U);
        for (uint64_t u = base; u < uend; ++u) {
            const uint32_t r = rv.unit_read[u];
            const uint64_t seg = u - rv.unit_ofs[r];
            const uint64_t o0 = rv.offs[r];
            const uint64_t len = rv.offs[r + 1] - o0;
            const uint64_t nk = num_kmers(len, k, 1);
            const uint64_t t0 = seg * kSegKmers;
            const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
            const uint64_t doc = rec_doc[r];
            if (doc >= bv.D) continue;
            const uint64_t g = doc / (8 * bv.page), bit = doc % (8 * bv.page);
            const GroupDesc gd = bv.groups[g];
            for (uint32_t tb = 0; tb < cnt; tb += 64) {
                if (tb + lane >= cnt) continue;
                Kmer c;
                kmer_at<KT, kKmerCobs>(rv, o0, len, t0 + tb + lane, k, c);
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
}

template <int KT>
__global__ void __launch_bounds__(kProbeThreads) build_bloom_kernel(ReadView rv, BloomView bv,
                                                                    uint32_t* bits) {
    const int lane = threadIdx.x & 63;
    const uint32_t k = KT ? KT : rv.k;
    const uint64_t U = rv.queue[0];
    for (;;) {
        const uint64_t base = grab_units(rv.queue, lane);
        if (base >= U) break;
        const uint64_t uend = min(base + kGrab, U);
        for (uint64_t u = base; u < uend; ++u) {
            const uint32_t r = rv.unit_read[u];
            const uint64_t seg = u - rv.unit_ofs[r];
            const uint64_t o0 = rv.offs[r];
            const uint64_t len = rv.offs[r + 1] - o0;
            const uint64_t nk = num_kmers(len, k, 1);
            const uint64_t t0 = seg * kSegKmers;
            const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
            for (uint32_t tb = 0; tb < cnt; tb += 64) {
                if (tb + lane >= cnt) continue;
                Kmer c;
                kmer_at<KT, kKmerBio>(rv, o0, len, t0 + tb + lane, k, c);
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
}

// ------------------------------------------------------------------ misc
// One block per column: sum of the per-block partial totals.
__global__ void __launch_bounds__(256) reduce_partials_kernel(const uint64_t* __restrict__ partials,
                                                              int blocks, uint64_t cols,
                                                              uint64_t* __restrict__ totals) {
    __shared__ uint64_t s[256];
    for (uint64_t c = blockIdx.x; c < cols; c += gridDim.x) {
        uint64_t v = 0;
        for (int b = threadIdx.x; b < blocks; b += blockDim.x) v += partials[(uint64_t)b * cols + c];
        s[threadIdx.x] = v;
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if ((int)threadIdx.x < w) s[threadIdx.x] += s[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) totals[c] = s[0];
        __syncthreads();
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

// ------------------------------------------------------------------ per-read best doc
// The doc with the most hits of each read, or kBestAmbiguous when several docs
// share the maximum: the per-read call of scripts/benchmark/main.nf:417-436
// ("ambiguous" on ties), made on the device so the n x D matrix stays in HBM.
// One wavefront per read; lanes stride over the docs.
__global__ void __launch_bounds__(256) best_doc_kernel(const uint32_t* __restrict__ hits, uint64_t n,
                                                       uint64_t D, uint32_t* __restrict__ best,
                                                       uint32_t* __restrict__ best_hits) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t r = wave; r < n; r += waves) {
        const uint32_t* row = hits + r * D;
        uint32_t m = 0, arg = kBestAmbiguous, cnt = 0;
        for (uint64_t d = (uint64_t)lane; d < D; d += 64) {
            const uint32_t v = row[d];
            if (cnt == 0 || v > m) {
                m = v;
                arg = (uint32_t)d;
                cnt = 1;
            } else if (v == m) {
                ++cnt;
            }
        }
        uint32_t wm = m;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) wm = max(wm, (uint32_t)__shfl_xor((int)wm, o, 64));
        uint32_t c = (cnt && m == wm) ? cnt : 0;
        uint32_t a = c ? arg : kBestAmbiguous;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            c += (uint32_t)__shfl_xor((int)c, o, 64);
            a = min(a, (uint32_t)__shfl_xor((int)a, o, 64));
        }
        if (lane == 0) {
            best[r] = c == 1 ? a : kBestAmbiguous;
            if (best_hits) best_hits[r] = wm;
        }
    }
}

// ------------------------------------------------------------------ read gather
// out read j = in read index[j], at out_offs[j] (computed by the caller): the
// device-side compaction of reads that passed the genus filter.  One wave per
// read, lanes copy bytes (coalesced 64-byte runs).
__global__ void __launch_bounds__(256) gather_reads_kernel(const uint8_t* __restrict__ seqs,
                                                           const uint64_t* __restrict__ offs,
                                                           const uint32_t* __restrict__ index, uint64_t m,
                                                           uint8_t* __restrict__ out,
                                                           const uint64_t* __restrict__ out_offs) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t j = wave; j < m; j += waves) {
        const uint32_t r = index[j];
        const uint64_t a = offs[r], len = offs[r + 1] - a, o = out_offs[j];
        for (uint64_t i = (uint64_t)lane; i < len; i += 64) out[o + i] = seqs[a + i];
    }
}

// ------------------------------------------------------------------ launchers
static inline int grid_for(uint64_t work, int per_block, int cap) {
    uint64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > (uint64_t)cap) g = cap;
    return (int)g;
}

// Resident blocks of `kernel` on the current device (blocks per CU x CUs),
// minus one block per CU of margin where the occupancy API over-reports
// (MI355X_MICROARCH.md, residency) — the work queue makes any grid correct;
// this only avoids a straggling second round.
template <class K>
static int resident_grid(K kernel, int threads, size_t lds) {
    int dev = 0, per_cu = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 1024;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    return per_cu * prop.multiProcessorCount;
}

hipError_t launch_units(const uint64_t* offs, uint64_t n, uint32_t k, uint32_t step,
                        uint64_t* nk_out, uint64_t* nseg, hipStream_t s) {
    if (n == 0) return hipSuccess;
    units_kernel<<<grid_for(n, 256, 4096), 256, 0, s>>>(offs, n, k, step, nk_out, nseg);
    return hipGetLastError();
}

size_t scan_temp_bytes(uint64_t n) {
    size_t bytes = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr,
                                           (uint64_t*)nullptr, (int)n);
    return bytes;
}

hipError_t launch_scan(void* temp, size_t temp_bytes, const uint64_t* in, uint64_t* out,
                       uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)n, s);
}

hipError_t launch_scatter_units(const uint64_t* nseg, const uint64_t* unit_ofs, uint64_t n,
                                uint32_t* unit_read, uint64_t* queue, uint32_t* hits_zero,
                                uint64_t D, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(queue, 0, 2 * sizeof(uint64_t), s);
    scatter_units_kernel<<<grid_for(n, 256, 4096), 256, 0, s>>>(nseg, unit_ofs, n, unit_read,
                                                               queue, hits_zero, D);
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

// The fast kernel covers classic banks of <= 128 docs whose image fits 32-bit
// row offsets, for the (k, h) pairs XspecT trains (species 21/7, MLST 31/1).
static bool cobs_fast(const CobsView& bv, uint32_t k) {
    return bv.G == 1 && bv.nchunks == 1 && bv.D <= 128 && bv.sig0 <= (1ull << 28) &&
           ((k == 21 && bv.h == 7) || (k == 31 && bv.h == 1));
}

static int load_policy() {
    static const int pol = [] {  // thread-safe one-time init
        const char* e = getenv("XSPECT2_AMD_LOADPOL");
        const int v = e ? atoi(e) : 0;
        return (v < 0 || v > 4) ? 0 : v;
    }();
    return pol;
}

// One grid size per kernel variant, computed on first use.  Banks may be
// queried from several host threads at once, hence the atomics.
template <class F>
static int cached_grid(std::atomic<int>& slot, F compute) {
    int v = slot.load(std::memory_order_relaxed);
    if (!v) {
        v = compute();
        slot.store(v, std::memory_order_relaxed);
    }
    return v;
}

template <int KT, int HT>
static hipError_t launch_fast_t(const ReadView& rv, const FastBank& fb, uint32_t* hits,
                                uint64_t* partials, int blocks, hipStream_t s) {
    switch (load_policy()) {
        case 1: probe_cobs_fast<KT, HT, 1><<<blocks, kProbeThreads, 0, s>>>(rv, fb, hits, partials); break;
        case 2: probe_cobs_fast<KT, HT, 2><<<blocks, kProbeThreads, 0, s>>>(rv, fb, hits, partials); break;
        case 3: probe_cobs_fast<KT, HT, 3><<<blocks, kProbeThreads, 0, s>>>(rv, fb, hits, partials); break;
        case 4: probe_cobs_fast<KT, HT, 4><<<blocks, kProbeThreads, 0, s>>>(rv, fb, hits, partials); break;
        default: probe_cobs_fast<KT, HT, 0><<<blocks, kProbeThreads, 0, s>>>(rv, fb, hits, partials); break;
    }
    return hipGetLastError();
}

template <int KT, int HT>
static hipError_t launch_cobs_t(const ReadView& rv, const CobsView& bv, uint32_t* hits,
                                uint64_t* partials, int blocks, int wpb, size_t lds,
                                uint32_t dpad, hipStream_t s) {
    probe_cobs_kernel<KT, HT><<<blocks, wpb * kWave, lds, s>>>(rv, bv, hits, partials, dpad);
    return hipGetLastError();
}

// Wide kernel chunk lanes for a classic bank of 2..16 data chunks (0: none).
static int wide_for(const CobsView& bv) {
    if (bv.G != 1 || bv.nchunks < 2 || bv.nchunks > 16 || bv.sig0 >= (1ull << 32)) return 0;
    return bv.nchunks == 2 ? 2 : bv.nchunks <= 4 ? 4 : bv.nchunks <= 8 ? 8 : 16;
}

using WideFn = void (*)(ReadView, CobsView, uint32_t*, uint64_t*, uint32_t);

// Two sub-tiles' row loads are issued before counting: measured against one
// and four at D = 200 / 600 / 1000 / 2000 (profiles/r01_wide16.txt).
constexpr int kWideInFlight = 2;

template <int KT, int HT>
static WideFn wide_fn(int c) {
    constexpr int P = kWideInFlight;
    return c == 2 ? probe_cobs_wide<KT, HT, 2, P> : c == 4 ? probe_cobs_wide<KT, HT, 4, P>
         : c == 8 ? probe_cobs_wide<KT, HT, 8, P> : probe_cobs_wide<KT, HT, 16, P>;
}

static WideFn pick_wide(uint32_t k, uint32_t h, int c);

// Slot kernel shape (GM groups x CM chunks) for a bank, or {0, 0} for the
// general kernel: classic rows of more than 8 chunks that the wide kernel does
// not take, compact rows of more than 16 slots.  D <= 16 * 128 follows, so the
// LDS totals need <= 16 KB.
struct SlotShape {
    int gm, cm;
};
static SlotShape slots_for(const CobsView& bv) {
    const uint64_t G = bv.G, c = bv.nchunks;
    if (G == 1) {  // classic rows of 2..16 chunks take the wide kernel first
        if (c <= 4) return {1, 4};
        if (c <= 8) return {1, 8};
        return {0, 0};
    }
    if (c == 1) return G <= 4 ? SlotShape{4, 1} : G <= 8 ? SlotShape{8, 1} : G <= 16 ? SlotShape{16, 1} : SlotShape{0, 0};
    if (c == 2) return G <= 4 ? SlotShape{4, 2} : G <= 8 ? SlotShape{8, 2} : SlotShape{0, 0};
    if (c <= 4) return G <= 2 ? SlotShape{2, 4} : G <= 3 ? SlotShape{3, 4} : G <= 4 ? SlotShape{4, 4} : SlotShape{0, 0};
    return {0, 0};
}

using SlotsFn = void (*)(ReadView, CobsView, uint32_t*, uint64_t*, uint32_t);

template <int KT, int HT>
static SlotsFn slots_fn_classic(SlotShape s) {
    return s.cm == 4 ? probe_cobs_slots<KT, HT, 1, 4> : probe_cobs_slots<KT, HT, 1, 8>;
}

template <int KT, int HT>
static SlotsFn slots_fn(SlotShape s) {
    if (s.gm == 1) return slots_fn_classic<KT, HT>(s);
    if (s.cm == 1) return s.gm == 4 ? probe_cobs_slots<KT, HT, 4, 1> : s.gm == 8 ? probe_cobs_slots<KT, HT, 8, 1>
                                                                                  : probe_cobs_slots<KT, HT, 16, 1>;
    if (s.cm == 2) return s.gm == 4 ? probe_cobs_slots<KT, HT, 4, 2> : probe_cobs_slots<KT, HT, 8, 2>;
    return s.gm == 2 ? probe_cobs_slots<KT, HT, 2, 4> : s.gm == 3 ? probe_cobs_slots<KT, HT, 3, 4>
                                                                  : probe_cobs_slots<KT, HT, 4, 4>;
}

static int kh_variant(uint32_t k, uint32_t h) { return (k == 21 && h == 7) ? 0 : (k == 31 && h == 1) ? 1 : 2; }

static SlotsFn pick_slots(uint32_t k, uint32_t h, SlotShape s) {
    switch (kh_variant(k, h)) {
        case 0: return s.gm == 1 ? slots_fn_classic<21, 7>(s) : slots_fn<0, 0>(s);  // species banks are classic
        case 1: return slots_fn<31, 1>(s);
        default: return slots_fn<0, 0>(s);
    }
}

static WideFn pick_wide(uint32_t k, uint32_t h, int c) {
    switch (kh_variant(k, h)) {
        case 0: return wide_fn<21, 7>(c);
        case 1: return wide_fn<31, 1>(c);
        default: return wide_fn<0, 0>(c);
    }
}

static int shape_index(SlotShape s) {  // 0..12, for the grid cache
    static const int gms[13] = {1, 1, 0, 0, 4, 8, 16, 4, 8, 2, 3, 4, 0};
    static const int cms[13] = {4, 8, 0, 0, 1, 1, 1, 2, 2, 4, 4, 4, 0};
    for (int i = 0; i < 12; ++i)
        if (gms[i] == s.gm && cms[i] == s.cm) return i;
    return 12;
}

static size_t slots_lds(const CobsView& bv) { return (size_t)((bv.D + 127) / 128 * 128) * sizeof(uint64_t); }

// Grid of the probe kernel launch_probe_cobs picks for this bank (partials
// are sized by it).  Cached per variant; every device of a run is an MI355X.
int probe_grid_cobs(const CobsView& bv, uint32_t k) {
    static std::atomic<int> fast21{0}, fast31{0}, generic[3], slots[3][13], wide[3][4];
    if (cobs_fast(bv, k)) {
        if (k == 21) return cached_grid(fast21, [] { return resident_grid(probe_cobs_fast<21, 7, 0>, kProbeThreads, 0); });
        return cached_grid(fast31, [] { return resident_grid(probe_cobs_fast<31, 1, 0>, kProbeThreads, 0); });
    }
    if (const int c = wide_for(bv)) {
        return cached_grid(wide[kh_variant(k, bv.h)][c == 2 ? 0 : c == 4 ? 1 : c == 8 ? 2 : 3],
                           [&] { return resident_grid(pick_wide(k, bv.h, c), kProbeThreads, 16 * c * 64); });
    }
    const SlotShape sh = slots_for(bv);
    if (sh.gm) {
        // LDS is 16 KB at most: residency is set by registers, not by D
        return cached_grid(slots[kh_variant(k, bv.h)][shape_index(sh)],
                           [&] { return resident_grid(pick_slots(k, bv.h, sh), kProbeThreads, 16384); });
    }
    int wpb;
    size_t lds;
    if (probe_blocks(bv.D, &wpb, &lds) != 0) return 0;
    return cached_grid(generic[wpb == 4 ? 0 : wpb == 2 ? 1 : 2],
                       [&] { return resident_grid(probe_cobs_kernel<0, 0>, wpb * kWave, lds); });
}

hipError_t launch_probe_cobs(const ReadView& rv, const CobsView& bv, uint32_t* hits,
                             uint64_t* partials, int blocks, hipStream_t s) {
    if (cobs_fast(bv, rv.k)) {
        FastBank fb;
        fb.rows = bv.rows;
        fb.sig = bv.sig0;
        fb.magic = barrett_magic(bv.sig0);
        fb.D = (uint32_t)bv.D;
        fb.nwords = (uint32_t)((bv.D + 31) / 32);
        fb.image_bytes = (uint32_t)min(bv.sig0 * 16ull, 0xFFFFFFFFull);
        if (rv.k == 21) return launch_fast_t<21, 7>(rv, fb, hits, partials, blocks, s);
        return launch_fast_t<31, 1>(rv, fb, hits, partials, blocks, s);
    }
    if (const int c = wide_for(bv)) {
        const size_t lds = slots_lds(bv);
        pick_wide(rv.k, bv.h, c)<<<blocks, kProbeThreads, lds, s>>>(rv, bv, hits, partials,
                                                                  (uint32_t)(lds / sizeof(uint64_t)));
        return hipGetLastError();
    }
    const SlotShape sh = slots_for(bv);
    if (sh.gm) {
        const size_t lds = slots_lds(bv);
        pick_slots(rv.k, bv.h, sh)<<<blocks, kProbeThreads, lds, s>>>(rv, bv, hits, partials,
                                                                    (uint32_t)(lds / sizeof(uint64_t)));
        return hipGetLastError();
    }
    int wpb;
    size_t lds;
    if (probe_blocks(bv.D, &wpb, &lds) != 0) return hipErrorInvalidValue;
    const uint32_t dpad = (uint32_t)((bv.D + 127) / 128 * 128);
    if (rv.k == 21 && bv.h == 7) return launch_cobs_t<21, 7>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
    if (rv.k == 31 && bv.h == 1) return launch_cobs_t<31, 1>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
    return launch_cobs_t<0, 0>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
}

// Bits tested before the rest (XSPECT2_AMD_BLOOM_SPLIT; 0 = all at once).
static int bloom_split() {
    static const int v = [] {  // thread-safe one-time init
        const char* e = getenv("XSPECT2_AMD_BLOOM_SPLIT");
        const int s = e ? atoi(e) : kBloomSplitDefault;
        return (s == 0 || s == 1 || s == 2 || s == 3) ? s : kBloomSplitDefault;
    }();
    return v;
}

int probe_grid_bloom() {
    static std::atomic<int> cache[4];
    const int sp = bloom_split();
    return cached_grid(cache[sp], [sp] {
        switch (sp) {
            case 1: return resident_grid(probe_bloom_kernel<21, 7, 1>, kProbeThreads, 0);
            case 2: return resident_grid(probe_bloom_kernel<21, 7, 2>, kProbeThreads, 0);
            case 3: return resident_grid(probe_bloom_kernel<21, 7, 3>, kProbeThreads, 0);
            default: return resident_grid(probe_bloom_kernel<21, 7, 0>, kProbeThreads, 0);
        }
    });
}

template <int SPLIT>
static void launch_bloom_t(const ReadView& rv, const BloomView& bv, uint32_t* hits, uint64_t* partials,
                           int blocks, hipStream_t s) {
    if (rv.k == 21 && bv.K == 7)
        probe_bloom_kernel<21, 7, SPLIT><<<blocks, kProbeThreads, 0, s>>>(rv, bv, hits, partials);
    else
        probe_bloom_kernel<0, 0, SPLIT><<<blocks, kProbeThreads, 0, s>>>(rv, bv, hits, partials);
}

hipError_t launch_probe_bloom(const ReadView& rv, const BloomView& bv, uint32_t* hits,
                              uint64_t* partials, int blocks, hipStream_t s) {
    switch (bloom_split()) {
        case 1: launch_bloom_t<1>(rv, bv, hits, partials, blocks, s); break;
        case 2: launch_bloom_t<2>(rv, bv, hits, partials, blocks, s); break;
        case 3: launch_bloom_t<3>(rv, bv, hits, partials, blocks, s); break;
        default: launch_bloom_t<0>(rv, bv, hits, partials, blocks, s); break;
    }
    return hipGetLastError();
}

hipError_t launch_reduce_partials(const uint64_t* partials, int blocks, uint64_t cols,
                                  uint64_t* totals, hipStream_t s) {
    reduce_partials_kernel<<<grid_for(cols, 1, 4096), 256, 0, s>>>(partials, blocks, cols, totals);
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

hipError_t launch_best_doc(const uint32_t* hits, uint64_t n, uint64_t D, uint32_t* best,
                           uint32_t* best_hits, hipStream_t s) {
    if (n == 0 || D == 0) return hipSuccess;
    best_doc_kernel<<<grid_for(n, 4, 16384), 256, 0, s>>>(hits, n, D, best, best_hits);
    return hipGetLastError();
}

hipError_t launch_gather_reads(const uint8_t* seqs, const uint64_t* offs, const uint32_t* index, uint64_t m,
                               uint8_t* out, const uint64_t* out_offs, hipStream_t s) {
    if (m == 0) return hipSuccess;
    gather_reads_kernel<<<grid_for(m, 4, 16384), 256, 0, s>>>(seqs, offs, index, m, out, out_offs);
    return hipGetLastError();
}

}  // namespace xs
