// xs_device.h — device helpers shared by the gfx950 kernel translation units
// (hashing, k-mer assembly, the unit queue, column-popcount counting) and the
// host-side launch helpers.  Internal; included only by the .hip sources.
#pragma once
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

// 64-bit rotate as two v_alignbit_b32 (the shift/or form compiles to three
// instructions, one of them a 64-bit shift); r is a constant at every call.
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if (r & 32) {
        const uint32_t t = lo;
        lo = hi;
        hi = t;
    }
    if ((r & 31) == 0) return ((uint64_t)hi << 32) | lo;
    const uint32_t s = 32 - (r & 31);
    return ((uint64_t)__builtin_amdgcn_alignbit(hi, lo, s) << 32) | __builtin_amdgcn_alignbit(lo, hi, s);
}

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
// The same for d < 2^30: the remainder before correction is below 3d < 2^32,
// so x - q*d is exact in 32 bits (the high words cancel) and the corrections
// are 32-bit compares.  Callers check d on the host.
__device__ __forceinline__ uint32_t fastmod_small(uint64_t x, uint32_t d, uint64_t m) {
    uint32_t r = (uint32_t)x - (uint32_t)__umul64hi(x, m) * d;
    r = r >= d ? r - d : r;
    return r >= d ? r - d : r;
}

// One step of the 128-bit LCG (state sh:sl): state = state * M + C mod 2^128.
// sl * Ml is formed once from four 32 x 32 partial products and gives both
// the low word and the carry into the high word.
__device__ __forceinline__ void lcg_step(uint64_t& sl, uint64_t& sh) {
    constexpr uint64_t ml = (uint32_t)kLcgMl, mh = kLcgMl >> 32;
    const uint64_t al = (uint32_t)sl, ah = sl >> 32;
    const uint64_t ll = al * ml, lh = al * mh, hl = ah * ml, hh = ah * mh;
    const uint64_t mid = (ll >> 32) + (uint32_t)lh + (uint32_t)hl;  // < 3 * 2^32
    const uint64_t plo = (mid << 32) | (uint32_t)ll;
    const uint64_t phi = hh + (lh >> 32) + (hl >> 32) + (mid >> 32);
    const uint64_t nl = plo + kLcgCl;
    sh = sh * kLcgMl + sl * kLcgMh + phi + kLcgCh + (nl < plo);
    sl = nl;
}

// The LCG's j-th state from a 64-bit start h (high word 0, as every rbloom index
// sequence starts): state_j = A_j * h + B_j mod 2^128 with A_j = M^j and
// B_j = C (M^(j-1) + ... + 1), constants folded at compile time.  Only the high
// word is needed; each j is independent of the others (no chain), and the
// product has a 64-bit factor: 7 multiplies instead of lcg_step's 10.
struct LcgJump {
    uint64_t ah, al, bh, bl;
};
constexpr LcgJump lcg_jump(int j) {
    unsigned __int128 m = ((unsigned __int128)kLcgMh << 64) | kLcgMl;
    unsigned __int128 c = ((unsigned __int128)kLcgCh << 64) | kLcgCl;
    unsigned __int128 a = 1, b = 0;
    for (int i = 0; i < j; ++i) {
        a = a * m;
        b = b * m + c;
    }
    return LcgJump{(uint64_t)(a >> 64), (uint64_t)a, (uint64_t)(b >> 64), (uint64_t)b};
}
template <int J>
__device__ __forceinline__ uint64_t lcg_high(uint64_t h) {
    constexpr LcgJump t = lcg_jump(J);
    constexpr uint64_t a0 = (uint32_t)t.al, a1 = t.al >> 32;
    const uint64_t h0 = (uint32_t)h, h1 = h >> 32;
    // al * h, full 128 bits, from four 32 x 32 partial products
    const uint64_t ll = a0 * h0, lh = a0 * h1, hl = a1 * h0, hh = a1 * h1;
    const uint64_t mid = (ll >> 32) + (uint32_t)lh + (uint32_t)hl;  // < 3 * 2^32
    const uint64_t plo = (mid << 32) | (uint32_t)ll;
    const uint64_t phi = hh + (lh >> 32) + (hl >> 32) + (mid >> 32);
    const uint64_t lo = plo + t.bl;
    return phi + t.ah * h + t.bh + (lo < plo);
}
// j = 1 .. 8 (a constant once the caller's loop is unrolled)
__device__ __forceinline__ uint64_t lcg_high_n(uint64_t h, int j) {
    switch (j) {
        case 1: return lcg_high<1>(h);
        case 2: return lcg_high<2>(h);
        case 3: return lcg_high<3>(h);
        case 4: return lcg_high<4>(h);
        case 5: return lcg_high<5>(h);
        case 6: return lcg_high<6>(h);
        case 7: return lcg_high<7>(h);
        default: return lcg_high<8>(h);
    }
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

// 0x80 in every byte of x that is A, C, G, T or N.  Their low 3 bits (1, 3,
// 7, 4, 6) are distinct, so v_perm_b32 looks up the one byte each could be
// in an 8-byte table {-, 'A', -, 'C', 'T', -, 'N', 'G'} (- = 0xFF, which no
// byte with those low bits equals) and the byte must equal its entry.
__device__ __forceinline__ uint32_t acgtn_bytes(uint32_t x) {
    return zero_bytes(__builtin_amdgcn_perm(0x474EFF54u, 0x43FF41FFu, x & 0x07070707u) ^ x);
}

// COBS normalisation of 4 bytes.  (b & 0xDF) is one of A/C/G/T only for
// A/C/G/T/a/c/g/t, so the upper-cased test is exact.  A, C, G, T have the
// distinct low 3 bits 1, 3, 7, 4: as in acgtn_bytes, v_perm_b32 looks up the
// one letter an upper-cased byte could be in {-, 'A', -, 'C', 'T', -, -, 'G'}
// (- = 0xFF) and the byte must equal it.
__device__ __forceinline__ uint32_t acgt_bytes(uint32_t u) {
    return zero_bytes(__builtin_amdgcn_perm(0x47FFFF54u, 0x43FF41FFu, u & 0x07070707u) ^ u);
}
__device__ __forceinline__ uint32_t cobs_norm4(uint32_t x) {
    const uint32_t u = x & 0xDFDFDFDFu;
    const uint32_t m = (acgt_bytes(u) >> 7) * 0xFFu;
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
    // global address space: plain global loads, counted on vmcnt only
    const __attribute__((address_space(1))) uint32_t* p =
        reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uintptr_t lim = reinterpret_cast<uintptr_t>(seq) + seq_bytes;
    const uint32_t nw = KT ? (KT + 3) / 4 : (k + 3) / 4;
    uint32_t raw[9];
    if (reinterpret_cast<uintptr_t>(p + nw) < lim) {  // every dword starts inside the buffer: no per-load guard
#pragma unroll
        for (int i = 0; i < 9; ++i) raw[i] = i <= (int)nw ? p[i] : 0u;
    } else {
#pragma unroll
        for (int i = 0; i < 9; ++i)
            raw[i] = (i <= (int)nw && reinterpret_cast<uintptr_t>(p + i) < lim) ? p[i] : 0u;
    }
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

// Hand out `grab` units per atomic (ReadView::grab: 4 balances ragged reads
// across waves; a small request takes 1, so every unit gets a wave).
__device__ __forceinline__ uint64_t grab_units(uint64_t* queue, int lane, uint32_t grab) {
    uint64_t base = 0;
    if (lane == 0) base = atomicAdd(reinterpret_cast<unsigned long long*>(queue + 1), (unsigned long long)grab);
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
            const uint32_t ok = acgtn_bytes(f[i]);
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

// ------------------------------------------------------------------ host launch helpers
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

inline int kh_variant(uint32_t k, uint32_t h) { return (k == 21 && h == 7) ? 0 : (k == 31 && h == 1) ? 1 : 2; }


// Bytes of the per-block doc totals (u64) the multi-chunk COBS kernels keep in LDS.
inline size_t slots_lds(const CobsView& bv) { return (size_t)((bv.D + 127) / 128 * 128) * sizeof(uint64_t); }

// ---- COBS probe families (one translation unit each) ---------------------
// xs_probe_fast.hip: classic D <= 128, species (21, 7) / MLST (31, 1)
bool cobs_fast(const CobsView& bv, uint32_t k);
int grid_cobs_fast(uint32_t k);
hipError_t launch_cobs_fast(const ReadView& rv, const CobsView& bv, uint32_t* hits, uint64_t* partials,
                            int blocks, hipStream_t s);
// xs_probe_wide.hip: classic rows of 2..16 chunks (0 = not taken)
int wide_for(const CobsView& bv);
int grid_cobs_wide(const CobsView& bv, uint32_t k);
hipError_t launch_cobs_wide(const ReadView& rv, const CobsView& bv, uint32_t* hits, uint64_t* partials,
                            int blocks, hipStream_t s);
// xs_probe_vslice.hip: compact, one hash, 3-4 groups of 64-byte pages (MLST loci)
bool vslice_take(const CobsView& bv);
int grid_cobs_vslice(const CobsView& bv, uint32_t k);
hipError_t launch_cobs_vslice(const ReadView& rv, const CobsView& bv, uint32_t* hits, uint64_t* partials,
                              int blocks, hipStream_t s);
// xs_probe_slots.hip: compile-time group x chunk layouts (false = not taken)
bool slots_take(const CobsView& bv);
int grid_cobs_slots(const CobsView& bv, uint32_t k);
hipError_t launch_cobs_slots(const ReadView& rv, const CobsView& bv, uint32_t* hits, uint64_t* partials,
                             int blocks, hipStream_t s);
// xs_probe_general.hip: anything the LDS counters hold
int grid_cobs_general(const CobsView& bv);
hipError_t launch_cobs_general(const ReadView& rv, const CobsView& bv, uint32_t* hits, uint64_t* partials,
                               int blocks, hipStream_t s);

}  // namespace xs
