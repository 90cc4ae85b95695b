// xs_probe_vslice.hip — COBS probe of banks of 1-4 groups of 64-byte pages with one hash
// (MLST loci of up to 2048 alleles), counting with bit-sliced adders.
#include "xs_device.h"

namespace xs {

// ------------------------------------------------------------------ COBS probe (bit-sliced)
// One wavefront per unit (<= kSegKmers k-mers of one read), as the other
// probes.  Hashing is one lane per k-mer.  Counting is one lane per 32 docs:
// a k-mer's G rows are one dword load across G * 16 lanes (each row one line),
// and each lane adds its word into a bit-sliced counter of its 32 docs.  With
// G = 1 or 2 the wave holds S = 4 or 2 such lane sets, each taking every S-th
// k-mer (slot, group, word = lane / 16G, lane / 16 % G, lane % 16); their
// counts are summed at the end.  Carry-save adders
// (Harley-Seal: 15 per 16 k-mers, 2 VALU each) put the whole k-mer's G * 512
// docs at ~2 VALU, where probe_cobs_wide's column-popcount transpose takes ~27
// VALU per 32-doc word and ran at the VALU issue limit on MLST loci
// (profiles/r06_pmc_mlst_wide.json: 2.97e9 VALU instructions per locus call,
// 0.94 of the issue rate).  At the end of a unit four 8x8 bit transposes per
// lane turn the planes into byte counts; they go through LDS in doc order, so
// the hit row is stored 64 consecutive docs per instruction.
constexpr int kVsBatch = 16;       // k-mers per carry-save round (row loads in flight per lane)
constexpr int kVsMinBlocks = 6;    // waves per SIMD the register budget is sized for (LDS allows 6-7)

// carry-save add of three bit vectors: hi = majority, lo = parity (one
// three-input v_bitop3_b32 each on gfx950)
__device__ __forceinline__ void csa(uint32_t& hi, uint32_t& lo, uint32_t a, uint32_t b, uint32_t c) {
    hi = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);  // truth table: two or three inputs set
    lo = __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // an odd number set
}

// Harley-Seal round: 16 words into the (ones, twos, fours, eights) state; the
// returned word carries weight 16.
__device__ __forceinline__ uint32_t hs16(uint32_t& ones, uint32_t& twos, uint32_t& fours, uint32_t& eights,
                                         const uint32_t (&x)[kVsBatch]) {
    uint32_t ta, tb, fa, fb, ea, eb, sixteens;
    csa(ta, ones, ones, x[0], x[1]);
    csa(tb, ones, ones, x[2], x[3]);
    csa(fa, twos, twos, ta, tb);
    csa(ta, ones, ones, x[4], x[5]);
    csa(tb, ones, ones, x[6], x[7]);
    csa(fb, twos, twos, ta, tb);
    csa(ea, fours, fours, fa, fb);
    csa(ta, ones, ones, x[8], x[9]);
    csa(tb, ones, ones, x[10], x[11]);
    csa(fa, twos, twos, ta, tb);
    csa(ta, ones, ones, x[12], x[13]);
    csa(tb, ones, ones, x[14], x[15]);
    csa(fb, twos, twos, ta, tb);
    csa(eb, fours, fours, fa, fb);
    csa(sixteens, eights, eights, ea, eb);
    return sixteens;
}

// Transpose of the 8x8 bit matrix whose row i is byte i of (lo, hi): byte j of
// the result holds bit j of every row, row i at bit i.
__device__ __forceinline__ void xpose8x8(uint32_t& lo, uint32_t& hi) {
    uint32_t t;
    t = (lo ^ (lo >> 7)) & 0x00AA00AAu;
    lo ^= t ^ (t << 7);
    t = (hi ^ (hi >> 7)) & 0x00AA00AAu;
    hi ^= t ^ (t << 7);
    t = (lo ^ (lo >> 14)) & 0x0000CCCCu;
    lo ^= t ^ (t << 14);
    t = (hi ^ (hi >> 14)) & 0x0000CCCCu;
    hi ^= t ^ (t << 14);
    const uint32_t l2 = (lo & 0x0F0F0F0Fu) | ((hi << 4) & 0xF0F0F0F0u);
    hi = (hi & 0xF0F0F0F0u) | ((lo >> 4) & 0x0F0F0F0Fu);
    lo = l2;
}

// Eight bit planes (weights 1..128) of 32 docs -> 32 byte counts, doc b at byte b.
__device__ __forceinline__ void planes_to_bytes(const uint32_t (&p)[8], uint32_t (&out)[8]) {
    // a[q]: bytes (p[2q].b0, p[2q+1].b0, p[2q].b1, p[2q+1].b1), c[q]: the same for bytes 2, 3
    uint32_t a[4], c[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        a[q] = __builtin_amdgcn_perm(p[2 * q + 1], p[2 * q], 0x05010400u);
        c[q] = __builtin_amdgcn_perm(p[2 * q + 1], p[2 * q], 0x07030602u);
    }
    // byte k of every plane, planes 0..3 in lo and 4..7 in hi, transposed to docs 8k..8k+7
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t* s = k < 2 ? a : c;
        const uint32_t sel = (k & 1) ? 0x07060302u : 0x05040100u;
        uint32_t lo = __builtin_amdgcn_perm(s[1], s[0], sel);
        uint32_t hi = __builtin_amdgcn_perm(s[3], s[2], sel);
        xpose8x8(lo, hi);
        out[2 * k] = lo;
        out[2 * k + 1] = hi;
    }
}

template <int KT, int GM>
__global__ void __launch_bounds__(kProbeThreads, kVsMinBlocks) probe_cobs_vslice(ReadView rv, CobsView bv,
                                                                                 uint32_t* __restrict__ hits,
                                                                                 uint64_t* __restrict__ partials) {
    constexpr int kDocs = GM * 512;  // docs of the bank's groups (D <= kDocs)
    constexpr int kWaves = kProbeThreads / kWave;
    constexpr int LW = GM * 16;                         // lanes per k-mer
    constexpr int S = GM == 1 ? 4 : GM == 2 ? 2 : 1;    // k-mer slots per wave
    constexpr int SK = kWave / S;                       // k-mers per slot per tile
    static_assert(GM >= 1 && GM <= 4 && S * kDocs <= kWave * 32, "counts of every slot fit the LDS buffer");
    // per wave: the tile's row offsets [group][slot][k-mer] while counting, then
    // the unit's byte counts [slot][doc] (the same bytes: one wave uses one at a time)
    __shared__ __attribute__((aligned(16))) uint32_t s_buf[kWaves][kWave * 8];
    __shared__ uint32_t s_p256[kWaves][kWave];  // weight-256 plane (a doc hit by all 256 k-mers of a unit)
    __shared__ uint64_t s_tot[kDocs];
    __shared__ uint64_t s_kmers[kWaves];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    for (int d = threadIdx.x; d < kDocs; d += kProbeThreads) s_tot[d] = 0;
    __syncthreads();

    const uint32_t k = KT ? KT : rv.k;
    const uint32_t step = rv.step;
    const uint32_t D = (uint32_t)bv.D;
    GroupDesc gd[GM];
#pragma unroll
    for (int g = 0; g < GM; ++g) gd[g] = bv.groups[g];
    // counting lane: slot my_slot, group my_g (at G = 3, lanes 48-63 repeat slot 0 group 0; their
    // counts land past the docs and are never read)
    const int my_slot = min(lane / LW, S - 1);
    const int my_g = min((lane % LW) >> 4, GM - 1);
    uint32_t my_base = (uint32_t)gd[0].base;
#pragma unroll
    for (int g = 1; g < GM; ++g)
        if (my_g == g) my_base = (uint32_t)gd[g].base;
    my_base += (uint32_t)(lane & 15) * 4u;
    const uint8_t* rows = bv.rows;
    uint8_t* s_cnt = reinterpret_cast<uint8_t*>(&s_buf[wid][0]);
    const uint64_t U = rv.queue[0];
    uint64_t kmer_total = 0;

    for (;;) {
        const uint64_t base = grab_units(rv.queue, lane, rv.grab);
        if (base >= U) break;
        const uint64_t uend = min(base + rv.grab, U);
        for (uint64_t u = base; u < uend; ++u) {
            const uint32_t r = rv.unit_read[u];
            const uint64_t seg = u - rv.unit_ofs[r];
            const uint64_t o0 = rv.offs[r];
            const uint64_t len = rv.offs[r + 1] - o0;
            const uint64_t nk = num_kmers(len, k, step);
            const uint64_t t0 = seg * kSegKmers;
            const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
            kmer_total += cnt;
            uint32_t ones = 0, twos = 0, fours = 0, eights = 0;
            uint32_t p16 = 0, p32 = 0, p64 = 0, p128 = 0, p256 = 0;
            for (uint32_t tb = 0; tb < cnt; tb += 64) {
                const uint32_t tile = min(64u, cnt - tb);
                uint32_t ri[GM];
#pragma unroll
                for (int g = 0; g < GM; ++g) ri[g] = 0;  // past the tile: row 0, loaded and dropped
                if ((uint32_t)lane < tile) {
                    Kmer c;
                    kmer_at<KT, kKmerCobs>(rv, o0, len, (t0 + tb + lane) * step, k, c);
                    Xxh64Pre pre;
                    xxh64_pre<KT>(c, k, pre);
                    const uint64_t hv = xxh64_seed<KT>(c, pre, k, 0);
#pragma unroll
                    for (int g = 0; g < GM; ++g) ri[g] = fastmod_small(hv, (uint32_t)gd[g].sig, gd[g].magic);
                }
                __builtin_amdgcn_wave_barrier();  // the previous unit's count reads are done
#pragma unroll
                for (int g = 0; g < GM; ++g) s_buf[wid][g * 64 + (lane % S) * SK + lane / S] = ri[g] * 64u;
                __builtin_amdgcn_wave_barrier();
                const uint32_t per_slot = (tile + S - 1) / S;
                for (uint32_t u0 = 0; u0 < per_slot; u0 += kVsBatch) {
                    const uint4* src = reinterpret_cast<const uint4*>(&s_buf[wid][my_g * 64 + my_slot * SK + u0]);
                    uint32_t x[kVsBatch];
#pragma unroll
                    for (int q = 0; q < kVsBatch / 4; ++q) {
                        const uint4 o = src[q];
                        x[4 * q + 0] = *reinterpret_cast<const uint32_t*>(rows + (my_base + o.x));
                        x[4 * q + 1] = *reinterpret_cast<const uint32_t*>(rows + (my_base + o.y));
                        x[4 * q + 2] = *reinterpret_cast<const uint32_t*>(rows + (my_base + o.z));
                        x[4 * q + 3] = *reinterpret_cast<const uint32_t*>(rows + (my_base + o.w));
                    }
                    if ((u0 + kVsBatch) * S > tile) {  // uniform: the k-mers past the tile add nothing
#pragma unroll
                        for (int q = 0; q < kVsBatch; ++q)
                            if ((u0 + q) * S + my_slot >= tile) x[q] = 0;
                    }
                    uint32_t carry = hs16(ones, twos, fours, eights, x), t;
                    t = p16 & carry; p16 ^= carry; carry = t;
                    t = p32 & carry; p32 ^= carry; carry = t;
                    t = p64 & carry; p64 ^= carry; carry = t;
                    t = p128 & carry; p128 ^= carry; carry = t;
                    p256 |= carry;  // <= 256 k-mers per slot: set only for a count of exactly 256 (S = 1)
                }
            }
            const uint32_t pl[8] = {ones, twos, fours, eights, p16, p32, p64, p128};
            uint32_t b[8];
            planes_to_bytes(pl, b);
            const bool any256 = __ballot(p256 != 0u) != 0ull;
            __builtin_amdgcn_wave_barrier();  // every lane has read its row indices
            uint4* dst = reinterpret_cast<uint4*>(s_cnt + lane * 32);
            dst[0] = make_uint4(b[0], b[1], b[2], b[3]);
            dst[1] = make_uint4(b[4], b[5], b[6], b[7]);
            if (any256) s_p256[wid][lane] = p256;
            __builtin_amdgcn_wave_barrier();
            const bool whole = nk <= kSegKmers;
            uint32_t* hrow = hits ? hits + (uint64_t)r * D : nullptr;
            for (uint32_t d = (uint32_t)lane; d < D; d += 64) {
                uint32_t v = s_cnt[d];
#pragma unroll
                for (int sl = 1; sl < S; ++sl) v += s_cnt[sl * kDocs + d];
                if (any256) v += ((s_p256[wid][d >> 5] >> (d & 31)) & 1u) << 8;
                if (v) atomicAdd(reinterpret_cast<unsigned long long*>(&s_tot[d]), (unsigned long long)v);
                if (hrow) {
                    if (whole) hrow[d] = v;
                    else if (v) atomicAdd(&hrow[d], v);
                }
            }
        }
    }
    if (lane == 0) s_kmers[wid] = kmer_total;
    __syncthreads();
    if (partials) {
        uint64_t* out = partials + (uint64_t)blockIdx.x * (D + 1);
        for (uint32_t d = threadIdx.x; d < D; d += kProbeThreads) out[d] = s_tot[d];
        if (threadIdx.x == 0) {
            uint64_t s = 0;
            for (int w = 0; w < kWaves; ++w) s += s_kmers[w];
            out[D] = s;
        }
    }
}

// ------------------------------------------------------------------ launch
// Banks of 1-4 groups of 64-byte pages (512 docs each) with one hash, whose
// image fits 32-bit offsets: XspecT's MLST loci of up to 2048 alleles.
bool vslice_take(const CobsView& bv) {
    return bv.G >= 1 && bv.G <= 4 && bv.h == 1 && bv.page == 64 && bv.pitch == 64 && bv.D <= bv.G * 512ull &&
           bv.sig_max < (1ull << 30) && (uint64_t)bv.G * bv.sig_max * 64 < (1ull << 32);
}

using VsFn = void (*)(ReadView, CobsView, uint32_t*, uint64_t*);

template <int KT>
static VsFn pick_vslice_g(uint32_t G) {
    return G == 1 ? probe_cobs_vslice<KT, 1> : G == 2 ? probe_cobs_vslice<KT, 2>
         : G == 3 ? probe_cobs_vslice<KT, 3> : probe_cobs_vslice<KT, 4>;
}

static VsFn pick_vslice(uint32_t k, uint32_t G) { return k == 31 ? pick_vslice_g<31>(G) : pick_vslice_g<0>(G); }

int grid_cobs_vslice(const CobsView& bv, uint32_t k) {
    static std::atomic<int> grid[2][4];  // k == 31 x G
    return cached_grid(grid[k == 31 ? 0 : 1][bv.G - 1],
                       [&] { return resident_grid(pick_vslice(k, bv.G), kProbeThreads, 0); });
}

hipError_t launch_cobs_vslice(const ReadView& rv, const CobsView& bv, uint32_t* hits, uint64_t* partials,
                              int blocks, hipStream_t s) {
    pick_vslice(rv.k, bv.G)<<<blocks, kProbeThreads, 0, s>>>(rv, bv, hits, partials);
    return hipGetLastError();
}

}  // namespace xs
