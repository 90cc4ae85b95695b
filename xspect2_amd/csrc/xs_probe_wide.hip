// xs_probe_wide.hip — COBS probe with C chunk lanes per k-mer: classic banks of 129..2048 docs,
// compact banks of 2..4 groups of 2..4-chunk pages (MLST loci).
#include "xs_device.h"

namespace xs {

// ------------------------------------------------------------------ COBS probe (wide rows)
// Classic banks of 129..2048 docs, and compact banks of GM = 2..4 groups
// (each group's rows probed the same way, group g's docs at g * 8 * page).  A
// row is C 16-byte chunks (C = 2, 4, 8 or 16, the next power of two of its
// data chunks; the pitch is padded so a row is one 128-byte line, or two
// aligned lines at C = 16).  Hashing stays one lane per k-mer, but the gathers
// run C lanes per k-mer: in sub-tile s, lane l loads chunk l % C of k-mer
// s * (64 / C) + l / C.  One load instruction then reads 64 / C whole rows, so
// the vector L1 sees each row line once instead of once per chunk.
// Counting: after the 32x32 transpose of a 32-lane half, bit r of lane t is
// lane r's bit t, and lanes r = c (mod C) hold chunk c: one masked popcount
// per chunk.
template <int C>
struct ChunkLanes {  // bits r of a 32-row column with r % C == 0
    static constexpr uint32_t m0 = C == 2 ? 0x55555555u : C == 4 ? 0x11111111u : C == 8 ? 0x01010101u : 0x00010001u;
};

// Min blocks per CU = waves per SIMD the register budget is sized for.  4/5/6
// force spills and run slower on every workload (profiles/r01_wide_occupancy.txt).
constexpr int kWideMinBlocks = 2;
template <int KT, int HT, int C, int P, int GM>
__global__ void __launch_bounds__(kProbeThreads, kWideMinBlocks) probe_cobs_wide(ReadView rv, CobsView bv,
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
    const uint32_t cpg = bv.nchunks;   // data chunks per group, <= C (host-checked)
    const uint64_t gdocs = 8 * bv.page;  // docs per group
    GroupDesc gd[GM];                  // G == GM, every sig < 2^30 (host-checked): 32-bit row indices
#pragma unroll
    for (int g = 0; g < GM; ++g) gd[g] = bv.groups[g];
    const uint32_t pitch = bv.pitch;
    const int my_c = lane % C, my_slot = lane / C;
    const bool my_chunk_on = (uint32_t)my_c < cpg;
    const uint32_t my_c_ofs = my_chunk_on ? (uint32_t)my_c * 16 : 0;
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
            // group g, chunk cc, words q: 16-bit counters, reg [g][2*cc + (q >> 1)]
            uint32_t acc[GM][2 * C];
#pragma unroll
            for (int g = 0; g < GM; ++g)
#pragma unroll
                for (int i = 0; i < 2 * C; ++i) acc[g][i] = 0;

            for (uint32_t tb = 0; tb < cnt; tb += 64) {
                const bool act = tb + lane < cnt;
                uint32_t ri[GM][NH];  // row index of hash j in group g
#pragma unroll
                for (int g = 0; g < GM; ++g)
#pragma unroll
                    for (int j = 0; j < NH; ++j) ri[g][j] = 0;
                if (act) {
                    Kmer c;
                    kmer_at<KT, kKmerCobs>(rv, o0, len, (t0 + tb + lane) * step, k, c);
                    Xxh64Pre pre;
                    xxh64_pre<KT>(c, k, pre);
#pragma unroll
                    for (int j = 0; j < NH; ++j)
                        if ((uint32_t)j < h) {
                            const uint64_t hv = xxh64_seed<KT>(c, pre, k, (uint64_t)j);
#pragma unroll
                            for (int g = 0; g < GM; ++g) ri[g][j] = fastmod_small(hv, (uint32_t)gd[g].sig, gd[g].magic);
                        }
                }
                const uint32_t tile = min(64u, cnt - tb);
#pragma unroll
                for (int s0 = 0; s0 < C; s0 += P) {
                    if ((uint32_t)(s0 * K) >= tile) continue;  // uniform
                    // P sub-tiles' row chunks of every group in flight before any
                    // counting.  The loads are unconditional (a lane without a
                    // k-mer has row 0, a lane past the data chunks reads chunk 0)
                    // and masked afterwards: a load under a divergent branch
                    // would be waited for before the branch joins, one row at a time.
                    uint4 mm[P][GM];
#pragma unroll
                    for (int p = 0; p < P; ++p) {
                        const int src = (s0 + p) * K + my_slot;
                        const bool on = (uint32_t)src < tile && my_chunk_on;
#pragma unroll
                        for (int g = 0; g < GM; ++g) {
                            const uint8_t* rows = bv.rows + gd[g].base;
                            uint4 v[NH];
#pragma unroll
                            for (int j = 0; j < NH; ++j) {
                                if ((uint32_t)j >= h) continue;
                                const uint32_t rj = (uint32_t)__shfl((int)ri[g][j], src, 64);
                                v[j] = *reinterpret_cast<const uint4*>(rows + (uint64_t)rj * pitch + my_c_ofs);
                            }
                            uint4 m = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
                            for (int j = 0; j < NH; ++j)
                                if ((uint32_t)j < h) m = and4(m, v[j]);
                            mm[p][g] = on ? m : make_uint4(0u, 0u, 0u, 0u);
                        }
                    }
#pragma unroll
                    for (int p = 0; p < P; ++p) {
#pragma unroll
                        for (int g = 0; g < GM; ++g) {
                            const uint32_t w[4] = {mm[p][g].x, mm[p][g].y, mm[p][g].z, mm[p][g].w};
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
#ifdef XS_WIDE_NOCOUNT  // measurement-only build: loads consumed, counting skipped (wrong hits)
                                acc[g][q] ^= w[q];
                                continue;
#endif
                                if (__ballot(w[q] != 0u) == 0ull) continue;
                                const uint32_t x = xpose32(w[q], X);
#pragma unroll
                                for (int cc = 0; cc < C; ++cc)
                                    acc[g][2 * cc + (q >> 1)] += (uint32_t)__popc(x & (M0 << cc)) << (16 * (q & 1));
                            }
                        }
                    }
                }
            }
            // lane t < 32 holds doc g * gdocs + 128 cc + 32 q + t after folding the halves
            const bool whole = nk <= kSegKmers;
#pragma unroll
            for (int g = 0; g < GM; ++g) {
#pragma unroll
                for (int cc = 0; cc < C; ++cc) {
                    if ((uint32_t)cc >= cpg) continue;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint64_t l0 = (uint64_t)cc * 128 + q * 32;  // doc within the group
                        const uint64_t d0 = (uint64_t)g * gdocs + l0;
                        if (l0 >= gdocs || d0 >= D) continue;
                        const uint32_t v = fold_halves((acc[g][2 * cc + (q >> 1)] >> (16 * (q & 1))) & 0xFFFFu);
                        const uint64_t d = d0 + (uint64_t)lane;
                        if (lane < 32 && l0 + lane < gdocs && d < D) {
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

// ------------------------------------------------------------------ launch
// Wide kernel chunk lanes for a bank (0: not taken): classic banks of 2..16
// data chunks; compact banks of 2..4 groups whose pages are 2..4 chunks (MLST
// loci: 3 groups of 64-byte pages).
int wide_for(const CobsView& bv) {
    if (bv.G < 1 || bv.G > 4 || bv.nchunks < 2 || bv.sig_max >= (1ull << 30)) return 0;  // fastmod_small
    if (bv.G == 1 && bv.nchunks > 16) return 0;
    if (bv.G > 1 && bv.nchunks > 4) return 0;
    return bv.nchunks == 2 ? 2 : bv.nchunks <= 4 ? 4 : bv.nchunks <= 8 ? 8 : 16;
}

using WideFn = void (*)(ReadView, CobsView, uint32_t*, uint64_t*, uint32_t);

// Two sub-tiles' row loads are issued before counting: measured against one
// and four at D = 200 / 600 / 1000 / 2000 (profiles/r01_wide16.txt) and on
// MLST loci (3 groups: 5.67 / 5.42 / 6.29 ms for 1 / 2 / 4; r01_wide_compact.txt).
constexpr int kWideInFlight = 2;

template <int KT, int HT, int GM>
static WideFn wide_fn_groups(int c) {
    constexpr int P = kWideInFlight;
    return c == 2 ? probe_cobs_wide<KT, HT, 2, P, GM> : probe_cobs_wide<KT, HT, 4, P, GM>;
}

template <int KT, int HT>
static WideFn wide_fn(int c, uint32_t G) {
    constexpr int P = kWideInFlight;
    if (G == 2) return wide_fn_groups<KT, HT, 2>(c);
    if (G == 3) return wide_fn_groups<KT, HT, 3>(c);
    if (G == 4) return wide_fn_groups<KT, HT, 4>(c);
    return c == 2 ? probe_cobs_wide<KT, HT, 2, P, 1> : c == 4 ? probe_cobs_wide<KT, HT, 4, P, 1>
         : c == 8 ? probe_cobs_wide<KT, HT, 8, P, 1> : probe_cobs_wide<KT, HT, 16, P, 1>;
}

static WideFn pick_wide(uint32_t k, uint32_t h, int c, uint32_t G) {
    switch (kh_variant(k, h)) {
        case 0: return G == 1 ? wide_fn<21, 7>(c, 1) : wide_fn<0, 0>(c, G);  // species banks are classic
        case 1: return wide_fn<31, 1>(c, G);
        default: return wide_fn<0, 0>(c, G);
    }
}

int grid_cobs_wide(const CobsView& bv, uint32_t k) {
    static std::atomic<int> wide[3][4][4];  // (k, h) variant x G x C
    const int c = wide_for(bv);
    return cached_grid(wide[kh_variant(k, bv.h)][bv.G - 1][c == 2 ? 0 : c == 4 ? 1 : c == 8 ? 2 : 3], [&] {
        return resident_grid(pick_wide(k, bv.h, c, bv.G), kProbeThreads, slots_lds(bv) > 8192 ? 16384 : 8192);
    });
}

hipError_t launch_cobs_wide(const ReadView& rv, const CobsView& bv, uint32_t* hits, uint64_t* partials,
                            int blocks, hipStream_t s) {
    const size_t lds = slots_lds(bv);
    pick_wide(rv.k, bv.h, wide_for(bv), bv.G)<<<blocks, kProbeThreads, lds, s>>>(
        rv, bv, hits, partials, (uint32_t)(lds / sizeof(uint64_t)));
    return hipGetLastError();
}

}  // namespace xs
