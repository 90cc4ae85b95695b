// xs_probe_slots.hip — COBS probe with a compile-time group x chunk row layout (MLST loci, compact banks).
#include "xs_device.h"

namespace xs {

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
    const uint32_t G = bv.G;               // <= GM (host-checked)
    const uint32_t cpg = bv.nchunks;       // <= CM (host-checked)
    const uint64_t gdocs = 8 * bv.page;    // docs per group
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
                uint4 mk[NS];
#pragma unroll
                for (int g = 0; g < GM; ++g) {
                    uint64_t ro[NH];
#pragma unroll
                    for (int j = 0; j < NH; ++j) ro[j] = 0;
                    if ((uint32_t)g < G) {
                        const GroupDesc gd = bv.groups[g];
#pragma unroll
                        for (int j = 0; j < NH; ++j)
                            if ((uint32_t)j < h) ro[j] = gd.base + fastmod(hv[j], gd.sig, gd.magic) * bv.pitch;
                    }
                    // row-major issue order: the chunks of one row leave back to back,
                    // so the vector L1 sees one row line in consecutive requests
                    const bool on = (uint32_t)g < G && act;
#pragma unroll
                    for (int cc = 0; cc < CM; ++cc)
                        mk[g * CM + cc] = (on && (uint32_t)cc < cpg) ? make_uint4(~0u, ~0u, ~0u, ~0u)
                                                                     : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
                    for (int j = 0; j < NH; ++j) {
                        if ((uint32_t)j >= h) continue;
#pragma unroll
                        for (int cc = 0; cc < CM; ++cc)
                            if (on && (uint32_t)cc < cpg)
                                mk[g * CM + cc] = and4(mk[g * CM + cc],
                                                       *reinterpret_cast<const uint4*>(bv.rows + ro[j] + cc * 16));
                    }
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

// ------------------------------------------------------------------ launch
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

static SlotsFn pick_slots(uint32_t k, uint32_t h, SlotShape s) {
    switch (kh_variant(k, h)) {
        case 0: return s.gm == 1 ? slots_fn_classic<21, 7>(s) : slots_fn<0, 0>(s);  // species banks are classic
        case 1: return slots_fn<31, 1>(s);
        default: return slots_fn<0, 0>(s);
    }
}

static int shape_index(SlotShape s) {  // 0..12, for the grid cache
    static const int gms[13] = {1, 1, 0, 0, 4, 8, 16, 4, 8, 2, 3, 4, 0};
    static const int cms[13] = {4, 8, 0, 0, 1, 1, 1, 2, 2, 4, 4, 4, 0};
    for (int i = 0; i < 12; ++i)
        if (gms[i] == s.gm && cms[i] == s.cm) return i;
    return 12;
}


bool slots_take(const CobsView& bv) { return slots_for(bv).gm != 0; }

int grid_cobs_slots(const CobsView& bv, uint32_t k) {
    static std::atomic<int> slots[3][13];
    const SlotShape sh = slots_for(bv);
    // LDS is 16 KB at most: residency is set by registers, not by D
    return cached_grid(slots[kh_variant(k, bv.h)][shape_index(sh)],
                       [&] { return resident_grid(pick_slots(k, bv.h, sh), kProbeThreads, 16384); });
}

hipError_t launch_cobs_slots(const ReadView& rv, const CobsView& bv, uint32_t* hits, uint64_t* partials,
                             int blocks, hipStream_t s) {
    const size_t lds = slots_lds(bv);
    pick_slots(rv.k, bv.h, slots_for(bv))<<<blocks, kProbeThreads, lds, s>>>(rv, bv, hits, partials,
                                                                           (uint32_t)(lds / sizeof(uint64_t)));
    return hipGetLastError();
}

}  // namespace xs
