// xs_probe_fast.hip — COBS probe of classic banks of <= 128 docs (one 16-byte row per hash).
#include "xs_device.h"

namespace xs {

// ------------------------------------------------------------------ COBS probe (fast)
// Classic bank with D <= 128 docs: one 16-byte row per hash, counters in
// registers.  One wavefront per unit (<= kSegKmers k-mers of one read), one
// lane per k-mer; units are handed out rv.grab at a time.
struct FastBank {
    const uint8_t* rows;
    uint64_t sig, magic;
    uint32_t D, nwords;  // nwords = ceil(D/32)
};

template <int KT, int HT>
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
                        off[j] = fastmod_small(xxh64_seed<KT>(c, pre, k, (uint64_t)j), (uint32_t)fb.sig, fb.magic) * 16u;
                    m = make_uint4(~0u, ~0u, ~0u, ~0u);
#pragma unroll
                    for (int j = 0; j < HT; ++j)
                        m = and4(m, *reinterpret_cast<const uint4*>(fb.rows + off[j]));
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

// ------------------------------------------------------------------ launch
// The fast kernel covers classic banks of <= 128 docs whose image fits 32-bit
// row offsets, for the (k, h) pairs XspecT trains (species 21/7, MLST 31/1).
bool cobs_fast(const CobsView& bv, uint32_t k) {
    return bv.G == 1 && bv.nchunks == 1 && bv.D <= 128 && bv.sig0 <= (1ull << 28) &&
           ((k == 21 && bv.h == 7) || (k == 31 && bv.h == 1));
}

template <int KT, int HT>
static hipError_t launch_fast_t(const ReadView& rv, const FastBank& fb, uint32_t* hits,
                                uint64_t* partials, int blocks, hipStream_t s) {
    probe_cobs_fast<KT, HT><<<blocks, kProbeThreads, 0, s>>>(rv, fb, hits, partials);
    return hipGetLastError();
}

int grid_cobs_fast(uint32_t k) {
    static std::atomic<int> g21{0}, g31{0};
    if (k == 21) return cached_grid(g21, [] { return resident_grid(probe_cobs_fast<21, 7>, kProbeThreads, 0); });
    return cached_grid(g31, [] { return resident_grid(probe_cobs_fast<31, 1>, kProbeThreads, 0); });
}

hipError_t launch_cobs_fast(const ReadView& rv, const CobsView& bv, uint32_t* hits, uint64_t* partials,
                            int blocks, hipStream_t s) {
    FastBank fb;
    fb.rows = bv.rows;
    fb.sig = bv.sig0;
    fb.magic = barrett_magic(bv.sig0);
    fb.D = (uint32_t)bv.D;
    fb.nwords = (uint32_t)((bv.D + 31) / 32);
    if (rv.k == 21) return launch_fast_t<21, 7>(rv, fb, hits, partials, blocks, s);
    return launch_fast_t<31, 1>(rv, fb, hits, partials, blocks, s);
}

}  // namespace xs
