// xs_probe_general.hip — COBS probe of any bank the LDS counters hold (the fallback layout).
#include "xs_device.h"

namespace xs {

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

// ------------------------------------------------------------------ launch
template <int KT, int HT>
static hipError_t launch_cobs_t(const ReadView& rv, const CobsView& bv, uint32_t* hits,
                                uint64_t* partials, int blocks, int wpb, size_t lds,
                                uint32_t dpad, hipStream_t s) {
    probe_cobs_kernel<KT, HT><<<blocks, wpb * kWave, lds, s>>>(rv, bv, hits, partials, dpad);
    return hipGetLastError();
}

int grid_cobs_general(const CobsView& bv) {
    static std::atomic<int> generic[3];
    int wpb;
    size_t lds;
    if (probe_blocks(bv.D, &wpb, &lds) != 0) return 0;
    return cached_grid(generic[wpb == 4 ? 0 : wpb == 2 ? 1 : 2],
                       [&] { return resident_grid(probe_cobs_kernel<0, 0>, wpb * kWave, lds); });
}

hipError_t launch_cobs_general(const ReadView& rv, const CobsView& bv, uint32_t* hits, uint64_t* partials,
                               int blocks, hipStream_t s) {
    int wpb;
    size_t lds;
    if (probe_blocks(bv.D, &wpb, &lds) != 0) return hipErrorInvalidValue;
    const uint32_t dpad = (uint32_t)((bv.D + 127) / 128 * 128);
    if (rv.k == 21 && bv.h == 7) return launch_cobs_t<21, 7>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
    if (rv.k == 31 && bv.h == 1) return launch_cobs_t<31, 1>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
    return launch_cobs_t<0, 0>(rv, bv, hits, partials, blocks, wpb, lds, dpad, s);
}

}  // namespace xs
