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

#include "xs_device.h"

namespace xs {

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

// ------------------------------------------------------------------ rbloom probe
// Filter bits tested before the rest: 2 measured fastest for member-heavy
// and foreign-heavy reads alike (all 7 at once: 15.69 against 13.43 ms per
// config-2 step).
constexpr int kBloomSplit = 2;
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
            lcg_step(sl, sh);
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
        const uint64_t base = grab_units(rv.queue, lane, rv.grab);
        if (base >= U) break;
        const uint64_t uend = min(base + rv.grab, U);
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
        const uint64_t base = grab_units(rv.queue, lane, rv.grab);
        if (base >= U) break;
        const uint64_t uend = min(base + rv.grab, U);
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
                    lcg_step(sl, sh);
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
                                uint64_t D, uint32_t threshold, unsigned long long* scores,
                                uint32_t* __restrict__ first) {
    const uint64_t total = n_chunks * D;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = hits[i];
        if (v > threshold) {
            const uint64_t c = i / D, d = i - c * D;
            const uint64_t o = (uint64_t)seq_of_chunk[c] * D + d;
            atomicAdd(&scores[o], (unsigned long long)v);
            if (first) atomicMin(&first[o], (uint32_t)c);
        }
    }
}

// The score of each (sequence, allele) in its first passing chunk (after
// mlst_sum_kernel has found that chunk): with the chunk index it gives the
// position at which the reference's all_counts dict first saw the allele.
__global__ void mlst_first_score_kernel(const uint32_t* __restrict__ hits,
                                        const uint32_t* __restrict__ seq_of_chunk, uint64_t n_chunks,
                                        uint64_t D, uint32_t threshold, const uint32_t* __restrict__ first,
                                        uint32_t* __restrict__ first_score) {
    const uint64_t total = n_chunks * D;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = hits[i];
        if (v > threshold) {
            const uint64_t c = i / D, d = i - c * D;
            const uint64_t o = (uint64_t)seq_of_chunk[c] * D + d;
            if (first[o] == (uint32_t)c) first_score[o] = v;
        }
    }
}

// ------------------------------------------------------------------ narrow hit rows
// Hit counts never exceed a read's k-mer count, so a host that wants the
// matrix back gets it in 1 or 2 bytes per (read, doc) when every read of the
// call has at most 255 / 65535 sampled k-mers: a quarter (half) of the PCIe
// bytes and of the host memory the caller has to touch.  Four counts per
// thread: one 16-B load, one 4- or 8-B store.
template <class T>
__global__ void narrow_hits_kernel(const uint32_t* __restrict__ src, T* __restrict__ dst, uint64_t n,
                                   uint32_t* __restrict__ overflow) {
    constexpr int kBits = 8 * sizeof(T);
    const uint64_t n4 = n / 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const bool vec = reinterpret_cast<uintptr_t>(src) % 16 == 0 && reinterpret_cast<uintptr_t>(dst) % (4 * sizeof(T)) == 0;
    uint32_t over = 0;  // any count that does not fit T (the caller's max_len was too small)
    if (vec) {
        for (uint64_t i = t0; i < n4; i += stride) {
            const uint4 v = reinterpret_cast<const uint4*>(src)[i];
            over |= (v.x | v.y | v.z | v.w) >> kBits;
            if constexpr (sizeof(T) == 1) {
                reinterpret_cast<uint32_t*>(dst)[i] = v.x | (v.y << 8) | (v.z << 16) | (v.w << 24);
            } else {
                reinterpret_cast<uint2*>(dst)[i] = make_uint2(v.x | (v.y << 16), v.z | (v.w << 16));
            }
        }
        for (uint64_t i = n4 * 4 + t0; i < n; i += stride) {
            over |= src[i] >> kBits;
            dst[i] = (T)src[i];
        }
    } else {
        for (uint64_t i = t0; i < n; i += stride) {
            over |= src[i] >> kBits;
            dst[i] = (T)src[i];
        }
    }
    if (over && overflow) overflow[0] = 1u;  // divergent: a vector store
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

// Grid of the probe kernel launch_probe_cobs picks for this bank (partials
// are sized by it).  Cached per variant; every device of a run is an MI355X.
// Order: fast (D <= 128), bit-sliced (MLST loci), wide (2..16 chunks), slots, general.
int probe_grid_cobs(const CobsView& bv, uint32_t k) {
    if (cobs_fast(bv, k)) return grid_cobs_fast(k);
    if (vslice_take(bv)) return grid_cobs_vslice(bv, k);
    if (wide_for(bv)) return grid_cobs_wide(bv, k);
    if (slots_take(bv)) return grid_cobs_slots(bv, k);
    return grid_cobs_general(bv);
}

hipError_t launch_probe_cobs(const ReadView& rv, const CobsView& bv, uint32_t* hits,
                             uint64_t* partials, int blocks, hipStream_t s) {
    if (cobs_fast(bv, rv.k)) return launch_cobs_fast(rv, bv, hits, partials, blocks, s);
    if (vslice_take(bv)) return launch_cobs_vslice(rv, bv, hits, partials, blocks, s);
    if (wide_for(bv)) return launch_cobs_wide(rv, bv, hits, partials, blocks, s);
    if (slots_take(bv)) return launch_cobs_slots(rv, bv, hits, partials, blocks, s);
    return launch_cobs_general(rv, bv, hits, partials, blocks, s);
}

int probe_grid_bloom() {
    static std::atomic<int> cache{0};
    return cached_grid(cache, [] { return resident_grid(probe_bloom_kernel<21, 7, kBloomSplit>, kProbeThreads, 0); });
}

hipError_t launch_probe_bloom(const ReadView& rv, const BloomView& bv, uint32_t* hits,
                              uint64_t* partials, int blocks, hipStream_t s) {
    if (rv.k == 21 && bv.K == 7)
        probe_bloom_kernel<21, 7, kBloomSplit><<<blocks, kProbeThreads, 0, s>>>(rv, bv, hits, partials);
    else
        probe_bloom_kernel<0, 0, kBloomSplit><<<blocks, kProbeThreads, 0, s>>>(rv, bv, hits, partials);
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
                           uint32_t* first, uint32_t* first_score, hipStream_t s) {
    if (n_chunks == 0 || D == 0) return hipSuccess;
    const unsigned g = grid_for(n_chunks * D, 256, 4096);
    mlst_sum_kernel<<<g, 256, 0, s>>>(hits, seq_of_chunk, n_chunks, D, threshold, scores, first);
    if (first && first_score)
        mlst_first_score_kernel<<<g, 256, 0, s>>>(hits, seq_of_chunk, n_chunks, D, threshold, first, first_score);
    return hipGetLastError();
}

hipError_t launch_narrow_hits(const uint32_t* src, void* dst, uint64_t n, int hit_bytes, hipStream_t s,
                              uint32_t* overflow) {
    if (n == 0) return hipSuccess;
    const unsigned g = grid_for((n + 3) / 4, 256, 8192);
    if (hit_bytes == 1) narrow_hits_kernel<uint8_t><<<g, 256, 0, s>>>(src, static_cast<uint8_t*>(dst), n, overflow);
    else narrow_hits_kernel<uint16_t><<<g, 256, 0, s>>>(src, static_cast<uint16_t*>(dst), n, overflow);
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
