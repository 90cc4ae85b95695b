// xs_probe_bloompart.hip — partitioned rbloom probe for filters far larger than L2.
//
// The direct probe (probe_bloom_kernel) gathers ~6 random filter words per
// k-mer; every one is a 128-B line fill from HBM, so it runs at the chip's
// random line-fill rate (~58 G lines/s).  Here the same membership test is
// reorganised around the filter instead of the k-mers:
//
//   counts  : per read k-mer count, exclusive scan -> global k-mer id g
//   bucket  : one block per 1024 k-mers: canonical k-mer, XXH3-64, the K
//             LCG bit indices (exactly as probe_bloom_kernel, kept in
//             registers), each binned by filter partition (2 MiB of
//             filter = 2^24 bits; smaller under 128 MiB, larger over 2 GiB)
//             with LDS counters, a block scan and LDS-sorted placement.  The block copies its
//             entries (u32 bit offset in the partition, u16 k-mer id)
//             partition-ordered into its own region with coalesced stores and
//             one u16 start per partition into a partition-major table.
//   lookup  : the workgroups of one XCD work through one partition at a time
//             (blocks b and b+8 share an XCD) from a per-partition queue, so
//             the filter bytes they test stay in that XCD's 4 MiB L2 while the
//             entries stream past; a zero bit sets the entry's miss byte.
//   resolve : per bucket block, miss bytes -> miss bits of its 1024 k-mers.
//   count   : per work unit, sampled k-mers minus missed k-mers -> hits per
//             read (direct store or atomicAdd for multi-unit reads) + totals.
//
// A k-mer is a member iff none of its K bits is zero: the same answer as
// rbloom's `kmer in bf` (probabilistic_single_filter_model.py:122-124), which
// stops at the first zero bit.  Parity: tests/test_gpu_parity.py (rbloom
// cases run through this path and the direct one).
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "xs_part.h"

namespace xs {

namespace {

template <int KT, int KB>
__global__ void __launch_bounds__(kBucketThreads) bloom_bucket_kernel(ReadView rv, BloomView bv,
                                                                      const uint64_t* __restrict__ kofs,
                                                                      uint32_t shift, uint32_t P, uint64_t tstride,
                                                                      uint32_t* __restrict__ eoff,
                                                                      uint16_t* __restrict__ eid,
                                                                      uint16_t* __restrict__ tbm,
                                                                      const uint32_t* __restrict__ blk_read) {
    using Scan = hipcub::BlockScan<uint32_t, kBucketThreads>;
    constexpr int ITEMS = kPartMax / kBucketThreads;
    constexpr int PER = kTK / kBucketThreads;  // k-mers per thread
    constexpr int NK = KB ? KB : kPartKMax;
    __shared__ uint32_t s_off[kTK * NK];  // partition-ordered bit offsets
    __shared__ uint16_t s_id[kTK * NK];   // their k-mer (0..kTK-1)
    __shared__ uint32_t cur[kPartMax];
    __shared__ typename Scan::TempStorage scan_tmp;
    __shared__ uint64_t s_kofs[kStageReads], s_offs[kStageReads];
    const int tid = threadIdx.x;
    const uint32_t K = KB ? KB : bv.K;
    const uint32_t k = KT ? KT : rv.k;
    const uint64_t Nk = kofs[rv.n];
    const uint64_t g0 = (uint64_t)blockIdx.x * kTK;
    if (g0 >= Nk) return;  // uniform per block
    const uint32_t m = (uint32_t)min((uint64_t)kTK, Nk - g0);
    for (uint32_t i = tid; i < kPartMax; i += kBucketThreads) cur[i] = 0;
    // reads of this block: from the one holding k-mer g0 to the one holding the
    // next block's first k-mer (or the last read); their k-mer and byte
    // offsets go to LDS when they fit, so a k-mer costs one global load (its
    // window) and every thread's windows are in flight together
    const uint64_t lo = blk_read[blockIdx.x];
    const uint64_t hi = g0 + kTK < Nk ? blk_read[blockIdx.x + 1] : rv.n - 1;
    const uint64_t nr = hi - lo + 2;  // kofs/offs entries lo .. hi+1
    const bool staged = nr <= kStageReads;
    // k-mer -> read (staged case) by a block-wide max-scan of the reads' first k-mers, as in
    // the COBS bucket pass (xs_probe_cobspart.hip); s_off is free until the entries are placed
    uint32_t* s_map = s_off;
    if (staged) {
        for (uint32_t x = tid; x < nr; x += kBucketThreads) {
            s_kofs[x] = kofs[lo + x];
            s_offs[x] = rv.offs[lo + x];
        }
        for (uint32_t i = tid; i < kTK; i += kBucketThreads) s_map[i] = 0;  // read 0 holds k-mer g0
    }
    __syncthreads();
    if (staged) {
        for (uint32_t x = 1 + tid; x + 1 < nr; x += kBucketThreads) {
            const uint64_t st = s_kofs[x] - g0;
            if (st < (uint64_t)kTK) atomicMax(&s_map[st], x);
        }
        __syncthreads();
        uint32_t mv[PER];
#pragma unroll
        for (int q = 0; q < PER; ++q) mv[q] = s_map[tid * PER + q];
        Scan(scan_tmp).InclusiveScan(mv, mv, hipcub::Max());
#pragma unroll
        for (int q = 0; q < PER; ++q) s_map[tid * PER + q] = mv[q];
        __syncthreads();
    }
    const uint64_t omask = (1ull << shift) - 1;
    Kmer c[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid + q * kBucketThreads;
        if (i < m) {
            const uint64_t g = g0 + i;
            uint64_t r, o0, o1, kr;
            if (staged) {
                const uint32_t a = s_map[i];  // largest x with s_kofs[x] <= g
                kr = s_kofs[a];
                o0 = s_offs[a];
                o1 = s_offs[a + 1];
            } else {
                r = read_of(kofs, lo, hi, g);
                kr = kofs[r];
                o0 = rv.offs[r];
                o1 = rv.offs[r + 1];
            }
            kmer_at<KT, kKmerBio>(rv, o0, o1 - o0, (g - kr) * rv.step, k, c[q]);
        }
    }
    uint64_t idx[PER][NK];  // the K bit indices of this thread's k-mers stay in registers,
    uint32_t rk[PER][NK];   // with each one's rank in its partition (one LDS atomic per index)
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid + q * kBucketThreads;
        if (i < m) {
            const uint64_t h = xxh3_kmer<KT>(c[q], k);
            static_assert(NK <= 8, "lcg_high_n covers 8 states");
#pragma unroll
            for (int j = 0; j < NK; ++j) {
                if ((uint32_t)j < K) {
                    idx[q][j] = fastmod(lcg_high_n(h, j + 1), bv.mbits, bv.magic);
                    rk[q][j] = atomicAdd(&cur[(uint32_t)(idx[q][j] >> shift)], 1u);
                }
            }
        }
    }
    __syncthreads();
    uint32_t v[ITEMS];
#pragma unroll
    for (int q = 0; q < ITEMS; ++q) v[q] = cur[tid * ITEMS + q];
    Scan(scan_tmp).ExclusiveSum(v, v);
    __syncthreads();  // every counter read before it becomes a cursor
#pragma unroll
    for (int q = 0; q < ITEMS; ++q) {
        const uint32_t p = tid * ITEMS + q;
        if (p < P) {
            cur[p] = v[q];
            tbm[(uint64_t)blockIdx.x * (P + 1) + p] = (uint16_t)v[q];
        }
    }
    if (tid == 0) tbm[(uint64_t)blockIdx.x * (P + 1) + P] = (uint16_t)(m * K);
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid + q * kBucketThreads;
        if (i < m) {
#pragma unroll
            for (int j = 0; j < NK; ++j) {
                if ((uint32_t)j < K) {
                    const uint32_t pos = cur[(uint32_t)(idx[q][j] >> shift)] + rk[q][j];
                    s_off[pos] = (uint32_t)(idx[q][j] & omask);
                    s_id[pos] = (uint16_t)i;
                }
            }
        }
    }
    __syncthreads();
    // coalesced copy-out (regions are kTK*K entries: 16-B aligned for both arrays)
    const uint64_t base = (uint64_t)blockIdx.x * kTK * K;
    const uint32_t tot = m * K;
    for (uint32_t e = tid * 4; e < tot; e += kBucketThreads * 4) {
        if (e + 4 <= tot) {
            *reinterpret_cast<uint4*>(eoff + base + e) = *reinterpret_cast<const uint4*>(s_off + e);
            *reinterpret_cast<uint2*>(eid + base + e) = *reinterpret_cast<const uint2*>(s_id + e);
        } else {
            for (uint32_t x = e; x < tot; ++x) {
                eoff[base + x] = s_off[x];
                eid[base + x] = s_id[x];
            }
        }
    }
}

// The waves of one XCD work through one partition at a time (its filter
// bytes stay in the XCD's 4 MiB L2 while the entries stream past), taking
// groups of 64 bucket blocks from the partition's queue counter.  A queue
// self-balances: with a static deal the wave scheduler lets some waves run
// partitions ahead and the L2 hit rate fell from 86 % to 44 %.  Each counter
// sits on its own 128-B line (a line's atomics are serialised at the memory
// side).  Every lane keeps kLookupUnroll entries in flight.

// Each group's entry -> block map is built in LDS per window of W entries, as
// in cobs_lookup_kernel (xs_probe_cobspart.hip): every lane writes its block's
// position base over its run's slots, then each entry reads its base back
// (positions are u32: the host keeps a call under 2^32 entries).
template <int kLookupUnroll, int W>
__global__ void __launch_bounds__(256) bloom_lookup_kernel(BloomView bv, const uint64_t* __restrict__ kofs,
                                                           uint64_t n, uint32_t K, uint32_t shift, uint32_t P,
                                                           uint64_t tstride, const uint32_t* __restrict__ eoff,
                                                           const uint16_t* __restrict__ tbl,
                                                           uint8_t* __restrict__ emiss, uint32_t* qctr) {
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    static_assert(W > 0, "window of the entry -> block map");
    __shared__ uint32_t s_base[4][W];  // entry -> position base
    const uint64_t nblk = (kofs[n] + kTK - 1) / kTK;
    const uint64_t cap = (uint64_t)kTK * K;
    const uint32_t xcd = blockIdx.x & 7;
    for (uint64_t p = xcd; p < P; p += 8) {
        const uint32_t* pb = bv.bits + (p << (shift - 5));
        const uint16_t* t0 = tbl + p * tstride;
        const uint16_t* t1 = t0 + tstride;
        for (;;) {
            uint32_t grp = 0;
            if (lane == 0) grp = atomicAdd(&qctr[p * kQStride], 1u);
            const uint64_t b0 = (uint64_t)__builtin_amdgcn_readfirstlane(grp) * 64;
            if (b0 >= nblk) break;
        {
            const uint64_t b = b0 + lane;
            uint32_t s = 0, len = 0;
            if (b < nblk) {
                s = t0[b];
                len = (uint32_t)t1[b] - s;
            }
            uint32_t inc = len;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t t = (uint32_t)__shfl_up((int)inc, d, 64);
                if (lane >= d) inc += t;
            }
            const uint32_t pre = inc - len;
            const uint32_t total = (uint32_t)__shfl((int)inc, 63, 64);
            const uint32_t base = (uint32_t)(b * cap + s) - pre;  // entry i sits at base + i (mod 2^32)
            for (uint32_t w0 = 0; w0 < total; w0 += W) {
            const uint32_t wend = min(total, w0 + W);
            {
                const uint32_t lo = max(pre, w0), hi = min(pre + len, wend);
                for (uint32_t x = lo; x < hi; ++x) s_base[wid][x - w0] = base;
                __builtin_amdgcn_wave_barrier();
            }
            for (uint32_t i0 = w0; i0 < wend; i0 += 64 * kLookupUnroll) {
                uint64_t pos[kLookupUnroll];
                uint32_t off[kLookupUnroll], w[kLookupUnroll];
#pragma unroll
                for (int u = 0; u < kLookupUnroll; ++u) {
                    const uint32_t i = i0 + u * 64 + lane;
                    pos[u] = i < wend ? s_base[wid][i - w0] + i : 0u;
                }
#pragma unroll
                for (int u = 0; u < kLookupUnroll; ++u)
                    off[u] = i0 + u * 64 + lane < wend ? eoff[pos[u]] : 0u;
#pragma unroll
                for (int u = 0; u < kLookupUnroll; ++u)
                    w[u] = i0 + u * 64 + lane < wend ? pb[off[u] >> 5] : ~0u;
#pragma unroll
                for (int u = 0; u < kLookupUnroll; ++u)
                    if (!((w[u] >> (off[u] & 31)) & 1u)) emiss[pos[u]] = 1;
            }
            __builtin_amdgcn_wave_barrier();  // bases read before the next window's writes
            }
        }
        }
    }
}

// Per bucket block: its entries' miss bytes -> the miss bits of its 1024 k-mers.
__global__ void __launch_bounds__(256) bloom_resolve_kernel(const uint64_t* __restrict__ kofs, uint64_t n,
                                                            uint32_t K, const uint16_t* __restrict__ eid,
                                                            const uint8_t* __restrict__ emiss,
                                                            uint32_t* __restrict__ miss) {
    __shared__ uint32_t s_m[kTK / 32];
    const uint64_t Nk = kofs[n];
    const uint64_t g0 = (uint64_t)blockIdx.x * kTK;
    if (g0 >= Nk) return;
    const uint32_t tot = (uint32_t)min((uint64_t)kTK, Nk - g0) * K;
    if (threadIdx.x < kTK / 32) s_m[threadIdx.x] = 0;
    __syncthreads();
    // 4 entries per lane: regions are multiples of 4 entries, and miss bytes
    // past `tot` are zero (memset per call, never written)
    const uint64_t base = (uint64_t)blockIdx.x * kTK * K;
    for (uint32_t e = threadIdx.x * 4; e < tot; e += blockDim.x * 4) {
        const uint32_t f = *reinterpret_cast<const uint32_t*>(emiss + base + e);
        if (f) {
            const uint2 ids = *reinterpret_cast<const uint2*>(eid + base + e);
            const uint32_t id4[4] = {ids.x & 0xFFFFu, ids.x >> 16, ids.y & 0xFFFFu, ids.y >> 16};
#pragma unroll
            for (int x = 0; x < 4; ++x)
                if ((f >> (8 * x)) & 0xFFu) atomicOr(&s_m[id4[x] >> 5], 1u << (id4[x] & 31));
        }
    }
    __syncthreads();
    if (threadIdx.x < kTK / 32) miss[(g0 >> 5) + threadIdx.x] = s_m[threadIdx.x];
}

__global__ void __launch_bounds__(256) bloom_count_kernel(ReadView rv, const uint64_t* __restrict__ kofs,
                                                          const uint32_t* __restrict__ miss, uint32_t K,
                                                          uint32_t* __restrict__ hits,
                                                          uint64_t* __restrict__ partials,
                                                          uint64_t* __restrict__ rows_read) {
    __shared__ uint64_t s_h[4], s_k[4];
    const uint32_t k = rv.k;
    const uint64_t U = rv.queue[0];
    uint64_t hit_total = 0, kmer_total = 0;
    for (uint64_t u = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; u < U;
         u += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = rv.unit_read[u];
        const uint64_t seg = u - rv.unit_ofs[r];
        const uint64_t nk = num_kmers(rv.offs[r + 1] - rv.offs[r], k, rv.step);
        const uint64_t t0 = seg * kSegKmers;
        const uint32_t cnt = (uint32_t)min((uint64_t)kSegKmers, nk - t0);
        const uint64_t g = kofs[r] + t0, ge = g + cnt;
        uint32_t missed = 0;
        for (uint64_t q = g; q < ge;) {
            const uint32_t bit = (uint32_t)(q & 31);
            const uint32_t take = (uint32_t)min((uint64_t)(32 - bit), ge - q);
            const uint32_t w = miss[q >> 5] >> bit;
            missed += (uint32_t)__popc(take == 32 ? w : (w & ((1u << take) - 1u)));
            q += take;
        }
        const uint32_t c = cnt - missed;
        if (hits) {
            if (nk <= kSegKmers) hits[r] = c;
            else if (c) atomicAdd(&hits[r], c);
        }
        hit_total += c;
        kmer_total += cnt;
    }
    // wave sums, then block sums
    for (int d = 32; d; d >>= 1) {
        hit_total += (uint64_t)__shfl_xor((long long)hit_total, d, 64);
        kmer_total += (uint64_t)__shfl_xor((long long)kmer_total, d, 64);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        s_h[wid] = hit_total;
        s_k[wid] = kmer_total;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t a = s_h[0] + s_h[1] + s_h[2] + s_h[3];
        const uint64_t b = s_k[0] + s_k[1] + s_k[2] + s_k[3];
        if (partials) {
            partials[blockIdx.x * 2ull] = a;
            partials[blockIdx.x * 2ull + 1] = b;
        }
        if (rows_read && b) atomicAdd(reinterpret_cast<unsigned long long*>(rows_read), (unsigned long long)(b * K));
    }
}

}  // namespace

// Partition shift for a filter of `mbits` bits: 2^24-bit (2 MiB) partitions
// (2 MiB: 8.92 ms per config-2 step; 1 MiB 9.31, 512 KiB 10.86, 4 MiB 10.00),
// halved down to 2^20 bits while that leaves fewer than 64 partitions (8 per
// XCD keep the XCDs evenly loaded), doubled while more than kPartMax.
static uint32_t part_shift(uint64_t mbits, uint32_t pref, uint32_t floor) {
    auto parts = [mbits](uint32_t s) { return (mbits + (1ull << s) - 1) >> s; };
    uint32_t s = pref;
    while (s > floor && parts(s) < 64) --s;
    while (parts(s) > kPartMax) ++s;
    return s;
}

// opt.bloom_part (ProbeOptions): 0 = direct probe only; 1 (default) =
// partitioned probe for filters of >= 16 MiB on member-rich input; 2 =
// partitioned for such filters whatever the input; 3 = partitioned for every
// filter, with partitions down to 1024 bits (tests reach many partitions on
// small filters).
bool bloom_part_plan(const BloomView& bv, uint64_t n, uint64_t seq_bytes, uint32_t step, double member_frac,
                     const ProbeOptions& opt, BloomPartPlan* plan) {
    const int mode = opt.bloom_part;
    if (mode <= 0 || bv.K == 0 || bv.K > (uint32_t)kPartKMax) return false;
    // member-poor input: the direct probe's early exit (2 bits first) wins
    if (mode == 1 && member_frac < kPartMinMembers) return false;
    const uint32_t shift = mode >= 3 ? part_shift(bv.mbits, 10, 10) : part_shift(bv.mbits, 24, 20);
    const uint64_t P = (bv.mbits + (1ull << shift) - 1) >> shift;
    // filters under 16 MiB stay L2/MALL resident: the direct probe is faster there
    if ((mode < 3 && bv.mbits < (128ull << 20)) || shift > 32) return false;
    const uint64_t kbound = seq_bytes / step + n + 1;  // >= sum of ceil((len-k+1)/step)
    if (kbound >= (1ull << 32)) return false;
    const uint64_t nblk = (kbound + kTK - 1) / kTK;
    plan->shift = shift;
    plan->P = (uint32_t)P;
    plan->tstride = nblk;
    plan->kbound = kbound;
    plan->entry_bytes = nblk * kTK * bv.K * (sizeof(uint32_t) + sizeof(uint16_t) + sizeof(uint8_t));
    plan->tbl_bytes = 2 * (P + 1) * nblk * sizeof(uint16_t);  // partition-major + block-major
    plan->miss_bytes = nblk * (kTK / 32) * sizeof(uint32_t);
    plan->aux_bytes = (nblk + 1 + kQStride) * sizeof(uint32_t) + (size_t)P * kQStride * sizeof(uint32_t);
    plan->nkc_bytes = (n + 1) * sizeof(uint64_t);
    size_t sb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, sb, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)(n + 1));
    plan->scan_bytes = sb;
    // entries are transient: cap the workspace (larger batches take the direct probe);
    // the lookup's u32 entry positions need fewer than 2^32 entries (7 B each: the cap keeps them)
    return plan->entry_bytes <= (24ull << 30) && nblk * kTK * bv.K < (1ull << 32);
}

// Entries in flight per lane: 4 / 8 / 16 measured 10.67 / 10.59 / 10.44 ms per
// config-2 step.  Blocks per CU: 3 (9.53 ms) beat the resident 5 (10.36 ms) and
// 2 (9.60 ms): fewer waves keep more of each partition in L2.  Running the
// bucket pass of sub-batch i+1 on a second stream beside the lookup of i
// saved a further 0.1 ms only, and is not done.
constexpr int kUnroll = 16;
constexpr int kLookupPerCu = 3;
// the entry -> block map's window: 1024 entries (lookup 5.27 -> 5.02-5.05 ms against
// round 2's shuffle binary search; 2048 / 512-entry windows 5.13 / 5.51, 24 / 12 entries
// per lane 5.09 / 5.21; profiles/r03_lookup_ownermap.txt)
constexpr int kLookupWindow = 1024;

static int lookup_grid() {
    static std::atomic<int> cache{0};
    return cached_grid(cache, [] {
        int dev = 0;
        hipDeviceProp_t prop;
        int per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 768;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bloom_lookup_kernel<kUnroll, kLookupWindow>, 256, 0) !=
                hipSuccess || per_cu < 1)
            per_cu = 1;
        const int g = std::min(per_cu, kLookupPerCu) * prop.multiProcessorCount;
        return g >= 8 ? g / 8 * 8 : 8;  // whole groups of 8 blocks (one per XCD)
    });
}

hipError_t launch_probe_bloom_part(const ReadView& rv, const BloomView& bv, const BloomPartPlan& plan,
                                   const BloomPartWs& ws, uint32_t* hits, uint64_t* partials, int blocks,
                                   hipStream_t s, PassRecorder* rec) {
    pass_mark(rec, kPassStart, s);
    part_counts_kernel<<<grid_for(rv.n + 1, 256, 4096), 256, 0, s>>>(rv.offs, rv.n, rv.k, rv.step, ws.nkc);
    size_t sb = ws.scan_bytes;
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(ws.scan_tmp, sb, ws.nkc, ws.kofs, (int)(rv.n + 1), s);
    if (e != hipSuccess) return e;
    const uint64_t ne = plan.tstride * kTK * bv.K;
    uint32_t* eoff = reinterpret_cast<uint32_t*>(ws.entries);
    uint16_t* eid = reinterpret_cast<uint16_t*>(eoff + ne);
    uint8_t* emiss = reinterpret_cast<uint8_t*>(eid + ne);
    if ((e = hipMemsetAsync(emiss, 0, ne, s)) != hipSuccess) return e;
    uint32_t* blk_read = ws.aux;
    uint16_t* tbm = ws.tbl + (uint64_t)(plan.P + 1) * plan.tstride;  // block-major copy
    part_map_kernel<<<grid_for(rv.n, 256, 4096), 256, 0, s>>>(ws.kofs, rv.n, blk_read);
    pass_mark(rec, kPassPrep, s);
    if (rv.k == 21 && bv.K == 7)
        bloom_bucket_kernel<21, 7><<<(unsigned)plan.tstride, kBucketThreads, 0, s>>>(
            rv, bv, ws.kofs, plan.shift, plan.P, plan.tstride, eoff, eid, tbm, blk_read);
    else
        bloom_bucket_kernel<0, 0><<<(unsigned)plan.tstride, kBucketThreads, 0, s>>>(
            rv, bv, ws.kofs, plan.shift, plan.P, plan.tstride, eoff, eid, tbm, blk_read);
    part_transpose_kernel<<<dim3((unsigned)((plan.tstride + 63) / 64), (plan.P + 1 + 63) / 64), 256, 0, s>>>(
        tbm, plan.P + 1, plan.tstride, ws.tbl, 0, plan.tstride);
    uint32_t* qctr = ws.aux + (plan.tstride + 1 + kQStride - 1) / kQStride * kQStride;  // 128-B aligned
    if ((e = hipMemsetAsync(qctr, 0, (size_t)plan.P * kQStride * sizeof(uint32_t), s)) != hipSuccess) return e;
    pass_mark(rec, kPassBucket, s);
    bloom_lookup_kernel<kUnroll, kLookupWindow><<<lookup_grid(), 256, 0, s>>>(
        bv, ws.kofs, rv.n, bv.K, plan.shift, plan.P, plan.tstride, eoff, ws.tbl, emiss, qctr);
    pass_mark(rec, kPassLookup, s);
    bloom_resolve_kernel<<<(unsigned)plan.tstride, 256, 0, s>>>(ws.kofs, rv.n, bv.K, eid, emiss, ws.miss);
    bloom_count_kernel<<<blocks, 256, 0, s>>>(rv, ws.kofs, ws.miss, bv.K, hits, partials, bv.rows_read);
    pass_mark(rec, kPassResolve, s);
    return hipGetLastError();
}

}  // namespace xs
