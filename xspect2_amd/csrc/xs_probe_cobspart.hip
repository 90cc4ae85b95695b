// xs_probe_cobspart.hip — partitioned COBS probe for classic banks far larger
// than L2 (species banks: D <= 128 docs, one 16-byte row per hash).
//
// The direct probe (probe_cobs_fast) gathers h random 16-B rows per k-mer;
// each is a 128-B line fill, so it runs at the chip's random line-fill rate
// (~57 G lines/s, 0.92 of HBM bandwidth at 128 B a line, 16 B of it used).
// Here the probe is reorganised around the bank, as the partitioned rbloom
// probe is (xs_probe_bloompart.hip):
//
//   counts  : per read k-mer count, exclusive scan -> global k-mer id g
//   bucket  : one block per CK (default 2048) k-mers: canonical k-mer, the h
//             XXH64 rows (exactly as the direct probe), each binned by bank
//             partition (2 MiB of rows) with one LDS atomic (its rank), a
//             block scan and LDS-sorted placement; one u32 entry per row =
//             (row in partition << 11 | k-mer in block), copied out
//             partition-ordered per block in runs padded to 4 entries, plus
//             one u16 start per partition into a partition-major table.
//   lookup  : the workgroups of one XCD work through one partition at a time
//             from a per-partition queue, so its 2 MiB of rows stay in that
//             XCD's 4 MiB L2 while the entries stream past; rows are gathered
//             by LDS-DMA, one gather instruction in flight per wave, and each
//             entry's 16-B row is written back in entry order (runs start on
//             64-B boundaries).
//   resolve : per bucket block: AND the h rows of each of its k-mers in LDS,
//             then count per (read, doc) with the column-popcount transpose
//             of the direct probe; reads inside the block are stored, reads
//             crossing a block edge are added atomically; per-doc totals.
//
// Same answer as the direct probe and the oracle (score[d] = number of
// sampled positions whose h rows all hold bit d; probabilistic_filter_model.py
// :227 -> cobs Search.search).  Parity: tests/test_gpu_parity.py runs the
// classic cases through both paths.
#include "xs_part.h"

namespace xs {

namespace {

// CK k-mers per bucket block (kCobsCK = 2048); an entry's low IDB bits name
// its k-mer within the block.
template <int CK>
constexpr int id_bits() { return CK == 4096 ? 12 : CK == 2048 ? 11 : 10; }
template <int CK>
constexpr int bucket_threads() { return CK / 2 < 1024 ? CK / 2 : 1024; }
constexpr int kMaxH = 8;     // rows per k-mer on this path

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 load_nt(const uint4* p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v[0], v[1], v[2], v[3]);
}

struct PartBank {
    const uint4* rows;  // 16-B rows
    uint64_t sig, magic;
    uint32_t D, nwords;
};

template <int KT, int HT, int CK>
__global__ void __launch_bounds__(bucket_threads<CK>(), CK == 4096 ? 1 : 2) cobs_bucket_kernel(ReadView rv, PartBank pb, uint32_t h,
                                                                     const uint64_t* __restrict__ kofs,
                                                                     uint32_t shift, uint32_t P,
                                                                     uint32_t* __restrict__ ent,
                                                                     uint16_t* __restrict__ tbm,
                                                                     const uint32_t* __restrict__ blk_read,
                                                                     uint64_t b_begin, uint64_t stride, uint32_t pad) {
    // entries and partition starts of block B go to row B - b_begin of the range's workspace;
    // with pad = 4 each partition's run is padded with kCobsPadEntry slots to a multiple
    // of 4 entries, so that the lookup's row runs are whole 64-B pieces (P <= kCobsPadParts)
    constexpr int BT = bucket_threads<CK>();
    constexpr int IDB = id_bits<CK>();
    using Scan = hipcub::BlockScan<uint32_t, BT>;
    constexpr int ITEMS = kPartMax / BT;
    constexpr int PER = CK / BT;  // k-mers per thread
    constexpr int NH = HT ? HT : kMaxH;
    __shared__ uint32_t s_ent[CK * NH + 3 * kCobsPadParts];  // partition-ordered entries (+ pad slots)
    __shared__ uint32_t cur[kPartMax];
    __shared__ typename Scan::TempStorage scan_tmp;
    __shared__ uint64_t s_kofs[kStageReads], s_offs[kStageReads];
    const int tid = threadIdx.x;
    const uint32_t H = HT ? HT : h;
    const uint32_t k = KT ? KT : rv.k;
    const uint64_t Nk = kofs[rv.n];
    const uint64_t B = b_begin + blockIdx.x;  // bucket block
    const uint64_t g0 = B * CK;
    if (g0 >= Nk) return;  // uniform per block
    const uint32_t m = (uint32_t)min((uint64_t)CK, Nk - g0);
    for (uint32_t i = tid; i < kPartMax; i += BT) cur[i] = 0;
    // reads of this block staged in LDS when they fit (one global load per k-mer: its window)
    const uint64_t lo = blk_read[B];
    const uint64_t hi = g0 + CK < Nk ? blk_read[B + 1] : rv.n - 1;
    const uint64_t nr = hi - lo + 2;
    const bool staged = nr <= kStageReads;
    // k-mer -> read (staged case): s_map[i] = the block-local read of k-mer g0 + i, from
    // each read's first k-mer marked and a block-wide max-scan (s_ent is free until the
    // entries are placed)
    uint32_t* s_map = s_ent;
    if (staged) {
        for (uint32_t x = tid; x < nr; x += BT) {
            s_kofs[x] = kofs[lo + x];
            s_offs[x] = rv.offs[lo + x];
        }
        for (uint32_t i = tid; i < CK; i += BT) s_map[i] = 0;  // read 0 holds k-mer g0
    }
    __syncthreads();
    if (staged) {
        // reads 1 .. nr-2 start inside the block or after it; empty reads share a start
        // with the next read, and the max keeps the later one
        for (uint32_t x = 1 + tid; x + 1 < nr; x += BT) {
            const uint64_t st = s_kofs[x] - g0;
            if (st < (uint64_t)CK) atomicMax(&s_map[st], x);
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
    Kmer c[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid + q * BT;
        if (i < m) {
            const uint64_t g = g0 + i;
            uint64_t kr, o0, o1;
            if (staged) {
                const uint32_t a = s_map[i];  // largest x with s_kofs[x] <= g
                kr = s_kofs[a];
                o0 = s_offs[a];
                o1 = s_offs[a + 1];
            } else {
                const uint64_t r = read_of(kofs, lo, hi, g);
                kr = kofs[r];
                o0 = rv.offs[r];
                o1 = rv.offs[r + 1];
            }
            kmer_at<KT, kKmerCobs>(rv, o0, o1 - o0, (g - kr) * rv.step, k, c[q]);
        }
    }
    uint32_t row[PER][NH];  // the h rows of this thread's k-mers stay in registers,
    uint32_t rk[PER][NH];   // with each row's rank in its partition (one LDS atomic per row)
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid + q * BT;
        if (i < m) {
            Xxh64Pre pre;
            xxh64_pre<KT>(c[q], k, pre);
#pragma unroll
            for (int j = 0; j < NH; ++j) {
                if ((uint32_t)j < H) {
                    row[q][j] = fastmod_small(xxh64_seed<KT>(c[q], pre, k, (uint64_t)j), (uint32_t)pb.sig, pb.magic);
                    rk[q][j] = atomicAdd(&cur[row[q][j] >> shift], 1u);
                }
            }
        }
    }
    __syncthreads();
    uint32_t v[ITEMS], c0[ITEMS], c1[ITEMS];
#pragma unroll
    for (int q = 0; q < ITEMS; ++q) {
        c0[q] = cur[tid * ITEMS + q];
        c1[q] = (c0[q] + pad - 1) & ~(pad - 1);
        v[q] = c1[q];
    }
    uint32_t tot;  // entries of the block, pad slots included
    Scan(scan_tmp).ExclusiveSum(v, v, tot);
    __syncthreads();  // every counter read before it becomes a cursor
#pragma unroll
    for (int q = 0; q < ITEMS; ++q) {
        const uint32_t p = tid * ITEMS + q;
        if (p < P) {
            cur[p] = v[q];
            tbm[(B - b_begin) * (P + 1) + p] = (uint16_t)v[q];
            for (uint32_t x = c0[q]; x < c1[q]; ++x) s_ent[v[q] + x] = kCobsPadEntry;
        }
    }
    if (tid == 0) tbm[(B - b_begin) * (P + 1) + P] = (uint16_t)tot;
    __syncthreads();
    const uint32_t omask = (1u << shift) - 1;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t i = tid + q * BT;
        if (i < m) {
#pragma unroll
            for (int j = 0; j < NH; ++j) {
                if ((uint32_t)j < H) {
                    s_ent[cur[row[q][j] >> shift] + rk[q][j]] = ((row[q][j] & omask) << IDB) | i;
                }
            }
        }
    }
    __syncthreads();
    // coalesced copy-out (regions of stride entries: 16-B aligned)
    const uint64_t base = (B - b_begin) * stride;  // the range reuses one workspace
    for (uint32_t e = tid * 4; e < tot; e += BT * 4) {
        if (e + 4 <= tot) {
            *reinterpret_cast<uint4*>(ent + base + e) = *reinterpret_cast<const uint4*>(s_ent + e);
        } else {
            for (uint32_t x = e; x < tot; ++x) ent[base + x] = s_ent[x];
        }
    }
}

// The waves of one XCD work through one partition at a time (its rows stay in
// the XCD's L2 while the entries stream past), taking groups of gb <= 64
// bucket blocks from the partition's queue counter (the rbloom lookup's
// scheme, xs_probe_bloompart.hip; gb shrinks for short ranges so that a
// partition still has a group for every wave of its XCD).  Each entry's row goes back in entry order; with
// EMB (D <= kEmbMaxDocs) the entry's k-mer id rides in the row's unused top
// bits (docs 118..127), so the resolve pass need not read the entries again.
template <int CK>
constexpr uint32_t emb_max_docs() { return 128 - id_bits<CK>(); }
// Rows are gathered by LDS-DMA (global_load_lds_dwordx4) into per-wave slots,
// one gather instruction in flight per wave: 1 in flight x 2 workgroups per CU
// beat 2, 3 or 6 in flight and 1, 3 or 4 workgroups (more requests per CU only
// lengthen the L2 wait; register gathers 12.64 vs 12.15 ms per step;
// DESIGN.md §6b items 8-9).  Rows go back with non-temporal dword stores (7.8
// vs 10.1 ms for one plain dwordx4 in tools/partgather.hip; the other store
// and load cache policies measured no better: profiles/r02_cobspart_ab.txt
// item 9).  The entry -> block map of a group is built in LDS per window of
// kWin entries (each lane writes its block's position base over its run's
// slots, then every entry reads its base: ~2 LDS operations per 64 entries)
// instead of a 6-step shuffle binary search per entry (8 shuffles per 64
// entries): lookup 6.33 -> 6.06 ms, and with 8 entries per lane over
// 2048-entry windows 5.84-5.88 ms (6 / 10 / 12 / 14 per lane: 6.06 / 6.08 /
// 6.55 / 6.78 ms; profiles/r03_lookup_ownermap.txt).  Positions are u32: the
// host keeps a range's workspace under 2^32 entries.
constexpr int kLookupUnroll = 8;
constexpr int kLookupWin = 2048;
constexpr int kLookupPerCu = 2;

template <bool EMB, int CK>
__global__ void __launch_bounds__(256) cobs_lookup_kernel(PartBank pb, const uint64_t* __restrict__ kofs,
                                                          uint64_t n, uint32_t H, uint32_t shift, uint32_t P,
                                                          uint64_t tstride, const uint32_t* __restrict__ ent,
                                                          const uint16_t* __restrict__ tbl,
                                                          uint4* __restrict__ out, uint32_t* qctr,
                                                          uint64_t b_begin, uint64_t b_end, uint32_t gb,
                                                          uint64_t stride) {
    constexpr int IDB = id_bits<CK>();
    constexpr int U = kLookupUnroll;
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    __shared__ uint4 s_rows[4][U][64];            // LDS-DMA landing slots
    __shared__ uint32_t s_base[4][kLookupWin];    // entry -> position base
    // this call's bucket blocks: b_begin .. b_end-1 (those past the batch's last k-mer
    // excluded), rows 0 .. nblk-1 of the range's workspace and partition tables
    const uint64_t last = min(b_end, (kofs[n] + CK - 1) / CK);
    const uint64_t nblk = last > b_begin ? last - b_begin : 0;
    const uint32_t xcd = blockIdx.x & 7;
    for (uint64_t p = xcd; p < P; p += 8) {
        const uint4* prow = pb.rows + (p << shift);
        const uint16_t* t0 = tbl + p * tstride;
        const uint16_t* t1 = t0 + tstride;
        for (;;) {
            uint32_t grp = 0;
            if (lane == 0) grp = atomicAdd(&qctr[p * kQStride], 1u);
            const uint64_t b0 = (uint64_t)__builtin_amdgcn_readfirstlane(grp) * gb;
            if (b0 >= nblk) break;
            const uint64_t b = b0 + lane;
            uint32_t s = 0, len = 0;
            if ((uint32_t)lane < gb && b < nblk) {
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
            // entry i of the group sits at its block's base + i (mod 2^32)
            const uint32_t base = (uint32_t)(b * stride + s) - pre;
            for (uint32_t w0 = 0; w0 < total; w0 += kLookupWin) {
                const uint32_t wend = min(total, w0 + kLookupWin);
                {
                    const uint32_t lo = max(pre, w0), hi = min(pre + len, wend);
                    for (uint32_t x = lo; x < hi; ++x) s_base[wid][x - w0] = base;
                    __builtin_amdgcn_wave_barrier();
                }
                for (uint32_t i0 = w0; i0 < wend; i0 += 64 * U) {
                    uint64_t pos[U];
                    uint32_t e[U];
                    uint4 v[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t i = i0 + u * 64 + lane;
                        pos[u] = i < wend ? s_base[wid][i - w0] + i : 0u;
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        e[u] = i0 + u * 64 + lane < wend ? __builtin_nontemporal_load(ent + pos[u]) : 0u;
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (i0 + u * 64 + lane < wend && e[u] != kCobsPadEntry) {
#if defined(__HIP_DEVICE_COMPILE__)  // a device-only builtin: the host pass must not see it
                            // one row gather in flight per wave: each waits for the one before
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                            __builtin_amdgcn_global_load_lds(prow + (e[u] >> IDB), &s_rows[wid][u][0], 16, 0, 0);
#endif
                        }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                    for (int u = 0; u < U; ++u) v[u] = s_rows[wid][u][lane];
                    // a pad slot's row is all ones, so ANDing it into any k-mer changes nothing; its id
                    // bits name the k-mer of its slot's position, spreading the pad rows' LDS ANDs in
                    // the resolve pass over the block instead of one address
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (e[u] == kCobsPadEntry) {
                            v[u] = make_uint4(~0u, ~0u, ~0u, ~0u);
                            e[u] = (uint32_t)pos[u] & (CK - 1);
                        }
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (i0 + u * 64 + lane < wend) {
                            if constexpr (EMB) v[u].w = (v[u].w & (0xFFFFFFFFu >> IDB)) | (e[u] << (32 - IDB));
                            uint32_t* o = reinterpret_cast<uint32_t*>(out + pos[u]);
                            __builtin_nontemporal_store(v[u].x, o);
                            __builtin_nontemporal_store(v[u].y, o + 1);
                            __builtin_nontemporal_store(v[u].z, o + 2);
                            __builtin_nontemporal_store(v[u].w, o + 3);
                        }
                }
                __builtin_amdgcn_wave_barrier();  // bases read before the next window's writes
            }
        }
    }
}

// Per bucket block: AND each k-mer's h rows in LDS, then count per (read, doc).
// Reads of the block whose k-mers all lie in it get their counts stored; the
// (at most two) reads crossing its edges are added atomically (hits zeroed
// beforehand).  Blocks with more reads than LDS counter rows (short reads)
// add every count atomically.
template <int CK>
constexpr int resolve_threads() { return CK / 4 < 1024 ? CK / 4 : 1024; }
template <int CK>
constexpr uint32_t cnt_reads() { return CK / 64; }  // reads per block with LDS counters
constexpr int kResolveUnroll = 8;


template <bool EMB, int CK>
__global__ void __launch_bounds__(resolve_threads<CK>()) cobs_resolve_kernel(ReadView rv, const uint64_t* __restrict__ kofs,
                                                                       uint32_t H, uint32_t D, uint32_t nwords,
                                                                       const uint32_t* __restrict__ ent,
                                                                       const uint4* __restrict__ rowv,
                                                                       const uint32_t* __restrict__ blk_read,
                                                                       uint32_t* __restrict__ hits,
                                                                       uint64_t* __restrict__ partials, int pblocks,
                                                                       uint64_t b_begin, uint64_t stride,
                                                                       const uint16_t* __restrict__ tbm, uint32_t P1) {
    __shared__ uint32_t acc[4][CK];
    constexpr int kResolveThreads = resolve_threads<CK>();
    constexpr uint32_t kCntReads = cnt_reads<CK>();
    __shared__ uint32_t cnt[kCntReads][128];
    __shared__ uint64_t s_kofs[kCntReads + 1];
    __shared__ uint32_t s_tot[128];  // the block's per-doc totals (<= CK each)
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint64_t n = rv.n;
    const uint64_t Nk = kofs[n];
    const uint64_t B = b_begin + blockIdx.x;  // bucket block
    const uint64_t g0 = B * CK;
    if (g0 >= Nk) return;
    const uint32_t m = (uint32_t)min((uint64_t)CK, Nk - g0);
    const uint64_t lo = blk_read[B];
    const uint64_t hi = g0 + CK < Nk ? blk_read[B + 1] : n - 1;
    // reads lo..hi hold the block's k-mers (empty reads between them hold none)
    const uint64_t nr = hi - lo + 1;
    const bool lds_cnt = nr <= kCntReads;
    if (tid < 128) s_tot[tid] = 0;
    for (uint32_t i = tid; i < CK; i += kResolveThreads) {
        acc[0][i] = ~0u;
        acc[1][i] = ~0u;
        acc[2][i] = ~0u;
        acc[3][i] = ~0u;
    }
    if (lds_cnt) {
        for (uint32_t x = tid; x < kCntReads * 128; x += kResolveThreads) (&cnt[0][0])[x] = 0;
        for (uint32_t x = tid; x <= nr; x += kResolveThreads) s_kofs[x] = kofs[lo + x];
    }
    __syncthreads();
    const uint64_t base = (B - b_begin) * stride;
    const uint32_t tot = tbm[(B - b_begin) * P1 + P1 - 1];  // m * H, plus the pad slots (all-ones rows)
    (void)H;
    // kResolveUnroll rows in flight per lane, then their LDS ANDs
    for (uint32_t e0 = tid; e0 < tot; e0 += kResolveThreads * kResolveUnroll) {
        uint4 v[kResolveUnroll];
        uint32_t id[kResolveUnroll];
#pragma unroll
        for (int u = 0; u < kResolveUnroll; ++u) {
            const uint32_t e = e0 + u * kResolveThreads;
            if (e < tot) {
                v[u] = load_nt(rowv + base + e);
                if (!EMB) {  // a pad slot's (all-ones) row goes to the k-mer of its position
                    const uint32_t ev = __builtin_nontemporal_load(ent + base + e);
                    id[u] = (ev == kCobsPadEntry ? e : ev) & (CK - 1);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kResolveUnroll; ++u) {
            if (e0 + u * kResolveThreads < tot) {
                const uint32_t i = EMB ? v[u].w >> (32 - id_bits<CK>()) : id[u];
                atomicAnd(&acc[0][i], v[u].x);
                if (nwords > 1) atomicAnd(&acc[1][i], v[u].y);
                if (nwords > 2) atomicAnd(&acc[2][i], v[u].z);
                if (nwords > 3) atomicAnd(&acc[3][i], v[u].w);
            }
        }
    }
    __syncthreads();
    Xpose X;
    xpose_init(lane, X);
    uint64_t doc_tot[4] = {0, 0, 0, 0};  // lane < 32: doc 32q + lane
    for (uint32_t t0 = (uint32_t)wid * 64; t0 < m; t0 += kResolveThreads) {
        const uint32_t i = t0 + lane;
        const bool valid = i < m;
        const uint64_t g = g0 + i;
        // read of each lane's k-mer
        uint64_t r;
        if (lds_cnt) {
            uint32_t a = 0, b = (uint32_t)(nr - 1);
            while (a < b) {
                const uint32_t mid = (a + b + 1) >> 1;
                if (s_kofs[mid] <= g) a = mid;
                else b = mid - 1;
            }
            r = lo + a;
        } else {
            r = read_of(kofs, lo, hi, valid ? g : g0);
        }
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) w[q] = valid ? acc[q][i] : 0u;
        // reads of this 64-k-mer tile: from lane 0's to the last valid lane's
        const uint64_t rfirst = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(r >> 32)) << 32) |
                                __builtin_amdgcn_readfirstlane((uint32_t)r);
        const uint32_t last = min(m - 1, t0 + 63) - t0;
        const uint64_t rlast = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(r >> 32), (int)last, 64) << 32) |
                               (uint32_t)__shfl((int)(uint32_t)r, (int)last, 64);
        for (uint64_t rr = rfirst; rr <= rlast; ++rr) {
            const bool mine = valid && r == rr;
            if (!__any(mine)) continue;  // an empty read between two others
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if ((uint32_t)q >= nwords) break;
                const uint32_t c = fold_halves(column_popc32(mine ? w[q] : 0u, X));
                const uint32_t d = q * 32 + (uint32_t)lane;
                if (lane < 32 && d < D && c) {
                    doc_tot[q] += c;
                    if (hits) {
                        if (lds_cnt) atomicAdd(&cnt[rr - lo][d], c);
                        else atomicAdd(&hits[rr * D + d], c);
                    }
                }
            }
        }
    }
    // per-doc totals of the block and its k-mer count: the waves' sums meet in LDS, then one
    // global atomic per doc instead of one per doc and wave
    if (partials) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t d = q * 32 + (uint32_t)lane;
            if (lane < 32 && d < D && doc_tot[q]) atomicAdd(&s_tot[d], (uint32_t)doc_tot[q]);
        }
    }
    __syncthreads();
    if (partials) {
        uint64_t* out = partials + (B % (uint32_t)pblocks) * (D + 1);
        if ((uint32_t)tid < D && s_tot[tid])
            atomicAdd(reinterpret_cast<unsigned long long*>(out + tid), (unsigned long long)s_tot[tid]);
        if (tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(out + D), (unsigned long long)m);
    }
    if (!hits || !lds_cnt) return;
    // reads wholly inside the block: stored; the edge reads: added
    for (uint32_t x = tid; x < nr * D; x += kResolveThreads) {
        const uint32_t ri = x / D, d = x - ri * D;
        const uint64_t rr = lo + ri;
        const bool inside = s_kofs[ri] >= g0 && s_kofs[ri + 1] <= g0 + m;
        const uint32_t c = cnt[ri][d];
        if (inside) hits[rr * D + d] = c;
        else if (c) atomicAdd(&hits[rr * D + d], c);
    }
}

// The hit rows cobs_resolve_kernel does not store whole are zeroed here, so the
// n x D matrix needs no memset: rows of reads without k-mers, of reads whose
// k-mers span two bucket blocks (added atomically by each), and of every read
// of a block with more reads than its LDS counter rows (all added atomically).
template <int CK>
__global__ void part_zero_rows_kernel(const uint64_t* __restrict__ kofs, uint64_t n,
                                      const uint32_t* __restrict__ blk_read, uint32_t D,
                                      uint32_t* __restrict__ hits) {
    const uint64_t Nk = kofs[n];
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = kofs[r], e = kofs[r + 1];
        bool zero = a == e;
        if (!zero) {
            const uint64_t b0 = a / CK, b1 = (e - 1) / CK;
            const uint64_t lo = blk_read[b0];
            const uint64_t hi = (b0 + 1) * CK < Nk ? blk_read[b0 + 1] : n - 1;
            zero = b0 != b1 || hi - lo + 1 > cnt_reads<CK>();
        }
        if (zero)
            for (uint32_t d = 0; d < D; ++d) hits[r * D + d] = 0;
    }
}

}  // namespace

// Bucket blocks of 2048 k-mers: 12.71-12.85 ms per config-2 step against 13.81
// at 1024 and 14.4 at 4096 when measured.
constexpr uint32_t kCobsCK = 2048;

// opt.cobs_part (ProbeOptions): 0 = direct probe only; 1 (default) = partitioned
// probe for classic banks of <= 128 docs of at least kCobsPartMinBankMiB and
// batches of at least kCobsPartMinKmers k-mers; 2 = partitioned for such banks
// of any size; 3 = as 2 with partitions down to 1024 rows (tests reach many
// partitions on small banks); 4 = as 2 with 1024-row partitions (tests reach
// more than kCobsPadParts partitions: unpadded runs).
bool cobs_part_plan(const CobsView& bv, uint32_t k, uint64_t n, uint64_t seq_bytes, uint32_t step,
                    const ProbeOptions& opt, CobsPartPlan* plan) {
    const int mode = opt.cobs_part;
    if (mode <= 0) return false;
    if (bv.G != 1 || bv.pitch != 16 || bv.D > 128 || bv.h == 0 || bv.h > (uint32_t)kMaxH || k > kMaxK) return false;
    const uint64_t sig = bv.sig0;
    if (sig >= (1ull << 30)) return false;  // fastmod_small in the bucket pass
    // banks that (nearly) fit the XCDs' L2s: the direct probe is as fast there
    // (15 MB: 11.09 vs 11.03 ms; 61 MB: 14.40 vs 11.53; profiles/r02_cobspart_banksize.txt)
    if (mode == 1 && sig * 16 < (kCobsPartMinBankMiB << 20)) return false;
    const uint32_t ck = kCobsCK, idb = id_bits<kCobsCK>();
    // 2^17 rows (2 MiB) per partition, fewer rows while that leaves under 64
    // partitions (8 per XCD), more while over kPartMax
    auto parts = [sig](uint32_t s) { return (sig + (1ull << s) - 1) >> s; };
    uint32_t shift = mode == 4 ? 10 : 17;
    const uint32_t floor_shift = mode >= 3 ? 10 : 13;
    while (mode != 4 && shift > floor_shift && parts(shift) < 64) --shift;
    while (parts(shift) > kPartMax) ++shift;
    // entry = (row in partition << idb) | k-mer in block: at shift + idb == 32 the
    // last row's last k-mer would encode to kCobsPadEntry (0xFFFFFFFF); sig < 2^30
    // and kPartMax partitions keep shift <= 20 (a guard, not a reachable case)
    if (shift + idb >= 32) return false;
    const uint64_t kbound = seq_bytes / step + n + 1;  // >= sum of ceil((len-k+1)/step)
    // small batches: the direct probe is faster below ~60-100 k reads of 150 bp
    // (profiles/r02_cobspart_small.txt)
    if (mode == 1 && kbound < kCobsPartMinKmers) return false;
    const uint64_t nblk = (kbound + ck - 1) / ck;
    const uint64_t P = parts(shift);
    // The bucket blocks run in ranges that reuse one workspace of at most
    // opt.workspace_mib MiB of entries + rows (default kCobsPartWsMiB), so
    // any batch size fits.  Runs are padded to 4 entries (64-B row pieces: 4.37
    // -> 3.51 ms for the lookup's write stream alone, tools/runwrite.hip) while
    // the pad slots fit the bucket block's LDS (P <= kCobsPadParts).
    const uint32_t pad = P <= kCobsPadParts ? 4 : 1;
    const uint64_t stride = ((uint64_t)ck * bv.h + (pad - 1) * P + 7) / 8 * 8;
    const uint64_t per_block = stride * (sizeof(uint32_t) + sizeof(uint4));
    const uint64_t cap = (uint64_t)std::max<uint32_t>(1, opt.workspace_mib) << 20;
    // a range holds fewer than 2^32 entries (the lookup's u32 positions)
    const uint64_t rblk = std::max<uint64_t>(1, std::min<uint64_t>({nblk, cap / per_block, ((1ull << 32) - 1) / stride}));
    plan->ck = ck;
    plan->shift = shift;
    plan->P = (uint32_t)P;
    plan->nblk = nblk;
    plan->rblk = rblk;
    plan->kbound = kbound;
    plan->pad = pad;
    plan->stride = stride;
    plan->entry_bytes = rblk * per_block + 128;                      // a range's entries, then their rows (128-B aligned)
    plan->tbl_bytes = 2 * (P + 1) * rblk * sizeof(uint16_t);         // partition- + block-major
    plan->aux_bytes = (nblk + 1 + kQStride) * sizeof(uint32_t) + (size_t)P * kQStride * sizeof(uint32_t);
    plan->nkc_bytes = (n + 1) * sizeof(uint64_t);
    size_t sb = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, sb, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)(n + 1));
    plan->scan_bytes = sb;
    return true;
}

static int cobs_lookup_grid() {
    static std::atomic<int> cache{0};
    return cached_grid(cache, [] {
        int dev = 0, per_cu = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return 768;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, cobs_lookup_kernel<true, kCobsCK>, 256, 0) !=
                hipSuccess || per_cu < 1)
            per_cu = 1;
        const int g = std::min(per_cu, kLookupPerCu) * prop.multiProcessorCount;
        return g >= 8 ? g / 8 * 8 : 8;  // whole groups of 8 blocks (one per XCD)
    });
}

// Ranges of plan.rblk bucket blocks, one after the other on stream s, each
// through bucket -> transpose -> lookup -> resolve in the same workspace.
template <int CK>
static hipError_t cobs_part_pipeline(const ReadView& rv, const PartBank& pb, uint32_t H, const CobsPartPlan& plan,
                                     const PartWs& ws, uint32_t* hits, uint64_t* partials, int blocks,
                                     hipStream_t s, PassRecorder* rec) {
    hipError_t e;
    const uint64_t ne = plan.rblk * plan.stride;
    uint32_t* ent = reinterpret_cast<uint32_t*>(ws.entries);
    uint4* rowv = reinterpret_cast<uint4*>(ent + (ne + 31) / 32 * 32);
    uint32_t* blk_read = ws.aux;
    uint16_t* tbm = ws.tbl + (uint64_t)(plan.P + 1) * plan.rblk;  // block-major copy
    uint32_t* qctr = ws.aux + (plan.nblk + 1 + kQStride - 1) / kQStride * kQStride;  // 128-B aligned
    part_map_kernel<CK><<<grid_for(rv.n, 256, 4096), 256, 0, s>>>(ws.kofs, rv.n, blk_read);
    if (hits)
        part_zero_rows_kernel<CK><<<grid_for(rv.n, 256, 4096), 256, 0, s>>>(ws.kofs, rv.n, blk_read, pb.D, hits);
    pass_mark(rec, kPassPrep, s);
    const bool emb = pb.D <= emb_max_docs<CK>();
    const int grid = cobs_lookup_grid();
    // groups per partition >= the XCD's waves (grid / 8 workgroups x 4 waves)
    const uint64_t waves = (uint64_t)grid / 8 * 4;
    for (uint64_t b0 = 0; b0 < plan.nblk; b0 += plan.rblk) {
        const uint64_t b1 = std::min(plan.nblk, b0 + plan.rblk);
        const unsigned nb = (unsigned)(b1 - b0);
        if (rv.k == 21 && H == 7)
            cobs_bucket_kernel<21, 7, CK><<<nb, bucket_threads<CK>(), 0, s>>>(rv, pb, H, ws.kofs, plan.shift, plan.P,
                                                                            ent, tbm, blk_read, b0, plan.stride,
                                                                            plan.pad);
        else
            cobs_bucket_kernel<0, 0, CK><<<nb, bucket_threads<CK>(), 0, s>>>(rv, pb, H, ws.kofs, plan.shift, plan.P,
                                                                           ent, tbm, blk_read, b0, plan.stride,
                                                                           plan.pad);
        part_transpose_kernel<<<dim3((nb + 63) / 64, (plan.P + 1 + 63) / 64), 256, 0, s>>>(
            tbm, plan.P + 1, plan.rblk, ws.tbl, 0, nb);
        if ((e = hipMemsetAsync(qctr, 0, (size_t)plan.P * kQStride * sizeof(uint32_t), s)) != hipSuccess) return e;
        pass_mark(rec, kPassBucket, s);
        const uint32_t gb = (uint32_t)std::min<uint64_t>(64, std::max<uint64_t>(1, (b1 - b0) / std::max<uint64_t>(1, waves)));
        if (emb)
            cobs_lookup_kernel<true, CK><<<grid, 256, 0, s>>>(pb, ws.kofs, rv.n, H, plan.shift, plan.P, plan.rblk, ent,
                                                              ws.tbl, rowv, qctr, b0, b1, gb, plan.stride);
        else
            cobs_lookup_kernel<false, CK><<<grid, 256, 0, s>>>(pb, ws.kofs, rv.n, H, plan.shift, plan.P, plan.rblk,
                                                               ent, ws.tbl, rowv, qctr, b0, b1, gb, plan.stride);
        pass_mark(rec, kPassLookup, s);
        if (emb)
            cobs_resolve_kernel<true, CK><<<nb, resolve_threads<CK>(), 0, s>>>(
                rv, ws.kofs, H, pb.D, pb.nwords, ent, rowv, blk_read, hits, partials, blocks, b0, plan.stride, tbm,
                plan.P + 1);
        else
            cobs_resolve_kernel<false, CK><<<nb, resolve_threads<CK>(), 0, s>>>(
                rv, ws.kofs, H, pb.D, pb.nwords, ent, rowv, blk_read, hits, partials, blocks, b0, plan.stride, tbm,
                plan.P + 1);
        pass_mark(rec, kPassResolve, s);
    }
    return hipGetLastError();
}

hipError_t launch_probe_cobs_part(const ReadView& rv, const CobsView& bv, const CobsPartPlan& plan,
                                  const PartWs& ws, uint32_t* hits, uint64_t* partials, int blocks,
                                  hipStream_t s, PassRecorder* rec) {
    pass_mark(rec, kPassStart, s);
    PartBank pb;
    pb.rows = reinterpret_cast<const uint4*>(bv.rows);
    pb.sig = bv.sig0;
    pb.magic = barrett_magic(bv.sig0);
    pb.D = (uint32_t)bv.D;
    pb.nwords = (uint32_t)((bv.D + 31) / 32);
    hipError_t e;
    // (the hit rows the resolve does not store are zeroed by part_zero_rows_kernel)
    if (partials && (e = hipMemsetAsync(partials, 0, (size_t)blocks * (bv.D + 1) * sizeof(uint64_t), s)) != hipSuccess)
        return e;
    part_counts_kernel<<<grid_for(rv.n + 1, 256, 4096), 256, 0, s>>>(rv.offs, rv.n, rv.k, rv.step, ws.nkc);
    size_t sb = ws.scan_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(ws.scan_tmp, sb, ws.nkc, ws.kofs, (int)(rv.n + 1), s)) != hipSuccess)
        return e;
    return cobs_part_pipeline<kCobsCK>(rv, pb, bv.h, plan, ws, hits, partials, blocks, s, rec);
}

}  // namespace xs
