// ldslookup.hip — can the COBS lookup serve its rows from LDS instead of L2?
//
// Today's lookup (xs_probe_cobspart.hip) gathers each entry's 16-B row from a
// 2 MiB bank partition kept in the XCD's L2; beside the entry reads and row
// stores that stream through the same L2s the gathers run at ~145 G/s
// (profiles/r02_l2gather_parts.txt), and the lookup is 55 % of the step.
// Variant B keeps a 128 KiB *fine* partition (8192 rows) in one CU's LDS: the
// bucket blocks' coarse runs are sorted by fine partition (16 per coarse
// partition) with one u8 start per (block, fine partition), and the workgroup
// that holds fine partition f reads only f's sub-runs (~3 entries a block at
// config 2), takes the rows from LDS and writes them back in entry order.  The
// 16 fine partitions of a coarse partition run at the same time on one XCD,
// so the sub-runs of one coarse run share their lines in that XCD's L2.
//
// Both lookups run here on the same synthetic config-2-shaped entries
// (38.37 M-row bank, 63477 blocks of 2048 k-mers x 7 rows, uniform random
// rows) and their row outputs are compared byte for byte.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ldslookup.hip -o tools/ldslookup
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                    \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

constexpr int CK = 2048, IDB = 11, H = 7;
constexpr uint32_t SHIFT = 17;      // coarse partition: 2^17 rows (2 MiB)
constexpr uint32_t FSHIFT = 13;     // fine partition: 2^13 rows (128 KiB)
constexpr uint32_t FPC = 1u << (SHIFT - FSHIFT);  // fine partitions per coarse one
constexpr uint32_t PAD_ENTRY = 0xFFFFFFFFu;
constexpr int GT = 1024;            // generator threads
constexpr uint32_t kPFMax = 8192;   // fine partitions the generator's LDS counters hold
constexpr uint32_t kQ = 32;         // u32 per queue counter (own 128-B line)

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

// One bucket block: 2048 k-mers x 7 uniform rows, binned by fine partition in
// LDS, coarse runs padded to 4 entries (pad slots after the run's last fine
// part), copied out; coarse starts (u16, P+1 per block) and fine starts
// within their coarse run (u8, PF per block).
__global__ void __launch_bounds__(GT) gen_kernel(uint32_t sig, uint32_t P, uint32_t PF, uint64_t stride,
                                                 uint32_t* __restrict__ ent, uint16_t* __restrict__ tbm,
                                                 uint8_t* __restrict__ fbm) {
    using Scan = hipcub::BlockScan<uint32_t, GT>;
    __shared__ typename Scan::TempStorage tmp;
    __shared__ uint32_t cnt[kPFMax];
    __shared__ uint32_t s_ent[CK * H + 3 * 1024];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    for (uint32_t f = tid; f < PF; f += GT) cnt[f] = 0;
    __syncthreads();
    constexpr int PER = CK * H / GT;  // 14
    uint32_t row[PER], rk[PER], kid[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t x = tid * PER + q;  // (k-mer, hash) pair
        kid[q] = x / H;
        row[q] = (uint32_t)(((uint64_t)mix32(b * 0x9E3779B1u ^ mix32(x + 0x1234567u)) * sig) >> 32);
        rk[q] = atomicAdd(&cnt[row[q] >> FSHIFT], 1u);
    }
    __syncthreads();
    // thread t owns coarse partition t (P <= GT): its fine counts, run length, pad
    uint32_t c[FPC], sum = 0;
    const uint32_t p = tid;
#pragma unroll
    for (uint32_t s = 0; s < FPC; ++s) {
        const uint32_t f = p * FPC + s;
        c[s] = (p < P && f < PF) ? cnt[f] : 0u;
        sum += c[s];
    }
    const uint32_t run = p < P ? (sum + 3) & ~3u : 0u;
    uint32_t cs, tot;
    Scan(tmp).ExclusiveSum(run, cs, tot);
    __syncthreads();
    if (p < P) {
        tbm[(uint64_t)b * (P + 1) + p] = (uint16_t)cs;
        uint32_t o = cs;
#pragma unroll
        for (uint32_t s = 0; s < FPC; ++s) {
            const uint32_t f = p * FPC + s;
            if (f < PF) {
                cnt[f] = o;
                fbm[(uint64_t)b * PF + f] = (uint8_t)(o - cs);
            }
            o += c[s];
        }
        for (; o < cs + run; ++o) s_ent[o] = PAD_ENTRY;
    }
    if (tid == 0) tbm[(uint64_t)b * (P + 1) + P] = (uint16_t)tot;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q)
        s_ent[cnt[row[q] >> FSHIFT] + rk[q]] = ((row[q] & ((1u << SHIFT) - 1)) << IDB) | kid[q];
    __syncthreads();
    for (uint32_t e = tid; e < tot; e += GT) ent[(uint64_t)b * stride + e] = s_ent[e];
}

template <typename T>
__global__ void transpose_kernel(const T* __restrict__ in, uint32_t cols, uint64_t rows, T* __restrict__ out) {
    // in: rows x cols (block-major), out: cols x rows (partition-major)
    __shared__ T t[64][65];
    const uint64_t r0 = (uint64_t)blockIdx.x * 64;
    const uint32_t c0 = blockIdx.y * 64;
    for (uint32_t x = threadIdx.x; x < 64 * 64; x += 256) {
        const uint32_t ri = x / 64, ci = x % 64;
        if (r0 + ri < rows && c0 + ci < cols) t[ri][ci] = in[(r0 + ri) * cols + c0 + ci];
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < 64 * 64; x += 256) {
        const uint32_t ci = x / 64, ri = x % 64;
        if (r0 + ri < rows && c0 + ci < cols) out[(c0 + ci) * rows + r0 + ri] = t[ri][ci];
    }
}

__device__ __forceinline__ void store_row(uint4* out, uint64_t pos, uint4 v, uint32_t e) {
    v.w = (v.w & (0xFFFFFFFFu >> IDB)) | (e << (32 - IDB));
    uint32_t* o = reinterpret_cast<uint32_t*>(out + pos);
    __builtin_nontemporal_store(v.x, o);
    __builtin_nontemporal_store(v.y, o + 1);
    __builtin_nontemporal_store(v.z, o + 2);
    __builtin_nontemporal_store(v.w, o + 3);
}

// A: today's lookup (cobs_lookup_kernel<6, EMB, 2048, DMA=1>), restated.
__global__ void __launch_bounds__(256) lookup_l2(const uint4* __restrict__ bank, uint32_t P, uint64_t nblk,
                                                 const uint32_t* __restrict__ ent, const uint16_t* __restrict__ tbl,
                                                 uint4* __restrict__ out, uint32_t* qctr, uint64_t stride) {
    constexpr int U = 6;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ uint4 s_rows[4][U][64];
    const uint32_t xcd = blockIdx.x & 7;
    for (uint64_t p = xcd; p < P; p += 8) {
        const uint4* prow = bank + (p << SHIFT);
        const uint16_t* t0 = tbl + p * nblk;
        const uint16_t* t1 = t0 + nblk;
        for (;;) {
            uint32_t grp = 0;
            if (lane == 0) grp = atomicAdd(&qctr[p * kQ], 1u);
            const uint64_t b0 = (uint64_t)__builtin_amdgcn_readfirstlane(grp) * 64;
            if (b0 >= nblk) break;
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
            for (uint32_t i0 = 0; i0 < total; i0 += 64 * U) {
                uint64_t pos[U];
                uint32_t e[U];
                uint4 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t i = i0 + u * 64 + lane;
                    int j = 0;
#pragma unroll
                    for (int st = 32; st; st >>= 1) {
                        const uint32_t pv = (uint32_t)__shfl((int)pre, j + st, 64);
                        if (pv <= i) j += st;
                    }
                    const uint32_t sj = (uint32_t)__shfl((int)s, j, 64);
                    const uint32_t pj = (uint32_t)__shfl((int)pre, j, 64);
                    pos[u] = (b0 + j) * stride + sj + (i - pj);
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    e[u] = i0 + u * 64 + lane < total ? __builtin_nontemporal_load(ent + pos[u]) : 0u;
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (i0 + u * 64 + lane < total && e[u] != PAD_ENTRY) {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        __builtin_amdgcn_global_load_lds(prow + (e[u] >> IDB), &s_rows[wid][u][0], 16, 0, 0);
                    }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int u = 0; u < U; ++u) v[u] = s_rows[wid][u][lane];
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (e[u] == PAD_ENTRY) {
                        v[u] = make_uint4(~0u, ~0u, ~0u, ~0u);
                        e[u] = (uint32_t)pos[u] & (CK - 1);
                    }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (i0 + u * 64 + lane < total) store_row(out, pos[u], v[u], e[u]);
            }
        }
    }
}

// A2: today's lookup with the entry -> block map built in LDS per window of W
// entries (each lane writes its block's position base over its run's slots,
// then every entry reads its base) instead of a 6-step shuffle binary search
// per entry: ~2 LDS operations per 64 entries instead of 8 shuffles.
template <int W>
__global__ void __launch_bounds__(256) lookup_l2_own(const uint4* __restrict__ bank, uint32_t P, uint64_t nblk,
                                                     const uint32_t* __restrict__ ent,
                                                     const uint16_t* __restrict__ tbl, uint4* __restrict__ out,
                                                     uint32_t* qctr, uint64_t stride) {
    constexpr int U = 6;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ uint4 s_rows[4][U][64];
    __shared__ uint32_t s_base[4][W];
    const uint32_t xcd = blockIdx.x & 7;
    for (uint64_t p = xcd; p < P; p += 8) {
        const uint4* prow = bank + (p << SHIFT);
        const uint16_t* t0 = tbl + p * nblk;
        const uint16_t* t1 = t0 + nblk;
        for (;;) {
            uint32_t grp = 0;
            if (lane == 0) grp = atomicAdd(&qctr[p * kQ], 1u);
            const uint64_t b0 = (uint64_t)__builtin_amdgcn_readfirstlane(grp) * 64;
            if (b0 >= nblk) break;
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
            // position of entry i of this group = base of its block + i (u32: the workspace
            // holds < 2^32 entries)
            const uint32_t base = (uint32_t)(b * stride + s - pre);
            for (uint32_t w0 = 0; w0 < total; w0 += W) {
                const uint32_t lo = max(pre, w0), hi = min(pre + len, w0 + W);
                for (uint32_t x = lo; x < hi; ++x) s_base[wid][x - w0] = base;
                __builtin_amdgcn_wave_barrier();
                const uint32_t wend = min(total, w0 + W);
                for (uint32_t i0 = w0; i0 < wend; i0 += 64 * U) {
                    uint32_t pos[U], e[U];
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
                        if (i0 + u * 64 + lane < wend && e[u] != PAD_ENTRY) {
                            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                            __builtin_amdgcn_global_load_lds(prow + (e[u] >> IDB), &s_rows[wid][u][0], 16, 0, 0);
                        }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                    for (int u = 0; u < U; ++u) v[u] = s_rows[wid][u][lane];
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (e[u] == PAD_ENTRY) {
                            v[u] = make_uint4(~0u, ~0u, ~0u, ~0u);
                            e[u] = pos[u] & (CK - 1);
                        }
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (i0 + u * 64 + lane < wend) store_row(out, pos[u], v[u], e[u]);
                }
                __builtin_amdgcn_wave_barrier();  // the window's bases are read before the next overwrite
            }
        }
    }
}

// B: fine partition f (8192 rows) in LDS; the workgroup's waves take groups of
// 64 blocks from an LDS counter and copy f's rows for their sub-runs.
template <int U, int WT>
__global__ void __launch_bounds__(WT, 1) lookup_lds(const uint4* __restrict__ bank, uint32_t sig, uint32_t P,
                                                    uint32_t PF, uint64_t nblk, const uint32_t* __restrict__ ent,
                                                    const uint16_t* __restrict__ tbl, const uint8_t* __restrict__ ftbl,
                                                    uint4* __restrict__ out, uint32_t* qx, uint64_t stride) {
    __shared__ uint4 s_part[1u << FSHIFT];
    __shared__ uint32_t s_f, s_g;
    const int lane = threadIdx.x & 63;
    const uint32_t xcd = blockIdx.x & 7;
    for (;;) {
        if (threadIdx.x == 0) {
            s_f = atomicAdd(&qx[xcd * kQ], 1u);
            s_g = 0;
        }
        __syncthreads();
        const uint32_t c = s_f;
        const uint32_t p = xcd + 8 * (c / FPC), f = p * FPC + c % FPC;
        if (p >= P) break;  // uniform: every wave leaves
        if (f < PF) {
            const uint32_t r0 = f << FSHIFT;
            const uint32_t nr = min(1u << FSHIFT, sig - r0);
            for (uint32_t r = threadIdx.x; r < nr; r += WT) s_part[r] = bank[r0 + r];
            __syncthreads();
            const uint16_t* t0 = tbl + (uint64_t)p * nblk;
            const uint16_t* t1 = t0 + nblk;
            const uint8_t* f0 = ftbl + (uint64_t)f * nblk;
            const bool last = (f + 1) % FPC == 0 || f + 1 == PF;  // its sub-run ends the coarse run
            const uint8_t* f1 = last ? nullptr : f0 + nblk;
            for (;;) {
                uint32_t grp = 0;
                if (lane == 0) grp = atomicAdd(&s_g, 1u);
                const uint64_t b0 = (uint64_t)__builtin_amdgcn_readfirstlane(grp) * 64;
                if (b0 >= nblk) break;
                const uint64_t b = b0 + lane;
                uint32_t s = 0, len = 0;
                if (b < nblk) {
                    const uint32_t cs = t0[b];
                    s = cs + f0[b];
                    len = (last ? (uint32_t)t1[b] : cs + f1[b]) - s;
                }
                uint32_t inc = len;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t t = (uint32_t)__shfl_up((int)inc, d, 64);
                    if (lane >= d) inc += t;
                }
                const uint32_t pre = inc - len;
                const uint32_t total = (uint32_t)__shfl((int)inc, 63, 64);
                for (uint32_t i0 = 0; i0 < total; i0 += 64 * U) {
                    uint64_t pos[U];
                    uint32_t e[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t i = i0 + u * 64 + lane;
                        int j = 0;
#pragma unroll
                        for (int st = 32; st; st >>= 1) {
                            const uint32_t pv = (uint32_t)__shfl((int)pre, j + st, 64);
                            if (pv <= i) j += st;
                        }
                        const uint32_t sj = (uint32_t)__shfl((int)s, j, 64);
                        const uint32_t pj = (uint32_t)__shfl((int)pre, j, 64);
                        pos[u] = (b0 + j) * stride + sj + (i - pj);
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        e[u] = i0 + u * 64 + lane < total ? __builtin_nontemporal_load(ent + pos[u]) : 0u;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if (i0 + u * 64 + lane < total) {
                            uint4 v;
                            uint32_t id = e[u];
                            if (e[u] == PAD_ENTRY) {
                                v = make_uint4(~0u, ~0u, ~0u, ~0u);
                                id = (uint32_t)pos[u] & (CK - 1);
                            } else {
                                v = s_part[(e[u] >> IDB) & ((1u << FSHIFT) - 1)];
                            }
                            store_row(out, pos[u], v, id);
                        }
                    }
                }
            }
        }
        __syncthreads();  // every wave is done with s_part and s_f
    }
}

__global__ void cmp_kernel(const uint4* a, const uint4* b, uint64_t n, unsigned long long* bad) {
    unsigned long long c = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 x = a[i], y = b[i];
        c += (x.x != y.x) | (x.y != y.y) | (x.z != y.z) | (x.w != y.w);
    }
    if (c) atomicAdd(bad, c);
}

__global__ void fill_bank(uint4* bank, uint32_t sig) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < sig; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t x = (uint32_t)i;
        bank[i] = make_uint4(mix32(x), mix32(x ^ 0x55555555u), mix32(x ^ 0xAAAAAAAAu), mix32(x + 7u) & 0xFu);
    }
}

int main(int argc, char** argv) {
    const uint32_t sig = 38371628u;
    const uint64_t nblk = argc > 1 ? strtoull(argv[1], nullptr, 10) : 63477;  // 130 M k-mers / 2048
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const uint32_t P = (sig + (1u << SHIFT) - 1) >> SHIFT;
    const uint32_t PF = (sig + (1u << FSHIFT) - 1) >> FSHIFT;
    const uint64_t stride = ((uint64_t)CK * H + 3 * P + 7) / 8 * 8;
    if (P > 1024 || PF > kPFMax) { fprintf(stderr, "bank too large for this tool\n"); return 1; }
    printf("sig %u rows, P %u coarse, PF %u fine, %llu blocks, stride %llu\n", sig, P, PF,
           (unsigned long long)nblk, (unsigned long long)stride);
    uint4 *bank, *outA, *outB;
    uint32_t *ent, *qctr, *qx;
    uint16_t *tbm, *tbl;
    uint8_t *fbm, *ftbl;
    unsigned long long* bad;
    CHK(hipMalloc(&bank, (size_t)sig * 16));
    CHK(hipMalloc(&ent, nblk * stride * 4));
    CHK(hipMalloc(&outA, nblk * stride * 16));
    CHK(hipMalloc(&outB, nblk * stride * 16));
    CHK(hipMalloc(&tbm, nblk * (P + 1) * 2));
    CHK(hipMalloc(&tbl, nblk * (P + 1) * 2));
    CHK(hipMalloc(&fbm, nblk * PF));
    CHK(hipMalloc(&ftbl, nblk * PF));
    CHK(hipMalloc(&qctr, (size_t)P * kQ * 4));
    CHK(hipMalloc(&qx, 8 * kQ * 4));
    CHK(hipMalloc(&bad, 8));
    fill_bank<<<4096, 256>>>(bank, sig);
    CHK(hipMemset(ent, 0, nblk * stride * 4));
    gen_kernel<<<(unsigned)nblk, GT>>>(sig, P, PF, stride, ent, tbm, fbm);
    CHK(hipGetLastError());
    transpose_kernel<uint16_t><<<dim3((unsigned)((nblk + 63) / 64), (P + 1 + 63) / 64), 256>>>(tbm, P + 1, nblk, tbl);
    transpose_kernel<uint8_t><<<dim3((unsigned)((nblk + 63) / 64), (PF + 63) / 64), 256>>>(fbm, PF, nblk, ftbl);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const double entries = (double)nblk * CK * H;
    int ncu = 256;
    {
        hipDeviceProp_t prop;
        CHK(hipGetDeviceProperties(&prop, 0));
        ncu = prop.multiProcessorCount;
    }
    auto run = [&](const char* name, auto launch, uint32_t* q, size_t qbytes) {
        float best = 1e30f, sum = 0;
        for (int r = 0; r < reps + 1; ++r) {
            CHK(hipMemset(q, 0, qbytes));
            CHK(hipEventRecord(e0));
            launch();
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            CHK(hipGetLastError());
            float ms;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            if (r == 0) continue;  // warm-up
            best = std::min(best, ms);
            sum += ms;
        }
        printf("%-34s best %.3f ms avg %.3f ms  %.1f G entries/s  %.2f TB/s streamed (4 B in + 16 B out)\n", name,
               best, sum / reps, entries / best / 1e6, entries * 20 / best / 1e9);
    };
    CHK(hipMemset(outA, 0, nblk * stride * 16));
    CHK(hipMemset(outB, 0, nblk * stride * 16));
    run("A: L2 partitions (today)", [&] { lookup_l2<<<2 * ncu, 256>>>(bank, P, nblk, ent, tbl, outA, qctr, stride); },
        qctr, (size_t)P * kQ * 4);
    unsigned long long nb = 0;
    auto compare = [&](const char* what) {
        CHK(hipMemset(bad, 0, 8));
        cmp_kernel<<<4096, 256>>>(outA, outB, nblk * stride, bad);
        CHK(hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost));
        printf("row slots differing between A and %s: %llu\n", what, nb);
        if (nb) exit(2);
        CHK(hipMemset(outB, 0, nblk * stride * 16));
    };
    run("A2: owner map W=1024", [&] { lookup_l2_own<1024><<<2 * ncu, 256>>>(bank, P, nblk, ent, tbl, outB, qctr, stride); },
        qctr, (size_t)P * kQ * 4);
    compare("A2");
    run("A2: owner map W=2048", [&] { lookup_l2_own<2048><<<2 * ncu, 256>>>(bank, P, nblk, ent, tbl, outB, qctr, stride); },
        qctr, (size_t)P * kQ * 4);
    compare("A2 W=2048");
    run("A: L2 partitions (today), again", [&] { lookup_l2<<<2 * ncu, 256>>>(bank, P, nblk, ent, tbl, outA, qctr, stride); },
        qctr, (size_t)P * kQ * 4);
    run("A2: owner map W=1024, again", [&] { lookup_l2_own<1024><<<2 * ncu, 256>>>(bank, P, nblk, ent, tbl, outB, qctr, stride); },
        qctr, (size_t)P * kQ * 4);
    compare("A2 again");
    if (argc > 3) return 0;  // owner-map A/B only
    run("B: LDS fine partitions, 1024 thr U4",
        [&] { lookup_lds<4, 1024><<<ncu, 1024>>>(bank, sig, P, PF, nblk, ent, tbl, ftbl, outB, qx, stride); }, qx,
        8 * kQ * 4);
    CHK(hipMemset(bad, 0, 8));
    cmp_kernel<<<4096, 256>>>(outA, outB, nblk * stride, bad);
    CHK(hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost));
    printf("row slots differing between A and B: %llu\n", nb);
    CHK(hipMemset(outB, 0, nblk * stride * 16));
    run("B: LDS fine partitions, 1024 thr U2",
        [&] { lookup_lds<2, 1024><<<ncu, 1024>>>(bank, sig, P, PF, nblk, ent, tbl, ftbl, outB, qx, stride); }, qx,
        8 * kQ * 4);
    run("B: LDS fine partitions, 512 thr U4",
        [&] { lookup_lds<4, 512><<<ncu, 512>>>(bank, sig, P, PF, nblk, ent, tbl, ftbl, outB, qx, stride); }, qx,
        8 * kQ * 4);
    CHK(hipMemset(bad, 0, 8));
    cmp_kernel<<<4096, 256>>>(outA, outB, nblk * stride, bad);
    CHK(hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost));
    printf("row slots differing between A and B (last variant): %llu\n", nb);
    return nb ? 2 : 0;
}
