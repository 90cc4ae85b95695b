// runwrite.hip — write pattern of the partitioned COBS lookup, isolated.
//
// The lookup writes each entry's 16-B row back in entry order: bucket block B
// owns a region of CK*h entries, split into P runs (one per bank partition,
// ~49 entries each at CK=2048, h=7, P=293), and the runs of partition p for a
// group of 64 blocks are written together, partition after partition.  This
// measures that write stream alone (no gathers) with the run starts at their
// natural 16-B offsets, padded to 64 B or 128 B, against one sequential
// stream of the same bytes.
//   hipcc -O3 --offload-arch=gfx950 tools/runwrite.hip -o tools/runwrite
//   tools/runwrite [blocks] [P]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHK(x)                                                      \
    do {                                                            \
        hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) {                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
            exit(1);                                                \
        }                                                           \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kGroup = 64;

// item = (partition p, group of kGroup blocks), partition-major
__global__ void __launch_bounds__(256) runs(const uint32_t* __restrict__ start,  // [NB][P+1] entry offsets
                                            const uint64_t* __restrict__ base,   // [NB] region start (entries)
                                            uint32_t NB, uint32_t P, uint32_t* ctr, u32x4* __restrict__ out) {
    __shared__ uint32_t s_it;
    const uint32_t ngroups = (NB + kGroup - 1) / kGroup;
    const uint32_t total = ngroups * P;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (;;) {
        if (threadIdx.x == 0) s_it = atomicAdd(ctr, 1u);
        __syncthreads();
        const uint32_t it = s_it;
        __syncthreads();
        if (it >= total) break;
        const uint32_t p = it / ngroups, g = it % ngroups;
        for (uint32_t b = g * kGroup + wave; b < min(NB, (g + 1) * kGroup); b += 4) {
            const uint32_t s0 = start[(uint64_t)b * (P + 1) + p], s1 = start[(uint64_t)b * (P + 1) + p + 1];
            for (uint32_t e = s0 + lane; e < s1; e += 64) {
                const u32x4 v = {e, p, b, 0x5A5A5A5Au};
                __builtin_nontemporal_store(v, out + base[b] + e);
            }
        }
    }
}

// The resolve's side of a partition-major layout: workgroup b reads block b's P runs, each
// stored at its partition's region (run (b, p) at pstart[p] + prefix over blocks < b).
__global__ void __launch_bounds__(256) runs_read(const uint32_t* __restrict__ cnt,   // [NB][P] run lengths
                                                 const uint64_t* __restrict__ at,    // [NB][P] run starts
                                                 uint32_t NB, uint32_t P, const u32x4* __restrict__ in,
                                                 uint32_t* __restrict__ sink) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t acc = 0;
    for (uint32_t b = blockIdx.x; b < NB; b += gridDim.x) {
        for (uint32_t p = wave; p < P; p += 4) {
            const uint32_t c = cnt[(uint64_t)b * P + p];
            const uint64_t a = at[(uint64_t)b * P + p];
            for (uint32_t e = lane; e < c; e += 64) {
                const u32x4 v = __builtin_nontemporal_load(in + a + e);
                acc += v[0] ^ v[3];
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) seq_read(uint64_t n, const u32x4* __restrict__ in, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const u32x4 v = __builtin_nontemporal_load(in + i);
        acc += v[0] ^ v[3];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) seq(uint64_t n, u32x4* __restrict__ out) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const u32x4 v = {(uint32_t)i, 1, 2, 3};
        __builtin_nontemporal_store(v, out + i);
    }
}

int main(int argc, char** argv) {
    const uint32_t NB = argc > 1 ? atoi(argv[1]) : 63477;
    const uint32_t P = argc > 2 ? atoi(argv[2]) : 293;
    const uint32_t per = 2048 * 7;
    std::mt19937_64 rng(7);
    // run lengths: multinomial(per, 1/P) per block
    std::vector<uint32_t> cnt((size_t)NB * P);
    for (uint32_t b = 0; b < NB; ++b) {
        uint32_t* c = &cnt[(size_t)b * P];
        for (uint32_t i = 0; i < per; ++i) c[rng() % P]++;
    }
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    u32x4* out = nullptr;
    const uint64_t cap = (uint64_t)NB * (per + P * 8) + 64;
    CHK(hipMalloc(&out, cap * 16));
    uint32_t* ctr = nullptr;
    CHK(hipMalloc(&ctr, 4));
    for (int align : {1, 4, 8}) {
        std::vector<uint32_t> st((size_t)NB * (P + 1));
        std::vector<uint64_t> bs(NB);
        uint64_t tot = 0, used = 0;
        for (uint32_t b = 0; b < NB; ++b) {
            uint32_t o = 0;
            for (uint32_t p = 0; p < P; ++p) {
                st[(size_t)b * (P + 1) + p] = o;
                o += (cnt[(size_t)b * P + p] + align - 1) / align * align;
                used += cnt[(size_t)b * P + p];
            }
            st[(size_t)b * (P + 1) + P] = o;
            bs[b] = tot;
            tot += (o + 7) / 8 * 8;
        }
        // lengths are padded; the kernel writes the padded runs (pad slots too)
        uint32_t* d_st = nullptr;
        uint64_t* d_bs = nullptr;
        CHK(hipMalloc(&d_st, st.size() * 4));
        CHK(hipMalloc(&d_bs, bs.size() * 8));
        CHK(hipMemcpy(d_st, st.data(), st.size() * 4, hipMemcpyHostToDevice));
        CHK(hipMemcpy(d_bs, bs.data(), bs.size() * 8, hipMemcpyHostToDevice));
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            CHK(hipMemset(ctr, 0, 4));
            CHK(hipEventRecord(e0));
            runs<<<cus * 3, 256>>>(d_st, d_bs, NB, P, ctr, out);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        printf("runs align %d entries: %.3f ms, %.2f GB written (%.2f GB useful), %.0f GB/s\n", align, best,
               tot * 16e-9, used * 16e-9, tot * 16e-9 / (best * 1e-3));
        CHK(hipFree(d_st));
        CHK(hipFree(d_bs));
    }
    const uint64_t n = (uint64_t)NB * per;
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHK(hipEventRecord(e0));
        seq<<<cus * 8, 256>>>(n, out);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    printf("sequential: %.3f ms, %.2f GB, %.0f GB/s\n", best, n * 16e-9, n * 16e-9 / (best * 1e-3));
    {
        // partition-major layout: run (b, p) at pbase[p] + sum of cnt[b' < b][p]
        std::vector<uint64_t> at((size_t)NB * P);
        uint64_t o = 0;
        for (uint32_t p = 0; p < P; ++p)
            for (uint32_t b = 0; b < NB; ++b) {
                at[(size_t)b * P + p] = o;
                o += cnt[(size_t)b * P + p];
            }
        uint32_t* d_cnt = nullptr;
        uint64_t* d_at = nullptr;
        uint32_t* sink = nullptr;
        CHK(hipMalloc(&d_cnt, cnt.size() * 4));
        CHK(hipMalloc(&d_at, at.size() * 8));
        CHK(hipMalloc(&sink, 4));
        CHK(hipMemcpy(d_cnt, cnt.data(), cnt.size() * 4, hipMemcpyHostToDevice));
        CHK(hipMemcpy(d_at, at.data(), at.size() * 8, hipMemcpyHostToDevice));
        for (int per : {2, 3, 4}) {
            float bt = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                CHK(hipEventRecord(e0));
                runs_read<<<cus * per, 256>>>(d_cnt, d_at, NB, P, out, sink);
                CHK(hipEventRecord(e1));
                CHK(hipEventSynchronize(e1));
                float ms = 0;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                bt = ms < bt ? ms : bt;
            }
            printf("partition-major runs read block by block (%d workgroups/CU): %.3f ms, %.0f GB/s\n", per, bt,
                   o * 16e-9 / (bt * 1e-3));
        }
        float bt = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            CHK(hipEventRecord(e0));
            seq_read<<<cus * 8, 256>>>(o, out, sink);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            bt = ms < bt ? ms : bt;
        }
        printf("sequential read: %.3f ms, %.0f GB/s\n", bt, o * 16e-9 / (bt * 1e-3));
    }
    CHK(hipFree(out));
    return 0;
}
