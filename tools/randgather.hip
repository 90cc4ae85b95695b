// randgather.hip — ceiling of random 16-byte row gathers on this GPU.
//
// Each lane draws pseudo-random row indices (splitmix64) into a table of
// `rows` 16-byte rows and ANDs NL rows per "k-mer" (NL loads in flight per
// lane, as the probe kernel issues its h = 7 row loads).  Reports gathered
// rows/s and GB/s at 64 B per row (one HBM/MALL transaction per row).
//   hipcc -O3 --offload-arch=gfx950 tools/randgather.hip -o /tmp/randgather
//   /tmp/randgather [table_MB ...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                         \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

template <int NL>
__global__ void __launch_bounds__(256) gather(const uint4* __restrict__ tab, uint64_t rows,
                                              uint64_t iters, uint32_t* out) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint64_t it = 0; it < iters; ++it) {
        uint4 m = make_uint4(~0u, ~0u, ~0u, ~0u);
        uint32_t idx[NL];
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            uint32_t x = (uint32_t)tid * 0x9E3779B1u + (uint32_t)(it * NL + j) * 0x85EBCA77u;
            x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
            idx[j] = (uint32_t)(((uint64_t)x * rows) >> 32);  // multiply-shift range map
        }
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const uint4 v = tab[idx[j]];
            m.x &= v.x; m.y &= v.y; m.z &= v.z; m.w &= v.w;
        }
        acc += m.x ^ m.y ^ m.z ^ m.w;
    }
    if (acc == 0x12345678u) out[0] = acc;  // keep the loads live
}

int main(int argc, char** argv) {
    std::vector<double> sizes;
    for (int i = 1; i < argc; ++i) sizes.push_back(atof(argv[i]));
    if (sizes.empty()) sizes = {16, 64, 200, 614, 2048, 8192};
    int dev = 0;
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, dev));
    const int cus = prop.multiProcessorCount;
    uint32_t* out;
    CHK(hipMalloc(&out, 4));
    printf("{\"cus\": %d, \"results\": [\n", cus);
    bool first = true;
    for (double mb : sizes) {
        const uint64_t bytes = (uint64_t)(mb * 1048576.0) / 16 * 16;
        const uint64_t rows = bytes / 16;
        uint4* tab;
        CHK(hipMalloc(&tab, bytes));
        CHK(hipMemset(tab, 0xA5, bytes));
        for (int blocks_per_cu : {4, 8}) {
            const int grid = cus * blocks_per_cu;
            const uint64_t threads = (uint64_t)grid * 256;
            const uint64_t iters = 64;
            hipEvent_t a, b;
            CHK(hipEventCreate(&a));
            CHK(hipEventCreate(&b));
            gather<7><<<grid, 256>>>(tab, rows, 4, out);  // warm
            CHK(hipDeviceSynchronize());
            CHK(hipEventRecord(a));
            gather<7><<<grid, 256>>>(tab, rows, iters, out);
            CHK(hipEventRecord(b));
            CHK(hipEventSynchronize(b));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, a, b));
            const double loads = (double)threads * iters * 7;
            printf("%s  {\"table_MB\": %.0f, \"blocks_per_cu\": %d, \"ms\": %.3f, \"Grows_per_s\": %.2f, "
                   "\"GBps_at_64B\": %.0f}", first ? "" : ",\n", mb, blocks_per_cu, ms,
                   loads / ms / 1e6, loads * 64 / ms / 1e6);
            first = false;
            CHK(hipEventDestroy(a));
            CHK(hipEventDestroy(b));
        }
        CHK(hipFree(tab));
    }
    printf("\n]}\n");
    return 0;
}
