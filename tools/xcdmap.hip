// Which XCD runs each block of a resident-sized grid (checks the blockIdx % 8
// grouping the partitioned rbloom lookup relies on for L2 affinity).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) who(unsigned* xcc, unsigned long long* sink, int spin) {
    if (threadIdx.x == 0) xcc[blockIdx.x] = __builtin_amdgcn_s_getreg((3 << 11) | 20) & 15;  // HW_REG_XCC_ID
    unsigned long long a = threadIdx.x;
    for (int i = 0; i < spin; ++i) a = a * 6364136223846793005ull + 1442695040888963407ull;
    if (a == 42) sink[0] = a;
}

int main() {
    int per_cu = 0;
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, who, 256, 0);
    for (int mult : {1, 2, 4}) {
        const int grid = per_cu * p.multiProcessorCount * mult / 8 * 8;
        unsigned* d;
        unsigned long long* s;
        hipMalloc(&d, grid * 4);
        hipMalloc(&s, 8);
        who<<<grid, 256>>>(d, s, 20000);
        hipDeviceSynchronize();
        std::vector<unsigned> h(grid);
        hipMemcpy(h.data(), d, grid * 4, hipMemcpyDeviceToHost);
        int bad = 0, hist[16] = {0};
        for (int b = 0; b < grid; ++b) {
            bad += h[b] != h[b % 8];
            hist[h[b] & 15]++;
        }
        printf("grid %d (%d per CU x %d CUs x %d): blocks whose XCD != XCD of block b%%8: %d; per-XCD counts:", grid,
               per_cu, p.multiProcessorCount, mult, bad);
        for (int x = 0; x < 8; ++x) printf(" %d", hist[x]);
        printf("\n");
        hipFree(d);
        hipFree(s);
    }
    return 0;
}
