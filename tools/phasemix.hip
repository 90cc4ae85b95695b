// phasemix.hip — does separating the HBM read stream from the HBM write stream in
// time raise the partitioned COBS lookup's rate (xs_probe_cobspart.hip)?
//
// tools/l2gather.hip m showed that L2-hit 16-B gathers run at ~227 G/s beside
// either a 4-B entry read stream or a 16-B row write stream alone, but at ~145 G/s
// beside both, also when the two streams come from different XCDs (~159 G/s):
// the reads and writes interfere chip-wide.  Here one persistent workgroup per
// slot alternates, in lock step with every other workgroup of the grid (a
// grid barrier between phases), a read phase (kEnt entries into LDS) and a
// write phase (one L2-hit gather + one 16-B streaming store per entry), so the
// chip sees reads only, then writes only.  Compared against the mixed form on
// the same number of entries.  The barrier spin is bounded (a flag reports a
// timeout instead of hanging when not all workgroups are resident).
//   hipcc -O3 --offload-arch=gfx950 tools/phasemix.hip -o tools/phasemix
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                      \
    do {                                                            \
        hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) {                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
            exit(1);                                                \
        }                                                           \
    } while (0)

constexpr uint32_t kRegionWords = (2u << 20) / 4;  // 2 MiB per XCD (L2-resident)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v;
}

__device__ __forceinline__ uint32_t row_of(uint32_t e, size_t i) {
    const uint32_t h = (e ^ (uint32_t)i) * 2654435761u;
    return ((h ^ (h >> 15)) * 2246822519u >> 8) % (kRegionWords / 4) * 4;
}

// Grid barrier: one lane per workgroup adds (agent scope, vector atomic), then polls.
__device__ __forceinline__ void grid_sync(uint32_t* bar, uint32_t target, uint32_t* err) {
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t n = 0;
        while (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (++n > (1u << 22)) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}

template <int KENT, int U, bool PHASED>
__global__ void __launch_bounds__(256) lookup_mix(const uint32_t* __restrict__ base, const uint32_t* __restrict__ ent,
                                                  uint4* __restrict__ out, uint32_t cycles, uint32_t* bar,
                                                  uint32_t* err) {
    __shared__ uint32_t s_e[PHASED ? KENT : 1];
    const uint32_t* reg = base + (size_t)xcc_id() * kRegionWords;
    const uint32_t nwg = gridDim.x, tid = threadIdx.x;
    for (uint32_t c = 0; c < cycles; ++c) {
        const size_t chunk = ((size_t)c * nwg + blockIdx.x) * KENT;
        if constexpr (PHASED) {
            for (uint32_t i = tid * 4; i < KENT; i += 1024) {
                const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ent + chunk + i));
                *reinterpret_cast<u32x4*>(&s_e[i]) = q;
            }
            grid_sync(bar, (2 * c + 1) * nwg, err);
        }
        for (uint32_t j0 = 0; j0 < KENT; j0 += 256 * U) {
            uint32_t e[U];
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t j = j0 + u * 256 + tid;
                e[u] = PHASED ? s_e[j] : __builtin_nontemporal_load(ent + chunk + j);
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                v[u] = *reinterpret_cast<const uint4*>(reg + row_of(e[u], chunk + j0 + u * 256 + tid));
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u32x4 q = {v[u].x, v[u].y, v[u].z, v[u].w};
                __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(out + chunk + j0 + u * 256 + tid));
            }
        }
        if constexpr (PHASED) grid_sync(bar, (2 * c + 2) * nwg, err);
    }
}

template <int KENT, int U, bool PHASED>
static void run(const uint32_t* base, const uint32_t* ent, uint4* out, uint32_t* bar, uint32_t* err, int cus,
                size_t total, hipEvent_t e0, hipEvent_t e1) {
    int per_cu = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lookup_mix<KENT, U, PHASED>, 256, 0));
    per_cu = per_cu > 2 ? 2 : per_cu;
    if (per_cu < 1) return;
    const int grid = cus * per_cu;
    const uint32_t cycles = (uint32_t)(total / ((size_t)grid * KENT));
    float best = 1e30f;
    uint32_t herr = 0;
    for (int r = 0; r < 3; ++r) {
        CHK(hipMemset(bar, 0, 4));
        CHK(hipMemset(err, 0, 4));
        CHK(hipEventRecord(e0));
        lookup_mix<KENT, U, PHASED><<<grid, 256>>>(base, ent, out, cycles, bar, err);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        uint32_t x = 0;
        CHK(hipMemcpy(&x, err, 4, hipMemcpyDeviceToHost));
        herr |= x;
    }
    const double n = (double)cycles * grid * KENT;
    printf("%s, %d entries per workgroup and phase, %d in flight, %d workgroups/CU, %u cycles: %.3f ms, "
           "%.1f G entries/s%s\n", PHASED ? "phased (reads, barrier, gathers + stores, barrier)" : "mixed",
           KENT, U, per_cu, cycles, best, n / (best * 1e-3) / 1e9, herr ? "  BARRIER TIMEOUT" : "");
}

int main() {
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t *base = nullptr, *ent = nullptr, *bar = nullptr, *err = nullptr;
    uint4* out = nullptr;
    const size_t total = (size_t)cus * 2 * 16384 * 32;  // entries per run (~268 M on 256 CUs)
    CHK(hipMalloc(&base, 8ull * kRegionWords * 4));
    CHK(hipMemset(base, 1, 8ull * kRegionWords * 4));
    CHK(hipMalloc(&ent, total * 4 + 4096));
    CHK(hipMemset(ent, 7, total * 4 + 4096));
    CHK(hipMalloc(&out, total * 16 + 4096));
    CHK(hipMalloc(&bar, 128));
    CHK(hipMalloc(&err, 128));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int r = 0; r < 2; ++r) {
        run<16384, 8, false>(base, ent, out, bar, err, cus, total, e0, e1);
        run<16384, 8, true>(base, ent, out, bar, err, cus, total, e0, e1);
        run<8192, 8, true>(base, ent, out, bar, err, cus, total, e0, e1);
        run<4096, 8, true>(base, ent, out, bar, err, cus, total, e0, e1);
    }
    return 0;
}
