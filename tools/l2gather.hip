// l2gather.hip — the chip's rate of random L2-hit gathers, the ceiling of the
// partitioned probes' lookup passes (xs_probe_cobspart.hip, xs_probe_bloompart.hip).
//
// Every workgroup reads random dwords (or 16-B rows) from a 2 MiB region of
// its own XCD (HW_REG_XCC_ID), so after the first touch every request is an
// L2 hit, as in the lookups where an XCD works through one 2 MiB bank
// partition at a time.  U loads in flight per lane, c workgroups of 256 per CU.
// Reports requests (lane loads) per second.
//   hipcc -O3 --offload-arch=gfx950 tools/l2gather.hip -o tools/l2gather
//   tools/l2gather
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

constexpr uint32_t kRegionWords = (2u << 20) / 4;  // 2 MiB per XCD

__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(v));
    return v;
}

template <int U, int W>  // W = dwords per request (1 or 4)
__global__ void __launch_bounds__(256) gather(const uint32_t* __restrict__ base, uint32_t iters,
                                              uint32_t* __restrict__ sink) {
    const uint32_t* reg = base + (size_t)xcc_id() * kRegionWords;
    uint32_t x = 2654435761u * (blockIdx.x * 256 + threadIdx.x + 1);
    uint32_t acc = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t v[U * W];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x = x * 1664525u + 1013904223u;
            const uint32_t o = (x >> 8) % (kRegionWords / W) * W;
            if constexpr (W == 4) {
                const uint4 q = *reinterpret_cast<const uint4*>(reg + o);
                v[4 * u] = q.x; v[4 * u + 1] = q.y; v[4 * u + 2] = q.z; v[4 * u + 3] = q.w;
            } else {
                v[u] = reg[o];
            }
        }
#pragma unroll
        for (int u = 0; u < U * W; ++u) acc += v[u];
    }
    if (acc == 0x12345678u) sink[0] = acc;  // keeps the loads
}

// The lookup's mix: per gathered 16-B row also one 4-B streaming entry load and one 16-B
// streaming row store (HBM), both contiguous per wave, as in cobs_lookup.  SL < 64: only
// lanes < SL store, contiguously per wave (the store stream of rows packed to 16 * SL / 64
// bytes, without the packing itself).
template <int U, int SL = 64>
__global__ void __launch_bounds__(256) gather_mix(const uint32_t* __restrict__ base, uint32_t iters,
                                                  const uint32_t* __restrict__ ent, uint4* __restrict__ out,
                                                  uint32_t* __restrict__ sink) {
    const uint32_t* reg = base + (size_t)xcc_id() * kRegionWords;
    const size_t t = blockIdx.x * 256 + threadIdx.x, nt = (size_t)gridDim.x * 256;
    const size_t lane = t & 63, wv = t >> 6, nw = nt >> 6;
    uint32_t acc = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) e[u] = __builtin_nontemporal_load(ent + ((size_t)(it * U + u) * nt + t));
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t h = (e[u] ^ (uint32_t)((it * U + u) * nt + t)) * 2654435761u;  // a random row
            const uint32_t o = ((h ^ (h >> 15)) * 2246822519u >> 8) % (kRegionWords / 4) * 4;
            v[u] = *reinterpret_cast<const uint4*>(reg + o);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 q = {v[u].x + e[u], v[u].y, v[u].z, v[u].w};
            if (SL == 64)
                __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(out + ((size_t)(it * U + u) * nt + t)));
            else if (lane < SL)
                __builtin_nontemporal_store(
                    q, reinterpret_cast<u32x4*>(out + (((size_t)(it * U + u) * nw + wv) * SL + lane)));
            acc += v[u].x;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// Parts of the mix: MODE 1 = gathers + row stores (addresses hashed from the index, no
// entry loads); 2 = entry loads + gathers (no stores); 3 = entry loads one iteration
// ahead of their gathers (software-prefetched), + stores.
template <int U, int MODE>
__global__ void __launch_bounds__(256) gather_part(const uint32_t* __restrict__ base, uint32_t iters,
                                                   const uint32_t* __restrict__ ent, uint4* __restrict__ out,
                                                   uint32_t* __restrict__ sink) {
    const uint32_t* reg = base + (size_t)xcc_id() * kRegionWords;
    const size_t t = blockIdx.x * 256 + threadIdx.x, nt = (size_t)gridDim.x * 256;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    uint32_t acc = 0;
    uint32_t en[U];
    if (MODE == 3) {
#pragma unroll
        for (int u = 0; u < U; ++u) en[u] = __builtin_nontemporal_load(ent + ((size_t)u * nt + t));
    }
    for (uint32_t it = 0; it < iters; ++it) {
        uint32_t e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t i = (size_t)(it * U + u) * nt + t;
            if (MODE == 1) e[u] = (uint32_t)i * 0x9E3779B1u;
            else if (MODE == 2) e[u] = __builtin_nontemporal_load(ent + i);
            else if (MODE == 4) e[u] = __builtin_nontemporal_load(ent + (i & ((256u << 10) - 1)));  // L2 hits
            else if (MODE == 5) e[u] = (xcc_id() & 1) ? (uint32_t)i * 0x9E3779B1u : __builtin_nontemporal_load(ent + i);
            else if (MODE == 6) e[u] = __builtin_nontemporal_load(reinterpret_cast<const uint16_t*>(ent) + i);  // 2-B entries
            else e[u] = en[u];
        }
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t h = (e[u] ^ (uint32_t)((it * U + u) * nt + t)) * 2654435761u;
            const uint32_t o = ((h ^ (h >> 15)) * 2246822519u >> 8) % (kRegionWords / 4) * 4;
            v[u] = *reinterpret_cast<const uint4*>(reg + o);
        }
        // the next iteration's entries are issued after this iteration's gathers, so that
        // waiting for the gathers (vmcnt counts in issue order) does not wait for them
        if (MODE == 3) __builtin_amdgcn_sched_barrier(0);  // gathers stay before the prefetches
        if (MODE == 3) {  // unconditional (the last iteration reloads its own entries), so that the
                          // compiler's vmcnt counts before the stores stay exact
            const uint32_t nx = it + 1 < iters ? it + 1 : it;
#pragma unroll
            for (int u = 0; u < U; ++u) en[u] = __builtin_nontemporal_load(ent + ((size_t)(nx * U + u) * nt + t));
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (MODE != 2 && (MODE != 5 || (xcc_id() & 1))) {  // (the row alone: e[u]'s registers are the next prefetch's in MODE 3)
                const u32x4 q = {v[u].x, v[u].y, v[u].z, v[u].w};
                __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(out + ((size_t)(it * U + u) * nt + t)));
            }
            acc += v[u].x;
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int U, int MODE>
static void run_part(const uint32_t* d, uint32_t* sink, int cus, int per_cu, hipEvent_t e0, hipEvent_t e1) {
    const int grid = cus * per_cu;
    const uint32_t iters = 2048 / U;
    const size_t n = (size_t)grid * 256 * iters * U;
    uint32_t* ent = nullptr;
    uint4* out = nullptr;
    CHK(hipMalloc(&ent, n * 4));
    CHK(hipMalloc(&out, n * 16));
    CHK(hipMemset(ent, 7, n * 4));
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CHK(hipEventRecord(e0));
        gather_part<U, MODE><<<grid, 256>>>(d, iters, ent, out, sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const char* what[] = {"", "gathers + 16-B row stores (no entry loads)", "4-B entry loads + gathers (no stores)",
                          "4-B entry loads one iteration ahead + gathers + 16-B row stores",
                          "4-B entry loads that hit L2 (a 1 MiB array) + gathers + 16-B row stores",
                          "XCDs split: even XCDs entry loads + gathers, odd XCDs gathers + row stores",
                          "2-B entry loads + gathers + 16-B row stores"};
    printf("%s, %d in flight, %d workgroups/CU: %.3f ms, %.1f G gathers/s\n", what[MODE], U, per_cu, best,
           n / (best * 1e-3) / 1e9);
    CHK(hipFree(ent));
    CHK(hipFree(out));
}

template <int U, int SL = 64>
static void run_mix(const uint32_t* d, uint32_t* sink, int cus, int per_cu, hipEvent_t e0, hipEvent_t e1) {
    const int grid = cus * per_cu;
    const uint32_t iters = 2048 / U;
    const size_t n = (size_t)grid * 256 * iters * U;
    uint32_t* ent = nullptr;
    uint4* out = nullptr;
    CHK(hipMalloc(&ent, n * 4));
    CHK(hipMalloc(&out, n * 16));
    CHK(hipMemset(ent, 7, n * 4));
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CHK(hipEventRecord(e0));
        gather_mix<U, SL><<<grid, 256>>>(d, iters, ent, out, sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    printf("16-B gathers + 4-B entry load + %.0f-B row store each, %d in flight, %d workgroups/CU: %.3f ms, "
           "%.1f G gathers/s, %.0f GB/s HBM streams\n", 16.0 * SL / 64, U, per_cu, best, n / (best * 1e-3) / 1e9,
           n * (4.0 + 16.0 * SL / 64) / (best * 1e-3) / 1e9);
    CHK(hipFree(ent));
    CHK(hipFree(out));
}

template <int U, int W>
static void run(const uint32_t* d, uint32_t* sink, int cus, int per_cu, hipEvent_t e0, hipEvent_t e1) {
    const uint32_t iters = 4096 / U;
    const int grid = cus * per_cu;
    gather<U, W><<<grid, 256>>>(d, 8, sink);  // warm: regions into L2
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        CHK(hipEventRecord(e0));
        gather<U, W><<<grid, 256>>>(d, iters, sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
    }
    const double req = (double)grid * 256 * iters * U;
    printf("%2d-B gathers, %2d in flight per lane, %d workgroups/CU: %.3f ms, %.1f G requests/s\n", 4 * W, U,
           per_cu, best, req / (best * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
    const bool packed = argc > 1 && argv[1][0] == 'p';  // store-stream width sweep only
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    uint32_t* d = nullptr;
    uint32_t* sink = nullptr;
    CHK(hipMalloc(&d, 8ull * kRegionWords * 4));
    CHK(hipMemset(d, 1, 8ull * kRegionWords * 4));
    CHK(hipMalloc(&sink, 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    if (argc > 1 && argv[1][0] == 'm') {  // which part of the mix costs the rate
        for (int r = 0; r < 2; ++r) {
            run_mix<8, 64>(d, sink, cus, 2, e0, e1);
            run_part<8, 1>(d, sink, cus, 2, e0, e1);
            run_part<8, 2>(d, sink, cus, 2, e0, e1);
            run_part<8, 3>(d, sink, cus, 2, e0, e1);
            run_part<8, 4>(d, sink, cus, 2, e0, e1);
            run_part<8, 5>(d, sink, cus, 2, e0, e1);
            run_part<8, 6>(d, sink, cus, 2, e0, e1);
            run<8, 4>(d, sink, cus, 2, e0, e1);
        }
        return 0;
    }
    if (packed) {  // rows packed to 14 / 12 B (D + 11 id bits in 112 / 96 bits), interleaved
        for (int r = 0; r < 3; ++r) {
            run_mix<8, 64>(d, sink, cus, 2, e0, e1);
            run_mix<8, 56>(d, sink, cus, 2, e0, e1);
            run_mix<8, 48>(d, sink, cus, 2, e0, e1);
        }
        return 0;
    }
    for (int c : {2, 4}) {
        run_mix<4>(d, sink, cus, c, e0, e1);
        run_mix<8>(d, sink, cus, c, e0, e1);
    }
    for (int c : {2, 4, 8}) {
        run<4, 1>(d, sink, cus, c, e0, e1);
        run<16, 1>(d, sink, cus, c, e0, e1);
        run<4, 4>(d, sink, cus, c, e0, e1);
        run<8, 4>(d, sink, cus, c, e0, e1);
    }
    return 0;
}
