// xs_part.h — pieces shared by the partitioned probes (xs_probe_bloompart.hip,
// xs_probe_cobspart.hip): per-read k-mer counts and their scan give every
// sampled k-mer a global id; bucket blocks of kPartKmers consecutive ids are
// mapped to the reads they start in; partition starts are transposed from
// block-major to partition-major for the per-XCD lookup queues.
#pragma once
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "xs_device.h"

namespace xs {

namespace {

constexpr int kTK = kPartKmers;  // k-mers per bucket block
constexpr int kBucketThreads = 512;
constexpr uint32_t kStageReads = 256;  // read offsets a bucket block keeps in LDS

__global__ void part_counts_kernel(const uint64_t* __restrict__ offs, uint64_t n, uint32_t k, uint32_t step,
                                   uint64_t* __restrict__ nkc) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r <= n;
         r += (uint64_t)gridDim.x * blockDim.x)
        nkc[r] = r < n ? num_kmers(offs[r + 1] - offs[r], k, step) : 0;
}

// Largest r in [lo, hi] with kofs[r] <= g (kofs non-decreasing, kofs[lo] <= g).
__device__ __forceinline__ uint64_t read_of(const uint64_t* __restrict__ kofs, uint64_t lo, uint64_t hi,
                                            uint64_t g) {
    while (lo < hi) {
        const uint64_t mid = (lo + hi + 1) >> 1;
        if (kofs[mid] <= g) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// blk_read[b] = the read holding k-mer b*TK (the first k-mer of bucket block b).
template <int TK = kTK>
__global__ void part_map_kernel(const uint64_t* __restrict__ kofs, uint64_t n, uint32_t* __restrict__ blk_read) {
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t fb = (kofs[r] + TK - 1) / TK, lb = (kofs[r + 1] + TK - 1) / TK;
        for (uint64_t b = fb; b < lb; ++b) blk_read[b] = (uint32_t)r;
    }
}

// Block-major partition starts (one coalesced row per bucket block) ->
// partition-major (the lookup reads 64 blocks' starts of one partition as one
// line), through a 64 x 64 LDS tile.
// Blocks b_begin .. b_end-1 (grid.x covers them in tiles of 64).
__global__ void __launch_bounds__(256) part_transpose_kernel(const uint16_t* __restrict__ tbm, uint32_t P1,
                                                             uint64_t tstride, uint16_t* __restrict__ tbl,
                                                             uint64_t b_begin, uint64_t b_end) {
    __shared__ uint16_t t[64][65];
    const uint64_t b0 = b_begin + (uint64_t)blockIdx.x * 64;
    const uint32_t p0 = blockIdx.y * 64;
    for (uint32_t x = threadIdx.x; x < 64 * 64; x += 256) {
        const uint32_t bi = x / 64, pi = x % 64;
        if (b0 + bi < b_end && p0 + pi < P1) t[bi][pi] = tbm[(b0 + bi) * P1 + p0 + pi];
    }
    __syncthreads();
    for (uint32_t x = threadIdx.x; x < 64 * 64; x += 256) {
        const uint32_t pi = x / 64, bi = x % 64;
        if (b0 + bi < b_end && p0 + pi < P1) tbl[(p0 + pi) * tstride + b0 + bi] = t[bi][pi];
    }
}

// u32 per lookup queue counter: each counter sits on its own 128-B line (a
// line's atomics are serialised at the memory side).
constexpr uint32_t kQStride = 32;  // u32 per queue counter

}  // namespace

}  // namespace xs
