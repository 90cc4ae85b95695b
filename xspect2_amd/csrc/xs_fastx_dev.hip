// xs_fastx_dev.hip — gfx950 record finding for the reader's device mode
// (xs_fastx_open_device / xs_fastx_next_device).
//
// The host only copies a window of file text (cut at a record start, as the
// host reader cuts it) into pinned memory and on to HBM; the records are found
// here, in passes over the text at HBM rate:
//   count     : '\n' per 16 KiB tile (SWAR byte compare, coalesced 16-B loads)
//   scan      : tile starts in the line index (hipCUB)
//   positions : every '\n' position, in text order (block scan per 4 KiB row)
//   records   : FASTQ, one thread per 4-line record: Biopython's checks
//               (FastqGeneralIterator, restated in xs_fastx.cpp), spans of the
//               sequence, id and title; FASTA, one thread per line: header or
//               sequence line, the line's kept length
//   scan      : output offsets of sequences, ids and titles
//   copy      : one wave per run (line, sequence, id), lanes copy bytes
// A window whose text the fast rules do not cover (wrapped FASTQ lines, blank
// lines between FASTQ records, an empty FASTQ sequence, ' ' or '\r' inside a
// FASTA sequence line, any FASTQ format error) is flagged and the host parses
// that window instead, so the result — or Biopython's error message — is the
// host reader's in every case.
#include <hipcub/hipcub.hpp>

#include "xs_device.h"

namespace xs {
namespace {

constexpr int kFxThreads = 256;
constexpr int kFqBlock = 256;  // FASTQ records per block of the record kernels
constexpr int kFxRow = kFxThreads * 16;  // bytes per coalesced row of a tile
static_assert(kFxTile == 4 * kFxRow, "a tile is four rows of 16 B per thread");

// Bit 7 of each byte of w set where that byte is '\n' (no carries cross bytes).
__device__ __forceinline__ uint32_t nl_bits(uint32_t w) {
    const uint32_t x = w ^ 0x0a0a0a0au;
    return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}

// Python's str.isspace() over ASCII (the host reader's is_ws).
__device__ __forceinline__ bool fx_ws(uint8_t c) {
    return c == ' ' || (c >= '\t' && c <= '\r') || (c >= 0x1c && c <= 0x1f);
}

__device__ __forceinline__ uint32_t fx_rstrip(const uint8_t* t, uint32_t b, uint32_t e) {
    while (e > b && fx_ws(t[e - 1])) --e;
    return e;
}

__device__ __forceinline__ uint32_t line_start(const uint32_t* nl, uint64_t j) { return j ? nl[j - 1] + 1 : 0; }

// Bit 7 of each byte of w set where that byte equals c (exact: no carries cross bytes).
__device__ __forceinline__ uint32_t eq_bits(uint32_t w, uint32_t c) {
    const uint32_t x = w ^ (c * 0x01010101u);
    return ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x) & 0x80808080u;
}

// First whitespace-separated token of [b, e): its start and length.
__device__ __forceinline__ void first_token(const uint8_t* t, uint32_t b, uint32_t e, uint32_t* s, uint64_t* len) {
    while (b < e && fx_ws(t[b])) ++b;
    uint32_t x = b;
    while (x < e && !fx_ws(t[x])) ++x;
    *s = b;
    *len = x - b;
}

__global__ void __launch_bounds__(kFxThreads) fx_count_kernel(const uint8_t* __restrict__ text,
                                                              uint64_t* __restrict__ tile_cnt) {
    using Reduce = hipcub::BlockReduce<uint32_t, kFxThreads>;
    __shared__ typename Reduce::TempStorage tmp;
    const uint8_t* p = text + (uint64_t)blockIdx.x * kFxTile + threadIdx.x * 16;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint4 v = *reinterpret_cast<const uint4*>(p + i * kFxRow);
        c += __popc(nl_bits(v.x)) + __popc(nl_bits(v.y)) + __popc(nl_bits(v.z)) + __popc(nl_bits(v.w));
    }
    const uint32_t total = Reduce(tmp).Sum(c);
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kFxThreads) fx_positions_kernel(const uint8_t* __restrict__ text,
                                                                  const uint64_t* __restrict__ tile_ofs,
                                                                  uint32_t* __restrict__ nl) {
    using Scan = hipcub::BlockScan<uint32_t, kFxThreads>;
    __shared__ typename Scan::TempStorage tmp;
    uint64_t base = tile_ofs[blockIdx.x];
    const uint32_t tile0 = blockIdx.x * (uint32_t)kFxTile;
    for (int i = 0; i < 4; ++i) {
        const uint32_t off = tile0 + i * kFxRow + threadIdx.x * 16;
        const uint4 v = *reinterpret_cast<const uint4*>(text + off);
        const uint32_t m[4] = {nl_bits(v.x), nl_bits(v.y), nl_bits(v.z), nl_bits(v.w)};
        const uint32_t c = __popc(m[0]) + __popc(m[1]) + __popc(m[2]) + __popc(m[3]);
        uint32_t pre, total;
        Scan(tmp).ExclusiveSum(c, pre, total);
        uint64_t o = base + pre;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            uint32_t mm = m[w];
            while (mm) {
                const uint32_t bit = __ffs(mm) - 1;  // 7, 15, 23 or 31
                nl[o++] = off + 4 * w + (bit >> 3);
                mm &= mm - 1;
            }
        }
        base += total;
        __syncthreads();  // tmp is reused by the next row's scan
    }
}

// FASTQ: record r = lines 4r .. 4r+3.  The checks are the host reader's
// (parse_fastq, xs_fastx.cpp), narrowed to the layouts where four lines are
// exactly one record; anything else sets *bad and the host parses the window.
__global__ void __launch_bounds__(kFqBlock) fq_records_kernel(const uint8_t* __restrict__ t,
                                                              const uint32_t* __restrict__ nl, uint64_t n,
                                                              FxRuns runs, uint32_t* __restrict__ bad,
                                                              FqBlockSums* __restrict__ blk) {
    const uint64_t r = blockIdx.x * (uint64_t)kFqBlock + threadIdx.x;
    uint64_t sl = 0, il = 0, dl = 0;
    // Pass 1, a record per lane: the line layout, the title, the caption and
    // the quality length.  The sequence line's ' '/'\t' check is pass 2.
    bool ok = false;
    uint32_t s1 = 0, se = 0, tb = 0, te = 0;
    if (r < n) {
        const uint32_t s0 = line_start(nl, 4 * r), e0 = nl[4 * r];
        s1 = e0 + 1;
        const uint32_t e1 = nl[4 * r + 1];
        const uint32_t s2 = e1 + 1, e2 = nl[4 * r + 2];
        const uint32_t s3 = e2 + 1, e3 = nl[4 * r + 3];
        ok = e0 > s0 && t[s0] == '@';
        tb = s0 + 1;
        te = ok ? fx_rstrip(t, tb, e0) : tb;
        // one sequence line, not empty, not itself a '+' line
        se = fx_rstrip(t, s1, e1);
        ok = ok && se > s1 && t[s1] != '+';
        ok = ok && e2 > s2 && t[s2] == '+';
        if (ok) {  // a caption, if any, repeats the title
            const uint32_t cb = s2 + 1, ce = fx_rstrip(t, cb, e2);
            if (ce > cb) {
                ok = ce - cb == te - tb;
                for (uint32_t i = 0; ok && i < ce - cb; ++i) ok = t[cb + i] == t[tb + i];
            }
        }
        ok = ok && fx_rstrip(t, s3, e3) - s3 == se - s1;  // one quality line of the same length
    }
    // Pass 2: no ' ' or '\t' in the sequence lines, read coalesced: a group of
    // 16 lanes scans one record's line in 16-B loads (256 B per step), four
    // records per wave step.  A lane scanning its own line alone put 64
    // scattered lines in flight per load (~0.8 ms per 256 MiB window, now ~4x less).
    {
        const int lane = threadIdx.x & 63, g = lane >> 4, gl = lane & 15;
        const uint4* t16 = reinterpret_cast<const uint4*>(t);
        bool clean = true;
        for (int j = 0; j < 64; j += 4) {
            const int owner = j + g;
            const uint32_t b = __shfl(s1, owner), e = __shfl(se, owner);
            const bool need = __shfl((int)ok, owner) != 0;
            bool dirty = false;
            if (need) {
                for (uint32_t p = (b & ~15u) + 16u * gl; p < e; p += 256u) {
                    const uint4 v = t16[p >> 4];
                    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint32_t at = p + 4u * q;
                        uint32_t keep = 0xffffffffu;
                        if (at + 4 <= b || at >= e) keep = 0;
                        else {
                            if (at < b) keep <<= 8 * (b - at);
                            if (e - at < 4) keep &= (1u << (8 * (e - at))) - 1u;
                        }
                        dirty |= ((eq_bits(w[q], ' ') | eq_bits(w[q], '\t')) & keep) != 0;
                    }
                }
            }
            const uint64_t m = __ballot(dirty);
            if (lane >= j && lane < j + 4) clean = ((m >> (16 * (lane - j))) & 0xffffull) == 0;
        }
        ok = ok && clean;
    }
    if (r < n) {
        if (!ok) {
            *bad = 1;
            runs.seq_src[r] = runs.id_src[r] = runs.desc_src[r] = 0;
        } else {
            runs.seq_src[r] = s1;
            sl = se - s1;
            runs.desc_src[r] = tb;
            dl = te - tb;
            first_token(t, tb, te, &runs.id_src[r], &il);
        }
        runs.seq_len[r] = sl;
        runs.id_len[r] = il;
        runs.desc_len[r] = dl;
    }
    // the block's sums and longest sequence, for fq_block_scan_kernel
    using Reduce = hipcub::BlockReduce<uint64_t, kFqBlock>;
    __shared__ typename Reduce::TempStorage tmp;
    const uint64_t a = Reduce(tmp).Sum(sl);
    __syncthreads();
    const uint64_t b = Reduce(tmp).Sum(il);
    __syncthreads();
    const uint64_t c = Reduce(tmp).Sum(dl);
    __syncthreads();
    const uint64_t m = Reduce(tmp).Reduce(sl, hipcub::Max());
    if (threadIdx.x == 0) blk[blockIdx.x] = FqBlockSums{a, b, c, m};
}

// One block: exclusive offsets of every record block's sequence, id and
// title bytes, and the window's totals into status ([0] bad, [1] records,
// [2] sequence bytes, [3] id bytes, [4] title bytes, [5] longest sequence).
__global__ void __launch_bounds__(1024) fq_block_scan_kernel(const FqBlockSums* __restrict__ blk, uint64_t nblk,
                                                             uint64_t n, const uint32_t* __restrict__ bad,
                                                             uint64_t* __restrict__ blk_ofs,
                                                             uint64_t* __restrict__ status) {
    using Scan = hipcub::BlockScan<uint64_t, 1024>;
    using Reduce = hipcub::BlockReduce<uint64_t, 1024>;
    __shared__ union {
        typename Scan::TempStorage scan;
        typename Reduce::TempStorage red;
    } tmp;
    const uint64_t per = (nblk + 1023) / 1024;
    const uint64_t b0 = threadIdx.x * per, b1 = b0 + per < nblk ? b0 + per : nblk;
    uint64_t tot[3] = {0, 0, 0}, mx = 0;
    for (uint64_t b = b0; b < b1; ++b) {
        tot[0] += blk[b].seq;
        tot[1] += blk[b].id;
        tot[2] += blk[b].desc;
        mx = blk[b].mx > mx ? blk[b].mx : mx;
    }
    for (int k = 0; k < 3; ++k) {
        uint64_t pre, all;
        Scan(tmp.scan).ExclusiveSum(tot[k], pre, all);
        __syncthreads();
        for (uint64_t b = b0; b < b1; ++b) {
            blk_ofs[3 * b + k] = pre;
            pre += k == 0 ? blk[b].seq : k == 1 ? blk[b].id : blk[b].desc;
        }
        if (threadIdx.x == 0) status[2 + k] = all;
    }
    const uint64_t m = Reduce(tmp.red).Reduce(mx, hipcub::Max());
    if (threadIdx.x == 0) {
        status[0] = *bad;
        status[1] = n;
        status[5] = m;
    }
}

// Record offsets of sequences, ids and titles (n+1 entries each): the block's
// exclusive scan of its records' lengths plus the block's offset.
__global__ void __launch_bounds__(kFqBlock) fq_offsets_kernel(FxRuns runs, uint64_t n,
                                                              const uint64_t* __restrict__ blk_ofs,
                                                              uint64_t* __restrict__ offs,
                                                              uint64_t* __restrict__ id_ofs,
                                                              uint64_t* __restrict__ desc_ofs) {
    using Scan = hipcub::BlockScan<uint64_t, kFqBlock>;
    __shared__ typename Scan::TempStorage tmp;
    const uint64_t r = blockIdx.x * (uint64_t)kFqBlock + threadIdx.x;
    const uint64_t* len[3] = {runs.seq_len, runs.id_len, runs.desc_len};
    uint64_t* out[3] = {offs, id_ofs, desc_ofs};
    for (int k = 0; k < 3; ++k) {
        const uint64_t v = r < n ? len[k][r] : 0;
        uint64_t pre;
        Scan(tmp).ExclusiveSum(v, pre);
        __syncthreads();
        pre += blk_ofs[3 * blockIdx.x + k];
        if (r < n) out[k][r] = pre;
        if (r + 1 == n) out[k][n] = pre + v;
    }
}

// FASTA pass 1: hdr[j] = line j is a header ('>' first).
__global__ void __launch_bounds__(256) fa_headers_kernel(const uint8_t* __restrict__ t,
                                                         const uint32_t* __restrict__ nl, uint64_t L,
                                                         uint64_t* __restrict__ hdr) {
    for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < L;
         j += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = line_start(nl, j), e = nl[j];
        hdr[j] = e > s && t[s] == '>';
    }
}

// FASTA pass 2, with hofs = exclusive scan of hdr: a header line opens record
// hofs[j] (its title and id); a sequence line after the first header keeps
// its right-stripped bytes; lines before the first header are skipped.
__global__ void __launch_bounds__(256) fa_lines_kernel(const uint8_t* __restrict__ t,
                                                       const uint32_t* __restrict__ nl, uint64_t L,
                                                       const uint64_t* __restrict__ hofs,
                                                       uint32_t* __restrict__ line_src,
                                                       uint64_t* __restrict__ line_len,
                                                       uint32_t* __restrict__ rec_line, FxRuns runs,
                                                       uint32_t* __restrict__ bad) {
    // a wave takes 64 lines at a time: a line per lane, then the whole wave
    // checks each kept sequence line for ' ' / '\r' in 16-B loads (1 KiB per
    // step), so an unwrapped multi-megabase line is not one lane's byte loop
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint4* t16 = reinterpret_cast<const uint4*>(t);
    for (uint64_t c = wave * 64; c < L; c += waves * 64) {
        const uint64_t j = c + lane;
        uint32_t s = 0, se = 0;
        if (j < L) {
            s = line_start(nl, j);
            const uint32_t e = nl[j];
            line_src[j] = s;
            if (e > s && t[s] == '>') {
                const uint64_t r = hofs[j];
                rec_line[r] = (uint32_t)j;
                const uint32_t tb = s + 1, te = fx_rstrip(t, tb, e);
                runs.desc_src[r] = tb;
                runs.desc_len[r] = te - tb;
                first_token(t, tb, te, &runs.id_src[r], &runs.id_len[r]);
                line_len[j] = 0;
            } else if (hofs[j] == 0) {
                line_len[j] = 0;
            } else {
                se = fx_rstrip(t, s, e);
                line_len[j] = se - s;
            }
        }
        bool dirty = false;
        for (int k = 0; k < 64; ++k) {  // sequence lines only (se > s)
            const uint32_t b = __shfl(s, k), e = __shfl(se, k);
            for (uint32_t p = (b & ~15u) + 16u * lane; p < e; p += 1024u) {
                const uint4 v = t16[p >> 4];
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t at = p + 4u * q;
                    uint32_t keep = 0xffffffffu;
                    if (at + 4 <= b || at >= e) keep = 0;
                    else {
                        if (at < b) keep <<= 8 * (b - at);
                        if (e - at < 4) keep &= (1u << (8 * (e - at))) - 1u;
                    }
                    dirty |= ((eq_bits(w[q], ' ') | eq_bits(w[q], '\r')) & keep) != 0;
                }
            }
        }
        if (dirty) *bad = 1;  // the host removes them inside the line
    }
}

// FASTA pass 3: record r's sequence starts where its header line's output
// does (a header keeps no bytes); lens[r] = its length.
// The record count n = hofs[L] is read on the device (the grid covers L).
__global__ void __launch_bounds__(256) fa_offsets_kernel(const uint32_t* __restrict__ rec_line,
                                                         const uint64_t* __restrict__ line_ofs, uint64_t L,
                                                         const uint64_t* __restrict__ n_dev,
                                                         uint64_t* __restrict__ offs,
                                                         uint64_t* __restrict__ lens) {
    const uint64_t n = *n_dev;
    for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t a = line_ofs[rec_line[r]];
        const uint64_t b = r + 1 < n ? line_ofs[rec_line[r + 1]] : line_ofs[L];
        offs[r] = a;
        lens[r] = b - a;
        if (r == n - 1) offs[n] = line_ofs[L];
    }
}

// Run i = src[i] .. + (dofs[i+1] - dofs[i]) bytes of t, to dst + dofs[i].
// A wave takes 64 runs at a time and loads their bounds in one coalesced
// load; G lanes copy one run (64 for sequences, 4-16 for ids and titles: the
// host picks G from the mean run length), 64/G runs per step, the bounds
// broadcast by shuffle, so consecutive runs' loads overlap instead of each
// run waiting on its own bounds.  Each lane writes whole aligned output dwords
// assembled from two aligned text dwords (alignbyte), and the bytes of a
// run's first and last dword that it shares with its neighbours one by one.
// dst is 4-B aligned; t is dword-readable 8 B past any run.
template <int G, bool kLong>
__global__ void __launch_bounds__(256) fx_copy_kernel(const uint8_t* __restrict__ t,
                                                      const uint32_t* __restrict__ src,
                                                      const uint64_t* __restrict__ dofs, uint64_t m,
                                                      uint8_t* __restrict__ dst) {
    constexpr int kPer = 64 / G;  // runs per step
    const int lane = threadIdx.x & 63, gl = lane % G, sub = lane / G;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(t);
    uint32_t* d32 = reinterpret_cast<uint32_t*>(dst);
    for (uint64_t c = wave * 64; c < m; c += waves * 64) {
        const uint64_t i = c + lane;
        const uint64_t my_o = i < m ? dofs[i] : 0, my_e = i < m ? dofs[i + 1] : 0;
        const uint64_t my_s = i < m ? src[i] : 0;
#pragma unroll 2
        for (int k = 0; k < G; ++k) {
            const int run = k * kPer + sub;  // lane of the run's bounds
            const uint64_t o = __shfl(my_o, run), end = __shfl(my_e, run), s = __shfl(my_s, run);
            if (end <= o) continue;  // empty run, or past m
            const uint64_t w0 = o >> 2, wl = (end - 1) >> 2;  // the run's output dwords
            if (!kLong) {
                for (uint64_t w = w0 + gl; w <= wl; w += G) {
                    const uint64_t q0 = w << 2;
                    if (q0 >= o && q0 + 4 <= end) {
                        const uint64_t x = s + (q0 - o);
                        d32[w] = __builtin_amdgcn_alignbyte(t32[(x >> 2) + 1], t32[x >> 2], (uint32_t)(x & 3));
                    } else {
                        for (uint64_t q = q0 > o ? q0 : o; q < q0 + 4 && q < end; ++q) dst[q] = t[s + (q - o)];
                    }
                }
                continue;
            }
            // long runs (unwrapped contig lines): four dwords per lane per pass,
            // all loaded before any is stored, 8 loads in flight (a separate
            // instantiation: its registers would slow the short-run copies)
            for (uint64_t w = w0 + gl; w <= wl; w += 4 * G) {
                uint32_t v[4];
                bool full[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint64_t ww = w + (uint64_t)u * G, q0 = ww << 2;
                    full[u] = ww <= wl && q0 >= o && q0 + 4 <= end;
                    if (full[u]) {
                        const uint64_t x = s + (q0 - o);
                        v[u] = __builtin_amdgcn_alignbyte(t32[(x >> 2) + 1], t32[x >> 2], (uint32_t)(x & 3));
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint64_t ww = w + (uint64_t)u * G, q0 = ww << 2;
                    if (full[u]) d32[ww] = v[u];
                    else if (ww <= wl)
                        for (uint64_t q = q0 > o ? q0 : o; q < q0 + 4 && q < end; ++q) dst[q] = t[s + (q - o)];
                }
            }
        }
    }
}

}  // namespace

size_t fx_temp_bytes(uint64_t n) {
    size_t a = 0, b = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)n);
    (void)hipcub::DeviceReduce::Max(nullptr, b, (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)n);
    return a > b ? a : b;
}

hipError_t launch_fx_count(const uint8_t* text, uint64_t tiles, uint64_t* tile_cnt, hipStream_t s) {
    if (!tiles) return hipSuccess;
    fx_count_kernel<<<(unsigned)tiles, kFxThreads, 0, s>>>(text, tile_cnt);
    return hipGetLastError();
}

hipError_t launch_fx_positions(const uint8_t* text, uint64_t tiles, const uint64_t* tile_ofs, uint32_t* nl,
                               hipStream_t s) {
    if (!tiles) return hipSuccess;
    fx_positions_kernel<<<(unsigned)tiles, kFxThreads, 0, s>>>(text, tile_ofs, nl);
    return hipGetLastError();
}

hipError_t launch_fq_records(const uint8_t* text, const uint32_t* nl, uint64_t n, const FxRuns& runs,
                             uint32_t* bad, FqBlockSums* blk, uint64_t* blk_ofs, uint64_t* offs, uint64_t* id_ofs,
                             uint64_t* desc_ofs, uint64_t* status, hipStream_t s) {
    const uint64_t nblk = (n + kFqBlock - 1) / kFqBlock;
    if (nblk) fq_records_kernel<<<(unsigned)nblk, kFqBlock, 0, s>>>(text, nl, n, runs, bad, blk);
    fq_block_scan_kernel<<<1, 1024, 0, s>>>(blk, nblk, n, bad, blk_ofs, status);
    if (nblk) fq_offsets_kernel<<<(unsigned)nblk, kFqBlock, 0, s>>>(runs, n, blk_ofs, offs, id_ofs, desc_ofs);
    return hipGetLastError();
}

hipError_t launch_fa_headers(const uint8_t* text, const uint32_t* nl, uint64_t L, uint64_t* hdr, hipStream_t s) {
    if (!L) return hipSuccess;
    fa_headers_kernel<<<grid_for(L, 256, 8192), 256, 0, s>>>(text, nl, L, hdr);
    return hipGetLastError();
}

hipError_t launch_fa_lines(const uint8_t* text, const uint32_t* nl, uint64_t L, const uint64_t* hofs,
                           uint32_t* line_src, uint64_t* line_len, uint32_t* rec_line, const FxRuns& runs,
                           uint32_t* bad, hipStream_t s) {
    if (!L) return hipSuccess;
    fa_lines_kernel<<<grid_for(L, 256, 8192), 256, 0, s>>>(text, nl, L, hofs, line_src, line_len, rec_line, runs,
                                                          bad);  // 64 lines per wave at a time
    return hipGetLastError();
}

hipError_t launch_fa_offsets(const uint32_t* rec_line, const uint64_t* line_ofs, uint64_t L, const uint64_t* n_dev,
                             uint64_t* offs, uint64_t* lens, hipStream_t s) {
    if (!L) return hipSuccess;
    fa_offsets_kernel<<<grid_for(L, 256, 8192), 256, 0, s>>>(rec_line, line_ofs, L, n_dev, offs, lens);
    return hipGetLastError();
}

hipError_t launch_fx_copy(const uint8_t* text, const uint32_t* src, const uint64_t* dofs, uint64_t m, uint64_t bytes,
                          uint8_t* dst, hipStream_t s) {
    if (!m || !bytes) return hipSuccess;
    const uint64_t mean = bytes / m;  // lanes per run: about one output dword each
    const int grid = grid_for(m, 256, 8192);  // 64 runs per wave at a time
    if (mean > 4096) fx_copy_kernel<64, true><<<grid, 256, 0, s>>>(text, src, dofs, m, dst);
    else if (mean > 64) fx_copy_kernel<64, false><<<grid, 256, 0, s>>>(text, src, dofs, m, dst);
    else if (mean > 16) fx_copy_kernel<16, false><<<grid, 256, 0, s>>>(text, src, dofs, m, dst);
    else fx_copy_kernel<4, false><<<grid, 256, 0, s>>>(text, src, dofs, m, dst);
    return hipGetLastError();
}

hipError_t launch_max_u64(void* temp, size_t temp_bytes, const uint64_t* in, uint64_t n, uint64_t* out,
                          hipStream_t s) {
    if (!n) return hipMemsetAsync(out, 0, sizeof(uint64_t), s);
    return hipcub::DeviceReduce::Max(temp, temp_bytes, in, out, (int)n, s);
}

}  // namespace xs
