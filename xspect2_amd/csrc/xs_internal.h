// xs_internal.h — shared between the host library (xs_api.cpp) and the
// gfx950 kernels (xs_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <exception>
#include <functional>
#include <new>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>
#include <stdint.h>

namespace xs {

// k-mers per work unit.  A read with more sampled k-mers is split into
// ceil(nk / kSegKmers) units whose partial counts are added atomically.
constexpr uint32_t kSegKmers = 256;
// Block geometry of the probe kernels (4 waves).
constexpr int kProbeThreads = 256;
constexpr int kWave = 64;
// Maximum k supported on the device (canonical k-mer held in 8 dwords).
constexpr uint32_t kMaxK = 32;
// Maximum hash functions per bank on the device.
constexpr uint32_t kMaxHashes = 16;
// Maximum 16-byte chunks per padded row of one group (1024 docs per group).
constexpr uint32_t kMaxChunks = 8;
// LDS budget per probe block for per-wave doc counters.
constexpr uint32_t kLdsBudget = 64 * 1024;

// How a k-mer's bytes are canonicalised: COBS (species, MLST) or rbloom/Biopython (genus).
enum KmerMode : int { kKmerCobs = 0, kKmerBio = 1 };

// One COBS doc group on the device.
struct GroupDesc {
    uint64_t sig;    // signature size (rows)
    uint64_t magic;  // floor((2^64-1)/sig) for Barrett reduction
    uint64_t base;   // byte offset of row 0 in the device image
};

struct CobsView {
    const uint8_t* rows;      // device image, rows of `pitch` bytes per group
    const GroupDesc* groups;  // device array [G]
    uint32_t G;
    uint32_t pitch;           // device bytes per row (multiple of 16)
    uint32_t nchunks;         // pitch / 16
    uint32_t h;
    uint64_t page;            // file bytes per row (docs per group = 8*page)
    uint64_t D;
    uint64_t sig0;            // host copy of groups[0].sig (fast-path selection)
    uint64_t sig_max;         // host copy of the largest group sig (32-bit row index paths)
};

struct BloomView {
    const uint32_t* bits;  // device image, padded to 16 bytes
    uint64_t mbits;        // number of bits (nbytes*8)
    uint64_t magic;        // floor((2^64-1)/mbits)
    uint32_t K;
    uint64_t* rows_read;   // when profiling: += filter words the probe loaded
};

// Reads / records laid out for one probe or build call.
struct ReadView {
    const uint8_t* seq;        // read bytes as handed over (no padding required)
    uint64_t seq_bytes;        // size of the seq buffer: loads stop there
    const uint64_t* offs;      // n+1
    const uint32_t* unit_read; // units -> read
    const uint64_t* unit_ofs;  // first unit of each read (n)
    uint64_t* queue;           // device: [0] = #units, [1] = next unit to hand out
    uint64_t n;
    uint32_t k;
    uint32_t step;
    uint32_t grab = 4;         // units a wave takes from the queue per atomic (small calls: 1)
};

// ---- launchers (xs_kernels.hip) -------------------------------------------
hipError_t launch_units(const uint64_t* offs, uint64_t n, uint32_t k, uint32_t step,
                        uint64_t* nk_out, uint64_t* nseg, hipStream_t s);
size_t scan_temp_bytes(uint64_t n);
hipError_t launch_scan(void* temp, size_t temp_bytes, const uint64_t* in, uint64_t* out,
                       uint64_t n, hipStream_t s);
hipError_t launch_scatter_units(const uint64_t* nseg, const uint64_t* unit_ofs, uint64_t n,
                                uint32_t* unit_read, uint64_t* queue, uint32_t* hits_zero,
                                uint64_t D, hipStream_t s);
int probe_blocks(uint64_t D, int* waves_per_block, size_t* lds_bytes);
int probe_grid_cobs(const CobsView& bv, uint32_t k);
int probe_grid_bloom();
hipError_t launch_probe_cobs(const ReadView& rv, const CobsView& bv, uint32_t* hits,
                             uint64_t* partials, int blocks, hipStream_t s);
hipError_t launch_probe_bloom(const ReadView& rv, const BloomView& bv, uint32_t* hits,
                              uint64_t* partials, int blocks, hipStream_t s);
// Profiling of the partitioned probes: an event recorded on the launch stream
// at each pass boundary, tagged with the pass that just ended (kPassStart opens
// a query).  xs_bank_pass_stats sums the gaps per pass.
enum PassTag { kPassStart = -1, kPassPrep = 0, kPassBucket = 1, kPassLookup = 2, kPassResolve = 3, kPassTags = 4 };
// Marks past kPassMarksMax since the last xs_bank_pass_stats are dropped, so
// a profiling run that never reads its stats does not grow the pool forever.
constexpr size_t kPassMarksMax = 1u << 16;
struct PassRecorder {
    std::vector<hipEvent_t>* pool;
    std::vector<int>* tags;
    size_t* used;
    hipError_t mark(int tag, hipStream_t s) {
        if (*used >= kPassMarksMax) return hipSuccess;
        if (*used == pool->size()) {
            hipEvent_t e;
            hipError_t err = hipEventCreate(&e);
            if (err != hipSuccess) return err;
            pool->push_back(e);
            tags->push_back(0);
        }
        (*tags)[*used] = tag;
        return hipEventRecord((*pool)[(*used)++], s);
    }
};
inline void pass_mark(PassRecorder* r, int tag, hipStream_t s) {
    if (r) (void)r->mark(tag, s);
}

// Probe path selection of one bank handle (xs_bank_set_probe_options; the
// defaults are what every production query takes).  Read by the planners at
// each query, under the handle's mutex; no environment variable changes them.
constexpr uint32_t kCobsPartWsMiB = 24 << 10;  // default cap of a range's entries + rows
struct ProbeOptions {
    // partitioned COBS probe: 0 = direct probe only; 1 = automatic (classic banks of
    // <= 128 docs of at least kCobsPartMinBankMiB, calls of at least kCobsPartMinKmers
    // k-mers); 2 = every such bank and call; 3 = as 2 with partitions down to 1024
    // rows; 4 = as 2 with partitions of 1024 rows (more than kCobsPadParts: unpadded runs)
    int cobs_part = 1;
    // partitioned rbloom probe: 0 = gather probe only; 1 = automatic (filters of
    // >= 16 MiB on member-rich input); 2 = such filters whatever the input; 3 =
    // every filter, with partitions down to 1024 bits
    int bloom_part = 1;
    uint32_t workspace_mib = kCobsPartWsMiB;  // cap of the partitioned COBS probe's workspace
    int small_calls = 1;                      // 0: small host calls take the regular pipeline
};

// Partitioned rbloom probe (xs_probe_bloompart.hip): k-mers per bucket block,
// most hash functions it takes, most filter partitions.
constexpr int kPartKmers = 1024;
constexpr int kPartKMax = 8;
constexpr uint32_t kPartMax = 1024;
struct BloomPartPlan {
    uint32_t shift;      // log2 filter bits per partition
    uint32_t P;          // partitions
    uint64_t tstride;    // bucket blocks (>= the call's k-mers / kPartKmers)
    uint64_t kbound;     // upper bound of the call's sampled k-mers
    size_t entry_bytes, tbl_bytes, miss_bytes, nkc_bytes, scan_bytes, aux_bytes;
};
struct BloomPartWs {
    uint64_t* nkc;       // n+1 per-read k-mer counts
    uint64_t* kofs;      // n+1 exclusive scan: first k-mer id of each read
    void* scan_tmp;
    size_t scan_bytes;
    uint64_t* entries;   // tstride regions of kPartKmers*K entries: u32 offsets, u16 k-mer ids, u8 miss flags
    uint16_t* tbl;       // (P+1) x tstride partition starts per bucket block
    uint32_t* miss;      // one bit per k-mer id: some filter bit was zero
    uint32_t* aux;       // bucket block -> read holding its first k-mer (tstride+1), then per-partition queue counters
};
// False when the direct probe should run (small filter, K > kPartKMax, a
// batch too large for the transient workspace, member-poor input -- the
// previous query's member fraction below kPartMinMembers -- or
// opt.bloom_part = 0).
constexpr double kPartMinMembers = 0.24;  // measured crossover, profiles/r01_bloom_crossover.txt
bool bloom_part_plan(const BloomView& bv, uint64_t n, uint64_t seq_bytes, uint32_t step, double member_frac,
                     const ProbeOptions& opt, BloomPartPlan* plan);
hipError_t launch_probe_bloom_part(const ReadView& rv, const BloomView& bv, const BloomPartPlan& plan,
                                   const BloomPartWs& ws, uint32_t* hits, uint64_t* partials, int blocks,
                                   hipStream_t s, PassRecorder* rec = nullptr);
// Partitioned COBS probe (xs_probe_cobspart.hip) for classic banks of <= 128
// docs (16-B rows) larger than the Infinity Cache.
constexpr uint64_t kCobsPartMinKmers = 1ull << 23;  // default mode: smaller batches take the direct probe
constexpr uint64_t kCobsPartMinBankMiB = 32;         // default mode: smaller banks take the direct probe
struct CobsPartPlan {
    uint32_t ck;         // k-mers per bucket block (1024, 2048 or 4096)
    uint32_t shift;      // log2 rows per partition
    uint32_t P;          // partitions
    uint64_t nblk;       // bucket blocks (>= the call's k-mers / ck)
    uint64_t rblk;       // bucket blocks per range (one workspace, reused range after range)
    uint64_t kbound;     // upper bound of the call's sampled k-mers
    uint32_t pad;        // each partition's run of a block padded to a multiple of pad entries (1 or 4)
    uint64_t stride;     // entries per bucket block region (ck * h, plus the padding, multiple of 8)
    size_t entry_bytes, tbl_bytes, nkc_bytes, scan_bytes, aux_bytes;
};
// Runs are padded (64-B aligned rows) only while P <= kCobsPadParts: the pad
// slots live in the bucket block's LDS.
constexpr uint32_t kCobsPadParts = 512;
constexpr uint32_t kCobsPadEntry = 0xFFFFFFFFu;  // pad slot: the lookup writes an all-ones row
struct PartWs {
    uint64_t* nkc;       // n+1 per-read k-mer counts
    uint64_t* kofs;      // n+1 exclusive scan: first k-mer id of each read
    void* scan_tmp;
    size_t scan_bytes;
    void* entries;       // a range's u32 entries (row in partition << id bits | k-mer in block), then their 16-B rows
    uint16_t* tbl;       // (P+1) x rblk partition starts per bucket block, + block-major copy
    uint32_t* aux;       // bucket block -> read holding its first k-mer, then per-partition queue counters
};
// False when the direct probe should run (bank not classic 16-B rows, under
// kCobsPartMinBankMiB, h > 8, fewer than kCobsPartMinKmers k-mers in the call, or
// opt.cobs_part = 0).
bool cobs_part_plan(const CobsView& bv, uint32_t k, uint64_t n, uint64_t seq_bytes, uint32_t step,
                    const ProbeOptions& opt, CobsPartPlan* plan);
hipError_t launch_probe_cobs_part(const ReadView& rv, const CobsView& bv, const CobsPartPlan& plan,
                                  const PartWs& ws, uint32_t* hits, uint64_t* partials, int blocks,
                                  hipStream_t s, PassRecorder* rec = nullptr);
hipError_t launch_reduce_partials(const uint64_t* partials, int blocks, uint64_t cols,
                                  uint64_t* totals, hipStream_t s);
hipError_t launch_build_cobs(const ReadView& rv, const uint32_t* rec_doc, const CobsView& bv,
                             uint32_t* rows_mut, int blocks, hipStream_t s);
hipError_t launch_build_bloom(const ReadView& rv, const BloomView& bv, uint32_t* bits_mut,
                              int blocks, hipStream_t s);
hipError_t launch_repack(const uint8_t* src, uint64_t src_pitch, uint8_t* dst, uint64_t dst_pitch,
                         uint64_t rows, uint64_t copy_bytes, hipStream_t s);
// Sum of hits[c][d] > threshold into scores[seq_of_chunk[c]][d]; with `first`
// (pre-filled with UINT32_MAX) also the first such chunk, and with first_score
// that chunk's count.
hipError_t launch_mlst_sum(const uint32_t* hits, const uint32_t* seq_of_chunk, uint64_t n_chunks,
                           uint64_t D, uint32_t threshold, unsigned long long* scores,
                           uint32_t* first, uint32_t* first_score, hipStream_t s);

// Host-side constants shared with the kernels.
inline uint64_t barrett_magic(uint64_t d) { return d ? (~0ull) / d : 0; }

// best_doc_kernel's value for reads whose maximum is shared (= XS_BEST_AMBIGUOUS).
constexpr uint32_t kBestAmbiguous = 0xFFFFFFFFu;
hipError_t launch_best_doc(const uint32_t* hits, uint64_t n, uint64_t D, uint32_t* best,
                           uint32_t* best_hits, hipStream_t s);

// dst[i] = src[i] as uint8 (hit_bytes 1) or uint16 (2); the caller guarantees the values fit.
hipError_t launch_narrow_hits(const uint32_t* src, void* dst, uint64_t n, int hit_bytes, hipStream_t s,
                              uint32_t* overflow = nullptr);

hipError_t launch_gather_reads(const uint8_t* seqs, const uint64_t* offs, const uint32_t* index, uint64_t m,
                               uint8_t* out, const uint64_t* out_offs, hipStream_t s);

// ---- device-mode reader (xs_fastx_dev.hip) ----------------------------------
// Text bytes per tile of the newline index (a window's device copy is padded
// with zeros to a whole tile).
constexpr uint64_t kFxTile = 16384;
// Per record: where its sequence / id / title start in the window's text and
// how long they are (the lengths, n+1 entries with [n] = 0, are scanned into
// output offsets).
struct FxRuns {
    uint32_t* seq_src;
    uint64_t* seq_len;
    uint32_t* id_src;
    uint64_t* id_len;
    uint32_t* desc_src;
    uint64_t* desc_len;
};
// FASTQ record blocks: sequence, id and title bytes, and the longest sequence
struct FqBlockSums {
    uint64_t seq, id, desc, mx;
};
size_t fx_temp_bytes(uint64_t n);
hipError_t launch_fx_count(const uint8_t* text, uint64_t tiles, uint64_t* tile_cnt, hipStream_t s);
hipError_t launch_fx_positions(const uint8_t* text, uint64_t tiles, const uint64_t* tile_ofs, uint32_t* nl,
                               hipStream_t s);
// FASTQ records (4 lines each) of the window, then in three kernels the
// offsets of their sequences, ids and titles (n+1 each) and the window's
// status ([0] bad, [1] records, [2] sequence, [3] id, [4] title bytes, [5]
// longest sequence): no host round trip between the passes.
hipError_t launch_fq_records(const uint8_t* text, const uint32_t* nl, uint64_t n, const FxRuns& runs,
                             uint32_t* bad, FqBlockSums* blk, uint64_t* blk_ofs, uint64_t* offs, uint64_t* id_ofs,
                             uint64_t* desc_ofs, uint64_t* status, hipStream_t s);
hipError_t launch_fa_headers(const uint8_t* text, const uint32_t* nl, uint64_t L, uint64_t* hdr, hipStream_t s);
hipError_t launch_fa_lines(const uint8_t* text, const uint32_t* nl, uint64_t L, const uint64_t* hofs,
                           uint32_t* line_src, uint64_t* line_len, uint32_t* rec_line, const FxRuns& runs,
                           uint32_t* bad, hipStream_t s);
hipError_t launch_fa_offsets(const uint32_t* rec_line, const uint64_t* line_ofs, uint64_t L, const uint64_t* n_dev,
                             uint64_t* offs, uint64_t* lens, hipStream_t s);
hipError_t launch_fx_copy(const uint8_t* text, const uint32_t* src, const uint64_t* dofs, uint64_t m, uint64_t bytes,
                          uint8_t* dst, hipStream_t s);
hipError_t launch_max_u64(void* temp, size_t temp_bytes, const uint64_t* in, uint64_t n, uint64_t* out,
                          hipStream_t s);

// Set the thread-local message xs_last_error() returns; returns `code`.
int set_error(int code, const char* msg);

// Page-locked host memory for DMA staging and callers' outputs.  Requests of
// 2 MiB and more are anonymous mappings backed by 2 MiB pages, faulted by up
// to 8 threads and registered with HIP (hipHostRegister): 2.2 ms per 128 MiB
// against 22.5 ms for hipHostMalloc on the MI355X boxes, at the same DMA rate
// (profiles/r05o_pin.json, tools/pin_probe.py).  Smaller requests, and any
// mapping HIP refuses to register, take hipHostMalloc.  Memory from
// pinned_alloc goes back through pinned_free only.  Contents start zeroed for
// the mapped kind, unspecified for the hipHostMalloc kind.
int pinned_alloc(size_t bytes, void** out);
void pinned_free(void* p);

// fn(t) for every t in [0, n): t = 0 on the calling thread, the others on the
// library's persistent host workers (started once, reused by every call: no
// thread is created per copy or pass).  Returns when all n have finished; an
// exception thrown by any fn(t) is rethrown here, on the calling thread, after
// the others have finished.  Calls from several threads at once share the
// workers; the caller itself runs tasks while it waits, so a call always
// completes even if no worker could be started.
void parallel_for(int n, const std::function<void(int)>& fn);

// Threads started for one call that must run beside it (a reader's loader, a
// writer behind the formatting), joined on every exit path: when a start
// fails, the threads already running finish before the exception leaves.
struct ThreadGroup {
    std::vector<std::thread> th;
    template <class... A>
    void start(A&&... a) {
        th.emplace_back(std::forward<A>(a)...);
    }
    void join() {
        for (auto& x : th)
            if (x.joinable()) x.join();
        th.clear();
    }
    ThreadGroup() = default;
    ThreadGroup(const ThreadGroup&) = delete;
    ThreadGroup& operator=(const ThreadGroup&) = delete;
    ~ThreadGroup() { join(); }
};

// Every C-ABI entry point runs its body under guard(): a C++ exception (a
// host vector that cannot be allocated, a worker thread that cannot start)
// becomes XS_ERR_NOMEM / XS_ERR_INTERNAL and a message instead of unwinding
// into the caller's C frames, where it would end the process.
template <class R>
R guard_failed(int code, const char* msg) noexcept {
    const int rc = set_error(code, msg);
    if constexpr (std::is_same_v<R, int>) return rc;
    else if constexpr (std::is_pointer_v<R>) return nullptr;
    else if constexpr (!std::is_void_v<R>) return R{};
}

template <class F>
auto guard(F&& f) noexcept -> decltype(f()) {
    using R = decltype(f());
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return guard_failed<R>(-6 /* XS_ERR_NOMEM */, "host memory allocation failed");
    } catch (const std::exception& e) {
        return guard_failed<R>(-7 /* XS_ERR_INTERNAL */, e.what());
    } catch (...) {
        return guard_failed<R>(-7 /* XS_ERR_INTERNAL */, "unknown C++ exception");
    }
}

}  // namespace xs
