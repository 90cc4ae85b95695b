/*
 * xspect_hip.h — C ABI of libxspect_hip.so, the MI355X (gfx950) k-mer x filter
 * probe engine behind the XspecT model classes.
 *
 * The reference crosses a Python<->native FFI once per READ (pybind11 into
 * cobs_index, PyO3 into rbloom with a Python callback per k-mer).  This ABI
 * replaces those crossings with one call per BATCH of reads.  Each entry point
 * names the reference interface it replaces (paths relative to the reference
 * repository):
 *
 *   xs_bank_open            cobs_index.Search(path, True/False)
 *                             src/xspect/models/probabilistic_filter_model.py:389
 *                             src/xspect/models/probabilistic_filter_svm_model.py:313
 *                             src/xspect/models/probabilistic_filter_mlst_model.py:188
 *                           rbloom.Bloom.load(path, hash_func=xxh3_64_intdigest)
 *                             src/xspect/models/probabilistic_single_filter_model.py:155-158
 *   xs_query                Search.search(str(seq), step=step), batched over reads
 *                             probabilistic_filter_model.py:227 (+ _count_kmers :462)
 *                             probabilistic_filter_mlst_model.py:242,274-276
 *                           sum(1 for kmer in _generate_kmers(seq, step) if kmer in bf)
 *                             probabilistic_single_filter_model.py:122-124
 *   xs_query_totals         ModelResult.get_total_hits() + sum(num_kmers)
 *                             src/xspect/models/result.py:57-72,76-90 (device-side)
 *   xs_query_device         same as xs_query on device-resident buffers/stream
 *   xs_bank_create_cobs,    cobs_index.ClassicIndexParameters/classic_construct_list
 *   xs_bank_build,            probabilistic_filter_model.py:186-192
 *   xs_bank_save            CompactIndexParameters/compact_construct_list
 *                             probabilistic_filter_mlst_model.py:132-141
 *   xs_bank_create_bloom    rbloom.Bloom(n, fpr, hash_func), .add(kmer), .save(path)
 *                             probabilistic_single_filter_model.py:88-96
 *
 * Conventions: every int-returning call returns XS_OK (0) or a negative
 * XS_ERR_* code; xs_last_error() returns a thread-local message for the last
 * failure on the calling thread.  No C++ exception leaves the library: a failed
 * host allocation inside a call is XS_ERR_NOMEM, any other C++ runtime failure
 * XS_ERR_INTERNAL (NULL from a pointer-returning call; nothing from a void
 * one).  Host buffers are borrowed for the duration of
 * the call only.  A bank handle owns its device memory and one HIP stream;
 * calls on one handle are serialised by an internal mutex, distinct handles are
 * independent.  The handle's device workspace is shared by all its calls: a
 * call enqueued on a different stream than the handle's previous call (the
 * *_device entry points take the caller's stream) is ordered after that call
 * on the device, so one handle may be used from several streams.  No
 * callbacks into the caller.
 */
#ifndef XSPECT_HIP_H
#define XSPECT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define XS_OK 0
#define XS_ERR_ARG (-1)
#define XS_ERR_IO (-2)
#define XS_ERR_FORMAT (-3)
#define XS_ERR_HIP (-4)
#define XS_ERR_UNSUPPORTED (-5)
#define XS_ERR_NOMEM (-6)    /* a host allocation failed inside the call */
#define XS_ERR_INTERNAL (-7) /* any other C++ runtime failure (e.g. a thread could not be started) */

#define XS_BANK_COBS_CLASSIC 0
#define XS_BANK_COBS_COMPACT 1
#define XS_BANK_RBLOOM 2

typedef struct xs_bank xs_bank;

typedef struct xs_bank_info_t {
    int32_t kind;             /* XS_BANK_* */
    int32_t device;           /* HIP device ordinal the bank is resident on */
    uint32_t term_size;       /* k */
    uint32_t num_hashes;      /* COBS h, or rbloom K */
    uint32_t canonicalize;    /* 1: canonical k-mers (always 1 for XspecT banks) */
    uint32_t reserved;
    uint64_t num_docs;        /* D (1 for rbloom) */
    uint64_t num_groups;      /* COBS doc groups (1 for classic) */
    uint64_t page_size;       /* bytes per row per group in the file layout */
    uint64_t signature_rows;  /* sum of signature sizes over groups */
    uint64_t bloom_bits;      /* rbloom bit count (0 for COBS) */
    uint64_t device_bytes;    /* device bytes held by the bank image */
    uint64_t device_row_pitch;/* padded device bytes per row per group */
} xs_bank_info_t;

int xs_version(void);
/* Build id: the first 16 hex digits of a SHA-256 over the library's sources,
 * headers, compiler flags and target, fixed when it was built
 * (xspect2_amd/build.py: source_id).  No reference counterpart: the
 * reference's native dependencies are unpinned (pyproject.toml:16-17), this
 * names exactly which sources a loaded library came from. */
const char* xs_build_id(void);
const char* xs_last_error(void);
int xs_device_count(int* count);

/* Open a bank file and make it resident on `device`.  kind = XS_BANK_*. */
int xs_bank_open(const char* path, int kind, int device, xs_bank** out);
/* A classic COBS index with only docs [doc_lo, doc_hi) resident: each row's
 * byte columns of those docs (doc_lo and doc_hi multiples of 8, or doc_hi the
 * doc count).  One bank column-split over ranks (SURVEY.md §8(e) config 5,
 * option b): every rank hashes every k-mer and reads its slice of each row;
 * the per-read hit columns are then all-gathered (xspect2_amd.distributed). */
int xs_bank_open_docs(const char* path, int device, uint64_t doc_lo, uint64_t doc_hi, xs_bank** out);

/* Create an empty COBS bank (classic: num_groups = 1 and page_size =
 * ceil(num_docs/8); compact: num_groups groups of 8*page_size docs each, the
 * last one partial).  sig[g] = signature size of group g.  doc_names may be
 * NULL (names "0", "1", ...). */
int xs_bank_create_cobs(int device, int kind, uint32_t term_size, uint32_t num_hashes,
                        uint64_t num_docs, uint64_t page_size, uint64_t num_groups,
                        const uint64_t* sig, const char* const* doc_names, xs_bank** out);

/* Create an empty rbloom bank of nbytes bytes and nhash index functions. */
int xs_bank_create_bloom(int device, uint32_t term_size, uint64_t nbytes, uint32_t nhash,
                         xs_bank** out);

/* Insert every k-mer (step 1) of n_rec host records; record r belongs to doc
 * rec_doc[r] (ignored for rbloom; may be NULL there). */
int xs_bank_build(xs_bank* bank, const char* seqs, const uint64_t* offsets,
                  const uint32_t* rec_doc, uint64_t n_rec);
/* Same with device-resident buffers, enqueued on `stream` (NULL = the null stream). */
int xs_bank_build_device(xs_bank* bank, const void* d_seqs, uint64_t seq_bytes,
                         const uint64_t* d_offsets, const uint32_t* d_rec_doc, uint64_t n_rec,
                         void* stream);

int xs_bank_save(xs_bank* bank, const char* path);
/* Copy the bank back in FILE layout (rows of page_size bytes, groups in order;
 * rbloom: the raw bit bytes). nbytes must equal the file payload size. */
int xs_bank_download(xs_bank* bank, void* host, uint64_t nbytes);
/* Replace the bank image from a FILE-layout payload (the inverse of download). */
int xs_bank_upload(xs_bank* bank, const void* host, uint64_t nbytes);

/* rbloom files carry no k-mer length (XspecT keeps it in the model JSON,
 * probabilistic_single_filter_model.py:143-151); set it after xs_bank_open. */
int xs_bank_set_term_size(xs_bank* bank, uint32_t term_size);

int xs_bank_info(const xs_bank* bank, xs_bank_info_t* out);
/* Signature size of each doc group (num_groups entries; COBS banks only). */
int xs_bank_signature_sizes(const xs_bank* bank, uint64_t* out, uint64_t n);
const char* xs_bank_doc_name(const xs_bank* bank, uint64_t i);

/* Probe n reads (host buffers): read r = seqs[offsets[r] .. offsets[r+1]).
 * hits_out: n x D uint32 (row-major, may be NULL), num_kmers_out: n (may be
 * NULL).  k-mers are taken at positions i*step, i < ceil((len-k+1)/step);
 * reads shorter than k contribute no k-mers. */
int xs_query(xs_bank* bank, const char* seqs, const uint64_t* offsets, uint64_t n, uint32_t step,
             uint32_t* hits_out, uint64_t* num_kmers_out);

/* xs_query with the hit matrix in hit_bytes = 1, 2 or 4 bytes per count
 * (uint8 / uint16 / uint32).  A count never exceeds its read's sampled k-mers,
 * so 150 bp reads (130 k-mers) come back in one byte: the matrix is narrowed
 * on the device and a quarter of the bytes cross PCIe.  Fails with XS_ERR_ARG
 * if some read has more k-mers than the width holds. */
int xs_query_hits(xs_bank* bank, const char* seqs, const uint64_t* offsets, uint64_t n, uint32_t step,
                  void* hits_out, int hit_bytes, uint64_t* num_kmers_out);
/* xs_query_hits / xs_query_totals for reads already in HBM (an
 * xs_fastx_dbatch: d_seqs, seq_bytes, d_offsets with [0] = 0, max_len = its
 * longest read, which bounds every count for the width check).  Outputs are
 * host memory, each optional: hits_out n x D (hit_bytes 1, 2 or 4), the
 * sampled k-mer counts, totals_out D+1 (per-doc sums, then the k-mer total).
 * The probe runs in read chunks whose hit rows go back while the next chunk
 * is probed. */
int xs_query_hits_device(xs_bank* bank, const void* d_seqs, uint64_t seq_bytes, const uint64_t* d_offsets,
                         uint64_t n, uint64_t max_len, uint32_t step, void* hits_out, int hit_bytes,
                         uint64_t* num_kmers_out, uint64_t* totals_out);

/* Blocking device -> host copy of `bytes` (e.g. an xs_fastx_dbatch's
 * sequences, for checks). */
int xs_memcpy_to_host(void* host, const void* dev, uint64_t bytes);

/* Device -> device copy of `bytes`, asynchronous on `stream` (e.g. a device
 * reader batch's sequences into a caller's buffer for a collective). */
int xs_memcpy_device(void* dst, const void* src, uint64_t bytes, void* stream);

/* Pinned (page-locked) host memory for outputs the caller reuses across calls:
 * results land there by DMA, with no page faults on a fresh pageable buffer. */
int xs_host_alloc(uint64_t bytes, void** out);
void xs_host_free(void* p);

/* totals_out[d] = sum over reads of hits[r][d] (D entries, uint64),
 * *total_kmers_out = sum of num_kmers.  No per-read matrix is materialised. */
int xs_query_totals(xs_bank* bank, const char* seqs, const uint64_t* offsets, uint64_t n,
                    uint32_t step, uint64_t* totals_out, uint64_t* total_kmers_out);

/* Device-resident variant, asynchronous on `stream` (NULL = the null stream,
 * ordered with all blocking streams; pass torch.cuda.current_stream().cuda_stream).
 * d_seqs holds seq_bytes bytes; d_offsets n+1 uint64.  Any of d_hits (n x D
 * uint32), d_num_kmers (n uint64) and d_totals (D+1 uint64: per-doc totals then
 * the k-mer total) may be NULL.  The bank must live on the current device. */
int xs_query_device(xs_bank* bank, const void* d_seqs, uint64_t seq_bytes,
                    const uint64_t* d_offsets, uint64_t n, uint32_t step, uint32_t* d_hits,
                    uint64_t* d_num_kmers, uint64_t* d_totals, void* stream);

/* Per-read best doc without materialising the hit matrix on the host:
 * best_doc[r] = the doc with the most hits of read r, or XS_BEST_AMBIGUOUS when
 * two or more docs share the maximum (the per-read call of the reference's
 * benchmark, scripts/benchmark/main.nf:417-436); best_hits[r] = that maximum.
 * best_hits, num_kmers_out and totals_out (D+1 entries, as xs_query_totals
 * then the k-mer total) may be NULL. */
#define XS_BEST_AMBIGUOUS 0xFFFFFFFFu
int xs_query_best(xs_bank* bank, const char* seqs, const uint64_t* offsets, uint64_t n, uint32_t step,
                  uint32_t* best_doc, uint32_t* best_hits, uint64_t* num_kmers_out, uint64_t* totals_out);
/* The same reduction over a device hit matrix (n x num_docs uint32) on `stream`. */
int xs_best_device(const uint32_t* d_hits, uint64_t n, uint64_t num_docs, uint32_t* d_best_doc,
                   uint32_t* d_best_hits, void* stream);

/* Device-side read compaction (the genus -> species hand-off of the fused
 * pipeline, replacing the filtered FASTA of src/xspect/main.py:116-145):
 * output read j = input read d_index[j], written at d_out_offsets[j] (m+1
 * entries, computed by the caller from the kept lengths), on `stream`. */
int xs_gather_reads_device(const void* d_seqs, const uint64_t* d_offsets, const uint32_t* d_index, uint64_t m,
                           void* d_out_seqs, const uint64_t* d_out_offsets, void* stream);

/* MLST chunk scoring (probabilistic_filter_mlst_model.py:237-256): for chunk
 * hit rows hits[c][d] whose owner is seq_of_chunk[c] (non-decreasing), sum
 * hits[c][d] into scores[seq][d] only where hits[c][d] > threshold
 * (get_cobs_result :378).  Host buffers; computed on the device. */
int xs_mlst_sum(xs_bank* bank, const uint32_t* hits, const uint32_t* seq_of_chunk,
                uint64_t n_chunks, uint64_t n_seqs, uint32_t threshold, uint64_t* scores);

/* One MLST locus in one call (probabilistic_filter_mlst_model.py:192-303; the
 * reference makes one cobs search per sequence, and per chunk of every
 * sequence >= 10 kbp, :236-286).  Records [0, n_direct) of seqs/offsets are
 * sequences probed whole: their hit rows come back in direct_hits
 * (n_direct x D uint32).  Records [n_direct, n_direct + n_chunks) are the
 * sequence_splitter chunks (:382-426) of the longer sequences, chunk c owned by
 * sequence chunk_owner[c] (non-decreasing, < n_owners); their rows stay on
 * the device, where per (owner, allele) the chunk scores > threshold
 * (get_cobs_result :377-380) are summed into owner_scores (n_owners x D,
 * :249-252), owner_first gets the first such chunk (index among the chunks,
 * UINT32_MAX if none) and owner_first_score its score: the position at which
 * the reference's all_counts dict first sees the allele, which orders ties of
 * its stable sort by -score (:254-256).  offsets: n_direct + n_chunks + 1
 * entries.  Every output may be NULL (owner_first_score needs owner_first). */
int xs_mlst_query(xs_bank* bank, const char* seqs, const uint64_t* offsets, uint64_t n_direct, uint64_t n_chunks,
                  const uint32_t* chunk_owner, uint64_t n_owners, uint32_t step, uint32_t threshold,
                  uint32_t* direct_hits, uint64_t* owner_scores, uint32_t* owner_first,
                  uint32_t* owner_first_score);

/* Record HIP events around the probe kernel of every query on this handle. */
int xs_bank_set_profiling(xs_bank* bank, int on);
/* Duration of the probe kernel of the last profiled query, milliseconds. */
int xs_bank_last_probe_ms(xs_bank* bank, float* ms);
/* Count, summed and maximum duration of every probe kernel launched since
 * profiling was enabled or the last call of this function (then resets). */
int xs_bank_probe_stats(xs_bank* bank, uint64_t* count, double* total_ms, float* max_ms);

/* Partitioned probes (xs_bank_probe_path == XS_PATH_PARTITIONED), profiling
 * on: time spent per pass since the last call (then resets), from HIP events
 * on the launch stream at the pass boundaries.  ms[4], count[4] indexed by
 * pass: 0 prep (k-mer counts, scan, block map), 1 bucket (hash, bin by bank
 * partition, transpose), 2 lookup (per-XCD L2-resident partition gathers),
 * 3 resolve (AND per k-mer and count; rbloom: resolve + count).  count =
 * pass instances (one per workspace range). */
int xs_bank_pass_stats(xs_bank* bank, double* ms, uint64_t* count);

/* rbloom banks: filter words the probe kernels loaded since profiling was
 * enabled or the last call (then resets).  The probe tests 2 bits first and
 * loads the other K-2 only for k-mers that pass them, as rbloom stops at the
 * first zero bit, so the count depends on the data; the partitioned path
 * (xs_bank_probe_path) tests all K.  0 for COBS banks, whose kernels read
 * exactly h rows per k-mer and doc group. */
int xs_bank_probe_rows(xs_bank* bank, uint64_t* rows);

/* Probe path of the last query on this handle: XS_PATH_GATHER (one random
 * filter/row gather per hash, every bank kind) or XS_PATH_PARTITIONED (rbloom
 * filters of >= 16 MiB: k-mer bit indices binned by 2 MiB filter partition,
 * each partition tested from one XCD's L2).  The partitioned path is taken
 * while the handle's previous query found at least 24 % of its k-mers in the
 * filter (member-rich input, where it is faster); xs_bank_set_probe_options
 * can disable it.  Both give identical results. */
#define XS_PATH_GATHER 0
#define XS_PATH_PARTITIONED 1
int xs_bank_probe_path(const xs_bank* bank, int* path);

/* Probe path selection of one handle.  The defaults (what xs_bank_open and
 * xs_bank_create_* set: 1, 1, 24576, 1) are the paths a production query takes;
 * the other values exist so tests can run every path on the same bank, and no
 * environment variable changes them.  Every path gives identical results.  No
 * reference counterpart (cobs_index / rbloom have one probe each,
 * pyproject.toml:16-17).  Applies to the handle's next query. */
typedef struct xs_probe_options_t {
    int32_t cobs_part;      /* COBS classic banks of <= 128 docs: 0 = direct probe only; 1 = the partitioned
                               probe for banks of >= 32 MiB and calls of >= 2^23 k-mers; 2 = partitioned for
                               every such bank and call; 3 = as 2 with partitions down to 1024 rows; 4 = as 2
                               with partitions of 1024 rows */
    int32_t bloom_part;     /* rbloom: 0 = gather probe only; 1 = partitioned for filters of >= 16 MiB on
                               member-rich input; 2 = such filters whatever the input; 3 = every filter, with
                               partitions down to 1024 bits */
    uint32_t workspace_mib; /* cap of the partitioned COBS probe's transient workspace (a larger call runs in
                               ranges that reuse it) */
    int32_t small_calls;    /* 1: calls of <= 4096 reads and <= 1 MiB go to the device in one round trip;
                               0: every call takes the regular chunked pipeline */
} xs_probe_options_t;
int xs_bank_set_probe_options(xs_bank* bank, const xs_probe_options_t* options);
int xs_bank_get_probe_options(const xs_bank* bank, xs_probe_options_t* options);

/* Device bytes of the handle's transient workspace (staging, reads, hit
 * matrices, the partitioned probes' entries and rows; not the bank image):
 * held now, and the most held at once since the handle was created.  For
 * memory planning beside other work on the GPU (288 GB per MI355X); a doc
 * slice (xs_bank_open_docs) stages one ~32 MiB piece of whole rows at a time,
 * never the whole bank. */
int xs_bank_workspace_bytes(const xs_bank* bank, uint64_t* held, uint64_t* peak);

void xs_bank_close(xs_bank* bank);

/* ---- Result output (src/xspect/models/result.py:151-202, json.dumps(indent=4)).
 * Appends the "hits", "scores" (with "total") and "num_kmers" sections of a
 * ModelResult JSON for an n x num_docs hit matrix to `path`; the caller writes
 * the fields before and after.  hits: counts of hit_bytes = 1, 2 or 4 bytes
 * (uint8/uint16/uint32: a matrix narrowed on the device stays narrow).
 * ids_json / labels_json: packed JSON string literals (quotes included) with
 * n+1 / num_docs+1 offsets; doc_mask (num_docs bytes, 1 = keep) may be NULL.
 * total_hits (num_docs sums), total_kmers and total_order_row (a hit row
 * whose COBS order orders the "total" labels): the whole job's totals for one
 * shard of a read-sharded job (n may then be 0); NULL: computed from this
 * matrix and its first row.  threads <= 0: 16. */
int xs_write_result_sections(const char* path, uint64_t n, uint64_t num_docs, const void* hits, int hit_bytes,
                             const uint64_t* num_kmers, const char* ids_json, const uint64_t* ids_off,
                             const char* labels_json, const uint64_t* labels_off, const uint8_t* doc_mask,
                             const uint64_t* total_hits, uint64_t total_kmers, const uint32_t* total_order_row,
                             int threads);

/* ---- Packed read ids (ASCII only; a byte >= 0x80 is XS_ERR_ARG and the caller
 * falls back to Python).  xs_ids_json_quote: json.dumps(id) of every id (the
 * "hits"/"scores"/"num_kmers" keys ModelResult.save writes, result.py:191-202),
 * packed with n+1 offsets; out_cap >= 6 * offs[n] + 2 * n.
 * xs_ids_has_duplicates: whether two ids are equal (the reference's hits dict
 * keeps the last record of a repeated id, probabilistic_filter_model.py:310). */
int xs_ids_json_quote(const char* buf, const uint64_t* offs, uint64_t n, char* out, uint64_t out_cap,
                      uint64_t* out_offs);
int xs_ids_has_duplicates(const char* buf, const uint64_t* offs, uint64_t n, int* has_dup);
/* out[2i], out[2i+1] = XXH64 of id i with seeds 0 and 0x27D4EB2F165667C5: the
 * 128-bit key by which the ranks of a read-sharded job find ids repeated
 * across their shards (the reference keeps the last record of a repeated id,
 * probabilistic_filter_model.py:310, and sums totals over that dict,
 * result.py:76-90).  Any bytes (not only ASCII). */
int xs_ids_hash128(const char* buf, const uint64_t* offs, uint64_t n, uint64_t* out);
/* out[i] = 1 if keys[i] is one of the m values of `set`, else 0: the owner
 * rank of a read-sharded job finding the records whose key half another
 * record shares (the candidates of a repeated id), in one pass over n keys
 * with a hash set of the (few) shared values.  set may hold repeats. */
int xs_u64_member_mask(const uint64_t* keys, uint64_t n, const uint64_t* set, uint64_t m, uint8_t* out);

/* ---- FASTA/FASTQ reader (host; replaces Bio.SeqIO.parse via
 * get_record_iterator, src/xspect/file_io.py:47-79, on the predict path
 * probabilistic_filter_model.py:316-330).  Records come out packed the way
 * xs_query takes them.  Semantics: see xspect2_amd/csrc/xs_fastx.cpp. */
#define XS_FASTX_FASTA 1
#define XS_FASTX_FASTQ 2
#define XS_FASTX_PINNED 1 /* flag: batch sequence/offset buffers in pinned host memory */

typedef struct xs_fastx xs_fastx;

typedef struct xs_fastx_batch {
    uint64_t n;                  /* records in this batch (0: end of file) */
    uint64_t seq_bytes;          /* bytes of seqs */
    const char* seqs;            /* record r = seqs[offsets[r] .. offsets[r+1]) */
    const uint64_t* offsets;     /* n+1 entries, offsets[0] = 0 */
    const char* ids;             /* record ids (first header token), packed */
    const uint64_t* id_offsets;  /* n+1 entries */
    uint64_t text_offset;        /* file offset parsed up to */
    uint64_t text_bytes;         /* end offset of the reader's text (file size, or its part's end) */
    const char* descs;           /* record titles (header line minus '>'/'@', right-stripped) */
    const uint64_t* desc_offsets;/* n+1 entries */
} xs_fastx_batch;

/* threads <= 0: up to 16.  The file is memory-mapped until xs_fastx_close. */
int xs_fastx_open(const char* path, int format, int threads, int flags, xs_fastx** out);
/* Part `part` of `parts` of the file, for one rank of a read-sharded job
 * (the reference reads the whole file in one
 * process, file_io.py:47-79): the reader yields only the records whose first
 * byte lies in [cut(part), cut(part+1)), cut(i) being the first record start at
 * or after file_size*i/parts.  The parts' records, concatenated in part order,
 * are exactly the file's records.  Each rank maps the file and parses its own
 * slice only.  xs_fastx_open(...) = xs_fastx_open_range(..., 0, 1, ...). */
int xs_fastx_open_range(const char* path, int format, int threads, int flags, uint32_t part, uint32_t parts,
                        xs_fastx** out);
/* Parse the next batch: about max_text_bytes of file text, cut at a record
 * start (one record at least).  Batches ramp up: for budgets of 64 MiB or
 * more, the reader's k-th window takes at most 32 MiB << k, so a pipeline's
 * first probe starts early.  The batch's buffers stay valid until the
 * SECOND following call, so batch i can be probed while batch i+1 is parsed.
 * Malformed records return XS_ERR_FORMAT with Biopython's message. */
int xs_fastx_next(xs_fastx* reader, uint64_t max_text_bytes, xs_fastx_batch* out);
void xs_fastx_close(xs_fastx* reader);

/* Device mode of the same reader (SURVEY.md §8 f1 on the GPU): each window of
 * text — cut exactly as xs_fastx_next cuts it — is copied into pinned memory
 * by host threads and on to HBM, and its records are found on `device`
 * (xs_fastx_dev.hip).  The next window's text is loaded while the caller works
 * on the returned batch.  A window outside the device rules (wrapped FASTQ,
 * blank lines between FASTQ records, empty FASTQ sequences, ' ' or '\r' inside
 * FASTA sequence lines, malformed records) is parsed by the host parser, so
 * batches, ids, titles and error messages equal xs_fastx_next's. */
typedef struct xs_fastx_dbatch {
    uint64_t n;                  /* records in this batch (0: end of the text) */
    uint64_t seq_bytes;          /* bytes of seqs */
    const void* seqs;            /* DEVICE: record r = seqs[offsets[r] .. offsets[r+1]), 64 zero bytes past the end */
    const uint64_t* offsets;     /* DEVICE: n+1 entries, offsets[0] = 0 */
    const uint64_t* host_offsets;/* host: the same n+1 offsets */
    uint64_t max_len;            /* longest record of the batch */
    const char* ids;             /* host: record ids (first header token), packed */
    const uint64_t* id_offsets;  /* host: n+1 entries */
    const char* descs;           /* host: record titles */
    const uint64_t* desc_offsets;/* host: n+1 entries */
    uint64_t text_offset;        /* file offset parsed up to */
    uint64_t text_bytes;         /* end offset of the reader's text */
    int parsed_on_device;        /* 0: this window went through the host parser */
    void* host_ready;            /* the host arrays (host_offsets, ids, descs and their offsets) are
                                    complete once this event has; NULL: already complete.
                                    Wait with xs_fastx_wait_host before reading them */
} xs_fastx_dbatch;

/* As xs_fastx_open_range, for xs_fastx_next_device on `device`. */
int xs_fastx_open_device(const char* path, int format, int threads, int device, uint32_t part, uint32_t parts,
                         xs_fastx** out);
/* Next batch, complete on the device when this returns.  Buffers stay valid
 * until the SECOND following call.  Errors as xs_fastx_next. */
int xs_fastx_next_device(xs_fastx* reader, uint64_t max_text_bytes, xs_fastx_dbatch* out);
/* Block until a device batch's host arrays have landed (their D2H copies run
 * behind the caller's probe of the batch, whose device data is complete when
 * xs_fastx_next_device returns). */
int xs_fastx_wait_host(const xs_fastx_dbatch* batch);

/* Write records as Bio.SeqIO.write(record, fh, "fasta") does (the genus
 * filter's output, src/xspect/file_io.py:166-191): ">" title, then the
 * sequence in lines of `width` (60) characters.  Records r = index[i] for
 * i < n (index NULL: r = i) of a packed batch (seqs/offsets, titles/desc_offs,
 * e.g. an xs_fastx_batch).  append = 0 truncates the file first. */
int xs_write_fasta(const char* path, int append, const char* seqs, const uint64_t* offsets,
                   const char* descs, const uint64_t* desc_offsets, const uint32_t* index, uint64_t n,
                   uint32_t width);

#ifdef __cplusplus
}
#endif
#endif /* XSPECT_HIP_H */
