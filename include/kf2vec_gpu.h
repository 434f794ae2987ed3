/*
 * kf2vec_gpu.h -- C-ABI of the MI355X (gfx950) k-mer frequency-vector builder.
 *
 * Drop-in boundary for kf2vec's `get_frequencies` hot path
 * (reference kf2vec/main.py:250-373).  The reference crosses a PROCESS boundary
 * there: it runs the external C++ counter Jellyfish twice per genome
 *     jellyfish count -m K -s 100M -t P -C <in> -o <x>.jf     (main.py:309-311)
 *     jellyfish dump -c <x>.jf_0 > <x>.dump                    (main.py:317-319)
 * then pandas-joins the dump onto the sorted canonical vocabulary
 * (main.py:278-296, 323-328), normalises (332-342) and formats one `.kf` line
 * (344-357).  This library replaces all of that with device kernels plus a
 * host formatter; the Python host (kf2vecfsw_amd/) binds it with ctypes.
 *
 * Conventions
 *   - plain pointers and sizes only; `d_` pointers are device (HBM) pointers,
 *     e.g. `torch.Tensor.data_ptr()` of a ROCm tensor; the CALLER owns every buffer;
 *   - `stream` is a hipStream_t (NULL = default stream); device entry points only
 *     enqueue work, so they can be graph-captured -- with one exception:
 *     kf_count_batch at k >= 10 allocates the library's workspace on first use
 *     and grows its piece table (a device sync) when n_genomes exceeds every
 *     earlier call; kf_workspace_reserve() does both up front;
 *   - return 0 on success, a negative KF_E* code on failure; the message is in
 *     kf_last_error() (thread-local).  Errors are never silent (deliberate
 *     deviation from main.py:309-311, which discards Jellyfish's stderr/status).
 *
 * Internal 2-bit base code ("kf code"): A=0 C=1 T=2 G=3, i.e. ((ascii >> 1) & 3)
 * for ACGTacgt; complement = code ^ 2.  A k-mer code has its first base in the
 * most significant pair.  Columns (bins) are the rank of the canonical k-mer in
 * the lexicographically sorted canonical vocabulary -- the order of the
 * reference's vocab files (kf2vec/data/) and hence of every `.kf` line.
 */
#ifndef KF2VEC_GPU_H
#define KF2VEC_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KF_ABI_VERSION 1

#define KF_OK 0
#define KF_EINVAL (-1)   /* bad argument (k out of range, null pointer, ...) */
#define KF_EHIP (-2)     /* HIP runtime error */
#define KF_ERANGE (-3)   /* output buffer too small / size overflow */
#define KF_EFORMAT (-4)  /* unparseable input */

#define KF_MIN_K 2
#define KF_MAX_K 12      /* dense device kernels; the CLI accepts 3..11 */
#define KF_SPARSE_MAX_K 31  /* kf_sparse_count (get_kmers, main.py:81-82) */

/* kf_count_batch flags */
#define KF_ACCUMULATE 1u /* do not zero d_counts / d_totals first */

/* input formats */
#define KF_FMT_AUTO 0    /* sniff: first byte '@' -> FASTQ, else FASTA */
#define KF_FMT_FASTA 1
#define KF_FMT_FASTQ 2

int kf_abi_version(void);
const char* kf_last_error(void);

/* Number of bins (= lines of the reference vocab file for k, main.py:278-296):
 * 4^k/2 for odd k, (4^k + 4^(k/2))/2 for even k.  0 if k is out of range. */
uint64_t kf_num_bins(int k);

/* Bin tables for k (replaces the vocab file read, main.py:278-296, and the
 * dump->vocab left-merge, main.py:323-328):
 *   code2col[4^k] : kf code of ANY k-mer -> column of its canonical class
 *   col2rep[nbins]: column -> the kf code the device kernels count it under
 *                   (min(code, revcomp(code)) in kf-code order)
 * Either pointer may be NULL.  *nbins receives kf_num_bins(k). */
int kf_tables(int k, uint32_t* code2col, uint32_t* col2rep, uint64_t* nbins);

/* Sorted canonical vocabulary as text, "KMER\n" per line (byte-identical to the
 * reference's kf2vec/data files for k=3..9).  cap >= nbins*(k+1). */
int kf_vocab_text(int k, char* out, uint64_t cap, uint64_t* written);

/* Record index of one FASTA/FASTQ buffer: the byte ranges that are NOT sequence
 * (FASTA header lines; FASTQ '@' header, '+' and quality lines), as sorted,
 * disjoint [start, end) pairs offset by `base` (the buffer's position inside the
 * device batch).  Newlines between sequence lines are not excluded: the device
 * kernel skips them, so k-mers span line breaks but never records.
 * out_iv holds cap_pairs pairs; on KF_ERANGE *n_pairs is the count needed. */
int kf_index_records(const uint8_t* bytes, uint64_t len, int fmt, uint64_t base,
                     uint64_t* out_iv, uint64_t cap_pairs, uint64_t* n_pairs,
                     int* fmt_detected);

/* Read n files into one host buffer (replaces the per-file open/read that the
 * reference leaves to Jellyfish, main.py:309-311): file i (sizes[i] bytes,
 * checked against the file) goes to dst + off[i], and the bytes
 * [off[i] + sizes[i], off[i+1]) are set to '\n' (transparent padding).  The reads
 * are cut into pieces of at most `piece` bytes (pread) shared by n_threads native
 * threads, so a few large files still keep every thread reading; no Python (or
 * its interpreter lock) runs per piece.  KF_EINVAL on an unreadable or
 * resized file (the message names it). */
int kf_read_files(const char* const* paths, int32_t n, const uint64_t* sizes, const uint64_t* off,
                  uint8_t* dst, uint64_t piece, int n_threads);

/* The FASTA record index of a batch resident in HBM (what kf_index_records finds
 * per file, found on the device so the host only copies the files): the header
 * lines -- a line starting with '>' at a genome start or after '\n', up to its
 * '\n' or the genome end -- as sorted [start, end) pairs d_excl[2i], d_excl[2i+1]
 * (absolute positions; adjacent header lines stay separate pairs, which the
 * count kernels treat alike).  *d_n_pairs (device) receives the number of
 * header lines; only the first cap_pairs are written, so a caller reads it back
 * and runs again with a larger table if it was exceeded.  batch_bytes = goff[n];
 * d_scratch >= ceil(batch_bytes / 4096) + 1 words.  FASTA only (FASTQ needs
 * kf_index_records' per-file state).  Asynchronous on `stream`. */
int kf_index_fasta(const uint8_t* d_bytes, const uint64_t* d_goff, int32_t n_genomes,
                   uint64_t batch_bytes, uint64_t* d_excl, uint64_t cap_pairs,
                   uint64_t* d_n_pairs, uint32_t* d_scratch, uint64_t scratch_words, void* stream);

/* Count canonical k-mers of a batch of genomes already resident in HBM
 * (replaces `jellyfish count -C` + `jellyfish dump -c`, main.py:309-323).
 *   d_bytes    : batch bytes, 16-byte aligned; genome g is
 *                d_bytes[d_goff[g], d_goff[g+1]); the allocation must be readable
 *                up to d_goff[n] rounded up to 16 bytes (vector loads)
 *   d_goff     : n_genomes+1 non-decreasing offsets (device)
 *   d_excl     : 2*n_excl sorted disjoint [start,end) pairs (device) from
 *                kf_index_records, positions absolute in d_bytes (may be NULL if 0)
 *   d_code2col, d_col2rep : kf_tables(k) uploaded to the device
 *   d_counts   : n_genomes x nbins uint32 (column order), zeroed first unless
 *                flags & KF_ACCUMULATE
 *   d_totals   : n_genomes uint64, number of k-mers counted per genome
 * Asynchronous on `stream`.  For k >= 10 the library counts through a device
 * workspace (about 9 GB on a 256-CU device: 2 bytes of sorted records per byte
 * of the 8 MiB genome piece each CU holds, in two slots for the staggered
 * phases) plus a piece table of n_genomes+1 words, kept until
 * kf_workspace_release().  Both are allocated on first use;
 * the piece table is re-allocated behind a hipDeviceSynchronize() when
 * n_genomes exceeds its capacity (it grows at least 2x).  Call
 * kf_workspace_reserve() first to keep every kf_count_batch asynchronous and
 * allocation-free.  Launches on different streams of one device that use the
 * workspace are ordered by the library. */
int kf_count_batch(const uint8_t* d_bytes, const uint64_t* d_goff, int32_t n_genomes,
                   const uint64_t* d_excl, uint64_t n_excl,
                   const uint32_t* d_code2col, const uint32_t* d_col2rep, int k,
                   uint32_t* d_counts, uint64_t* d_totals, uint32_t flags, void* stream);

/* Allocate up front, on the current device, everything kf_count_batch(k, n)
 * needs for any n <= max_genomes: the k >= 10 bucket tables, workspace and
 * piece table, and the kernel attributes of k.  Afterwards such calls neither
 * allocate nor synchronise.  Synchronous; may be called again with a larger
 * max_genomes. */
int kf_workspace_reserve(int k, int32_t max_genomes);

/* Grid the count kernel will use on the current device for k (workgroups,
 * threads per workgroup, dynamic LDS bytes); for roofline accounting.
 * Kernel choice: k <= 7 the pair kernel K1x (k1x_kernel<k>: (k+1)-mer pairs
 * plus single k-mers in LDS), k = 8 its single-pass form (k1x_kernel<8>),
 * k = 9 its byte-counter form (k1x_kernel<9>: all 131,072 canonical classes
 * as u8 LDS counters, carries corrected exactly from the adds' returns), k >= 10
 * the two-phase bucket kernels (bucket_kernel<k>).
 * No environment variable changes the choice in the product library. */
int kf_count_launch_info(int k, int* grid, int* block, int* lds_bytes);

/* ---- get_kmers at any k = 2..31 (replaces `jellyfish count -m K -C` +
 * `jellyfish dump -c -t` of main.py:133-160, which keep the PRESENT canonical
 * k-mers only).  For every genome of a batch laid out as for kf_count_batch:
 * its distinct canonical k-mers in ascending standard 2-bit code (A0 C1 G2 T3,
 * first base most significant: lexicographic order of the k-mer strings, the
 * order of the vocab files) and their counts.  Same input semantics as
 * kf_count_batch.  Genome g's results are d_keys[goff[g] + i] and
 * d_counts[goff[g] + i] for i < d_nuniq[g] (a genome has at most goff[g+1] -
 * goff[g] distinct k-mers, so both arrays hold batch_bytes = goff[n] entries).
 * The device counts each genome's keys per bucket (their top min(10, 2k)
 * bits), scatters every window's key once into its bucket (decoupled
 * look-back per bucket), packs whole buckets into chunks of <= 16,384 keys
 * (12,288 for k <= 16) and
 * sorts each chunk in LDS (10-bit MSD passes plus a fix-up of runs of equal
 * top bits); buckets larger than a chunk are sorted by LSD passes in an
 * overflow area.  Then run-length encoding.  d_work must hold
 * kf_sparse_workspace_bytes(k, batch_bytes, n_genomes) bytes: two key areas of
 * 4 (k <= 16) or 8 B per input byte plus ~1 B per byte of tables, so with the
 * outputs a call needs ~21 (k <= 16) or ~29 device bytes per input byte.  batch_bytes < 2^32 and d_bytes
 * 16-byte aligned (KF_EINVAL otherwise, as kf_count_batch).
 * Asynchronous on `stream`, no allocation, no host synchronisation.  The
 * offsets are checked on the device: if d_goff decreases or d_goff[n] >
 * batch_bytes, nothing is read or written and every d_nuniq[g] is UINT64_MAX.
 * The sorted keys are checked on the device too: a genome whose keys are not
 * in order, or a sort pass whose tile-to-tile prefix exchange (decoupled
 * look-back) stalled past its bound, makes every d_nuniq[g] UINT64_MAX - 1
 * (fail loudly, never silently or by hanging). */
uint64_t kf_sparse_workspace_bytes(int k, uint64_t batch_bytes, int32_t n_genomes);
int kf_sparse_count(const uint8_t* d_bytes, const uint64_t* d_goff, int32_t n_genomes,
                    uint64_t batch_bytes, const uint64_t* d_excl, uint64_t n_excl, int k,
                    void* d_work, uint64_t work_bytes, uint64_t* d_keys, uint32_t* d_counts,
                    uint64_t* d_nuniq, void* stream);

/* Hash of the sources this library was built from (csrc/ + this header, as
 * kf2vecfsw_amd/build.py computes it): 16 hex digits, with a "+<tag>" suffix for
 * profiling builds.  The Python binding refuses a library whose id differs from
 * the sources next to it. */
const char* kf_build_id(void);

/* Measurement aid (bench.py): read d_bytes[0, n) with the fastest read pattern
 * measured on gfx950 (3 KiB blocks dealt grid-stride over the waves, coalesced
 * 16-byte lanes, four blocks in flight per wave) and XOR-fold it into *d_out
 * (device).  Time it to get the practical HBM read ceiling.  Needs n rounded up
 * to 16 readable. */
int kf_stream_probe(const uint8_t* d_bytes, uint64_t n, uint32_t* d_out, void* stream);

/* Free the large-k workspace and tables of the current device (synchronises the
 * device).  The next large-k kf_count_batch allocates them again. */
int kf_workspace_release(void);

/* Synthetic FASTA generator on the device (benchmark/test input; spec in
 * DESIGN.md "Synthetic genomes"): genome i has id g = g0 + i*g_stride (so a rank
 * of a round-robin shard passes g0 = rank, g_stride = world) and seed seed0 + g;
 * it is written to d_bytes[d_goff[i], d_goff[i+1]) as ">syn_<g>\n" + seq_len
 * bases in `width`-column lines + '\n' padding.  d_goff must be 16-aligned. */
int kf_synth_fasta(uint8_t* d_bytes, const uint64_t* d_goff, int32_t n_genomes,
                   int64_t g0, int64_t g_stride, uint64_t seed0, uint64_t seq_len,
                   int width, uint64_t n_period, void* stream);

/* Host-side layout for kf_synth_fasta: genome sizes rounded up to `align`. */
uint64_t kf_synth_genome_bytes(int64_t g, uint64_t seq_len, int width, uint64_t align);
uint64_t kf_synth_header_len(int64_t g);

/* One `.kf` line, byte-identical to main.py:331-357:
 *   "<name>," + ",".join(str(v)) + "\n"
 * with v = counts (+0.5 if pseudocount) (/ sum unless raw_cnt), float64,
 * printed like Python repr(float); raw counts with no empty bin print as
 * integers (pandas keeps int64 when the left-merge introduces no NaN), and so
 * do the zeros of a genome with no k-mer at all (an empty dump).
 * On KF_ERANGE *written is the size needed. */
int kf_format_kf(const char* name, const uint32_t* counts, uint64_t nbins,
                 int pseudocount, int raw_cnt, char* out, uint64_t cap, uint64_t* written);

/* Format and write many `.kf` files with n_threads host threads:
 * file i = dir + "/" + names[i] + ".kf", counts row i of counts[n x nbins]. */
int kf_write_kf_files(const char* dir, const char* const* names, int32_t n,
                      const uint32_t* counts, uint64_t nbins, int pseudocount,
                      int raw_cnt, int n_threads);

/* get_chunks (main.py:869-915): the rows of many windows in ONE file, in order:
 * path = the file, row i = names[i] + counts row i, formatted by n_threads host
 * threads (as kf_format_kf) and written in row order. */
int kf_write_kf_rows(const char* path, const char* const* names, int32_t n,
                     const uint32_t* counts, uint64_t nbins, int pseudocount,
                     int raw_cnt, int n_threads);

/* get_chunks, many genomes at once: segment g is rows [seg_row0[g],
 * seg_row0[g+1]) of counts (seg_row0[0] = 0, non-decreasing), written in row
 * order to paths[g] (distinct), appended if seg_append && seg_append[g] (a genome
 * whose windows span several count launches), else truncated.  Row i is named
 * names[i], or, with names == NULL, prefixes[row_prefix[i]] followed by
 * "<s+1>-<s+win_len>" for s = row_start[i] (the window names of main.py:905-915).
 * n_threads host threads format rows into private arenas and write each
 * segment's file once its rows are formatted (formatting and writing overlap). */
int kf_write_kf_segments(int32_t n_seg, const char* const* paths, const int32_t* seg_row0,
                         const uint8_t* seg_append, const char* const* names,
                         const char* const* prefixes, const uint32_t* row_prefix,
                         const uint64_t* row_start, uint32_t win_len,
                         const uint32_t* counts, uint64_t nbins, int pseudocount,
                         int raw_cnt, int n_threads);

/* kf_write_kf_segments for u16 counts (a get_chunks window of 10 kbp has every
 * count below 2^16, so its rows cross PCIe at half the bytes). */
int kf_write_kf_segments16(int32_t n_seg, const char* const* paths, const int32_t* seg_row0,
                           const uint8_t* seg_append, const char* const* names,
                           const char* const* prefixes, const uint32_t* row_prefix,
                           const uint64_t* row_start, uint32_t win_len,
                           const uint16_t* counts, uint64_t nbins, int pseudocount,
                           int raw_cnt, int n_threads);

/* ---- get_chunks device pre-pass (replaces seqtk seq -l 0 | awk N-collapse |
 * seqkit seq -g -m, main.py:726-760).  d_seq holds n_rec sorted, disjoint
 * [start, end) byte ranges of record sequences (the bytes between a header's
 * '\n' and the next header).  Writes each record's processed sequence --
 * newlines and line-end '\r' dropped, the gap letters "- \t." dropped, runs of
 * N / n / '|' (awk runs before seqkit: gap letters split a run) collapsed to
 * one 'N' -- back to back into d_out (>= len bytes) and its [start, end) into
 * d_out_se[2r], d_out_se[2r+1].  d_scratch: >= ceil(len / 4096) + 1 words.
 * len < 2^32 (KF_EINVAL otherwise).  Asynchronous on `stream`. */
int kf_chunk_compact(const uint8_t* d_bytes, uint64_t len, const uint64_t* d_seq, int32_t n_rec,
                     uint8_t* d_out, uint64_t* d_out_se, uint32_t* d_scratch, uint64_t scratch_words,
                     void* stream);

/* Window w = d_src[d_win_src[w], + win_len) to d_dst[w * win_len, + win_len)
 * (the seqkit sliding windows of main.py:813-824, laid out for kf_count_batch). */
int kf_chunk_gather(const uint8_t* d_src, const uint64_t* d_win_src, int32_t n_win, uint32_t win_len,
                    uint8_t* d_dst, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* KF2VEC_GPU_H */
