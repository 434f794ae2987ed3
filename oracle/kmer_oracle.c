/*
 * kmer_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C CPU restatement of the counting half of kf2vec's `get_frequencies`
 * (reference: kf2vec/main.py:250-373).  The reference does not count k-mers
 * itself: it shells out to the third-party C++ counter Jellyfish
 * (`jellyfish count -m K -s 100M -t P -C <in> -o <jf>` then `jellyfish dump -c`,
 * main.py:309-319; pinned `kmer-jellyfish=1.1.12`, kf2vec_env.yml:35, NOT vendored
 * in /root/reference and not installed in this image).  What follows restates the
 * published Jellyfish semantics that kf2vec relies on:
 *
 *   - canonical k-mers (`-C`): a k-mer and its reverse complement are one bin,
 *     represented by the lexicographically smaller string over A<C<G<T;
 *   - FASTA: a line starting with '>' is a header and ends the previous record;
 *     k-mers span line breaks inside a record but never a record boundary;
 *   - any byte that is not A/C/G/T (either case) breaks the k-mer (N, IUPAC, '\r');
 *   - FASTQ: '@' header, sequence lines up to a '+' line, then quality lines
 *     whose total length equals the sequence length; only sequence bytes count;
 *   - exact counts; `jellyfish dump -c` + the pandas left-merge onto the sorted
 *     vocabulary (main.py:323-328) is the same as indexing counts by the rank of
 *     the canonical k-mer in sorted order (vocab files under kf2vec/data/).
 *
 * Pinning: tests/test_oracle_golden.py reproduces the 7 committed toy `.kf`
 * files (normalised) and the 3 committed chunk `.kf` files (raw counts)
 * byte-for-byte from their `.fna` through this file + oracle/kf_oracle.py.
 * Policies the fixtures do not pin (lowercase, '\r', FASTQ) are documented in
 * DESIGN.md section "Input policy".
 *
 * Build: see oracle/Makefile (gcc -O2 -fopenmp -shared).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORACLE_MAX_K 13

/* Standard 2-bit code, lexicographic order: A0 C1 G2 T3; -1 = breaks the k-mer. */
static int std_code(uint8_t c) {
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return -1;
    }
}

static uint64_t revcomp_std(uint64_t x, int k) {
    uint64_t r = 0;
    for (int i = 0; i < k; ++i) { r = (r << 2) | (3u - (x & 3u)); x >>= 2; }
    return r;
}

/* Number of canonical bins = number of lines of the vocab file (main.py:278-296). */
uint64_t oracle_nbins(int k) {
    if (k < 1 || k > ORACLE_MAX_K) return 0;
    uint64_t n = 1ull << (2 * k);
    uint64_t pal = (k % 2 == 0) ? (1ull << k) : 0; /* 4^(k/2) palindromes for even k */
    return (n + pal) / 2;
}

/* rank[std_code] = column of the canonical class in the sorted vocab. */
int oracle_rank_std(int k, uint32_t* rank) {
    if (k < 1 || k > ORACLE_MAX_K) return -1;
    uint64_t n = 1ull << (2 * k);
    uint32_t next = 0;
    /* ascending numeric order of std codes == lexicographic string order */
    for (uint64_t x = 0; x < n; ++x) {
        uint64_t r = revcomp_std(x, k);
        if (x <= r) rank[x] = next++;
    }
    for (uint64_t x = 0; x < n; ++x) {
        uint64_t r = revcomp_std(x, k);
        if (r < x) rank[x] = rank[r];
    }
    return 0;
}

/* Writes the sorted canonical vocabulary ("KMER\n" lines) into out (nbins*(k+1) bytes). */
int oracle_vocab(int k, char* out) {
    if (k < 1 || k > ORACLE_MAX_K) return -1;
    static const char B[4] = {'A', 'C', 'G', 'T'};
    uint64_t n = 1ull << (2 * k);
    char* p = out;
    for (uint64_t x = 0; x < n; ++x) {
        if (x > revcomp_std(x, k)) continue;
        for (int i = k - 1; i >= 0; --i) *p++ = B[(x >> (2 * i)) & 3];
        *p++ = '\n';
    }
    return 0;
}

typedef struct {
    int k;
    uint64_t mask, fw, rc, len;
    const uint32_t* rank;
    uint32_t* counts;
    uint64_t total;
    uint64_t* keys;      /* sparse mode (oracle_sparse_count): canonical codes appended here */
} kstate;

static inline void ks_reset(kstate* s) { s->len = 0; }

static inline void ks_push(kstate* s, uint8_t c) {
    int code = std_code(c);
    if (code < 0) { s->len = 0; return; }
    s->fw = ((s->fw << 2) | (uint64_t)code) & s->mask;
    s->rc = (s->rc >> 2) | ((uint64_t)(3 - code) << (2 * s->k - 2));
    if (++s->len >= (uint64_t)s->k) {
        uint64_t canon = s->fw < s->rc ? s->fw : s->rc;
        if (s->keys) s->keys[s->total] = canon;
        else s->counts[s->rank[canon]] += 1;
        s->total += 1;
    }
}

/* FASTA scan (main.py:309-311 via Jellyfish): '>' at line start opens a header
 * line (record boundary), '\n' is transparent inside a record. */
static void scan_fasta(kstate* s, const uint8_t* b, uint64_t n) {
    int at_line_start = 1, in_header = 0;
    for (uint64_t i = 0; i < n; ++i) {
        uint8_t c = b[i];
        if (at_line_start && c == '>') { in_header = 1; ks_reset(s); }
        at_line_start = (c == '\n');
        if (c == '\n') { in_header = 0; continue; }
        if (in_header) continue;
        ks_push(s, c);
    }
}

/* FASTQ scan: '@' header line, sequence lines until a line starting with '+',
 * then quality lines until their total length reaches the sequence length. */
static void scan_fastq(kstate* s, const uint8_t* b, uint64_t n) {
    enum { HDR, SEQ, QUAL } st = HDR;
    uint64_t seqlen = 0, qlen = 0, i = 0;
    while (i < n) {
        uint64_t j = i;
        while (j < n && b[j] != '\n') ++j;       /* line = b[i, j) */
        uint64_t L = j - i;
        if (st == HDR) {
            if (L > 0 && b[i] == '@') { st = SEQ; seqlen = 0; ks_reset(s); }
        } else if (st == SEQ) {
            if (L > 0 && b[i] == '+') { st = QUAL; qlen = 0; ks_reset(s); if (seqlen == 0) st = HDR; }
            else { for (uint64_t t = i; t < j; ++t) ks_push(s, b[t]); seqlen += L; }
        } else {
            qlen += L;
            if (qlen >= seqlen) st = HDR;
        }
        i = j + 1;
    }
}

/* fmt: 0 = sniff (first byte '@' -> FASTQ), 1 = FASTA, 2 = FASTQ */
static int sniff(const uint8_t* b, uint64_t n, int fmt) {
    if (fmt) return fmt;
    return (n > 0 && b[0] == '@') ? 2 : 1;
}

/* Counts every canonical k-mer of one genome into counts[nbins] (rank order),
 * adds; total receives the number of k-mers counted (sum of counts). */
int oracle_count(const uint8_t* bytes, uint64_t len, int k, int fmt,
                 const uint32_t* rank_std, uint32_t* counts, uint64_t* total) {
    if (k < 1 || k > ORACLE_MAX_K) return -1;
    kstate s;
    memset(&s, 0, sizeof s);
    s.k = k;
    s.mask = (k == 32) ? ~0ull : ((1ull << (2 * k)) - 1);
    s.rank = rank_std;
    s.counts = counts;
    if (sniff(bytes, len, fmt) == 2) scan_fastq(&s, bytes, len);
    else scan_fasta(&s, bytes, len);
    *total = s.total;
    return 0;
}

/* Many genomes (concatenated; genome g = bytes[off[g], off[g+1])), OpenMP over
 * genomes.  Used as the CPU baseline leg of bench.py (kind "port"). */
int oracle_count_many(const uint8_t* bytes, const uint64_t* off, int n_genomes, int k, int fmt,
                      const uint32_t* rank_std, uint32_t* counts, uint64_t* totals, int n_threads) {
    uint64_t nb = oracle_nbins(k);
    if (!nb) return -1;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int g = 0; g < n_genomes; ++g) {
        memset(counts + (uint64_t)g * nb, 0, nb * sizeof(uint32_t));
        oracle_count(bytes + off[g], off[g + 1] - off[g], k, fmt, rank_std,
                     counts + (uint64_t)g * nb, totals + g);
    }
    return 0;
}

/* FASTA scan of bytes [from, n) that counts only the k-mers ending at bytes in
 * [a, e).  `from` must be a line start (or 0); the bytes [from, a) only rebuild
 * the k-mer context and the header state, exactly as scan_fasta would have them
 * at a (a record boundary or non-ACGT byte in between resets it the same way). */
static void scan_fasta_part(kstate* s, const uint8_t* b, uint64_t from, uint64_t a, uint64_t e) {
    int at_line_start = 1, in_header = 0;
    for (uint64_t i = from; i < e; ++i) {
        uint8_t c = b[i];
        if (at_line_start && c == '>') { in_header = 1; ks_reset(s); }
        at_line_start = (c == '\n');
        if (c == '\n') { in_header = 0; continue; }
        if (in_header) continue;
        if (i < a) {   /* context only: push without counting */
            int code = std_code(c);
            if (code < 0) { s->len = 0; continue; }
            s->fw = ((s->fw << 2) | (uint64_t)code) & s->mask;
            s->rc = (s->rc >> 2) | ((uint64_t)(3 - code) << (2 * s->k - 2));
            ++s->len;
            continue;
        }
        ks_push(s, c);
    }
}

/* As oracle_count_many, with every FASTA genome cut into parts of about
 * `part_bytes` bytes and OpenMP over all (genome, part) pairs, so that the
 * threads are not capped by the number of genomes (bench.py's CPU baseline on
 * the GPU box's nproc threads).  Part j of a genome counts the k-mers whose
 * last base lies in its byte range; it rebuilds its context by scanning from
 * the start of the line holding the k-th non-newline byte before the range (a
 * FASTA line start is a state-free restart point).  FASTQ genomes are one part each.
 * Each part counts into a thread-private row, added to the genome's row under
 * an atomic per non-zero bin. */
int oracle_count_many_parts(const uint8_t* bytes, const uint64_t* off, int n_genomes, int k, int fmt,
                            const uint32_t* rank_std, uint32_t* counts, uint64_t* totals, int n_threads,
                            uint64_t part_bytes) {
    uint64_t nb = oracle_nbins(k);
    if (!nb || part_bytes == 0) return -1;
    uint64_t* first = (uint64_t*)malloc(((size_t)n_genomes + 1) * sizeof(uint64_t));
    if (!first) return -1;
    first[0] = 0;
    for (int g = 0; g < n_genomes; ++g) {
        const uint64_t len = off[g + 1] - off[g];
        const int fq = sniff(bytes + off[g], len, fmt) == 2;
        const uint64_t np = (fq || len == 0) ? 1 : (len + part_bytes - 1) / part_bytes;
        first[g + 1] = first[g] + np;
        memset(counts + (uint64_t)g * nb, 0, nb * sizeof(uint32_t));
        totals[g] = 0;
    }
    const int64_t ntask = (int64_t)first[n_genomes];
    int rc = 0;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel
#endif
    {
        uint32_t* loc = (uint32_t*)calloc(nb, sizeof(uint32_t));
        if (!loc) {
#ifdef _OPENMP
#pragma omp atomic write
#endif
            rc = -1;
        }
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t t = 0; t < ntask; ++t) {
            if (!loc) continue;
            int g = 0, lo = 0, hi = n_genomes;   /* genome of task t: last g with first[g] <= t */
            while (hi - lo > 1) { int m = (lo + hi) / 2; if (first[m] <= (uint64_t)t) lo = m; else hi = m; }
            g = lo;
            const uint8_t* b = bytes + off[g];
            const uint64_t len = off[g + 1] - off[g], np = first[g + 1] - first[g], j = (uint64_t)t - first[g];
            kstate s;
            memset(&s, 0, sizeof s);
            s.k = k;
            s.mask = (1ull << (2 * k)) - 1;
            s.rank = rank_std;
            s.counts = loc;
            if (np == 1) {
                if (sniff(b, len, fmt) == 2) scan_fastq(&s, b, len);
                else scan_fasta(&s, b, len);
            } else {
                const uint64_t a = len / np * j + (len % np) * j / np;
                const uint64_t e = j + 1 == np ? len : len / np * (j + 1) + (len % np) * (j + 1) / np;
                /* back over k non-newline bytes (k bases of context, or a reset
                 * among them), then to the start of that line */
                uint64_t from = a;
                for (int seen = 0; from > 0 && seen < k;)
                    if (b[--from] != '\n') ++seen;
                while (from > 0 && b[from - 1] != '\n') --from;
                scan_fasta_part(&s, b, from, a, e);
            }
            uint32_t* row = counts + (uint64_t)g * nb;
            for (uint64_t i = 0; i < nb; ++i) {
                if (!loc[i]) continue;
#ifdef _OPENMP
#pragma omp atomic
#endif
                row[i] += loc[i];
                loc[i] = 0;
            }
#ifdef _OPENMP
#pragma omp atomic
#endif
            totals[g] += s.total;
        }
        free(loc);
    }
    free(first);
    return rc;
}

static int cmp_u64(const void* a, const void* b) {
    const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return x < y ? -1 : x > y;
}

/* get_kmers at any k = 1..31 (main.py:133-160: `jellyfish count -C` + `dump -c`
 * keep the PRESENT canonical k-mers): the canonical standard code (A0 C1 G2 T3,
 * the smaller of a k-mer and its reverse complement) of every window, sorted and
 * run-length encoded: keys[i] ascending with counts[i], i < *n_out.  keys and
 * counts hold at least len entries (keys is also the scratch of the sort). */
int oracle_sparse_count(const uint8_t* bytes, uint64_t len, int k, int fmt, uint64_t* keys, uint32_t* counts,
                        uint64_t* n_out) {
    if (k < 1 || k > 31) return -1;
    kstate s;
    memset(&s, 0, sizeof s);
    s.k = k;
    s.mask = (1ull << (2 * k)) - 1;
    s.keys = keys;
    if (sniff(bytes, len, fmt) == 2) scan_fastq(&s, bytes, len);
    else scan_fasta(&s, bytes, len);
    qsort(keys, s.total, sizeof(uint64_t), cmp_u64);
    uint64_t n = 0;
    for (uint64_t i = 0; i < s.total; ++i) {
        if (n && keys[n - 1] == keys[i]) { counts[n - 1] += 1; continue; }
        keys[n] = keys[i];
        counts[n] = 1;
        ++n;
    }
    *n_out = n;
    return 0;
}

/* oracle_sparse_count over many genomes (genome g = bytes[off[g], off[g+1])),
 * OpenMP over genomes, in the device counter's layout: genome g's present
 * k-mers at keys[off[g] ...] / counts[off[g] ...], their number in nuniq[g]
 * (keys and counts hold off[n] entries).  For the full-size GPU parity test. */
int oracle_sparse_count_many(const uint8_t* bytes, const uint64_t* off, int n_genomes, int k, int fmt,
                             uint64_t* keys, uint32_t* counts, uint64_t* nuniq, int n_threads) {
    if (k < 1 || k > 31) return -1;
    int rc = 0;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int g = 0; g < n_genomes; ++g) {
        if (oracle_sparse_count(bytes + off[g], off[g + 1] - off[g], k, fmt, keys + off[g], counts + off[g],
                                nuniq + g) != 0) {
#ifdef _OPENMP
#pragma omp atomic write
#endif
            rc = -1;
        }
    }
    return rc;
}

int oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ---------------------------------------------------------------------------
 * Synthetic genome generator: bit-identical CPU twin of the device generator
 * kf_synth_fasta (kf2vecfsw_amd/csrc/kf_kernels.hip).  Spec:
 *   key      = splitmix64(seed)
 *   base i   = "ACGT"[(splitmix64(key + (i >> 5)) >> (2*(i & 31))) & 3]
 *   N runs   : block b = i >> 12; h = splitmix64(key ^ 0xA5A5A5A5A5A5A5A5 + b);
 *              if n_period && h % n_period == 0: run [b*4096 + (h>>16)%4096, +1+(h>>32)%100)
 *   layout   : ">syn_<g>\n", bases in lines of `width`, each line '\n'-terminated,
 *              then '\n' padding up to `size` bytes.
 * ------------------------------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

static int in_nrun(uint64_t key, uint64_t i, uint64_t n_period) {
    if (!n_period) return 0;
    uint64_t b = i >> 12;
    for (int d = 0; d < 2; ++d) {
        if (d == 1) { if (b == 0) break; b -= 1; }
        uint64_t h = splitmix64((key ^ 0xA5A5A5A5A5A5A5A5ull) + b);
        if (h % n_period) continue;
        uint64_t st = (b << 12) + ((h >> 16) % 4096), ln = 1 + ((h >> 32) % 100);
        if (i >= st && i < st + ln) return 1;
    }
    return 0;
}

uint64_t oracle_synth_header_len(int64_t g) {
    char tmp[32];
    return (uint64_t)snprintf(tmp, sizeof tmp, ">syn_%lld\n", (long long)g);
}

int oracle_synth_genome(int64_t g, uint64_t seed, uint64_t seq_len, int width, uint64_t n_period,
                        uint8_t* out, uint64_t size) {
    static const char B[4] = {'A', 'C', 'G', 'T'};
    char hdr[32];
    uint64_t h = (uint64_t)snprintf(hdr, sizeof hdr, ">syn_%lld\n", (long long)g);
    uint64_t need = h + seq_len + (seq_len + width - 1) / width;
    if (need > size || width < 1) return -1;
    memcpy(out, hdr, h);
    uint64_t key = splitmix64(seed), p = h;
    for (uint64_t i = 0; i < seq_len; ++i) {
        uint8_t c = B[(splitmix64(key + (i >> 5)) >> (2 * (i & 31))) & 3];
        if (in_nrun(key, i, n_period)) c = 'N';
        out[p++] = c;
        if ((i + 1) % (uint64_t)width == 0 || i + 1 == seq_len) out[p++] = '\n';
    }
    while (p < size) out[p++] = '\n';
    return 0;
}
