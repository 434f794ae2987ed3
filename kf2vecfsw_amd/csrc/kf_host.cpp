// kf_host.cpp -- host half of the kf2vec_gpu C-ABI (include/kf2vec_gpu.h):
// bin tables / vocabulary, FASTA/FASTQ record index, byte-exact `.kf` formatting
// and the parallel `.kf` writer.
#include <emmintrin.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <memory>
#include <charconv>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kf_internal.h"

namespace {
thread_local std::string g_err;

inline uint64_t kf_rc(uint64_t x, int k) {
    // reverse complement in kf code (complement = ^2)
    uint64_t r = 0;
    for (int i = 0; i < k; ++i) {
        r = (r << 2) | ((x & 3u) ^ 2u);
        x >>= 2;
    }
    return r;
}
// kf code (A0 C1 T2 G3) -> lexicographic code (A0 C1 G2 T3), per pair: std = kf ^ (kf >> 1)
inline uint64_t kf_to_std(uint64_t x, int k) {
    const uint64_t lo = 0x5555555555555555ull & ((k >= 32) ? ~0ull : ((1ull << (2 * k)) - 1));
    return x ^ ((x >> 1) & lo);
}
inline uint64_t std_rc(uint64_t x, int k) {
    uint64_t r = 0;
    for (int i = 0; i < k; ++i) {
        r = (r << 2) | (3u - (x & 3u));
        x >>= 2;
    }
    return r;
}
}  // namespace

int kf_fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

extern "C" int kf_abi_version(void) { return KF_ABI_VERSION; }
extern "C" const char* kf_last_error(void) { return g_err.c_str(); }

extern "C" uint64_t kf_num_bins(int k) {
    if (k < 1 || k > 15) return 0;
    const uint64_t n = 1ull << (2 * k);
    const uint64_t pal = (k % 2 == 0) ? (1ull << k) : 0;
    return (n + pal) / 2;
}

// main.py:278-296 (vocab file per k) + main.py:327-328 (left merge onto it).
extern "C" int kf_tables(int k, uint32_t* code2col, uint32_t* col2rep, uint64_t* nbins) {
    if (k < 1 || k > KF_MAX_K) return kf_fail(KF_EINVAL, "k=%d out of range [1, %d]", k, KF_MAX_K);
    const uint64_t n = 1ull << (2 * k);
    // columns: canonical classes in ascending lexicographic (std code) order
    std::vector<uint32_t> std_col(n, 0xFFFFFFFFu);
    uint32_t next = 0;
    for (uint64_t s = 0; s < n; ++s)
        if (s <= std_rc(s, k)) std_col[s] = next++;
    for (uint64_t x = 0; x < n; ++x) {
        const uint64_t s = kf_to_std(x, k);
        const uint64_t c = std::min(s, std_rc(s, k));
        const uint32_t col = std_col[c];
        if (code2col) code2col[x] = col;
        if (col2rep && x <= kf_rc(x, k)) col2rep[col] = (uint32_t)x;   // kernel counts under min(code, rc)
    }
    if (nbins) *nbins = next;
    return KF_OK;
}

extern "C" int kf_vocab_text(int k, char* out, uint64_t cap, uint64_t* written) {
    if (k < 1 || k > KF_MAX_K) return kf_fail(KF_EINVAL, "k=%d out of range", k);
    const uint64_t need = kf_num_bins(k) * (uint64_t)(k + 1);
    if (written) *written = need;
    if (!out || cap < need) return kf_fail(KF_ERANGE, "vocab buffer too small (%llu < %llu)",
                                           (unsigned long long)cap, (unsigned long long)need);
    static const char B[4] = {'A', 'C', 'G', 'T'};
    const uint64_t n = 1ull << (2 * k);
    char* p = out;
    for (uint64_t s = 0; s < n; ++s) {
        if (s > std_rc(s, k)) continue;
        for (int i = k - 1; i >= 0; --i) *p++ = B[(s >> (2 * i)) & 3];
        *p++ = '\n';
    }
    return KF_OK;
}

// ------------------------------------------------------------------ record index
namespace {
struct IvOut {
    uint64_t* out;
    uint64_t cap, n, base, last_e;
    void add(uint64_t s, uint64_t e) {
        if (e <= s) return;
        if (n && s <= last_e + 1) {   // merge (gap of at most the one '\n' between lines)
            last_e = std::max(last_e, e);
            if (out && n <= cap) out[2 * (n - 1) + 1] = last_e + base;
            return;
        }
        if (out && n < cap) {
            out[2 * n] = s + base;
            out[2 * n + 1] = e + base;
        }
        ++n;
        last_e = e;
    }
};

inline uint64_t line_end(const uint8_t* b, uint64_t i, uint64_t len) {
    const void* p = memchr(b + i, '\n', len - i);
    return p ? (uint64_t)((const uint8_t*)p - b) : len;
}
}  // namespace

extern "C" int kf_index_records(const uint8_t* bytes, uint64_t len, int fmt, uint64_t base,
                                uint64_t* out_iv, uint64_t cap_pairs, uint64_t* n_pairs, int* fmt_detected) {
    if (!bytes && len) return kf_fail(KF_EINVAL, "null input");
    if (fmt == KF_FMT_AUTO) fmt = (len > 0 && bytes[0] == '@') ? KF_FMT_FASTQ : KF_FMT_FASTA;
    if (fmt != KF_FMT_FASTA && fmt != KF_FMT_FASTQ) return kf_fail(KF_EINVAL, "unknown format %d", fmt);
    if (fmt_detected) *fmt_detected = fmt;
    IvOut iv{out_iv, cap_pairs, 0, base, 0};
    if (fmt == KF_FMT_FASTA) {
        // header = a line starting with '>' (record boundary), up to its '\n'
        uint64_t i = 0;
        while (i < len) {
            const void* p = memchr(bytes + i, '>', len - i);
            if (!p) break;
            const uint64_t j = (uint64_t)((const uint8_t*)p - bytes);
            if (j == 0 || bytes[j - 1] == '\n') {
                const uint64_t e = line_end(bytes, j, len);
                iv.add(j, e);
                i = e;
            } else {
                i = j + 1;   // mid-line '>' is an ordinary invalid byte (k-mer reset)
            }
        }
    } else {
        // FASTQ: '@' header, sequence lines until '+', quality lines until their
        // length reaches the sequence length (same rules as oracle scan_fastq)
        enum { HDR, SEQ, QUAL } st = HDR;
        uint64_t seqlen = 0, qlen = 0, i = 0;
        while (i < len) {
            const uint64_t j = line_end(bytes, i, len), L = j - i;
            if (st == HDR) {
                iv.add(i, j);
                if (L > 0 && bytes[i] == '@') { st = SEQ; seqlen = 0; }
            } else if (st == SEQ) {
                if (L > 0 && bytes[i] == '+') {
                    iv.add(i, j);
                    st = QUAL;
                    qlen = 0;
                    if (seqlen == 0) st = HDR;
                } else {
                    seqlen += L;
                }
            } else {
                iv.add(i, j);
                qlen += L;
                if (qlen >= seqlen) st = HDR;
            }
            i = j + 1;
        }
    }
    if (n_pairs) *n_pairs = iv.n;
    if (iv.n > cap_pairs) return kf_fail(KF_ERANGE, "record index needs %llu pairs", (unsigned long long)iv.n);
    return KF_OK;
}

// ------------------------------------------------------------------ .kf formatting
namespace {
// Python repr(float) (PyOS_double_to_string mode 'r'): shortest round-trip digits,
// exponent form iff decpt <= -4 or decpt > 16, ".0" appended to integral values.
inline char* fmt_repr(double v, char* p) {
    if (v != v) { memcpy(p, "nan", 3); return p + 3; }
    if (v == 0.0) { memcpy(p, "0.0", 3); return p + 3; }
    if (v < 0) { *p++ = '-'; v = -v; }
    if (v == __builtin_inf()) { memcpy(p, "inf", 3); return p + 3; }
    char tmp[40];
    auto r = std::to_chars(tmp, tmp + sizeof tmp, v, std::chars_format::scientific);
    // tmp = d[.ddd]e(+|-)XX
    char digs[24];
    int nd = 0;
    const char* q = tmp;
    while (q < r.ptr && *q != 'e') {
        if (*q != '.') digs[nd++] = *q;
        ++q;
    }
    int e10 = 0;
    std::from_chars(q + 1 + (q[1] == '+'), r.ptr, e10);
    const int decpt = e10 + 1;
    if (decpt <= -4 || decpt > 16) {
        *p++ = digs[0];
        if (nd > 1) {
            *p++ = '.';
            memcpy(p, digs + 1, nd - 1);
            p += nd - 1;
        }
        *p++ = 'e';
        *p++ = e10 < 0 ? '-' : '+';
        int a = e10 < 0 ? -e10 : e10;
        if (a >= 100) { *p++ = (char)('0' + a / 100); a %= 100; }
        *p++ = (char)('0' + a / 10);
        *p++ = (char)('0' + a % 10);
    } else if (decpt <= 0) {
        *p++ = '0';
        *p++ = '.';
        for (int i = 0; i < -decpt; ++i) *p++ = '0';
        memcpy(p, digs, nd);
        p += nd;
    } else if (decpt >= nd) {
        memcpy(p, digs, nd);
        p += nd;
        for (int i = nd; i < decpt; ++i) *p++ = '0';
        *p++ = '.';
        *p++ = '0';
    } else {
        memcpy(p, digs, decpt);
        p += decpt;
        *p++ = '.';
        memcpy(p, digs + decpt, nd - decpt);
        p += nd - decpt;
    }
    return p;
}

inline char* fmt_u64(uint64_t v, char* p) {
    auto r = std::to_chars(p, p + 24, v);
    return r.ptr;
}

// Small counts are most of a row (a 10 kbp get_chunks window has 8,192 columns
// at k=7, nearly all 0-3).  Single digits go eight columns at a time through SSE2
// (one add per column: "d.0," is the little-endian word 0x2C302E30 + d); the rest
// come from a table built once, each entry with its trailing comma:
//   txt[0][c] = "c,", txt[1][c] = "c.5," (pseudocount), txt[2][c] = "c.0,"
constexpr uint32_t kSmall = 1024;
struct SmallText {
    char txt[3][kSmall][8];
    uint8_t len[3][kSmall];
    SmallText() {
        for (uint32_t c = 0; c < kSmall; ++c) {
            for (int m = 0; m < 3; ++m) {
                char* p = txt[m][c];
                char* e = fmt_u64(c, p);
                if (m == 1) { *e++ = '.'; *e++ = '5'; }
                if (m == 2) { *e++ = '.'; *e++ = '0'; }
                *e++ = ',';
                len[m][c] = (uint8_t)(e - p);
            }
        }
    }
};
const SmallText& small_text() {
    static const SmallText t;
    return t;
}

// eight counts from c (u32 or u16) as two vectors of four u32
inline void load8(const uint32_t* c, __m128i& a, __m128i& b) {
    a = _mm_loadu_si128((const __m128i*)c);
    b = _mm_loadu_si128((const __m128i*)(c + 4));
}
inline void load8(const uint16_t* c, __m128i& a, __m128i& b) {
    const __m128i x = _mm_loadu_si128((const __m128i*)c);
    a = _mm_unpacklo_epi16(x, _mm_setzero_si128());
    b = _mm_unpackhi_epi16(x, _mm_setzero_si128());
}

// columns [0, n) of one raw row, each followed by ','; m as in SmallText.  Adds the
// number of zero columns to *zeros.
template <typename CT>
inline char* raw_columns(const CT* c, uint64_t n, int m, char* p, uint64_t* zeros) {
    const SmallText& T = small_text();
    auto one = [&](uint32_t v) {
        if (v < kSmall) {
            memcpy(p, T.txt[m][v], 8);   // the row buffer has >= 26 B per column
            p += T.len[m][v];
        } else {
            p = fmt_u64(v, p);
            if (m == 1) { *p++ = '.'; *p++ = '5'; }
            if (m == 2) { *p++ = '.'; *p++ = '0'; }
            *p++ = ',';
        }
    };
    const __m128i sgn = _mm_set1_epi32((int)0x80000000u);
    const __m128i lim = _mm_set1_epi32((int)0x8000000Au);   // unsigned v < 10 as a signed compare
    const __m128i w4 = _mm_set1_epi32(m == 1 ? 0x2C352E30 : 0x2C302E30);   // "0.5," / "0.0,"
    const __m128i w2 = _mm_set1_epi16(0x2C30);                            // "0,"
    const __m128i zero = _mm_setzero_si128();
    uint64_t zs = 0, i = 0;
    while (i + 8 <= n) {
        __m128i z = _mm_setzero_si128();   // 32-bit lane counters, folded every 2^30 groups
        const uint64_t end = std::min<uint64_t>(n & ~7ull, i + (8ull << 30));
        for (; i < end; i += 8) {
            __m128i a, b;
            load8(c + i, a, b);
            z = _mm_sub_epi32(z, _mm_add_epi32(_mm_cmpeq_epi32(a, zero), _mm_cmpeq_epi32(b, zero)));
            const __m128i ok = _mm_and_si128(_mm_cmplt_epi32(_mm_xor_si128(a, sgn), lim),
                                             _mm_cmplt_epi32(_mm_xor_si128(b, sgn), lim));
            if (_mm_movemask_epi8(ok) != 0xFFFF) {
                for (int j = 0; j < 8; ++j) one(c[i + j]);
            } else if (m == 0) {
                _mm_storeu_si128((__m128i*)p, _mm_add_epi16(_mm_packs_epi32(a, b), w2));
                p += 16;
            } else {
                _mm_storeu_si128((__m128i*)p, _mm_add_epi32(a, w4));
                _mm_storeu_si128((__m128i*)(p + 16), _mm_add_epi32(b, w4));
                p += 32;
            }
        }
        alignas(16) uint32_t zl[4];
        _mm_store_si128((__m128i*)zl, z);
        zs += (uint64_t)zl[0] + zl[1] + zl[2] + zl[3];
    }
    for (; i < n; ++i) {
        zs += c[i] == 0;
        one(c[i]);
    }
    *zeros += zs;
    return p;
}

uint64_t kf_line_cap(size_t name_len, uint64_t nbins) { return name_len + 2 + nbins * 26; }

// Per-thread memo of one row's normalised column texts by count (format_line).
struct NormMemo {
    static constexpr uint32_t kMemo = 4096;   // counts memoised (larger ones are formatted each time)
    static constexpr uint32_t kSlot = 24;     // bytes copied per column: repr of a double is <= 24 chars
    uint32_t row = 0;                         // generation of the current row
    uint32_t gen[kMemo] = {};
    uint8_t len[kMemo];
    char txt[kMemo][kSlot];
};
NormMemo& norm_memo() {
    thread_local std::unique_ptr<NormMemo> m(new NormMemo);   // ~120 KB per formatting thread
    return *m;
}

// main.py:327-357
template <typename T>
uint64_t format_line(const char* name, const T* c, uint64_t nb, int pseudo, int raw, char* out) {
    char* p = out;
    const size_t nl = strlen(name);
    memcpy(p, name, nl);
    p += nl;
    *p++ = ',';
    // Integer text ("54", not "54.0") in raw mode without pseudocount when the
    // merged column is not float64: every vocab k-mer is in the dump (pd.merge
    // keeps the dump's int64 column), or the dump is empty (an object column of
    // NaN, which fillna(0) fills with the int 0).  Pinned by
    // tests/golden/ref_postproc (dense_k3_raw, empty_k7_raw).
    if (raw) {
        // raw counts: "c" (integer text), "c.5" (pseudocount) or "c.0" -- what
        // repr prints for an integral float64 below 1e16 (and c + 0.5 < 2^33).
        // Written as float text first; the rare integer-text row (no zero column,
        // or all zero) is written again.
        uint64_t zeros = 0;
        char* const p0 = p;
        p = raw_columns(c, nb, pseudo ? 1 : 2, p0, &zeros);
        if (!pseudo && (zeros == 0 || zeros == nb)) p = raw_columns(c, nb, 0, p0, &zeros);
        if (nb) --p;   // the last column's ','
    } else {
        uint64_t usum = 0;
        for (uint64_t i = 0; i < nb; ++i) usum += c[i];
        double sum = (double)usum;              // exact: integers < 2^53
        if (pseudo) sum += 0.5 * (double)nb;   // exact: multiples of 0.5 < 2^53
        // A row holds few distinct counts (k=7, 5 Mbp: ~1-2 thousand values over
        // 8,192 columns), and a column's text depends on its count only: each
        // count below kMemo is formatted once per row and copied after that.
        NormMemo& M = norm_memo();
        if (++M.row == 0) {   // generation counter wrapped: forget every entry
            memset(M.gen, 0, sizeof M.gen);
            M.row = 1;
        }
        for (uint64_t i = 0; i < nb; ++i) {
            if (i) *p++ = ',';
            const uint32_t ci = (uint32_t)c[i];
            if (ci < NormMemo::kMemo) {
                if (M.gen[ci] != M.row) {
                    M.gen[ci] = M.row;
                    M.len[ci] = (uint8_t)(fmt_repr(((double)ci + (pseudo ? 0.5 : 0.0)) / sum, M.txt[ci]) - M.txt[ci]);
                }
                memcpy(p, M.txt[ci], NormMemo::kSlot);   // the row buffer has >= 26 B per column
                p += M.len[ci];
            } else {
                p = fmt_repr(((double)ci + (pseudo ? 0.5 : 0.0)) / sum, p);
            }
        }
    }
    *p++ = '\n';
    return (uint64_t)(p - out);
}
}  // namespace

// ------------------------------------------------------------------ host worker pool
// One process-wide pool of native worker threads for the host-side batch work
// (file reads, .kf formatting): a call submits n independent items and takes part
// itself; no threads are created per call, and concurrent calls (the CLI reads
// the next batches while the writer formats the last one) share the workers
// instead of oversubscribing the CPUs.
namespace {
struct PoolJob {
    std::function<void(uint64_t)> fn;
    uint64_t n = 0;
    int max_helpers = 0;                 // pool workers allowed on this job
    std::atomic<uint64_t> next{0}, done{0};
    std::atomic<int> helpers{0};
    std::mutex mu;
    std::condition_variable cv;
};
struct HostPool {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::shared_ptr<PoolJob>> jobs;
    std::vector<std::thread> th;
    void ensure(int n) {   // caller holds mu
        while ((int)th.size() < n) th.emplace_back([this] { loop(); });
    }
    void loop() {
        for (;;) {
            std::shared_ptr<PoolJob> j;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !jobs.empty(); });
                for (auto& x : jobs)
                    if (x->next.load() < x->n && x->helpers.load() < x->max_helpers) {
                        j = x;
                        break;
                    }
                if (!j) {   // every queued job is fully handed out: wait for a new one
                    cv.wait(lk);
                    continue;
                }
                j->helpers.fetch_add(1);
            }
            run(*j);
            j->helpers.fetch_sub(1);
        }
    }
    static void run(PoolJob& j) {
        for (;;) {
            const uint64_t t = j.next.fetch_add(1);
            if (t >= j.n) return;
            j.fn(t);
            if (j.done.fetch_add(1) + 1 == j.n) {
                std::lock_guard<std::mutex> lk(j.mu);
                j.cv.notify_all();
            }
        }
    }
};
HostPool& host_pool() {
    static HostPool* p = new HostPool;   // never destroyed: workers outlive static teardown
    return *p;
}
}  // namespace

// Runs fn(0..n-1) on up to n_threads threads (the caller plus pool workers).
static void host_parallel(uint64_t n, int n_threads, const std::function<void(uint64_t)>& fn) {
    if (n == 0) return;
    if (n_threads <= 1 || n == 1) {
        for (uint64_t i = 0; i < n; ++i) fn(i);
        return;
    }
    auto j = std::make_shared<PoolJob>();
    j->fn = fn;
    j->n = n;
    j->max_helpers = (int)std::min<uint64_t>((uint64_t)n_threads - 1, n - 1);
    HostPool& P = host_pool();
    {
        std::lock_guard<std::mutex> lk(P.mu);
        P.ensure(std::min(n_threads - 1, 255));
        P.jobs.push_back(j);
    }
    P.cv.notify_all();
    HostPool::run(*j);
    {
        std::unique_lock<std::mutex> lk(j->mu);
        j->cv.wait(lk, [&] { return j->done.load() == j->n; });
    }
    std::lock_guard<std::mutex> lk(P.mu);
    for (auto it = P.jobs.begin(); it != P.jobs.end(); ++it)
        if (*it == j) {
            P.jobs.erase(it);
            break;
        }
}

extern "C" int kf_read_files(const char* const* paths, int32_t n, const uint64_t* sizes, const uint64_t* off,
                             uint8_t* dst, uint64_t piece, int n_threads) {
    if (n < 0 || (n && (!paths || !sizes || !off || !dst))) return kf_fail(KF_EINVAL, "null argument");
    if (n == 0) return KF_OK;
    if (piece < 4096) piece = 4096;
    if (n_threads < 1) n_threads = 1;
    std::vector<int> fds((size_t)n, -1);
    std::vector<uint64_t> first((size_t)n + 1, 0);   // first piece of each file
    for (int32_t i = 0; i < n; ++i) {
        if (off[i + 1] < off[i] + sizes[i]) return kf_fail(KF_EINVAL, "file %d does not fit its slot", i);
        first[i + 1] = first[i] + (sizes[i] + piece - 1) / piece;
    }
    const uint64_t npiece = first[n];
    std::atomic<int> err{0};
    std::string errmsg;
    std::mutex mu;
    auto fail = [&](const std::string& m) {
        std::lock_guard<std::mutex> lk(mu);
        if (!err.exchange(1)) errmsg = m;
    };
    for (int32_t i = 0; i < n; ++i) {   // open (and check the sizes) first: a missing file fails before any read
        fds[i] = open(paths[i], O_RDONLY | O_CLOEXEC);
        struct stat st;
        if (fds[i] < 0 || fstat(fds[i], &st) != 0 || (uint64_t)st.st_size != sizes[i]) {
            fail(std::string("cannot read ") + paths[i] + (fds[i] < 0 ? "" : " (size changed)"));
            break;
        }
    }
    auto piece_fn = [&](uint64_t t) {
        {
            if (err.load()) return;
            const int32_t i = (int32_t)(std::upper_bound(first.begin(), first.end(), t) - first.begin()) - 1;
            const uint64_t a = (t - first[i]) * piece, e = std::min(sizes[i], a + piece);
            uint64_t got = a;
            while (got < e) {
                const ssize_t r = pread(fds[i], dst + off[i] + got, e - got, (off_t)got);
                if (r < 0 && errno == EINTR) continue;
                if (r <= 0) {
                    fail(std::string("short read on ") + paths[i]);
                    return;
                }
                got += (uint64_t)r;
            }
            if (e == sizes[i]) memset(dst + off[i] + sizes[i], '\n', off[i + 1] - off[i] - sizes[i]);
        }
    };
    if (!err.load()) host_parallel(npiece, n_threads, piece_fn);
    for (int32_t i = 0; i < n; ++i)
        if (fds[i] >= 0) close(fds[i]);
    for (int32_t i = 0; i < n; ++i)   // empty files: their padding (no piece covers them)
        if (sizes[i] == 0) memset(dst + off[i], '\n', off[i + 1] - off[i]);
    if (err.load()) return kf_fail(KF_EINVAL, "%s", errmsg.c_str());
    return KF_OK;
}

extern "C" int kf_format_kf(const char* name, const uint32_t* counts, uint64_t nbins, int pseudocount,
                            int raw_cnt, char* out, uint64_t cap, uint64_t* written) {
    if (!name || (!counts && nbins)) return kf_fail(KF_EINVAL, "null argument");
    const uint64_t need = kf_line_cap(strlen(name), nbins);
    if (!out || cap < need) {
        if (written) *written = need;
        return kf_fail(KF_ERANGE, "output buffer too small (need %llu)", (unsigned long long)need);
    }
    const uint64_t w = format_line(name, counts, nbins, pseudocount, raw_cnt, out);
    if (written) *written = w;
    return KF_OK;
}

constexpr uint64_t kKeepLineBuf = 16ull << 20;   // a worker's line buffer above this is freed after its item

extern "C" int kf_write_kf_files(const char* dir, const char* const* names, int32_t n, const uint32_t* counts,
                                 uint64_t nbins, int pseudocount, int raw_cnt, int n_threads) {
    if (!dir || (!names && n) || (!counts && n)) return kf_fail(KF_EINVAL, "null argument");
    if (n <= 0) return KF_OK;
    std::atomic<int> err{0};
    std::string errmsg;
    std::mutex mu;
    host_parallel((uint64_t)n, std::max(1, n_threads), [&](uint64_t gi) {
        const int32_t i = (int32_t)gi;
        if (err.load()) return;
        thread_local std::vector<char> buf;   // per worker, kept across calls
        thread_local std::string path;
        buf.resize(kf_line_cap(strlen(names[i]), nbins));
        const uint64_t w = format_line(names[i], counts + (uint64_t)i * nbins, nbins, pseudocount, raw_cnt,
                                       buf.data());
        path.assign(dir);
        path += "/";
        path += names[i];
        path += ".kf";
        FILE* f = fopen(path.c_str(), "wb");
        bool ok = f && fwrite(buf.data(), 1, w, f) == w;
        if (f) ok = (fclose(f) == 0) && ok;
        if (!ok) {
            std::lock_guard<std::mutex> lk(mu);
            if (!err.exchange(1)) errmsg = "cannot write " + path;
        }
        // the pool's workers never exit: a large-k line buffer (~54 MB at k=11)
        // is not kept past its item, so a library caller does not hold
        // threads x 54 MB of host memory after the writes
        if (buf.capacity() > kKeepLineBuf) std::vector<char>().swap(buf);
    });
    if (err.load()) return kf_fail(KF_EINVAL, "%s", errmsg.c_str());
    return KF_OK;
}

// Row arenas, kept across calls: fresh blocks would page-fault (and be zeroed by
// the kernel) on every launch's 130 MB of text.  Up to 1 GiB stays pooled.
constexpr uint64_t kArena = 16ull << 20;
struct ArenaPool {
    std::mutex mu;
    std::vector<char*> free;
};
ArenaPool& arena_pool() {
    static ArenaPool* p = new ArenaPool;   // never destroyed: worker threads may outlive static teardown
    return *p;
}
char* arena_get(uint64_t sz) {
    if (sz == kArena) {
        ArenaPool& P = arena_pool();
        std::lock_guard<std::mutex> lk(P.mu);
        if (!P.free.empty()) {
            char* a = P.free.back();
            P.free.pop_back();
            return a;
        }
    }
    const uint64_t al = 2ull << 20;
    char* a = (char*)aligned_alloc(al, (sz + al - 1) / al * al);
    if (a) madvise(a, sz, MADV_HUGEPAGE);
    return a;
}
void arena_put(char* a, uint64_t sz) {
    if (sz == kArena) {
        ArenaPool& P = arena_pool();
        std::lock_guard<std::mutex> lk(P.mu);
        if (P.free.size() < 64) {
            P.free.push_back(a);
            return;
        }
    }
    free(a);
}

// write all of buf at file offset off, resuming after short writes
bool pwrite_all(int fd, const char* buf, uint64_t len, uint64_t off) {
    while (len) {
        const ssize_t w = pwrite(fd, buf, len, (off_t)off);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        buf += w;
        len -= (uint64_t)w;
        off += (uint64_t)w;
    }
    return true;
}

// get_chunks' writer.  The rows are cut into blocks (about 1 MB of text, never
// across a segment); a pool of n_threads workers claims blocks in order, formats
// each into its own arena and writes it with pwrite as soon as its file offset is
// known, i.e. once every earlier block of the segment is formatted (the thread
// that completes that prefix writes the blocks it releases).  So a file is written
// while its later rows are still being formatted, and the tail after the last row
// is one block.  Row i's name is names[i], or, with names == NULL,
// prefixes[row_prefix[i]] + "<s+1>-<s+win_len>", s = row_start[i] (the seqkit
// sliding window name of main.py:905-915).
namespace {
template <typename T>
int write_segments(int32_t n_seg, const char* const* paths, const int32_t* seg_row0, const uint8_t* seg_append,
                   const char* const* names, const char* const* prefixes, const uint32_t* row_prefix,
                   const uint64_t* row_start, uint32_t win_len, const T* counts, uint64_t nbins, int pseudocount,
                   int raw_cnt, int n_threads) {
    if (n_seg < 0 || (n_seg && (!paths || !seg_row0))) return kf_fail(KF_EINVAL, "null argument");
    if (n_seg == 0) return KF_OK;
    const int32_t n = seg_row0[n_seg];
    if (seg_row0[0] != 0 || n < 0) return kf_fail(KF_EINVAL, "seg_row0 must start at 0");
    for (int32_t g = 0; g < n_seg; ++g)
        if (seg_row0[g + 1] < seg_row0[g]) return kf_fail(KF_EINVAL, "seg_row0 must be non-decreasing");
    if (n && (!counts || (!names && (!prefixes || !row_prefix || !row_start))))
        return kf_fail(KF_EINVAL, "null argument");
    if (n_threads < 1) n_threads = 1;
    // files: opened up front (an empty segment still creates / truncates its file)
    std::vector<int> fd((size_t)n_seg, -1);
    std::vector<uint64_t> base((size_t)n_seg, 0);
    auto close_all = [&]() {
        bool ok = true;
        for (int f : fd)
            if (f >= 0) ok = (close(f) == 0) && ok;
        return ok;
    };
    for (int32_t g = 0; g < n_seg; ++g) {
        const bool app = seg_append && seg_append[g];
        fd[g] = open(paths[g], O_WRONLY | O_CREAT | (app ? 0 : O_TRUNC), 0666);
        const off_t end = fd[g] >= 0 && app ? lseek(fd[g], 0, SEEK_END) : 0;
        if (fd[g] < 0 || end < 0) {
            close_all();
            return kf_fail(KF_EINVAL, "cannot write %s", paths[g]);
        }
        base[g] = (uint64_t)end;
    }
    // blocks
    struct Block {
        int32_t g, r0, r1;
        bool done;
        char* buf;
        uint64_t len;
    };
    const uint64_t row_text = 4 * std::max<uint64_t>(nbins, 1) + 64;
    const int32_t per = (int32_t)std::max<uint64_t>(1, std::min<uint64_t>(64, (1ull << 20) / row_text));
    std::vector<Block> blk;
    std::vector<int32_t> front((size_t)n_seg), blk_end((size_t)n_seg);
    std::vector<std::vector<std::pair<int32_t, uint64_t>>> pending((size_t)n_seg);   // (block, file offset)
    std::vector<uint8_t> writing((size_t)n_seg, 0);
    for (int32_t g = 0; g < n_seg; ++g) {
        front[g] = (int32_t)blk.size();
        for (int32_t r = seg_row0[g]; r < seg_row0[g + 1]; r += per)
            blk.push_back({g, r, std::min(r + per, seg_row0[g + 1]), false, nullptr, 0});
        blk_end[g] = (int32_t)blk.size();
    }
    const int32_t nb = (int32_t)blk.size();
    // claim order: every segment at the same relative pace, so concurrent workers
    // hold different files (writes to one file serialise on its inode) and the
    // segments finish together
    std::vector<int32_t> order((size_t)nb);
    {
        std::vector<std::pair<double, int32_t>> key((size_t)nb);
        for (int32_t g = 0, b0 = 0; g < n_seg; b0 = blk_end[g], ++g)
            for (int32_t b = b0; b < blk_end[g]; ++b)
                key[b] = {(b - b0 + 0.5) / (double)(blk_end[g] - b0), b};
        std::sort(key.begin(), key.end());
        for (int32_t j = 0; j < nb; ++j) order[j] = key[j].second;
    }
    const int nw = std::min<int>(n_threads, std::max<int32_t>(nb, 1));
    std::vector<std::vector<std::pair<char*, uint64_t>>> arenas((size_t)nw);
    std::atomic<int32_t> next{0};
    std::atomic<int> err{0};
    std::string errmsg;
    std::mutex mu;
    auto fail = [&](const std::string& m) {
        std::lock_guard<std::mutex> lk(mu);
        if (!err.exchange(1)) errmsg = m;
    };
    auto work = [&](int t) {
        char* pos = nullptr;
        uint64_t left_b = 0;
        std::string nm;
        std::vector<std::pair<int32_t, uint64_t>> release;
        for (;;) {
            const int32_t j = next.fetch_add(1);
            if (j >= nb || err.load()) return;
            Block& B = blk[order[j]];
            // the block's capacity: one arena holds the whole block
            uint64_t cap = 0;
            for (int32_t i = B.r0; i < B.r1; ++i)
                cap += kf_line_cap(names ? strlen(names[i]) : strlen(prefixes[row_prefix[i]]) + 48, nbins);
            if (left_b < cap) {
                const uint64_t sz = std::max(kArena, cap);
                char* a = arena_get(sz);
                if (!a) {
                    fail("out of host memory formatting rows");
                    return;
                }
                arenas[t].emplace_back(a, sz);
                pos = a;
                left_b = sz;
            }
            char* const start = pos;
            for (int32_t i = B.r0; i < B.r1; ++i) {
                const char* name = names ? names[i] : nullptr;
                if (!name) {
                    char tmp[48];
                    const uint64_t s0 = row_start[i];
                    const int m = snprintf(tmp, sizeof tmp, "%llu-%llu", (unsigned long long)(s0 + 1),
                                           (unsigned long long)(s0 + win_len));
                    nm.assign(prefixes[row_prefix[i]]);
                    nm.append(tmp, (size_t)m);
                    name = nm.c_str();
                }
                pos += format_line(name, counts + (uint64_t)i * nbins, nbins, pseudocount, raw_cnt, pos);
            }
            left_b -= (uint64_t)(pos - start);
            const int32_t g = B.g;
            release.clear();
            {
                std::lock_guard<std::mutex> lk(mu);
                B.buf = start;
                B.len = (uint64_t)(pos - start);
                B.done = true;
                while (front[g] < blk_end[g] && blk[front[g]].done) {
                    pending[g].emplace_back(front[g], base[g]);
                    base[g] += blk[front[g]].len;
                    ++front[g];
                }
                // one writer per file at a time: a busy file's blocks are written by
                // the thread already writing it, this one goes back to formatting
                if (writing[g] || pending[g].empty()) continue;
                writing[g] = 1;
                release.swap(pending[g]);
            }
            for (;;) {
                for (auto& r : release)
                    if (!pwrite_all(fd[g], blk[r.first].buf, blk[r.first].len, r.second)) {
                        fail(std::string("cannot write ") + paths[g]);
                        return;
                    }
                release.clear();
                std::lock_guard<std::mutex> lk(mu);
                if (pending[g].empty()) {
                    writing[g] = 0;
                    break;
                }
                release.swap(pending[g]);
            }
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 1; t < nw; ++t) th.emplace_back(work, t);
        work(0);
        for (auto& t : th) t.join();
    }
    for (auto& v : arenas)
        for (auto& a : v) arena_put(a.first, a.second);
    if (!close_all() && !err.load()) {
        err = 1;
        errmsg = "cannot close an output file";
    }
    if (err.load()) return kf_fail(errmsg.rfind("out of", 0) == 0 ? KF_ERANGE : KF_EINVAL, "%s", errmsg.c_str());
    return KF_OK;
}
}  // namespace

extern "C" int kf_write_kf_segments(int32_t n_seg, const char* const* paths, const int32_t* seg_row0,
                                    const uint8_t* seg_append, const char* const* names,
                                    const char* const* prefixes, const uint32_t* row_prefix, const uint64_t* row_start,
                                    uint32_t win_len, const uint32_t* counts, uint64_t nbins, int pseudocount,
                                    int raw_cnt, int n_threads) {
    return write_segments(n_seg, paths, seg_row0, seg_append, names, prefixes, row_prefix, row_start, win_len, counts,
                          nbins, pseudocount, raw_cnt, n_threads);
}

extern "C" int kf_write_kf_segments16(int32_t n_seg, const char* const* paths, const int32_t* seg_row0,
                                      const uint8_t* seg_append, const char* const* names,
                                      const char* const* prefixes, const uint32_t* row_prefix,
                                      const uint64_t* row_start, uint32_t win_len, const uint16_t* counts,
                                      uint64_t nbins, int pseudocount, int raw_cnt, int n_threads) {
    return write_segments(n_seg, paths, seg_row0, seg_append, names, prefixes, row_prefix, row_start, win_len, counts,
                          nbins, pseudocount, raw_cnt, n_threads);
}

extern "C" int kf_write_kf_rows(const char* path, const char* const* names, int32_t n, const uint32_t* counts,
                                uint64_t nbins, int pseudocount, int raw_cnt, int n_threads) {
    if (!path || (!names && n) || (!counts && n) || n < 0) return kf_fail(KF_EINVAL, "null argument");
    const int32_t row0[2] = {0, n};
    return kf_write_kf_segments(1, &path, row0, nullptr, names, nullptr, nullptr, nullptr, 0, counts, nbins, pseudocount,
                                raw_cnt, n_threads);
}

// ------------------------------------------------------------------ synthetic layout
extern "C" uint64_t kf_synth_header_len(int64_t g) {
    char tmp[32];
    return (uint64_t)snprintf(tmp, sizeof tmp, ">syn_%lld\n", (long long)g);
}

extern "C" uint64_t kf_synth_genome_bytes(int64_t g, uint64_t seq_len, int width, uint64_t align) {
    if (width < 1) return 0;
    const uint64_t need = kf_synth_header_len(g) + seq_len + (seq_len + (uint64_t)width - 1) / (uint64_t)width;
    if (align < 1) align = 1;
    return (need + align - 1) / align * align;
}

// ------------------------------------------------------------------ build provenance
#ifndef KF_BUILD_ID
#define KF_BUILD_ID "unknown"
#endif
// "KF_BUILD_ID=<id>" is kept whole in the binary so build.py can read the id
// without loading the library.
static const char kBuildId[] = "KF_BUILD_ID=" KF_BUILD_ID;
extern "C" const char* kf_build_id(void) { return kBuildId + 12; }
