// kf_host.cpp -- host half of the kf2vec_gpu C-ABI (include/kf2vec_gpu.h):
// bin tables / vocabulary, FASTA/FASTQ record index, byte-exact `.kf` formatting
// and the parallel `.kf` writer.
#include <fcntl.h>
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
// at k=7, nearly all 0-3): their text comes from a table built once.
//   kSmallInt[c] = "c", kSmallHalf[c] = "c.5" (pseudocount), kSmallF[c] = "c.0"
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
                len[m][c] = (uint8_t)(e - p);
            }
        }
    }
};
const SmallText& small_text() {
    static const SmallText t;
    return t;
}

uint64_t kf_line_cap(size_t name_len, uint64_t nbins) { return name_len + 2 + nbins * 26; }

// writev all of iov (bytes in total), resuming after short writes.
bool write_all_v(int fd, struct iovec* iov, int cnt, uint64_t bytes) {
    while (bytes) {
        const ssize_t w = writev(fd, iov, cnt);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        bytes -= (uint64_t)w;
        uint64_t d = (uint64_t)w;
        while (cnt && d >= iov->iov_len) {
            d -= iov->iov_len;
            ++iov;
            --cnt;
        }
        if (cnt) {
            iov->iov_base = (char*)iov->iov_base + d;
            iov->iov_len -= d;
        }
    }
    return true;
}

// main.py:327-357
uint64_t format_line(const char* name, const uint32_t* c, uint64_t nb, int pseudo, int raw, char* out) {
    char* p = out;
    const size_t nl = strlen(name);
    memcpy(p, name, nl);
    p += nl;
    *p++ = ',';
    bool all_present = nb > 0;
    double sum = 0.0;
    for (uint64_t i = 0; i < nb; ++i) {
        all_present &= c[i] > 0;
        sum += (double)c[i];        // exact: integers < 2^53
    }
    if (pseudo) sum += 0.5 * (double)nb;   // exact: multiples of 0.5 < 2^53
    // Integer text ("54", not "54.0") in raw mode without pseudocount when the
    // merged column is not float64: every vocab k-mer is in the dump (pd.merge
    // keeps the dump's int64 column), or the dump is empty (an object column of
    // NaN, which fillna(0) fills with the int 0).  Pinned by
    // tests/golden/ref_postproc (dense_k3_raw, empty_k7_raw).
    const bool int_text = raw && !pseudo && (all_present || sum == 0.0);
    if (raw) {
        // raw counts: "c" (integer text), "c.5" (pseudocount) or "c.0" -- what
        // repr prints for an integral float64 below 1e16 (and c + 0.5 < 2^33)
        const SmallText& T = small_text();
        const int m = int_text ? 0 : (pseudo ? 1 : 2);
        for (uint64_t i = 0; i < nb; ++i) {
            if (i) *p++ = ',';
            const uint32_t v = c[i];
            if (v < kSmall) {
                memcpy(p, T.txt[m][v], 8);   // the row buffer has >= 26 B per column
                p += T.len[m][v];
            } else {
                p = fmt_u64(v, p);
                if (m == 1) { *p++ = '.'; *p++ = '5'; }
                if (m == 2) { *p++ = '.'; *p++ = '0'; }
            }
        }
    } else {
        for (uint64_t i = 0; i < nb; ++i) {
            if (i) *p++ = ',';
            const double v = ((double)c[i] + (pseudo ? 0.5 : 0.0)) / sum;
            p = fmt_repr(v, p);
        }
    }
    *p++ = '\n';
    return (uint64_t)(p - out);
}
}  // namespace

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

extern "C" int kf_write_kf_files(const char* dir, const char* const* names, int32_t n, const uint32_t* counts,
                                 uint64_t nbins, int pseudocount, int raw_cnt, int n_threads) {
    if (!dir || (!names && n) || (!counts && n)) return kf_fail(KF_EINVAL, "null argument");
    if (n_threads < 1) n_threads = 1;
    n_threads = std::min<int>(n_threads, std::max<int32_t>(n, 1));
    std::atomic<int32_t> next{0};
    std::atomic<int> err{0};
    std::string errmsg;
    std::mutex mu;
    auto work = [&]() {
        std::vector<char> buf;
        std::string path;
        for (;;) {
            const int32_t i = next.fetch_add(1);
            if (i >= n || err.load()) break;
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
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < n_threads; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    if (err.load()) return kf_fail(KF_EINVAL, "%s", errmsg.c_str());
    return KF_OK;
}

// get_chunks' writer.  One pool of n_threads workers: a worker writes a segment
// whose rows are all formatted (one writev stream per file, rows in order) and
// otherwise formats the next row into its own arenas (no per-row allocation or
// copy), so formatting and writing overlap.  Row i's name is names[i], or, with
// names == NULL, prefixes[row_prefix[i]] + "<s+1>-<s+win_len>", s = row_start[i]
// (the seqkit sliding window name of main.py:905-915).
extern "C" int kf_write_kf_segments(int32_t n_seg, const char* const* paths, const int32_t* seg_row0,
                                    const uint8_t* seg_append, const char* const* names,
                                    const char* const* prefixes, const uint32_t* row_prefix, const uint64_t* row_start,
                                    uint32_t win_len, const uint32_t* counts, uint64_t nbins, int pseudocount,
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
    std::vector<char*> rp((size_t)n, nullptr);
    std::vector<uint64_t> rl((size_t)n, 0);
    std::vector<int32_t> seg_of((size_t)n);
    std::unique_ptr<std::atomic<int32_t>[]> left(new std::atomic<int32_t>[n_seg]);
    std::vector<int32_t> ready;   // segments whose rows are all formatted, not yet claimed
    for (int32_t g = 0; g < n_seg; ++g) {
        left[g].store(seg_row0[g + 1] - seg_row0[g]);
        for (int32_t i = seg_row0[g]; i < seg_row0[g + 1]; ++i) seg_of[i] = g;
        if (seg_row0[g + 1] == seg_row0[g]) ready.push_back(g);
    }
    const int nw = std::min<int>(n_threads, std::max<int32_t>(n, n_seg));
    std::vector<std::vector<std::unique_ptr<char[]>>> arenas((size_t)nw);
    std::atomic<int32_t> next_row{0};
    int32_t written = 0;
    int err = 0;
    std::string errmsg;
    std::mutex mu;
    std::condition_variable cv;
    auto write_seg = [&](int32_t g, std::vector<struct iovec>& iov) -> bool {
        const int fd = open(paths[g], O_WRONLY | O_CREAT | ((seg_append && seg_append[g]) ? O_APPEND : O_TRUNC), 0666);
        bool ok = fd >= 0;
        for (int32_t i = seg_row0[g]; ok && i < seg_row0[g + 1];) {
            iov.clear();
            uint64_t bytes = 0;
            for (; i < seg_row0[g + 1] && iov.size() < 512; ++i) {
                iov.push_back({rp[i], (size_t)rl[i]});
                bytes += rl[i];
            }
            ok = write_all_v(fd, iov.data(), (int)iov.size(), bytes);
        }
        if (fd >= 0) ok = (close(fd) == 0) && ok;
        return ok;
    };
    auto work = [&](int t) {
        constexpr uint64_t kArena = 16ull << 20;
        char* pos = nullptr;
        uint64_t left_b = 0;
        std::vector<struct iovec> iov;
        std::string nm;
        for (;;) {
            int32_t g = -1;
            {
                std::unique_lock<std::mutex> lk(mu);
                for (;;) {
                    if (err || written == n_seg) return;
                    if (!ready.empty()) {
                        g = ready.back();
                        ready.pop_back();
                        break;
                    }
                    if (next_row.load() < n) break;   // rows left to format
                    cv.wait(lk);
                }
            }
            if (g >= 0) {
                const bool ok = write_seg(g, iov);
                std::lock_guard<std::mutex> lk(mu);
                if (!ok && !err) {
                    err = 1;
                    errmsg = std::string("cannot write ") + paths[g];
                }
                ++written;
                cv.notify_all();
                continue;
            }
            const int32_t i = next_row.fetch_add(1);
            if (i >= n) continue;
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
            const uint64_t cap = kf_line_cap(strlen(name), nbins);
            if (left_b < cap) {
                const uint64_t sz = std::max(kArena, cap);
                char* a = new (std::nothrow) char[sz];
                if (!a) {
                    std::lock_guard<std::mutex> lk(mu);
                    if (!err) { err = 1; errmsg = "out of host memory formatting rows"; }
                    cv.notify_all();
                    return;
                }
                arenas[t].emplace_back(a);
                pos = a;
                left_b = sz;
            }
            const uint64_t w = format_line(name, counts + (uint64_t)i * nbins, nbins, pseudocount, raw_cnt, pos);
            rp[i] = pos;
            rl[i] = w;
            pos += w;
            left_b -= w;
            if (left[seg_of[i]].fetch_sub(1) == 1) {   // the segment's last row: it can be written
                std::lock_guard<std::mutex> lk(mu);
                ready.push_back(seg_of[i]);
                cv.notify_one();
            }
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 1; t < nw; ++t) th.emplace_back(work, t);
        work(0);
        for (auto& t : th) t.join();
    }
    if (err) return kf_fail(errmsg.rfind("out of", 0) == 0 ? KF_ERANGE : KF_EINVAL, "%s", errmsg.c_str());
    return KF_OK;
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
