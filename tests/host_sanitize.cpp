// host_sanitize.cpp -- drives every host-side entry point of libkf2vec_gpu
// (kf2vecfsw_amd/csrc/kf_host.cpp: vocab tables, record index, .kf formatter,
// threaded .kf writer, synthetic layout) under AddressSanitizer and
// UndefinedBehaviorSanitizer.  Built and run by tests/test_host_sanitize.py via
// `python -m kf2vecfsw_amd.build --sanitize` (g++ -fsanitize=address,undefined,
// host code only: the HIP kernels are not part of this binary).
//
// Besides "no sanitizer report", it checks invariants of each result:
//   * kf_tables: code2col and col2rep are inverse on representatives, every
//     column has one or two codes (a k-mer and its reverse complement);
//   * kf_index_records: sorted, disjoint, in-range intervals; the ERANGE path
//     reports the pair count the full call then returns;
//   * kf_format_kf: every field parses back (strtod) to count/sum, count+0.5 or
//     the integer count, as main.py:327-345 defines them; written <= capacity;
//   * kf_write_kf_files (8 threads): each file equals kf_format_kf's line.
#include <dirent.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <random>
#include <string>
#include <vector>

#include "../include/kf2vec_gpu.h"

static int g_fail = 0;
#define CHECK(c)                                                                        \
    do {                                                                                \
        if (!(c)) {                                                                     \
            fprintf(stderr, "CHECK failed %s:%d: %s (%s)\n", __FILE__, __LINE__, #c,    \
                    kf_last_error());                                                   \
            ++g_fail;                                                                   \
        }                                                                               \
    } while (0)

static void tables() {
    for (int k = 2; k <= 11; ++k) {
        const uint64_t nb = kf_num_bins(k);
        std::vector<uint32_t> c2c((size_t)1 << (2 * k)), c2r(nb);
        uint64_t n = 0;
        CHECK(kf_tables(k, c2c.data(), c2r.data(), &n) == KF_OK && n == nb);
        std::vector<uint8_t> seen(nb, 0);
        for (uint64_t x = 0; x < c2c.size(); ++x) {
            CHECK(c2c[x] < nb);
            if (c2c[x] < nb && seen[c2c[x]] < 255) ++seen[c2c[x]];
        }
        for (uint64_t c = 0; c < nb; ++c) {
            CHECK(seen[c] == 1 || seen[c] == 2);
            CHECK(c2r[c] < c2c.size() && c2c[c2r[c]] == c);
        }
        if (k <= 9) {
            std::vector<char> v(nb * (k + 1));
            uint64_t w = 0;
            CHECK(kf_vocab_text(k, v.data(), v.size(), &w) == KF_OK && w == v.size());
            CHECK(kf_vocab_text(k, v.data(), v.size() - 1, &w) == KF_ERANGE);
        }
    }
    CHECK(kf_num_bins(1) == 0 || kf_num_bins(1) == 2);
    CHECK(kf_tables(13, nullptr, nullptr, nullptr) != KF_OK);
}

static void index_records(std::mt19937_64& rng) {
    const char alpha[] = "ACGTN\n\n>@+acgt\r";
    for (int t = 0; t < 400; ++t) {
        const size_t len = rng() % 3000;
        std::vector<uint8_t> b(len);
        for (auto& x : b) x = (rng() % 8 == 0) ? (uint8_t)(rng() & 0xFF) : (uint8_t)alpha[rng() % (sizeof alpha - 1)];
        if (len && t % 3 == 0) b[0] = '@';
        const int fmt = (int)(t % 3);   // auto, FASTA, FASTQ
        const uint64_t base = rng() % 1000;
        uint64_t n = 0;
        int det = -1;
        std::vector<uint64_t> iv(2);
        int rc = kf_index_records(b.data(), len, fmt, base, iv.data(), 1, &n, &det);
        CHECK(rc == KF_OK || rc == KF_ERANGE);
        if (rc == KF_ERANGE) {
            iv.resize(2 * n);
            uint64_t n2 = 0;
            CHECK(kf_index_records(b.data(), len, fmt, base, iv.data(), n, &n2, &det) == KF_OK && n2 == n);
        }
        for (uint64_t i = 0; i < n; ++i) {
            CHECK(iv[2 * i] <= iv[2 * i + 1]);
            CHECK(iv[2 * i] >= base && iv[2 * i + 1] <= base + len);
            if (i) CHECK(iv[2 * i - 1] <= iv[2 * i]);
        }
        CHECK(det == 1 || det == 2);
    }
    uint64_t n = 0;
    CHECK(kf_index_records(nullptr, 0, 0, 0, nullptr, 0, &n, nullptr) == KF_OK && n == 0);
    CHECK(kf_index_records(nullptr, 5, 0, 0, nullptr, 0, &n, nullptr) == KF_EINVAL);
}

// fields of one .kf line after the name
static std::vector<std::string> fields(const char* s, uint64_t w) {
    std::vector<std::string> out;
    const char* p = (const char*)memchr(s, ',', w);
    if (!p) return out;
    const char* e = s + w;
    CHECK(w > 0 && s[w - 1] == '\n');
    ++p;
    if (e - p == 1 && *p == '\n') return out;   // no bins: "name,\n"
    while (p < e) {
        const char* q = p;
        while (q < e && *q != ',' && *q != '\n') ++q;
        out.emplace_back(p, q);
        p = q + 1;
    }
    return out;
}

static void format(std::mt19937_64& rng) {
    for (int t = 0; t < 300; ++t) {
        const uint64_t nb = t < 3 ? (uint64_t)t : 1 + rng() % 2100;
        std::vector<uint32_t> c(nb);
        const int mode = t % 4;   // sparse, all present, huge, zero
        for (auto& x : c) {
            if (mode == 0) x = (rng() % 3) ? 0 : (uint32_t)(rng() % 100);
            else if (mode == 1) x = 1 + (uint32_t)(rng() % 1000);
            else if (mode == 2) x = (uint32_t)(rng() >> 32);
            else x = 0;
        }
        for (int pseudo = 0; pseudo < 2; ++pseudo)
            for (int raw = 0; raw < 2; ++raw) {
                uint64_t need = 0;
                CHECK(kf_format_kf("s", c.data(), nb, pseudo, raw, nullptr, 0, &need) == KF_ERANGE);
                std::vector<char> buf(need);
                uint64_t w = 0;
                CHECK(kf_format_kf("s", c.data(), nb, pseudo, raw, buf.data(), buf.size(), &w) == KF_OK);
                CHECK(w <= need);
                const auto f = fields(buf.data(), w);
                CHECK(f.size() == nb);
                double sum = 0;
                bool all = nb > 0;
                for (auto x : c) sum += x + (pseudo ? 0.5 : 0.0), all &= x > 0;
                for (uint64_t i = 0; i < f.size() && i < nb; ++i) {
                    double v = c[i] + (pseudo ? 0.5 : 0.0);
                    if (!raw) v = v / sum;
                    if (raw && !pseudo && (all || sum == 0.0)) {
                        CHECK(f[i] == std::to_string(c[i]));
                    } else if (v != v) {
                        CHECK(f[i] == "nan");
                    } else {
                        CHECK(strtod(f[i].c_str(), nullptr) == v);
                        CHECK(f[i].find_first_of(".en") != std::string::npos);
                    }
                }
            }
    }
}

static void writer(std::mt19937_64& rng) {
    char tmpl[] = "/tmp/kf_host_sanitize_XXXXXX";
    const char* dir = mkdtemp(tmpl);
    CHECK(dir != nullptr);
    if (!dir) return;
    const int n = 37;
    const uint64_t nb = 512;
    std::vector<uint32_t> c((size_t)n * nb);
    for (auto& x : c) x = (uint32_t)(rng() % 50);
    std::vector<std::string> nm(n);
    std::vector<const char*> names(n);
    for (int i = 0; i < n; ++i) {
        nm[i] = "genome_" + std::to_string(i);
        names[i] = nm[i].c_str();
    }
    CHECK(kf_write_kf_files(dir, names.data(), n, c.data(), nb, 1, 0, 8) == KF_OK);
    for (int i = 0; i < n; ++i) {
        uint64_t need = 0;
        kf_format_kf(names[i], c.data() + (size_t)i * nb, nb, 1, 0, nullptr, 0, &need);
        std::vector<char> exp(need);
        uint64_t w = 0;
        CHECK(kf_format_kf(names[i], c.data() + (size_t)i * nb, nb, 1, 0, exp.data(), need, &w) == KF_OK);
        const std::string path = std::string(dir) + "/" + nm[i] + ".kf";
        FILE* f = fopen(path.c_str(), "rb");
        CHECK(f != nullptr);
        if (!f) continue;
        std::vector<char> got(w + 16);
        const size_t r = fread(got.data(), 1, got.size(), f);
        fclose(f);
        CHECK(r == w && memcmp(got.data(), exp.data(), w) == 0);
        unlink(path.c_str());
    }
    CHECK(kf_write_kf_files("/nonexistent_dir_kf", names.data(), 2, c.data(), nb, 0, 0, 2) != KF_OK);
    rmdir(dir);
}

int main() {
    std::mt19937_64 rng(20260101);
    CHECK(kf_abi_version() == 1);
    tables();
    index_records(rng);
    format(rng);
    writer(rng);
    for (int64_t g : {0, 7, 12345, -3}) {
        CHECK(kf_synth_header_len(g) >= 7);
        CHECK(kf_synth_genome_bytes(g, 5000, 80, 256) % 256 == 0);
    }
    CHECK(kf_synth_genome_bytes(0, 10, 0, 16) == 0);
    if (g_fail) {
        fprintf(stderr, "host_sanitize: %d checks failed\n", g_fail);
        return 1;
    }
    printf("host_sanitize: all checks passed (ASan + UBSan)\n");
    return 0;
}
