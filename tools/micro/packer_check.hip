// packer_check.hip — host-only check of the matcher's pinned-block packer (match_common.h): plain items and
// row-gather items (add_rows) filled by fill() and by fill_parallel() over 4 MiB pieces give the bytes of a
// straightforward reference pack.  Built against the product library (osg_parallel_for) by
// tests/test_host_runtime.py; no GPU calls.
#include <random>

#include "match_common.h"

extern "C" int packer_check(unsigned seed, int n_items, int threads)
{
    std::mt19937 rng(seed);
    std::vector<std::vector<uint8_t>> src(n_items);
    std::vector<std::vector<int32_t>> idx(n_items);
    std::vector<size_t> row(n_items, 0);
    osg_packer pk;
    std::vector<size_t> off(n_items);
    for (int i = 0; i < n_items; i++) {
        const bool rows = rng() % 2;
        static const size_t row_sizes[3] = {4, 32, 12};  // 12: rows split by the 4 MiB pieces
        const size_t rb = rows ? row_sizes[rng() % 3] : 0;
        if (rows) {  // up to ~1.5 MiB of rows gathered from a larger source, indices in any order
            const size_t n_src = 1 + rng() % 40000, n_rows = 1 + rng() % (1 + (1 << 20) / rb);
            src[i].resize(n_src * rb);
            for (auto &b : src[i]) b = (uint8_t)rng();
            idx[i].resize(n_rows);
            for (auto &k : idx[i]) k = (int32_t)(rng() % n_src);
            row[i] = rb;
            off[i] = pk.add_rows(src[i].data(), idx[i].data(), n_rows, rb);
        } else {
            src[i].resize(1 + rng() % (3 << 20));
            for (auto &b : src[i]) b = (uint8_t)rng();
            off[i] = pk.add(src[i].data(), src[i].size());
        }
    }
    std::vector<uint8_t> ref(pk.total, 0), a(pk.total, 0), b(pk.total, 0);
    for (int i = 0; i < n_items; i++) {
        if (!row[i]) {
            std::memcpy(&ref[off[i]], src[i].data(), src[i].size());
            continue;
        }
        for (size_t r = 0; r < idx[i].size(); r++)
            std::memcpy(&ref[off[i] + r * row[i]], &src[i][(size_t)idx[i][r] * row[i]], row[i]);
    }
    pk.fill(a.data());
    pk.fill_parallel(b.data(), threads);
    if (std::memcmp(ref.data(), a.data(), ref.size()) != 0) return 1;
    if (std::memcmp(ref.data(), b.data(), ref.size()) != 0) return 2;
    return 0;
}
