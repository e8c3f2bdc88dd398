// match_common.h — host/device helpers shared by the matcher kernels (match.hip).
#pragma once
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "osg_internal.h"

// Packs many host arrays into one pinned staging block so a call moves its inputs with a single
// hipMemcpyAsync (and its outputs back with one more).  Offsets are 256-byte aligned.
struct osg_packer {
    // a plain item copies `bytes` from src; a row item (idx != nullptr) gathers `bytes / row` rows of
    // `row` bytes, row r from src + idx[r] * row, straight into the block (no host staging copy)
    struct item {
        const void *src;
        size_t bytes;
        size_t off;
        const int32_t *idx;
        size_t row;
    };
    std::vector<item> items;
    size_t total = 0;
    // returns the offset, or SIZE_MAX for a null/empty source
    size_t add(const void *src, size_t bytes)
    {
        if (!src || bytes == 0) return SIZE_MAX;
        const size_t off = total;
        items.push_back({src, bytes, off, nullptr, 0});
        total = (total + bytes + 255) & ~size_t(255);
        return off;
    }
    // rows src[idx[0]], src[idx[1]], ... of `row` bytes each; idx must stay valid until the fill
    size_t add_rows(const void *src, const int32_t *idx, size_t rows, size_t row)
    {
        if (!src || !idx || rows == 0 || row == 0) return SIZE_MAX;
        const size_t off = total;
        items.push_back({src, rows * row, off, idx, row});
        total = (total + rows * row + 255) & ~size_t(255);
        return off;
    }
    // bytes [a, b) of item `it` (offsets relative to the item) into dst + it.off + a
    static void copy_part(char *dst, const item &it, size_t a, size_t b)
    {
        if (!it.idx) {
            std::memcpy(dst + it.off + a, (const char *)it.src + a, b - a);
            return;
        }
        const char *src = (const char *)it.src;
        const size_t rb = it.row;
        // whole rows inside [a, b) with a fixed-size copy (inlined for the 32-byte descriptor and 4-byte
        // rows), the split rows at a piece's edges byte-exact
        const size_t r0 = (a + rb - 1) / rb, r1 = b / rb;
        auto part = [&](size_t r) {
            const size_t lo = std::max(a, r * rb), hi = std::min(b, (r + 1) * rb);
            if (lo < hi) std::memcpy(dst + it.off + lo, src + (size_t)it.idx[r] * rb + (lo - r * rb), hi - lo);
        };
        if (r0 > r1) {  // [a, b) inside one row
            part(a / rb);
            return;
        }
        if (a < r0 * rb) part(r0 - 1);
        char *d = dst + it.off + r0 * rb;
        if (rb == 32)
            for (size_t r = r0; r < r1; r++, d += 32) std::memcpy(d, src + (size_t)it.idx[r] * 32, 32);
        else if (rb == 4)
            for (size_t r = r0; r < r1; r++, d += 4) std::memcpy(d, src + (size_t)it.idx[r] * 4, 4);
        else
            for (size_t r = r0; r < r1; r++, d += rb) std::memcpy(d, src + (size_t)it.idx[r] * rb, rb);
        if (r1 * rb < b) part(r1);
    }
    void fill(void *dst) const
    {
        for (const item &it : items) copy_part((char *)dst, it, 0, it.bytes);
    }
    // the same copy split into 4 MiB pieces over up to `nthreads` host threads (the calling one and
    // budgeted workers, osg_parallel_for) for large batches
    void fill_parallel(void *dst, int nthreads) const
    {
        if (nthreads <= 1 || total < (size_t(8) << 20)) {
            fill(dst);
            return;
        }
        constexpr size_t PIECE = size_t(4) << 20;
        const int np = (int)((total + PIECE - 1) / PIECE);
        osg_parallel_for(np, nthreads, [&](int p) {
            const size_t lo = (size_t)p * PIECE, hi = std::min(total, lo + PIECE);
            // the items overlapping [lo, hi): items are in offset order
            size_t k = std::upper_bound(items.begin(), items.end(), lo,
                                        [](size_t v, const item &it) { return v < it.off; }) - items.begin();
            if (k > 0) k--;
            for (; k < items.size() && items[k].off < hi; k++) {
                const item &it = items[k];
                const size_t a = std::max(lo, it.off), b = std::min(hi, it.off + it.bytes);
                if (a < b) copy_part((char *)dst, it, a - it.off, b - it.off);
            }
        });
    }
};

template <typename T>
static inline T *osg_dptr(void *base, size_t off)
{
    return off == SIZE_MAX ? nullptr : (T *)((char *)base + off);
}
