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
    struct item {
        const void *src;
        size_t bytes;
        size_t off;
    };
    std::vector<item> items;
    size_t total = 0;
    // returns the offset, or SIZE_MAX for a null/empty source
    size_t add(const void *src, size_t bytes)
    {
        if (!src || bytes == 0) return SIZE_MAX;
        const size_t off = total;
        items.push_back({src, bytes, off});
        total = (total + bytes + 255) & ~size_t(255);
        return off;
    }
    void fill(void *dst) const
    {
        for (const item &it : items) std::memcpy((char *)dst + it.off, it.src, it.bytes);
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
                if (a < b) std::memcpy((char *)dst + a, (const char *)it.src + (a - it.off), b - a);
            }
        });
    }
};

template <typename T>
static inline T *osg_dptr(void *base, size_t off)
{
    return off == SIZE_MAX ? nullptr : (T *)((char *)base + off);
}
