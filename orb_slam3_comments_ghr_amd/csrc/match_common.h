// match_common.h — host/device helpers shared by the matcher kernels (match.hip).
#pragma once
#include <cstdint>
#include <cstring>
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
};

template <typename T>
static inline T *osg_dptr(void *base, size_t off)
{
    return off == SIZE_MAX ? nullptr : (T *)((char *)base + off);
}
