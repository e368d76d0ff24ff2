// heap.h -- the Emscripten-style linear heap behind the N-API addon (h264mi_napi.cc): a first-fit
// allocator over one pinned host block, addressed by byte offsets (offset 0 = NULL), and the bounds
// checks every entry point applies to the offsets the JS glue passes in. Plain C++ (no Node, no HIP):
// also compiled into the sanitizer harness tests/native/host_fuzz.cc.
#pragma once
#include <cstddef>
#include <cstdint>
#include <map>

namespace {

struct Heap {
    uint8_t *base = nullptr;
    size_t size = 0;
    std::map<uint32_t, uint32_t> free_;  // offset -> bytes (coalesced)
    std::map<uint32_t, uint32_t> used_;
    void init(uint8_t *b, size_t n) {
        base = b; size = n;
        free_.clear(); used_.clear();
        if (n > 16) free_[16] = (uint32_t)(n - 16);
    }
    uint32_t alloc(size_t n) {
        if (n == 0) n = 1;
        if (n > size) return 0;
        const uint32_t need = (uint32_t)((n + 15) & ~(size_t)15);
        for (auto it = free_.begin(); it != free_.end(); ++it) {
            if (it->second < need) continue;
            const uint32_t off = it->first, rest = it->second - need;
            free_.erase(it);
            if (rest) free_[off + need] = rest;
            used_[off] = need;
            return off;
        }
        return 0;
    }
    void release(uint32_t off) {
        auto u = used_.find(off);
        if (u == used_.end()) return;
        uint32_t o = off, n = u->second;
        used_.erase(u);
        auto nx = free_.lower_bound(o);
        if (nx != free_.end() && nx->first == o + n) { n += nx->second; free_.erase(nx); }
        auto pv = free_.lower_bound(o);
        if (pv != free_.begin()) {
            --pv;
            if (pv->first + pv->second == o) { o = pv->first; n += pv->second; free_.erase(pv); }
        }
        free_[o] = n;
    }
    // [off, off + n) lies inside the heap; off > 0 (0 is NULL). Written so that no sum can overflow
    // whatever the (double-converted) arguments are.
    bool ok(int64_t off, int64_t n) const {
        return off > 0 && n >= 0 && (uint64_t)off <= size && (uint64_t)n <= size - (uint64_t)off;
    }
    uint8_t *at(int64_t off) const { return base + off; }
};

}  // namespace
