// Process-wide recycling of large record blocks (fe_picture.h PoolAlloc): a freed block of at least
// kPoolMin bytes is kept (up to kPoolCap idle bytes) and handed to the next request it fits, so a
// parser thread's coefficient arena and TB array reuse pages that are already mapped.
#include <cstdlib>
#include <mutex>
#include <new>
#include <vector>

#include "fe_picture.h"

namespace p265fe {

namespace {

constexpr size_t kHeader = 64;                 // block header: capacity (keeps 64-B data alignment)
constexpr size_t kPoolMin = 256u << 10;        // smaller blocks go straight back to malloc
constexpr size_t kPoolCap = 2048ull << 20;     // idle bytes kept at most (≈200 1080p pictures)

struct Pool {
    std::mutex mu;
    std::vector<std::pair<size_t, void*>> free;   // (capacity, base)
    size_t idle = 0;
};

Pool& pool() {
    static Pool* p = new Pool();                // never destroyed: blocks may be freed at process exit
    return *p;
}

}  // namespace

void* pool_alloc(size_t bytes) {
    if (bytes >= kPoolMin) {
        Pool& P = pool();
        std::lock_guard<std::mutex> lk(P.mu);
        size_t best = P.free.size();
        for (size_t i = 0; i < P.free.size(); ++i)     // smallest idle block that fits (and is not 4x too big)
            if (P.free[i].first >= bytes && P.free[i].first <= 4 * bytes &&
                (best == P.free.size() || P.free[i].first < P.free[best].first))
                best = i;
        if (best < P.free.size()) {
            void* base = P.free[best].second;
            P.idle -= P.free[best].first;
            P.free[best] = P.free.back();
            P.free.pop_back();
            return static_cast<char*>(base) + kHeader;
        }
        bytes = (bytes + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);   // 1 MB granules: reusable sizes
    }
    void* base = std::aligned_alloc(kHeader, (bytes + 2 * kHeader - 1) & ~(kHeader - 1));
    if (!base) throw std::bad_alloc();
    *static_cast<size_t*>(base) = bytes;
    return static_cast<char*>(base) + kHeader;
}

void pool_free(void* p) {
    if (!p) return;
    void* base = static_cast<char*>(p) - kHeader;
    const size_t cap = *static_cast<size_t*>(base);
    if (cap >= kPoolMin) {
        Pool& P = pool();
        std::lock_guard<std::mutex> lk(P.mu);
        if (P.idle + cap <= kPoolCap) {
            P.free.emplace_back(cap, base);
            P.idle += cap;
            return;
        }
    }
    std::free(base);
}

}  // namespace p265fe
