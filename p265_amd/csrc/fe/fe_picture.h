// Slice segment data decoding of one picture into back-end records (see fe_picture.cpp).
#pragma once
#include <cstdint>
#include <memory>
#include <utility>
#include <vector>

#include "../../../include/p265r.h"
#include "fe_ps.h"

namespace p265fe {

// an allocator whose value-less construct() leaves the element uninitialised: resize() of the
// coefficient arena neither zeroes nor touches its pages (each block is zeroed when carved out)
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U> struct rebind { using other = DefaultInitAlloc<U>; };
    DefaultInitAlloc() = default;
    template <class U> DefaultInitAlloc(const DefaultInitAlloc<U>&) {}
    template <class U> void construct(U* p) { ::new (static_cast<void*>(p)) U; }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
};

// Recycled large blocks for a picture's big record arrays (coefficient arena, TB array).  Those arrays
// live until the host frees the picture; fresh multi-MB allocations come straight from mmap, and every
// first touch of their pages faults (measured: the coefficient arena's zeroing was ≈6 % of a parser
// thread's time, and the faults serialise the parser threads on the process's address-space lock).
// Blocks of at least kPoolMin bytes go back to a process-wide free list (bounded) and are reused.
void* pool_alloc(size_t bytes);
void pool_free(void* p);

template <class T>
struct PoolAlloc {
    using value_type = T;
    PoolAlloc() = default;
    template <class U> PoolAlloc(const PoolAlloc<U>&) {}
    template <class U> struct rebind { using other = PoolAlloc<U>; };
    T* allocate(size_t n) { return static_cast<T*>(pool_alloc(n * sizeof(T))); }
    void deallocate(T* p, size_t) { pool_free(p); }
    // value-less construct() leaves the element uninitialised (resize() does not touch the pages)
    template <class U> void construct(U* p) { ::new (static_cast<void*>(p)) U; }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
    template <class U> bool operator==(const PoolAlloc<U>&) const { return true; }
    template <class U> bool operator!=(const PoolAlloc<U>&) const { return false; }
};

struct PictureRecords {
    std::vector<p265r_ctu> ctus;      // raster order
    std::vector<p265r_tb, PoolAlloc<p265r_tb>> tbs;        // grouped by CTU (raster), decode order inside a CTU
    std::vector<int16_t, PoolAlloc<int16_t>> coef;         // decode order
    std::vector<uint8_t> nofilter;    // empty = none
    uint32_t n_cus = 0;
};

struct SliceRef {
    const SliceHeader* hdr;
    const uint8_t* rbsp;
    size_t size;
};

// Decode every slice segment of one picture (in decode order) into records.
// Throws BitstreamError / Unsupported.
void decode_picture(const Active& act, const std::vector<SliceRef>& slices, PictureRecords& out);

// Context-variable initialization values (Tables 9-5..9-37, initType 0 = I slices), exposed
// for the tests' parity with decoder/cabac.py:13-63.
int context_init_values(const uint8_t** vals);

}  // namespace p265fe
