// HBM bandwidth probe (tools only, not part of the library): streaming copy / read / write
// kernels with 16-B accesses per lane, timed with HIP events, to compare the memory-bound phases
// (residual, SAO) with what the box's HBM actually delivers for a plain stream, and to pick the copy
// form libp265probe.so's ceiling uses.
//   hipcc -O3 --offload-arch=gfx950 -o tools/bw_probe tools/bw_probe.hip && tools/bw_probe [GiB]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy_k(const u4* __restrict__ a, u4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}
__global__ __launch_bounds__(256) void copy_unroll_k(const u4* __restrict__ a, u4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const u4 x0 = a[i], x1 = a[i + stride], x2 = a[i + 2 * stride], x3 = a[i + 3 * stride];
        b[i] = x0; b[i + stride] = x1; b[i + 2 * stride] = x2; b[i + 3 * stride] = x3;
    }
    for (; i < n; i += stride) b[i] = a[i];
}
// one contiguous chunk per workgroup (no grid stride): block b copies [b * per, (b + 1) * per)
template <int U>
__global__ __launch_bounds__(256) void copy_chunk_k(const u4* __restrict__ a, u4* __restrict__ b, size_t n, size_t per) {
    const size_t lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
    for (size_t i = lo + threadIdx.x; i < hi; i += 256 * U) {
        u4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + 256 * u < hi) x[u] = a[i + 256 * u];
#pragma unroll
        for (int u = 0; u < U; ++u) if (i + 256 * u < hi) b[i + 256 * u] = x[u];
    }
}
__global__ __launch_bounds__(256) void copy_nt_k(const u4* __restrict__ a, u4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256;
    size_t i = blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const u4 x0 = __builtin_nontemporal_load(a + i), x1 = __builtin_nontemporal_load(a + i + stride);
        const u4 x2 = __builtin_nontemporal_load(a + i + 2 * stride), x3 = __builtin_nontemporal_load(a + i + 3 * stride);
        __builtin_nontemporal_store(x0, b + i); __builtin_nontemporal_store(x1, b + i + stride);
        __builtin_nontemporal_store(x2, b + i + 2 * stride); __builtin_nontemporal_store(x3, b + i + 3 * stride);
    }
    for (; i < n; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}
__global__ __launch_bounds__(256) void read_k(const u4* __restrict__ a, u4* __restrict__ sink, size_t n) {
    u4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= a[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}
__global__ __launch_bounds__(256) void write_k(u4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = u4{1, 2, 3, 4};
}
__global__ __launch_bounds__(256) void write_nt_k(u4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        __builtin_nontemporal_store(u4{1, 2, 3, (unsigned)i}, b + i);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
    const size_t gib = argc > 1 ? (size_t)atoi(argv[1]) : 2;
    const size_t bytes = gib << 30, n = bytes / 16;
    u4 *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    static const char* names[] = {"copy", "copy x4", "copy nt", "chunk x4", "chunk x8", "read", "write", "write nt"};
    const int grids[] = {cus, cus * 2, cus * 4, cus * 8, cus * 16, cus * 32};
    for (int k = 0; k < 8; ++k) {
        for (int gi = 0; gi < 6; ++gi) {
            const int grid = grids[gi];
            const size_t per = (n + grid - 1) / grid;
            float best = 1e30f;
            for (int rep = 0; rep < 6; ++rep) {
                CK(hipEventRecord(e0, 0));
                switch (k) {
                    case 0: copy_k<<<grid, 256>>>(a, b, n); break;
                    case 1: copy_unroll_k<<<grid, 256>>>(a, b, n); break;
                    case 2: copy_nt_k<<<grid, 256>>>(a, b, n); break;
                    case 3: copy_chunk_k<4><<<grid, 256>>>(a, b, n, per); break;
                    case 4: copy_chunk_k<8><<<grid, 256>>>(a, b, n, per); break;
                    case 5: read_k<<<grid, 256>>>(a, b, n); break;
                    case 6: write_k<<<grid, 256>>>(b, n); break;
                    default: write_nt_k<<<grid, 256>>>(b, n); break;
                }
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep > 0 && ms < best) best = ms;
            }
            const double moved = (k <= 4 ? 2.0 : 1.0) * (double)bytes;
            printf("%zu GiB grid %6d (%2d/CU)  %-9s %7.3f ms  %7.1f GB/s\n", gib, grid, grid / cus, names[k], best,
                   moved / (best * 1e-3) / 1e9);
        }
    }
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipEventRecord(e0, 0));
        CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0));
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
    }
    printf("hipMemcpy D2D        %7.3f ms  %7.1f GB/s\n", best, 2.0 * bytes / (best * 1e-3) / 1e9);
    return 0;
}
