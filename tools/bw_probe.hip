// HBM bandwidth probe (tools only, not part of the library): streaming copy / read / write
// kernels with 16-B accesses per lane, timed with HIP events, to compare the memory-bound phases
// (residual, SAO) with what the box's HBM actually delivers for a plain stream.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/bw_probe tools/bw_probe.hip && /tmp/bw_probe
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
__global__ __launch_bounds__(256) void read_k(const u4* __restrict__ a, u4* __restrict__ sink, size_t n) {
    u4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= a[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}
__global__ __launch_bounds__(256) void write_k(u4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = u4{1, 2, 3, 4};
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const size_t bytes = (size_t)2 << 30, n = bytes / 16;
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
    const int grids[] = {cus * 4, cus * 8, cus * 16, cus * 32};
    for (int gi = 0; gi < 4; ++gi) {
        const int grid = grids[gi];
        for (int k = 0; k < 4; ++k) {
            float best = 1e30f;
            for (int rep = 0; rep < 6; ++rep) {
                CK(hipEventRecord(e0, 0));
                if (k == 0) copy_k<<<grid, 256>>>(a, b, n);
                else if (k == 1) copy_unroll_k<<<grid, 256>>>(a, b, n);
                else if (k == 2) read_k<<<grid, 256>>>(a, b, n);
                else write_k<<<grid, 256>>>(b, n);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep > 0 && ms < best) best = ms;
            }
            const double moved = (k <= 1 ? 2.0 : 1.0) * (double)bytes;
            static const char* names[] = {"copy", "copy x4", "read", "write"};
            printf("grid %6d  %-8s %7.3f ms  %7.1f GB/s\n", grid, names[k], best, moved / (best * 1e-3) / 1e9);
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
