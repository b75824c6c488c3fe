// issue_probe.hip -- measured instruction-issue ceiling of the row kernel's job loop (bench.py
// "issue" block).  Not part of the product path: libp265probe.so, loaded by bench.py.
//
// The row kernel (intra_rows.h) is said to be bound by instruction issue: per job its waves issue
// V VALU, S SALU and L LDS instructions (rocprofv3 SQ_INSTS_* / jobs), 24 waves per CU (two W = 12
// workgroups, 6 per SIMD).  This kernel issues exactly that mix per "job" with NO dependency
// between instructions (four independent VGPR / SGPR chains, LDS reads waited for once per job, as
// a job waits for its last LDS result), at the same occupancy, and measures cycles per job and CU
// with s_memtime.  Its result is the issue ceiling of the mix: the fastest the row kernel could run
// if latency and dependencies cost nothing.  The row kernel's own cycles per job and CU divided by
// this ceiling say how much of its time is issue.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace {

template <int V, int S, int L>
__device__ __forceinline__ void job_mix(uint32_t (&v)[4], uint32_t (&s)[4], uint32_t lds_addr) {
    constexpr int N = V > S ? (V > L ? V : L) : (S > L ? S : L);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if (i < V) asm volatile("v_add_u32 %0, %0, 1" : "+v"(v[i & 3]));
        if (i * S / N < (i + 1) * S / N) asm volatile("s_add_u32 %0, %0, 1" : "+s"(s[i & 3]) :: "scc");
        if (i * L / N < (i + 1) * L / N) {
            uint32_t r;   // (never read: the job's one wait below stands for its uses)
            asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(lds_addr) : "memory");
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// 64 * W threads per workgroup, WPE waves per SIMD (the row kernel's occupancy: two W = 12
// workgroups per CU at 80 VGPRs); out[block * W + wave] = cycles of this wave over `jobs` jobs
template <int V, int S, int L, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(6))) void issue_probe_kernel(int jobs, uint32_t* out,
                                                                                                     uint32_t* sink) {
    __shared__ uint32_t buf[64 * W];
    buf[threadIdx.x] = threadIdx.x;
    __syncthreads();
    uint32_t v[4] = {threadIdx.x, threadIdx.x + 1, threadIdx.x + 2, threadIdx.x + 3};
    uint32_t s[4] = {0, 1, 2, 3};
    const uint32_t a = (uint32_t)(uintptr_t)&buf[threadIdx.x];
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < jobs; ++j) job_mix<V, S, L>(v, s, a);
    const long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * W + (threadIdx.x >> 6)] = (uint32_t)(t1 - t0);
    if (v[0] + v[1] + v[2] + v[3] + s[0] + s[1] + s[2] + s[3] == 0x7fffffffu) sink[0] = 1;   // keep the chains live
}

template <int V, int S, int L>
int run(int device, int jobs, double* cycles_per_job_cu, double* ms) {
    constexpr int W = 12;
    if (hipSetDevice(device) != hipSuccess) return -3;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return -3;
    const int grid = 2 * cus;                          // two workgroups per CU, as the row kernel
    uint32_t *out = nullptr, *sink = nullptr;
    if (hipMalloc(&out, sizeof(uint32_t) * grid * W) != hipSuccess) return -2;
    if (hipMalloc(&sink, sizeof(uint32_t)) != hipSuccess) { (void)hipFree(out); return -2; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    issue_probe_kernel<V, S, L, W><<<grid, 64 * W>>>(jobs / 8, out, sink);          // warm-up (clocks, code)
    (void)hipEventRecord(e0, nullptr);
    issue_probe_kernel<V, S, L, W><<<grid, 64 * W>>>(jobs, out, sink);
    (void)hipEventRecord(e1, nullptr);
    hipError_t e = hipEventSynchronize(e1);
    float t = 0;
    if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
    uint32_t* h = new uint32_t[grid * W];
    if (e == hipSuccess) e = hipMemcpy(h, out, sizeof(uint32_t) * grid * W, hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < grid * W && e == hipSuccess; ++i) mx = h[i] > mx ? h[i] : mx;
    delete[] h;
    (void)hipFree(out);
    (void)hipFree(sink);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (e != hipSuccess) return -3;
    // the CU runs 2 x W waves, each `jobs` jobs: CU-cycles per job = wave cycles / (2 W)
    *cycles_per_job_cu = mx / jobs / (2.0 * W);
    *ms = t;
    return 0;
}

// ---- achievable HBM stream rates (bench.py roofline.achievable): 16 B per lane; the fastest of a few
// copy / read / write forms and grids measured on the box (tools/bw_probe.hip: grid-stride plain copy at
// 8-32 workgroups per CU, one contiguous chunk per workgroup with 4 loads in flight per lane at 1-4 per
// CU; non-temporal stores for the write).  What the bandwidth-bound phases (residual, SAO) are compared
// against; the guide quotes 6.29 TB/s for a float4 copy (MI355X_MICROARCH.md).
typedef unsigned int probe_u4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void copy_probe_kernel(const probe_u4* __restrict__ a, probe_u4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}
__global__ __launch_bounds__(256) void copy_chunk_probe_kernel(const probe_u4* __restrict__ a, probe_u4* __restrict__ b,
                                                               size_t n, size_t per) {
    const size_t lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
    for (size_t i = lo + threadIdx.x; i < hi; i += 256 * 4) {
        probe_u4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) if (i + 256 * u < hi) x[u] = a[i + 256 * u];
#pragma unroll
        for (int u = 0; u < 4; ++u) if (i + 256 * u < hi) b[i + 256 * u] = x[u];
    }
}
__global__ __launch_bounds__(256) void read_probe_kernel(const probe_u4* __restrict__ a, probe_u4* __restrict__ sink, size_t n) {
    probe_u4 acc = {0u, 0u, 0u, 0u};
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= a[i];
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;
}
__global__ __launch_bounds__(256) void write_probe_kernel(probe_u4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        __builtin_nontemporal_store(probe_u4{1u, 2u, 3u, (unsigned)i}, b + i);
}

}  // namespace

extern "C" {

// Best rate over the forms above (5 timed repetitions each, after one warm-up) of a copy (read + write
// bytes), a read and a write of `bytes`-sized buffers, in GB/s.  Returns 0, or < 0 on a HIP error /
// allocation failure.
int p265probe_stream(int device, double bytes, double* copy_gbs, double* read_gbs, double* write_gbs) {
    if (!copy_gbs || !read_gbs || !write_gbs || bytes < (1 << 20)) return -1;
    if (hipSetDevice(device) != hipSuccess) return -3;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return -3;
    const size_t nb = (size_t)bytes / 16 * 16, n = nb / 16;
    probe_u4 *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, nb) != hipSuccess) return -2;
    if (hipMalloc(&b, nb) != hipSuccess) { (void)hipFree(a); return -2; }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipError_t e = hipMemset(a, 1, nb);
    if (e == hipSuccess) e = hipMemset(b, 0, nb);
    double best[3] = {0, 0, 0};
    // (kind, workgroups per CU): copy plain 8 / 16 / 32, copy chunked 1 / 2 / 4, read 8 / 16 / 32, write 4 / 8 / 16
    const int forms[12][2] = {{0, 8}, {0, 16}, {0, 32}, {1, 1}, {1, 2}, {1, 4}, {2, 8}, {2, 16}, {2, 32}, {3, 4}, {3, 8}, {3, 16}};
    for (int f = 0; f < 12 && e == hipSuccess; ++f) {
        const int kind = forms[f][0], grid = forms[f][1] * cus;
        const size_t per = (n + grid - 1) / grid;
        for (int rep = 0; rep < 6 && e == hipSuccess; ++rep) {
            (void)hipEventRecord(e0, nullptr);
            switch (kind) {
                case 0: copy_probe_kernel<<<grid, 256>>>(a, b, n); break;
                case 1: copy_chunk_probe_kernel<<<grid, 256>>>(a, b, n, per); break;
                case 2: read_probe_kernel<<<grid, 256>>>(a, b, n); break;
                default: write_probe_kernel<<<grid, 256>>>(b, n); break;
            }
            (void)hipEventRecord(e1, nullptr);
            e = hipEventSynchronize(e1);
            float ms = 0;
            if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
            const int k = kind <= 1 ? 0 : kind - 1;
            const double moved = (k == 0 ? 2.0 : 1.0) * (double)nb;
            if (e == hipSuccess && rep > 0 && ms > 0) best[k] = std::max(best[k], moved / (ms * 1e-3) / 1e9);
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(a);
    (void)hipFree(b);
    if (e != hipSuccess) return -3;
    *copy_gbs = best[0]; *read_gbs = best[1]; *write_gbs = best[2];
    return 0;
}

// which: 0 = the round-5 row-kernel mix (VALU 131, SALU 81, LDS 15 per job), 1 = its VALU alone,
// 2 = its SALU alone, 3 = its LDS alone.  -> CU-cycles per job (s_memtime, the slowest wave) and the
// launch time.  Returns 0, or < 0 on a HIP error.
int p265probe_issue(int device, int which, int jobs, double* cycles_per_job_cu, double* ms) {
    if (!cycles_per_job_cu || !ms || jobs < 8) return -1;
    switch (which) {
        case 0: return run<131, 81, 15>(device, jobs, cycles_per_job_cu, ms);
        case 1: return run<131, 0, 0>(device, jobs, cycles_per_job_cu, ms);
        case 2: return run<0, 81, 0>(device, jobs, cycles_per_job_cu, ms);
        case 3: return run<0, 0, 15>(device, jobs, cycles_per_job_cu, ms);
        default: return -1;
    }
}

}  // extern "C"
