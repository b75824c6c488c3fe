// ISA probe (not built by the Makefile): one job per loop iteration, to read the per-job
// instruction stream of a job kind in isolation (PROBE = 0 luma quad, 1 chroma quad,
// 2 fast luma 8x8, 3 fast luma 16x16).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S -DPROBE=0 tools/isa_probe.hip
#include "../p265_amd/csrc/intra_rows.h"
using namespace p265r;
#ifndef PROBE
#define PROBE 0
#endif
__global__ __launch_bounds__(64) void probe(const uint32_t* __restrict__ w, int n, uint32_t lt) {
    extern __shared__ unsigned char smem[];
    const int lane = threadIdx.x;
    const uint32_t lbase = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)smem;
    const uint32_t tab = lbase + 8192u;   // AngTab4 stand-in
    for (int t = 0; t < n; ++t) {
        const uint32_t w0 = __builtin_amdgcn_readfirstlane(w[8 * t]), w1 = __builtin_amdgcn_readfirstlane(w[8 * t + 1]);
        const uint32_t w2 = __builtin_amdgcn_readfirstlane(w[8 * t + 2]), w5 = __builtin_amdgcn_readfirstlane(w[8 * t + 3]);
        const int r16 = (int)w[8 * t + 64 + lane];
#if PROBE == 0
        recon_quad<false>(lbase, lt, 0u, w0, w1, w2, tab, r16, lane);
#elif PROBE == 1
        recon_quad<true>(lbase, lt, 960u, w0, w1, w2, tab, r16, lane);
#elif PROBE == 2
        recon_fast<3, false>(lbase, lt, w0, w1, w5, r16, lane, tab);
#else
        recon_fast16(lbase, lt, w0, w1, w5, make_uint4(r16, r16, 0, 0), lane);
#endif
    }
}
