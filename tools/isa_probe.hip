// ISA probe (not built by the Makefile): one fast job per loop iteration, to read the
// per-job instruction stream of recon_fast in isolation.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 --save-temps -c tools/isa_probe.hip
#include "../p265_amd/csrc/intra_rows.h"
using namespace p265r;
__global__ __launch_bounds__(64) void probe(const uint32_t* __restrict__ w, int n, const uint8_t* lt) {
    __shared__ WaveLds L;
    const int lane = threadIdx.x;
    for (int t = 0; t < n; ++t) {
        const uint32_t w0 = __builtin_amdgcn_readfirstlane(w[4 * t]), w1 = __builtin_amdgcn_readfirstlane(w[4 * t + 1]);
        const uint32_t w5 = __builtin_amdgcn_readfirstlane(w[4 * t + 2]);
        const int r16 = (int)w[4 * t + 3 + lane];
        recon_fast<2, false>(L, lt, w0, w1, w5, r16, lane);
    }
}
