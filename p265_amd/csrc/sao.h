// SAO (H.265 8.7.3) helpers shared by the in-loop filter kernel (loopfilter.h).
//
// The reference only parses the SAO syntax (decoder/sao.py:15-136) and never filters
// a sample.  8.7.3.2: a sample's edge-offset neighbour in another CTB is usable only if
// that CTB is inside the picture, in the same tile (unless loop_filter_across_tiles),
// and - across slices - the slice containing the later of the two samples allows it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/p265r.h"
#include "intra.h"

namespace p265r {

__device__ __forceinline__ bool ts_before(const p265r_ctu& a, int ra, const p265r_ctu& b, int rb) {
    // CtbAddrRsToTs[a] < CtbAddrRsToTs[b]; tiles are numbered in tile-scan order
    return a.tile_id < b.tile_id || (a.tile_id == b.tile_id && ra < rb);
}

__device__ __forceinline__ int sgn(int v) { return (v > 0) - (v < 0); }

// may samples of CTB rs use samples of the neighbouring CTB (dx, dy)?  (8.7.3.2)
__device__ __forceinline__ bool sao_allow(const p265r_ctu* ctus, const p265r_ctu& me, int rs, int rx, int ry,
                                          int dx, int dy, const Geo& g) {
    const int nx = rx + dx, ny = ry + dy;
    if (nx < 0 || ny < 0 || nx >= g.wc || ny >= g.hc) return false;
    if (!dx && !dy) return true;
    const int ro = ny * g.wc + nx;
    const p265r_ctu o = ctus[ro];
    bool ok = true;
    if (o.slice_addr != me.slice_addr) {
        // the flag of the slice containing the LATER of the two samples
        ok = ts_before(o, ro, me, rs) ? (me.flags & P265R_CTU_LF_ACROSS_SLICES) != 0
                                      : (o.flags & P265R_CTU_LF_ACROSS_SLICES) != 0;
    }
    if (!g.lf_tiles && o.tile_id != me.tile_id) ok = false;
    return ok;
}

}  // namespace p265r
