// Host-side exhaustive check: ref_avail_mask() == the unit-by-unit nb_available_wh() loop.
// Build + run (CPU only): hipcc --offload-arch=gfx950 -O2 tools/avail_check.hip -o /tmp/avail_check && /tmp/avail_check
#include <cstdio>
#include "../p265_amd/csrc/intra.h"
using namespace p265r;

int main() {
    long long checked = 0, bad = 0, bad32 = 0;
    for (int ctb_log2 = 4; ctb_log2 <= 6; ++ctb_log2) {
        const int ctb = 1 << ctb_log2;
        for (int c = 0; c < 2; ++c)
            for (int lg = 2; lg <= 5; ++lg) {
                const int n = 1 << lg, sub = c ? 1 : 0;
                if ((n << sub) > ctb || (c && lg == 5)) continue;
                for (int yr = 0; (yr << sub) < ctb; yr += n)
                    for (int xr = 0; (xr << sub) < ctb; xr += n)
                        for (unsigned flags = 0; flags < 16; ++flags)
                            for (int px = 0; px < 3; ++px)
                                for (int py = 0; py < 3; ++py) {
                                    // CTB origin and picture size: interior, or picture edge cutting the CTB
                                    const int x0 = 2 * ctb, y0 = 2 * ctb;
                                    const int w = px == 0 ? x0 + 4 * ctb : x0 + ((xr << sub) + (n << sub) + 8 * px) / 8 * 8;
                                    const int h = py == 0 ? y0 + 4 * ctb : y0 + ((yr << sub) + (n << sub) + 8 * py) / 8 * 8;
                                    if (x0 + (xr << sub) + (n << sub) > w || y0 + (yr << sub) + (n << sub) > h) continue;
                                    const int us_log = c ? 1 : 2, L = (2 * n) >> us_log;
                                    const int xc = xr << sub, yc = yr << sub;
                                    unsigned long long ref = 0;
                                    for (int u = 0; u <= 2 * L; ++u) {
                                        int dx, dy;
                                        if (u < L) { dx = -1; dy = 2 * n - 1 - (u << us_log); }
                                        else if (u == L) { dx = -1; dy = -1; }
                                        else { dx = (u - L - 1) << us_log; dy = -1; }
                                        if (nb_available_wh((xr + dx) << sub, (yr + dy) << sub, xc, yc, x0, y0, w, h, ctb, flags))
                                            ref |= 1ull << u;
                                    }
                                    const unsigned long long got = ref_avail_mask(c, xr, yr, n, x0, y0, w, h, ctb, flags);
                                    uint32_t hi32 = 0;
                                    const int s = __builtin_ctz((unsigned)(n << sub)) - 2;
                                    const uint32_t lo32 = ref_avail_mask32(c, xr, yr, n, x0, y0, w, h, ctb, flags,
                                                                           avail_ztab_word(s, yc >> 2), hi32);
                                    const unsigned long long got32 = (unsigned long long)lo32 | (unsigned long long)hi32 << 32;
                                    if (got32 != ref && bad32++ < 10)
                                        printf("MISMATCH32 ctb %d c %d n %d xr %d yr %d flags %u w %d h %d: %llx vs %llx\n", ctb, c,
                                               n, xr, yr, flags, w, h, got32, ref);
                                    ++checked;
                                    if (got != ref && bad++ < 10)
                                        printf("MISMATCH ctb %d c %d n %d xr %d yr %d flags %u w %d h %d: %llx vs %llx\n", ctb, c, n,
                                               xr, yr, flags, w, h, got, ref);
                                }
            }
    }
    printf("checked %lld, mismatches %lld\n", checked, bad + bad32);
    return (bad + bad32) ? 1 : 0;
}
