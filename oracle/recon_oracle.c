/*
 * recon_oracle.c -- scalar C restatement of the HEVC intra reconstruction path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/recon_oracle.py for the policy): used by
 * tests/ as a fast checker at full picture sizes and by bench.py as the timed CPU
 * baseline ("kind": "port").  Never linked into libp265r.so.
 *
 * Same algorithm as oracle/recon_oracle.py, written independently of the HIP code:
 * spec-form availability (6.4.1, global MinTbAddrZs), substitution (8.4.4.2.2),
 * filtering (8.4.4.2.3), planar/DC/angular (8.4.4.2.4-6), scaling (8.6.3), inverse
 * DCT/DST as plain O(N^3) matrix products (8.6.4.2), residual (8.6.2), construction
 * (8.6.7), deblocking (8.7.2) and SAO (8.7.3).  Reference file:line for each piece: see
 * the Python twin.
 *
 * Build: make -C oracle   ->  oracle/build/liboracle_p265.so
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/p265r.h"

#ifdef _OPENMP
#include <omp.h>
#endif

static const int COS64[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                              61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};
static const int DST4[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};
static const int ANGLE[35] = {0,  0,  32, 26, 21, 17, 13, 9,  5,  2,  0,  -2, -5, -9, -13, -17, -21, -26,
                              -32, -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32};
static const int INVANG[35] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, -4096, -1638, -910, -630, -482, -390, -315,
                               -256, -315, -390, -482, -630, -910, -1638, -4096, 0, 0, 0, 0, 0, 0, 0, 0, 0};
static const int LEVEL_SCALE[6] = {40, 45, 51, 57, 64, 72};

static int DCT[32][32];
static int dct_ready = 0;

static void init_dct(void) {
    if (dct_ready) return;
    for (int k = 0; k < 32; ++k)
        for (int n = 0; n < 32; ++n) {
            int a = (k * (2 * n + 1)) % 128, v;
            if (k == 0) v = 64;
            else if (a <= 32) v = COS64[a];
            else if (a < 64) v = -COS64[64 - a];
            else if (a <= 96) v = -COS64[a - 64];
            else v = COS64[128 - a];
            DCT[k][n] = v;
        }
    dct_ready = 1;
}

static inline int clip3(int lo, int hi, long long v) { return v < lo ? lo : (v > hi ? hi : (int)v); }

typedef struct {
    int w, h, ctb_log2, ctb, wc, hc, mintb_log2, shift;
    const p265r_ctu* ctus;
    int* rs2ts;
} geo_t;

static void geo_init(geo_t* g, const p265r_params* p, const p265r_ctu* ctus, int* rs2ts) {
    g->w = p->pic_width; g->h = p->pic_height;
    g->ctb_log2 = p->ctb_log2_size; g->ctb = 1 << g->ctb_log2;
    g->wc = (g->w + g->ctb - 1) >> g->ctb_log2; g->hc = (g->h + g->ctb - 1) >> g->ctb_log2;
    g->mintb_log2 = p->min_tb_log2_size; g->shift = g->ctb_log2 - g->mintb_log2;
    g->ctus = ctus; g->rs2ts = rs2ts;
    /* tile-scan order = (tile_id, raster) lexicographic */
    const int n = g->wc * g->hc;
    int ts = 0, max_tile = 0;
    for (int i = 0; i < n; ++i) if (ctus[i].tile_id > max_tile) max_tile = ctus[i].tile_id;
    for (int t = 0; t <= max_tile; ++t)
        for (int i = 0; i < n; ++i) if (ctus[i].tile_id == t) rs2ts[i] = ts++;
}

static inline int ctb_of(const geo_t* g, int x, int y) { return (y >> g->ctb_log2) * g->wc + (x >> g->ctb_log2); }

static inline long long min_tb_addr_zs(const geo_t* g, int x, int y) {
    const int m = g->ctb - 1;
    const int tx = (x & m) >> g->mintb_log2, ty = (y & m) >> g->mintb_log2;
    long long v = 0;
    for (int i = 0; i < g->shift; ++i) {
        const int b = 1 << i;
        v += ((tx & b) ? (long long)b * b : 0) + ((ty & b) ? 2LL * b * b : 0);
    }
    return ((long long)g->rs2ts[ctb_of(g, x, y)] << (2 * g->shift)) + v;
}

/* 6.4.1 z-scan availability (decoder/image.py:38-73) */
static int available(const geo_t* g, int xc, int yc, int xn, int yn) {
    if (xn < 0 || yn < 0 || xn >= g->w || yn >= g->h) return 0;
    if (min_tb_addr_zs(g, xn, yn) > min_tb_addr_zs(g, xc, yc)) return 0;
    const int a = ctb_of(g, xc, yc), b = ctb_of(g, xn, yn);
    if (a != b && (g->ctus[a].slice_addr != g->ctus[b].slice_addr || g->ctus[a].tile_id != g->ctus[b].tile_id))
        return 0;
    return 1;
}

/* residual r[y*n+x] of one TB (8.6.2-8.6.4); m: the TB's ScalingFactor m[y*n+x] (NULL: flat 16) */
static void residual(const int16_t* lvl, int log2, int c, int qp, int flags, int bd, const uint8_t* m, int* r) {
    const int n = 1 << log2, nn = n * n;
    if (flags & (P265R_TB_BYPASS | P265R_TB_PCM)) {
        for (int i = 0; i < nn; ++i) r[i] = lvl[i];
        return;
    }
    int d[1024];
    const int bds = bd + log2 - 5;
    for (int i = 0; i < nn; ++i) {
        long long v = ((long long)lvl[i] * (m ? m[i] : 16) * LEVEL_SCALE[qp % 6]) << (qp / 6);
        d[i] = clip3(-32768, 32767, (v + (1LL << (bds - 1))) >> bds);
    }
    const int bd2 = 20 - bd;
    if (flags & P265R_TB_TSKIP) {
        for (int i = 0; i < nn; ++i) r[i] = (int)((((long long)d[i] << (5 + log2)) + (1 << (bd2 - 1))) >> bd2);
        return;
    }
    const int dst = (log2 == 2 && c == 0);
    const int step = 1 << (5 - log2);
    int g[1024];
    for (int x = 0; x < n; ++x)          /* columns: e[y][x] = sum_j T[j][y] d[j][x] */
        for (int y = 0; y < n; ++y) {
            long long e = 0;
            for (int j = 0; j < n; ++j) e += (long long)(dst ? DST4[j][y] : DCT[j * step][y]) * d[j * n + x];
            g[y * n + x] = clip3(-32768, 32767, (e + 64) >> 7);
        }
    for (int y = 0; y < n; ++y)          /* rows */
        for (int x = 0; x < n; ++x) {
            long long e = 0;
            for (int j = 0; j < n; ++j) e += (long long)(dst ? DST4[j][x] : DCT[j * step][x]) * g[y * n + j];
            r[y * n + x] = (int)((e + (1 << (bd2 - 1))) >> bd2);
        }
}

/* linear reference array order: k<2n: p[-1][2n-1-k]; k=2n: p[-1][-1]; k>2n: p[k-2n-1][-1] */
static void predict(const int* p, int n, int mode, int c, int bd, int* pred) {
    const int log2 = n == 4 ? 2 : n == 8 ? 3 : n == 16 ? 4 : 5;
    const int maxv = (1 << bd) - 1;
#define LEFT(yy) p[2 * n - 1 - (yy)]
#define TOP(xx) p[2 * n + 1 + (xx)]
    if (mode == 0) {
        for (int y = 0; y < n; ++y)
            for (int x = 0; x < n; ++x)
                pred[y * n + x] = ((n - 1 - x) * LEFT(y) + (x + 1) * TOP(n) + (n - 1 - y) * TOP(x) + (y + 1) * LEFT(n) + n) >>
                                  (log2 + 1);
        return;
    }
    if (mode == 1) {
        int s = n;
        for (int i = 0; i < n; ++i) s += TOP(i) + LEFT(i);
        const int dc = s >> (log2 + 1);
        for (int i = 0; i < n * n; ++i) pred[i] = dc;
        if (c == 0 && n < 32) {
            pred[0] = (LEFT(0) + 2 * dc + TOP(0) + 2) >> 2;
            for (int x = 1; x < n; ++x) pred[x] = (TOP(x) + 3 * dc + 2) >> 2;
            for (int y = 1; y < n; ++y) pred[y * n] = (LEFT(y) + 3 * dc + 2) >> 2;
        }
        return;
    }
    const int ang = ANGLE[mode], vert = mode >= 18;
    int refbuf[3 * 64 + 1];
    int* ref = refbuf + 64;             /* ref[-64 .. 128] */
    for (int x = 0; x <= 2 * n; ++x) ref[x] = vert ? TOP(x - 1) : LEFT(x - 1);
    if (ang < 0 && ((n * ang) >> 5) < -1) {
        const int inv = INVANG[mode];
        for (int x = (n * ang) >> 5; x < 0; ++x) {
            const int k = -1 + ((x * inv + 128) >> 8);
            ref[x] = vert ? LEFT(k) : TOP(k);
        }
    }
    for (int a = 0; a < n; ++a) {
        const int idx = ((a + 1) * ang) >> 5, fact = ((a + 1) * ang) & 31;
        for (int b = 0; b < n; ++b) {
            int v = fact ? ((32 - fact) * ref[b + idx + 1] + fact * ref[b + idx + 2] + 16) >> 5 : ref[b + idx + 1];
            if (vert) pred[a * n + b] = v;
            else pred[b * n + a] = v;
        }
    }
    if (c == 0 && n < 32) {
        if (mode == 26)
            for (int y = 0; y < n; ++y) pred[y * n] = clip3(0, maxv, TOP(0) + ((LEFT(y) - LEFT(-1)) >> 1));
        if (mode == 10)
            for (int x = 0; x < n; ++x) pred[x] = clip3(0, maxv, LEFT(0) + ((TOP(x) - TOP(-1)) >> 1));
    }
#undef LEFT
#undef TOP
}

/* Sample planes are uint16_t inside the oracle whatever the bit depth (8..12); the caller's planes are
 * uint8_t for BitDepth 8 and uint16_t (little-endian) above (p265r_picture). */
typedef uint16_t pel;

/* byte offset of the intra ScalingFactor of (log2 size, component) in the 2032-byte array
 * (include/p265r.h p265r_set_scaling_factors) */
static int sf_offset(int log2, int c) {
    static const int OFF[4][3] = {{0, 16, 32}, {48, 112, 176}, {240, 496, 752}, {1008, -1, -1}};
    return OFF[log2 - 2][c];
}

static void recon_tb(const geo_t* g, const p265r_params* prm, const uint8_t* sf, pel* planes[3], const int stride[3],
                     const p265r_tb* t, const int16_t* coef) {
    const int c = t->c_idx, log2 = t->log2_size, n = 1 << log2, sub = c ? 1 : 0;
    const int bd = c ? prm->bit_depth_chroma : prm->bit_depth_luma;
    const int maxv = (1 << bd) - 1;
    const int x0 = t->x, y0 = t->y;
    pel* pl = planes[c];
    const int st = stride[c];
    int res[1024], pred[1024];
    if (t->flags & (P265R_TB_CBF | P265R_TB_PCM))
        residual(coef + t->coef_off, log2, c, t->qp, t->flags, bd, sf ? sf + sf_offset(log2, c) : NULL, res);
    else memset(res, 0, sizeof(int) * n * n);
    if (t->flags & P265R_TB_PCM) {
        memset(pred, 0, sizeof(int) * n * n);
    } else {
        const int nref = 4 * n + 1;
        int p[129], av[129], any = 0;
        for (int k = 0; k < nref; ++k) {
            const int dx = k <= 2 * n ? -1 : k - 2 * n - 1;
            const int dy = k < 2 * n ? 2 * n - 1 - k : -1;
            av[k] = available(g, x0 << sub, y0 << sub, (x0 + dx) << sub, (y0 + dy) << sub);
            p[k] = av[k] ? pl[(y0 + dy) * st + x0 + dx] : 0;
            any |= av[k];
        }
        if (!any) {
            for (int k = 0; k < nref; ++k) p[k] = 1 << (bd - 1);
        } else {
            if (!av[0]) {
                int k = 1;
                while (!av[k]) ++k;
                p[0] = p[k];
            }
            for (int k = 1; k < nref; ++k) if (!av[k]) p[k] = p[k - 1];
        }
        int filt = 0;
        if (c == 0 && t->pred_mode != 1 && n != 4) {
            const int m = t->pred_mode;
            const int dist = abs(m - 26) < abs(m - 10) ? abs(m - 26) : abs(m - 10);
            filt = dist > (n == 8 ? 7 : n == 16 ? 1 : 0);
        }
        if (filt) {
            int f[129];
            const int corner = p[2 * n], bl = p[0], tr = p[4 * n];
            if (prm->strong_intra_smoothing && n == 32 && abs(corner + tr - 2 * p[3 * n]) < (1 << (bd - 5)) &&
                abs(corner + bl - 2 * p[n]) < (1 << (bd - 5))) {
                f[2 * n] = corner;
                for (int y = 0; y < 63; ++y) f[2 * n - 1 - y] = ((63 - y) * corner + (y + 1) * bl + 32) >> 6;
                f[0] = bl;
                for (int x = 0; x < 63; ++x) f[2 * n + 1 + x] = ((63 - x) * corner + (x + 1) * tr + 32) >> 6;
                f[4 * n] = tr;
            } else {
                f[0] = p[0];
                f[4 * n] = p[4 * n];
                for (int k = 1; k < 4 * n; ++k) f[k] = (p[k - 1] + 2 * p[k] + p[k + 1] + 2) >> 2;
            }
            memcpy(p, f, sizeof(int) * nref);
        }
        predict(p, n, t->pred_mode, c, bd, pred);
    }
    for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x) pl[(y0 + y) * st + x0 + x] = (pel)clip3(0, maxv, (long long)pred[y * n + x] + res[y * n + x]);
}

static inline int sgn(int v) { return (v > 0) - (v < 0); }

static void sao(const geo_t* g, const p265r_params* prm, const p265r_picture* pic, pel* rec[3], pel* out[3],
                const int stride[3]) {
    const int nfw = (g->w + 7) / 8;
    for (int rs = 0; rs < g->wc * g->hc; ++rs) {
        const p265r_ctu* me = &g->ctus[rs];
        const int rx = rs % g->wc, ry = rs / g->wc;
        int allow[9];
        for (int i = 0; i < 9; ++i) {
            const int dx = i % 3 - 1, dy = i / 3 - 1, nx = rx + dx, ny = ry + dy;
            int ok = 1;
            if (nx < 0 || ny < 0 || nx >= g->wc || ny >= g->hc) ok = 0;
            else if (dx || dy) {
                const int ro = ny * g->wc + nx;
                const p265r_ctu* o = &g->ctus[ro];
                if (o->slice_addr != me->slice_addr)
                    ok = g->rs2ts[ro] < g->rs2ts[rs] ? (me->flags & P265R_CTU_LF_ACROSS_SLICES) != 0
                                                     : (o->flags & P265R_CTU_LF_ACROSS_SLICES) != 0;
                if (!prm->loop_filter_across_tiles && o->tile_id != me->tile_id) ok = 0;
            }
            allow[i] = ok;
        }
        for (int c = 0; c < 3; ++c) {
            const int sub = c ? 1 : 0, cs = g->ctb >> sub;
            const int W = g->w >> sub, H = g->h >> sub;
            const int xb = rx * cs, yb = ry * cs;
            const int x1 = xb + cs < W ? xb + cs : W, y1 = yb + cs < H ? yb + cs : H;
            const int typ = me->sao_type[c];
            const int bd = c ? prm->bit_depth_chroma : prm->bit_depth_luma, maxv = (1 << bd) - 1;
            const int off[5] = {0, me->sao_offset[c][0], me->sao_offset[c][1], me->sao_offset[c][2], me->sao_offset[c][3]};
            const int cls = me->sao_class[c];
            static const int EO[4][4] = {{-1, 0, 1, 0}, {0, -1, 0, 1}, {-1, -1, 1, 1}, {1, -1, -1, 1}};
            for (int y = yb; y < y1; ++y)
                for (int x = xb; x < x1; ++x) {
                    const int v = rec[c][y * stride[c] + x];
                    int r = v;
                    int skip = typ == 0;
                    if (!skip && pic->nofilter) skip = pic->nofilter[((y << sub) >> 3) * nfw + ((x << sub) >> 3)] != 0;
                    if (!skip && typ == 1) {
                        int table[32] = {0};
                        for (int k = 0; k < 4; ++k) table[(k + cls) & 31] = k + 1;
                        r = clip3(0, maxv, v + off[table[v >> (bd - 5)]]);
                    } else if (!skip) {
                        const int xa = x + EO[cls][0], ya = y + EO[cls][1], xc = x + EO[cls][2], yc = y + EO[cls][3];
                        int ok = xa >= 0 && ya >= 0 && xa < W && ya < H && xc >= 0 && yc >= 0 && xc < W && yc < H;
                        if (ok) {
                            const int da = (xa < xb ? 0 : xa >= xb + cs ? 2 : 1) + 3 * (ya < yb ? 0 : ya >= yb + cs ? 2 : 1);
                            const int dc = (xc < xb ? 0 : xc >= xb + cs ? 2 : 1) + 3 * (yc < yb ? 0 : yc >= yb + cs ? 2 : 1);
                            ok = allow[da] && allow[dc];
                        }
                        if (ok) {
                            int e = 2 + sgn(v - rec[c][ya * stride[c] + xa]) + sgn(v - rec[c][yc * stride[c] + xc]);
                            e = e == 2 ? 0 : (e < 2 ? e + 1 : e);
                            r = clip3(0, maxv, v + off[e]);
                        }
                    }
                    out[c][y * stride[c] + x] = (pel)r;
                }
        }
    }
}

/* ---- deblocking (8.7.2; all-intra: bS = 2 on transform-block edges of the 8x8 grid) ---- */
static const int BETA_T[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                               8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                               34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
static const int TC_T[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                             2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

static int qpc_of(int qpi) {
    static const int T[14] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37, 37};
    return qpi < 30 ? qpi : (qpi >= 43 ? qpi - 6 : T[qpi - 30]);
}
static inline int nib(int v) { return v >= 8 ? v - 16 : v; }

typedef struct {
    const geo_t* g;
    const p265r_params* prm;
    const uint8_t* nofilter;
    int nfw, w4;
    uint32_t* org;   /* per 4x4 luma unit: origin (x | y << 16) of the luma TB covering it */
    int16_t* qpy;    /* per 4x4 luma unit: QpY (negative down to -QpBdOffsetY above 8 bits)  */
    int bdl, bdc;    /* BitDepthY, BitDepthC                                             */
} dbk_t;

/* bS == 2 && filterEdgeFlag for the edge between luma samples p0 (xp,yp) and q0 (xq,yq) */
static int dbk_edge(const dbk_t* d, int xp, int yp, int xq, int yq) {
    if (d->org[(yp >> 2) * d->w4 + (xp >> 2)] == d->org[(yq >> 2) * d->w4 + (xq >> 2)]) return 0;
    const geo_t* g = d->g;
    const int a = ctb_of(g, xq, yq), b = ctb_of(g, xp, yp);
    const p265r_ctu* cq = &g->ctus[a];
    if (!(cq->flags & P265R_CTU_DEBLOCK)) return 0;
    if (a != b) {
        if (!d->prm->loop_filter_across_tiles && g->ctus[b].tile_id != cq->tile_id) return 0;
        if (g->ctus[b].slice_addr != cq->slice_addr && !(cq->flags & P265R_CTU_LF_ACROSS_SLICES)) return 0;
    }
    return 1;
}
static inline int dbk_nf(const dbk_t* d, int x, int y) { return d->nofilter && d->nofilter[(y >> 3) * d->nfw + (x >> 3)]; }
static inline int dbk_qp(const dbk_t* d, int x, int y) { return d->qpy[(y >> 2) * d->w4 + (x >> 2)]; }

/* s[i*step_i + k*step_k]: sample at distance i from the edge (i < 0: P side, p_i = s[-(i+1)]) on line k */
static void dbk_luma_seg(pel* s, int step_i, int step_k, int qpp, int qpq, int boff, int toff, int nop, int noq, int bd) {
#define PS(i, k) s[-((i) + 1) * step_i + (k) * step_k]
#define QS(i, k) s[(i) * step_i + (k) * step_k]
    const int qpl = (qpq + qpp + 1) >> 1;
    const int beta = BETA_T[clip3(0, 51, qpl + 2 * boff)] * (1 << (bd - 8));      /* 8.7.2.5.3: beta' and tC' scaled */
    const int tc = TC_T[clip3(0, 53, qpl + 2 + 2 * toff)] * (1 << (bd - 8));
    const int maxv = (1 << bd) - 1;
    const int dp0 = abs(PS(2, 0) - 2 * PS(1, 0) + PS(0, 0)), dp3 = abs(PS(2, 3) - 2 * PS(1, 3) + PS(0, 3));
    const int dq0 = abs(QS(2, 0) - 2 * QS(1, 0) + QS(0, 0)), dq3 = abs(QS(2, 3) - 2 * QS(1, 3) + QS(0, 3));
    if (dp0 + dq0 + dp3 + dq3 >= beta) return;
    int strong = 1;
    for (int j = 0; j < 2; ++j) {
        const int k = j ? 3 : 0, dpq = 2 * (j ? dp3 + dq3 : dp0 + dq0);
        if (!(dpq < (beta >> 2) && abs(PS(3, k) - PS(0, k)) + abs(QS(0, k) - QS(3, k)) < (beta >> 3) &&
              abs(PS(0, k) - QS(0, k)) < ((5 * tc + 1) >> 1)))
            strong = 0;
    }
    const int side = (beta + (beta >> 1)) >> 3;
    const int dep = dp0 + dp3 < side, deq = dq0 + dq3 < side;
    for (int k = 0; k < 4; ++k) {
        const int p0 = PS(0, k), p1 = PS(1, k), p2 = PS(2, k), p3 = PS(3, k);
        const int q0 = QS(0, k), q1 = QS(1, k), q2 = QS(2, k), q3 = QS(3, k);
        if (strong) {
            if (!nop) {
                PS(0, k) = (pel)clip3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
                PS(1, k) = (pel)clip3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2);
                PS(2, k) = (pel)clip3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
            }
            if (!noq) {
                QS(0, k) = (pel)clip3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
                QS(1, k) = (pel)clip3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2);
                QS(2, k) = (pel)clip3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3);
            }
        } else {
            int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
            if (abs(delta) >= tc * 10) continue;
            delta = clip3(-tc, tc, delta);
            if (!nop) {
                PS(0, k) = (pel)clip3(0, maxv, p0 + delta);
                if (dep) PS(1, k) = (pel)clip3(0, maxv, p1 + clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1));
            }
            if (!noq) {
                QS(0, k) = (pel)clip3(0, maxv, q0 - delta);
                if (deq) QS(1, k) = (pel)clip3(0, maxv, q1 + clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1));
            }
        }
    }
#undef PS
#undef QS
}

static void deblock(const geo_t* g, const p265r_params* prm, const p265r_picture* pic, pel* pl[3], const int stride[3]) {
    int any = 0;
    for (int i = 0; i < g->wc * g->hc; ++i) any |= g->ctus[i].flags & P265R_CTU_DEBLOCK;
    if (!any) return;
    dbk_t d;
    d.g = g; d.prm = prm; d.nofilter = pic->nofilter; d.nfw = (g->w + 7) / 8; d.w4 = g->w >> 2;
    d.bdl = prm->bit_depth_luma; d.bdc = prm->bit_depth_chroma;
    const int h4 = g->h >> 2;
    d.org = (uint32_t*)calloc((size_t)d.w4 * h4, sizeof(uint32_t));
    d.qpy = (int16_t*)calloc((size_t)d.w4 * h4, sizeof(int16_t));
    for (uint32_t t = 0; t < pic->n_tbs; ++t) {
        const p265r_tb* tb = &pic->tbs[t];
        if (tb->c_idx) continue;
        const int n4 = 1 << (tb->log2_size - 2);
        for (int j = 0; j < n4; ++j)
            for (int i = 0; i < n4; ++i) {
                const size_t u = (size_t)((tb->y >> 2) + j) * d.w4 + (tb->x >> 2) + i;
                d.org[u] = (uint32_t)tb->x | (uint32_t)tb->y << 16;
                d.qpy[u] = (int16_t)(tb->qp - 6 * (d.bdl - 8));   /* QpY = Qp'Y - QpBdOffsetY */
            }
    }
    for (int dir = 0; dir < 2; ++dir) {          /* 0: vertical edges, 1: horizontal edges */
        /* luma */
        const int emax = dir ? g->h : g->w, smax = dir ? g->w : g->h;
        for (int e = 8; e < emax; e += 8)
            for (int s0 = 0; s0 < smax; s0 += 4) {
                const int xq = dir ? s0 : e, yq = dir ? e : s0, xp = dir ? xq : xq - 1, yp = dir ? yq - 1 : yq;
                if (!dbk_edge(&d, xp, yp, xq, yq)) continue;
                const uint8_t off = g->ctus[ctb_of(g, xq, yq)].deblock_offsets;
                pel* s = pl[0] + (size_t)yq * stride[0] + xq;
                dbk_luma_seg(s, dir ? stride[0] : 1, dir ? 1 : stride[0], dbk_qp(&d, xp, yp), dbk_qp(&d, xq, yq),
                             nib(off & 15), nib(off >> 4), dbk_nf(&d, xp, yp), dbk_nf(&d, xq, yq), d.bdl);
            }
        /* chroma */
        for (int c = 1; c < 3; ++c) {
            const int cw = g->w >> 1, ch = g->h >> 1;
            const int cemax = dir ? ch : cw, csmax = dir ? cw : ch;
            const int cqp = c == 1 ? prm->pps_cb_qp_offset : prm->pps_cr_qp_offset;
            for (int e = 8; e < cemax; e += 8)
                for (int s0 = 0; s0 < csmax; s0 += 4) {
                    const int xq = dir ? s0 : e, yq = dir ? e : s0;
                    const int lxq = xq << 1, lyq = yq << 1, lxp = dir ? lxq : lxq - 1, lyp = dir ? lyq - 1 : lyq;
                    if (!dbk_edge(&d, lxp, lyp, lxq, lyq)) continue;
                    const int toff = nib(g->ctus[ctb_of(g, lxq, lyq)].deblock_offsets >> 4);
                    const int qpc = qpc_of(((dbk_qp(&d, lxq, lyq) + dbk_qp(&d, lxp, lyp) + 1) >> 1) + cqp);
                    const int tc = TC_T[clip3(0, 53, qpc + 2 + 2 * toff)] * (1 << (d.bdc - 8));
                    const int maxc = (1 << d.bdc) - 1;
                    const int nop = dbk_nf(&d, lxp, lyp), noq = dbk_nf(&d, lxq, lyq);
                    const int si = dir ? stride[c] : 1, sk = dir ? 1 : stride[c];
                    for (int k = 0; k < 4; ++k) {
                        pel* q = pl[c] + (size_t)yq * stride[c] + xq + k * sk;
                        const int p0 = q[-si], p1 = q[-2 * si], q0 = q[0], q1 = q[si];
                        const int delta = clip3(-tc, tc, ((((q0 - p0) * 4) + p1 - q1 + 4) >> 3));
                        if (!nop) q[-si] = (pel)clip3(0, maxc, p0 + delta);
                        if (!noq) q[0] = (pel)clip3(0, maxc, q0 - delta);
                    }
                }
        }
    }
    free(d.org);
    free(d.qpy);
}

/* caller plane <-> oracle plane (uint8_t samples at BitDepth 8, uint16_t above) */
static void plane_out(void* dst, const pel* src, size_t n, int bd) {
    if (bd > 8) memcpy(dst, src, n * sizeof(pel));
    else for (size_t i = 0; i < n; ++i) ((uint8_t*)dst)[i] = (uint8_t)src[i];
}

/* Decode n pictures: writes pics[i].recon[] (if set) and pics[i].out[] (if set).  sf: the intra
 * ScalingFactor arrays (2032 bytes, layout of p265r_set_scaling_factors) when scaling_list_enabled.
 * Returns 0 or a negative P265R_* code.  n_threads <= 0: OpenMP default. */
int oracle_decode_sl(const p265r_params* prm, const uint8_t* sf, const p265r_picture* pics, int n, int n_threads) {
    if (!prm || !pics || n < 0) return P265R_EINVAL;
    if (prm->scaling_list_enabled && !sf) return P265R_EINVAL;
    if (!prm->scaling_list_enabled) sf = NULL;
    if (prm->bit_depth_luma < 8 || prm->bit_depth_luma > 12 || prm->bit_depth_chroma < 8 || prm->bit_depth_chroma > 12 ||
        prm->chroma_format_idc != 1)
        return P265R_EUNSUPPORTED;
    init_dct();
    int err = 0;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (int i = 0; i < n; ++i) {
        geo_t g;
        const int nc = ((prm->pic_width + (1 << prm->ctb_log2_size) - 1) >> prm->ctb_log2_size) *
                       ((prm->pic_height + (1 << prm->ctb_log2_size) - 1) >> prm->ctb_log2_size);
        int* rs2ts = (int*)malloc(sizeof(int) * nc);
        const int stride[3] = {prm->pic_width, prm->pic_width / 2, prm->pic_width / 2};
        const int bd[3] = {prm->bit_depth_luma, prm->bit_depth_chroma, prm->bit_depth_chroma};
        size_t sz[3];
        pel* rec[3];
        for (int c = 0; c < 3; ++c) {
            sz[c] = (size_t)stride[c] * (c ? prm->pic_height / 2 : prm->pic_height);
            rec[c] = (pel*)malloc(sz[c] * sizeof(pel));
        }
        geo_init(&g, prm, pics[i].ctus, rs2ts);
        /* CTUs in tile-scan order, TBs in record order */
        int* order = (int*)malloc(sizeof(int) * nc);
        for (int rs = 0; rs < nc; ++rs) order[rs2ts[rs]] = rs;
        for (int ts = 0; ts < nc; ++ts) {
            const p265r_ctu* cu = &pics[i].ctus[order[ts]];
            for (uint32_t k = cu->tb_begin; k < cu->tb_begin + cu->tb_count; ++k)
                recon_tb(&g, prm, sf, rec, stride, &pics[i].tbs[k], pics[i].coef);
        }
        for (int c = 0; c < 3; ++c)
            if (pics[i].recon[c]) plane_out(pics[i].recon[c], rec[c], sz[c], bd[c]);
        if (pics[i].out[0] && pics[i].out[1] && pics[i].out[2]) {
            /* in-loop filters: deblocking into a scratch copy (rec stays the filter input), then SAO */
            pel* dbk[3];
            pel* out[3];
            for (int c = 0; c < 3; ++c) {
                dbk[c] = (pel*)malloc(sz[c] * sizeof(pel));
                out[c] = (pel*)malloc(sz[c] * sizeof(pel));
                memcpy(dbk[c], rec[c], sz[c] * sizeof(pel));
            }
            deblock(&g, prm, &pics[i], dbk, stride);
            if (prm->sample_adaptive_offset) sao(&g, prm, &pics[i], dbk, out, stride);
            else
                for (int c = 0; c < 3; ++c) memcpy(out[c], dbk[c], sz[c] * sizeof(pel));
            for (int c = 0; c < 3; ++c) {
                plane_out(pics[i].out[c], out[c], sz[c], bd[c]);
                free(dbk[c]);
                free(out[c]);
            }
        }
        for (int c = 0; c < 3; ++c) free(rec[c]);
        free(order);
        free(rs2ts);
    }
    return err ? P265R_EINVAL : P265R_OK;
}

int oracle_decode(const p265r_params* prm, const p265r_picture* pics, int n, int n_threads) {
    return oracle_decode_sl(prm, NULL, pics, n, n_threads);
}
