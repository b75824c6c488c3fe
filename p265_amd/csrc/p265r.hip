// p265r.hip -- host side of the C ABI declared in include/p265r.h.
//
// Build (see Makefile):  hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o p265_amd/libp265r.so
//
// One context = one HIP device + one non-blocking stream + one parameter set.
// A batch = one device allocation holding every picture's records, the re-packed
// coefficient pool, the residual job lists and the output planes.  Run order on the
// stream: residual kernels (one per job class) -> intra wavefront steps -> SAO.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/p265r.h"
#include "digest.h"
#include "intra.h"
#include "intra_prep.h"
#include "intra_rows.h"
#include "loopfilter.h"
#include "loopfilter16.h"
#include "sao16.h"
#include "residual.h"
#include "sao.h"
#include "sao_strip16.h"
#include "sao_rows.h"
#include "tables.h"

using namespace p265r;

// Experiment knobs (measured-slower or diagnostic variants) are compiled in only with
// -DP265R_EXPERIMENTS=1 (make variant V=exp FLAGS=-DP265R_EXPERIMENTS=1): P265R_SKIP, P265R_STREAM_PRIO,
// P265R_PIPE_WAVES, P265R_LEAN=0, P265R_FORK_PREP=2, P265R_ROW_WAVES 4 / 6 / 10 / 16, P265R_DEBUG_SYNC.
// The product build reads only the knobs the GPU parity matrix sets (tests/test_gpu_parity.py).
#ifndef P265R_EXPERIMENTS
#define P265R_EXPERIMENTS 0
#endif
// Stream plan of pipelined contexts (round 5: one interleaved A/B of round 3's head against every round-4
// step): the round-4 additions below each cost 5-8 % of the pipelined C3 step by adding
// streams -- a process's streams map round-robin onto GPU_MAX_HW_QUEUES hardware queues (4), so every
// extra stream changes which lanes' kernels queue behind which -- and are off (A/B macros only):
#ifndef P265R_EARLY_RESIDUAL
#define P265R_EARLY_RESIDUAL 0     // re-runs: residual + prep start when the batch's previous intra phase ends
#endif
#ifndef P265R_PHASE_ORDER
#define P265R_PHASE_ORDER 0        // pipelined contexts: one intra phase at a time; residual + prep overlap loop filters
#endif
#ifndef P265R_SAO_AUX
#define P265R_SAO_AUX 0            // pipelined chip-filling batches: prep on the lane stream, the loop filters on the
                                   // lane's aux stream, so the next run's residual + prep overlap this run's SAO
#endif
#ifndef P265R_UP_STREAM
#define P265R_UP_STREAM 0          // 0: a batch uploads on its own lane stream; 1: on an upload stream created with
                                   // the context; 2: created at the first upload (after the lanes)
#endif
#ifndef P265R_SPLIT_W16
#define P265R_SPLIT_W16 1          // small split batches: W = 16 row kernel (0: the by-run W, A/B)
#endif

namespace {

thread_local std::string g_last_hip_error;

int hip_fail(hipError_t e, const char* what) {
    g_last_hip_error = std::string(what) + ": " + hipGetErrorString(e);
    return P265R_EHIP;
}

#define HIP_TRY(expr)                                        \
    do {                                                     \
        hipError_t _e = (expr);                              \
        if (_e != hipSuccess) return hip_fail(_e, #expr);    \
    } while (0)

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

enum { RC_RAW = RC_NUM, N_POOLS = RC_NUM + 1 };

constexpr size_t kDlHalf = 24u << 20;   // download bounce buffer half (p265r_batch_download)

int tb_class(const p265r_tb& t) {
    if (t.flags & (P265R_TB_BYPASS | P265R_TB_PCM)) return RC_RAW;
    if (t.flags & P265R_TB_TSKIP) return RC_TSKIP;
    switch (t.log2_size) {
        case 2: return t.c_idx == 0 ? RC_DST4 : RC_DCT4;
        case 3: return RC_DCT8;
        case 4: return RC_DCT16;
        default: return RC_DCT32;
    }
}

bool params_ok(const p265r_params& p) {
    return p.version == P265R_ABI_VERSION && p.chroma_format_idc == 1 && p.pic_width > 0 && p.pic_height > 0 &&
           p.pic_width % 8 == 0 && p.pic_height % 8 == 0 && p.ctb_log2_size >= 4 && p.ctb_log2_size <= 6 &&
           p.min_tb_log2_size >= 2 && p.max_tb_log2_size <= 5 && p.min_tb_log2_size <= p.max_tb_log2_size;
}

}  // namespace

struct p265r_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t up_stream = nullptr;   // uploads: never queued behind a lane's kernels, so batch k+1
                                       // uploads while batch k decodes (the host waits for it alone)
    p265r_params params{};
    Geo geo{};
    int n_ctus = 0;
    bool timing = false;
    // per timed run: 4 events (start, after residual, after intra, after loop filter) + the
    // launch counts; kept for every run since p265r_set_timing(ctx, 1) so runs can be queued
    // back to back and read once (p265r_timings_total)
    struct Run { hipEvent_t ev[4]; p265r_timings counts; };
    std::vector<Run> runs;
    std::vector<hipEvent_t> spare;
    bool have_timing = false;
    p265r_batch* pending = nullptr;
    std::vector<p265r_picture> pending_pics;
    int schedule = 1;          // 0: one launch per anti-diagonal, 1: CU-local row pipeline
    int row_waves = 0;         // waves per workgroup of the row pipeline (P265R_ROW_WAVES 8, 12; experiments
                               // build also 4, 6, 10, 16); 0 = by run: a batch alone 12 (6 per SIMD, 80 VGPRs:
                               // lowest latency), overlapping other lanes' batches 8 (80 VGPRs: room beside it)
    unsigned lane_busy = 0;    // lanes with a run enqueued since the API last synchronised them (p265r_sync,
                               // p265r_batch_download / p265r_batch_status of a batch on the lane): the row
                               // kernel build of a run follows from the call sequence, not from device timing
    int sao_rows = 1;          // SAO-only batches: 1 16-B strip kernel (CTB 32 / 64; 4-B strip kernel for
                               // CTB 16), 2 4-B strip kernel, 0 loop-filter window kernel (P265R_SAO_ROWS)
    int skip = 0;              // P265R_SKIP (timing experiments on batch re-runs, p265r_batch_run)
    int lean = 1;              // experiments: W = 8 row kernel build 0 unconstrained (P265R_LEAN=0), 1 register-lean
    int split = 1;             // component split of small batches (P265R_SPLIT=0: off; launch_rows_w)
    int xg = 4;                // workgroups per chain of the cross-group row kernel (P265R_XG; 0: off; launch_rows)
    bool last_split = false;   // the last row-kernel launch was split (p265r_describe)
    bool last_xg = false;      // ... was the cross-group kernel
    long long row_launches[5] = {0, 0, 0, 0, 0};   // row-kernel launches per build: W = 12, W = 8, W = 16 split,
                                                   // cross-group, other (experiments) -- p265r_describe
    int luma_lead = -1;        // rows the luma chain leads the chroma chain in the row queue (P265R_LUMA_LEAD);
                               // -1 = by run: 8 for a batch alone, 5 beside other lanes' batches (round 3,
                               // 2 reps: alone lead 5/7/8/10 -> 4.28/4.23/4.19/4.22 ms, pipelined
                               // 45.5/44.9/44.4/44.7 M CTU/s; round 1, W=8: lead 0/1/2/3/5/8/17 ->
                               // 10.40/10.10/10.40/10.09/10.07/10.35/10.38 ms)
    bool stream_prio = false;
    // occupancy caps by dynamic-LDS padding of the SAO / residual launches (P265R_SAO_LDS /
    // P265R_RES_LDS bytes per block, experiments builds): fewer waves per CU streamed faster in the
    // HBM probe (tools/bw_probe.hip)
    int sao_lds = 0, res_lds = 0, prep_lds = 0;
    int prep_last = 0;             // experiments: P265R_PREP_LAST=1 enqueues the prep kernel after the residual kernels
    int order_r = 1;               // P265R_ORDER_R=0 (experiments): ordered runs' residual phase waits only for its own batch  // lanes at the highest stream priority, prep streams at the lowest (P265R_STREAM_PRIO)
    int pipe_waves = 8;        // row pipeline waves per workgroup while other lanes have work (experiments:
                               // P265R_PIPE_WAVES 4, 6, 8)
    int num_cus = 256;
    bool debug_sync = false;   // P265R_DEBUG_SYNC=1: synchronise + log after every phase (P265R_DEBUG_DIAG
                               // builds also trace the row kernel's waves and print placement statistics)
    // reused across batches: pinned host staging (grow-only) and one freed device allocation
    unsigned char* stage = nullptr;
    size_t stage_bytes = 0;
    bool stage_pinned = false;
    void* cache_mem = nullptr;
    size_t cache_bytes = 0;
    // batch pipelining (p265r_set_pipeline): batches are bound round-robin to `pipeline`
    // streams (lane 0 = stream), so one batch's residual / loop-filter phases run beside
    // another batch's intra kernel
    int pipeline = 1;
    int next_lane = 0;
    std::vector<hipStream_t> lanes;   // lanes[0] == stream
    // job prep forked onto a second stream per lane (P265R_FORK_PREP, default on): the prep
    // kernel (latency-bound, LDS/VGPR-limited occupancy) runs beside the residual kernels
    // (HBM-bound) instead of after them; the intra kernel waits for both
    int fork_prep = 1;
    std::vector<hipStream_t> aux;     // aux[i]: lane i's prep stream (created on first use)
    std::vector<hipEvent_t> fork_ev, join_ev;
    std::vector<hipStream_t> aux2;    // aux2[i]: lane i's residual stream (early residual phase)
    std::vector<hipEvent_t> join2_ev;
    // phase order of a pipelined context (P265R_PHASE_ORDER): the last intra launch and the last
    // loop-filter launch of ANY lane, recorded on their lane streams
    hipEvent_t last_intra_ev = nullptr, last_lf_ev = nullptr;
    bool last_intra_valid = false, last_lf_valid = false;
    std::string describe;             // p265r_describe text
    uint8_t* d_sf = nullptr;           // scaling lists: the intra ScalingFactor table (p265r_set_scaling_factors)
    unsigned char* dl_stage = nullptr;  // pinned download bounce buffer, 2 x kDlHalf (first download)
    hipEvent_t dl_ev[2] = {nullptr, nullptr};
};

struct p265r_batch {
    int n_pics = 0;
    void* mem = nullptr;
    size_t bytes = 0;
    DevPic* d_pics = nullptr;
    int16_t* d_pool = nullptr;
    int16_t* d_res = nullptr;
    int* d_err = nullptr;
    ResJob* d_jobs[RC_NUM] = {};
    uint32_t slab[RC_NUM] = {};    // int16 offset of each class's packed TBs in the pool (fixed-size classes)
    BatchView view{};
    int n_jobs[RC_NUM] = {};
    std::vector<DevPic> h_pics;
    hipStream_t stream = nullptr;  // the context lane this batch runs on
    int lane = 0;
    bool sao = false;
    bool dbk = false;          // some CTU of the batch has deblocking on
    bool recon_input = false;  // P265R_PIC_RECON_INPUT: only the in-loop filters run
    bool ragged = false;       // some picture is smaller than the context size (Geo::ragged)
    int* d_xg_prog = nullptr;  // cross-group row kernel (intra_rows.h XgBuf): progress words (zeroed per run
    uint8_t* d_xg_lines = nullptr;  // with the CU slots), the rows' bottom lines; null: batch too large
    std::vector<std::array<int, 2>> size;   // per picture: luma width, height
    int runs = 0;              // p265r_batch_run calls so far
    hipEvent_t sao_done = nullptr;     // P265R_SAO_AUX: recorded on the aux stream after a run's loop filters
    bool sao_pending = false;          // ... and not yet joined into the lane stream (join_sao)
    unsigned long long* d_dig = nullptr;   // p265r_batch_digest_async slots: P265R_DIGEST_SLOTS x n_pics x 3
    hipEvent_t intra_done = nullptr;   // recorded after each run's intra phase (the last reader of the
                                       // residual pool and job lists): the next run's residual + prep
                                       // phase waits for it instead of for the whole previous run
};

namespace {

// Run fn(i) for i in [0, n) on up to 16 host threads (picture-level packing work).
template <class F>
void parallel_for(int n, F fn) {
    const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
    const int nt = std::min(std::min(hw, 16), n);
    if (nt <= 1) {
        for (int i = 0; i < n; ++i) fn(i);
        return;
    }
    std::atomic<int> next{0};
    std::vector<std::thread> th;
    th.reserve(nt);
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&]() {
            for (int i; (i = next.fetch_add(1)) < n;) fn(i);
        });
    for (auto& t : th) t.join();
}

// a lane stream: default priority, or the device's highest with P265R_STREAM_PRIO (then the
// dispatcher prefers the lanes' residual / intra / SAO workgroups over the prep streams')
hipError_t lane_stream_create(const p265r_ctx* ctx, hipStream_t* st) {
    if (!ctx->stream_prio) return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e != hipSuccess) return e;
    return hipStreamCreateWithPriority(st, hipStreamNonBlocking, greatest);
}

// a picture's luma size: its own (p265r_picture.pic_width / pic_height) or the context's
std::array<int, 2> pic_size(const p265r_ctx* ctx, const p265r_picture& pic) {
    return {pic.pic_width ? (int)pic.pic_width : (int)ctx->params.pic_width,
            pic.pic_height ? (int)pic.pic_height : (int)ctx->params.pic_height};
}

int validate_picture(const p265r_ctx* ctx, const p265r_picture& pic) {
    const p265r_params& p = ctx->params;
    const auto sz = pic_size(ctx, pic);
    const int pw = sz[0], ph = sz[1];
    if (pw > p.pic_width || ph > p.pic_height || pw % 8 || ph % 8 || pw <= 0 || ph <= 0) return P265R_EINVAL;
    if (pic.reserved) return P265R_EINVAL;
    Geo g = ctx->geo;
    g.wc = (pw + (1 << g.ctb_log2) - 1) >> g.ctb_log2;
    g.hc = (ph + (1 << g.ctb_log2) - 1) >> g.ctb_log2;
    const int n_ctus = g.wc * g.hc;
    if (!pic.ctus || (!pic.tbs && pic.n_tbs) || (!pic.coef && pic.n_coef)) return P265R_EINVAL;
    if (pic.flags & ~P265R_PIC_RECON_INPUT) return P265R_EINVAL;
    if ((pic.flags & P265R_PIC_RECON_INPUT) && (!pic.recon[0] || !pic.recon[1] || !pic.recon[2])) return P265R_EINVAL;
    const int ctb = 1 << p.ctb_log2_size;
    const int max_tbs = 3 * (ctb / 4) * (ctb / 4) / 2;                  // all-4x4 luma + 4x4 chroma per 8x8
    for (int rs = 0; rs < n_ctus; ++rs) {
        const p265r_ctu& c = pic.ctus[rs];
        if ((uint64_t)c.tb_begin + c.tb_count > pic.n_tbs) return P265R_ERANGE;
        if (c.tb_count > max_tbs) return P265R_EINVAL;                  // more TBs than 4x4 units
        for (int k = 0; k < 2; ++k) {
            const int v = ((c.deblock_offsets >> (4 * k)) & 15) ^ 8;   // biased: -6..6 -> 2..14
            if (v < 2 || v > 14) return P265R_EINVAL;
        }
        for (int k = 0; k < 3; ++k) {
            if (c.sao_type[k] > 2) return P265R_EINVAL;
            if (c.sao_type[k] == 2 && c.sao_class[k] > 3) return P265R_EINVAL;
            if (c.sao_type[k] == 1 && c.sao_class[k] > 31) return P265R_EINVAL;
        }
        // Cb and Cr share SaoTypeIdx and SaoEoClass (7.4.9.3.2; sao.py:57-59, 75-77)
        if (c.sao_type[1] != c.sao_type[2] || (c.sao_type[1] == 2 && c.sao_class[1] != c.sao_class[2])) return P265R_EINVAL;
        const int cx0 = (rs % g.wc) * ctb, cy0 = (rs / g.wc) * ctb;
        int n_luma = 0, n_chroma = 0;
        for (uint32_t i = c.tb_begin; i < c.tb_begin + c.tb_count; ++i) {
            const p265r_tb& t = pic.tbs[i];
            if (t.c_idx == 0 && ++n_luma > (ctb / 4) * (ctb / 4)) return P265R_EINVAL;   // intra_prep.h kMaxCtuLuma
            if (t.c_idx && ++n_chroma > 2 * (ctb / 8) * (ctb / 8)) return P265R_EINVAL;  // kMaxCtuChroma
            if (t.log2_size < 2 || t.log2_size > 5 || t.c_idx > 2 || t.pred_mode > 34) return P265R_EINVAL;
            if (t.c_idx && t.log2_size > 4) return P265R_EINVAL;        // 4:2:0 chroma TBs are 4..16
            const int sub = t.c_idx ? 1 : 0;
            const int n = 1 << t.log2_size;
            const int xl = t.x << sub, yl = t.y << sub, nl = n << sub;
            if (xl + nl > pw || yl + nl > ph) return P265R_ERANGE;
            if (xl < cx0 || yl < cy0 || xl + nl > cx0 + ctb || yl + nl > cy0 + ctb) return P265R_ERANGE;
            if ((t.x & 3) || (t.y & 3) || (t.x & (n - 1)) || (t.y & (n - 1))) return P265R_EINVAL;
            if (t.flags & (P265R_TB_CBF | P265R_TB_PCM)) {
                if ((uint64_t)t.coef_off + (uint64_t)n * n > pic.n_coef) return P265R_ERANGE;
            }
            if (t.flags & ~0x0fu) return P265R_EINVAL;
        }
    }
    return P265R_OK;
}

#ifdef P265R_DEBUG_DIAG
// Row-kernel diagnostics (P265R_DEBUG_DIAG builds with P265R_DEBUG_SYNC=1): wave trace of a hung
// launch, dependency-wait share, workgroup lifetimes and placement, per-job-class cycles
// (P265R_JOB_STATS builds).  Not compiled into the product library.
void rows_diag(hipStream_t st, const int* dbg, int grid, int W) {
    for (int it = 0; it < 100; ++it) {
        if (hipStreamQuery(st) == hipSuccess) break;
        struct timespec ts{0, 100000000};
        nanosleep(&ts, nullptr);
        if (it == 99) {
            fprintf(stderr, "[p265r] rows kernel still running after 10 s; wave trace:\n");
            for (int i = 0; i < grid * W && i < 64; ++i) fprintf(stderr, "  wg %d wave %d: code %d (0x%x)\n", i / W, i % W, dbg[i] & 0xff, dbg[i]);
            fflush(stderr);
            std::abort();
        }
    }
    double tot = 0, wt = 0;
    for (int i = 0; i < grid * W; ++i) { tot += dbg[grid * W + 2 * i]; wt += dbg[grid * W + 2 * i + 1]; }
    fprintf(stderr, "[p265r] rows kernel: %.1f%% of wave time in dependency waits (%d waves)\n", 100.0 * wt / (tot > 0 ? tot : 1), grid * W);
    std::vector<int> life(grid, 0);          // workgroup lifetimes (longest wave, 256-cycle units)
    for (int i = 0; i < grid * W; ++i) life[i / W] = std::max(life[i / W], dbg[grid * W + 2 * i]);
    double sx[16] = {}; int nx[16] = {};
    for (int i = 0; i < grid; ++i) { const int x = dbg[3 * grid * W + 2 * i] & 15; sx[x] += life[i]; ++nx[x]; }
    fprintf(stderr, "[p265r] mean workgroup lifetime per XCC (Mcycles):");
    for (int x = 0; x < 16; ++x) if (nx[x]) fprintf(stderr, " x%d:%.2f(%d)", x, sx[x] / nx[x] * 256e-6, nx[x]);
    fprintf(stderr, "\n");
    std::vector<std::pair<int, int>> byhw;
    for (int i = 0; i < grid; ++i) byhw.push_back({dbg[3 * grid * W + 2 * i] * 256 + ((dbg[3 * grid * W + 2 * i + 1] >> 8) & 255), life[i]});
    std::sort(byhw.begin(), byhw.end());
    int same = 0; double dsum = 0;
    for (size_t i = 1; i < byhw.size(); ++i)
        if (byhw[i].first == byhw[i - 1].first) { ++same; dsum += std::abs(byhw[i].second - byhw[i - 1].second); }
    fprintf(stderr, "[p265r] workgroups sharing a CU: %d pairs, mean lifetime difference %.2f Mcycles\n", same, same ? dsum / same * 256e-6 : 0.0);
    static const char* names[14] = {"luma quad", "chroma quad", "fast Y4", "fast Y8", "fast Y16", "fast C4 pair",
                                    "fast C8 pair", "gen Y4", "gen Y8", "gen Y16", "gen Y32", "gen C4", "gen C8", "gen C16"};
    const int* js = dbg + 3 * grid * W + 2 * grid;
    double jt = 0;
    for (int k = 0; k < 14; ++k) jt += 16.0 * (unsigned)js[2 * k];
    for (int k = 0; k < 14; ++k)
        if (js[2 * k + 1])
            fprintf(stderr, "[p265r] jobs %-13s %9d  %7.0f cycles/job  %5.1f %%\n", names[k], js[2 * k + 1],
                    16.0 * (unsigned)js[2 * k] / js[2 * k + 1], 100.0 * 16.0 * (unsigned)js[2 * k] / (jt > 0 ? jt : 1));
    std::sort(life.begin(), life.end());
    if (grid > 0)
        fprintf(stderr, "[p265r] rows kernel workgroup lifetime (Mcycles): min %.2f p10 %.2f p50 %.2f p90 %.2f max %.2f\n",
                life[0] * 256e-6, life[grid / 10] * 256e-6, life[grid / 2] * 256e-6, life[grid * 9 / 10] * 256e-6,
                life[grid - 1] * 256e-6);
}
#endif

// P265R_SAO_AUX: order the batch's lane stream after its last run's loop filters (host-facing reads)
int join_sao(p265r_batch* b) {
    if (b->sao_pending) {
        HIP_TRY(hipStreamWaitEvent(b->stream, b->sao_done, 0));
        b->sao_pending = false;
    }
    return P265R_OK;
}

// dynamic LDS of the row kernel with W waves and f picture slots (launch_rows_w)
template <typename T>
size_t rows_lds_bytes(const Geo& g, int W, int f) {
    return 256 + (size_t)((f * 2 * g.hc * 4 + 15) & ~15) + W * sizeof(WaveLdsT<T>) +
           (size_t)f * 2 * (g.w + 2 * g.cw) * sizeof(T) + kAngTabBytes;
}

template <int W, int WPE, bool XG = false, bool TRCHK = false, typename T = uint8_t>
int launch_rows_w(p265r_ctx* ctx, p265r_batch* b, hipStream_t st, bool alone) {
    Geo g = ctx->geo;
    // picture slots: the W rows in flight are consecutive in the queue, so they span at
    // most ceil(W / hc) + 1 pictures; a slot is reused only after its previous picture is
    // complete (the kernel waits for that, so fewer slots would still be correct)
    int fs = std::min(32, (W + 2 * g.hc - 1) / (2 * g.hc) + 1);     // 2 row units (luma, chroma) per CTU row
    auto lds_of = [&](int f) { return rows_lds_bytes<T>(g, W, f); };
    while (fs > 2 && lds_of(fs) > 160 * 1024) --fs;
    auto fn = intra_rows_kernel<W, WPE, XG, TRCHK, T>;
    bool split = false;
    {
        // every workgroup resident at once and holding a single picture: one slot is enough
        // (a second picture would only wait for the first), and the smaller LDS footprint can
        // fit one more workgroup per CU
        int pc1 = 0;
        HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_of(1)));
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc1, fn, 64 * W, lds_of(1)));
        if (pc1 >= 1 && b->n_pics <= pc1 * ctx->num_cus) fs = 1;
        // component split: a picture's luma chain and its chroma chain on two workgroups of their own
        // (on different CUs) when all of them fit at once -- the latency regime of a few large
        // pictures / tile units, where one workgroup's W waves on one CU bound the picture's time
        split = ctx->split && pc1 >= 1 && 2 * (long long)b->n_pics <= (long long)pc1 * ctx->num_cus;
        if (XG) { fs = 1; split = true; }
    }
    const size_t lds = lds_of(fs);
    if (lds > 160 * 1024) return P265R_EUNSUPPORTED;
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int per_cu = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * W, lds));
    if (per_cu < 1) return P265R_EUNSUPPORTED;
    const int grid = XG ? 2 * b->n_pics * ctx->xg : split ? 2 * b->n_pics : std::min(b->n_pics, per_cu * ctx->num_cus);
    // fair CU sharing pairs the two workgroups of a CU (rank = arrival order & 1): only valid
    // when exactly two fit per CU and all of them are resident for the whole launch (grid <= 2
    // per CU, no workgroup starts after another ends) -- and only worth it for a batch alone
    g.fair = g.fair && alone && per_cu == 2 && !split;
    // (XG: the progress words were cleared with the CU slots this run, so one tag serves every run)
    const XgBuf xb{XG ? b->d_xg_prog : nullptr, XG ? b->d_xg_lines : nullptr,
                   XG ? b->d_xg_prog + 2 * (size_t)g.hc * b->n_pics : nullptr, XG ? ctx->xg : 0, 1};
    g.ragged = b->ragged ? 1 : 0;
    int* dbg = nullptr;
#ifdef P265R_DEBUG_DIAG
    if (ctx->debug_sync) {
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&dbg), sizeof(int) * (grid * W * 3 + grid * 2 + 32), hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(dbg, 0, sizeof(int) * (grid * W * 3 + grid * 2 + 32));
        fprintf(stderr, "[p265r] rows kernel W=%d WPE=%d fair=%d grid=%d lds=%zu fs=%d per_cu=%d\n", W, WPE, g.fair, grid, lds, fs, per_cu);
    }
#endif
    const int lead = ctx->luma_lead >= 0 ? ctx->luma_lead : (alone ? 8 : 5);
    fn<<<grid, 64 * W, lds, st>>>(b->d_pics, b->d_pool, b->d_res, g, b->n_pics, fs, lead, b->d_err, dbg, split ? 1 : 0, xb);
    ctx->last_split = split;
    ctx->last_xg = XG;
    ++ctx->row_launches[XG ? 3 : (W == 16 ? 2 : (W == 8 ? 1 : (W == 12 ? 0 : 4)))];
    HIP_TRY(hipGetLastError());
#ifdef P265R_DEBUG_DIAG
    if (dbg) {
        rows_diag(st, dbg, grid, W);
        (void)hipHostFree(dbg);
    }
#endif
    return P265R_OK;
}

// alone: no other lane of the context has a run enqueued (ctx->lane_busy), so this batch's kernels
// have the GPU to themselves: W = 12 with fair CU sharing; otherwise W = 8 (80 VGPRs, so the residual /
// prep / SAO waves of the neighbouring batches fit beside it on every SIMD)
#ifndef P265R_W10_WPE
#define P265R_W10_WPE 5                  // experiments: the pipelined W = 10 build's waves-per-SIMD attribute
#endif
int launch_rows(p265r_ctx* ctx, p265r_batch* b, hipStream_t st, bool alone) {
#if P265R_EXPERIMENTS
    switch (ctx->row_waves) {
        case 4: return launch_rows_w<4, 1>(ctx, b, st, alone);
        case 6: return launch_rows_w<6, 1>(ctx, b, st, alone);
        case 10: return launch_rows_w<10, 5>(ctx, b, st, alone);
        case 16: return launch_rows_w<16, 1>(ctx, b, st, alone);
        default: break;
    }
    if (ctx->row_waves == 0 && !alone && ctx->pipe_waves == 4) return launch_rows_w<4, 1>(ctx, b, st, alone);
    if (ctx->row_waves == 0 && !alone && ctx->pipe_waves == 6) return launch_rows_w<6, 1>(ctx, b, st, alone);
    if (ctx->row_waves == 0 && !alone && ctx->pipe_waves == 10 && !(ctx->split && 2 * (long long)b->n_pics <= ctx->num_cus))
        return launch_rows_w<10, P265R_W10_WPE>(ctx, b, st, alone);
    if (ctx->lean == 0 && (ctx->row_waves == 8 || (ctx->row_waves == 0 && !alone))) return launch_rows_w<8, 1>(ctx, b, st, alone);
#endif
    // a batch small enough for the component split with one workgroup per CU (the latency regime:
    // tile units, the decoder's small batches): W = 16, so every CTU row of a picture's chain can
    // be in flight at once (a 2-CTU-lag wavefront of 17 rows needs 17 waves; with 12 the rows
    // after the 12th wait for a whole row to finish)
    // 16-bit samples (BitDepth 9..12): the same row pipeline on 16-bit LDS tiles and line buffers
    // (one workgroup per CU: twice the LDS of a wave); W = 12 alone, W = 8 beside other lanes' work
    if (ctx->geo.pel16) {
        // (wide pictures: W = 12 only while its two picture slots fit the 160 KB of LDS; p265r_create keeps
        // the per-diagonal schedule for pictures too wide for W = 8)
        int w = ctx->row_waves ? ctx->row_waves : (alone ? 12 : 8);
        if (w == 12 && rows_lds_bytes<uint16_t>(ctx->geo, 12, 2) > 160 * 1024) w = 8;
        if (ctx->geo.bd[0] > 10)                    // BitDepth 11..12: int16_t tags the split angular sums (pang)
            return w == 12 ? launch_rows_w<12, 1, false, false, int16_t>(ctx, b, st, alone)
                           : launch_rows_w<8, 1, false, false, int16_t>(ctx, b, st, alone);
        return w == 12 ? launch_rows_w<12, 1, false, false, uint16_t>(ctx, b, st, alone)
                       : launch_rows_w<8, 1, false, false, uint16_t>(ctx, b, st, alone);
    }
    // smaller still (every chain on xg CUs of its own): the cross-group kernel, one wave per SIMD
    if (ctx->row_waves == 0 && b->d_xg_prog && 2 * (long long)b->n_pics * ctx->xg <= ctx->num_cus)
        return ctx->geo.tr_check ? launch_rows_w<4, 1, true, true>(ctx, b, st, alone)     // (test build of it)
                                 : launch_rows_w<4, 1, true>(ctx, b, st, alone);
    if (ctx->row_waves == 0 && ctx->split && P265R_SPLIT_W16 && 2 * (long long)b->n_pics <= ctx->num_cus)
        return launch_rows_w<16, 4>(ctx, b, st, alone);
    const int w = ctx->row_waves ? ctx->row_waves : (alone ? 12 : 8);
    return w == 12 ? launch_rows_w<12, 6>(ctx, b, st, alone) : launch_rows_w<8, 6>(ctx, b, st, alone);
}

}  // namespace

extern "C" {

uint32_t p265r_abi_version(void) { return P265R_ABI_VERSION; }

const char* p265r_last_hip_error(void) { return g_last_hip_error.c_str(); }

const char* p265r_strerror(int code) {
    switch (code) {
        case P265R_OK: return "ok";
        case P265R_EINVAL: return "invalid argument or malformed record";
        case P265R_ENOMEM: return "out of memory";
        case P265R_EHIP: return "HIP runtime error";
        case P265R_EUNSUPPORTED: return "unsupported stream feature";
        case P265R_ERANGE: return "record points outside the picture or its buffers";
        case P265R_ESTATE: return "call out of order";
        case P265R_ENODEV: return "no such HIP device";
        default: return "unknown error";
    }
}

int p265r_device_count(void) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e == hipErrorNoDevice) return 0;
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
    return n;
}

int p265r_create(int device, const p265r_params* params, p265r_ctx** out) {
    if (!params || !out) return P265R_EINVAL;
    *out = nullptr;
    const p265r_params& p = *params;
    if (!params_ok(p)) return P265R_EINVAL;
    // BitDepth 8 (uint8_t planes) or 9..12 with one depth for luma and chroma (uint16_t planes; 13..14 would
    // need SaoOffsetVal beyond the int8 of the CTU record)
    if (p.bit_depth_luma < 8 || p.bit_depth_luma > 12 || p.bit_depth_chroma != p.bit_depth_luma || p.scaling_list_enabled > 1)
        return P265R_EUNSUPPORTED;
    const int n = p265r_device_count();
    if (n < 0) return n;
    if (device < 0 || device >= n) return P265R_ENODEV;
    p265r_ctx* ctx = new (std::nothrow) p265r_ctx();
    if (!ctx) return P265R_ENOMEM;
    ctx->device = device;
    ctx->params = p;
    Geo& g = ctx->geo;
    g.w = p.pic_width; g.h = p.pic_height;
    g.cw = g.w / 2; g.ch = g.h / 2;
    g.stride[0] = (int)align_up(g.w, 64);
    g.stride[1] = g.stride[2] = (int)align_up(g.cw, 64);
    g.ctb_log2 = p.ctb_log2_size;
    g.wc = (g.w + (1 << g.ctb_log2) - 1) >> g.ctb_log2;
    g.hc = (g.h + (1 << g.ctb_log2) - 1) >> g.ctb_log2;
    g.bd[0] = p.bit_depth_luma; g.bd[1] = g.bd[2] = p.bit_depth_chroma;
    g.pel16 = p.bit_depth_luma > 8 ? 1 : 0;
    g.strong = p.strong_intra_smoothing;
    g.lf_tiles = p.loop_filter_across_tiles;
    g.nf_w = (g.w + 7) / 8;
    g.cqp[0] = p.pps_cb_qp_offset;
    g.cqp[1] = p.pps_cr_qp_offset;
    g.fair = 1;
    if (const char* v = std::getenv("P265R_FAIR")) g.fair = v[0] != '0';
    g.quad = 3;
    g.tr_check = 0;
    g.tr_info = 1;
    if (const char* v = std::getenv("P265R_QUAD")) g.quad = std::atoi(v) & 7;
    ctx->n_ctus = g.wc * g.hc;
    // test knobs of the GPU parity matrix (bench.py refuses to run with any P265R_* variable set)
    for (const char* k : {"P265R_FAIR", "P265R_QUAD", "P265R_SCHEDULE", "P265R_SAO_ROWS", "P265R_LUMA_LEAD", "P265R_ROW_WAVES",
                          "P265R_FORK_PREP", "P265R_SPLIT", "P265R_XG", "P265R_TR_CHECK"})
        if (std::getenv(k)) ctx->describe += std::string(ctx->describe.empty() ? "" : ", ") + "\"" + k + "\"";
    if (const char* v = std::getenv("P265R_SCHEDULE")) ctx->schedule = std::strcmp(v, "steps") == 0 ? 0 : 1;
    // 16-bit samples: the row pipeline while a W = 8 workgroup's LDS tiles and two line-buffer slots fit
    // 160 KB (pictures up to ≈ 4K wide), else the per-diagonal kernel (BitDepth 11..12 too: the row kernel's
    // packed Cb | Cr angular sums are split into 6-bit halves there, pang in intra_rows.h)
    if (g.pel16 && rows_lds_bytes<uint16_t>(g, 8, 2) > 160 * 1024) ctx->schedule = 0;
    if (const char* v = std::getenv("P265R_SAO_ROWS")) ctx->sao_rows = std::atoi(v) == 2 ? 2 : (v[0] != '0' ? 1 : 0);
    if (const char* v = std::getenv("P265R_LUMA_LEAD")) ctx->luma_lead = std::max(0, std::atoi(v));
    if (const char* v = std::getenv("P265R_SPLIT")) ctx->split = v[0] != '0';
    if (const char* v = std::getenv("P265R_TR_CHECK")) g.tr_check = v[0] == '1';
    if (const char* v = std::getenv("P265R_XG")) { const int x = std::atoi(v); ctx->xg = (x == 2 || x == 4 || x == 8) ? x : 0; }
    if (const char* v = std::getenv("P265R_FORK_PREP")) ctx->fork_prep = std::atoi(v) != 0 ? 1 : 0;
    if (const char* v = std::getenv("P265R_ROW_WAVES")) {
        const int w = std::atoi(v);
        if (w == 8 || w == 12) ctx->row_waves = w;
#if P265R_EXPERIMENTS
        if (w == 4 || w == 6 || w == 10 || w == 16) ctx->row_waves = w;
#endif
    }
#if P265R_EXPERIMENTS
    for (const char* k : {"P265R_DEBUG_SYNC", "P265R_SKIP", "P265R_LEAN", "P265R_PIPE_WAVES", "P265R_STREAM_PRIO"})
        if (std::getenv(k)) ctx->describe += std::string(ctx->describe.empty() ? "" : ", ") + "\"" + k + "\"";
    if (const char* v = std::getenv("P265R_DEBUG_SYNC")) ctx->debug_sync = v[0] == '1';
    if (const char* v = std::getenv("P265R_SKIP")) ctx->skip = std::atoi(v) & 7;
    if (const char* v = std::getenv("P265R_LEAN")) ctx->lean = std::atoi(v) == 0 ? 0 : 1;
    if (const char* v = std::getenv("P265R_FORK_PREP")) ctx->fork_prep = std::min(2, std::max(0, std::atoi(v)));
    if (const char* v = std::getenv("P265R_PIPE_WAVES")) {
        const int w = std::atoi(v);
        if (w == 4 || w == 6 || w == 8 || w == 10) ctx->pipe_waves = w;
    }
    if (const char* v = std::getenv("P265R_STREAM_PRIO")) ctx->stream_prio = std::atoi(v) != 0;
    for (const char* k : {"P265R_SAO_LDS", "P265R_RES_LDS", "P265R_PREP_LDS", "P265R_PREP_LAST"})
        if (std::getenv(k)) ctx->describe += std::string(ctx->describe.empty() ? "" : ", ") + "\"" + k + "\"";
    if (const char* v = std::getenv("P265R_ORDER_R")) ctx->order_r = std::atoi(v) != 0;
    if (const char* v = std::getenv("P265R_SAO_LDS")) ctx->sao_lds = std::min(65536, std::max(0, std::atoi(v)));
    if (const char* v = std::getenv("P265R_RES_LDS")) ctx->res_lds = std::min(32768, std::max(0, std::atoi(v)));
    if (const char* v = std::getenv("P265R_PREP_LDS")) ctx->prep_lds = std::min(65536, std::max(0, std::atoi(v)));
    if (const char* v = std::getenv("P265R_PREP_LAST")) ctx->prep_last = std::atoi(v) != 0;
#endif
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&ctx->num_cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e == hipSuccess) e = lane_stream_create(ctx, &ctx->stream);
    if (e == hipSuccess) ctx->lanes.push_back(ctx->stream);
    if (e == hipSuccess && P265R_UP_STREAM == 1) e = hipStreamCreateWithFlags(&ctx->up_stream, hipStreamNonBlocking);
    if (e == hipSuccess) {
        int8_t ang[35];
        int16_t inv[35];
        for (int i = 0; i < 35; ++i) { ang[i] = (int8_t)kIntraPredAngle[i]; inv[i] = (int16_t)kInvAngle[i]; }
        uint32_t angw[35];
        for (int i = 0; i < 35; ++i) angw[i] = (uint32_t)(uint8_t)ang[i] | (uint32_t)(inv[i] ? -inv[i] : 256) << 8;
        e = hipMemcpyToSymbol(HIP_SYMBOL(c_angle), ang, sizeof(ang));
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_inv_angle), inv, sizeof(inv));
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_angw), angw, sizeof(angw));
        uint32_t ztab[64];
        for (int i = 0; i < 64; ++i) ztab[i] = avail_ztab_word(i >> 4, i & 15);
        if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(c_ztab), ztab, sizeof(ztab));
    }
    if (e != hipSuccess) {
        int rc = hip_fail(e, "p265r_create");
        p265r_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return P265R_OK;
}

void p265r_destroy(p265r_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    for (hipStream_t st : ctx->lanes) (void)hipStreamSynchronize(st);
    for (hipStream_t st : ctx->aux) if (st) (void)hipStreamSynchronize(st);
    for (hipStream_t st : ctx->aux2) if (st) (void)hipStreamSynchronize(st);
    if (ctx->pending) p265r_batch_free(ctx, ctx->pending);
    for (hipStream_t st : ctx->aux) if (st) (void)hipStreamDestroy(st);
    for (hipStream_t st : ctx->aux2) if (st) (void)hipStreamDestroy(st);
    for (hipEvent_t e : ctx->join2_ev) if (e) (void)hipEventDestroy(e);
    if (ctx->last_intra_ev) (void)hipEventDestroy(ctx->last_intra_ev);
    if (ctx->last_lf_ev) (void)hipEventDestroy(ctx->last_lf_ev);
    for (hipEvent_t e : ctx->fork_ev) if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->join_ev) if (e) (void)hipEventDestroy(e);
    for (auto& r : ctx->runs) for (auto& e : r.ev) (void)hipEventDestroy(e);
    for (auto& e : ctx->spare) (void)hipEventDestroy(e);
    for (size_t i = 1; i < ctx->lanes.size(); ++i) (void)hipStreamDestroy(ctx->lanes[i]);
    if (ctx->up_stream) (void)hipStreamDestroy(ctx->up_stream);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->cache_mem) (void)hipFree(ctx->cache_mem);
    if (ctx->d_sf) (void)hipFree(ctx->d_sf);
    if (ctx->dl_stage) (void)hipHostFree(ctx->dl_stage);
    for (hipEvent_t e : ctx->dl_ev) if (e) (void)hipEventDestroy(e);
    if (ctx->stage) { if (ctx->stage_pinned) (void)hipHostFree(ctx->stage); else std::free(ctx->stage); }
    delete ctx;
}

int p265r_batch_upload(p265r_ctx* ctx, const p265r_picture* pics, int n_pics, p265r_batch** out) {
    if (!ctx || !pics || n_pics <= 0 || !out) return P265R_EINVAL;
#if P265R_EXPERIMENTS
    // P265R_UPLOAD_TIMES=1 (experiments build): wall time of the upload's stages on stderr
    const bool ut = std::getenv("P265R_UPLOAD_TIMES") != nullptr;
    std::vector<std::pair<const char*, std::chrono::steady_clock::time_point>> tp;
#define P265R_UT(name) do { if (ut) tp.emplace_back(name, std::chrono::steady_clock::now()); } while (0)
#else
#define P265R_UT(name) do { } while (0)
#endif
    P265R_UT("start");
    *out = nullptr;
    if (n_pics > 65535) return P265R_ERANGE;                     // pictures index a grid dimension
    for (int i = 0; i < n_pics; ++i)
        if ((pics[i].flags ^ pics[0].flags) & P265R_PIC_RECON_INPUT) return P265R_EINVAL;
    const bool recon_input = (pics[0].flags & P265R_PIC_RECON_INPUT) != 0;
    const Geo& g = ctx->geo;
    const int nc = ctx->n_ctus;                  // per-picture slots of the context size
    // per picture: luma size, CTUs, no-filter map bytes (a ragged batch mixes sizes)
    std::vector<std::array<int, 2>> psize(n_pics);
    std::vector<int> pnc(n_pics);
    std::vector<size_t> pnf(n_pics);
    bool ragged = false;
    for (int i = 0; i < n_pics; ++i) {
        psize[i] = pic_size(ctx, pics[i]);
        const int wc = (psize[i][0] + (1 << g.ctb_log2) - 1) >> g.ctb_log2, hc = (psize[i][1] + (1 << g.ctb_log2) - 1) >> g.ctb_log2;
        pnc[i] = wc * hc;
        pnf[i] = (size_t)((psize[i][0] + 7) / 8) * ((psize[i][1] + 7) / 8);
        ragged |= psize[i][0] != g.w || psize[i][1] != g.h;
    }
    // ---- pool sizing per class (per picture, so pictures can be packed in parallel) ----
    std::vector<std::array<size_t, N_POOLS>> cnt_pool(n_pics);
    std::vector<std::array<int, RC_NUM>> cnt_job(n_pics);
    std::vector<int> crc(n_pics, 0);
    parallel_for(n_pics, [&](int i) {
        // every record of every picture is checked (on up to 16 host threads: pictures are independent; the
        // first failing picture's code is returned), then its coded TBs are counted per class with
        // thread-local counters, stored once (neighbouring pictures' counters share cache lines).  Every TB
        // of the array is packed, so the fields the packing reads are checked here for all of them
        // (validate_picture checks the TBs the CTUs reference, by position); one pass per picture right
        // after its validation, while its TB array is still in the cache
        const p265r_picture& pic = pics[i];
        if ((crc[i] = validate_picture(ctx, pic)) != 0) return;
        std::array<size_t, N_POOLS> cp{};
        std::array<int, RC_NUM> cj{};
        for (uint32_t t = 0; t < pic.n_tbs; ++t) {
            const p265r_tb& tb = pic.tbs[t];
            if (!(tb.flags & (P265R_TB_CBF | P265R_TB_PCM))) continue;
            if (tb.log2_size < 2 || tb.log2_size > 5) { crc[i] = P265R_EINVAL; return; }
            if ((uint64_t)tb.coef_off + ((uint64_t)1 << (2 * tb.log2_size)) > pic.n_coef) { crc[i] = P265R_ERANGE; return; }
            const int cls = tb_class(tb);
            cp[cls] += (size_t)1 << (2 * tb.log2_size);
            if (cls < RC_NUM) ++cj[cls];
        }
        cnt_pool[i] = cp;
        cnt_job[i] = cj;
    });
    for (int i = 0; i < n_pics; ++i)
        if (crc[i]) return crc[i];
    P265R_UT("validate+count");
    size_t pool_sz[N_POOLS] = {};
    size_t n_tbs_total = 0;
    int n_jobs[RC_NUM] = {};
    for (int i = 0; i < n_pics; ++i) {
        n_tbs_total += pics[i].n_tbs;
        for (int c = 0; c < N_POOLS; ++c) pool_sz[c] += cnt_pool[i][c];
        for (int c = 0; c < RC_NUM; ++c) n_jobs[c] += cnt_job[i][c];
    }
    size_t pool_base[N_POOLS];
    size_t pool_total = 0;
    for (int c = 0; c < N_POOLS; ++c) { pool_base[c] = pool_total; pool_total += pool_sz[c]; }
    // the row kernel addresses every residual as a signed 32-bit int16 offset relative to the
    // residual pool: raw samples down to -(pool_total + 128) (coefficient pool + its pad), the
    // zero block and the fast jobs' over-read up to pool_total + 512 + 64
    if (pool_total + 2048 > (size_t)INT32_MAX) return P265R_ERANGE;
    // ---- device layout -----------------------------------------------------------
    const bool sao = ctx->params.sample_adaptive_offset != 0;
    bool dbk = false;
    for (int i = 0; i < n_pics && !dbk; ++i)
        for (int rs = 0; rs < pnc[i]; ++rs)
            if (pics[i].ctus[rs].flags & P265R_CTU_DEBLOCK) { dbk = true; break; }
    const bool lf = sao || dbk;                  // separate output planes
    const size_t pb = g.pel16 ? 2 : 1;          // bytes per sample
    const size_t plane_bytes[3] = {(size_t)g.stride[0] * g.h * pb, (size_t)g.stride[1] * g.ch * pb, (size_t)g.stride[2] * g.ch * pb};
    const size_t pic_plane_bytes = align_up(plane_bytes[0], 256) + 2 * align_up(plane_bytes[1], 256);
    size_t off = 0;
    const size_t o_pics = off; off = align_up(off + sizeof(DevPic) * n_pics, 256);
    // error word (+ the row kernel's per-CU workgroup slots, kRowCuSlots x 16 B, intra_rows.h)
    // cross-group row kernel (a batch whose chains fit xg workgroups each on the CUs): its progress words
    // follow the CU slots (cleared together per run), its lines get their own range
    const bool xg_ok = ctx->xg > 0 && ctx->split && 2 * (long long)n_pics * ctx->xg <= ctx->num_cus;
    // (+ one row ticket per chain)
    const size_t xg_prog_bytes = xg_ok ? sizeof(int) * 2 * ((size_t)g.hc + 1) * n_pics : 0;
    const size_t o_err = off; off = align_up(off + 256 + kRowCuSlots * 16 + xg_prog_bytes, 256);
    const size_t o_xgl = off;
    if (xg_ok) off = align_up(off + 2 * (size_t)g.hc * ((size_t)(g.wc + 2) << g.ctb_log2) * n_pics, 256);
    const size_t o_ctus = off; off = align_up(off + sizeof(p265r_ctu) * nc * (size_t)n_pics, 256);
    const size_t o_tbs = off; off = align_up(off + sizeof(p265r_tb) * n_tbs_total, 256);
    // both pools padded by 64 B: the intra kernel reads fixed-shape 32-B runs
    // (the row kernel reads every residual relative to the residual pool: raw TBs at negative
    // offsets into the coefficient pool, uncoded halves from a zero block after the residuals;
    // fast jobs read one sample per lane, lanes past the TB up to 126 B beyond it)
    const size_t o_pool = off; off = align_up(off + sizeof(int16_t) * pool_total + 256, 256);
    const size_t o_res = off; off = align_up(off + sizeof(int16_t) * pool_total + 1024, 256);
    size_t o_jobs[RC_NUM];
    for (int c = 0; c < RC_NUM; ++c) { o_jobs[c] = off; off = align_up(off + sizeof(ResJob) * n_jobs[c], 256); }
    // intra jobs (same index space as the TB records) + per-CTU job counts
    const size_t o_ijobs = off; off = align_up(off + sizeof(IntraJob) * n_tbs_total, 256);
    const size_t o_jcount = off; off = align_up(off + 4 * sizeof(uint32_t) * nc * (size_t)n_pics, 256);
    size_t o_nf = off;
    size_t nf_bytes = (size_t)g.nf_w * ((g.h + 7) / 8);
    size_t n_nf = 0;
    for (int i = 0; i < n_pics; ++i) n_nf += pics[i].nofilter ? 1 : 0;
    off = align_up(off + nf_bytes * n_nf, 256);
    const size_t map_bytes = nf_bytes << g.pel16;                  // uint16 entries above 8 bits (loopfilter.h)
    const size_t o_map = off; if (dbk) off = align_up(off + map_bytes * n_pics, 256);
    const size_t o_rec = off; off += pic_plane_bytes * n_pics;
    const size_t o_out = off; if (lf) off += pic_plane_bytes * n_pics;
    const size_t total = align_up(off, 256);
    P265R_UT("layout");

    // ---- host staging: [0, o_res) | jobs [o_jobs[0], o_ijobs) | no-filter maps, compact ---------
    const size_t jobs_bytes = o_ijobs - o_jobs[0];
    const size_t s_jobs = o_res, s_nf = o_res + jobs_bytes;
    const size_t stage_need = s_nf + nf_bytes * n_nf;
    (void)hipSetDevice(ctx->device);
    if (ctx->stage_bytes < stage_need) {
        if (ctx->stage) { if (ctx->stage_pinned) (void)hipHostFree(ctx->stage); else std::free(ctx->stage); }
        ctx->stage = nullptr;
        ctx->stage_bytes = 0;
        const size_t want = stage_need + stage_need / 4;
        void* ptr = nullptr;
        if (hipHostMalloc(&ptr, want, hipHostMallocDefault) == hipSuccess) {
            ctx->stage_pinned = true;
        } else {
            (void)hipGetLastError();
            ptr = std::malloc(want);
            ctx->stage_pinned = false;
            if (!ptr) return P265R_ENOMEM;
        }
        ctx->stage = static_cast<unsigned char*>(ptr);
        ctx->stage_bytes = want;
    }
    unsigned char* host = ctx->stage;
    p265r_batch* b = new (std::nothrow) p265r_batch();
    if (!b) return P265R_ENOMEM;
    hipError_t e = hipSuccess;
    if (ctx->cache_mem && ctx->cache_bytes >= total) {      // reuse the last freed allocation
        b->mem = ctx->cache_mem;
        b->bytes = ctx->cache_bytes;
        ctx->cache_mem = nullptr;
        ctx->cache_bytes = 0;
    } else {
        e = hipMalloc(&b->mem, total);
        if (e != hipSuccess && ctx->cache_mem) {             // make room: drop the cached one
            (void)hipGetLastError();
            (void)hipFree(ctx->cache_mem);
            ctx->cache_mem = nullptr;
            ctx->cache_bytes = 0;
            e = hipMalloc(&b->mem, total);
        }
        if (e != hipSuccess) { delete b; return e == hipErrorOutOfMemory ? P265R_ENOMEM : hip_fail(e, "hipMalloc"); }
        b->bytes = total;
    }
    b->n_pics = n_pics;
    b->stream = ctx->stream;
    if (ctx->pipeline > 1) {
        b->lane = ctx->next_lane++ % ctx->pipeline;
        b->stream = ctx->lanes[b->lane];
    }
    b->sao = sao;
    b->dbk = dbk;
    b->recon_input = recon_input;
    b->ragged = ragged;
    b->size = psize;
    unsigned char* dbase = static_cast<unsigned char*>(b->mem);
    b->d_pics = reinterpret_cast<DevPic*>(dbase + o_pics);
    b->d_pool = reinterpret_cast<int16_t*>(dbase + o_pool);
    b->d_res = reinterpret_cast<int16_t*>(dbase + o_res);
    b->d_err = reinterpret_cast<int*>(dbase + o_err);
    b->d_xg_prog = xg_ok ? b->d_err + 64 + kRowCuSlots * 4 : nullptr;
    b->d_xg_lines = xg_ok ? dbase + o_xgl : nullptr;
    for (int c = 0; c < RC_NUM; ++c) {
        b->d_jobs[c] = reinterpret_cast<ResJob*>(dbase + o_jobs[c]);
        b->n_jobs[c] = n_jobs[c];
        b->slab[c] = (uint32_t)pool_base[c];
    }
    b->h_pics.resize(n_pics);

    P265R_UT("alloc");
    p265r_ctu* h_ctus = reinterpret_cast<p265r_ctu*>(host + o_ctus);
    p265r_tb* h_tbs = reinterpret_cast<p265r_tb*>(host + o_tbs);
    int16_t* h_pool = reinterpret_cast<int16_t*>(host + o_pool);
    ResJob* h_jobs[RC_NUM];
    for (int c = 0; c < RC_NUM; ++c) h_jobs[c] = reinterpret_cast<ResJob*>(host + s_jobs + (o_jobs[c] - o_jobs[0]));
    // per-picture start offsets in every pool / job list / TB array / no-filter slot
    std::vector<std::array<size_t, N_POOLS>> pool_at(n_pics);
    std::vector<std::array<int, RC_NUM>> job_at(n_pics);
    std::vector<size_t> tb_at(n_pics), nf_at(n_pics);
    {
        size_t pf[N_POOLS];
        std::copy(pool_base, pool_base + N_POOLS, pf);
        int jf[RC_NUM] = {};
        size_t tf = 0, nf = 0;
        for (int i = 0; i < n_pics; ++i) {
            for (int c = 0; c < N_POOLS; ++c) { pool_at[i][c] = pf[c]; pf[c] += cnt_pool[i][c]; }
            for (int c = 0; c < RC_NUM; ++c) { job_at[i][c] = jf[c]; jf[c] += cnt_job[i][c]; }
            tb_at[i] = tf;
            tf += pics[i].n_tbs;
            nf_at[i] = nf;
            nf += pics[i].nofilter ? 1 : 0;
        }
    }
    auto pack_pic = [&](int i) {
        const p265r_picture& pic = pics[i];
        std::memcpy(h_ctus + (size_t)i * nc, pic.ctus, sizeof(p265r_ctu) * pnc[i]);
        if (pnc[i] < nc) std::memset(h_ctus + (size_t)i * nc + pnc[i], 0, sizeof(p265r_ctu) * (nc - pnc[i]));
        p265r_tb* tb_dst = h_tbs + tb_at[i];
        size_t pool_fill[N_POOLS];
        int job_fill[RC_NUM];
        for (int c = 0; c < N_POOLS; ++c) pool_fill[c] = pool_at[i][c];
        for (int c = 0; c < RC_NUM; ++c) job_fill[c] = job_at[i][c];
        for (uint32_t t = 0; t < pic.n_tbs; ++t) {
            p265r_tb tb = pic.tbs[t];
            if (tb.flags & (P265R_TB_CBF | P265R_TB_PCM)) {
                const int cls = tb_class(tb);
                const size_t nn = (size_t)1 << (2 * tb.log2_size);
                int16_t* dst = h_pool + pool_fill[cls];
                const int16_t* src = pic.coef + tb.coef_off;
                switch (tb.log2_size) {                // fixed sizes: inlined vector moves, no memcpy call per TB
                    case 2: std::memcpy(dst, src, 16 * sizeof(int16_t)); break;
                    case 3: std::memcpy(dst, src, 64 * sizeof(int16_t)); break;
                    case 4: std::memcpy(dst, src, 256 * sizeof(int16_t)); break;
                    default: std::memcpy(dst, src, 1024 * sizeof(int16_t)); break;
                }
                tb.coef_off = (uint32_t)pool_fill[cls];
                if (cls < RC_NUM) h_jobs[cls][job_fill[cls]++] = ResJob{tb.coef_off, tb.qp, tb.flags, tb.log2_size, tb.c_idx};
                pool_fill[cls] += nn;
            }
            tb_dst[t] = tb;
        }
        DevPic& dp = b->h_pics[i];
        dp.ctus = reinterpret_cast<const p265r_ctu*>(dbase + o_ctus) + (size_t)i * nc;
        dp.tbs = reinterpret_cast<const p265r_tb*>(dbase + o_tbs) + tb_at[i];
        dp.jobs = reinterpret_cast<IntraJob*>(dbase + o_ijobs) + tb_at[i];
        dp.jcount = reinterpret_cast<uint32_t*>(dbase + o_jcount) + 4 * (size_t)i * nc;
        unsigned char* rec = dbase + o_rec + pic_plane_bytes * i;
        dp.rec[0] = rec;
        dp.rec[1] = rec + align_up(plane_bytes[0], 256);
        dp.rec[2] = dp.rec[1] + align_up(plane_bytes[1], 256);
        dp.dbk_map = dbk ? dbase + o_map + map_bytes * i : nullptr;
        dp.pool_rel = -(int32_t)((o_res - o_pool) / sizeof(int16_t));
        dp.zero_off = (uint32_t)pool_total;
        dp.wh = (uint32_t)psize[i][0] | (uint32_t)psize[i][1] << 16;
        dp.pad_ = 0;
        if (lf) {
            unsigned char* o = dbase + o_out + pic_plane_bytes * i;
            dp.out[0] = o;
            dp.out[1] = o + align_up(plane_bytes[0], 256);
            dp.out[2] = dp.out[1] + align_up(plane_bytes[1], 256);
        } else {
            for (int c = 0; c < 3; ++c) dp.out[c] = dp.rec[c];
        }
        if (pic.nofilter) {
            std::memcpy(host + s_nf + nf_at[i] * nf_bytes, pic.nofilter, pnf[i]);   // (slot of the context size)
            dp.nofilter = dbase + o_nf + nf_at[i] * nf_bytes;
        } else {
            dp.nofilter = nullptr;
        }
        };
    // Packing and H2D overlap: the pictures go in chunks; a chunk's ranges of every array (CTU and TB
    // records, each class slab of the coefficient pool, each residual job list, no-filter maps) are
    // enqueued as soon as the chunk is packed, so the DMA engine copies chunk k while the host packs
    // chunk k + 1 (the staging ranges of different chunks are disjoint).  The DevPic table and the
    // error word follow last; the gaps between the arrays are zeroed on the device.
    (void)hipSetDevice(ctx->device);
    if (P265R_UP_STREAM == 2 && !ctx->up_stream && e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->up_stream, hipStreamNonBlocking);
    hipStream_t st = P265R_UP_STREAM ? ctx->up_stream : b->stream;
    auto h2d = [&](size_t dev_off, size_t host_off, size_t bytes) {
        if (e == hipSuccess && bytes) e = hipMemcpyAsync(dbase + dev_off, host + host_off, bytes, hipMemcpyHostToDevice, st);
    };
    if (e == hipSuccess) e = hipMemsetAsync(dbase + o_res, 0, o_ijobs - o_res, st);   // residual pool, job lists
    if (e == hipSuccess) e = hipMemsetAsync(dbase + o_ijobs, 0, o_rec - o_ijobs, st);
    // (16 chunks of 32 pictures at 512: the first H2D starts after 1/16 of the packing; 4 chunks measured
    // 78 ms per 512 1080p pictures, H2D-bound from the first chunk on)
    const int n_chunks = std::max(1, std::min(n_pics / 8, 16));
    for (int k = 0; k < n_chunks; ++k) {
        const int p0 = (int)((long long)n_pics * k / n_chunks), p1 = (int)((long long)n_pics * (k + 1) / n_chunks);
        parallel_for(p1 - p0, [&](int j) { pack_pic(p0 + j); });
        h2d(o_ctus + sizeof(p265r_ctu) * nc * (size_t)p0, o_ctus + sizeof(p265r_ctu) * nc * (size_t)p0,
            sizeof(p265r_ctu) * nc * (size_t)(p1 - p0));
        const size_t t1 = p1 < n_pics ? tb_at[p1] : n_tbs_total;
        h2d(o_tbs + sizeof(p265r_tb) * tb_at[p0], o_tbs + sizeof(p265r_tb) * tb_at[p0], sizeof(p265r_tb) * (t1 - tb_at[p0]));
        for (int c = 0; c < N_POOLS; ++c) {
            const size_t q0 = pool_at[p0][c], q1 = p1 < n_pics ? pool_at[p1][c] : pool_base[c] + pool_sz[c];
            h2d(o_pool + sizeof(int16_t) * q0, o_pool + sizeof(int16_t) * q0, sizeof(int16_t) * (q1 - q0));
        }
        for (int c = 0; c < RC_NUM; ++c) {
            const size_t j0 = (size_t)job_at[p0][c], j1 = p1 < n_pics ? (size_t)job_at[p1][c] : (size_t)n_jobs[c];
            h2d(o_jobs[c] + sizeof(ResJob) * j0, s_jobs + (o_jobs[c] - o_jobs[0]) + sizeof(ResJob) * j0, sizeof(ResJob) * (j1 - j0));
        }
        const size_t f1 = p1 < n_pics ? nf_at[p1] : n_nf;
        h2d(o_nf + nf_bytes * nf_at[p0], s_nf + nf_bytes * nf_at[p0], nf_bytes * (f1 - nf_at[p0]));
    }
    P265R_UT("pack");
    std::memcpy(host + o_pics, b->h_pics.data(), sizeof(DevPic) * n_pics);
    b->view.rec0 = dbase + o_rec;
    b->view.out0 = lf ? dbase + o_out : dbase + o_rec;
    b->view.pic_bytes = pic_plane_bytes;
    b->view.plane_off[0] = 0;
    b->view.plane_off[1] = align_up(plane_bytes[0], 256);
    b->view.plane_off[2] = b->view.plane_off[1] + align_up(plane_bytes[1], 256);
    b->view.ctus0 = reinterpret_cast<const p265r_ctu*>(dbase + o_ctus);
    b->view.err = b->d_err;
    std::memset(host + o_err, 0, o_ctus - o_err);                                        // error word
    std::memset(host + o_pics + sizeof(DevPic) * n_pics, 0, o_err - (o_pics + sizeof(DevPic) * n_pics));
    // alignment gaps between the arrays and the coefficient pool's pad: zero on the device, as the device
    // image always had them; then the DevPic table and the error word (complete before returning: the
    // staging buffer is refilled by the next upload)
    {
        const size_t ctus_end = o_ctus + sizeof(p265r_ctu) * nc * (size_t)n_pics;
        const size_t tbs_end = o_tbs + sizeof(p265r_tb) * n_tbs_total;
        const size_t pool_end = o_pool + sizeof(int16_t) * pool_total;
        if (e == hipSuccess && o_tbs > ctus_end) e = hipMemsetAsync(dbase + ctus_end, 0, o_tbs - ctus_end, st);
        if (e == hipSuccess && o_pool > tbs_end) e = hipMemsetAsync(dbase + tbs_end, 0, o_pool - tbs_end, st);
        if (e == hipSuccess && o_res > pool_end) e = hipMemsetAsync(dbase + pool_end, 0, o_res - pool_end, st);
    }
    h2d(0, 0, o_ctus);
    if (e == hipSuccess && recon_input) {
        for (int i = 0; i < n_pics && e == hipSuccess; ++i)
            for (int c = 0; c < 3 && e == hipSuccess; ++c) {
                const int wd[3] = {psize[i][0], psize[i][0] / 2, psize[i][0] / 2}, ht[3] = {psize[i][1], psize[i][1] / 2, psize[i][1] / 2};
                e = hipMemcpy2DAsync(b->h_pics[i].rec[c], g.stride[c] * pb, pics[i].recon[c], wd[c] * pb, wd[c] * pb, ht[c],
                                     hipMemcpyHostToDevice, st);
            }
    }
    P265R_UT("enqueue");
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    P265R_UT("h2d");
#if P265R_EXPERIMENTS
    if (ut) {
        fprintf(stderr, "[p265r] upload %d pictures, %.1f MB staged:", n_pics, (double)(o_res + jobs_bytes) / 1e6);
        for (size_t i = 1; i < tp.size(); ++i)
            fprintf(stderr, " %s %.2f ms", tp[i].first, std::chrono::duration<double, std::milli>(tp[i].second - tp[i - 1].second).count());
        fprintf(stderr, "\n");
    }
#endif
#undef P265R_UT
    if (e != hipSuccess) { int rc = hip_fail(e, "upload"); (void)hipFree(b->mem); delete b; return rc; }
    *out = b;
    return P265R_OK;
}

int p265r_batch_run(p265r_ctx* ctx, p265r_batch* b) {
    if (!ctx || !b) return P265R_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    hipStream_t s = b->stream;
    Geo g = ctx->geo;
    g.ragged = b->ragged ? 1 : 0;
    p265r_timings tm{};
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    if (ctx->timing) {
        for (auto& e : ev) {
            if (!ctx->spare.empty()) { e = ctx->spare.back(); ctx->spare.pop_back(); }
            else HIP_TRY(hipEventCreate(&e));
        }
        HIP_TRY(hipEventRecord(ev[0], s));
    }
    // ---- residual phase ----------------------------------------------------------
    const int bdl = g.bd[0], bdc = g.bd[1];
    const bool recon = !b->recon_input;
    // timing experiments only (P265R_SKIP bit 0: residual kernels, bit 1: job preparation, bit 2:
    // loop filters) on RE-RUNS of a resident batch: its residuals / job lists from the previous
    // run are still in place, so the output is unchanged while the skipped phase costs nothing
    const int skip = b->runs > 0 ? ctx->skip : 0;
    if (ctx->params.scaling_list_enabled && !ctx->d_sf && !b->recon_input) return P265R_ESTATE;   // factors not set
    const uint8_t* sf = ctx->params.scaling_list_enabled ? ctx->d_sf : nullptr;
    ++b->runs;
    ctx->lane_busy |= 1u << b->lane;
    const bool prep = recon && ctx->schedule == 1 && !(skip & 2);
    hipStream_t ps = s;                              // the prep kernel's stream
    // Stream plan of one run (no phase timing):
    // * a batch smaller than the chip (< 1 picture per CU: tile units, decoder batches, a few workgroups
    //   per launch) keeps every phase on its lane stream, and such batches run side by side: extra prep /
    //   residual streams would outnumber the hardware queues (4 by default) and put one lane's kernels
    //   behind another's (C5, 4 lanes: 2.3 M CTU/s forked vs 3.0 M unforked; 5.2 M unforked at
    //   GPU_MAX_HW_QUEUES=8, round 4);
    // * a chip-filling batch in a pipelined context runs in PHASE ORDER: its residual + prep phase (on
    //   two streams of the lane's own) waits for the last intra launch of ANY lane and runs beside the
    //   previous batch's loop filters; its intra phase waits for the last loop-filter launch, so the row
    //   kernel (W = 12, all of every CU's registers) always runs alone -- overlapping it with the other
    //   phases cost as much as it hid (3 lanes unordered = serial, 43.0 vs 43.5 M CTU/s, round 4);
    // * otherwise (a lone lane's re-runs) the EARLY residual phase: residual + prep start when this
    //   batch's previous intra phase ends, beside its previous loop filters.
    const bool big = b->n_pics >= ctx->num_cus;
    // P265R_SAO_AUX: the loop filters of this run go to the lane's aux stream (after its intra phase), the
    // prep kernel stays on the lane, so the next run's residual + prep phase overlaps this run's loop filters
    const bool sao_aux = P265R_SAO_AUX && !P265R_PHASE_ORDER && !P265R_EARLY_RESIDUAL && ctx->pipeline > 1 && big && prep &&
                         !ctx->timing && ctx->fork_prep == 1 && (b->sao || b->dbk) && !(skip & 4);
    const int fork_prep = big && !sao_aux ? ctx->fork_prep : 0;
    const bool ordered = P265R_PHASE_ORDER && ctx->pipeline > 1 && prep && fork_prep == 1 && !ctx->timing;
    const bool early = !ordered && P265R_EARLY_RESIDUAL && prep && fork_prep == 1 && !ctx->timing && b->intra_done &&
                       !(skip & 1);
    hipEvent_t r_after = ordered ? (ctx->last_intra_valid ? ctx->last_intra_ev : nullptr) : (early ? b->intra_done : nullptr);
    if (ordered && ctx->order_r == 0) r_after = b->intra_done;     // (A/B: residual phase not held back)
    hipStream_t rs = s;                              // the residual kernels' stream
    if ((ordered || early) && r_after) {
        const size_t li = (size_t)b->lane;
        if (ctx->aux2.size() <= li) { ctx->aux2.resize(li + 1, nullptr); ctx->join2_ev.resize(li + 1, nullptr); }
        if (!ctx->aux2[li]) {
            HIP_TRY(hipStreamCreateWithFlags(&ctx->aux2[li], hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&ctx->join2_ev[li], hipEventDisableTiming));
        }
        rs = ctx->aux2[li];
        HIP_TRY(hipStreamWaitEvent(rs, r_after, 0));
        // the batch's own previous intra phase (the last reader of its residual pool and job lists):
        // r_after is the last intra launch of ANY lane, which only orders after it when every intra
        // launch of the context ran phase-ordered (a small or timed batch on another lane does not)
        if (b->intra_done && r_after != b->intra_done) HIP_TRY(hipStreamWaitEvent(rs, b->intra_done, 0));
    }
    if (prep && fork_prep) {
        // fork_prep 2: one prep stream shared by all lanes (fewer streams than HW queues, so no
        // lane's intra kernel sits in front of a prep kernel in a shared hardware queue)
        const size_t li = fork_prep == 2 ? 0 : (size_t)b->lane;
        if (ctx->aux.size() <= li) {
            ctx->aux.resize(li + 1, nullptr); ctx->fork_ev.resize(li + 1, nullptr); ctx->join_ev.resize(li + 1, nullptr);
        }
        if (!ctx->aux[li]) {
            if (ctx->stream_prio) {
                int least = 0, greatest = 0;
                HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
                HIP_TRY(hipStreamCreateWithPriority(&ctx->aux[li], hipStreamNonBlocking, least));
            } else {
                HIP_TRY(hipStreamCreateWithFlags(&ctx->aux[li], hipStreamNonBlocking));
            }
            HIP_TRY(hipEventCreateWithFlags(&ctx->fork_ev[li], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&ctx->join_ev[li], hipEventDisableTiming));
        }
        ps = ctx->aux[li];
        if ((ordered || early) && r_after) {
            HIP_TRY(hipStreamWaitEvent(ps, r_after, 0));
            if (b->intra_done && r_after != b->intra_done) HIP_TRY(hipStreamWaitEvent(ps, b->intra_done, 0));
        } else {
            HIP_TRY(hipEventRecord(ctx->fork_ev[li], s));
            HIP_TRY(hipStreamWaitEvent(ps, ctx->fork_ev[li], 0));
        }
    }
    auto launch_prep = [&]() -> int {
        // intra job preparation (availability, filter decisions, Cb/Cr pairing): independent
        // of the residuals, timed with the residual phase; enqueued first so that, forked, its
        // waves start before the residual kernels fill the chip
        // (a superset of launch_rows' latency layouts: the cross-group kernel and the W = 16 split need
        // 2 n_pics <= CUs, the experiments' fixed W = 16 any size)
        Geo gp = g;
        gp.tr_info = (2 * (long long)b->n_pics <= ctx->num_cus || ctx->row_waves == 16) ? 1 : 0;
        intra_prep_kernel<<<dim3(g.wc, g.hc, b->n_pics), 64, ctx->prep_lds, ps>>>(b->d_pics, gp, b->view);
        ++tm.residual_launches;
        if (ps != s) HIP_TRY(hipEventRecord(ctx->join_ev[fork_prep == 2 ? 0 : (size_t)b->lane], ps));
        return P265R_OK;
    };
    if (prep && !ctx->prep_last) { int rc = launch_prep(); if (rc) return rc; }
    // (scaling lists: the SL instances, which read m from the context's ScalingFactor table)
#define P265R_RES_LAUNCH(K, KSL, blocks, ...)                                                                     \
    do {                                                                                                          \
        if (sf) KSL<<<(blocks), 256, ctx->res_lds, rs>>>(__VA_ARGS__, sf);                                        \
        else K<<<(blocks), 256, ctx->res_lds, rs>>>(__VA_ARGS__, nullptr);                                        \
        ++tm.residual_launches;                                                                                   \
    } while (0)
    if (recon && !(skip & 1) && b->n_jobs[RC_DST4])
        P265R_RES_LAUNCH((residual4_kernel<true, false>), (residual4_kernel<true, true>), (b->n_jobs[RC_DST4] + 255) / 256,
                         b->d_pool, b->d_res, b->d_jobs[RC_DST4], b->n_jobs[RC_DST4], bdl, b->slab[RC_DST4]);
    if (recon && !(skip & 1) && b->n_jobs[RC_DCT4])
        P265R_RES_LAUNCH((residual4_kernel<false, false>), (residual4_kernel<false, true>), (b->n_jobs[RC_DCT4] + 255) / 256,
                         b->d_pool, b->d_res, b->d_jobs[RC_DCT4], b->n_jobs[RC_DCT4], bdc, b->slab[RC_DCT4]);
    if (recon && !(skip & 1) && b->n_jobs[RC_DCT8])
        P265R_RES_LAUNCH((residualN_kernel<3, false>), (residualN_kernel<3, true>), (b->n_jobs[RC_DCT8] + 31) / 32,
                         b->d_pool, b->d_res, b->d_jobs[RC_DCT8], b->n_jobs[RC_DCT8], bdl, bdc, b->slab[RC_DCT8]);
    if (recon && !(skip & 1) && b->n_jobs[RC_DCT16])
        P265R_RES_LAUNCH((residualN_kernel<4, false>), (residualN_kernel<4, true>), (b->n_jobs[RC_DCT16] + 15) / 16,
                         b->d_pool, b->d_res, b->d_jobs[RC_DCT16], b->n_jobs[RC_DCT16], bdl, bdc, b->slab[RC_DCT16]);
    if (recon && !(skip & 1) && b->n_jobs[RC_DCT32])
        P265R_RES_LAUNCH((residualN_kernel<5, false>), (residualN_kernel<5, true>), (b->n_jobs[RC_DCT32] + 7) / 8,
                         b->d_pool, b->d_res, b->d_jobs[RC_DCT32], b->n_jobs[RC_DCT32], bdl, bdc, b->slab[RC_DCT32]);
#undef P265R_RES_LAUNCH
    if (recon && !(skip & 1) && b->n_jobs[RC_TSKIP]) {
        residual_tskip_kernel<<<(b->n_jobs[RC_TSKIP] + 255) / 256, 256, 0, rs>>>(b->d_pool, b->d_res, b->d_jobs[RC_TSKIP], b->n_jobs[RC_TSKIP], bdl, bdc, sf);
        ++tm.residual_launches;
    }
    if (prep && ctx->prep_last) { int rc = launch_prep(); if (rc) return rc; }
    if (prep && ps != s) HIP_TRY(hipStreamWaitEvent(s, ctx->join_ev[fork_prep == 2 ? 0 : (size_t)b->lane], 0));
    if (rs != s) {
        HIP_TRY(hipEventRecord(ctx->join2_ev[(size_t)b->lane], rs));
        HIP_TRY(hipStreamWaitEvent(s, ctx->join2_ev[(size_t)b->lane], 0));
    }
    if (b->dbk) {
        // deblocking edge / QpY map: depends on the records only
        if (g.pel16) dbk_map_kernel<uint16_t><<<dim3(ctx->n_ctus, b->n_pics), 64, 0, s>>>(b->d_pics, g);
        else dbk_map_kernel<uint8_t><<<dim3(ctx->n_ctus, b->n_pics), 64, 0, s>>>(b->d_pics, g);   // (context-size grid)
        ++tm.residual_launches;
    }
    HIP_TRY(hipGetLastError());
    if (ctx->debug_sync) { fprintf(stderr, "[p265r] residual phase enqueued\n"); HIP_TRY(hipStreamSynchronize(s)); fprintf(stderr, "[p265r] residual phase done\n"); }
    if (ctx->timing) HIP_TRY(hipEventRecord(ev[1], s));
    // ---- intra wavefront ---------------------------------------------------------------
    if (recon && ctx->schedule == 1) {
        // per-CU workgroup slots cleared per run; the error word (d_err[0]) is sticky from upload on,
        // so p265r_batch_status / p265r_batch_download report a give-up in ANY run of the batch
        // (and the cross-group kernel's progress words behind them)
        HIP_TRY(hipMemsetAsync(b->d_err + 64, 0, kRowCuSlots * 16 + (b->d_xg_prog ? sizeof(int) * 2 * ((size_t)g.hc + 1) * b->n_pics : 0), s));
        // the previous run's loop filters (on the aux stream) read the planes this run writes
        if (b->sao_pending) { HIP_TRY(hipStreamWaitEvent(s, b->sao_done, 0)); b->sao_pending = false; }
        if (ordered && ctx->last_lf_valid) HIP_TRY(hipStreamWaitEvent(s, ctx->last_lf_ev, 0));
        // does another lane have a run enqueued that the API has not synchronised since?  (host
        // state only, so the build a run gets is a function of the call sequence)
        // (phase order: the intra phase has the GPU to itself by construction)
        bool alone = ordered || (ctx->lane_busy & ~(1u << b->lane)) == 0u;
#ifdef P265R_ALONE_PIPE
        alone = alone && ctx->pipeline == 1;       // A/B: a pipelined context never runs the W = 12 build
#endif
        int rc = launch_rows(ctx, b, s, alone);
        if (rc) return rc;
        ++tm.intra_launches;
    }
    const int n_steps = (recon && ctx->schedule == 0) ? (g.wc - 1) + 2 * (g.hc - 1) + 1 : 0;
    for (int step = 0; step < n_steps; ++step) {
        const int d = step - (g.wc - 1);
        const int cy_min = d > 0 ? (d + 1) / 2 : 0;
        const int cy_max = std::min(g.hc - 1, step / 2);
        if (cy_max < cy_min) continue;
        dim3 grid(cy_max - cy_min + 1, b->n_pics);
        if (g.pel16) intra_step_kernel<uint16_t><<<grid, 64, 0, s>>>(b->d_pics, b->d_pool, b->d_res, g, step, cy_min);
        else intra_step_kernel<uint8_t><<<grid, 64, 0, s>>>(b->d_pics, b->d_pool, b->d_res, g, step, cy_min);
        ++tm.intra_launches;
    }
    HIP_TRY(hipGetLastError());
    if (recon) {                                     // the residual pool and job lists are free again
        if (!b->intra_done) HIP_TRY(hipEventCreateWithFlags(&b->intra_done, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(b->intra_done, s));
        if (!ctx->last_intra_ev) HIP_TRY(hipEventCreateWithFlags(&ctx->last_intra_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ctx->last_intra_ev, s));
        ctx->last_intra_valid = true;
    }
    if (ctx->debug_sync) { fprintf(stderr, "[p265r] intra phase enqueued\n"); HIP_TRY(hipStreamSynchronize(s)); fprintf(stderr, "[p265r] intra phase done\n"); }
    if (ctx->timing) HIP_TRY(hipEventRecord(ev[2], s));
    // ---- in-loop filters: deblocking + SAO ----------------------------------------------
    const hipStream_t lane_s = s;
    if (sao_aux) {
        const size_t li = (size_t)b->lane;
        if (ctx->aux.size() <= li) {
            ctx->aux.resize(li + 1, nullptr); ctx->fork_ev.resize(li + 1, nullptr); ctx->join_ev.resize(li + 1, nullptr);
        }
        if (!ctx->aux[li]) {
            HIP_TRY(hipStreamCreateWithFlags(&ctx->aux[li], hipStreamNonBlocking));
            HIP_TRY(hipEventCreateWithFlags(&ctx->fork_ev[li], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&ctx->join_ev[li], hipEventDisableTiming));
        }
        if (!b->sao_done) HIP_TRY(hipEventCreateWithFlags(&b->sao_done, hipEventDisableTiming));
        s = ctx->aux[li];
        HIP_TRY(hipStreamWaitEvent(s, b->intra_done, 0));
    }
    if (g.pel16 && b->sao && !b->dbk && !(skip & 4)) {
        // 16-bit samples, SAO only: the strip kernel (sao16.h), 8 samples per lane, one wave per (picture,
        // CTB row, component, 496-sample strip), 4 waves per block, blocks dealt XCD-aware
        const long long waves = (long long)sao16b_units(g) * b->n_pics;
        if (waves >= (1ll << 31) - 64) return P265R_ERANGE;
        const unsigned blocks = (unsigned)((waves + 3) / 4 + 7) / 8 * 8;
        sao16_strip_kernel<<<blocks, 256, 0, s>>>(b->d_pics, g, b->view, b->n_pics);
        ++tm.sao_launches;
        HIP_TRY(hipGetLastError());
    } else if (g.pel16 && (b->dbk || b->sao) && !(skip & 4)) {
        // 16-bit samples (Main 10): deblocking + SAO in loopfilter16.h, with or without deblocking
        const long long units = (long long)ctx->n_ctus * b->n_pics;
        if (units >= (1ll << 31) - 8) return P265R_ERANGE;
        const dim3 grid((unsigned)((units + 7) / 8 * 8));
        const int so = b->sao ? 1 : 0, np = b->n_pics;
        switch (g.ctb_log2 * 2 + (b->dbk ? 1 : 0)) {
            case 12: loopfilter16_kernel<6, false><<<grid, 256, 0, s>>>(b->d_pics, g, so, np); break;
            case 13: loopfilter16_kernel<6, true><<<grid, 256, 0, s>>>(b->d_pics, g, so, np); break;
            case 10: loopfilter16_kernel<5, false><<<grid, 256, 0, s>>>(b->d_pics, g, so, np); break;
            case 11: loopfilter16_kernel<5, true><<<grid, 256, 0, s>>>(b->d_pics, g, so, np); break;
            case 8: loopfilter16_kernel<4, false><<<grid, 256, 0, s>>>(b->d_pics, g, so, np); break;
            default: loopfilter16_kernel<4, true><<<grid, 256, 0, s>>>(b->d_pics, g, so, np); break;
        }
        ++tm.sao_launches;
        HIP_TRY(hipGetLastError());
    } else if (b->sao && !b->dbk && ctx->sao_rows == 1 && g.ctb_log2 >= 5 && g.h % 8 == 0 && !(skip & 4)) {
        // SAO only, CTB 32 / 64: the 16-samples-per-lane strip kernel (sao_strip16.h), one wave per
        // (picture, CTB row, component, 992-sample strip), 4 waves per block, blocks dealt XCD-aware;
        // it filters 4-row chunks and takes plane heights in multiples of 4 (luma a multiple of
        // MinCbSizeY >= 8 in a conforming stream; anything else goes to the 4-B strip kernel)
        const long long waves = (long long)sao16_units(g) * b->n_pics;
        if (waves >= (1ll << 31) - 64) return P265R_ERANGE;
        const unsigned blocks = (unsigned)((waves + 3) / 4 + 7) / 8 * 8;
        if (g.ctb_log2 == 6) sao_strip16_kernel<6><<<blocks, 256, ctx->sao_lds, s>>>(b->d_pics, g, b->view, b->n_pics);
        else sao_strip16_kernel<5><<<blocks, 256, ctx->sao_lds, s>>>(b->d_pics, g, b->view, b->n_pics);
        ++tm.sao_launches;
        HIP_TRY(hipGetLastError());
    } else if (b->sao && !b->dbk && ctx->sao_rows && !(skip & 4)) {
        // SAO only, CTB 16 (or P265R_SAO_ROWS=2): the strip kernel (sao_rows.h), one wave per
        // (picture, component, CTB row, 248-sample strip), 4 waves per block, blocks dealt XCD-aware
        const long long waves = (long long)sao_rows_units(g) * b->n_pics;
        if (waves >= (1ll << 31) - 64) return P265R_ERANGE;
        const long long blocks = (waves + 3) / 4;
        sao_rows_kernel<<<(unsigned)((blocks + 7) / 8 * 8), 256, 0, s>>>(b->d_pics, g, b->n_pics);
        ++tm.sao_launches;
        HIP_TRY(hipGetLastError());
    } else if ((b->dbk || b->sao) && !(skip & 4)) {
        const long long units = (long long)ctx->n_ctus * b->n_pics;
        if (units >= (1ll << 31) - 8) return P265R_ERANGE;
        const dim3 grid((unsigned)((units + 7) / 8 * 8));
        const int so = b->sao ? 1 : 0, np = b->n_pics;
        switch (g.ctb_log2 * 2 + (b->dbk ? 1 : 0)) {
            case 12: loopfilter_kernel<6, false><<<grid, LfShape<6>::threads(false), 0, s>>>(b->d_pics, g, so, np); break;
            case 13: loopfilter_kernel<6, true><<<grid, LfShape<6>::threads(true), 0, s>>>(b->d_pics, g, so, np); break;
            case 10: loopfilter_kernel<5, false><<<grid, LfShape<5>::threads(false), 0, s>>>(b->d_pics, g, so, np); break;
            case 11: loopfilter_kernel<5, true><<<grid, LfShape<5>::threads(true), 0, s>>>(b->d_pics, g, so, np); break;
            case 8: loopfilter_kernel<4, false><<<grid, LfShape<4>::threads(false), 0, s>>>(b->d_pics, g, so, np); break;
            default: loopfilter_kernel<4, true><<<grid, LfShape<4>::threads(true), 0, s>>>(b->d_pics, g, so, np); break;
        }
        ++tm.sao_launches;
        HIP_TRY(hipGetLastError());
    }
    if (sao_aux) {
        HIP_TRY(hipEventRecord(b->sao_done, s));
        b->sao_pending = true;
        s = lane_s;
    }
    if (ordered) {                                   // the next batch's intra phase starts after this
        if (!ctx->last_lf_ev) HIP_TRY(hipEventCreateWithFlags(&ctx->last_lf_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(ctx->last_lf_ev, s));
        ctx->last_lf_valid = true;
    }
    if (ctx->timing) {
        HIP_TRY(hipEventRecord(ev[3], s));
        p265r_ctx::Run run;
        for (int i = 0; i < 4; ++i) run.ev[i] = ev[i];
        run.counts = tm;
        ctx->runs.push_back(run);
        ctx->have_timing = true;
    }
    return P265R_OK;
}

int p265r_batch_download(p265r_ctx* ctx, p265r_batch* b, const p265r_picture* pics, int n_pics) {
    if (!ctx || !b || !pics || n_pics != b->n_pics) return P265R_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = join_sao(b)) return rc;
    const Geo& g = ctx->geo;
    // planes to copy: (host destination, device source, row pitch, width, height)
    struct Item { void* dst; const unsigned char* src; int pitch, w, h; size_t bytes; };
    std::vector<Item> items;
    const int pb = g.pel16 ? 2 : 1;                          // bytes per sample
    for (int i = 0; i < n_pics; ++i)
        for (int c = 0; c < 3; ++c) {
            const int sub = c ? 1 : 0;
            const int w = (b->size[i][0] >> sub) * pb, h = b->size[i][1] >> sub;     // (w in bytes)
            const int pitch = (c ? g.stride[1] : g.stride[0]) * pb;
            if (pics[i].out[c]) items.push_back({pics[i].out[c], b->h_pics[i].out[c], pitch, w, h, (size_t)w * h});
            if (pics[i].recon[c] && !b->recon_input)
                items.push_back({pics[i].recon[c], b->h_pics[i].rec[c], pitch, w, h, (size_t)w * h});
        }
    // D2H through two halves of a pinned bounce buffer (DMA at pinned speed; the copy into the
    // caller's pageable planes runs on host threads while the next chunk's DMA is in flight)
    if (!ctx->dl_stage) {
        if (hipHostMalloc(reinterpret_cast<void**>(&ctx->dl_stage), 2 * kDlHalf, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            ctx->dl_stage = nullptr;
        }
    }
    if (!ctx->dl_stage) {                                   // no pinned memory: straight pageable copies
        for (const Item& it : items)
            HIP_TRY(hipMemcpy2DAsync(it.dst, it.w, it.src, it.pitch, it.w, it.h, hipMemcpyDeviceToHost, b->stream));
        return p265r_batch_status(ctx, b);
    }
    if (!ctx->dl_ev[0]) {
        HIP_TRY(hipEventCreateWithFlags(&ctx->dl_ev[0], hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&ctx->dl_ev[1], hipEventDisableTiming));
    }
    // chunks: consecutive items of at most kDlHalf bytes (an item larger than that goes alone, direct)
    std::vector<std::pair<size_t, size_t>> chunks;          // [first, last) item
    for (size_t i = 0; i < items.size();) {
        size_t j = i, bytes = 0;
        while (j < items.size() && (j == i || bytes + items[j].bytes <= kDlHalf)) bytes += items[j++].bytes;
        chunks.push_back({i, j});
        i = j;
    }
    auto enqueue = [&](size_t k) -> hipError_t {
        unsigned char* st = ctx->dl_stage + (k & 1) * kDlHalf;
        size_t off = 0;
        for (size_t i = chunks[k].first; i < chunks[k].second; ++i) {
            const Item& it = items[i];
            hipError_t e = it.bytes > kDlHalf
                ? hipMemcpy2DAsync(it.dst, it.w, it.src, it.pitch, it.w, it.h, hipMemcpyDeviceToHost, b->stream)
                : hipMemcpy2DAsync(st + off, it.w, it.src, it.pitch, it.w, it.h, hipMemcpyDeviceToHost, b->stream);
            if (e != hipSuccess) return e;
            off += it.bytes;
        }
        return hipEventRecord(ctx->dl_ev[k & 1], b->stream);
    };
    if (!chunks.empty()) HIP_TRY(enqueue(0));
    for (size_t k = 0; k < chunks.size(); ++k) {
        if (k + 1 < chunks.size()) HIP_TRY(enqueue(k + 1));          // into the other half (its copy-out is done)
        HIP_TRY(hipEventSynchronize(ctx->dl_ev[k & 1]));
        const unsigned char* st = ctx->dl_stage + (k & 1) * kDlHalf;
        const size_t first = chunks[k].first, n = chunks[k].second - first;
        std::vector<size_t> offs(n);
        for (size_t i = 0, off = 0; i < n; ++i) { offs[i] = off; off += items[first + i].bytes; }
        parallel_for((int)n, [&](int i) {
            const Item& it = items[first + i];
            if (it.bytes <= kDlHalf) std::memcpy(it.dst, st + offs[i], it.bytes);
        });
    }
    return p265r_batch_status(ctx, b);
}

int p265r_batch_status(p265r_ctx* ctx, p265r_batch* b) {
    if (!ctx || !b) return P265R_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = join_sao(b)) return rc;
    HIP_TRY(hipStreamSynchronize(b->stream));
    // the lane is idle now (every run on it, of any batch, has completed)
    ctx->lane_busy &= ~(1u << b->lane);
    int err = 0;
    HIP_TRY(hipMemcpy(&err, b->d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (err) {
        g_last_hip_error = (err & 1) ? "intra row pipeline: dependency wait timed out"
                                     : "job prep self-check (P265R_TR_CHECK): a job covering the bottom row's left half "
                                       "comes after the half-CTU publish point";
        return P265R_EHIP;
    }
    return P265R_OK;
}

int p265r_batch_digest(p265r_ctx* ctx, p265r_batch* b, int which, uint64_t* out, int n) {
    if (!ctx || !b || !out || n != 3 * b->n_pics || (which != 0 && which != 1)) return P265R_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = join_sao(b)) return rc;
    // after every run enqueued on the batch's lane (stream order); one device buffer per call
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d), sizeof(uint64_t) * (size_t)n));
    hipError_t e = hipMemsetAsync(d, 0, sizeof(uint64_t) * (size_t)n, b->stream);
    if (e == hipSuccess) {
        const dim3 grid((unsigned)((ctx->geo.h + kDigestRows - 1) / kDigestRows), 3, (unsigned)b->n_pics);
        digest_kernel<<<grid, 256, 0, b->stream>>>(b->d_pics, ctx->geo, which == 0 ? 1 : 0, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(out, d, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToHost, b->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(b->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return hip_fail(e, "p265r_batch_digest");
    return p265r_batch_status(ctx, b);
}

int p265r_batch_digest_async(p265r_ctx* ctx, p265r_batch* b, int which, int slot) {
    if (!ctx || !b || (which != 0 && which != 1) || slot < 0 || slot >= P265R_DIGEST_SLOTS) return P265R_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = join_sao(b)) return rc;
    const size_t per_slot = sizeof(uint64_t) * 3 * (size_t)b->n_pics;
    if (!b->d_dig) {
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&b->d_dig), per_slot * P265R_DIGEST_SLOTS));
        HIP_TRY(hipMemsetAsync(b->d_dig, 0, per_slot * P265R_DIGEST_SLOTS, b->stream));
    }
    unsigned long long* d = b->d_dig + 3 * (size_t)b->n_pics * slot;
    HIP_TRY(hipMemsetAsync(d, 0, per_slot, b->stream));
    const dim3 grid((unsigned)((ctx->geo.h + kDigestRows - 1) / kDigestRows), 3, (unsigned)b->n_pics);
    digest_kernel<<<grid, 256, 0, b->stream>>>(b->d_pics, ctx->geo, which == 0 ? 1 : 0, d);
    HIP_TRY(hipGetLastError());
    ctx->lane_busy |= 1u << b->lane;
    return P265R_OK;
}

int p265r_batch_digest_slots(p265r_ctx* ctx, p265r_batch* b, uint64_t* out, int n_slots) {
    if (!ctx || !b || !out || n_slots < 1 || n_slots > P265R_DIGEST_SLOTS) return P265R_EINVAL;
    if (!b->d_dig) return P265R_ESTATE;
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = join_sao(b)) return rc;
    HIP_TRY(hipMemcpyAsync(out, b->d_dig, sizeof(uint64_t) * 3 * (size_t)b->n_pics * n_slots, hipMemcpyDeviceToHost,
                           b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return p265r_batch_status(ctx, b);
}

int p265r_batch_job_count(p265r_ctx* ctx, p265r_batch* b, uint64_t* luma, uint64_t* chroma) {
    if (!ctx || !b || !luma || !chroma) return P265R_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    HIP_TRY(hipStreamSynchronize(b->stream));
    // per CTU slot: luma jobs | chroma jobs << 16, top-right indices (intra_prep.h), context-size slots
    const size_t n = (size_t)ctx->n_ctus * b->n_pics;
    std::vector<uint32_t> jc(4 * n);
    HIP_TRY(hipMemcpy(jc.data(), b->h_pics[0].jcount, 4 * sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
    uint64_t l = 0, c = 0;
    for (size_t i = 0; i < n; ++i) { l += jc[4 * i] & 0xffffu; c += jc[4 * i] >> 16; }
    *luma = l;
    *chroma = c;
    return P265R_OK;
}

int p265r_batch_free(p265r_ctx* ctx, p265r_batch* b) {
    if (!ctx || !b) return P265R_EINVAL;
    (void)hipSetDevice(ctx->device);
    (void)join_sao(b);
    if (ctx->pending == b) ctx->pending = nullptr;
    // its lane may still run it: the allocation is reused by the next upload (another stream); the
    // lane stream's last run waited for every residual / prep kernel of the batch
    hipError_t e = b->stream ? hipStreamSynchronize(b->stream) : hipSuccess;
    if (b->intra_done) (void)hipEventDestroy(b->intra_done);
    if (b->sao_done) (void)hipEventDestroy(b->sao_done);
    if (b->d_dig) (void)hipFree(b->d_dig);
    if (b->mem) {
        // keep the larger of (cache, this allocation) for the next upload (its runs are complete)
        if (!ctx->cache_mem || b->bytes > ctx->cache_bytes) {
            if (ctx->cache_mem) e = hipFree(ctx->cache_mem);
            ctx->cache_mem = b->mem;
            ctx->cache_bytes = b->bytes;
        } else {
            e = hipFree(b->mem);
        }
    }
    delete b;
    return e == hipSuccess ? P265R_OK : hip_fail(e, "hipFree");
}

int p265r_submit(p265r_ctx* ctx, const p265r_picture* pics, int n_pics) {
    if (!ctx) return P265R_EINVAL;
    if (ctx->pending) return P265R_ESTATE;
    p265r_batch* b = nullptr;
    int rc = p265r_batch_upload(ctx, pics, n_pics, &b);
    if (rc) return rc;
    rc = p265r_batch_run(ctx, b);
    if (rc) { p265r_batch_free(ctx, b); return rc; }
    ctx->pending = b;
    ctx->pending_pics.assign(pics, pics + n_pics);
    return P265R_OK;
}

int p265r_wait(p265r_ctx* ctx) {
    if (!ctx) return P265R_EINVAL;
    if (!ctx->pending) return P265R_ESTATE;
    p265r_batch* b = ctx->pending;
    int rc = p265r_batch_download(ctx, b, ctx->pending_pics.data(), (int)ctx->pending_pics.size());
    ctx->pending = nullptr;
    ctx->pending_pics.clear();
    int rc2 = p265r_batch_free(ctx, b);
    return rc ? rc : rc2;
}

int p265r_sync(p265r_ctx* ctx) {
    if (!ctx) return P265R_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    for (hipStream_t st : ctx->lanes) HIP_TRY(hipStreamSynchronize(st));
    for (hipStream_t st : ctx->aux) if (st) HIP_TRY(hipStreamSynchronize(st));
    for (hipStream_t st : ctx->aux2) if (st) HIP_TRY(hipStreamSynchronize(st));
    ctx->lane_busy = 0;
    return P265R_OK;
}

int p265r_set_pipeline(p265r_ctx* ctx, int depth) {
    if (!ctx || depth < 1 || depth > 16) return P265R_EINVAL;
    HIP_TRY(hipSetDevice(ctx->device));
    while ((int)ctx->lanes.size() < depth) {
        hipStream_t st = nullptr;
        HIP_TRY(lane_stream_create(ctx, &st));
        ctx->lanes.push_back(st);
    }
    ctx->pipeline = depth;
    ctx->next_lane = 0;
    return P265R_OK;
}

// GPU_MAX_HW_QUEUES as the HIP runtime read it at initialisation (HIP's default 4 when unset)
static const char* hwq_env() {
    const char* v = std::getenv("GPU_MAX_HW_QUEUES");
    return (v && std::strlen(v) < 8 && std::strspn(v, "0123456789") == std::strlen(v)) ? v : "default";
}

int p265r_describe(p265r_ctx* ctx, char* buf, int size) {
    if (!ctx || size < 0 || (size > 0 && !buf)) return P265R_EINVAL;
    const Geo& g = ctx->geo;
    char tmp[2048];
    const int n = snprintf(tmp, sizeof(tmp),
        "{\"schedule\": \"%s\", \"row_waves\": %d, \"row_waves_by_run\": \"%s\", \"lean\": %d, "
        "\"fair\": %d, \"quad\": %d, \"luma_lead\": %d, \"sao_rows\": %d, \"skip\": %d, \"debug_sync\": %d, "
        "\"pipeline\": %d, \"fork_prep\": %d, \"pipe_waves\": %d, \"hw_queues\": \"%s\", \"num_cus\": %d, \"diag_build\": %d, "
        "\"experiments_build\": %d, \"split\": %d, \"last_launch_split\": %d, \"xg\": %d, \"last_launch_xg\": %d, "
        "\"phase_order\": %d, \"early_residual\": %d, \"bit_depth\": %d, \"row_launches\": {\"w12\": %lld, \"w8\": %lld, \"w16_split\": %lld, \"xg\": %lld, \"other\": %lld}, "
        "\"env_overrides\": [%s]}",
        ctx->schedule ? "rows" : "steps", ctx->row_waves,
        ctx->row_waves ? "fixed" : (P265R_PHASE_ORDER
                                   ? "batches of >= 1 picture per CU in a pipelined context: W=12, one intra launch at a time "
                                     "(phase order); small batches (< 1 picture per CU: component split, W=16): side by side; "
                                     "otherwise W=12 while no other lane has a run enqueued since the API synchronised it, "
                                     "else pipe_waves"
                                   : "batches of <= CUs / (2 xg) pictures: every luma / chroma chain on xg workgroups of W=4 "
                                     "(cross-group rows, progress and lines in global memory); small batches (< 1 picture per "
                                     "CU: component split, W=16); otherwise W=12 while no other "
                                     "lane has a run enqueued since the API synchronised it, else pipe_waves (W=8, 80 VGPRs: "
                                     "the other lanes' residual / prep / SAO waves fit beside it)"),
        ctx->lean, g.fair, g.quad, ctx->luma_lead, ctx->sao_rows, ctx->skip, ctx->debug_sync ? 1 : 0,
        ctx->pipeline, ctx->fork_prep, ctx->pipe_waves, hwq_env(), ctx->num_cus,
#ifdef P265R_DEBUG_DIAG
        1,
#else
        0,
#endif
        P265R_EXPERIMENTS, ctx->split, ctx->last_split ? 1 : 0, ctx->xg, ctx->last_xg ? 1 : 0, P265R_PHASE_ORDER, P265R_EARLY_RESIDUAL,
        (int)ctx->params.bit_depth_luma, ctx->row_launches[0], ctx->row_launches[1], ctx->row_launches[2], ctx->row_launches[3], ctx->row_launches[4],
        ctx->describe.c_str());
    if (n < 0) return P265R_EINVAL;
    if (size > 0) {
        const int k = std::min(n, size - 1);
        std::memcpy(buf, tmp, (size_t)k);
        buf[k] = 0;
    }
    return n;
}

int p265r_set_scaling_factors(p265r_ctx* ctx, const uint8_t* factors, int n_bytes) {
    if (!ctx || !factors || n_bytes != P265R_SCALING_FACTOR_BYTES) return P265R_EINVAL;
    if (!ctx->params.scaling_list_enabled) return P265R_ESTATE;
    for (int i = 0; i < n_bytes; ++i)
        if (factors[i] == 0) return P265R_EINVAL;              // ScalingFactor is 1..255 (7.4.5)
    HIP_TRY(hipSetDevice(ctx->device));
    if (int rc = p265r_sync(ctx)) return rc;                    // no run in flight reads the old table
    if (!ctx->d_sf) HIP_TRY(hipMalloc(reinterpret_cast<void**>(&ctx->d_sf), P265R_SCALING_FACTOR_BYTES));
    HIP_TRY(hipMemcpy(ctx->d_sf, factors, P265R_SCALING_FACTOR_BYTES, hipMemcpyHostToDevice));
    return P265R_OK;
}

int p265r_set_row_waves(p265r_ctx* ctx, int waves) {
    if (!ctx || (waves != 0 && waves != 8 && waves != 12)) return P265R_EINVAL;
    ctx->row_waves = waves;
    return P265R_OK;
}

int p265r_set_timing(p265r_ctx* ctx, int enable) {
    if (!ctx) return P265R_EINVAL;
    ctx->timing = enable != 0;
    if (enable) {                               // start a new accumulation
        for (auto& r : ctx->runs) for (auto& e : r.ev) ctx->spare.push_back(e);
        ctx->runs.clear();
        ctx->have_timing = false;
    }
    return P265R_OK;
}

namespace {
int run_times(const p265r_ctx::Run& r, p265r_timings* t) {
    HIP_TRY(hipEventSynchronize(r.ev[3]));
    float a = 0, b = 0, c = 0, tt = 0;
    HIP_TRY(hipEventElapsedTime(&a, r.ev[0], r.ev[1]));
    HIP_TRY(hipEventElapsedTime(&b, r.ev[1], r.ev[2]));
    HIP_TRY(hipEventElapsedTime(&c, r.ev[2], r.ev[3]));
    HIP_TRY(hipEventElapsedTime(&tt, r.ev[0], r.ev[3]));
    *t = r.counts;
    t->residual_ms = a; t->intra_ms = b; t->sao_ms = c; t->total_ms = tt;
    return P265R_OK;
}
}  // namespace

int p265r_last_timings(p265r_ctx* ctx, p265r_timings* out) {
    if (!ctx || !out) return P265R_EINVAL;
    if (!ctx->have_timing || ctx->runs.empty()) return P265R_ESTATE;
    HIP_TRY(hipSetDevice(ctx->device));
    return run_times(ctx->runs.back(), out);
}

int p265r_timings_total(p265r_ctx* ctx, p265r_timings* out, int* n_runs) {
    if (!ctx || !out) return P265R_EINVAL;
    if (!ctx->have_timing || ctx->runs.empty()) return P265R_ESTATE;
    HIP_TRY(hipSetDevice(ctx->device));
    p265r_timings sum{};
    for (const auto& r : ctx->runs) {
        p265r_timings t{};
        int rc = run_times(r, &t);
        if (rc) return rc;
        sum.total_ms += t.total_ms; sum.residual_ms += t.residual_ms; sum.intra_ms += t.intra_ms; sum.sao_ms += t.sao_ms;
        sum.intra_launches += t.intra_launches; sum.residual_launches += t.residual_launches;
        sum.sao_launches += t.sao_launches;
    }
    if (n_runs) *n_runs = (int)ctx->runs.size();
    *out = sum;
    return P265R_OK;
}

}  // extern "C"
