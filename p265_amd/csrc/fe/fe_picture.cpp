// Slice segment data of all-intra pictures -> back-end records (H.265 7.3.8, 9.3).
//
// Reference counterparts (decoder/): SliceSegmentData.parse (slice.py:234-296), Ctu.parse
// (ctu.py:24-30), Sao.parse (sao.py:15-220), Cu.parse / parse_leaf / parse_intra_pred_mode /
// parse__split_cu_flag / parse__part_mode (cu.py:41-471), Cu.decode_qp (cu.py:496-593),
// Tu.parse / parse_leaf / parse_residual_coding and the per-syntax-element context
// selection (tu.py:11-665), and the context tables of cabac.py:13-63.  The reference
// builds an object tree per CTU and hands leaf CUs to Cu.decode_leaf (cu.py:483); here
// each leaf CU directly appends its records in the layout PictureBuilder.add_cu /
// add_ctu (p265_amd/frontend.py) produces, which is what the GPU back-end consumes.
//
// Beyond the reference (which raises or is wrong there): tiles, WPP
// context synchronisation, dependent slice segments, cu_qp_delta, PCM,
// cu_transquant_bypass, SAO EO sign inference, end_of_subset_one_bit.
#include "fe_picture.h"

#include <algorithm>
#include <cstring>

namespace p265fe {

const uint8_t kLpsTable[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205}, {116, 142, 169, 195},
    {111, 135, 160, 185}, {105, 128, 152, 175}, {100, 122, 144, 166}, {95, 116, 137, 158}, {90, 110, 130, 150},
    {85, 104, 123, 142},  {81, 99, 117, 135},   {77, 94, 111, 128},   {73, 89, 105, 122},  {69, 85, 100, 116},
    {66, 80, 95, 110},    {62, 76, 90, 104},    {59, 72, 86, 99},     {56, 69, 81, 94},    {53, 65, 77, 89},
    {51, 62, 73, 85},     {48, 59, 69, 80},     {46, 56, 66, 76},     {43, 53, 63, 72},    {41, 50, 59, 69},
    {39, 48, 56, 65},     {37, 45, 54, 62},     {35, 43, 51, 59},     {33, 41, 48, 56},    {32, 39, 46, 53},
    {30, 37, 43, 50},     {29, 35, 41, 48},     {27, 33, 39, 45},     {26, 31, 37, 43},    {24, 30, 35, 41},
    {23, 28, 33, 39},     {22, 27, 32, 37},     {21, 26, 30, 35},     {20, 24, 29, 33},    {19, 23, 27, 31},
    {18, 22, 26, 30},     {17, 21, 25, 28},     {16, 20, 23, 27},     {15, 19, 22, 25},    {14, 18, 21, 24},
    {14, 17, 20, 23},     {13, 16, 19, 22},     {12, 15, 18, 21},     {12, 14, 17, 20},    {11, 14, 16, 19},
    {11, 13, 15, 18},     {10, 12, 15, 17},     {10, 12, 14, 16},     {9, 11, 13, 15},     {9, 11, 12, 14},
    {8, 10, 12, 14},      {8, 9, 11, 13},       {7, 9, 11, 12},       {7, 9, 10, 12},      {7, 8, 10, 11},
    {6, 8, 9, 11},        {6, 7, 9, 10},        {6, 7, 8, 9},         {2, 2, 2, 2}};
const uint8_t kNextStateMps[64] = {1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16,
                                   17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32,
                                   33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47, 48,
                                   49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 62, 63};
const uint8_t kNextStateLps[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12,
                                   13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, 24,
                                   24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33,
                                   33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};

// kTransTable[(pStateIdx << 1) | valMps][bin is the LPS]: kNextStateMps / kNextStateLps folded per state word,
// with the valMps flip of an LPS at pStateIdx 0 (9.3.4.3.2.2); generated from the two tables above
const uint8_t kTransTable[128][2] = {
    {2, 1}, {3, 0}, {4, 0}, {5, 1}, {6, 2}, {7, 3}, {8, 4}, {9, 5},
    {10, 4}, {11, 5}, {12, 8}, {13, 9}, {14, 8}, {15, 9}, {16, 10}, {17, 11},
    {18, 12}, {19, 13}, {20, 14}, {21, 15}, {22, 16}, {23, 17}, {24, 18}, {25, 19},
    {26, 18}, {27, 19}, {28, 22}, {29, 23}, {30, 22}, {31, 23}, {32, 24}, {33, 25},
    {34, 26}, {35, 27}, {36, 26}, {37, 27}, {38, 30}, {39, 31}, {40, 30}, {41, 31},
    {42, 32}, {43, 33}, {44, 32}, {45, 33}, {46, 36}, {47, 37}, {48, 36}, {49, 37},
    {50, 38}, {51, 39}, {52, 38}, {53, 39}, {54, 42}, {55, 43}, {56, 42}, {57, 43},
    {58, 44}, {59, 45}, {60, 44}, {61, 45}, {62, 46}, {63, 47}, {64, 48}, {65, 49},
    {66, 48}, {67, 49}, {68, 50}, {69, 51}, {70, 52}, {71, 53}, {72, 52}, {73, 53},
    {74, 54}, {75, 55}, {76, 54}, {77, 55}, {78, 56}, {79, 57}, {80, 58}, {81, 59},
    {82, 58}, {83, 59}, {84, 60}, {85, 61}, {86, 60}, {87, 61}, {88, 60}, {89, 61},
    {90, 62}, {91, 63}, {92, 64}, {93, 65}, {94, 64}, {95, 65}, {96, 66}, {97, 67},
    {98, 66}, {99, 67}, {100, 66}, {101, 67}, {102, 68}, {103, 69}, {104, 68}, {105, 69},
    {106, 70}, {107, 71}, {108, 70}, {109, 71}, {110, 70}, {111, 71}, {112, 72}, {113, 73},
    {114, 72}, {115, 73}, {116, 72}, {117, 73}, {118, 74}, {119, 75}, {120, 74}, {121, 75},
    {122, 74}, {123, 75}, {124, 76}, {125, 77}, {124, 76}, {125, 77}, {126, 126}, {127, 127},
};

// Flat context index layout (initType 0 only: I slices).
enum {
    C_SAO_MERGE = 0, C_SAO_TYPE = 1, C_SPLIT_CU = 2, C_TQ_BYPASS = 5, C_PART_MODE = 6, C_PREV_INTRA = 7,
    C_CHROMA_MODE = 8, C_SPLIT_TF = 9, C_CBF_LUMA = 12, C_CBF_CHROMA = 14, C_QP_DELTA = 19, C_TSKIP = 21,
    C_LAST_X = 23, C_LAST_Y = 41, C_CSBF = 59, C_SIG = 63, C_GT1 = 107, C_GT2 = 131, C_NUM = 137
};

// initValue per context (initType 0 columns of Tables 9-5..9-37; cabac.py:13-63)
static const uint8_t kInit[C_NUM] = {
    153,                                   // sao_merge_left/up_flag
    200,                                   // sao_type_idx_luma/chroma
    139, 141, 157,                         // split_cu_flag
    154,                                   // cu_transquant_bypass_flag
    184,                                   // part_mode
    184,                                   // prev_intra_luma_pred_flag
    63,                                    // intra_chroma_pred_mode
    153, 138, 138,                         // split_transform_flag
    111, 141,                              // cbf_luma
    94, 138, 182, 154, 154,                // cbf_cb / cbf_cr
    154, 154,                              // cu_qp_delta_abs
    139, 139,                              // transform_skip_flag (luma, chroma)
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,   // last_sig_coeff_x_prefix
    110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,   // last_sig_coeff_y_prefix
    91, 171, 134, 141,                     // coded_sub_block_flag
    111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107,              // sig_coeff_flag
    125, 141, 179, 153, 125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152,
    136, 152, 136, 153, 136, 139, 111, 136, 139, 111, 141, 111,
    140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152,                // coeff_abs_level_greater1_flag
    140, 179, 166, 182, 140, 227, 122, 197,
    138, 153, 136, 167, 152, 152,          // coeff_abs_level_greater2_flag
};

int context_init_values(const uint8_t** vals) {
    *vals = kInit;
    return C_NUM;
}

// ScanOrder[log2BlockSize][scanIdx][sPos] (6.5.3-6.5.5), positions packed as x | y << 4.
struct ScanTables {
    uint8_t pos[4][3][64];
    ScanTables() {
        for (int lg = 0; lg < 4; ++lg) {
            int n = 1 << lg;
            int i = 0, x = 0, y = 0;
            bool stop = false;
            while (!stop) {                           // up-right diagonal (6-10)
                while (y >= 0) {
                    if (x < n && y < n) pos[lg][0][i++] = (uint8_t)(x | (y << 4));
                    --y;
                    ++x;
                }
                y = x;
                x = 0;
                if (i >= n * n) stop = true;
            }
            i = 0;
            for (y = 0; y < n; ++y)
                for (x = 0; x < n; ++x) pos[lg][1][i++] = (uint8_t)(x | (y << 4));   // horizontal
            i = 0;
            for (x = 0; x < n; ++x)
                for (y = 0; y < n; ++y) pos[lg][2][i++] = (uint8_t)(x | (y << 4));   // vertical
            for (int sc = 0; sc < 3; ++sc)
                for (int k = 0; k < n * n; ++k) inv[lg][sc][pos[lg][sc][k]] = (uint8_t)k;
        }
    }
    uint8_t inv[4][3][128];                           // scan index of position x | y << 4
};
static const ScanTables kScan;

// sig_coeff_flag context index (9.3.4.2.5, absolute, incl. the component's base) of every
// position of a 4x4 sub-block, in the sub-block's scan order: [c != 0][log2 - 2][scanIdx]
// [prevCsbf][first sub-block of the TB][n]
struct SigCtxTables {
    uint8_t t[2][4][3][4][2][16];
    SigCtxTables() : t() {
        static const uint8_t ctx_idx_map[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
        static const uint8_t pattern[4][16] = {
            {2, 1, 1, 0, 1, 1, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0},     // prevCsbf 0: by xP + yP ([yP][xP] order)
            {2, 2, 2, 2, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0},     // 1: by yP
            {2, 1, 0, 0, 2, 1, 0, 0, 2, 1, 0, 0, 2, 1, 0, 0},     // 2: by xP
            {2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2}};
        for (int c = 0; c < 2; ++c)
            for (int lg = 2; lg <= 5; ++lg)
                for (int sc = 0; sc < 3; ++sc)
                    for (int prev = 0; prev < 4; ++prev)
                        for (int first = 0; first < 2; ++first)
                            for (int nn = 0; nn < 16; ++nn) {
                                const int pos = kScan.pos[2][sc][nn];
                                const int k = ((pos >> 4) << 2) + (pos & 15);
                                const int base = 63 + (c ? 27 : 0);          // C_SIG + chroma offset
                                int v;
                                if (lg == 2) {
                                    v = base + ctx_idx_map[k];
                                } else {
                                    const int add = c == 0 ? (first ? 0 : 3) + (lg == 3 ? (sc == 0 ? 9 : 15) : 21)
                                                           : (lg == 3 ? 9 : 12);
                                    v = base + add + pattern[prev][k];
                                    if (first && k == 0) v = base;            // DC of the TB: sigCtx 0
                                }
                                t[c][lg - 2][sc][prev][first][nn] = (uint8_t)v;
                            }
    }
};
static const SigCtxTables kSigCtx;

static inline int clip3(int lo, int hi, int v) { return v < lo ? lo : (v > hi ? hi : v); }

// QpC as a function of qPi for ChromaArrayType == 1 (Table 8-10; cu.py:575-591)
static inline int qpc_from_qpi(int qpi) {
    static const int t[13] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37};
    if (qpi < 30) return qpi;
    if (qpi >= 43) return qpi - 6;
    return t[qpi - 30];
}

namespace {

class PicDecoder {
public:
    PicDecoder(const Active& a, PictureRecords& out) : a_(a), sps_(a.sps), pps_(a.pps), out_(out) {
        W_ = a.w_ctb;
        log2ctb_ = sps_.log2_ctb;
        min_cb_w_ = sps_.width >> sps_.log2_min_cb;
        min_cb_h_ = sps_.height >> sps_.log2_min_cb;
        w4_ = (sps_.width + 3) >> 2;
        h4_ = (sps_.height + 3) >> 2;
        ctb_slice_.assign(a.size_ctb, -1);
        ct_depth_.assign((size_t)min_cb_w_ * min_cb_h_, 0);
        qp_map_.assign((size_t)min_cb_w_ * min_cb_h_, 0);
        ipm_.assign((size_t)w4_ * h4_, 1);
        // every sample is covered by at most one coded TB (or PCM block) per component: the dense
        // blocks are carved from one arena sized once (uninitialised; trimmed in finish()); the TB
        // array is reserved for its bound (one luma TB per 4 x 4 and a chroma pair per 8 x 8) and
        // filled in decode order, each CTU's TBs contiguous
        out_.coef.resize((size_t)sps_.width * sps_.height * 3 / 2 + 1024);
        out_.tbs.reserve((size_t)w4_ * h4_ * 3 / 2 + 64);
        coef_used_ = 0;
        out_.ctus.assign(a.size_ctb, p265r_ctu{});
        for (auto& c : out_.ctus) c.flags = P265R_CTU_LF_ACROSS_SLICES;
        qp_bd_y_ = 6 * (sps_.bit_depth_y - 8);
        qp_bd_c_ = 6 * (sps_.bit_depth_c - 8);
    }

    void decode_segment(const SliceRef& s) {
        const SliceHeader& h = *s.hdr;
        hdr_ = &h;
        rbsp_ = s.rbsp;
        rbsp_size_ = s.size;
        if (!h.dependent) slice_addr_ = h.segment_address;
        else if (slice_addr_ < 0) bs_fail("dependent slice segment starts the picture");
        slice_qp_ = h.slice_qp_y;
        int rs = h.segment_address;
        int ts = a_.rs_to_ts[rs];
        if (ctb_slice_[rs] != -1) bs_fail("slice segment address of an already decoded CTB");
        cabac_.start(rbsp_, rbsp_size_, h.data_byte_offset);
        bool first = true;
        for (;;) {
            if (ts >= a_.size_ctb) bs_fail("slice segment runs past the end of the picture");
            rs = a_.ts_to_rs[ts];
            if (ctb_slice_[rs] != -1) bs_fail("CTB decoded twice");
            int tile = a_.tile_id_ts[ts];
            int cx = rs % W_, cy = rs / W_;
            int tile_col0 = a_.col_bd[a_.ctb_col_tile[cx]];
            int tile_row0 = a_.row_bd[a_.ctb_row_tile[cy]];
            bool first_in_tile = (cx == tile_col0 && cy == tile_row0);
            bool wpp_row_start = pps_.entropy_coding_sync && cx == tile_col0;
            cur_tile_ = tile;
            ctb_slice_[rs] = slice_addr_;
            // context initialization at this CTU (9.3.1, 9.3.2.2)
            if (first || first_in_tile || wpp_row_start) {
                if (first_in_tile) {
                    init_contexts();
                } else if (wpp_row_start) {
                    int trx = cx + 1, try_ = cy - 1;
                    bool avail = trx < W_ && try_ >= 0 && ctb_avail(try_ * W_ + trx);
                    if (avail && wpp_valid_) std::memcpy(ctx_, wpp_ctx_, sizeof(ctx_));
                    else init_contexts();
                } else if (h.dependent && rs == h.segment_address) {
                    if (!ds_valid_) bs_fail("dependent slice segment without stored contexts");
                    std::memcpy(ctx_, ds_ctx_, sizeof(ctx_));
                } else {
                    init_contexts();
                }
                // first quantization group in a slice / tile / CTB row of a tile with WPP (8.6.1)
                if ((first && !h.dependent) || first_in_tile || wpp_row_start) first_qg_ = true;
            }
            first = false;
            decode_ctu(rs, ts);
            if (pps_.entropy_coding_sync && cx == tile_col0 + 1) {   // storage after the 2nd CTB of a tile row
                std::memcpy(wpp_ctx_, ctx_, sizeof(ctx_));
                wpp_valid_ = true;
            }
            int end_of_slice_segment = cabac_.terminate();
            if (cabac_.overrun()) bs_fail("slice data truncated");
            ++ts;
            if (end_of_slice_segment) break;
            if (ts >= a_.size_ctb) bs_fail("end_of_slice_segment_flag missing at the end of the picture");
            int nrs = a_.ts_to_rs[ts];
            int ncx = nrs % W_, ncy = nrs / W_;
            bool new_tile = pps_.tiles && a_.tile_id_ts[ts] != a_.tile_id_ts[ts - 1];
            bool new_row = pps_.entropy_coding_sync && ncx == a_.col_bd[a_.ctb_col_tile[ncx]];
            (void)ncy;
            if (new_tile || new_row) {
                if (!cabac_.terminate()) bs_fail("end_of_subset_one_bit != 1");
                cabac_.start(rbsp_, rbsp_size_, cabac_.aligned_byte_after_terminate());
                first = true;   // re-evaluate context initialization at the next CTU
            }
        }
        if (pps_.dependent_slice_segments) {
            std::memcpy(ds_ctx_, ctx_, sizeof(ctx_));
            ds_valid_ = true;
        }
    }

    // n zeroed coefficients at the end of the picture's arena
    int16_t* coef_alloc(size_t n, uint32_t& off) {
        off = (uint32_t)coef_used_;
        if (coef_used_ + n > out_.coef.size()) out_.coef.resize(std::max(out_.coef.size() * 2, coef_used_ + n));
        coef_used_ += n;
        int16_t* p = out_.coef.data() + off;
        std::memset(p, 0, n * sizeof(int16_t));
        return p;
    }

    void finish() {
        out_.coef.resize(coef_used_);
        for (int rs = 0; rs < a_.size_ctb; ++rs)
            if (ctb_slice_[rs] < 0) bs_fail("picture incomplete: CTB not covered by any slice segment");
        // TBs were emitted in decode (tile-scan) order; the records list them by raster CTU
        bool raster = true;
        size_t next = 0;
        for (int rs = 0; rs < a_.size_ctb && raster; ++rs) {
            raster = out_.ctus[rs].tb_begin == next;
            next += out_.ctus[rs].tb_count;
        }
        if (!raster) {
            std::vector<p265r_tb, PoolAlloc<p265r_tb>> v;
            v.reserve(out_.tbs.size());
            for (int rs = 0; rs < a_.size_ctb; ++rs) {
                p265r_ctu& c = out_.ctus[rs];
                const size_t b = c.tb_begin;
                c.tb_begin = (uint32_t)v.size();
                v.insert(v.end(), out_.tbs.begin() + b, out_.tbs.begin() + b + c.tb_count);
            }
            out_.tbs.swap(v);
        }
    }

private:
    // ---------------------------------------------------------------- helpers
    void init_contexts() {   // 9.3.2.2 (cabac.py:163-186)
        int qp = clip3(0, 51, slice_qp_);
        for (int i = 0; i < C_NUM; ++i) {
            int v = kInit[i];
            int m = (v >> 4) * 5 - 45, n = ((v & 15) << 3) - 16;
            int pre = clip3(1, 126, ((m * qp) >> 4) + n);
            int mps = pre <= 63 ? 0 : 1;
            int st = mps ? pre - 64 : 63 - pre;
            ctx_[i] = (uint16_t)((st << 1) | mps);
        }
    }
    // CTB of a neighbouring location is available: decoded, same slice, same tile (6.4.1)
    inline bool ctb_avail(int rs) const {
        return ctb_slice_[rs] == slice_addr_ && a_.tile_id_rs(rs) == cur_tile_;
    }
    inline bool loc_avail(int x, int y) const {
        if (x < 0 || y < 0 || x >= sps_.width || y >= sps_.height) return false;
        return ctb_avail((y >> log2ctb_) * W_ + (x >> log2ctb_));
    }
    inline int dec(int c) { return cabac_.decision(ctx_[c]); }

    // ---------------------------------------------------------------- CTU / SAO
    void decode_ctu(int rs, int ts) {
        p265r_ctu& c = out_.ctus[rs];
        const SliceHeader& h = *hdr_;
        c.slice_addr = (uint32_t)slice_addr_;
        c.tile_id = (uint16_t)a_.tile_id_ts[ts];
        c.flags = (uint8_t)((h.loop_filter_across_slices ? P265R_CTU_LF_ACROSS_SLICES : 0) |
                            (h.deblocking_disabled ? 0 : P265R_CTU_DEBLOCK));
        c.deblock_offsets = h.deblocking_disabled ? 0 : P265R_DEBLOCK_OFFSETS(h.beta_offset_div2, h.tc_offset_div2);
        cur_ctu_ = rs;
        int cx = rs % W_, cy = rs / W_;
        if (h.sao_luma || h.sao_chroma) parse_sao(rs, ts, cx, cy, c);
        const size_t tb0 = out_.tbs.size();
        coding_quadtree(cx << log2ctb_, cy << log2ctb_, log2ctb_, 0);
        const size_t ntb = out_.tbs.size() - tb0;
        if (ntb > 0xFFFF) bs_fail("too many TBs in a CTU");
        c.tb_begin = (uint32_t)tb0;
        c.tb_count = (uint16_t)ntb;
    }

    // sao(rx, ry) (7.3.8.3; sao.py:15-136), SaoOffsetVal with EO signs inferred (7.4.9.3.2)
    void parse_sao(int rs, int ts, int rx, int ry, p265r_ctu& c) {
        const SliceHeader& h = *hdr_;
        int merge_left = 0, merge_up = 0;
        if (rx > 0) {
            bool in_slice = rs > slice_addr_;
            bool in_tile = a_.tile_id_ts[ts] == a_.tile_id_rs(rs - 1);
            if (in_slice && in_tile) merge_left = dec(C_SAO_MERGE);
        }
        if (ry > 0 && !merge_left) {
            bool in_slice = (rs - W_) >= slice_addr_;
            bool in_tile = a_.tile_id_ts[ts] == a_.tile_id_rs(rs - W_);
            if (in_slice && in_tile) merge_up = dec(C_SAO_MERGE);
        }
        if (merge_left || merge_up) {
            const p265r_ctu& src = out_.ctus[merge_left ? rs - 1 : rs - W_];
            std::memcpy(c.sao_type, src.sao_type, 3);
            std::memcpy(c.sao_class, src.sao_class, 3);
            std::memcpy(c.sao_offset, src.sao_offset, sizeof(c.sao_offset));
            return;
        }
        for (int ci = 0; ci < 3; ++ci) {
            c.sao_type[ci] = 0;
            c.sao_class[ci] = 0;
            std::memset(c.sao_offset[ci], 0, 4);
            if (!((h.sao_luma && ci == 0) || (h.sao_chroma && ci > 0))) continue;
            int type;
            if (ci == 2) {
                type = c.sao_type[1];
            } else {                                // TR cMax = 2: ctx bin, bypass bin (sao.py:148-160)
                type = dec(C_SAO_TYPE) ? (cabac_.bypass() ? 2 : 1) : 0;
            }
            c.sao_type[ci] = (uint8_t)type;
            if (!type) continue;
            int bd = ci ? sps_.bit_depth_c : sps_.bit_depth_y;
            int cmax = (1 << (std::min(bd, 10) - 5)) - 1, absv[4];   // TR cMax of sao_offset_abs
            for (int i = 0; i < 4; ++i) {           // TR bypass (sao.py:172-191)
                int v = 0;
                while (v < cmax && cabac_.bypass()) ++v;
                absv[i] = v;
            }
            int shift = bd - std::min(bd, 10);
            if (type == 1) {
                for (int i = 0; i < 4; ++i) {
                    int sgn = (absv[i] != 0) ? cabac_.bypass() : 0;
                    c.sao_offset[ci][i] = (int8_t)((sgn ? -absv[i] : absv[i]) * (1 << shift));
                }
                c.sao_class[ci] = (uint8_t)cabac_.bypass_bits(5);   // sao_band_position
            } else {
                for (int i = 0; i < 4; ++i) c.sao_offset[ci][i] = (int8_t)((i >= 2 ? -absv[i] : absv[i]) * (1 << shift));
                if (ci == 0) c.sao_class[0] = (uint8_t)cabac_.bypass_bits(2);
                else if (ci == 1) c.sao_class[1] = (uint8_t)cabac_.bypass_bits(2);
                else c.sao_class[2] = c.sao_class[1];
            }
        }
    }

    // ---------------------------------------------------------------- coding quadtree / CU
    // coding_quadtree (7.3.8.4; cu.py:41-98, split flag context cu.py:367-395)
    void coding_quadtree(int x0, int y0, int log2, int depth) {
        int size = 1 << log2;
        int split;
        if (x0 + size <= sps_.width && y0 + size <= sps_.height && log2 > sps_.log2_min_cb) {
            int inc = 0;
            if (loc_avail(x0 - 1, y0) && ct_depth_at(x0 - 1, y0) > depth) ++inc;
            if (loc_avail(x0, y0 - 1) && ct_depth_at(x0, y0 - 1) > depth) ++inc;
            split = dec(C_SPLIT_CU + inc);
        } else {
            split = log2 > sps_.log2_min_cb;
        }
        if (split) {
            int h = size >> 1;
            coding_quadtree(x0, y0, log2 - 1, depth + 1);
            if (x0 + h < sps_.width) coding_quadtree(x0 + h, y0, log2 - 1, depth + 1);
            if (y0 + h < sps_.height) coding_quadtree(x0, y0 + h, log2 - 1, depth + 1);
            if (x0 + h < sps_.width && y0 + h < sps_.height) coding_quadtree(x0 + h, y0 + h, log2 - 1, depth + 1);
        } else {
            coding_unit(x0, y0, log2, depth);
        }
    }

    inline int ct_depth_at(int x, int y) const {
        return ct_depth_[(size_t)(y >> sps_.log2_min_cb) * min_cb_w_ + (x >> sps_.log2_min_cb)];
    }
    inline int qp_at(int x, int y) const {
        return qp_map_[(size_t)(y >> sps_.log2_min_cb) * min_cb_w_ + (x >> sps_.log2_min_cb)];
    }

    // candModeList derivation (8.4.2) for the PB at (xPb, yPb); cu.py:175-263
    int derive_luma_mode(int xPb, int yPb, int prev_flag, int mpm_idx, int rem) {
        int a = 1, b = 1;   // INTRA_DC when unavailable / PCM (ipm_ stores DC for PCM CUs)
        if (loc_avail(xPb - 1, yPb)) a = ipm_[(size_t)(yPb >> 2) * w4_ + ((xPb - 1) >> 2)];
        if (yPb - 1 >= ((yPb >> log2ctb_) << log2ctb_) && loc_avail(xPb, yPb - 1))
            b = ipm_[(size_t)((yPb - 1) >> 2) * w4_ + (xPb >> 2)];
        int cand[3];
        if (a == b) {
            if (a < 2) { cand[0] = 0; cand[1] = 1; cand[2] = 26; }
            else { cand[0] = a; cand[1] = 2 + ((a + 29) % 32); cand[2] = 2 + ((a - 2 + 1) % 32); }
        } else {
            cand[0] = a; cand[1] = b;
            if (a != 0 && b != 0) cand[2] = 0;
            else if (a != 1 && b != 1) cand[2] = 1;
            else cand[2] = 26;
        }
        if (prev_flag) return cand[mpm_idx];
        if (cand[0] > cand[1]) std::swap(cand[0], cand[1]);
        if (cand[0] > cand[2]) std::swap(cand[0], cand[2]);
        if (cand[1] > cand[2]) std::swap(cand[1], cand[2]);
        int m = rem;
        for (int i = 0; i < 3; ++i)
            if (m >= cand[i]) ++m;
        return m;
    }

    void set_ipm(int x0, int y0, int size, int mode) {
        int n4 = size >> 2;
        for (int j = 0; j < n4; ++j) {
            int yy = (y0 >> 2) + j;
            if (yy >= h4_) break;
            for (int i = 0; i < n4; ++i) {
                int xx = (x0 >> 2) + i;
                if (xx < w4_) ipm_[(size_t)yy * w4_ + xx] = (uint8_t)mode;
            }
        }
    }

    void fill_cb_map(std::vector<int8_t>& m, int x0, int y0, int log2, int v) {
        int n = 1 << (log2 - sps_.log2_min_cb);
        for (int j = 0; j < n; ++j) {
            int yy = (y0 >> sps_.log2_min_cb) + j;
            if (yy >= min_cb_h_) break;
            for (int i = 0; i < n; ++i) {
                int xx = (x0 >> sps_.log2_min_cb) + i;
                if (xx < min_cb_w_) m[(size_t)yy * min_cb_w_ + xx] = (int8_t)v;
            }
        }
    }
    void fill_depth(int x0, int y0, int log2, int depth) {
        int n = 1 << (log2 - sps_.log2_min_cb);
        for (int j = 0; j < n; ++j) {
            int yy = (y0 >> sps_.log2_min_cb) + j;
            if (yy >= min_cb_h_) break;
            for (int i = 0; i < n; ++i) {
                int xx = (x0 >> sps_.log2_min_cb) + i;
                if (xx < min_cb_w_) ct_depth_[(size_t)yy * min_cb_w_ + xx] = (uint8_t)depth;
            }
        }
    }

    void mark_nofilter(int x0, int y0, int log2) {
        int nw = (sps_.width + 7) >> 3, nh = (sps_.height + 7) >> 3;
        if (out_.nofilter.empty()) out_.nofilter.assign((size_t)nw * nh, 0);
        int n8 = std::max(1, (1 << log2) >> 3);
        for (int j = 0; j < n8; ++j)
            for (int i = 0; i < n8; ++i) {
                int bx = (x0 >> 3) + i, by = (y0 >> 3) + j;
                if (bx < nw && by < nh) out_.nofilter[(size_t)by * nw + bx] = 1;
            }
    }

    // coding_unit (7.3.8.5) for I slices; cu.py:99-174, 310-365, 397-471
    void coding_unit(int x0, int y0, int log2, int depth) {
        ++out_.n_cus;
        int size = 1 << log2;
        int mask = (1 << a_.log2_min_cu_qp_delta) - 1;
        if ((x0 & mask) == 0 && (y0 & mask) == 0) {
            // start of a quantization group: qPY_PREV, qPY_A, qPY_B -> qPY_PRED (8.6.1)
            if (pps_.cu_qp_delta) { is_cu_qp_delta_coded_ = 0; cu_qp_delta_val_ = 0; }
            int prev = first_qg_ ? slice_qp_ : last_qp_y_;
            first_qg_ = false;
            int ctb_mask = (1 << log2ctb_) - 1;
            int qa = (x0 & ctb_mask) ? qp_at(x0 - 1, y0) : prev;
            int qb = (y0 & ctb_mask) ? qp_at(x0, y0 - 1) : prev;
            qg_pred_ = (qa + qb + 1) >> 1;
        }
        fill_depth(x0, y0, log2, depth);
        cu_bypass_ = 0;
        if (pps_.transquant_bypass) cu_bypass_ = dec(C_TQ_BYPASS);
        int part_nxn = 0;
        if (log2 == sps_.log2_min_cb) {
            part_nxn = !dec(C_PART_MODE);
        }
        int pcm = 0;
        if (!part_nxn && sps_.pcm && log2 >= sps_.log2_min_pcm && log2 <= sps_.log2_max_pcm) pcm = cabac_.terminate();
        cu_tbs_.clear();
        int mode_c = 0;
        if (pcm) {
            set_ipm(x0, y0, size, 1);
            pcm_sample(x0, y0, log2);
        } else {
            int nparts = part_nxn ? 4 : 1;
            int pb = part_nxn ? size >> 1 : size;
            int prev[4], mpm[4] = {0, 0, 0, 0}, rem[4] = {0, 0, 0, 0};
            for (int i = 0; i < nparts; ++i) prev[i] = dec(C_PREV_INTRA);
            for (int i = 0; i < nparts; ++i) {
                if (prev[i]) {                    // mpm_idx: TR cMax 2, bypass
                    mpm[i] = cabac_.bypass() ? (cabac_.bypass() ? 2 : 1) : 0;
                } else {
                    rem[i] = (int)cabac_.bypass_bits(5);
                }
                int xp = x0 + pb * (i & 1), yp = y0 + pb * (i >> 1);
                modes_y_[i] = derive_luma_mode(xp, yp, prev[i], mpm[i], rem[i]);
                set_ipm(xp, yp, pb, modes_y_[i]);
            }
            // intra_chroma_pred_mode (9.3.3.8 binarization; 8.4.3 derivation, Table 8-2/8-3)
            int icpm = 4;
            if (dec(C_CHROMA_MODE)) icpm = (int)cabac_.bypass_bits(2);
            if (icpm == 4) {
                mode_c = modes_y_[0];
            } else {
                static const int tab[4] = {0, 26, 10, 1};
                mode_c = tab[icpm];
                if (mode_c == modes_y_[0]) mode_c = 34;
            }
            mode_c_ = mode_c;
            part_nxn_ = part_nxn;
            cu_x_ = x0; cu_y_ = y0; cu_log2_ = log2;
            max_trafo_depth_ = sps_.max_th_depth_intra + part_nxn;
            transform_tree(x0, y0, x0, y0, log2, 0, 0, 1, 1);
        }
        // QpY of the CU (8-283) and chroma QPs (8-285..8-287)
        int qpy = ((qg_pred_ + cu_qp_delta_val_ + 52 + 2 * qp_bd_y_) % (52 + qp_bd_y_)) - qp_bd_y_;
        last_qp_y_ = qpy;
        fill_cb_map(qp_map_, x0, y0, log2, qpy);
        int qcb = qpc_from_qpi(clip3(-qp_bd_c_, 57, qpy + pps_.cb_qp_offset + hdr_->cb_qp_offset)) + qp_bd_c_;
        int qcr = qpc_from_qpi(clip3(-qp_bd_c_, 57, qpy + pps_.cr_qp_offset + hdr_->cr_qp_offset)) + qp_bd_c_;
        uint8_t qps[3] = {(uint8_t)(qpy + qp_bd_y_), (uint8_t)qcb, (uint8_t)qcr};
        for (auto& t : cu_tbs_) {
            t.qp = qps[t.c_idx];
            out_.tbs.push_back(t);
        }
        if (cu_bypass_ || (pcm && sps_.pcm_loop_filter_disabled)) mark_nofilter(x0, y0, log2);
    }

    // pcm_sample() (7.3.8.7) after pcm_flag; the engine restarts after the samples (9.3.2.5)
    void pcm_sample(int x0, int y0, int log2) {
        size_t byte = cabac_.aligned_byte_after_terminate();   // pcm_alignment_zero_bit(s) skipped
        BitReader br(rbsp_, rbsp_size_, byte * 8);
        for (int c = 0; c < 3; ++c) {
            int lg = c ? log2 - 1 : log2;
            int n = 1 << lg;
            int pbd = c ? sps_.pcm_bit_depth_c : sps_.pcm_bit_depth_y;
            int bd = c ? sps_.bit_depth_c : sps_.bit_depth_y;
            uint32_t off;
            int16_t* dst = coef_alloc((size_t)n * n, off);
            for (int k = 0; k < n * n; ++k) dst[k] = (int16_t)(br.u(pbd) << (bd - pbd));
            p265r_tb t{};
            t.x = (uint16_t)(c ? x0 >> 1 : x0);
            t.y = (uint16_t)(c ? y0 >> 1 : y0);
            t.log2_size = (uint8_t)lg;
            t.c_idx = (uint8_t)c;
            t.pred_mode = 0;
            t.flags = P265R_TB_PCM;
            t.coef_off = off;
            cu_tbs_.push_back(t);
        }
        if (!br.byte_aligned()) bs_fail("PCM samples not byte aligned");
        cabac_.start(rbsp_, rbsp_size_, br.pos() >> 3);
    }

    // ---------------------------------------------------------------- transform tree
    // transform_tree (7.3.8.8; tu.py:11-83, split flag / cbf contexts tu.py:342-394)
    void transform_tree(int x0, int y0, int xb, int yb, int log2, int depth, int blk, int parent_cb, int parent_cr) {
        int split;
        if (log2 <= sps_.log2_max_tb && log2 > sps_.log2_min_tb && depth < max_trafo_depth_ && !(part_nxn_ && depth == 0))
            split = dec(C_SPLIT_TF + 5 - log2);
        else
            split = (log2 > sps_.log2_max_tb || (part_nxn_ && depth == 0)) ? 1 : 0;
        int cbf_cb = 0, cbf_cr = 0;
        if (log2 > 2) {
            if (depth == 0 || parent_cb) cbf_cb = dec(C_CBF_CHROMA + depth);
            if (depth == 0 || parent_cr) cbf_cr = dec(C_CBF_CHROMA + depth);
        }
        if (split) {
            int h = 1 << (log2 - 1);
            transform_tree(x0, y0, x0, y0, log2 - 1, depth + 1, 0, cbf_cb, cbf_cr);
            transform_tree(x0 + h, y0, x0, y0, log2 - 1, depth + 1, 1, cbf_cb, cbf_cr);
            transform_tree(x0, y0 + h, x0, y0, log2 - 1, depth + 1, 2, cbf_cb, cbf_cr);
            transform_tree(x0 + h, y0 + h, x0, y0, log2 - 1, depth + 1, 3, cbf_cb, cbf_cr);
            return;
        }
        int cbf_luma = dec(C_CBF_LUMA + (depth == 0 ? 1 : 0));
        // transform_unit (7.3.8.10); for a 4x4 luma TB the chroma cbfs are the parent's
        int ccb = log2 > 2 ? cbf_cb : parent_cb;
        int ccr = log2 > 2 ? cbf_cr : parent_cr;
        if (cbf_luma || ccb || ccr) {
            if (pps_.cu_qp_delta && !is_cu_qp_delta_coded_) {
                int v = 0;                                   // prefix TR cMax 5, suffix EG0 (9.3.3.10)
                while (v < 5 && dec(C_QP_DELTA + (v == 0 ? 0 : 1))) ++v;
                if (v == 5) {
                    int k = 0;
                    while (cabac_.bypass()) {
                        v += 1 << k;
                        if (++k > 30) bs_fail("cu_qp_delta_abs suffix too long");
                    }
                    v += (int)cabac_.bypass_bits(k);
                }
                if (v && cabac_.bypass()) v = -v;
                is_cu_qp_delta_coded_ = 1;
                cu_qp_delta_val_ = v;
                int lim = 26 + qp_bd_y_ / 2;
                if (v < -lim || v > lim - 1) bs_fail("CuQpDeltaVal out of range");
            }
        }
        int mode_y = modes_y_[part_nxn_ ? (((y0 - cu_y_) >= (1 << (cu_log2_ - 1))) * 2 + ((x0 - cu_x_) >= (1 << (cu_log2_ - 1)))) : 0];
        emit_tb(x0, y0, log2, 0, mode_y, cbf_luma);
        if (log2 > 2) {
            emit_tb(x0 >> 1, y0 >> 1, log2 - 1, 1, mode_c_, cbf_cb);
            emit_tb(x0 >> 1, y0 >> 1, log2 - 1, 2, mode_c_, cbf_cr);
        } else if (blk == 3) {
            emit_tb(xb >> 1, yb >> 1, 2, 1, mode_c_, parent_cb);
            emit_tb(xb >> 1, yb >> 1, 2, 2, mode_c_, parent_cr);
        }
    }

    void emit_tb(int x, int y, int log2, int c, int mode, int cbf) {
        p265r_tb t{};
        t.x = (uint16_t)x;
        t.y = (uint16_t)y;
        t.log2_size = (uint8_t)log2;
        t.c_idx = (uint8_t)c;
        t.pred_mode = (uint8_t)mode;
        t.flags = (uint8_t)(cu_bypass_ ? P265R_TB_BYPASS : 0);
        if (cbf) {
            t.flags |= P265R_TB_CBF;
            int tskip = 0;
            t.coef_off = residual_coding(log2, c, mode, &tskip);
            if (tskip) t.flags |= P265R_TB_TSKIP;
        }
        cu_tbs_.push_back(t);
    }

    // ---------------------------------------------------------------- residual coding
    // residual_coding (7.3.8.11) with the context selection of 9.3.4.2.3-9.3.4.2.7
    // (tu.py:137-340, 396-665).  Returns the coefficient offset of the dense N x N block.
    uint32_t residual_coding(int log2, int c, int pred_mode, int* tskip_out) {
        int n = 1 << log2;
        uint32_t off;
        int16_t* blk = coef_alloc((size_t)n * n, off);
        // the engine lives in registers for the whole TB (copied back at the end)
        Cabac e = cabac_;
        uint16_t* const cx = ctx_;
        int tskip = 0;
        if (pps_.transform_skip && !cu_bypass_ && log2 <= 2) tskip = e.decision(cx[C_TSKIP + (c ? 1 : 0)]);
        *tskip_out = tskip;
        // last_sig_coeff_x/y_prefix (TR, cMax (log2 << 1) - 1), suffix (FL bypass)
        int off_ctx, shift;
        if (c == 0) { off_ctx = 3 * (log2 - 2) + ((log2 - 1) >> 2); shift = (log2 + 1) >> 2; }
        else { off_ctx = 15; shift = log2 - 2; }
        int cmax = (log2 << 1) - 1;
        int px = 0, py = 0;
        while (px < cmax && e.decision(cx[C_LAST_X + off_ctx + (px >> shift)])) ++px;
        while (py < cmax && e.decision(cx[C_LAST_Y + off_ctx + (py >> shift)])) ++py;
        int last_x = px, last_y = py;
        if (px > 3) {
            int nb = (px >> 1) - 1;
            last_x = (1 << nb) * (2 + (px & 1)) + (int)e.bypass_bits(nb);
        }
        if (py > 3) {
            int nb = (py >> 1) - 1;
            last_y = (1 << nb) * (2 + (py & 1)) + (int)e.bypass_bits(nb);
        }
        // scanIdx (7.4.9.11): mode dependent for 4x4, and 8x8 luma
        int scan = 0;
        if (log2 == 2 || (log2 == 3 && c == 0)) {
            if (pred_mode >= 6 && pred_mode <= 14) scan = 2;
            else if (pred_mode >= 22 && pred_mode <= 30) scan = 1;
        }
        if (scan == 2) std::swap(last_x, last_y);
        if (last_x >= n || last_y >= n) bs_fail("last significant coefficient outside the TB");
        const int lsb = log2 - 2;                 // log2 of the sub-block grid size
        const uint8_t* sb_scan = kScan.pos[lsb][scan];
        const uint8_t* c_scan = kScan.pos[2][scan];
        int sbw = 1 << lsb;
        // sub-block and in-sub-block scan positions of the last coefficient
        const int last_sb = kScan.inv[lsb][scan][(last_x >> 2) | ((last_y >> 2) << 4)];
        const int last_pos = kScan.inv[2][scan][(last_x & 3) | ((last_y & 3) << 4)];
        uint8_t csbf[8][8];
        std::memset(csbf, 0, sizeof(csbf));
        const bool sdh = pps_.sign_data_hiding && !cu_bypass_;
        int greater1_state = 1;   // "c1" carried across sub-blocks (9.3.4.2.6)
        bool first_sb_done = false;
        // sig_coeff_flag contexts per position of a sub-block (9.3.4.2.5), tabulated (kSigCtx)
        const int cc = c ? 1 : 0;
        for (int i = last_sb; i >= 0; --i) {
            int xs = sb_scan[i] & 15, ys = sb_scan[i] >> 4;
            int infer_dc = 0;
            if (i < last_sb && i > 0) {
                int right = (xs + 1 < sbw) ? csbf[xs + 1][ys] : 0;
                int below = (ys + 1 < sbw) ? csbf[xs][ys + 1] : 0;
                int inc = std::min(right + below, 1) + (c ? 2 : 0);
                csbf[xs][ys] = (uint8_t)e.decision(cx[C_CSBF + inc]);
                infer_dc = 1;
            } else {
                csbf[xs][ys] = 1;
            }
            // significant coefficients of the sub-block, in decoding (reverse scan) order
            int sig_pos[16], nsig = 0;
            int start = 15;
            if (i == last_sb) {
                start = last_pos - 1;
                sig_pos[nsig++] = last_pos;
            }
            if (csbf[xs][ys]) {
                int prev = 0;
                if (xs + 1 < sbw) prev |= csbf[xs + 1][ys];
                if (ys + 1 < sbw) prev |= csbf[xs][ys + 1] << 1;
                const uint8_t* sctx = kSigCtx.t[cc][log2 - 2][scan][prev][(xs | ys) == 0 ? 1 : 0];
                // branch-free on the decoded bins (an LPS-rate branch mispredicts on every few bins)
                for (int nn = start; nn > 0; --nn) {
                    const int b = e.decision(cx[sctx[nn]]);
                    sig_pos[nsig] = nn;
                    nsig += b;
                    infer_dc &= b ^ 1;
                }
                if (start >= 0) {
                    // DC: decoded, or inferred significant when no other coefficient of the coded sub-block is
                    const int b = infer_dc ? 1 : e.decision(cx[sctx[0]]);
                    sig_pos[nsig] = 0;
                    nsig += b;
                }
            }
            if (nsig == 0) continue;
            // coeff_abs_level_greater1_flag (<= 8) / greater2_flag (1)
            int ctx_set = (i == 0 || c > 0) ? 0 : 2;
            if (first_sb_done && greater1_state == 0) ++ctx_set;
            first_sb_done = true;
            greater1_state = 1;
            int g1[16] = {}, g2[16] = {};
            int first_g1_idx = -1;
            int ng1 = std::min(nsig, 8);
            const int g1_base = C_GT1 + ctx_set * 4 + (c ? 16 : 0);
            for (int k = 0; k < ng1; ++k) {
                const int b = e.decision(cx[g1_base + greater1_state]);
                g1[k] = b;
                // (9.3.4.2.6) greater1Ctx: 0 after a 1, else 1 -> 2 -> 3 (saturating); branch-free
                const int inc = (greater1_state > 0) & (greater1_state < 3);
                greater1_state = b ? 0 : greater1_state + inc;
                first_g1_idx = (first_g1_idx < 0 && b) ? k : first_g1_idx;
            }
            if (first_g1_idx >= 0) g2[first_g1_idx] = e.decision(cx[C_GT2 + ctx_set + (c ? 4 : 0)]);
            bool hidden = sdh && (sig_pos[0] - sig_pos[nsig - 1] > 3);
            // coeff_sign_flag (bypass), last one skipped when hidden
            int nsign = hidden ? nsig - 1 : nsig;
            uint32_t signs = nsign ? e.bypass_bits(nsign) << (32 - nsign) : 0;   // first sign in the MSB
            // coeff_abs_level_remaining + levels
            int rice = 0, sum_abs = 0;
            for (int k = 0; k < nsig; ++k) {
                int base = 1 + g1[k] + g2[k];
                int level = base;
                int thr = (k < 8) ? ((k == first_g1_idx) ? 3 : 2) : 1;
                if (base == thr) {
                    int prefix = 0;
                    while (e.bypass()) {
                        if (++prefix > 32) bs_fail("coeff_abs_level_remaining prefix too long");
                    }
                    int rem;
                    if (prefix <= 3) {
                        rem = (prefix << rice) + (int)e.bypass_bits(rice);
                    } else {
                        int nb = prefix - 3 + rice;
                        if (nb > 28) bs_fail("coeff_abs_level_remaining too large");
                        rem = (((1 << (prefix - 3)) + 2) << rice) + (int)e.bypass_bits(nb);
                    }
                    level = base + rem;
                    if (level > 3 * (1 << rice)) rice = std::min(rice + 1, 4);
                }
                int v = level;
                if (k < nsign && ((signs << k) & 0x80000000u)) v = -v;
                if (hidden) {
                    sum_abs += level;
                    if (k == nsig - 1 && (sum_abs & 1)) v = -v;
                }
                int pos = c_scan[sig_pos[k]];
                int x = (xs << 2) + (pos & 15), y = (ys << 2) + (pos >> 4);
                blk[y * n + x] = (int16_t)clip3(-32768, 32767, v);
            }
        }
        cabac_ = e;
        return off;
    }

    // ---------------------------------------------------------------- state
    const Active& a_;
    const Sps& sps_;
    const Pps& pps_;
    PictureRecords& out_;
    int W_ = 0, log2ctb_ = 0, min_cb_w_ = 0, min_cb_h_ = 0, w4_ = 0, h4_ = 0;
    int qp_bd_y_ = 0, qp_bd_c_ = 0;
    std::vector<int> ctb_slice_;
    std::vector<uint8_t> ct_depth_;
    std::vector<int8_t> qp_map_;
    std::vector<uint8_t> ipm_;
    std::vector<p265r_tb> cu_tbs_;
    size_t coef_used_ = 0;
    const SliceHeader* hdr_ = nullptr;
    const uint8_t* rbsp_ = nullptr;
    size_t rbsp_size_ = 0;
    Cabac cabac_;
    uint16_t ctx_[C_NUM], wpp_ctx_[C_NUM], ds_ctx_[C_NUM];
    bool wpp_valid_ = false, ds_valid_ = false;
    int slice_addr_ = -1, slice_qp_ = 26, cur_tile_ = 0, cur_ctu_ = 0;
    // quantization group state (8.6.1)
    bool first_qg_ = true;
    int last_qp_y_ = 26, qg_pred_ = 26, is_cu_qp_delta_coded_ = 0, cu_qp_delta_val_ = 0;
    // current CU
    int cu_bypass_ = 0, part_nxn_ = 0, mode_c_ = 0, max_trafo_depth_ = 0, cu_x_ = 0, cu_y_ = 0, cu_log2_ = 3;
    int modes_y_[4] = {1, 1, 1, 1};
};

}  // namespace

void decode_picture(const Active& act, const std::vector<SliceRef>& slices, PictureRecords& out) {
    if (act.sps.chroma_format_idc != 1) throw Unsupported("chroma_format_idc != 1 (4:2:0 only)");
    if (act.sps.range_extension_flags || act.pps.range_extension_flags)
        throw Unsupported("range extension coding tools");
    out = PictureRecords{};
    PicDecoder d(act, out);
    for (const auto& s : slices) d.decode_segment(s);
    d.finish();
}

}  // namespace p265fe
