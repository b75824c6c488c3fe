// Parameter sets and slice segment headers (H.265 7.3.2.1-7.3.2.3, 7.3.3, 7.3.4, 7.3.6,
// 7.3.7, E.2.1).  See fe_ps.h for the reference counterparts.
#include "fe_ps.h"

#include <cstring>

#include <algorithm>

namespace p265fe {

static int ceil_log2(int v) {
    int r = 0;
    while ((1 << r) < v) ++r;
    return r;
}

// profile_tier_level(1, maxNumSubLayersMinus1) (7.3.3; ptl.py:5)
static void parse_ptl(BitReader& br, int max_sub_layers_minus1) {
    br.skip(8 + 32 + 4 + 43 + 1);   // general profile space/tier/idc, compat flags, 4 source flags, 43+1 bits
    br.skip(8);                     // general_level_idc
    int prof[8] = {}, lvl[8] = {};
    for (int i = 0; i < max_sub_layers_minus1; ++i) {
        prof[i] = br.flag();
        lvl[i] = br.flag();
    }
    if (max_sub_layers_minus1 > 0)
        for (int i = max_sub_layers_minus1; i < 8; ++i) br.skip(2);
    for (int i = 0; i < max_sub_layers_minus1; ++i) {
        if (prof[i]) br.skip(88);
        if (lvl[i]) br.skip(8);
    }
}

// Table 7-6: default ScalingList of the 8x8 and larger matrices, intra (matrixId 0..2) and inter (3..5),
// in coefficient order i (Table 7-5: the 4x4 default is flat 16); the reference's sld.py:13-33 tables
static const uint8_t kSlIntra[64] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 16, 17, 16, 17, 18, 17, 18, 18, 17, 18, 21,
                                     19, 20, 21, 20, 19, 21, 24, 22, 22, 24, 24, 22, 22, 24, 25, 25, 27, 30, 27, 25, 25, 29,
                                     31, 35, 35, 31, 29, 36, 41, 44, 41, 36, 47, 54, 54, 47, 65, 70, 65, 88, 88, 115};
static const uint8_t kSlInter[64] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 17, 18, 18, 18, 18, 18, 18, 20,
                                     20, 20, 20, 20, 20, 20, 24, 24, 24, 24, 24, 24, 24, 24, 25, 25, 25, 25, 25, 25, 25, 28,
                                     28, 28, 28, 28, 28, 33, 33, 33, 33, 33, 41, 41, 41, 41, 54, 54, 54, 71, 71, 91};

static void default_list(int size_id, int matrix_id, ScalingLists& sl) {
    for (int i = 0; i < 64; ++i)
        sl.list[size_id][matrix_id][i] = size_id == 0 ? 16 : (matrix_id < 3 ? kSlIntra[i] : kSlInter[i]);
    sl.dc[size_id][matrix_id] = 16;
}

ScalingLists default_scaling_lists() {
    ScalingLists sl;
    for (int size_id = 0; size_id < 4; ++size_id)
        for (int matrix_id = 0; matrix_id < 6; ++matrix_id) default_list(size_id, matrix_id, sl);
    return sl;
}

// 6.5.3 up-right diagonal scan position i of a blk x blk block
static void diag_pos(int blk, int i, int& x, int& y) {
    int k = 0;
    for (int d = 0;; ++d)
        for (int yy = d, xx = 0; yy >= 0; --yy, ++xx)
            if (xx < blk && yy < blk && k++ == i) { x = xx; y = yy; return; }
}

void scaling_factors(const ScalingLists& sl, uint8_t out[2032]) {
    static const int kOff[4][3] = {{0, 16, 32}, {48, 112, 176}, {240, 496, 752}, {1008, -1, -1}};
    for (int size_id = 0; size_id < 4; ++size_id)
        for (int m = 0; m < (size_id == 3 ? 1 : 3); ++m) {
            const int n = 4 << size_id, blk = size_id == 0 ? 4 : 8, rep = n / blk;
            uint8_t* f = out + kOff[size_id][m];
            for (int i = 0; i < blk * blk; ++i) {
                int x = 0, y = 0;
                diag_pos(blk, i, x, y);
                for (int j = 0; j < rep; ++j)
                    for (int k = 0; k < rep; ++k) f[(y * rep + j) * n + x * rep + k] = sl.list[size_id][m][i];
            }
            if (size_id > 1) f[0] = sl.dc[size_id][m];
        }
}

// scaling_list_data() (7.3.4; sld.py:63-117) resolved per 7.4.5 (the numbering of matrixId of the 2016+
// editions: 0 and 3 for sizeId 3, refMatrixId = matrixId - delta * 3 there; v1's 0 / 1 code the same lists)
static void parse_scaling_list_data(BitReader& br, ScalingLists& sl) {
    for (int size_id = 0; size_id < 4; ++size_id)
        for (int matrix_id = 0; matrix_id < 6; matrix_id += (size_id == 3) ? 3 : 1) {
            if (!br.flag()) {                                      // scaling_list_pred_mode_flag = 0
                const uint32_t delta = br.ue();                    // scaling_list_pred_matrix_id_delta
                const int step = size_id == 3 ? 3 : 1;
                if (delta > (uint32_t)(matrix_id / step)) bs_fail("scaling_list_pred_matrix_id_delta out of range");
                if (delta == 0) {
                    default_list(size_id, matrix_id, sl);
                } else {
                    const int ref = matrix_id - (int)delta * step;
                    std::memcpy(sl.list[size_id][matrix_id], sl.list[size_id][ref], 64);
                    sl.dc[size_id][matrix_id] = sl.dc[size_id][ref];
                }
            } else {
                int next = 8;
                const int coef_num = std::min(64, 1 << (4 + (size_id << 1)));
                if (size_id > 1) {
                    const int dc = br.se();                        // scaling_list_dc_coef_minus8
                    if (dc < -7 || dc > 247) bs_fail("scaling_list_dc_coef_minus8 out of range");
                    next = dc + 8;
                    sl.dc[size_id][matrix_id] = (uint8_t)next;
                }
                for (int i = 0; i < coef_num; ++i) {
                    const int d = br.se();                         // scaling_list_delta_coef
                    if (d < -128 || d > 127) bs_fail("scaling_list_delta_coef out of range");
                    next = (next + d + 256) % 256;
                    if (next == 0) bs_fail("ScalingList value 0");
                    sl.list[size_id][matrix_id][i] = (uint8_t)next;
                }
            }
        }
}

// st_ref_pic_set(stRpsIdx) (7.3.7) + derivation (7.4.8); st_rps.py:5
static StRps parse_st_rps(BitReader& br, int idx, int num_sets, const std::vector<StRps>& sets) {
    StRps r;
    int inter = 0;
    if (idx != 0) inter = br.flag();
    if (inter) {
        int delta_idx_minus1 = 0;
        if (idx == num_sets) delta_idx_minus1 = (int)br.ue();
        if (delta_idx_minus1 + 1 > idx) bs_fail("delta_idx_minus1 out of range");
        int ref_idx = idx - (delta_idx_minus1 + 1);
        int sign = br.flag();
        int abs_minus1 = (int)br.ue();
        int delta_rps = (1 - 2 * sign) * (abs_minus1 + 1);
        const StRps& ref = sets[ref_idx];
        int n = ref.num_delta_pocs();
        uint8_t used[33] = {}, use_delta[33];
        for (int j = 0; j <= n; ++j) {
            used[j] = (uint8_t)br.flag();
            use_delta[j] = 1;
            if (!used[j]) use_delta[j] = (uint8_t)br.flag();
        }
        // (7-61)
        int i = 0;
        for (int j = ref.num_positive - 1; j >= 0; --j) {
            int dpoc = ref.delta_poc_s1[j] + delta_rps;
            if (dpoc < 0 && use_delta[ref.num_negative + j]) {
                if (i >= 16) bs_fail("st_rps too large");
                r.delta_poc_s0[i] = dpoc; r.used_s0[i++] = used[ref.num_negative + j];
            }
        }
        if (delta_rps < 0 && use_delta[n]) {
            if (i >= 16) bs_fail("st_rps too large");
            r.delta_poc_s0[i] = delta_rps; r.used_s0[i++] = used[n];
        }
        for (int j = 0; j < ref.num_negative; ++j) {
            int dpoc = ref.delta_poc_s0[j] + delta_rps;
            if (dpoc < 0 && use_delta[j]) {
                if (i >= 16) bs_fail("st_rps too large");
                r.delta_poc_s0[i] = dpoc; r.used_s0[i++] = used[j];
            }
        }
        r.num_negative = i;
        // (7-62)
        i = 0;
        for (int j = ref.num_negative - 1; j >= 0; --j) {
            int dpoc = ref.delta_poc_s0[j] + delta_rps;
            if (dpoc > 0 && use_delta[j]) {
                if (i >= 16) bs_fail("st_rps too large");
                r.delta_poc_s1[i] = dpoc; r.used_s1[i++] = used[j];
            }
        }
        if (delta_rps > 0 && use_delta[n]) {
            if (i >= 16) bs_fail("st_rps too large");
            r.delta_poc_s1[i] = delta_rps; r.used_s1[i++] = used[n];
        }
        for (int j = 0; j < ref.num_positive; ++j) {
            int dpoc = ref.delta_poc_s1[j] + delta_rps;
            if (dpoc > 0 && use_delta[ref.num_negative + j]) {
                if (i >= 16) bs_fail("st_rps too large");
                r.delta_poc_s1[i] = dpoc; r.used_s1[i++] = used[ref.num_negative + j];
            }
        }
        r.num_positive = i;
    } else {
        r.num_negative = (int)br.ue();
        r.num_positive = (int)br.ue();
        if (r.num_negative > 16 || r.num_positive > 16 || r.num_negative + r.num_positive > 16)
            bs_fail("num_negative_pics/num_positive_pics out of range");
        int poc = 0;
        for (int i = 0; i < r.num_negative; ++i) {
            poc -= (int)br.ue() + 1;
            r.delta_poc_s0[i] = poc;
            r.used_s0[i] = (uint8_t)br.flag();
        }
        poc = 0;
        for (int i = 0; i < r.num_positive; ++i) {
            poc += (int)br.ue() + 1;
            r.delta_poc_s1[i] = poc;
            r.used_s1[i] = (uint8_t)br.flag();
        }
    }
    return r;
}

// sub_layer_hrd_parameters() (E.2.3)
static void parse_sub_layer_hrd(BitReader& br, int cpb_cnt, int sub_pic) {
    for (int i = 0; i <= cpb_cnt; ++i) {
        br.ue(); br.ue();
        if (sub_pic) { br.ue(); br.ue(); }
        br.skip(1);
    }
}

// hrd_parameters() (E.2.2)
static void parse_hrd(BitReader& br, int common, int max_sub_layers_minus1) {
    int nal = 0, vcl = 0, sub_pic = 0;
    if (common) {
        nal = br.flag();
        vcl = br.flag();
        if (nal || vcl) {
            sub_pic = br.flag();
            if (sub_pic) br.skip(8 + 5 + 1 + 5);
            br.skip(4 + 4);
            if (sub_pic) br.skip(4);
            br.skip(5 + 5 + 5);
        }
    }
    for (int i = 0; i <= max_sub_layers_minus1; ++i) {
        int fixed_general = br.flag();
        int fixed_cvs = 1;
        if (!fixed_general) fixed_cvs = br.flag();
        int low_delay = 0;
        if (fixed_cvs) br.ue();
        else low_delay = br.flag();
        int cpb_cnt = 0;
        if (!low_delay) cpb_cnt = (int)br.ue();
        if (cpb_cnt > 31) bs_fail("cpb_cnt_minus1 out of range");
        if (nal) parse_sub_layer_hrd(br, cpb_cnt, sub_pic);
        if (vcl) parse_sub_layer_hrd(br, cpb_cnt, sub_pic);
    }
}

// vui_parameters() (E.2.1); the reference stops here (sps.py:131 calls an undefined object)
static void parse_vui(BitReader& br, int max_sub_layers_minus1) {
    if (br.flag()) {                       // aspect_ratio_info_present_flag
        if (br.u(8) == 255) br.skip(32);   // sar_width, sar_height
    }
    if (br.flag()) br.skip(1);             // overscan
    if (br.flag()) {                       // video_signal_type_present_flag
        br.skip(3 + 1);
        if (br.flag()) br.skip(24);
    }
    if (br.flag()) { br.ue(); br.ue(); }   // chroma_loc_info
    br.skip(3);                            // neutral_chroma, field_seq, frame_field_info
    if (br.flag()) { br.ue(); br.ue(); br.ue(); br.ue(); }   // default display window
    if (br.flag()) {                       // vui_timing_info_present_flag
        br.skip(64);
        if (br.flag()) br.ue();
        if (br.flag()) parse_hrd(br, 1, max_sub_layers_minus1);
    }
    if (br.flag()) {                       // bitstream_restriction_flag
        br.skip(3);
        br.ue(); br.ue(); br.ue(); br.ue(); br.ue();
    }
}

void parse_vps(BitReader& br) {
    br.u(4);   // vps_video_parameter_set_id; nothing of the VPS reaches the reconstruction
}

Sps parse_sps(BitReader& br) {
    Sps s;
    s.vps_id = (int)br.u(4);
    s.max_sub_layers_minus1 = (int)br.u(3);
    if (s.max_sub_layers_minus1 > 6) bs_fail("sps_max_sub_layers_minus1 > 6");
    br.skip(1);
    parse_ptl(br, s.max_sub_layers_minus1);
    s.sps_id = (int)br.ue();
    if (s.sps_id > 15) bs_fail("sps_seq_parameter_set_id > 15");
    s.chroma_format_idc = (int)br.ue();
    if (s.chroma_format_idc > 3) bs_fail("chroma_format_idc > 3");
    if (s.chroma_format_idc == 3) s.separate_colour_plane = br.flag();
    s.width = (int)br.ue();
    s.height = (int)br.ue();
    if (s.width <= 0 || s.height <= 0 || s.width > 16888 || s.height > 16888) bs_fail("picture size out of range");
    if (br.flag()) {
        s.conf_left = (int)br.ue(); s.conf_right = (int)br.ue();
        s.conf_top = (int)br.ue(); s.conf_bottom = (int)br.ue();
    }
    s.bit_depth_y = 8 + (int)br.ue();
    s.bit_depth_c = 8 + (int)br.ue();
    if (s.bit_depth_y > 16 || s.bit_depth_c > 16) bs_fail("bit depth out of range");
    s.log2_max_poc_lsb = 4 + (int)br.ue();
    if (s.log2_max_poc_lsb > 16) bs_fail("log2_max_pic_order_cnt_lsb_minus4 > 12");
    int ordering = br.flag();
    for (int i = ordering ? 0 : s.max_sub_layers_minus1; i <= s.max_sub_layers_minus1; ++i) {
        br.ue();                                       // sps_max_dec_pic_buffering_minus1
        s.max_num_reorder = (int)br.ue();              // sps_max_num_reorder_pics (HighestTid = last)
        br.ue();                                       // sps_max_latency_increase_plus1
    }
    if (s.max_num_reorder > 16) bs_fail("sps_max_num_reorder_pics > 16");
    s.log2_min_cb = 3 + (int)br.ue();
    s.log2_ctb = s.log2_min_cb + (int)br.ue();
    s.log2_min_tb = 2 + (int)br.ue();
    s.log2_max_tb = s.log2_min_tb + (int)br.ue();
    s.max_th_depth_inter = (int)br.ue();
    s.max_th_depth_intra = (int)br.ue();
    if (s.log2_ctb > 6 || s.log2_ctb < 4 || s.log2_max_tb > 5 || s.log2_min_tb >= s.log2_min_cb ||
        s.log2_max_tb > s.log2_ctb || s.max_th_depth_intra > s.log2_ctb - s.log2_min_tb)
        bs_fail("SPS block sizes out of range");
    if ((s.width & ((1 << s.log2_min_cb) - 1)) || (s.height & ((1 << s.log2_min_cb) - 1)))
        bs_fail("picture size not a multiple of MinCbSizeY");
    s.scaling_list_enabled = br.flag();
    s.scaling = default_scaling_lists();
    if (s.scaling_list_enabled) {
        s.scaling_list_data_present = br.flag();
        if (s.scaling_list_data_present) parse_scaling_list_data(br, s.scaling);
    }
    s.amp = br.flag();
    s.sao = br.flag();
    s.pcm = br.flag();
    if (s.pcm) {
        s.pcm_bit_depth_y = 1 + (int)br.u(4);
        s.pcm_bit_depth_c = 1 + (int)br.u(4);
        s.log2_min_pcm = 3 + (int)br.ue();
        s.log2_max_pcm = s.log2_min_pcm + (int)br.ue();
        s.pcm_loop_filter_disabled = br.flag();
        if (s.pcm_bit_depth_y > s.bit_depth_y || s.pcm_bit_depth_c > s.bit_depth_c || s.log2_max_pcm > 5 ||
            s.log2_max_pcm > s.log2_ctb)
            bs_fail("PCM parameters out of range");
    }
    int num_sets = (int)br.ue();
    if (num_sets > 64) bs_fail("num_short_term_ref_pic_sets > 64");
    for (int i = 0; i < num_sets; ++i) s.st_rps.push_back(parse_st_rps(br, i, num_sets, s.st_rps));
    s.long_term_refs_present = br.flag();
    if (s.long_term_refs_present) {
        s.num_long_term_ref_pics_sps = (int)br.ue();
        if (s.num_long_term_ref_pics_sps > 32) bs_fail("num_long_term_ref_pics_sps > 32");
        for (int i = 0; i < s.num_long_term_ref_pics_sps; ++i) br.skip((size_t)s.log2_max_poc_lsb + 1);
    }
    s.temporal_mvp = br.flag();
    s.strong_intra_smoothing = br.flag();
    if (br.flag()) parse_vui(br, s.max_sub_layers_minus1);
    if (br.flag()) {                                  // sps_extension_present_flag
        int range = br.flag();
        br.skip(3);                                   // multilayer, 3d, scc
        br.skip(4);
        if (range) s.range_extension_flags = (int)br.u(9);
    }
    return s;
}

Pps parse_pps(BitReader& br) {
    Pps p;
    p.pps_id = (int)br.ue();
    if (p.pps_id > 63) bs_fail("pps_pic_parameter_set_id > 63");
    p.sps_id = (int)br.ue();
    if (p.sps_id > 15) bs_fail("pps_seq_parameter_set_id > 15");
    p.dependent_slice_segments = br.flag();
    p.output_flag_present = br.flag();
    p.num_extra_slice_header_bits = (int)br.u(3);
    p.sign_data_hiding = br.flag();
    p.cabac_init_present = br.flag();
    br.ue(); br.ue();                                 // num_ref_idx_l0/l1_default_active_minus1
    p.init_qp = 26 + br.se();
    p.constrained_intra_pred = br.flag();
    p.transform_skip = br.flag();
    p.cu_qp_delta = br.flag();
    if (p.cu_qp_delta) p.diff_cu_qp_delta_depth = (int)br.ue();
    p.cb_qp_offset = br.se();
    p.cr_qp_offset = br.se();
    if (p.cb_qp_offset < -12 || p.cb_qp_offset > 12 || p.cr_qp_offset < -12 || p.cr_qp_offset > 12)
        bs_fail("pps_cb/cr_qp_offset out of range");
    p.slice_chroma_qp_offsets_present = br.flag();
    p.weighted_pred = br.flag();
    p.weighted_bipred = br.flag();
    p.transquant_bypass = br.flag();
    p.tiles = br.flag();
    p.entropy_coding_sync = br.flag();
    if (p.tiles) {
        p.num_tile_cols = (int)br.ue() + 1;
        p.num_tile_rows = (int)br.ue() + 1;
        if (p.num_tile_cols > 64 || p.num_tile_rows > 64) bs_fail("too many tiles");
        p.uniform_spacing = br.flag();
        if (!p.uniform_spacing) {
            for (int i = 0; i < p.num_tile_cols - 1; ++i) p.col_width_minus1.push_back((int)br.ue());
            for (int i = 0; i < p.num_tile_rows - 1; ++i) p.row_height_minus1.push_back((int)br.ue());
        }
        p.loop_filter_across_tiles = br.flag();
    }
    p.loop_filter_across_slices = br.flag();
    p.deblocking_control_present = br.flag();
    if (p.deblocking_control_present) {
        p.deblocking_override_enabled = br.flag();
        p.deblocking_disabled = br.flag();
        if (!p.deblocking_disabled) {
            p.beta_offset_div2 = br.se();
            p.tc_offset_div2 = br.se();
            if (p.beta_offset_div2 < -6 || p.beta_offset_div2 > 6 || p.tc_offset_div2 < -6 || p.tc_offset_div2 > 6)
                bs_fail("pps_beta/tc_offset_div2 out of range");
        }
    }
    p.scaling_list_data_present = br.flag();
    p.scaling = default_scaling_lists();
    if (p.scaling_list_data_present) parse_scaling_list_data(br, p.scaling);
    p.lists_modification_present = br.flag();
    p.log2_parallel_merge_level = 2 + (int)br.ue();
    p.slice_header_extension_present = br.flag();
    if (br.flag()) {                                  // pps_extension_present_flag
        int range = br.flag();
        br.skip(3 + 4);
        if (range) {
            int any = 0;
            if (p.transform_skip) any |= (br.ue() != 0);   // log2_max_transform_skip_block_size_minus2
            any |= br.flag();                              // cross_component_prediction_enabled_flag
            if (br.flag()) any = 1;                        // chroma_qp_offset_list_enabled_flag
            else {
                any |= (br.ue() != 0);                     // log2_sao_offset_scale_luma
                any |= (br.ue() != 0);                     // log2_sao_offset_scale_chroma
            }
            p.range_extension_flags = any;
        }
    }
    return p;
}

std::shared_ptr<const Active> activate(const Sps& sps, const Pps& pps) {
    auto a = std::make_shared<Active>();
    a->sps = sps;
    a->pps = pps;
    int W = sps.pic_w_ctb(), H = sps.pic_h_ctb();
    a->w_ctb = W; a->h_ctb = H; a->size_ctb = W * H;
    int nc = pps.num_tile_cols, nr = pps.num_tile_rows;
    if (nc > W || nr > H) bs_fail("more tile columns/rows than CTBs");
    std::vector<int> cw(nc), rh(nr);
    if (pps.uniform_spacing) {                       // (6-3), (6-4)
        for (int i = 0; i < nc; ++i) cw[i] = ((i + 1) * W) / nc - (i * W) / nc;
        for (int j = 0; j < nr; ++j) rh[j] = ((j + 1) * H) / nr - (j * H) / nr;
    } else {
        int sum = 0;
        for (int i = 0; i < nc - 1; ++i) { cw[i] = pps.col_width_minus1[i] + 1; sum += cw[i]; }
        if (sum >= W) bs_fail("tile columns exceed picture width");
        cw[nc - 1] = W - sum;
        sum = 0;
        for (int j = 0; j < nr - 1; ++j) { rh[j] = pps.row_height_minus1[j] + 1; sum += rh[j]; }
        if (sum >= H) bs_fail("tile rows exceed picture height");
        rh[nr - 1] = H - sum;
    }
    a->col_bd.assign(nc + 1, 0);
    a->row_bd.assign(nr + 1, 0);
    for (int i = 0; i < nc; ++i) a->col_bd[i + 1] = a->col_bd[i] + cw[i];
    for (int j = 0; j < nr; ++j) a->row_bd[j + 1] = a->row_bd[j] + rh[j];
    a->ctb_col_tile.assign(W, 0);
    a->ctb_row_tile.assign(H, 0);
    for (int i = 0; i < nc; ++i)
        for (int x = a->col_bd[i]; x < a->col_bd[i + 1]; ++x) a->ctb_col_tile[x] = i;
    for (int j = 0; j < nr; ++j)
        for (int y = a->row_bd[j]; y < a->row_bd[j + 1]; ++y) a->ctb_row_tile[y] = j;
    // CtbAddrRsToTs (6-5), CtbAddrTsToRs, TileId (6-7); pps.py:152-228
    a->rs_to_ts.assign(a->size_ctb, 0);
    a->ts_to_rs.assign(a->size_ctb, 0);
    a->tile_id_ts.assign(a->size_ctb, 0);
    for (int rs = 0; rs < a->size_ctb; ++rs) {
        int tbx = rs % W, tby = rs / W;
        int ti = a->ctb_col_tile[tbx], tj = a->ctb_row_tile[tby];
        int v = 0;
        for (int i = 0; i < ti; ++i) v += rh[tj] * cw[i];
        for (int j = 0; j < tj; ++j) v += W * rh[j];
        v += (tby - a->row_bd[tj]) * cw[ti] + tbx - a->col_bd[ti];
        a->rs_to_ts[rs] = v;
        a->ts_to_rs[v] = rs;
    }
    for (int j = 0, tid = 0; j < nr; ++j)
        for (int i = 0; i < nc; ++i, ++tid)
            for (int y = a->row_bd[j]; y < a->row_bd[j + 1]; ++y)
                for (int x = a->col_bd[i]; x < a->col_bd[i + 1]; ++x) a->tile_id_ts[a->rs_to_ts[y * W + x]] = tid;
    a->log2_min_cu_qp_delta = sps.log2_ctb - pps.diff_cu_qp_delta_depth;
    if (a->log2_min_cu_qp_delta < sps.log2_min_cb) bs_fail("diff_cu_qp_delta_depth out of range");
    // ScalingFactor (7.4.5): the PPS lists when present, else the SPS lists (the defaults when the SPS
    // codes none)
    if (sps.scaling_list_enabled) scaling_factors(pps.scaling_list_data_present ? pps.scaling : sps.scaling, a->scaling_factor.data());
    return a;
}

int peek_slice_pps_id(const std::vector<uint8_t>& rbsp, int nal_type, int* first_in_pic) {
    BitReader br(rbsp.data(), rbsp.size());
    *first_in_pic = br.flag();
    if (nal_type >= 16 && nal_type <= 23) br.skip(1);
    return (int)br.ue();
}

SliceHeader parse_slice_header(BitReader& br, int nal_type, const std::shared_ptr<const Active>& act,
                               const SliceHeader* prev_indep) {
    const Sps& sps = act->sps;
    const Pps& pps = act->pps;
    SliceHeader h;
    h.first_slice_segment_in_pic = br.flag();
    if (nal_type >= 16 && nal_type <= 23) h.no_output_of_prior_pics = br.flag();
    h.pps_id = (int)br.ue();
    if (!h.first_slice_segment_in_pic) {
        if (pps.dependent_slice_segments) h.dependent = br.flag();
        h.segment_address = (int)br.u(ceil_log2(act->size_ctb));
        if (h.segment_address >= act->size_ctb) bs_fail("slice_segment_address out of range");
    }
    if (h.dependent) {
        if (!prev_indep) bs_fail("dependent slice segment without a preceding independent segment");
        SliceHeader d = *prev_indep;
        d.first_slice_segment_in_pic = h.first_slice_segment_in_pic;
        d.no_output_of_prior_pics = h.no_output_of_prior_pics;
        d.pps_id = h.pps_id;
        d.dependent = 1;
        d.segment_address = h.segment_address;
        d.entry_point_offsets.clear();
        d.num_entry_points = 0;
        h = d;
    } else {
        br.skip(pps.num_extra_slice_header_bits);
        h.slice_type = (int)br.ue();
        if (h.slice_type > 2) bs_fail("slice_type > 2");
        if (h.slice_type != 2) throw Unsupported("P/B slices (the back-end reconstructs all-intra streams)");
        if (pps.output_flag_present) h.pic_output_flag = br.flag();
        if (sps.separate_colour_plane) h.colour_plane_id = (int)br.u(2);
        if (nal_type != 19 && nal_type != 20) {      // not IDR_W_RADL / IDR_N_LP
            h.poc_lsb = (int)br.u(sps.log2_max_poc_lsb);
            int st_sps = br.flag();
            int num_sets = (int)sps.st_rps.size();
            if (!st_sps) {
                parse_st_rps(br, num_sets, num_sets, sps.st_rps);
            } else if (num_sets > 1) {
                br.u(ceil_log2(num_sets));
            } else if (num_sets == 0) {
                bs_fail("short_term_ref_pic_set_sps_flag with no SPS sets");
            }
            if (sps.long_term_refs_present) {
                int num_lt_sps = 0;
                if (sps.num_long_term_ref_pics_sps > 0) num_lt_sps = (int)br.ue();
                int num_lt_pics = (int)br.ue();
                if (num_lt_sps > sps.num_long_term_ref_pics_sps || num_lt_pics > 32) bs_fail("long-term picture count");
                for (int i = 0; i < num_lt_sps + num_lt_pics; ++i) {
                    if (i < num_lt_sps) {
                        if (sps.num_long_term_ref_pics_sps > 1) br.u(ceil_log2(sps.num_long_term_ref_pics_sps));
                    } else {
                        br.u(sps.log2_max_poc_lsb);
                        br.skip(1);
                    }
                    if (br.flag()) br.ue();   // delta_poc_msb_present_flag -> delta_poc_msb_cycle_lt
                }
            }
            if (sps.temporal_mvp) br.skip(1);
        }
        if (sps.sao) {
            h.sao_luma = br.flag();
            if (sps.chroma_format_idc != 0) h.sao_chroma = br.flag();
        }
        h.slice_qp_delta = br.se();
        h.slice_qp_y = pps.init_qp + h.slice_qp_delta;
        int qp_bd = 6 * (sps.bit_depth_y - 8);
        if (h.slice_qp_y < -qp_bd || h.slice_qp_y > 51) bs_fail("SliceQpY out of range");
        if (pps.slice_chroma_qp_offsets_present) {
            h.cb_qp_offset = br.se();
            h.cr_qp_offset = br.se();
            if (h.cb_qp_offset < -12 || h.cb_qp_offset > 12 || h.cr_qp_offset < -12 || h.cr_qp_offset > 12 ||
                pps.cb_qp_offset + h.cb_qp_offset < -12 || pps.cb_qp_offset + h.cb_qp_offset > 12 ||
                pps.cr_qp_offset + h.cr_qp_offset < -12 || pps.cr_qp_offset + h.cr_qp_offset > 12)
                bs_fail("slice_cb/cr_qp_offset out of range");
        }
        int override_flag = 0;
        if (pps.deblocking_override_enabled) override_flag = br.flag();
        h.deblocking_disabled = pps.deblocking_disabled;
        h.beta_offset_div2 = pps.beta_offset_div2;
        h.tc_offset_div2 = pps.tc_offset_div2;
        if (override_flag) {                          // slice.py:177 raises here
            h.deblocking_disabled = br.flag();
            if (!h.deblocking_disabled) {
                h.beta_offset_div2 = br.se();
                h.tc_offset_div2 = br.se();
                if (h.beta_offset_div2 < -6 || h.beta_offset_div2 > 6 || h.tc_offset_div2 < -6 || h.tc_offset_div2 > 6)
                    bs_fail("slice_beta/tc_offset_div2 out of range");
            }
        }
        h.loop_filter_across_slices = pps.loop_filter_across_slices;
        if (pps.loop_filter_across_slices && (h.sao_luma || h.sao_chroma || !h.deblocking_disabled))
            h.loop_filter_across_slices = br.flag();
    }
    if (pps.tiles || pps.entropy_coding_sync) {       // slice.py:181-186 raises here
        h.num_entry_points = (int)br.ue();
        if (h.num_entry_points > act->size_ctb) bs_fail("num_entry_point_offsets out of range");
        if (h.num_entry_points > 0) {
            int len = (int)br.ue() + 1;
            if (len > 32) bs_fail("offset_len_minus1 > 31");
            for (int i = 0; i < h.num_entry_points; ++i) h.entry_point_offsets.push_back(br.u(len) + 1);
        }
    }
    if (pps.slice_header_extension_present) {         // slice.py:188-189 raises here
        int len = (int)br.ue();
        br.skip((size_t)len * 8);
    }
    br.byte_alignment();
    h.data_byte_offset = br.pos() >> 3;
    return h;
}

}  // namespace p265fe
