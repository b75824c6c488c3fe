// Parameter sets and slice segment headers of the native front-end (H.265 7.3.2-7.3.6).
//
// Reference counterparts: Vps.parse (decoder/vps.py:9), Sps.parse (sps.py:24-140) and its
// derived sizes (sps.py:142-171), Pps.parse (pps.py:16-150) with the tile scan conversion
// (pps.py:152-228), ShortTermRefPicSet.decode (st_rps.py:5), ScalingListData.decode
// (sld.py:63), SliceSegmentHeader.parse (slice.py:35-191).  Where the reference raises
// "Unimplemented" (VUI/HRD sps.py:131, deblocking override slice.py:177, entry points
// slice.py:185, header extension slice.py:189, tiles pps.py:61-93) this parses the syntax.
#pragma once
#include <array>
#include <cstdint>
#include <memory>
#include <vector>

#include "fe_bits.h"

namespace p265fe {

struct StRps {            // st_ref_pic_set() (7.3.7) with its derived lists (7.4.8)
    int num_negative = 0, num_positive = 0;
    int delta_poc_s0[16] = {}, delta_poc_s1[16] = {};
    uint8_t used_s0[16] = {}, used_s1[16] = {};
    int num_delta_pocs() const { return num_negative + num_positive; }
};

// scaling_list_data() (7.3.4) resolved by 7.4.5: ScalingList[sizeId][matrixId][i] (predicted lists copied,
// defaults of Table 7-5 / 7-6 filled in) and the 16x16 / 32x32 DC values
struct ScalingLists {
    uint8_t list[4][6][64] = {};
    uint8_t dc[4][6] = {};
};
ScalingLists default_scaling_lists();
// ScalingFactor (7.4.5) of the intra matrices 4:2:0 uses, in p265r_set_scaling_factors' layout (2032 B)
void scaling_factors(const ScalingLists& sl, uint8_t out[2032]);

struct Sps {
    int sps_id = 0, vps_id = 0, max_sub_layers_minus1 = 0;
    int chroma_format_idc = 1, separate_colour_plane = 0;
    int width = 0, height = 0;
    int conf_left = 0, conf_right = 0, conf_top = 0, conf_bottom = 0;   // in chroma units (7.4.3.2.1)
    int bit_depth_y = 8, bit_depth_c = 8;
    int log2_max_poc_lsb = 4;
    int max_num_reorder = 0;          // sps_max_num_reorder_pics[sps_max_sub_layers_minus1] (C.5.2.2 bumping)
    int log2_min_cb = 3, log2_ctb = 4, log2_min_tb = 2, log2_max_tb = 5;
    int max_th_depth_inter = 0, max_th_depth_intra = 0;
    int scaling_list_enabled = 0, scaling_list_data_present = 0;
    ScalingLists scaling;             // sps_scaling_list_data (defaults when not present)
    int amp = 0, sao = 0;
    int pcm = 0, pcm_bit_depth_y = 8, pcm_bit_depth_c = 8, log2_min_pcm = 3, log2_max_pcm = 3, pcm_loop_filter_disabled = 0;
    std::vector<StRps> st_rps;
    int long_term_refs_present = 0, num_long_term_ref_pics_sps = 0;
    int temporal_mvp = 0, strong_intra_smoothing = 0;
    int range_extension_flags = 0;   // any sps_range_extension() flag set (unsupported)
    // derived (7.4.3.2.1)
    int ctb_size() const { return 1 << log2_ctb; }
    int pic_w_ctb() const { return (width + ctb_size() - 1) >> log2_ctb; }
    int pic_h_ctb() const { return (height + ctb_size() - 1) >> log2_ctb; }
    int pic_size_ctb() const { return pic_w_ctb() * pic_h_ctb(); }
};

struct Pps {
    int pps_id = 0, sps_id = 0;
    int dependent_slice_segments = 0, output_flag_present = 0, num_extra_slice_header_bits = 0;
    int sign_data_hiding = 0, cabac_init_present = 0;
    int init_qp = 26, constrained_intra_pred = 0, transform_skip = 0;
    int cu_qp_delta = 0, diff_cu_qp_delta_depth = 0;
    int cb_qp_offset = 0, cr_qp_offset = 0, slice_chroma_qp_offsets_present = 0;
    int weighted_pred = 0, weighted_bipred = 0, transquant_bypass = 0;
    int tiles = 0, entropy_coding_sync = 0;
    int num_tile_cols = 1, num_tile_rows = 1, uniform_spacing = 1;
    std::vector<int> col_width_minus1, row_height_minus1;   // explicit spacing
    int loop_filter_across_tiles = 1, loop_filter_across_slices = 0;
    int deblocking_control_present = 0, deblocking_override_enabled = 0, deblocking_disabled = 0;
    int beta_offset_div2 = 0, tc_offset_div2 = 0;
    int scaling_list_data_present = 0, lists_modification_present = 0, log2_parallel_merge_level = 2;
    ScalingLists scaling;             // pps_scaling_list_data (when present)
    int slice_header_extension_present = 0;
    int range_extension_flags = 0;   // any pps_range_extension() feature used (unsupported)
};

// SPS + PPS of one picture with the PPS-derived scan conversion arrays (6.5.1).
struct Active {
    Sps sps;
    Pps pps;
    int w_ctb = 0, h_ctb = 0, size_ctb = 0;
    std::vector<int> col_bd, row_bd;          // tile boundaries in CTBs (num+1 entries)
    std::vector<int> rs_to_ts, ts_to_rs, tile_id_ts;
    std::vector<int> ctb_col_tile, ctb_row_tile;   // tile column / row of a CTB column / row
    int log2_min_cu_qp_delta = 0;
    std::array<uint8_t, 2032> scaling_factor{};   // ScalingFactor (PPS lists, else SPS lists, else defaults)
                                                  // when sps.scaling_list_enabled
    int tile_id_rs(int rs) const { return tile_id_ts[rs_to_ts[rs]]; }
};
std::shared_ptr<const Active> activate(const Sps& sps, const Pps& pps);

struct SliceHeader {
    int first_slice_segment_in_pic = 0, no_output_of_prior_pics = 0, pps_id = 0;
    int dependent = 0, segment_address = 0;
    int slice_type = 2, pic_output_flag = 1, colour_plane_id = 0;
    int poc_lsb = 0;
    int sao_luma = 0, sao_chroma = 0;
    int slice_qp_delta = 0, slice_qp_y = 26;
    int cb_qp_offset = 0, cr_qp_offset = 0;
    int deblocking_disabled = 0, beta_offset_div2 = 0, tc_offset_div2 = 0;
    int loop_filter_across_slices = 0;
    int num_entry_points = 0;
    std::vector<uint32_t> entry_point_offsets;
    size_t data_byte_offset = 0;     // first byte of slice_segment_data() in the RBSP
};

// Parsers.  `sps_table`/`pps_table` are indexed by id; nullptr = not received.
void parse_vps(BitReader& br);
Sps parse_sps(BitReader& br);
Pps parse_pps(BitReader& br);
// Parse a slice segment header; fields of a dependent segment are copied from `prev_indep`
// (the header of the preceding independent segment of the same picture).
SliceHeader parse_slice_header(BitReader& br, int nal_type, const std::shared_ptr<const Active>& act,
                               const SliceHeader* prev_indep);
// slice_pic_parameter_set_id of a slice segment header (after first_slice_segment_in_pic_flag
// and no_output_of_prior_pics_flag)
int peek_slice_pps_id(const std::vector<uint8_t>& rbsp, int nal_type, int* first_in_pic);

}  // namespace p265fe
