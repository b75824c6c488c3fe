/*
 * p265fe.h -- C ABI of the native (host, C++) HEVC syntax front-end that feeds the
 * MI355X reconstruction back-end (p265r.h).
 *
 * It replaces the reference's Python parsing stack for all-intra streams
 * (SURVEY.md §8(f) item 2 and item 4):
 *     Decoder.decode NAL loop                      (dec.py:18-64, nalu.py:73-131)
 *     BitStreamBuffer start codes / u / ue / se    (bsb.py:58-176)
 *     Vps/Sps/Pps.parse                            (vps.py:9, sps.py:24-171, pps.py:16-262)
 *     SliceSegmentHeader.parse                     (slice.py:35-191; entry points slice.py:181-189)
 *     SliceSegmentData.parse, Ctu.parse            (slice.py:234-296, ctu.py:24-30)
 *     Cabac engine + context tables                (cabac.py:4-293)
 *     Sao.parse                                    (sao.py:15-220)
 *     Cu.parse / parse_leaf / intra modes / QP     (cu.py:41-593)
 *     Tu.parse / parse_leaf / residual_coding      (tu.py:11-665)
 * and emits, per picture, exactly the records that the reference's per-CU hook
 * (Cu.decode_leaf, cu.py:483) hands to the back-end through the Python
 * PictureBuilder (p265_amd/frontend.py): p265r_ctu[PicSizeInCtbsY] in raster order,
 * p265r_tb per transform block (grouped by CTU, decode order inside a CTU), dense
 * int16 coefficients in decode order, and the optional no-filter map.
 *
 * Scope: 4:2:0, 8..14-bit syntax (the back-end reconstructs 8-bit), I slices only
 * (P/B slices -> P265FE_EUNSUPPORTED), tiles, WPP (entropy_coding_sync), multiple
 * and dependent slice segments, PCM, cu_transquant_bypass, transform_skip, sign data
 * hiding, cu_qp_delta, deblocking/SAO syntax, decoded-picture-hash SEI.  Scaling lists
 * and range extensions are parsed where needed and reported as unsupported.
 *
 * Conventions: every function returns int (0 = P265FE_OK, < 0 = error); the decoder
 * owns every output buffer it returns (valid until p265fe_destroy or the next
 * p265fe_decode on the same decoder).  Not thread-safe per decoder object; the
 * decoder itself runs pictures on `n_threads` worker threads.
 */
#ifndef P265FE_H
#define P265FE_H

#include <stddef.h>
#include <stdint.h>

#include "p265r.h"

#ifdef __cplusplus
extern "C" {
#endif

#define P265FE_ABI_VERSION 4u   /* 3: P265FE_ASYNC, p265fe_wait; 4: scaling_factors */

#define P265FE_OK            0
#define P265FE_EINVAL       -1   /* bad argument                                   */
#define P265FE_ENOMEM       -2
#define P265FE_EBITSTREAM   -8   /* malformed / truncated bitstream                */
#define P265FE_EUNSUPPORTED -4   /* stream feature outside this front-end's scope  */

/* p265fe_picture_info.hash_type */
#define P265FE_HASH_NONE     -1
#define P265FE_HASH_MD5       0
#define P265FE_HASH_CRC       1
#define P265FE_HASH_CHECKSUM  2

/* p265fe_feed flags */
#define P265FE_FLUSH          1   /* end of stream: the last access unit is complete */
#define P265FE_ASYNC          2   /* parse the complete access units on the decoder's persistent
                                     workers and return at once (p265fe_wait / p265fe_take) */

typedef struct p265fe_picture_info {
    p265r_params     params;        /* back-end parameters of this picture's SPS/PPS         */
    const p265r_ctu* ctus;          /* PicSizeInCtbsY records, raster order                  */
    const p265r_tb*  tbs;
    uint32_t         n_tbs;
    uint32_t         n_ctus;
    const int16_t*   coef;
    uint64_t         n_coef;
    const uint8_t*   nofilter;      /* NULL when no PCM(loop filter off)/bypass block exists  */
    int32_t          poc;           /* PicOrderCntVal                                        */
    int32_t          output_rank;   /* position in output order (-1 = not output)            */
    uint16_t         crop_left, crop_right, crop_top, crop_bottom; /* conformance window, luma samples */
    uint8_t          nal_unit_type; /* of the first slice segment                            */
    int8_t           hash_type;     /* P265FE_HASH_*                                         */
    uint16_t         n_slices;      /* slice segments                                        */
    uint32_t         n_cus;         /* coding units parsed                                   */
    uint8_t          hash[3][16];   /* decoded picture hash per component (MD5: 16 B, CRC: 2 B BE, checksum: 4 B BE) */
    int32_t          cvs_id;        /* coded video sequence counter (IRAP with NoRaslOutputFlag = 1) */
    uint8_t          max_num_reorder; /* sps_max_num_reorder_pics: output "bumping" (C.5.2.2)   */
    uint8_t          output_flag;   /* PicOutputFlag                                             */
    uint16_t         reserved;
    const uint8_t*   scaling_factors; /* params.scaling_list_enabled: the intra ScalingFactor table of
                                       its SPS / PPS (7.4.5; PPS lists, else SPS lists, else the
                                       defaults), P265R_SCALING_FACTOR_BYTES in the layout of
                                       p265r_set_scaling_factors; NULL otherwise                  */
} p265fe_picture_info;

typedef struct p265fe_pictures p265fe_pictures;

typedef struct p265fe_decoder p265fe_decoder;

int  p265fe_create(p265fe_decoder** out);
void p265fe_destroy(p265fe_decoder* dec);

/* Parse a whole Annex-B byte stream (start-code delimited NAL units).  Parameter sets,
 * slice headers and POC are processed in stream order; the slice data of the pictures
 * is parsed on n_threads worker threads (0 = hardware concurrency).  Returns the number
 * of pictures (>= 0) or an error code (p265fe_last_error gives the text). */
int  p265fe_decode(p265fe_decoder* dec, const uint8_t* data, size_t size, int n_threads);

/* Picture i (decode order) of the last p265fe_decode. */
int  p265fe_picture(p265fe_decoder* dec, int i, p265fe_picture_info* out);

/* Streaming.  Feed the byte stream in order, in chunks of any size (flags = P265FE_FLUSH
 * with the last one, which may be empty).  Parameter sets, POC state, the access unit being
 * assembled and an incomplete trailing NAL unit carry over between calls; access units that
 * are complete (the next access unit has started, or FLUSH) are parsed on n_threads workers
 * and queued.  Returns the number of queued pictures, or an error code.  (p265fe_decode
 * resets this state.) */
int  p265fe_feed(p265fe_decoder* dec, const uint8_t* data, size_t size, int n_threads, int flags);
/* Move the queued pictures (decode order) into a new set owned by the caller; returns its
 * size.  output_rank is -1 in a set: output order is the caller's (cvs_id, poc,
 * max_num_reorder, output_flag give what the bumping process needs). */
int  p265fe_take(p265fe_decoder* dec, p265fe_pictures** out);
/* P265FE_ASYNC: every feed of a decoder passes it (no mixing).  Access units are parsed in the
 * background on n_threads persistent workers (those of the first async feed), so parsing of a
 * chunk overlaps the slowest pictures of the previous one; p265fe_feed returns the number of
 * pictures submitted and not yet taken.  p265fe_take then hands out the PARSED PREFIX in decode
 * order (possibly empty; a picture that failed to parse ends the prefix and its error code is
 * returned once the pictures before it are taken -- that take reports it once and drops the failed
 * picture, so the next take continues with the pictures after it).  p265fe_wait blocks until the next picture in
 * decode order is parsed (all = 0) or every submitted one is (all = 1), and returns how many are
 * ready to take. */
int  p265fe_wait(p265fe_decoder* dec, int all);
int  p265fe_pictures_get(const p265fe_pictures* set, int i, p265fe_picture_info* out);
void p265fe_pictures_free(p265fe_pictures* set);

/* Decoded picture hash (D.3.19) of one 8-bit sample plane (width x height, row stride in
 * bytes): P265FE_HASH_MD5 -> 16 bytes, _CRC -> 2 bytes big-endian, _CHECKSUM -> 4 bytes
 * big-endian, as carried by the decoded_picture_hash SEI. */
int  p265fe_plane_hash(const uint8_t* plane, int width, int height, int stride, int hash_type, uint8_t out[16]);

/* Text of the last error of this decoder ("" if none). */
const char* p265fe_last_error(p265fe_decoder* dec);
uint32_t    p265fe_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* P265FE_H */
