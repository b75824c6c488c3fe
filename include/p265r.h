/*
 * p265r.h -- C ABI of the MI355X (gfx950) HEVC intra reconstruction back-end.
 *
 * Drop-in boundary for the reconstruction hook of the p265 reference decoder.
 * The reference has no FFI: its boundary is the Python call
 *     Cu.parse -> Cu.decode_leaf()                 (decoder/cu.py:96-97, cu.py:483-494)
 * which (were it not dead, cu.py:487-488) would run, per leaf CU,
 *     Cu.decode_intra -> IntraPu.decode            (cu.py:595-615, intra.py:39-70)
 *       -> scaling.inverse_scaling                 (scaling.py:4-47)
 *       -> transform.inverse_transform             (transform.py:89-109)
 *       -> reconstruction.reconstruction           (reconstruction.py:4-27)
 * with the picture served back through Cu.get_reconstructed_sample (cu.py:617-632),
 * and the per-CTU SAO syntax of Sao.parse (sao.py:15-136) that nothing consumes.
 *
 * Here decode_leaf() only APPENDS records (one p265r_tb per transform block, one
 * p265r_ctu per CTU); at end of picture (slice.py:284-286) the host submits a batch
 * of pictures; the device runs dequant + inverse DCT/DST + intra prediction +
 * reconstruction + SAO and writes the decoded planes.  See INTEGRATION.md for the
 * ctypes binding the reference would add.
 *
 * Conventions: every function returns int (0 = P265R_OK, < 0 = error code, see
 * p265r_strerror); no exception or C++ type crosses this boundary.  All host
 * buffers are owned by the caller.  A context is bound to one device and is not
 * thread-safe: use one context per GPU per thread/process.
 */
#ifndef P265R_H
#define P265R_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define P265R_ABI_VERSION 2u   /* 2: per-picture size in p265r_picture */

/* error codes */
#define P265R_OK            0
#define P265R_EINVAL       -1   /* bad argument / malformed record              */
#define P265R_ENOMEM       -2   /* host or device allocation failed             */
#define P265R_EHIP         -3   /* HIP runtime error (see p265r_last_hip_error) */
#define P265R_EUNSUPPORTED -4   /* stream feature outside this back-end's scope */
#define P265R_ERANGE       -5   /* record points outside picture / buffers      */
#define P265R_ESTATE       -6   /* call out of order (e.g. wait without submit) */
#define P265R_ENODEV       -7   /* no such HIP device                           */

/* p265r_tb.flags */
#define P265R_TB_CBF     0x01u  /* coefficients present at coef_off (N*N int16, raster)        */
#define P265R_TB_TSKIP   0x02u  /* transform_skip_flag (tu.py:142-143)                        */
#define P265R_TB_BYPASS  0x04u  /* cu_transquant_bypass_flag (cu.py:102-105)                 */
#define P265R_TB_PCM     0x08u  /* PCM block: coef holds samples at BitDepth; no prediction    */

/* p265r_picture.flags */
#define P265R_PIC_RECON_INPUT 0x01u /* recon[] holds the reconstruction (input): residual and intra
                                       phases are skipped, only the in-loop filters run (tile halo
                                       decoding, p265_amd/tiles.py).  All pictures of a batch must
                                       agree on this flag. */

/* p265r_ctu.flags */
#define P265R_CTU_LF_ACROSS_SLICES 0x01u  /* slice_loop_filter_across_slices_enabled_flag of its slice */
#define P265R_CTU_DEBLOCK          0x02u  /* deblocking on in its slice (!slice_deblocking_filter_disabled_flag,
                                             slice.py:170-175 / pps.py:122-131); 0 = the edges this CTU's
                                             coding blocks own (left/top/internal) are not filtered     */

/* p265r_ctu.deblock_offsets: slice_beta_offset_div2 in bits 0..3, slice_tc_offset_div2 in bits
 * 4..7, each a 4-bit two's-complement value in -6..6 (inherited from pps_*_offset_div2) */
#define P265R_DEBLOCK_OFFSETS(beta_div2, tc_div2) ((uint8_t)(((beta_div2) & 15) | (((tc_div2) & 15) << 4)))

/* Sequence-level parameters (SPS/PPS-derived fields the path reads; sps.py:59-62,
 * sps.py:142-171, sps.py:120, pps.py:38, pps.py:49-50).  POD, 32 bytes: RCCL-broadcastable. */
typedef struct p265r_params {
    uint32_t version;                 /* = P265R_ABI_VERSION                      */
    uint16_t pic_width;               /* pic_width_in_luma_samples                */
    uint16_t pic_height;              /* pic_height_in_luma_samples               */
    uint8_t  chroma_format_idc;       /* 1 (4:2:0) only                           */
    uint8_t  bit_depth_luma;          /* BitDepthY: 8, or 9..12 (uint16_t planes)   */
    uint8_t  bit_depth_chroma;        /* BitDepthC: equal to bit_depth_luma        */
    uint8_t  ctb_log2_size;           /* CtbLog2SizeY, 4..6                       */
    uint8_t  min_tb_log2_size;        /* MinTbLog2SizeY, 2..5                     */
    uint8_t  max_tb_log2_size;        /* MaxTbLog2SizeY, <= 5                     */
    uint8_t  strong_intra_smoothing;  /* strong_intra_smoothing_enabled_flag      */
    uint8_t  constrained_intra_pred;  /* constrained_intra_pred_flag (no effect: all-intra) */
    uint8_t  sample_adaptive_offset;  /* sample_adaptive_offset_enabled_flag      */
    uint8_t  loop_filter_across_tiles;/* loop_filter_across_tiles_enabled_flag    */
    uint8_t  scaling_list_enabled;    /* scaling_list_enabled_flag: 1 = dequantise with the ScalingFactor
                                         table given by p265r_set_scaling_factors (sps.py:86-90,
                                         scaling.py:32-44)                          */
    int8_t   pps_cb_qp_offset;        /* cQpPicOffset of Cb chroma deblocking (8.7.2.5.5) */
    int8_t   pps_cr_qp_offset;        /* cQpPicOffset of Cr chroma deblocking     */
    uint8_t  reserved[11];
} p265r_params;

/* One CTU, raster order, PicSizeInCtbsY per picture.  32 bytes. */
typedef struct p265r_ctu {
    uint32_t tb_begin;        /* first p265r_tb of this CTU (its TBs are contiguous, decode order) */
    uint16_t tb_count;
    uint16_t tile_id;         /* TileId (tiles numbered in tile-scan order)                    */
    uint32_t slice_addr;      /* SliceAddrRs of the slice containing this CTU                  */
    uint8_t  flags;           /* P265R_CTU_*                                                   */
    uint8_t  sao_type[3];     /* SaoTypeIdx[cIdx]: 0 off, 1 band offset, 2 edge offset         */
    uint8_t  sao_class[3];    /* sao_band_position (type 1) or SaoEoClass (type 2)             */
    uint8_t  deblock_offsets; /* P265R_DEBLOCK_OFFSETS(slice_beta_offset_div2, slice_tc_offset_div2) */
    int8_t   sao_offset[3][4];/* SaoOffsetVal[cIdx][1..4]: signed, << log2OffsetScale          */
} p265r_ctu;

/* One transform block, in decode order within its CTU.  16 bytes.
 * Luma TBs of a TU precede its Cb and Cr TBs; for a luma 4x4 quad the single
 * 4x4 Cb/Cr pair follows blkIdx 3 (tu.py:127-135). */
typedef struct p265r_tb {
    uint16_t x, y;            /* top-left, in samples of component c_idx                       */
    uint8_t  log2_size;       /* 2..5                                                          */
    uint8_t  c_idx;           /* 0 Y, 1 Cb, 2 Cr                                               */
    uint8_t  pred_mode;       /* IntraPredModeY / IntraPredModeC, 0..34                        */
    uint8_t  flags;           /* P265R_TB_*                                                    */
    uint8_t  qp;              /* qP for scaling: Qp'Y or Qp'Cb / Qp'Cr (incl. QpBdOffset); luma
                                 TBs (PCM ones too) also give QpY + QpBdOffsetY to deblocking    */
    uint8_t  reserved[3];
    uint32_t coef_off;        /* int16 offset of the N*N TransCoeffLevel[y][x] (iff CBF|PCM)   */
} p265r_tb;

/* One picture of a batch (host memory, caller-owned). */
typedef struct p265r_picture {
    const p265r_ctu* ctus;    /* PicSizeInCtbsY entries, raster order                          */
    const p265r_tb*  tbs;
    uint32_t         n_tbs;
    uint32_t         flags;   /* P265R_PIC_*                                                   */
    const int16_t*   coef;
    uint64_t         n_coef;
    const uint8_t*   nofilter;/* optional (NULL): per 8x8 luma block, raster, ceil(W/8) wide;
                                 1 = deblocking and SAO leave the block's samples untouched
                                 (pcm_loop_filter_disabled && pcm, or cu_transquant_bypass)   */
    void*            out[3];  /* decoded (post-deblocking, post-SAO) planes Y, Cb, Cr; stride =
                                 plane width in samples; uint8_t samples at BitDepth 8, uint16_t
                                 at 9..12.  NULL = do not download                              */
    void*            recon[3];/* optional in-loop-filter input (reconstruction before deblocking
                                 and SAO), same layout; NULL = skip.  Written by download, or
                                 read by upload with P265R_PIC_RECON_INPUT                     */
    uint16_t         pic_width;  /* this picture's size in luma samples; 0 = the context's      */
    uint16_t         pic_height; /* (p265r_params).  A batch may mix sizes up to the context's --
                                 the uneven tiles of one picture decoded as sub-pictures (the
                                 reference's column / row widths, pps.py:152-227) run in ONE
                                 launch.  Multiples of 8; the CTU records (PicSizeInCtbsY),
                                 planes, nofilter map and TB positions are of this size          */
    uint32_t         reserved;
} p265r_picture;

/* Per-phase device time of the last run, from HIP events on the context's stream. */
typedef struct p265r_timings {
    double   total_ms;        /* first kernel start -> last kernel end                     */
    double   residual_ms;     /* dequant + inverse transform kernels                       */
    double   intra_ms;        /* intra prediction + reconstruction (all wavefront steps)   */
    double   sao_ms;          /* in-loop filter kernel (deblocking + SAO)                  */
    int32_t  intra_launches;  /* kernel launches in the intra phase                        */
    int32_t  residual_launches;
    int32_t  sao_launches;
    int32_t  reserved;
} p265r_timings;

typedef struct p265r_ctx   p265r_ctx;
typedef struct p265r_batch p265r_batch;

/* Context on HIP device `device` for a sequence with parameters `params`. */
int  p265r_create(int device, const p265r_params* params, p265r_ctx** out);
void p265r_destroy(p265r_ctx* ctx);

/* Validate the records of n_pics pictures and copy them (plus output planes) into a
 * device-resident batch.  Synchronous w.r.t. the host buffers. */
int  p265r_batch_upload(p265r_ctx* ctx, const p265r_picture* pics, int n_pics, p265r_batch** out);
/* Enqueue reconstruction + SAO of every picture of the batch on the context stream. */
int  p265r_batch_run(p265r_ctx* ctx, p265r_batch* batch);
/* Wait for the batch and copy its planes into pics[i].out / pics[i].recon; returns what
 * p265r_batch_status returns afterwards. */
int  p265r_batch_download(p265r_ctx* ctx, p265r_batch* batch, const p265r_picture* pics, int n_pics);
/* Wait for every run enqueued on the batch's stream and report whether any run of the batch
 * since its upload failed on the device: P265R_OK, or P265R_EHIP when the intra row pipeline
 * gave up a (capped) dependency wait -- its output is then incomplete (p265r_last_hip_error
 * says which).  Lets a caller that re-runs a resident batch (a benchmark) check the work it
 * timed without downloading it.  No counterpart in the reference (which cannot fail this way). */
int  p265r_batch_status(p265r_ctx* ctx, p265r_batch* batch);
/* Per-picture digest of a batch's planes after every run enqueued on it, computed on the device
 * (no plane download): which = 0 the decoded (output) planes, 1 the reconstruction before the
 * in-loop filters.  out[3 * i + c] = sum over the 4-sample words of plane c of picture i (row y,
 * word k; the picture's own width W, W/4 words per row) of mix64(word | (y * W/4 + k) << 32)
 * mod 2^64, mix64 = the splitmix64 finalizer (p265_amd/digest.py restates it on the host);
 * n = 3 * the batch's pictures.  Returns what p265r_batch_status returns afterwards.  Lets a
 * benchmark check every picture it timed.  No counterpart in the reference. */
int  p265r_batch_digest(p265r_ctx* ctx, p265r_batch* batch, int which, uint64_t* out, int n);
/* The same digest ENQUEUED on the batch's lane after every run enqueued so far, into slot `slot`
 * (0 .. P265R_DIGEST_SLOTS-1) of the batch's digest buffer; returns without waiting (the buffer is
 * allocated at the first call).  p265r_batch_digest_slots waits for the lane and copies slots
 * [0, n_slots): out[(s * n_pics + i) * 3 + c].  Lets a caller check EVERY run of a pipelined schedule,
 * not only the last (a run's output is otherwise overwritten by the batch's next run).  A slot
 * written twice holds the later digest.  No counterpart in the reference. */
#define P265R_DIGEST_SLOTS 64
int  p265r_batch_digest_async(p265r_ctx* ctx, p265r_batch* batch, int which, int slot);
int  p265r_batch_digest_slots(p265r_ctx* ctx, p265r_batch* batch, uint64_t* out, int n_slots);
/* Intra jobs of the batch's last run (after job preparation: a 4x4 quad counts once, a Cb+Cr pair
 * once), luma and chroma, summed over its pictures; waits for the batch's lane.  For measurement
 * (bench.py: the row kernel's cycles per job).  No counterpart in the reference. */
int  p265r_batch_job_count(p265r_ctx* ctx, p265r_batch* batch, uint64_t* luma, uint64_t* chroma);
int  p265r_batch_free(p265r_ctx* ctx, p265r_batch* batch);

/* Convenience: upload + run (asynchronous) ... */
int  p265r_submit(p265r_ctx* ctx, const p265r_picture* pics, int n_pics);
/* ... then block until outputs are written into the pictures given to submit. */
int  p265r_wait(p265r_ctx* ctx);

/* Block until the context's streams are idle. */
int  p265r_sync(p265r_ctx* ctx);
/* Batch pipelining (no counterpart in the reference; a throughput knob of this back-end):
 * batches uploaded afterwards are bound round-robin to `depth` (1..16) HIP streams, so the
 * residual and loop-filter phases of one batch run beside the intra phase of another (small
 * batches: whole batches side by side).  Every stream wants a hardware queue of its own: HIP's
 * default GPU_MAX_HW_QUEUES=4 serves depth <= 3 (+ the upload stream); set GPU_MAX_HW_QUEUES >=
 * depth + 1 before the process first touches HIP for deeper pipelines (min(32, 2 x depth + 2) for
 * batches of >= one picture per CU, whose prep / residual phases get streams of their own; the
 * runtime accepts at most 32, so past depth 15 such batches share hardware queues).
 * Runs of one batch stay ordered; p265r_sync waits for every stream.  Default 1. */
int  p265r_set_pipeline(p265r_ctx* ctx, int depth);
/* Scaling lists (scaling_list_enabled = 1; decoder/scaling.py:32-44, m[x][y] = ScalingFactor[sizeId]
 * [matrixId][x][y]): the intra ScalingFactor arrays, 2032 bytes, each matrix row-major m[y][x] (y the
 * row): 4x4 Y, Cb, Cr at byte 0, 16, 32; 8x8 Y, Cb, Cr at 48, 112, 176; 16x16 Y, Cb, Cr at 240, 496,
 * 752 (DC included); 32x32 Y at 1008 -- the derivation of 7.4.5 from the SPS / PPS scaling_list_data
 * (default lists included) is the caller's (libp265fe.so delivers it with every picture).  Values
 * 1..255.  Applies to every later run of the context (waits for the runs in flight first); a context
 * with scaling_list_enabled refuses to run (P265R_ESTATE) until it is set. */
#define P265R_SCALING_FACTOR_BYTES 2032
int  p265r_set_scaling_factors(p265r_ctx* ctx, const uint8_t* factors, int n_bytes);
/* Measurement knob (no counterpart in the reference): force the intra row kernel's build for this
 * context's later runs -- 8 or 12 waves per workgroup -- or 0 (default) to pick it per run (12 for a
 * batch alone, 8 beside other lanes' runs, the latency layouts for small batches).  Lets a benchmark
 * time the build its pipelined steps run, in isolation. */
int  p265r_set_row_waves(p265r_ctx* ctx, int waves);
/* Enable (1, which also starts a new accumulation) / disable (0) per-phase HIP-event
 * timing of every p265r_batch_run; read the last run's timings, or the sums over all runs
 * since enabling (runs may be queued back to back: nothing here waits per run). */
int  p265r_set_timing(p265r_ctx* ctx, int enable);
int  p265r_last_timings(p265r_ctx* ctx, p265r_timings* out);
int  p265r_timings_total(p265r_ctx* ctx, p265r_timings* out, int* n_runs);

/* Effective configuration of a context as a JSON object (intra schedule, waves per workgroup,
 * loop-filter kernel choice, pipeline depth, and which P265R_* environment knobs overrode the
 * defaults): writes at most size-1 bytes + NUL into buf, returns the full length (like snprintf)
 * or an error code.  Lets a benchmark record what it measured. */
int  p265r_describe(p265r_ctx* ctx, char* buf, int size);

/* Number of HIP devices visible (>= 0), or an error code. */
int  p265r_device_count(void);
const char* p265r_strerror(int code);
/* Text of the last HIP error seen by this library (thread-local), "" if none. */
const char* p265r_last_hip_error(void);
/* Library ABI version (P265R_ABI_VERSION). */
uint32_t p265r_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* P265R_H */
