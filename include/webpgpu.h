/*
 * webpgpu.h -- C ABI of libwebpgpu.so, the MI355X (gfx950) implementation of
 * the deepteams/webp internal/dsp hot path.
 *
 * This header is the drop-in boundary.  Every entry point is extern "C",
 * takes plain pointers / sizes, and replaces one reference interface (cited
 * as path:line relative to the reference root).  Conventions:
 *
 *  - All buffer pointers are DEVICE pointers (hipMalloc / torch CUDA tensor
 *    storage) unless the name ends in _host.  `stream` is a hipStream_t
 *    (NULL = default stream).  Calls are asynchronous on `stream`.
 *  - Return value: WG_OK (0) or a negative WG_E* status.  A HIP runtime
 *    failure is reported, never papered over: there is no CPU fallback in
 *    this library.  wg_last_error() returns a message for the calling thread.
 *  - "Batched" entry points run the reference's per-block function over n
 *    independent instances.  Instance i's buffer starts at base + i*stride.
 *  - Frame entry points take `n_images` same-sized images laid out back to
 *    back with the given per-image byte pitch (image_pitch).
 *  - Persistent kernels (wg_encode_mbs, wg_decode_frames,
 *    wg_vp8l_inverse_predictor, the gradient wg_alpha_unfilter) hand rows
 *    across workgroups and bound every wait (2 s); a wait that times out makes
 *    the *_status call fail.  Issue a first kernel on every stream before
 *    running them concurrently with other streams: the first kernel on a new
 *    stream makes the runtime create a hardware queue, which on MI355X
 *    stalled a persistent kernel already running on another queue past that
 *    bound.  A timeout is reported once, by the first *_status call of that
 *    kernel family on the device after it; later clean launches report WG_OK.
 *  - Device state (timeout records, the encoder's constant tables) belongs
 *    to the device of `stream`; the frame entry points require it to be the
 *    calling thread's current device.
 *
 * The Go-side binding a maintainer adds (cgo) is shown in INTEGRATION.md.
 */
#ifndef WEBPGPU_H
#define WEBPGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WG_OK 0
#define WG_EINVAL (-1)   /* bad argument (shape, mode, NULL) */
#define WG_EHIP (-2)     /* HIP runtime / launch failure */
#define WG_ENODEV (-3)   /* no gfx950 device */
#define WG_ENOMEM (-4)

#define WG_BPS 32 /* internal/dsp/dsp.go:5 */
/* reference work-buffer layout, internal/lossy/constants.go:70-75 */
#define WG_YUV_SIZE (WG_BPS * 17 + WG_BPS * 9)
#define WG_YOFF (WG_BPS * 1 + 8)
#define WG_UOFF (WG_YOFF + WG_BPS * 16 + WG_BPS)
#define WG_VOFF (WG_UOFF + 16)

const char* wg_last_error(void);
/* ABI version of this header; WG_ABI_VERSION when the library matches it.
 * 2: wg_alpha_unfilter_work_bytes(width, height, n) (was (height, n)). */
#define WG_ABI_VERSION 2
int wg_version(void);
/* Checks that the current device is gfx950 and the kernels are loadable. */
int wg_device_check(void);
/* Diagnostics: records one timed-out dependency wait in the device's record
 * of kernel family `family` (0 encode, 16 decode, 32 VP8L inverse, 48 alpha)
 * as a persistent kernel's timed-out wait would, so tests can check how the
 * *_status entry points report and recover.  Not used by the product path. */
int wg_debug_inject_timeout(int32_t family, void* stream);

/* ===================================================================== *
 * 1. Block-level layer: the internal/dsp function variables, batched.
 *    Each replaces the Go function variable / table named in the comment
 *    (internal/dsp/dsp.go:10-37, ssim.go:251-254).
 * ===================================================================== */

/* PredLuma4[mode](buf, off) -- predict_lossy.go:185-451, dsp.go:36.
 * For i < n: PredLuma4[modes[i]](bufs + i*buf_stride, offs ? offs[i] : off). */
int wg_pred_luma4(const uint8_t* modes, uint8_t* bufs, int64_t buf_stride, const int32_t* offs, int32_t off,
                  int32_t n, void* stream);
/* PredLuma16[mode] -- predict_lossy.go:27-102, dsp.go:34 */
int wg_pred_luma16(const uint8_t* modes, uint8_t* bufs, int64_t buf_stride, const int32_t* offs, int32_t off,
                   int32_t n, void* stream);
/* PredChroma8[mode] -- predict_lossy.go:106-181, dsp.go:35 */
int wg_pred_chroma8(const uint8_t* modes, uint8_t* bufs, int64_t buf_stride, const int32_t* offs, int32_t off,
                    int32_t n, void* stream);

/* Decoder transforms, dsp.go:18-24.  coeffs: int16[n][coeff_pitch]; dst
 * blocks at dst + i*dst_stride, BPS row stride.
 * kind: 0 Transform(doTwo=0) 1 Transform(doTwo=1) 2 TransformAC3 3 TransformDC
 *       4 TransformUV 5 TransformDCUV  (transforms.go:139-216) */
int wg_transform(int32_t kind, const int16_t* coeffs, int64_t coeff_pitch, uint8_t* dst, int64_t dst_stride,
                 int32_t n, void* stream);
/* TransformWHT (transforms.go:223): in int16[n][16] -> out int16[n][256] */
int wg_transform_wht(const int16_t* in, int16_t* out, int32_t n, void* stream);
/* FTransformWHT (transforms.go:500): in int16[n][16] (flat) -> out int16[n][16] */
int wg_ftransform_wht(const int16_t* in, int16_t* out, int32_t n, void* stream);
/* ITransform(ref, in, dst, doTwo) (transforms.go:256): ref/dst blocks at
 * +i*blk_stride (BPS rows), in int16[n][32]. */
int wg_itransform(const uint8_t* ref, const int16_t* in, uint8_t* dst, int64_t blk_stride, int32_t do_two,
                  int32_t n, void* stream);
/* FTransform / FTransform2 (transforms.go:371,487): out int16[n][16 or 32] */
int wg_ftransform(const uint8_t* src, const uint8_t* ref, int64_t blk_stride, int16_t* out, int32_t two,
                  int32_t n, void* stream);

/* MetricFunc SSE4x4/SSE16x16/TDisto4x4/TDisto16x16 (ssim.go:188-335).
 * kind: 0 SSE4x4 1 SSE16x16 2 TDisto4x4 3 TDisto16x16.  out int32[n]. */
int wg_metric(int32_t kind, const uint8_t* pix, const uint8_t* ref, int64_t blk_stride, int32_t* out,
              int32_t n, void* stream);
/* SSIMGet / SSIMGetClipped (ssim.go:116,132). xywh: int32[n][4] (xo,yo,W,H)
 * or NULL for the unclipped 7x7 window at the buffer origin.  out double[n]. */
int wg_ssim_get(const uint8_t* s1, const uint8_t* s2, int64_t buf_stride, int32_t row_stride,
                const int32_t* xywh, double* out, int32_t n, void* stream);

/* Loop filters (filter.go:93-242), applied in place to each instance buffer
 * p + i*buf_stride at `base` with row `stride`.
 * kind: 0 SimpleVFilter16 1 SimpleHFilter16 2 SimpleVFilter16i 3 SimpleHFilter16i
 *       4 VFilter16 5 HFilter16 6 VFilter16i 7 HFilter16i
 *       8 VFilter8 9 HFilter8 10 VFilter8i 11 HFilter8i (u = p, v = p + uv_delta)
 * thresh/ithresh/hev are per instance (int32[n]); ithresh/hev unused by kinds 0-3. */
int wg_filter(int32_t kind, uint8_t* p, int64_t buf_stride, int32_t base, int32_t stride, int32_t uv_delta,
              const int32_t* thresh, const int32_t* ithresh, const int32_t* hev, int32_t n, void* stream);

/* UpsampleLinePair (internal/dsp/upsample.go:45, format 0: RGB, 3 B/px) and
 * UpsampleLinePairNRGBA (upsample_direct_amd64.go:10 / upsample_direct_noasm.go,
 * format 1: NRGBA, 4 B/px; alpha rows may be NULL -> 255) over n line pairs:
 * pair i reads top_y/bot_y + i*y_step, the four chroma rows + i*uv_step, and
 * writes top_dst/bot_dst + i*dst_step (and alpha_* + i*alpha_step).  bot_y
 * NULL = the last row of an odd-height image (bot_dst unused), as in Go.
 * width >= 0; n <= 65535; NRGBA rows 4-byte aligned. */
int wg_upsample_line_pairs(int32_t format, const uint8_t* top_y, const uint8_t* bot_y, int64_t y_step,
                           const uint8_t* top_u, const uint8_t* top_v, const uint8_t* bot_u, const uint8_t* bot_v,
                           int64_t uv_step, uint8_t* top_dst, uint8_t* bot_dst, int64_t dst_step,
                           const uint8_t* alpha_top, const uint8_t* alpha_bot, int64_t alpha_step, int32_t width,
                           int32_t n, void* stream);

/* PointSampleRow(y, u, v, dst, width) (internal/dsp/upsample.go:238-245) over
 * n rows: y + i*y_step, u/v + i*uv_step (chroma sample x>>1 per pixel), RGB
 * (3 B/px) to dst + i*dst_step.  n <= 65535. */
int wg_point_sample_rows(const uint8_t* y, const uint8_t* u, const uint8_t* v, int64_t y_step, int64_t uv_step,
                         uint8_t* dst, int64_t dst_step, int32_t width, int32_t n, void* stream);

/* ConvertARGBToY(argb, y, width) (internal/dsp/yuv.go:270-278) over n rows:
 * packed 0xAARRGGBB words at argb + i*argb_pitch (elements), Y bytes at
 * y + i*y_pitch.  n <= 65535. */
int wg_convert_argb_to_y(const uint32_t* argb, int64_t argb_pitch, uint8_t* y, int64_t y_pitch, int32_t width,
                         int32_t n, void* stream);
/* ConvertARGBToUV(argb, u, v, srcWidth, doStore) (yuv.go:291-330) over n
 * rows: (src_width + 1) / 2 U and V samples at u/v + i*uv_pitch; do_store 0
 * averages each into the sample already there, as the Go call does. */
int wg_convert_argb_to_uv(const uint32_t* argb, int64_t argb_pitch, uint8_t* u, uint8_t* v, int64_t uv_pitch,
                          int32_t src_width, int32_t do_store, int32_t n, void* stream);

/* AccumulateRGBA(r, g, b, a, stride, dst, width) (internal/dsp/yuv.go:486-547)
 * over n row pairs: planar channel rows at r/g/b/a + i*in_pitch (second row
 * at +stride), dst uint16 (R, G, B, A) quads at dst + i*dst_pitch (elements).
 * n <= 65535. */
int wg_accumulate_rgba(const uint8_t* r, const uint8_t* g, const uint8_t* b, const uint8_t* a, int32_t stride,
                       int64_t in_pitch, uint16_t* dst, int64_t dst_pitch, int32_t width, int32_t n, void* stream);
/* ConvertRGBA32ToUV(rgb, u, v, width) (yuv.go:553) over n rows: rgb uint16
 * quads at rgb + i*rgb_pitch (elements), u/v + i*uv_pitch.  n <= 65535. */
int wg_convert_rgba32_to_uv(const uint16_t* rgb, int64_t rgb_pitch, uint8_t* u, uint8_t* v, int64_t uv_pitch,
                            int32_t width, int32_t n, void* stream);
/* VP8Random (internal/dsp/random.go:17-21): the generator state a dithered
 * conversion advances.  232 bytes. */
typedef struct wg_random {
  int32_t index1, index2;
  uint32_t tab[55];
  int32_t amp;
} wg_random;
/* InitRandom(rg, dithering) (random.go:39-52), host memory */
void wg_random_init_host(wg_random* rg, float dithering);
/* ConvertRGBA32ToUVDithered(rgb, u, v, width, rg) (yuv.go:568-576) over n
 * rows, row i with its own generator state[i] (device), advanced in place
 * exactly as the Go call advances rg (two RandomBits(18) draws per pixel). */
int wg_convert_rgba32_to_uv_dithered(const uint16_t* rgb, int64_t rgb_pitch, uint8_t* u, uint8_t* v, int64_t uv_pitch,
                                     int32_t width, wg_random* state, int32_t n, void* stream);

/* SSE(pix, ref, width, height, pixStride, refStride) (ssim.go:172) over n
 * blocks at pix + i*pix_pitch / ref + i*ref_pitch: out uint64[n]. n <= 65535. */
int wg_sse_planes(const uint8_t* pix, const uint8_t* ref, int32_t width, int32_t height, int32_t pix_stride,
                  int32_t ref_stride, int64_t pix_pitch, int64_t ref_pitch, uint64_t* out, int32_t n, void* stream);
/* PSNRFromSSE(sse, count) (ssim.go:163): out double[n] (Go's math.Log10). */
int wg_psnr_from_sse(const uint64_t* sse, const int64_t* count, double* out, int32_t n, void* stream);
/* DistoStats (ssim.go:12-17), Go's uint32 fields (wrapping sums). */
typedef struct wg_disto_stats {
  uint32_t w, xm, ym, xxm, xym, yym;
} wg_disto_stats;
/* The DistoStats SSIMFromBlocks accumulates (Accumulate per pixel,
 * ssim.go:19-27, :103-112) over n blocks: out[n]. n <= 65535. */
int wg_disto_stats_blocks(const uint8_t* pix, const uint8_t* ref, int32_t width, int32_t height, int32_t pix_stride,
                          int32_t ref_stride, int64_t pix_pitch, int64_t ref_pitch, wg_disto_stats* out, int32_t n,
                          void* stream);
/* SSIMFromStats (ssim.go:88, clipped = 0) / SSIMFromStatsClipped (:97,
 * clipped = 1) of n stats: out double[n]. */
int wg_ssim_from_stats(const wg_disto_stats* stats, int32_t clipped, double* out, int32_t n, void* stream);

/* ===================================================================== *
 * 2. Frame layer: the reference's row/frame seams.
 * ===================================================================== */

/* Parsed macroblock (mirrors MBData internal/lossy/decode.go:115-126 and
 * FInfo :107-112).  32 bytes.  Coefficients travel separately as
 * int16[n_mb][384] (Coeffs, already dequantised, I16 DC already WHT'd). */
typedef struct wg_mb_info {
  uint32_t non_zero_y;  /* 2-bit nz code per luma block, block 0 in bits 31..30 */
  uint32_t non_zero_uv; /* U codes in bits 0..7, V in bits 8..15 */
  uint8_t imodes[16];   /* I16: imodes[0]; I4: 16 sub-block modes, raster order */
  uint8_t is_i4x4;
  uint8_t uv_mode;
  uint8_t skip;
  uint8_t segment;
  uint8_t f_limit;      /* FInfo.FLimit; 0 disables filtering of this MB */
  uint8_t f_ilevel;
  uint8_t f_inner;
  uint8_t hev_thresh;
} wg_mb_info;

/* Decoder reconstruct + loop filter for whole frames: replaces the
 * reconstructRow / filterRowAt calls of parseFrame
 * (internal/lossy/decode.go:532-560, decode_frame.go:83-342).
 * Output planes: Y stride 16*mbw (16*mbh rows), U/V stride 8*mbw, like the
 * decoder caches (decode.go:441-530).  filter_type: 0 none, 1 simple, 2 normal.
 * `work` is scratch of wg_decode_work_bytes(mbw, mbh, n_images) bytes. */
size_t wg_decode_work_bytes(int32_t mbw, int32_t mbh, int32_t n_images);
int wg_decode_frames(const wg_mb_info* mb, const int16_t* coeffs, int32_t filter_type, int32_t mbw, int32_t mbh,
                     int32_t n_images, uint8_t* y, uint8_t* u, uint8_t* v, void* work, void* stream);
/* Which kernel wg_decode_frames launches for a batch of n_images frames of
 * mbh macroblock rows on the current device: 1 = k_decode_split (two waves a
 * row; few rows), 2 = k_decode_bands (one wave a row; batches past twice the
 * resident split rows), or a negative error code.  No reference counterpart:
 * a query for reports (bench.py labels its decode roofline with it). */
int wg_decode_kernel(int32_t mbh, int32_t n_images);

/* VP8 bitstream parse (HOST memory in and out; no device work): the CPU
 * half of the reference's decoder as a parse-all-rows-first pass that feeds
 * wg_decode_frames.  Replaces the parsing in DecodeFrame / parseFrame
 * (internal/lossy/decode.go:207-560: parseHeaders, parseIntraModeRow
 * decode_tree.go:35, decodeMB / parseResiduals decode_mb.go:272-430,
 * precomputeFilterStrengths decode_frame.go:220).  `data` is a RIFF/WEBP
 * file with a "VP8 " chunk, or a raw VP8 key frame.  dims[5] receives
 * width, height, filter_type, mbw, mbh.  With mb == NULL only the headers
 * are parsed; otherwise mb[mbw*mbh] and coeffs[mbw*mbh][384] (dequantised,
 * I16 DCs already inverse-WHT'd, as the decoder stores them) are filled. */
int wg_vp8_parse(const uint8_t* data, size_t size, int32_t* dims, wg_mb_info* mb, int16_t* coeffs,
                 int64_t max_mbs);

/* Encoder macroblock RD loop: Phase A of encodeFrameParallel
 * (internal/lossy/encode_parallel.go:168-1495; encodeRow :252-338), methods
 * 3-6: methods 4-6 run the same Phase A (trellis quantisation in the I4 RD
 * and the final I16 residuals, :793, :1202), method 3 quantises plainly
 * there (pickBestI4ModeRDParallel :842-929).  Methods 0-2 return WG_EINVAL
 * (encode.go:1356 encodes them with the serial encodeFrame).
 * Frames with mbh < 4 (height <= 48) return WG_EINVAL: EncodeFrame
 * (internal/lossy/encode.go:1356) encodes those with the serial encodeFrame.
 * out / work must be 16-byte aligned, the planes 4-byte aligned.
 * y/u/v: the encoder's padded planes (importImage output: Y stride 16*mbw,
 * U/V 8*mbw), pitches per image.  segments: per-MB segment id (NULL = all 0).
 * segs: 4 x wg_segment per image (device, 16-byte aligned), segs_pitch bytes
 * apart (0: the same 4 for every image; wg_segment_analysis writes them).  proba: the 4x8x3x11 coefficient
 * probabilities Phase A prices tokens with (device; ResetProba gives
 * CoeffsProba0).  out: n_images*mbw*mbh wg_mb_enc.  ry/ru/rv receive the
 * reconstruction (exportParallel writes it over the source planes; passing
 * the source pointers does the same).  work: wg_encode_work_bytes(). */
typedef struct wg_squant {  /* SegmentQuant, internal/lossy/encode.go:311-323 */
  int32_t quant, iquant, bias, zthresh;
  int32_t dc_quant, dc_iquant, dc_bias, dc_zthresh;
  int16_t sharpen[16];
} wg_squant;
typedef struct wg_segment { /* SegmentInfo fields Phase A reads, encode.go:278-309 */
  wg_squant y1, y2, uv;
  int32_t lambda_i4, lambda_i16, lambda_uv, lambda_mode;
  int32_t tlambda_i4, tlambda_i16, tlambda_uv, tlambda_sd;
} wg_segment;
typedef struct wg_mb_enc {  /* MBEncInfo, encode.go:241-276 (Phase A outputs) */
  int16_t coeffs[400];      /* levels: 16 Y, 4 U, 4 V blocks (raster), then the I16 WHT block */
  uint8_t modes[16];        /* I4 modes */
  uint8_t nz_y[16];         /* zigzag nz count per block */
  uint8_t nz_uv[8];
  uint32_t non_zero_y;      /* bit b: Y block b non-zero; bit 24: WHT block */
  uint32_t non_zero_uv;
  uint8_t mb_type;          /* 0 I16, 1 I4 */
  uint8_t i16_mode, uv_mode, nz_dc, skip, segment, pad0, pad1;
  uint64_t score;
} wg_mb_enc;
/* setupSegment (encode.go:1085-1181) for quantiser index q and the frame's
 * dq deltas {y1_dc, y2_dc, y2_ac, uv_dc, uv_ac}; host memory. */
int wg_setup_segment(int32_t q, const int32_t* dq5, int32_t method, int32_t sns_strength, wg_segment* out);
/* Encoder configuration the analysis reads: the EncodeConfig fields of
 * internal/lossy/encode.go:30-63 (DefaultConfig(75) :66-86 = quality 75,
 * method 4, sns 50, filter strength 60, sharpness 0, type 1, 4 segments,
 * preprocessing 0).  seg_quant[a + 127] is setSegmentParams' quantiser for a
 * segment alpha a in [-127, 127] (encode_analysis.go:128-142, the one
 * floating-point step, built on the host by wg_encoder_config). */
typedef struct wg_enc_config {
  int32_t quality, method, sns_strength, filter_strength, filter_sharpness, filter_type, segments, preprocessing;
  uint8_t seg_quant[256];
} wg_enc_config;
int wg_encoder_config(int32_t quality, int32_t method, int32_t sns_strength, int32_t filter_strength,
                      int32_t filter_sharpness, int32_t filter_type, int32_t segments, int32_t preprocessing,
                      wg_enc_config* out);
/* Per image, what analysis() and setSegmentProbas leave for Phase A / B and
 * the segment header (encode_analysis.go:29-73, :852-903). */
typedef struct wg_frame_segs {
  int32_t num_segments;   /* after simplifySegments */
  int32_t base_quant;     /* dqm[0].Quant */
  int32_t global_uv_alpha;
  int32_t dq_uv_ac, dq_uv_dc;
  int32_t filter_level;   /* filterHdr.Level */
  int32_t update_map;     /* segmentHdr.UpdateMap after setSegmentProbas */
  int32_t pad;
  int32_t quant[4], fstrength[4], alpha[4], beta[4];
  uint8_t seg_proba[4];   /* proba.Segments[0..2] */
  int32_t pad2[3];
} wg_frame_segs;          /* 112 bytes */
/* Segment analysis after computeAlphas, on the device, per image: assignSegments
 * (encode_analysis.go:737-849, smoothSegmentMap :76-119), setSegmentParams
 * (:122-195: per-segment quantiser, dq_uv deltas, setupFilterStrength
 * encode.go:1276, simplifySegments :197), setSegmentProbas' map reset
 * (:874-903) and setupSegment (encode.go:1084) for all 4 segments.
 * cfg: HOST pointer.  alphas [n][mbw*mbh], uv_sum [n] as wg_analysis_alphas
 * writes them.  Outputs seg_ids [n][mbw*mbh], segs (4 wg_segment per image,
 * segs_pitch bytes apart, 16-byte aligned) for wg_encode_mbs, and info [n]
 * (may be NULL). */
int wg_segment_analysis(const wg_enc_config* cfg, const int32_t* alphas, const int32_t* uv_sum, int32_t mbw,
                        int32_t mbh, int32_t n_images, uint8_t* seg_ids, void* segs, int64_t segs_pitch,
                        wg_frame_segs* info, void* stream);
size_t wg_encode_work_bytes(int32_t mbw, int32_t mbh, int32_t n_images);
/* Phase A of encodeFrameParallel (encode_parallel.go:168-232) for n frames of
 * one size: y / u / v planes [n] at y_pitch / uv_pitch bytes apart, rows
 * 16*mbw / 8*mbw bytes (the reference's padded layout); y and ry 16-byte
 * aligned with y_pitch a multiple of 16, u, v, ru, rv 8-byte aligned with
 * uv_pitch a multiple of 8; out (wg_mb_enc [n][mbh][mbw]) and work 16-byte
 * aligned.  Methods 3-6, mbh >= 4 (else WG_EINVAL).  Launches whose rows fit
 * the device's wave slots twice walk each row with a wave pair (I4 RD beside
 * the I16 / chroma work), larger ones with one wave a row; the outputs are the
 * same (environment WG_ENCODE_PAIR=0 / 1 forces either schedule). */
int wg_encode_mbs(const uint8_t* y, const uint8_t* u, const uint8_t* v, int64_t y_pitch, int64_t uv_pitch,
                  int32_t width, int32_t height, int32_t n_images, const uint8_t* segments, const void* segs,
                  int64_t segs_pitch, const uint8_t* proba, int32_t method, int32_t quality, void* out, uint8_t* ry, uint8_t* ru,
                  uint8_t* rv, void* work, void* stream);
/* The row schedule of wg_encode_mbs for a batch, from computeAlphas' per-MB
 * alphas [n_images][mbw*mbh] (device): the rows of frames with textured
 * macroblocks (low mean alpha; the slow ones, whose wavefront ends the
 * launch) are dequeued up to mbh/4 rows ahead of the others.  Written into
 * `work` (wg_encode_work_bytes; kept across wg_encode_mbs calls on the same
 * work and row count, until the next wg_encode_row_order); without it the
 * rows go in (row, frame) order.  Scheduling only: the outputs are the same. */
int wg_encode_row_order(const int32_t* alphas, int32_t mbw, int32_t mbh, int32_t n_images, void* work, void* stream);
/* After wg_encode_mbs on the same stream: WG_OK, or WG_EHIP if a row wait of
 * the last launch on `work` -- or of any encoder launch since the library
 * loaded (a device-wide count that is never reset) -- timed out.  Synchronises. */
int wg_encode_status(const void* work, int32_t mbw, int32_t n_images, void* stream);
/* The multi-device batch variant of the encode DSP path (one host process
 * driving several GPUs, as a cgo host would): n_images RGBA frames (w x h,
 * tightly packed, n_images * w * h * 4 bytes of HOST memory); frame i is
 * encoded on devices[i % n_devices] (an entry may repeat a device: each
 * entry gets its own stream and buffers), each device
 * running wg_import_rgba -> wg_analysis_alphas -> wg_segment_analysis (cfg,
 * host) -> wg_encode_mbs over its frames on its own stream, with the default
 * token probabilities (CoeffsProba0).  The outputs are gathered into HOST
 * buffers in frame order: mb_out wg_mb_enc [n][mbh*mbw]; ry [n][16*mbh][16*mbw],
 * ru / rv [n][8*mbh][8*mbw], seg_ids [n][mbh*mbw], info [n] (each may be NULL
 * but mb_out).  Replaces the per-frame EncodeFrame calls up to Phase A
 * (internal/lossy/encode.go:1324-1366) for a batch of independent frames
 * (C4); blocks until every device is done.  WG_EINVAL for mbh < 4. */
int wg_encode_frames_devices(const int32_t* devices, int32_t n_devices, const uint8_t* rgba, int32_t w, int32_t h,
                             int32_t n_images, int32_t has_alpha, const wg_enc_config* cfg, void* mb_out, uint8_t* ry,
                             uint8_t* ru, uint8_t* rv, uint8_t* seg_ids, wg_frame_segs* info);
/* VP8FixedCostsI4[top][left][mode] (encode_analysis.go:1498-1520) as
 * uploaded by wg_encode_mbs; host memory, 1000 uint16. */
int wg_fixed_costs_i4_host(uint16_t* out);

/* After wg_decode_frames on the same stream: WG_OK, or WG_EHIP if a row
 * dependency wait of the last launch on `work`, or of any decoder launch since
 * the library loaded, timed out inside the kernel (output invalid).
 * Synchronises the stream. */
int wg_decode_status(const void* work, int32_t mbw, int32_t n_images, void* stream);

/* RGBA -> YUV420 import: replaces VP8Encoder.importImage
 * (internal/lossy/encode.go:671-943, non-dithered path; dithered below).  rgba: w x h, row
 * pitch `stride`, image pitch rgba_pitch.  Outputs padded planes (Y stride
 * 16*mbw, U/V stride 8*mbw) with per-image pitches y_pitch / uv_pitch. */
int wg_import_rgba(const uint8_t* rgba, int32_t w, int32_t h, int32_t stride, int64_t rgba_pitch,
                   int32_t has_alpha, uint8_t* y, uint8_t* u, uint8_t* v, int64_t y_pitch, int64_t uv_pitch,
                   int32_t n_images, void* stream);

/* Dithered import (webp.Encode Preprocessing bit 1): importImage's dithered
 * path (internal/lossy/encode.go:690-695, :793-809, :903-940:
 * RGBToYRounding with RandomBits(16) over every padded pixel, then
 * ConvertRGBA32ToUVDithered with RandomBits(18) for U and V,
 * internal/dsp/yuv.go:568-576).  The VP8Random stream (random.go) is the same
 * for every image of a padded size, so it is built once into `plan`
 * (wg_dither_plan_bytes device bytes, 16-byte aligned; wg_dither_plan builds
 * it on the host, copies it and synchronises `stream`).  amp: the generator's
 * amplitude, wg_dither_amp(quality, preprocessing) for webp.Encode's options
 * (encode.go (root):517-521, InitRandom random.go:39). */
int32_t wg_dither_amp(float quality, int32_t preprocessing);
size_t wg_dither_plan_bytes(int32_t w, int32_t h);
int wg_dither_plan(int32_t w, int32_t h, void* plan, void* stream);
/* the same plan in host memory (no device work; tests) */
int wg_dither_plan_host(int32_t w, int32_t h, void* plan_host);
int wg_import_rgba_dithered(const uint8_t* rgba, int32_t w, int32_t h, int32_t stride, int64_t rgba_pitch,
                            int32_t has_alpha, int32_t amp, const void* plan, uint8_t* y, uint8_t* u, uint8_t* v,
                            int64_t y_pitch, int64_t uv_pitch, int32_t n_images, void* stream);

/* Encoder analysis: replaces computeAlphas (internal/lossy/encode_analysis.go:245-307).
 * Outputs per MB: alphas (mixed), lum/uv parts (may be NULL); uv_sum[img] is
 * the sum of uv alphas (the reference's return value = uv_sum / nMB). */
int wg_analysis_alphas(const uint8_t* y, const uint8_t* u, const uint8_t* v, int32_t w, int32_t h,
                       int64_t y_pitch, int64_t uv_pitch, int32_t n_images, int32_t* alphas, int32_t* lum,
                       int32_t* uva, int32_t* uv_sum, void* stream);

/* Fancy upsampling YUV420 -> NRGBA: replaces buildNRGBA (webp.go:379-450)
 * -> dsp.UpsampleLinePairNRGBA (upsample_direct_amd64.go:10).  alpha may be
 * NULL (A = 255) else w x h plane with pitch a_pitch per image.
 * out: h rows of 4*w bytes, out_pitch per image. */
int wg_upsample_nrgba(const uint8_t* y, int32_t y_stride, int64_t y_pitch, const uint8_t* u, const uint8_t* v,
                      int32_t uv_stride, int64_t uv_pitch, const uint8_t* alpha, int64_t a_pitch, int32_t w,
                      int32_t h, uint8_t* out, int64_t out_pitch, int32_t n_images, void* stream);

/* Plane SSIM (libwebp AccumulateSSIM built from SSIMGet/SSIMGetClipped,
 * ssim.go:116-160): out[img] = sum over pixels of the clipped-window SSIM.
 * `work` needs wg_plane_ssim_work_bytes(w, h, n_images) bytes. */
size_t wg_plane_ssim_work_bytes(int32_t w, int32_t h, int32_t n_images);
/* Partial sums per 16-row tile row of a w-wide plane (one per 58-column
 * strip): the layout of wg_plane_ssim_rows' output. */
int32_t wg_plane_ssim_row_partials(int32_t w);
int wg_plane_ssim(const uint8_t* a, int32_t a_stride, int64_t a_pitch, const uint8_t* b, int32_t b_stride,
                  int64_t b_pitch, int32_t w, int32_t h, int32_t n_images, double* out, void* work,
                  void* stream);

/* Row-band form for sharding one large plane over GPUs (SSIM
 * shards by row bands with a 3-row halo).  Tile rows [ty_begin, ty_end) of
 * 16 pixel rows each; a and b must hold rows 16*ty_begin - 3 .. 16*ty_end + 2
 * (clipped to the plane) at their full-plane positions.  partial receives
 * wg_plane_ssim_row_partials(w) * (ty_end - ty_begin) doubles per image
 * (image-major, tile-row-major).  The
 * bands' partials concatenated in tile-row order and passed to
 * wg_plane_ssim_reduce give exactly wg_plane_ssim's sum. */
int wg_plane_ssim_rows(const uint8_t* a, int32_t a_stride, int64_t a_pitch, const uint8_t* b, int32_t b_stride,
                       int64_t b_pitch, int32_t w, int32_t h, int32_t ty_begin, int32_t ty_end, int32_t n_images,
                       double* partial, void* stream);
/* Plane SSIM of one large pair over several devices (C5, from one host
 * process): 16-row tile bands, device k computing band k from its rows plus
 * 3 halo rows each side (wg_plane_ssim_rows); the per-tile partial sums are
 * gathered and reduced on the first device in the one-device order, so *out
 * (HOST) equals wg_plane_ssim's sum bit for bit.  a, b: HOST planes. */
int wg_plane_ssim_devices(const int32_t* devices, int32_t n_devices, const uint8_t* a, int32_t a_stride,
                          const uint8_t* b, int32_t b_stride, int32_t w, int32_t h, double* out);
/* out[img] = the fixed-order sum of partial[img][0 .. per_image) */
int wg_plane_ssim_reduce(const double* partial, int64_t per_image, int32_t n_images, double* out, void* stream);

/* ===================================================================== *
 * 3. VP8L (lossless) predictor transform.
 *    ARGB images are uint32 [n_images][image_pitch] (width*height used),
 *    one 0xAARRGGBB word per pixel like the reference's []uint32.
 * ===================================================================== */

/* lossless.ResidualImage (internal/lossless/encode_predictor.go:378-455):
 * per 2^bits tile the predictor with the lowest entropy estimate among the
 * first 4 / 8 / 14 (quality <25 / <50 / else), written as mode<<8|0xff000000
 * to modes[n_images][tiles_y*tiles_x]; residuals[n_images][image_pitch] =
 * ARGB -mod prediction from the original pixels.  bits in [2, 9]. */
int wg_vp8l_residual_image(const uint32_t* argb, int32_t width, int32_t height, int64_t image_pitch,
                           int32_t bits, int32_t quality, int32_t n_images, uint32_t* modes, uint32_t* residuals,
                           void* stream);
/* Row-band form for sharding one large image over GPUs (the
 * residual shards by tile rows with a 1-row halo): only tile rows
 * [ty_begin, ty_end) (2^bits pixel rows each) are selected and their pixel
 * rows' residuals written, at their full-image positions in modes and
 * residuals.  argb must hold pixel rows (ty_begin << bits) - 1 ..
 * min(ty_end << bits, height) - 1. */
int wg_vp8l_residual_image_rows(const uint32_t* argb, int32_t width, int32_t height, int64_t image_pitch,
                                int32_t bits, int32_t quality, int32_t ty_begin, int32_t ty_end, int32_t n_images,
                                uint32_t* modes, uint32_t* residuals, void* stream);
/* One large image over several devices (C5), from one host
 * process: device k of n_devices takes the contiguous tile-row band k (the
 * first tiles % n devices one row more) and computes it through
 * wg_vp8l_residual_image_rows from its rows plus the row above; modes
 * [tiles_y*tiles_x] and residuals [height*width] land in HOST memory at
 * their places, identical to wg_vp8l_residual_image.  argb: HOST, width *
 * height words.  Blocks until done. */
int wg_vp8l_residual_image_devices(const int32_t* devices, int32_t n_devices, const uint32_t* argb, int32_t width,
                                   int32_t height, int32_t bits, int32_t quality, uint32_t* modes, uint32_t* residuals);
/* predictorInverseTransform (internal/lossless/decode_transform.go:202-360):
 * out = residuals +mod prediction from reconstructed pixels.  `work` needs
 * wg_vp8l_inverse_work_bytes(width, height, n_images) bytes, 16-B aligned (the
 * band-to-band hand-off of each band's last row). */
size_t wg_vp8l_inverse_work_bytes(int32_t width, int32_t height, int32_t n_images);
int wg_vp8l_inverse_predictor(const uint32_t* modes, int32_t bits, int32_t width, int32_t height,
                              int64_t image_pitch, int32_t n_images, const uint32_t* residuals, uint32_t* out,
                              void* work, void* stream);
/* After wg_vp8l_inverse_predictor on the same stream: WG_OK or WG_EHIP if a
 * band wait timed out.  Synchronises the stream. */
int wg_vp8l_inverse_status(const void* work, void* stream);
/* SubtractGreen (encode_predictor.go:461) when add == 0, AddGreenToBlueAndRed
 * (dsp/lossless_dsp.go:12) when add != 0; in place over n pixels. */
int wg_vp8l_green(uint32_t* argb, int64_t n, int32_t add, void* stream);
/* The fastSLog2 table (encode_histogram.go:359-368) the selection uses, host copy. */
int wg_vp8l_slog2_lut_host(double* out, int32_t n);

/* ColorSpaceTransform (internal/lossless/encode_predictor.go:727-770): per
 * 2^bits tile the green->red, green->blue and red->blue multipliers
 * (findBestMultipliers :514-585), written as g2r | g2b << 8 | r2b << 16
 * (packMultipliers :489) to data[n_images][tiles_y*tiles_x], and the forward
 * transform applied to argb IN PLACE.  bits in [2, 9]. */
int wg_vp8l_color_space_transform(uint32_t* argb, int32_t width, int32_t height, int64_t image_pitch, int32_t bits,
                                  int32_t n_images, uint32_t* data, void* stream);
/* colorSpaceInverseTransform (internal/lossless/decode_transform.go:454-520). */
int wg_vp8l_color_space_inverse(const uint32_t* data, int32_t bits, int32_t width, int32_t height, int64_t image_pitch,
                                int32_t n_images, const uint32_t* src, uint32_t* dst, void* stream);
/* colorIndexInverseTransform (internal/lossless/decode_transform.go:560-612):
 * src rows hold (width + 2^xbits - 1) >> xbits packed index words (index in
 * the green byte, 8 >> xbits bits per pixel), palette (<= 256 entries, shared
 * by the n images); indices past the palette leave dst untouched. */
int wg_vp8l_color_index_inverse(const uint32_t* palette, int32_t palette_size, int32_t xbits, int32_t width,
                                int32_t height, int32_t n_images, const uint32_t* src, int64_t src_pitch, uint32_t* dst,
                                int64_t dst_pitch, void* stream);

/* ===================================================================== *
 * 3c. Alpha plane: the ALPH filters of
 *     internal/lossy/alpha.go and the alpha processing of
 *     internal/dsp/alpha_proc.go.  Alpha planes are w x h bytes, row stride w,
 *     images `pitch` bytes apart.  filter: 0 none, 1 horizontal, 2 vertical,
 *     3 gradient (AlphaFilter* constants).
 * ===================================================================== */

/* alphaFilterHorizontal / Vertical / Gradient (alpha.go:387-454); filter 0
 * copies.  in and out must not alias. */
int wg_alpha_filter(int32_t filter, const uint8_t* in, uint8_t* out, int32_t width, int32_t height, int64_t pitch,
                    int32_t n_images, void* stream);

/* alphaUnfilterHorizontal / Vertical / Gradient (alpha.go:128-203), in place.
 * work: wg_alpha_unfilter_work_bytes(width, height, n_images) device bytes,
 * 16-B aligned (gradient only: band dequeue, progress counters and the bands'
 * hand-off rows; zeroed by the call). */
size_t wg_alpha_unfilter_work_bytes(int32_t width, int32_t height, int32_t n_images);
int wg_alpha_unfilter(int32_t filter, uint8_t* data, int32_t width, int32_t height, int64_t pitch, int32_t n_images,
                      void* work, void* stream);
/* synchronises `stream`; WG_EHIP if a gradient band wait timed out */
int wg_alpha_unfilter_status(const void* work, void* stream);

/* estimateBestFilter (alpha.go:321-385) and getNumColors (:302-317) per image:
 * best_filter[n], num_colors[n] (device int32).  work:
 * wg_alpha_estimate_work_bytes(n_images) device bytes. */
size_t wg_alpha_estimate_work_bytes(int32_t n_images);
int wg_alpha_estimate_filter(const uint8_t* data, int32_t width, int32_t height, int64_t pitch, int32_t n_images,
                             int32_t* best_filter, int32_t* num_colors, void* work, void* stream);

/* ApplyAlphaMultiply (alpha_proc.go:74-104): 4-byte pixels, alpha at byte 0
 * (alpha_first) or 3; rows `stride` bytes apart; images `pitch` apart. */
int wg_apply_alpha_multiply(uint8_t* rgba, int32_t alpha_first, int32_t width, int32_t height, int32_t stride,
                            int64_t pitch, int32_t n_images, int32_t inverse, void* stream);
/* MultARGBRow (alpha_proc.go:28-46) over n words */
int wg_mult_argb(uint32_t* argb, int64_t n, int32_t inverse, void* stream);
/* ApplyAlphaMultiply4444 (alpha_proc.go:106-135): 2-byte RGBA4444 pixels */
int wg_apply_alpha_multiply_4444(uint8_t* data, int32_t width, int32_t height, int32_t stride, int64_t pitch,
                                 int32_t n_images, void* stream);
/* DispatchAlpha (alpha_proc.go:140-155): *has_transparency (device int32)
 * = 1 when any alpha != 0xff (the Go bool result) */
int wg_dispatch_alpha(const uint8_t* alpha, int32_t alpha_stride, int32_t width, int32_t height, uint8_t* dst,
                      int32_t dst_stride, int32_t alpha_off, int32_t* has_transparency, void* stream);
/* ExtractAlpha (alpha_proc.go:158-176): *all_opaque (device int32) = 1 when
 * every alpha is 0xff (the Go int result) */
int wg_extract_alpha(const uint8_t* src, int32_t src_stride, int32_t width, int32_t height, uint8_t* alpha,
                     int32_t alpha_stride, int32_t alpha_off, int32_t* all_opaque, void* stream);
/* HasAlpha8b (step 1) / HasAlpha32b (step 4) (alpha_proc.go:178-197):
 * *any_transparent (device int32) = the Go bool */
int wg_has_alpha(const uint8_t* src, int64_t length, int32_t step, int32_t* any_transparent, void* stream);
/* AlphaReplace (alpha_proc.go:199-206) */
int wg_alpha_replace(uint32_t* argb, int64_t length, uint32_t color, void* stream);
/* DispatchAlphaToGreen (alpha_proc.go:209-219); dst_stride in pixels */
int wg_dispatch_alpha_to_green(const uint8_t* alpha, int32_t alpha_stride, int32_t width, int32_t height,
                               uint32_t* dst, int32_t dst_stride, void* stream);
/* ExtractGreen (alpha_proc.go:221-226) */
int wg_extract_green(const uint32_t* argb, uint8_t* alpha, int64_t size, void* stream);
/* PackRGB (alpha_proc.go:229-238) */
int wg_pack_rgb(const uint8_t* r, const uint8_t* g, const uint8_t* b, int64_t length, int32_t step, uint32_t* out,
                void* stream);

/* ===================================================================== *
 * 3d. Row rescaler: internal/dsp/rescale.go's Rescaler
 *     (RescalerInit :63, RescalerImportRow :110, RescalerExportRow :185),
 *     driven over whole planes: import a source row while RescalerNeedsSrcRow,
 *     else export a destination row, until dst_height rows are out or the
 *     source is exhausted.  The Go arithmetic is kept as written (it is not
 *     libwebp's: no x_add-1 adjustment, FYScale only when expanding), so for
 *     some sizes fewer than dst_height rows come out; `rows` reports how many.
 * ===================================================================== */

/* device bytes of a plan for dst_width x dst_height */
size_t wg_rescaler_plan_bytes(int32_t dst_width, int32_t dst_height);
/* Builds the plan (the size-only walk of the Go state machine) on the host
 * and copies it into `plan` (device memory) on `stream`, synchronising it;
 * *rows (host) = destination rows the driver writes. */
int wg_rescaler_plan(int32_t src_width, int32_t src_height, int32_t dst_width, int32_t dst_height, void* plan,
                     int32_t* rows, void* stream);
/* the same plan into host memory (no device work; for inspection and tests).
 * Layout: a 64-byte header, 32 bytes per destination column, 16 per row. */
int wg_rescaler_plan_host(int32_t src_width, int32_t src_height, int32_t dst_width, int32_t dst_height,
                          void* plan_host, int32_t* rows);
/* Rescales n_images planes (images src_pitch / dst_pitch bytes apart) with a
 * plan built for these sizes; rows and dst_width as returned / planned. */
int wg_rescale(const void* plan, int32_t dst_width, int32_t rows, const uint8_t* src, int64_t src_stride,
               int64_t src_pitch, uint8_t* dst, int64_t dst_stride, int64_t dst_pitch, int32_t n_images, void* stream);

/* ===================================================================== *
 * 4. SharpYUV: sharpyuv.Convert with SharpEnabled and the
 *    sRGB transfer (sharpyuv/sharpyuv.go:39-64, convertSharp :170-269).
 * ===================================================================== */

/* rgb: packed 8-bit RGB (3 bytes per pixel), row stride rgb_stride, image
 * pitch rgb_pitch.  matrix_host: 12 ints (HOST memory), ConversionMatrix
 * RGBToY[4], RGBToU[4], RGBToV[4] (sharpyuv/csp.go:62-90; WebP's matrix is
 * what the encoder uses).  Outputs Y (stride y_stride, pitch y_pitch) and
 * U / V ((width+1)/2 x (height+1)/2, stride uv_stride, pitch uv_pitch).
 * `work`: wg_sharpyuv_work_bytes(width, height, n_images).  width <= 16384. */
size_t wg_sharpyuv_work_bytes(int32_t width, int32_t height, int32_t n_images);
int wg_sharpyuv_convert(const uint8_t* rgb, int32_t width, int32_t height, int32_t rgb_stride, int64_t rgb_pitch,
                        const int32_t* matrix_host, int32_t n_images, uint8_t* y, int32_t y_stride, int64_t y_pitch,
                        uint8_t* u, uint8_t* v, int32_t uv_stride, int64_t uv_pitch, void* work, void* stream);
/* sharpyuv.Convert with Options{Matrix, TransferType, SharpEnabled}
 * (sharpyuv.go:17-64): transfer is the H.273 code (gamma.go:11-28; 13 = sRGB,
 * the default, as in wg_sharpyuv_convert); sharp_enabled = 0 runs
 * convertStandard (:68-115, 2x2 average, no work buffer needed). */
int wg_sharpyuv_convert_ex(const uint8_t* rgb, int32_t width, int32_t height, int32_t rgb_stride, int64_t rgb_pitch,
                           const int32_t* matrix_host, int32_t transfer, int32_t sharp_enabled, int32_t n_images,
                           uint8_t* y, int32_t y_stride, int64_t y_pitch, uint8_t* u, uint8_t* v, int32_t uv_stride,
                           int64_t uv_pitch, void* work, void* stream);
/* GammaToLinear over the 1024 10-bit codes (g2l) and the LinearToGamma table
 * (l2g, *n entries; l2g may be NULL to query n) the kernels use for a
 * transfer function other than sRGB (gamma.go:360-446); host memory. */
int wg_sharpyuv_transfer_tables_host(int32_t tf, uint32_t* g2l, uint16_t* l2g, int32_t* n);
/* The gamma tables used (gamma.go:48-88), host copies: g2l[1026], l2g[514]. */
int wg_sharpyuv_tables_host(uint32_t* g2l, uint32_t* l2g);
/* After wg_sharpyuv_convert on `work` (same stream): the refinement
 * iterations each image ran, the count the reference's early exit gives
 * (sharpyuv.go:254-263; 2..4).  Synchronises the stream; WG_EHIP if a
 * pipeline dependency wait timed out (the output is then invalid). */
int wg_sharpyuv_iterations(const void* work, int32_t width, int32_t height, int32_t n_images, int32_t* out,
                           void* stream);

#ifdef __cplusplus
}
#endif
#endif /* WEBPGPU_H */
