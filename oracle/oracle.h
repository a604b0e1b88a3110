/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the deepteams/webp internal/dsp hot path (and the
 * lossy/webp callers that drive it), written from the Go source so that the
 * HIP kernels in webp_amd/ can be checked bit-for-bit.  Every function cites
 * the reference file:line it follows (paths relative to the reference root).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline -- never as the
 * product path.  The product library (webp_amd/libwebpgpu.so) does not link
 * it and has no CPU fallback.
 *
 * Integer widths: Go `int` is 64-bit, so arithmetic that Go does in `int`
 * and that can exceed 2^31 (IDCT second pass) is done in int64_t here.
 */
#ifndef WEBP_ORACLE_H
#define WEBP_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_BPS 32 /* internal/dsp/dsp.go:5 */
/* internal/lossy/constants.go:70-75 */
#define OR_YUV_SIZE (OR_BPS * 17 + OR_BPS * 9)
#define OR_YOFF (OR_BPS * 1 + 8)
#define OR_UOFF (OR_YOFF + OR_BPS * 16 + OR_BPS)
#define OR_VOFF (OR_UOFF + 16)

/* ---- clip helpers (internal/dsp/cliptables.go) ---- */
int or_clip8b(int64_t v);

/* ---- transforms (internal/dsp/transforms.go) ---- */
void or_transform(const int16_t* in, uint8_t* dst, int do_two);   /* transformTwo :139 */
void or_transform_dc(const int16_t* in, uint8_t* dst);            /* :148 */
void or_transform_ac3(const int16_t* in, uint8_t* dst);           /* :170 */
void or_transform_uv(const int16_t* in, uint8_t* dst);            /* :197 */
void or_transform_dcuv(const int16_t* in, uint8_t* dst);          /* :203 */
void or_transform_wht(const int16_t* in, int16_t* out);           /* :223 */
void or_itransform(const uint8_t* ref, const int16_t* in, uint8_t* dst, int do_two); /* :256 */
void or_ftransform(const uint8_t* src, const uint8_t* ref, int16_t* out);            /* :371 */
void or_ftransform2(const uint8_t* src, const uint8_t* ref, int16_t* out);           /* :487 */
void or_ftransform_wht(const int16_t* in, int16_t* out);          /* :500 */

/* ---- intra predictors (internal/dsp/predict_lossy.go); buf+off is the block origin ---- */
void or_pred_luma16(int mode, uint8_t* buf, int off);   /* :27-102 */
void or_pred_chroma8(int mode, uint8_t* buf, int off);  /* :106-181 */
void or_pred_luma4(int mode, uint8_t* buf, int off);    /* :185-451 */

/* ---- loop filters (internal/dsp/filter.go) ---- */
void or_simple_vfilter16(uint8_t* p, int base, int stride, int thresh);  /* :93 */
void or_simple_hfilter16(uint8_t* p, int base, int stride, int thresh);  /* :109 */
void or_simple_vfilter16i(uint8_t* p, int base, int stride, int thresh); /* :126 */
void or_simple_hfilter16i(uint8_t* p, int base, int stride, int thresh); /* :134 */
void or_vfilter16(uint8_t* p, int base, int stride, int thresh, int ithresh, int hev_t);  /* :194 */
void or_hfilter16(uint8_t* p, int base, int stride, int thresh, int ithresh, int hev_t);  /* :199 */
void or_vfilter16i(uint8_t* p, int base, int stride, int thresh, int ithresh, int hev_t); /* :217 */
void or_hfilter16i(uint8_t* p, int base, int stride, int thresh, int ithresh, int hev_t); /* :224 */
void or_vfilter8(uint8_t* u, uint8_t* v, int ubase, int vbase, int stride, int thresh, int ithresh, int hev_t);  /* :205 */
void or_hfilter8(uint8_t* u, uint8_t* v, int ubase, int vbase, int stride, int thresh, int ithresh, int hev_t);  /* :211 */
void or_vfilter8i(uint8_t* u, uint8_t* v, int ubase, int vbase, int stride, int thresh, int ithresh, int hev_t); /* :232 */
void or_hfilter8i(uint8_t* u, uint8_t* v, int ubase, int vbase, int stride, int thresh, int ithresh, int hev_t); /* :238 */

/* ---- YUV <-> RGB (internal/dsp/yuv.go) ---- */
void or_yuv_to_rgb(int y, int u, int v, uint8_t* rgb);          /* YUVToRGB :105 */
int or_rgb_to_y(int r, int g, int b);                            /* :151 */
int or_rgb_to_u(int r, int g, int b, int rounding);              /* :164 */
int or_rgb_to_v(int r, int g, int b, int rounding);              /* :169 */
uint32_t or_gamma_to_linear(int v);                              /* :226 */
int or_linear_to_gamma(uint32_t base, int shift);               /* :236 */
void or_accumulate_rgba(const uint8_t* r, const uint8_t* g, const uint8_t* b, const uint8_t* a,
                        int stride, uint16_t* dst, int width);   /* :486 */
void or_convert_rgba32_to_uv(const uint16_t* rgb, uint8_t* u, uint8_t* v, int width); /* :553 */
void or_convert_argb_to_y(const uint32_t* argb, uint8_t* y, int width);           /* :270 */
void or_convert_argb_to_uv(const uint32_t* argb, uint8_t* u, uint8_t* v, int src_width,
                           int do_store);                                         /* :291 */

/* ---- VP8Random (internal/dsp/random.go) ---- */
typedef struct { int index1, index2; uint32_t tab[55]; int amp; } or_random;
void or_random_init(or_random* rg, float dithering);            /* :39 */
int or_random_bits2(or_random* rg, int num_bits, int amp);      /* :54 */
void or_convert_rgba32_to_uv_dithered(const uint16_t* rgb, uint8_t* u, uint8_t* v, int width,
                                      or_random* rg);            /* yuv.go:568 */
float or_dithering_strength(float quality);                      /* encode.go (root):517-521 */
void or_import_rgba_dithered(const uint8_t* rgba, int w, int h, int stride, int has_alpha, float dithering,
                             uint8_t* Y, uint8_t* U, uint8_t* V); /* internal/lossy/encode.go:690-940 */

/* ---- upsampling (internal/dsp/upsample.go, webp.go) ---- */
void or_upsample_line_pair_nrgba(const uint8_t* top_y, const uint8_t* bot_y,
                                 const uint8_t* top_u, const uint8_t* top_v,
                                 const uint8_t* bot_u, const uint8_t* bot_v,
                                 uint8_t* top_dst, uint8_t* bot_dst,
                                 const uint8_t* alpha_top, const uint8_t* alpha_bot, int width); /* :130 */
void or_upsample_line_pair_rgb(const uint8_t* top_y, const uint8_t* bot_y,
                               const uint8_t* top_u, const uint8_t* top_v,
                               const uint8_t* bot_u, const uint8_t* bot_v,
                               uint8_t* top_dst, uint8_t* bot_dst, int width); /* :45 */
void or_point_sample_row(const uint8_t* y, const uint8_t* u, const uint8_t* v, uint8_t* dst,
                         int width); /* PointSampleRow :240 */
/* buildNRGBA (webp.go:379-450): alpha may be NULL (then A=255); out stride = 4*w */
void or_build_nrgba(int w, int h, const uint8_t* y, int y_stride, const uint8_t* u, const uint8_t* v,
                    int uv_stride, const uint8_t* alpha, uint8_t* out);

/* ---- distortion / SSIM (internal/dsp/ssim.go) ---- */
int or_sse4x4(const uint8_t* a, const uint8_t* b);               /* :188 */
int or_sse16x16(const uint8_t* a, const uint8_t* b);             /* :220 */
int or_tdisto4x4(const uint8_t* a, const uint8_t* b);            /* :315 */
int or_tdisto16x16(const uint8_t* a, const uint8_t* b);          /* :327 */
double or_ssim_get(const uint8_t* s1, int st1, const uint8_t* s2, int st2);   /* :116 */
double or_ssim_get_clipped(const uint8_t* s1, int st1, const uint8_t* s2, int st2,
                           int xo, int yo, int w, int h);         /* :132 */
/* plane SSIM sum = libwebp AccumulateSSIM: sum over all pixels of SSIMGetClipped */
double or_plane_ssim(const uint8_t* a, int sa, const uint8_t* b, int sb, int w, int h);
uint64_t or_sse_plane(const uint8_t* a, int sa, const uint8_t* b, int sb, int w, int h); /* SSE :172 */
void or_disto_stats(const uint8_t* pix, int ps, const uint8_t* ref, int rs, int w, int h, uint32_t out[6]); /* :103 */
double or_ssim_from_stats(const uint32_t st[6], int clipped);   /* :88, :97 */
double or_psnr_from_sse(uint64_t sse, int64_t count);           /* :163 */

/* ---- lossy encoder DSP drivers ---- */
/* importImage (internal/lossy/encode.go:671-943), non-dithered direct path:
 * rgba (stride bytes) w x h -> Y (stride 16*mbW, 16*mbH rows), U/V (stride 8*mbW, 8*mbH rows).
 * has_alpha=0 forces A=255 for chroma averaging (encode.go:862-866). */
void or_import_rgba(const uint8_t* rgba, int w, int h, int stride, int has_alpha,
                    uint8_t* y, uint8_t* u, uint8_t* v);
/* computeAlphas (encode_analysis.go:245-307): alphas[mbW*mbH] mixed alpha, returns uv alpha avg.
 * lum_alpha/uv_alpha (optional, may be NULL) receive the per-MB parts. */
int or_compute_alphas(const uint8_t* y, const uint8_t* u, const uint8_t* v, int w, int h,
                      int32_t* alphas, int32_t* lum_alpha, int32_t* uv_alpha);

/* ---- lossy decoder reconstruct + loop filter (internal/lossy/decode_frame.go) ---- */
/* Parsed macroblock, the GPU wire format (mirrors MBData decode.go:115-126 and FInfo :107-112). */
typedef struct {
  uint32_t non_zero_y;   /* 2 bits/block, block 0 in bits 31..30 */
  uint32_t non_zero_uv;  /* U in bits 0..7, V in bits 8..15 */
  uint8_t imodes[16];    /* I16: imodes[0]; I4: 16 sub-block modes (raster) */
  uint8_t is_i4x4;
  uint8_t uv_mode;
  uint8_t skip;
  uint8_t segment;
  uint8_t f_limit;       /* FInfo.FLimit (0 = no filtering) */
  uint8_t f_ilevel;      /* FInfo.FILevel */
  uint8_t f_inner;       /* FInfo.FInner */
  uint8_t hev_thresh;    /* FInfo.HevThresh */
} or_mb_info;            /* 32 bytes */

/* reconstructRow over all rows (decode_frame.go:83-218): coeffs int16[nMB][384].
 * Planes have stride 16*mbW (Y) and 8*mbW (U/V), like the decoder caches (decode.go:441-530). */
void or_decode_reconstruct(const or_mb_info* mb, const int16_t* coeffs, int mbw, int mbh,
                           uint8_t* y, uint8_t* u, uint8_t* v);
/* filterRowAt/doFilter over all rows, raster MB order (decode_frame.go:283-342). */
void or_decode_filter(const or_mb_info* mb, int filter_type, int mbw, int mbh,
                      uint8_t* y, uint8_t* u, uint8_t* v);
/* parseFrame order (decode.go:532-560): reconstruct row then filter row. */
void or_decode_frame(const or_mb_info* mb, const int16_t* coeffs, int filter_type, int mbw, int mbh,
                     uint8_t* y, uint8_t* u, uint8_t* v);

/* ---- VP8L predictor transform (lossless.c; encode_predictor.go, decode_transform.go) ---- */
double or_go_log2(double x);
void or_vp8l_slog2_lut(double* out, int n);
uint32_t or_vp8l_predict(int mode, uint32_t l, uint32_t t, uint32_t tr, uint32_t tl);
double or_vp8l_estimate_entropy(const uint32_t* argb, int width, int height, int tx, int ty, int bits, int mode);
void or_vp8l_residual_image(const uint32_t* argb, int width, int height, int bits, int quality, uint32_t* modes,
                            uint32_t* residuals);
void or_vp8l_inverse_predictor(const uint32_t* modes, int bits, int width, int height, const uint32_t* in,
                               uint32_t* out);
void or_vp8l_subtract_green(uint32_t* argb, size_t n);
void or_vp8l_add_green(uint32_t* argb, size_t n);
void or_vp8l_color_space_transform(uint32_t* argb, int width, int height, int bits, uint32_t* data);
void or_vp8l_color_space_inverse(const uint32_t* data, int bits, int width, int height, const uint32_t* src,
                                 uint32_t* dst);
void or_vp8l_color_index_inverse(const uint32_t* palette, int palette_size, int xbits, int width, int height,
                                 const uint32_t* src, uint32_t* dst);

/* vp8l_dec.c: entropy decoding of a VP8L bitstream up to the inverse transforms */
typedef struct {
  int width, height, has_alpha, tw, n_transforms;
  int type[4], bits[4], xsize[4], dsize[4];
} or_vp8l_info;
int or_vp8l_decode(const uint8_t* payload, size_t len, or_vp8l_info* info, uint32_t* pixels, uint32_t** tdata);

/* alpha.c: alpha-plane filters and alpha processing */
void or_alpha_filter(int filter, const uint8_t* in, int width, int height, uint8_t* out);
void or_alpha_unfilter(int filter, uint8_t* data, int width, int height);
int or_alpha_estimate_best_filter(const uint8_t* data, int width, int height);
int or_alpha_num_colors(const uint8_t* data, int width, int height);
void or_apply_alpha_multiply(uint8_t* rgba, int alpha_first, int width, int height, int stride, int inverse);
void or_mult_argb(uint32_t* argb, size_t n, int inverse);
void or_apply_alpha_multiply_4444(uint8_t* data, int width, int height, int stride);
int or_dispatch_alpha(const uint8_t* alpha, int alpha_stride, int width, int height, uint8_t* dst, int dst_stride,
                      int alpha_off);
int or_extract_alpha(const uint8_t* src, int src_stride, int width, int height, uint8_t* alpha, int alpha_stride,
                     int alpha_off);
int or_has_alpha(const uint8_t* src, size_t length, int step);
void or_alpha_replace(uint32_t* argb, size_t length, uint32_t color);
void or_dispatch_alpha_to_green(const uint8_t* alpha, int alpha_stride, int width, int height, uint32_t* dst,
                                int dst_stride);
void or_extract_green(const uint32_t* argb, uint8_t* alpha, size_t size);
void or_pack_rgb(const uint8_t* r, const uint8_t* g, const uint8_t* b, size_t length, int step, uint32_t* out);

/* rescale.c: the row rescaler (internal/dsp/rescale.go) */
typedef struct {          /* dsp.Rescaler (rescale.go:14-41) */
  int src_width, src_height, dst_width, dst_height;
  int x_expand, y_expand;
  int32_t* frow;
  int32_t* irow;
  int64_t y_accum;
  int y_add, y_sub, x_add, x_sub;
  uint32_t fx_scale, fy_scale, fxy_scale;
  int src_y, dst_y;
} or_rescaler;
void or_rescaler_init(or_rescaler* r, int sw, int sh, int dw, int dh);
void or_rescaler_free(or_rescaler* r);
void or_rescaler_import_row(or_rescaler* r, const uint8_t* src);
int or_rescaler_export_row(or_rescaler* r, uint8_t* dst);
/* plane driver: returns the number of destination rows written */
int or_rescale_plane(const uint8_t* src, int sw, int sh, int src_stride, uint8_t* dst, int dw, int dh,
                     int dst_stride);

/* ---- Encoder MB RD loop (lossy_rd.c; encode_parallel.go Phase A) ---- */
typedef struct {          /* SegmentQuant (encode.go:311-323) */
  int32_t quant, iquant, bias, zthresh;
  int32_t dc_quant, dc_iquant, dc_bias, dc_zthresh;
  int16_t sharpen[16];
} or_squant;              /* 64 bytes */
typedef struct {          /* SegmentInfo fields Phase A reads (encode.go:278-309) */
  or_squant y1, y2, uv;
  int32_t lambda_i4, lambda_i16, lambda_uv, lambda_mode;
  int32_t tlambda_i4, tlambda_i16, tlambda_uv, tlambda_sd;
} or_segment;             /* 224 bytes */
typedef struct {          /* MBEncInfo (encode.go:241-276), Phase A outputs */
  int16_t coeffs[400];    /* 16 Y, 4 U, 4 V blocks (raster), then the WHT DC block */
  uint8_t modes[16];
  uint8_t nz_y[16];
  uint8_t nz_uv[8];
  uint32_t non_zero_y;    /* bit b: Y block b has a non-zero level; bit 24: DC block */
  uint32_t non_zero_uv;   /* bit ch*4+b */
  uint8_t mb_type, i16_mode, uv_mode, nz_dc;
  uint8_t skip, segment, pad0, pad1;
  uint64_t score;
} or_mb_enc;              /* 864 bytes */
void or_setup_segment(int q, int dq_y1_dc, int dq_y2_dc, int dq_y2_ac, int dq_uv_dc, int dq_uv_ac, int method,
                      int sns_strength, or_segment* seg);
void or_fixed_costs_i4(uint16_t* out /* [10][10][10] */);
int or_quantize_coeffs(const int16_t* in, int16_t* out, const or_squant* sq, int first);
void or_dequant_coeffs(const int16_t* in, int16_t* out, const or_squant* sq);
uint64_t or_rd_score(int disto, int rate, int lambda);
int or_token_cost(const int16_t* coeffs, int nz_count, int type, const uint8_t* proba, int ctx0, int first);
int or_trellis_quantize(const int16_t* in, int16_t* out, const or_squant* sq, int first, int ctx_type, int init_ctx,
                        const uint8_t* proba, int lambda);
void or_encode_frame_rd(uint8_t* y, uint8_t* u, uint8_t* v, int width, int height, int mbw, int mbh,
                        const uint8_t* segments, const or_segment* segs, const uint8_t* proba, int method,
                        int quality, or_mb_enc* out);

/* ---- segment analysis (segments.c; encode_analysis.go:29-903) ---- */
typedef struct { /* the EncodeConfig fields the analysis reads (internal/lossy/encode.go:30-63) */
  int quality, method, sns_strength, filter_strength, filter_sharpness, filter_type, segments, preprocessing;
} or_enc_config;
typedef struct { /* what analysis() + setSegmentProbas leave for Phase A/B (= wg_frame_segs) */
  int32_t num_segments, base_quant, global_uv_alpha, dq_uv_ac, dq_uv_dc, filter_level, update_map, pad;
  int32_t quant[4], fstrength[4], alpha[4], beta[4];
  uint8_t seg_proba[4];
  int32_t pad2[3];
} or_frame_segs;        /* 112 bytes */
double or_quality_to_compression(int quality);
int or_quality_to_qindex(int quality);
int or_segment_quant(int quality, int sns_strength, int seg_alpha);
void or_segment_analysis(const int32_t* alphas, int mbw, int mbh, int uv_alpha_sum, const or_enc_config* cfg,
                         uint8_t* seg_ids, or_frame_segs* info);

/* ---- SharpYUV (sharpyuv.c; sharpyuv/sharpyuv.go, gamma.go) ---- */
void or_sharpyuv_tables(uint32_t* g2l_out /* 1026 */, uint32_t* l2g_out /* 514 */);
int or_sharpyuv_convert(const uint8_t* rgb, int width, int height, int rgb_stride, uint8_t* y, int y_stride,
                        uint8_t* u, uint8_t* v, int uv_stride, const int32_t* matrix /* 12 */);
int or_sharpyuv_convert_tf(const uint8_t* rgb, int width, int height, int rgb_stride, uint8_t* y, int y_stride,
                           uint8_t* u, uint8_t* v, int uv_stride, const int32_t* matrix, int tf);
void or_sharpyuv_convert_standard(const uint8_t* rgb, int width, int height, int rgb_stride, uint8_t* y, int y_stride,
                                  uint8_t* u, uint8_t* v, int uv_stride, const int32_t* matrix);
uint32_t or_sharpyuv_gamma_to_linear(uint16_t v, int bit_depth, int tf);
void or_sharpyuv_tf_long_double(int on);
uint16_t or_sharpyuv_linear_to_gamma(uint32_t v, int bit_depth, int tf);

#ifdef __cplusplus
}
#endif
#endif
