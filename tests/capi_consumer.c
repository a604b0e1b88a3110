/*
 * capi_consumer.c -- TEST: a C program built with gcc against
 * include/webpgpu.h and linked to webp_amd/libwebpgpu.so, standing in for the
 * cgo preambles of INTEGRATION.md (cgo compiles exactly such C with a C
 * compiler).  Built and run by tests/test_capi_consumer.py.
 *
 *   capi_consumer cpu <file.webp>
 *       host-only entry points and the argument validation paths: version,
 *       invalid arguments, work-size helpers, wg_setup_segment,
 *       wg_fixed_costs_i4_host, wg_random_init_host, wg_vp8_parse; prints
 *       key=value lines the test compares with the Python binding.
 *   capi_consumer gpu <file.webp> <out.bin>     (built with -DWG_WITH_HIP)
 *       the INTEGRATION.md call sequences through hipMalloc'd buffers:
 *       dsp_hip.go's ITransform override (wg_itransform, doTwo) and
 *       decode_hip.go's decodeFrameHIP (wg_vp8_parse -> wg_decode_frames ->
 *       wg_decode_status); writes ITransform's ref / coefficients / output and
 *       the decoded Y, U, V planes to out.bin for the test to check against
 *       the oracle.
 *   capi_consumer encode <frame.bin> <out.bin>   (built with -DWG_WITH_HIP)
 *       INTEGRATION.md's encodeFramePhaseAHIP over the whole device encode
 *       path, as encode_hip.go calls it for one frame: wg_encoder_config ->
 *       wg_import_rgba -> wg_analysis_alphas -> wg_segment_analysis ->
 *       wg_encode_row_order -> wg_encode_mbs -> wg_encode_status.  frame.bin:
 *       int32 w, h, quality, method, then w*h*4 RGBA bytes, then the 1056
 *       token probabilities (enc.proba.Bands).  out.bin: the wg_mb_enc
 *       records, the reconstruction (Y, U, V), the segment ids and the
 *       wg_frame_segs record, for the test to compare with the oracle.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "webpgpu.h"
#ifdef WG_WITH_HIP
#include <hip/hip_runtime_api.h>
#endif

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #c, wg_last_error()); \
      fails++;                                                     \
    }                                                              \
  } while (0)

static uint8_t* read_file(const char* path, size_t* n) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *n = (size_t)ftell(f);
  fseek(f, 0, SEEK_SET);
  uint8_t* buf = (uint8_t*)malloc(*n);
  if (buf && fread(buf, 1, *n, f) != *n) {
    free(buf);
    buf = NULL;
  }
  fclose(f);
  return buf;
}

static uint64_t fnv(const void* p, size_t n) {
  const uint8_t* b = (const uint8_t*)p;
  uint64_t h = 1469598103934665603ull;
  for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

/* the host-side parse every mode starts from */
static int parse(const uint8_t* data, size_t n, int32_t dims[5], wg_mb_info** mb, int16_t** co) {
  if (wg_vp8_parse(data, n, dims, NULL, NULL, 0) != WG_OK) return -1;
  const int64_t nmb = (int64_t)dims[3] * dims[4];
  *mb = (wg_mb_info*)calloc((size_t)nmb, sizeof(wg_mb_info));
  *co = (int16_t*)calloc((size_t)nmb * 384, sizeof(int16_t));
  return wg_vp8_parse(data, n, dims, *mb, *co, nmb);
}

static int run_cpu(const uint8_t* data, size_t n) {
  CHECK(wg_version() == WG_ABI_VERSION);
  /* invalid arguments are rejected before any device work */
  CHECK(wg_decode_frames(NULL, NULL, 2, 1, 1, 1, NULL, NULL, NULL, NULL, NULL) == WG_EINVAL);
  CHECK(strstr(wg_last_error(), "invalid argument") != NULL);
  CHECK(wg_transform(9, NULL, 0, NULL, 0, 1, NULL) == WG_EINVAL);
  CHECK(wg_convert_argb_to_uv(NULL, 0, NULL, NULL, 0, 4, 1, 1, NULL) == WG_EINVAL);
  CHECK(wg_decode_work_bytes(0, 68, 2) == 0);
  printf("decode_work_bytes=%zu\n", wg_decode_work_bytes(120, 68, 2));
  printf("encode_work_bytes=%zu\n", wg_encode_work_bytes(120, 68, 64));
  wg_segment seg;
  const int32_t dq[5] = {0, 0, 0, 0, 0};
  CHECK(wg_setup_segment(30, dq, 4, 50, &seg) == WG_OK);
  printf("segment_fnv=%llu\n", (unsigned long long)fnv(&seg, sizeof(seg)));
  uint16_t fixed[1000];
  CHECK(wg_fixed_costs_i4_host(fixed) == WG_OK);
  printf("fixed_i4_fnv=%llu\n", (unsigned long long)fnv(fixed, sizeof(fixed)));
  wg_random rg;
  wg_random_init_host(&rg, 0.5f);
  CHECK(rg.index1 == 0 && rg.index2 == 31 && rg.amp == 128);
  int32_t dims[5];
  wg_mb_info* mb = NULL;
  int16_t* co = NULL;
  CHECK(parse(data, n, dims, &mb, &co) == WG_OK);
  const size_t nmb = (size_t)dims[3] * dims[4];
  printf("dims=%d,%d,%d,%d,%d\n", dims[0], dims[1], dims[2], dims[3], dims[4]);
  printf("mb_fnv=%llu\n", (unsigned long long)fnv(mb, nmb * sizeof(wg_mb_info)));
  printf("coeffs_fnv=%llu\n", (unsigned long long)fnv(co, nmb * 384 * sizeof(int16_t)));
  free(mb);
  free(co);
  return fails;
}

#ifdef WG_WITH_HIP
static int run_gpu(const uint8_t* data, size_t n, const char* out_path) {
  CHECK(wg_device_check() == WG_OK);
  if (fails) return fails;
  FILE* out = fopen(out_path, "wb");
  if (!out) return 1;
  /* dsp_hip.go: ITransform(ref, in, dst, doTwo) on one BPS buffer */
  {
    uint8_t host[WG_YUV_SIZE];
    int16_t coef[32];
    uint32_t x = 12345u;
    for (int i = 0; i < WG_YUV_SIZE; i++) host[i] = (uint8_t)((x = x * 1664525u + 1013904223u) >> 24);
    for (int i = 0; i < 32; i++) coef[i] = (int16_t)(((x = x * 1664525u + 1013904223u) >> 20) - 2048);
    void *dev_buf = NULL, *dev_coef = NULL;
    CHECK(hipMalloc(&dev_buf, WG_YUV_SIZE) == hipSuccess && hipMalloc(&dev_coef, 64) == hipSuccess);
    CHECK(hipMemcpy(dev_buf, host, WG_YUV_SIZE, hipMemcpyHostToDevice) == hipSuccess);
    CHECK(hipMemcpy(dev_coef, coef, 64, hipMemcpyHostToDevice) == hipSuccess);
    CHECK(wg_itransform((const uint8_t*)dev_buf, (const int16_t*)dev_coef, (uint8_t*)dev_buf, 0, 1, 1, NULL) == WG_OK);
    uint8_t res[WG_YUV_SIZE];
    CHECK(hipMemcpy(res, dev_buf, WG_YUV_SIZE, hipMemcpyDeviceToHost) == hipSuccess);
    fwrite(host, 1, WG_YUV_SIZE, out);
    fwrite(coef, 2, 32, out);
    fwrite(res, 1, WG_YUV_SIZE, out);
    (void)hipFree(dev_buf);
    (void)hipFree(dev_coef);
  }
  /* decode_hip.go: decodeFrameHIP over the all-rows parse */
  {
    int32_t dims[5];
    wg_mb_info* mb = NULL;
    int16_t* co = NULL;
    CHECK(parse(data, n, dims, &mb, &co) == WG_OK);
    const int mbw = dims[3], mbh = dims[4];
    const size_t nmb = (size_t)mbw * mbh, ysz = 256 * nmb, uvsz = 64 * nmb;
    const size_t work = wg_decode_work_bytes(mbw, mbh, 1);
    void *d_mb = NULL, *d_co = NULL, *d_y = NULL, *d_u = NULL, *d_v = NULL, *d_work = NULL;
    CHECK(hipMalloc(&d_mb, 32 * nmb) == hipSuccess && hipMalloc(&d_co, 768 * nmb) == hipSuccess &&
          hipMalloc(&d_y, ysz) == hipSuccess && hipMalloc(&d_u, uvsz) == hipSuccess &&
          hipMalloc(&d_v, uvsz) == hipSuccess && hipMalloc(&d_work, work) == hipSuccess);
    CHECK(hipMemcpy(d_mb, mb, 32 * nmb, hipMemcpyHostToDevice) == hipSuccess);
    CHECK(hipMemcpy(d_co, co, 768 * nmb, hipMemcpyHostToDevice) == hipSuccess);
    int rc = wg_decode_frames((const wg_mb_info*)d_mb, (const int16_t*)d_co, dims[2], mbw, mbh, 1, (uint8_t*)d_y,
                              (uint8_t*)d_u, (uint8_t*)d_v, d_work, NULL);
    if (rc == WG_OK) rc = wg_decode_status(d_work, mbw, 1, NULL);
    CHECK(rc == WG_OK);
    uint8_t* planes = (uint8_t*)malloc(ysz + 2 * uvsz);
    CHECK(hipMemcpy(planes, d_y, ysz, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(hipMemcpy(planes + ysz, d_u, uvsz, hipMemcpyDeviceToHost) == hipSuccess);
    CHECK(hipMemcpy(planes + ysz + uvsz, d_v, uvsz, hipMemcpyDeviceToHost) == hipSuccess);
    fwrite(planes, 1, ysz + 2 * uvsz, out);
    void* ps[6] = {d_mb, d_co, d_y, d_u, d_v, d_work};
    for (int i = 0; i < 6; i++) (void)hipFree(ps[i]);
    free(planes);
    free(mb);
    free(co);
  }
  fclose(out);
  return fails;
}

static int run_encode(const uint8_t* in, size_t n, const char* out_path) {
  CHECK(wg_device_check() == WG_OK);
  if (fails || n < 16) return fails + 1;
  int32_t hdr[4];
  memcpy(hdr, in, sizeof(hdr));
  const int32_t w = hdr[0], h = hdr[1], quality = hdr[2], method = hdr[3];
  const size_t rgba_bytes = (size_t)w * h * 4;
  if (n != 16 + rgba_bytes + 1056) return fails + 1;
  const uint8_t* rgba = in + 16;
  const uint8_t* proba = in + 16 + rgba_bytes;
  const int32_t mbw = (w + 15) / 16, mbh = (h + 15) / 16, nmb = mbw * mbh;
  const size_t ysz = (size_t)256 * nmb, uvsz = (size_t)64 * nmb;
  /* EncodeConfig: DefaultConfig(quality) with the method asked for (encode.go:66-86) */
  wg_enc_config cfg;
  CHECK(wg_encoder_config(quality, method, 50, 60, 0, 1, 4, 0, &cfg) == WG_OK);
  void *d_rgba = NULL, *d_y = NULL, *d_u = NULL, *d_v = NULL, *d_alpha = NULL, *d_uvsum = NULL, *d_ids = NULL,
       *d_segs = NULL, *d_info = NULL, *d_proba = NULL, *d_out = NULL, *d_work = NULL;
  const size_t work = wg_encode_work_bytes(mbw, mbh, 1);
  CHECK(hipMalloc(&d_rgba, rgba_bytes) == hipSuccess && hipMalloc(&d_y, ysz) == hipSuccess &&
        hipMalloc(&d_u, uvsz) == hipSuccess && hipMalloc(&d_v, uvsz) == hipSuccess &&
        hipMalloc(&d_alpha, 4 * (size_t)nmb) == hipSuccess && hipMalloc(&d_uvsum, 4) == hipSuccess &&
        hipMalloc(&d_ids, (size_t)nmb) == hipSuccess && hipMalloc(&d_segs, 4 * sizeof(wg_segment)) == hipSuccess &&
        hipMalloc(&d_info, sizeof(wg_frame_segs)) == hipSuccess && hipMalloc(&d_proba, 1056) == hipSuccess &&
        hipMalloc(&d_out, sizeof(wg_mb_enc) * (size_t)nmb) == hipSuccess && hipMalloc(&d_work, work) == hipSuccess);
  if (fails) return fails;
  CHECK(hipMemcpy(d_rgba, rgba, rgba_bytes, hipMemcpyHostToDevice) == hipSuccess);
  CHECK(hipMemcpy(d_proba, proba, 1056, hipMemcpyHostToDevice) == hipSuccess);
  /* importImage (encode.go:671-943), no alpha */
  int rc = wg_import_rgba((const uint8_t*)d_rgba, w, h, 4 * w, (int64_t)rgba_bytes, 0, (uint8_t*)d_y,
                          (uint8_t*)d_u, (uint8_t*)d_v, (int64_t)ysz, (int64_t)uvsz, 1, NULL);
  CHECK(rc == WG_OK);
  /* computeAlphas -> analysis() -> setSegmentParams / setupSegment, on the device */
  if (rc == WG_OK)
    rc = wg_analysis_alphas((const uint8_t*)d_y, (const uint8_t*)d_u, (const uint8_t*)d_v, w, h, (int64_t)ysz,
                            (int64_t)uvsz, 1, (int32_t*)d_alpha, NULL, NULL, (int32_t*)d_uvsum, NULL);
  CHECK(rc == WG_OK);
  if (rc == WG_OK)
    rc = wg_segment_analysis(&cfg, (const int32_t*)d_alpha, (const int32_t*)d_uvsum, mbw, mbh, 1, (uint8_t*)d_ids,
                             d_segs, 4 * sizeof(wg_segment), (wg_frame_segs*)d_info, NULL);
  CHECK(rc == WG_OK);
  if (rc == WG_OK) rc = wg_encode_row_order((const int32_t*)d_alpha, mbw, mbh, 1, d_work, NULL);
  CHECK(rc == WG_OK);
  /* encodeFrameParallel Phase A; the reconstruction goes to separate planes */
  void *d_ry = NULL, *d_ru = NULL, *d_rv = NULL;
  CHECK(hipMalloc(&d_ry, ysz) == hipSuccess && hipMalloc(&d_ru, uvsz) == hipSuccess &&
        hipMalloc(&d_rv, uvsz) == hipSuccess);
  if (rc == WG_OK)
    rc = wg_encode_mbs((const uint8_t*)d_y, (const uint8_t*)d_u, (const uint8_t*)d_v, (int64_t)ysz, (int64_t)uvsz, w,
                       h, 1, (const uint8_t*)d_ids, d_segs, 0, (const uint8_t*)d_proba, cfg.method, cfg.quality,
                       d_out, (uint8_t*)d_ry, (uint8_t*)d_ru, (uint8_t*)d_rv, d_work, NULL);
  if (rc == WG_OK) rc = wg_encode_status(d_work, mbw, 1, NULL);
  CHECK(rc == WG_OK);
  FILE* out = fopen(out_path, "wb");
  if (!out) return fails + 1;
  const size_t host_bytes = sizeof(wg_mb_enc) * (size_t)nmb + ysz + 2 * uvsz + (size_t)nmb + sizeof(wg_frame_segs);
  uint8_t* host = (uint8_t*)malloc(host_bytes);
  uint8_t* p = host;
  CHECK(hipMemcpy(p, d_out, sizeof(wg_mb_enc) * (size_t)nmb, hipMemcpyDeviceToHost) == hipSuccess);
  p += sizeof(wg_mb_enc) * (size_t)nmb;
  CHECK(hipMemcpy(p, d_ry, ysz, hipMemcpyDeviceToHost) == hipSuccess);
  CHECK(hipMemcpy(p + ysz, d_ru, uvsz, hipMemcpyDeviceToHost) == hipSuccess);
  CHECK(hipMemcpy(p + ysz + uvsz, d_rv, uvsz, hipMemcpyDeviceToHost) == hipSuccess);
  p += ysz + 2 * uvsz;
  CHECK(hipMemcpy(p, d_ids, (size_t)nmb, hipMemcpyDeviceToHost) == hipSuccess);
  CHECK(hipMemcpy(p + nmb, d_info, sizeof(wg_frame_segs), hipMemcpyDeviceToHost) == hipSuccess);
  fwrite(host, 1, host_bytes, out);
  fclose(out);
  free(host);
  void* ps[15] = {d_rgba, d_y, d_u, d_v, d_alpha, d_uvsum, d_ids, d_segs, d_info, d_proba, d_out, d_work,
                  d_ry, d_ru, d_rv};
  for (int i = 0; i < 15; i++) (void)hipFree(ps[i]);
  return fails;
}
#endif

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s cpu|gpu file.webp [out.bin] | encode frame.bin out.bin\n", argv[0]);
    return 2;
  }
  size_t n = 0;
  uint8_t* data = read_file(argv[2], &n);
  if (!data) return 2;
  int rc;
  if (strcmp(argv[1], "cpu") == 0) {
    rc = run_cpu(data, n);
  } else if (strcmp(argv[1], "encode") == 0) {
#ifdef WG_WITH_HIP
    rc = argc > 3 ? run_encode(data, n, argv[3]) : 2;
#else
    fprintf(stderr, "built without -DWG_WITH_HIP\n");
    rc = 2;
#endif
  } else {
#ifdef WG_WITH_HIP
    rc = argc > 3 ? run_gpu(data, n, argv[3]) : 2;
#else
    fprintf(stderr, "built without -DWG_WITH_HIP\n");
    rc = 2;
#endif
  }
  free(data);
  printf("fails=%d\n", rc);
  return rc ? 1 : 0;
}
