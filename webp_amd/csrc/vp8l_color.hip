// vp8l_color.hip -- the VP8L cross-colour transform and the colour inverse
// transforms on gfx950.
//
//   k_cc_select   ColorSpaceTransform (internal/lossless/encode_predictor.go:
//                 727-770): per tile, the three multipliers
//                 (findBestMultipliers :514-585) and the forward transform of
//                 the tile in place (applyColorTransformTile :774-792)
//   k_cc_inverse  colorSpaceInverseTransform (decode_transform.go:454-520)
//   k_ci_inverse  colorIndexInverseTransform (decode_transform.go:560-612)
//
// k_cc_select: one 256-lane workgroup per tile.  A multiplier search is a
// first-minimum over candidate multipliers of sum_i |t_i - (m * int8(s_i)) >> 5|
// (mod 256, folded at 128; multiplierCost :645-718 -- its threshold early exit
// returns a partial sum above the running best, which never changes the
// argmin, so the full sums are used).  Each pass gives a lane one candidate and
// a strided share of the tile's pixels; the per-candidate sums are reduced in
// LDS and one lane then applies the reference's scan order (coarse m = -128,
// -120, ..., 120 with strict '<', then m = best-7..best+7 with strict '<'
// against the running best).  Passes: coarse green->red and green->blue
// together (64 candidates), their fine searches (2 x 15), coarse red->blue on
// the adjusted red / blue (32), its fine search (15), then the transform.
// All integer; bit-exact with oracle/lossless.c.
#include "wg_common.h"

namespace {

constexpr int CC_THREADS = 256;
constexpr int CC_LDS_PIXELS = 64 * 64;  // tiles up to bits = 6 are staged in LDS

__device__ __forceinline__ int cc_delta(int m, int c) { return (m * (int)(int8_t)c) >> 5; }
// |t - delta| folded as the reference does: r = uint8(t - delta); r > 128 ? 256 - r : r
// (= |int8(t - delta)|: r < 128 -> r, r = 128 -> 128, r > 128 -> 256 - r)
__device__ __forceinline__ int cc_term(int m, int s, int t) {
  const int v = (int)(int8_t)(uint8_t)(t - cc_delta(m, s));
  return v < 0 ? -v : v;
}

struct CcArgs {
  uint32_t* argb;
  uint32_t* data;
  int64_t pitch;
  int width, height, bits, tiles_x, tiles_y;
};

__global__ __launch_bounds__(CC_THREADS) void k_cc_select(CcArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t px[CC_LDS_PIXELS];
  __shared__ int part[CC_THREADS];
  __shared__ int cost[64];
  __shared__ int best[3];
  const int tid = threadIdx.x;
  const int tiles = a.tiles_x * a.tiles_y;
  const int img = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const int tx = tile % a.tiles_x, ty = tile / a.tiles_x, ts = 1 << a.bits;
  const int x0 = tx * ts, y0 = ty * ts;
  const int tw = min(ts, a.width - x0), th = min(ts, a.height - y0), n = tw * th;
  uint32_t* base = a.argb + img * a.pitch + (int64_t)y0 * a.width + x0;
  const bool staged = n <= CC_LDS_PIXELS;
  if (staged) {
    for (int i = tid; i < n; i += CC_THREADS) px[i] = base[(int64_t)(i / tw) * a.width + i % tw];
    __syncthreads();
  }
  auto pixel = [&](int i) -> uint32_t { return staged ? px[i] : base[(int64_t)(i / tw) * a.width + i % tw]; };

  // one search pass: lane = (candidate c < ncand, pixel group g of ngroups)
  // -> cost[c]; src/dst channel selectors: 0 green, 1 red, 2 blue, 3 adjusted
  // red, 4 adjusted blue (after the green multipliers in best[0], best[1])
  auto pass = [&](int ncand, int first_m, int step, int sel_mode) {
    const int ngroups = CC_THREADS / ncand;  // ncand in {32, 64}
    const int c = tid % ncand, g = tid / ncand;
    int sum = 0;
    // sel_mode 0: c < 32 green->red, c >= 32 green->blue (coarse, 64 candidates)
    // sel_mode 1: c < 16 green->red fine, 16..31 green->blue fine
    // sel_mode 2: adjusted red -> adjusted blue (coarse or fine by step)
    int m, ch;
    if (sel_mode == 0) {
      m = -128 + 8 * (c & 31);
      ch = c >> 5;
    } else if (sel_mode == 1) {
      ch = c >> 4;
      m = best[ch] - 7 + (c & 15);
    } else {
      ch = 2;
      m = step ? -128 + 8 * c : best[2] - 7 + c;
    }
    const bool live = (sel_mode == 1 ? (c & 15) < 15 : (sel_mode == 2 && !step ? c < 15 : true)) && m >= -128 && m <= 127;
    // (sel_mode is uniform; within modes 0 / 1 the target channel is a
    // per-lane shift, not a branch: the lanes of one wave search both the
    // green->red and the green->blue candidates, and a branch on the channel
    // ran both bodies for every pixel)
    // staged: group g sums a contiguous chunk of the tile, 4 pixels an LDS
    // read (the sums are integers: any order gives the reference's)
    const int chunk = ((n + ngroups - 1) / ngroups + 3) & ~3;
    const int i0 = staged ? g * chunk : g, i1 = staged ? min(n, i0 + chunk) : n, di = staged ? 1 : ngroups;
    if (live && sel_mode != 2) {
      const int tsh = ch == 0 ? 16 : 0;  // red or blue
      auto term = [&](uint32_t p) { return cc_term(m, (p >> 8) & 0xff, (p >> tsh) & 0xff); };
      int i = i0;
      if (staged)
        for (; i + 4 <= i1; i += 4) {
          const uint4 q = *reinterpret_cast<const uint4*>(&px[i]);
          sum += term(q.x) + term(q.y) + term(q.z) + term(q.w);
        }
      for (; i < i1; i += di) sum += term(pixel(i));
    } else if (live) {
      const int g2r = best[0], g2b = best[1];
      auto term = [&](uint32_t p) {
        const int gr = (p >> 8) & 0xff, rd = (p >> 16) & 0xff, bl = p & 0xff;
        return cc_term(m, (rd - cc_delta(g2r, gr)) & 0xff, (bl - cc_delta(g2b, gr)) & 0xff);
      };
      int i = i0;
      if (staged)
        for (; i + 4 <= i1; i += 4) {
          const uint4 q = *reinterpret_cast<const uint4*>(&px[i]);
          sum += term(q.x) + term(q.y) + term(q.z) + term(q.w);
        }
      for (; i < i1; i += di) sum += term(pixel(i));
    }
    part[tid] = live ? sum : 0x7fffffff;
    __syncthreads();
    if (tid < ncand) {
      int s = 0;
      bool ok = part[tid] != 0x7fffffff;
      for (int k = 0; k < ngroups; k++) s += part[tid + k * ncand];
      cost[tid] = ok ? s : 0x7fffffff;
    }
    __syncthreads();
  };

  // coarse green->red and green->blue
  if (tid < 3) best[tid] = 0;
  __syncthreads();
  pass(64, -128, 8, 0);
  __shared__ int coarse_cost[3];
  if (tid < 2) {  // first minimum in the reference's scan order
    int bm = 0, bc = 0x7fffffff;
    for (int k = 0; k < 32; k++)
      if (cost[32 * tid + k] < bc) {
        bc = cost[32 * tid + k];
        bm = -128 + 8 * k;
      }
    best[tid] = bm;
    coarse_cost[tid] = bc;
  }
  __syncthreads();
  pass(32, 0, 0, 1);
  if (tid < 2) {
    int bm = best[tid], bc = coarse_cost[tid];
    for (int k = 0; k < 15; k++) {
      const int m = best[tid] - 7 + k;
      if (m < -128 || m > 127) continue;
      const int cst = cost[16 * tid + k];
      if (cst < bc) {
        bc = cst;
        bm = m;
      }
    }
    part[tid] = bm;  // (part is free here)
  }
  __syncthreads();
  if (tid < 2) best[tid] = part[tid];
  __syncthreads();
  // red->blue on the adjusted channels
  pass(32, -128, 1, 2);
  if (tid == 0) {
    int bm = 0, bc = 0x7fffffff;
    for (int k = 0; k < 32; k++)
      if (cost[k] < bc) {
        bc = cost[k];
        bm = -128 + 8 * k;
      }
    best[2] = bm;
    coarse_cost[2] = bc;
  }
  __syncthreads();
  pass(32, 0, 0, 2);
  if (tid == 0) {
    int bm = best[2], bc = coarse_cost[2];
    for (int k = 0; k < 15; k++) {
      const int m = best[2] - 7 + k;
      if (m < -128 || m > 127) continue;
      if (cost[k] < bc) {
        bc = cost[k];
        bm = m;
      }
    }
    part[0] = bm;
  }
  __syncthreads();
  const int g2r = best[0], g2b = best[1], r2b = part[0];
  if (tid == 0)
    a.data[(int64_t)img * tiles + tile] = (uint32_t)(uint8_t)g2r | (uint32_t)(uint8_t)g2b << 8 | (uint32_t)(uint8_t)r2b << 16;
  // applyColorTransformPixel (:497-507) over the tile, in place
  for (int i = tid; i < n; i += CC_THREADS) {
    const uint32_t p = pixel(i);
    const int gr = (p >> 8) & 0xff, rd = (p >> 16) & 0xff, bl = p & 0xff;
    const int nr = (rd - cc_delta(g2r, gr)) & 0xff;
    const int nb = (bl - cc_delta(g2b, gr) - cc_delta(r2b, rd)) & 0xff;
    base[(int64_t)(i / tw) * a.width + i % tw] = (p & 0xff00ff00u) | ((uint32_t)nr << 16) | (uint32_t)nb;
  }
}

// ---- k_cc_select_q: the same search for tiles of at most 32 x 32 (bits <= 5)
// on packed byte arithmetic, one 256-lane workgroup a tile.
//
// A candidate's cost is sum_i |int8(t_i - delta(m, s_i))|.  With t' = t + 128
// (mod 256) that is sum_i |u_i - 128| for the byte u_i = t'_i - delta (mod
// 256), so four pixels' terms are one v_sad_u8 against 0x80808080 once their
// four u bytes sit in one word.  The tile is staged once as 4-pixel groups:
// the sources as two packed int16 pairs (sign-extended bytes: delta of two
// pixels is one v_pk_mul_lo_u16 and one v_pk_ashrrev_i16 -- m * int8(s) fits
// int16 and its low byte is all that counts), and each target as T1 = t' |
// 0x80 and T2 = (t' & 0x80) ^ 0x80 per byte, so the byte-wise subtraction
// mod 256 is (T1 - (d & 0x7f..)) ^ T2 ^ (d & 0x80..) with no borrow crossing a
// byte.  Lane = candidate: every lane of a wave reads the same group (an LDS
// broadcast) and adds 4 terms per ~10 VALU instructions.  Groups past the
// tile's pixels are padding (source 0, t' = 128: term 0).
//   A  coarse green->red (lanes 0-31) and green->blue (32-63), m = -128 + 8j;
//      wave w sums groups 64w .. 64w + 63
//   B  their fine searches (m = best - 7 + j, j < 15), a pixel half per
//      half-wave
//   C  red->blue coarse on the adjusted channels (restaged), a half a half-wave
//   D  its fine search, a pixel quarter per 16 lanes
// Each search's winner is the reference's: the first strict minimum in scan
// order (the minimum of cost << 5 | j), and a fine candidate replaces the
// coarse best only with a strictly lower cost.  Sums are integers, so the
// order they are added in does not matter.
constexpr int CQ_GROUPS = 256;  // 4-pixel groups of a 32 x 32 tile
typedef short cq_s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t cq_sext_pair(uint32_t a, uint32_t b) {  // int8 bytes a, b -> int16 pair
  return ((uint32_t)(int32_t)(int8_t)a & 0xffffu) | (uint32_t)(int32_t)(int8_t)b << 16;
}
// T1 / T2 of four target bytes (t' = t + 128)
__device__ __forceinline__ uint2 cq_target(uint32_t t4) {
  const uint32_t tp = t4 ^ 0x80808080u;
  return make_uint2(tp | 0x80808080u, (tp & 0x80808080u) ^ 0x80808080u);
}
// four terms of candidate mm (m in both int16 halves) on one group
__device__ __forceinline__ uint32_t cq_terms(uint32_t mm, uint2 src, uint2 tgt, uint32_t acc) {
  const cq_s16x2 m2 = __builtin_bit_cast(cq_s16x2, mm);
  const cq_s16x2 p0 = (m2 * __builtin_bit_cast(cq_s16x2, src.x)) >> (cq_s16x2){5, 5};
  const cq_s16x2 p1 = (m2 * __builtin_bit_cast(cq_s16x2, src.y)) >> (cq_s16x2){5, 5};
  const uint32_t d = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, p1), __builtin_bit_cast(uint32_t, p0), 0x06040200u);
  const uint32_t z = tgt.x - (d & 0x7f7f7f7fu);
  const uint32_t u = z ^ tgt.y ^ (d & 0x80808080u);
  return __builtin_amdgcn_sad_u8(u, 0x80808080u, acc);
}
__device__ __forceinline__ int cq_min(int v, int width) {  // min over aligned groups of `width` lanes
  for (int o = width >> 1; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}

__global__ __launch_bounds__(256) void k_cc_select_q(CcArgs a) {
  __shared__ uint2 gsrc[CQ_GROUPS];     // source int16 pairs (pixels 0, 1 | 2, 3)
  __shared__ uint2 gtgt[CQ_GROUPS][2];  // target T1 / T2: [0] red (then adjusted blue), [1] blue
  __shared__ int part[4][64];
  __shared__ int best[3], cbest[3];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles = a.tiles_x * a.tiles_y;
  const int img = blockIdx.x / tiles, tile = blockIdx.x % tiles;
  const int tx = tile % a.tiles_x, ty = tile / a.tiles_x, ts = 1 << a.bits;
  const int x0 = tx * ts, y0 = ty * ts;
  const int tw = min(ts, a.width - x0), th = min(ts, a.height - y0), n = tw * th;
  uint32_t* base = a.argb + img * a.pitch + (int64_t)y0 * a.width + x0;
  // this thread's group: pixels 4 tid .. 4 tid + 3 of the tile (row-major), kept for the transform
  uint32_t px[4];
  bool in[4];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int i = 4 * tid + k;
    in[k] = i < n;
    px[k] = in[k] ? base[(int64_t)(i / tw) * a.width + i % tw] : 0u;
  }
  auto bytes4 = [&](int sh) {  // channel byte at shift sh of the 4 pixels (padding: 0)
    return ((px[0] >> sh) & 0xffu) | ((px[1] >> sh) & 0xffu) << 8 | ((px[2] >> sh) & 0xffu) << 16 |
           ((px[3] >> sh) & 0xffu) << 24;
  };
  {
    const uint32_t g4 = bytes4(8);
    gsrc[tid] = make_uint2(cq_sext_pair(g4, g4 >> 8), cq_sext_pair(g4 >> 16, g4 >> 24));
    gtgt[tid][0] = cq_target(bytes4(16));
    gtgt[tid][1] = cq_target(bytes4(0));
  }
  __syncthreads();
  auto pack_m = [](int m) { return ((uint32_t)m & 0xffffu) | (uint32_t)m << 16; };
  // ---- A: coarse green->red / green->blue ----
  {
    const int ch = lane >> 5, j = lane & 31;
    const uint32_t mm = pack_m(-128 + 8 * j);
    uint32_t acc = 0;
    for (int g = 64 * wave; g < 64 * wave + 64; g++) acc = cq_terms(mm, gsrc[g], gtgt[g][ch], acc);
    part[wave][lane] = (int)acc;
  }
  __syncthreads();
  if (wave == 0) {
    const int cost = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    const int key = cq_min(cost * 32 + (lane & 31), 32);
    if ((lane & 31) == 0) {
      best[lane >> 5] = -128 + 8 * (key & 31);
      cbest[lane >> 5] = key >> 5;
    }
  }
  __syncthreads();
  // ---- B: fine green->red (lanes 0-15 of a half) / green->blue (16-31) ----
  {
    const int h = lane >> 5, ch = (lane >> 4) & 1, j = lane & 15;
    const uint32_t mm = pack_m(best[ch] - 7 + j);
    uint32_t acc = 0;
    for (int g = 64 * wave + 32 * h; g < 64 * wave + 32 * h + 32; g++) acc = cq_terms(mm, gsrc[g], gtgt[g][ch], acc);
    acc += __shfl_xor(acc, 32, 64);
    if (lane < 32) part[wave][lane] = (int)acc;
  }
  __syncthreads();
  if (wave == 0 && lane < 32) {
    const int ch = lane >> 4, j = lane & 15, m = best[ch] - 7 + j;
    const int cost = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    const bool valid = j < 15 && m >= -128 && m <= 127;
    const int key = cq_min(valid ? cost * 16 + j : 0x7fffffff, 16);
    if (j == 0 && (key >> 4) < cbest[ch]) best[ch] = best[ch] - 7 + (key & 15);
  }
  __syncthreads();
  // ---- C: restage: adjusted red -> sources, adjusted blue -> targets; coarse red->blue ----
  const int g2r = best[0], g2b = best[1];
  {
    uint32_t ar = 0, ab = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int gr = (px[k] >> 8) & 0xff, rd = (px[k] >> 16) & 0xff, bl = px[k] & 0xff;
      const uint32_t r2 = in[k] ? (uint32_t)((rd - cc_delta(g2r, gr)) & 0xff) : 0u;
      const uint32_t b2 = in[k] ? (uint32_t)((bl - cc_delta(g2b, gr)) & 0xff) : 0u;
      ar |= r2 << (8 * k);
      ab |= b2 << (8 * k);
    }
    gsrc[tid] = make_uint2(cq_sext_pair(ar, ar >> 8), cq_sext_pair(ar >> 16, ar >> 24));
    gtgt[tid][0] = cq_target(ab);
  }
  __syncthreads();
  {
    const int h = lane >> 5, j = lane & 31;
    const uint32_t mm = pack_m(-128 + 8 * j);
    uint32_t acc = 0;
    for (int g = 64 * wave + 32 * h; g < 64 * wave + 32 * h + 32; g++) acc = cq_terms(mm, gsrc[g], gtgt[g][0], acc);
    acc += __shfl_xor(acc, 32, 64);
    if (lane < 32) part[wave][lane] = (int)acc;
  }
  __syncthreads();
  if (wave == 0 && lane < 32) {
    const int cost = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    const int key = cq_min(cost * 32 + lane, 32);
    if (lane == 0) {
      best[2] = -128 + 8 * (key & 31);
      cbest[2] = key >> 5;
    }
  }
  __syncthreads();
  // ---- D: fine red->blue, a pixel quarter per 16 lanes ----
  {
    const int q = lane >> 4, j = lane & 15;
    const uint32_t mm = pack_m(best[2] - 7 + j);
    uint32_t acc = 0;
    for (int g = 64 * wave + 16 * q; g < 64 * wave + 16 * q + 16; g++) acc = cq_terms(mm, gsrc[g], gtgt[g][0], acc);
    acc += __shfl_xor(acc, 16, 64);
    acc += __shfl_xor(acc, 32, 64);
    if (lane < 16) part[wave][lane] = (int)acc;
  }
  __syncthreads();
  if (wave == 0 && lane < 16) {
    const int j = lane, m = best[2] - 7 + j;
    const int cost = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
    const bool valid = j < 15 && m >= -128 && m <= 127;
    const int key = cq_min(valid ? cost * 16 + j : 0x7fffffff, 16);
    if (j == 0 && (key >> 4) < cbest[2]) best[2] = best[2] - 7 + (key & 15);
  }
  __syncthreads();
  const int r2b = best[2];
  if (tid == 0)
    a.data[(int64_t)img * tiles + tile] = (uint32_t)(uint8_t)g2r | (uint32_t)(uint8_t)g2b << 8 | (uint32_t)(uint8_t)r2b << 16;
  // applyColorTransformPixel (:497-507) over the thread's group, in place
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (!in[k]) continue;
    const int i = 4 * tid + k;
    const uint32_t p = px[k];
    const int gr = (p >> 8) & 0xff, rd = (p >> 16) & 0xff, bl = p & 0xff;
    const int nr = (rd - cc_delta(g2r, gr)) & 0xff;
    const int nb = (bl - cc_delta(g2b, gr) - cc_delta(r2b, rd)) & 0xff;
    base[(int64_t)(i / tw) * a.width + i % tw] = (p & 0xff00ff00u) | ((uint32_t)nr << 16) | (uint32_t)nb;
  }
}

struct CiArgs {
  const uint32_t* data;
  const uint32_t* src;
  uint32_t* dst;
  int64_t pitch;
  int width, height, bits, tiles_x;
};

// one thread per pixel; the tile's multipliers come from the (cached) data row
__global__ __launch_bounds__(256) void k_cc_inverse(CiArgs a, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t per = (int64_t)a.width * a.height;
  const int img = (int)(i / per);
  const int64_t r = i - img * per;
  const int y = (int)(r / a.width), x = (int)(r % a.width);
  const int tiles = a.tiles_x * ((a.height + (1 << a.bits) - 1) >> a.bits);
  const uint32_t code = a.data[(int64_t)img * tiles + (y >> a.bits) * a.tiles_x + (x >> a.bits)];
  const int g2r = (int8_t)code, g2b = (int8_t)(code >> 8), r2b = (int8_t)(code >> 16);
  const uint32_t p = a.src[img * a.pitch + r];
  const int green = (int8_t)(p >> 8);
  int red = (int)((p >> 16) & 0xff), blue = (int)(p & 0xff);
  red = (red + ((g2r * green) >> 5)) & 0xff;
  blue = (blue + ((g2b * green) >> 5) + ((r2b * (int)(int8_t)red) >> 5)) & 0xff;
  a.dst[img * a.pitch + r] = (p & 0xff00ff00u) | ((uint32_t)red << 16) | (uint32_t)blue;
}

struct IxArgs {
  const uint32_t* palette;
  const uint32_t* src;
  uint32_t* dst;
  int64_t src_pitch, dst_pitch;
  int palette_size, xbits, width, height, packed_w;
};

// one thread per output pixel: its packed word, its index bits, the palette
__global__ __launch_bounds__(256) void k_ci_inverse(IxArgs a, int64_t total) {
  __shared__ uint32_t pal[256];
  for (int k = threadIdx.x; k < a.palette_size; k += 256) pal[k] = a.palette[k];
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int64_t per = (int64_t)a.width * a.height;
  const int img = (int)(i / per);
  const int64_t r = i - img * per;
  const int y = (int)(r / a.width), x = (int)(r % a.width);
  const int bpp = 8 >> a.xbits;
  const uint32_t word = (a.src[img * a.src_pitch + (int64_t)y * a.packed_w + (x >> a.xbits)] >> 8) & 0xff;
  const uint32_t idx = bpp < 8 ? (word >> (bpp * (x & ((1 << a.xbits) - 1)))) & ((1u << bpp) - 1) : word;
  if ((int)idx < a.palette_size) a.dst[img * a.dst_pitch + r] = pal[idx];
}

}  // namespace

extern "C" int wg_vp8l_color_space_transform(uint32_t* argb, int32_t width, int32_t height, int64_t image_pitch,
                                             int32_t bits, int32_t n_images, uint32_t* data, void* stream) {
  WG_REQUIRE(argb && data && width > 0 && height > 0 && n_images > 0);
  WG_REQUIRE(bits >= 2 && bits <= 9 && image_pitch >= (int64_t)width * height);
  CcArgs a;
  a.argb = argb;
  a.data = data;
  a.pitch = image_pitch;
  a.width = width;
  a.height = height;
  a.bits = bits;
  a.tiles_x = (width + (1 << bits) - 1) >> bits;
  a.tiles_y = (height + (1 << bits) - 1) >> bits;
  const int64_t blocks = (int64_t)a.tiles_x * a.tiles_y * n_images;
  WG_REQUIRE(blocks < (1ll << 31));
  if (bits <= 5) {  // tiles of at most 1024 pixels: the packed-byte search
    hipLaunchKernelGGL(k_cc_select_q, dim3((unsigned)blocks), dim3(256), 0, wg::as_stream(stream), a);
    return wg::check_launch("k_cc_select_q");
  }
  hipLaunchKernelGGL(k_cc_select, dim3((unsigned)blocks), dim3(CC_THREADS), 0, wg::as_stream(stream), a);
  return wg::check_launch("k_cc_select");
}

extern "C" int wg_vp8l_color_space_inverse(const uint32_t* data, int32_t bits, int32_t width, int32_t height,
                                           int64_t image_pitch, int32_t n_images, const uint32_t* src, uint32_t* dst,
                                           void* stream) {
  WG_REQUIRE(data && src && dst && width > 0 && height > 0 && n_images > 0);
  WG_REQUIRE(bits >= 2 && bits <= 9 && image_pitch >= (int64_t)width * height);
  CiArgs a;
  a.data = data;
  a.src = src;
  a.dst = dst;
  a.pitch = image_pitch;
  a.width = width;
  a.height = height;
  a.bits = bits;
  a.tiles_x = (width + (1 << bits) - 1) >> bits;
  const int64_t total = (int64_t)width * height * n_images;
  hipLaunchKernelGGL(k_cc_inverse, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, wg::as_stream(stream), a, total);
  return wg::check_launch("k_cc_inverse");
}

extern "C" int wg_vp8l_color_index_inverse(const uint32_t* palette, int32_t palette_size, int32_t xbits, int32_t width,
                                           int32_t height, int32_t n_images, const uint32_t* src, int64_t src_pitch,
                                           uint32_t* dst, int64_t dst_pitch, void* stream) {
  WG_REQUIRE(palette && src && dst && width > 0 && height > 0 && n_images > 0);
  WG_REQUIRE(palette_size >= 1 && palette_size <= 256 && xbits >= 0 && xbits <= 3);
  const int packed_w = (width + (1 << xbits) - 1) >> xbits;
  WG_REQUIRE(src_pitch >= (int64_t)packed_w * height && dst_pitch >= (int64_t)width * height);
  IxArgs a;
  a.palette = palette;
  a.src = src;
  a.dst = dst;
  a.src_pitch = src_pitch;
  a.dst_pitch = dst_pitch;
  a.palette_size = palette_size;
  a.xbits = xbits;
  a.width = width;
  a.height = height;
  a.packed_w = packed_w;
  const int64_t total = (int64_t)width * height * n_images;
  hipLaunchKernelGGL(k_ci_inverse, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, wg::as_stream(stream), a, total);
  return wg::check_launch("k_ci_inverse");
}
