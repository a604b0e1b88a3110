/* TEST INFRASTRUCTURE ONLY: the entropy-decoding half of the reference's VP8L
 * decoder, restated in C so the parity tests can feed real VP8L bitstreams
 * (the reference's own testdata/ files) to the GPU inverse transforms.
 *
 * The lossless entropy coder is outside the hot path; this file
 * stops where the hot path starts: it returns the entropy-decoded pixel array
 * (before any inverse transform) and each transform's parameters and
 * sub-image, in bitstream order.  The inverse transforms themselves are the
 * hot path (A25, §8(f)#3) and are applied by the caller -- lossless.c on the
 * CPU, libwebpgpu.so on the GPU.
 *
 * Follows internal/lossless/:
 *   decode.go:199-222 (decodeHeader), :227-289 (decodeImageStream),
 *   :293-331 (decodeSubImage);
 *   decode_transform.go:23-79 (readTransform), :81-109 (expandColorMap);
 *   decode_image.go:13-83 (readHuffmanCodeLengths), :86-166 (readHuffmanCode),
 *   :175-333 (readHuffmanCodes), :368-392 (meta index), :394-410 (copy
 *   distance / length), :451-713 (decodeImageData);
 *   huffman.go:76-235 (canonical code construction);
 *   constants.go:98-160 (code-length order, alphabet sizes, CodeToPlane,
 *   PlaneCodeToDistance); colorcache.go:29-37 (hash, insert).
 * Huffman decoding here walks the canonical code bit by bit instead of the
 * reference's two-level tables; for a valid stream both read the same
 * symbols with the same bit counts.  The colour cache is updated pixel by
 * pixel; the reference's deferred insertion (lastCached) flushes before every
 * lookup, so both see the same cache contents.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

enum { NUM_LITERAL = 256, NUM_LENGTH = 24, NUM_DISTANCE = 40, CL_CODES = 19, MAX_LEN = 15 };

static const int kCodeLengthOrder[CL_CODES] = {17, 18, 0, 1, 2, 3, 4, 5, 16, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
static const int kAlphabetBase[5] = {NUM_LITERAL + NUM_LENGTH, NUM_LITERAL, NUM_LITERAL, NUM_LITERAL, NUM_DISTANCE};
static const uint8_t kCodeToPlane[120] = {
    0x18, 0x07, 0x17, 0x19, 0x28, 0x06, 0x27, 0x29, 0x16, 0x1a, 0x26, 0x2a, 0x38, 0x05, 0x37, 0x39, 0x15, 0x1b,
    0x36, 0x3a, 0x25, 0x2b, 0x48, 0x04, 0x47, 0x49, 0x14, 0x1c, 0x35, 0x3b, 0x46, 0x4a, 0x24, 0x2c, 0x58, 0x45,
    0x4b, 0x34, 0x3c, 0x03, 0x57, 0x59, 0x13, 0x1d, 0x56, 0x5a, 0x23, 0x2d, 0x44, 0x4c, 0x55, 0x5b, 0x33, 0x3d,
    0x68, 0x02, 0x67, 0x69, 0x12, 0x1e, 0x66, 0x6a, 0x22, 0x2e, 0x54, 0x5c, 0x43, 0x4d, 0x65, 0x6b, 0x32, 0x3e,
    0x78, 0x01, 0x77, 0x79, 0x53, 0x5d, 0x11, 0x1f, 0x64, 0x6c, 0x42, 0x4e, 0x76, 0x7a, 0x21, 0x2f, 0x75, 0x7b,
    0x31, 0x3f, 0x63, 0x6d, 0x52, 0x5e, 0x00, 0x74, 0x7c, 0x41, 0x4f, 0x10, 0x20, 0x62, 0x6e, 0x30, 0x73, 0x7d,
    0x51, 0x5f, 0x40, 0x72, 0x7e, 0x61, 0x6f, 0x50, 0x71, 0x7f, 0x60, 0x70};

typedef struct {
  const uint8_t* buf;
  size_t len;
  size_t bitpos;
  int eos;
} BitReader;

static uint32_t read_bits(BitReader* br, int n) {  // LSB first (bitio LosslessReader)
  uint32_t v = 0;
  for (int i = 0; i < n; i++) {
    const size_t byte = br->bitpos >> 3;
    if (byte >= br->len) {
      br->eos = 1;
      return 0;
    }
    v |= (uint32_t)((br->buf[byte] >> (br->bitpos & 7)) & 1) << i;
    br->bitpos++;
  }
  return v;
}

/* Canonical Huffman code (huffman.go:76-235): codes assigned by length, then
 * symbol; the first bit read is the code's most significant bit. */
typedef struct {
  int count[MAX_LEN + 1];
  int first[MAX_LEN + 1];  // first code of each length
  int offset[MAX_LEN + 1];  // index into sym of that code
  int* sym;
  int single;  // >= 0: the only symbol, read with zero bits
} Huff;

static int huff_build(Huff* h, const int* lengths, int n) {
  memset(h->count, 0, sizeof h->count);
  h->sym = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
  h->single = -1;
  int nonzero = 0, last = -1;
  for (int i = 0; i < n; i++) {
    if (lengths[i] < 0 || lengths[i] > MAX_LEN) return -1;
    if (lengths[i] > 0) {
      h->count[lengths[i]]++;
      nonzero++;
      last = i;
    }
  }
  if (nonzero == 0) return -1;
  if (nonzero == 1) {  // huffman.go: a lone symbol takes zero bits
    h->single = last;
    return 0;
  }
  int code = 0, idx = 0;
  for (int len = 1; len <= MAX_LEN; len++) {
    h->first[len] = code;
    h->offset[len] = idx;
    idx += h->count[len];
    code = (code + h->count[len]) << 1;
  }
  int fill[MAX_LEN + 1];
  memcpy(fill, h->offset, sizeof fill);
  for (int i = 0; i < n; i++)
    if (lengths[i] > 0) h->sym[fill[lengths[i]]++] = i;
  return 0;
}

static void huff_free(Huff* h) {
  free(h->sym);
  h->sym = NULL;
}

static int huff_read(const Huff* h, BitReader* br) {
  if (h->single >= 0) return h->single;
  int code = 0;
  for (int len = 1; len <= MAX_LEN; len++) {
    code |= (int)read_bits(br, 1);
    const int k = code - h->first[len];
    if (k >= 0 && k < h->count[len]) return h->sym[h->offset[len] + k];
    code <<= 1;
  }
  br->eos = 1;
  return 0;
}

/* readHuffmanCode (decode_image.go:86-166) + readHuffmanCodeLengths (:13-83) */
static int read_huffman_code(BitReader* br, int alphabet, Huff* out) {
  int* lengths = (int*)calloc((size_t)alphabet, sizeof(int));
  int rc = 0;
  if (read_bits(br, 1)) {  // simple code: one or two symbols
    const int nsym = (int)read_bits(br, 1) + 1;
    const int first_bits = read_bits(br, 1) ? 8 : 1;
    const int s0 = (int)read_bits(br, first_bits);
    if (s0 >= alphabet) rc = -1;
    else lengths[s0] = 1;
    if (nsym == 2) {
      const int s1 = (int)read_bits(br, 8);
      if (s1 >= alphabet) rc = -1;
      else lengths[s1] = 1;
    }
  } else {
    int cl_len[CL_CODES] = {0};
    int ncodes = (int)read_bits(br, 4) + 4;
    if (ncodes > CL_CODES) ncodes = CL_CODES;
    for (int i = 0; i < ncodes; i++) cl_len[kCodeLengthOrder[i]] = (int)read_bits(br, 3);
    Huff cl;
    if (huff_build(&cl, cl_len, CL_CODES) < 0) {
      huff_free(&cl);
      free(lengths);
      return -1;
    }
    int max_symbol = alphabet;
    if (read_bits(br, 1)) {
      const int nbits = 2 + 2 * (int)read_bits(br, 3);
      max_symbol = 2 + (int)read_bits(br, nbits);
      if (max_symbol > alphabet) rc = -1;
    }
    int prev = 8;  // DefaultCodeLength
    for (int s = 0; rc == 0 && s < alphabet && max_symbol-- > 0;) {
      const int c = huff_read(&cl, br);
      if (c < 16) {
        lengths[s++] = c;
        if (c != 0) prev = c;
      } else {
        static const int extra[3] = {2, 3, 7}, base[3] = {3, 3, 11};
        const int n = (int)read_bits(br, extra[c - 16]) + base[c - 16];
        if (s + n > alphabet) {
          rc = -1;
          break;
        }
        for (int i = 0; i < n; i++) lengths[s++] = c == 16 ? prev : 0;
      }
    }
    huff_free(&cl);
  }
  if (rc == 0 && !br->eos) rc = huff_build(out, lengths, alphabet);
  else rc = -1;
  free(lengths);
  return rc;
}

typedef struct {
  int cache_bits;
  int meta_bits;  // 0: one group
  int meta_xsize;
  uint32_t* meta;  // group index per meta tile
  int ngroups;
  Huff* groups;  // 5 per group
} Level;

static void level_free(Level* L) {
  for (int i = 0; i < 5 * L->ngroups; i++) huff_free(&L->groups[i]);
  free(L->groups);
  free(L->meta);
}

static int subsample(int size, int bits) { return (size + (1 << bits) - 1) >> bits; }

static int decode_image_data(BitReader* br, const Level* L, uint32_t* data, int width, int height);

/* decodeImageStream + decodeSubImage (decode.go:227-331) for a level without
 * transforms; `allow_meta` only on level 0. */
static int read_level(BitReader* br, int xsize, int ysize, int allow_meta, Level* L) {
  memset(L, 0, sizeof *L);
  if (read_bits(br, 1)) {
    L->cache_bits = (int)read_bits(br, 4);
    if (L->cache_bits < 1 || L->cache_bits > 11) return -1;
  }
  int nmax = 1;
  if (allow_meta && read_bits(br, 1)) {  // readHuffmanCodes :181-231
    L->meta_bits = 2 + (int)read_bits(br, 3);
    L->meta_xsize = subsample(xsize, L->meta_bits);
    const int mh = subsample(ysize, L->meta_bits);
    Level sub;
    if (read_level(br, L->meta_xsize, mh, 0, &sub) < 0) return -1;
    L->meta = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)L->meta_xsize * mh);
    const int rc = decode_image_data(br, &sub, L->meta, L->meta_xsize, mh);
    level_free(&sub);
    if (rc < 0) return -1;
    for (int i = 0; i < L->meta_xsize * mh; i++) {
      L->meta[i] = (L->meta[i] >> 8) & 0xffff;
      if ((int)L->meta[i] + 1 > nmax) nmax = (int)L->meta[i] + 1;
    }
  }
  L->ngroups = nmax;
  L->groups = (Huff*)calloc((size_t)5 * nmax, sizeof(Huff));
  for (int g = 0; g < nmax; g++)
    for (int j = 0; j < 5; j++) {
      const int alphabet = kAlphabetBase[j] + (j == 0 && L->cache_bits ? 1 << L->cache_bits : 0);
      if (read_huffman_code(br, alphabet, &L->groups[5 * g + j]) < 0) return -1;
    }
  return br->eos ? -1 : 0;
}

static int copy_value(int sym, BitReader* br) {  // getCopyDistance / getCopyLength (:394-410)
  if (sym < 4) return sym + 1;
  const int extra = (sym - 2) >> 1;
  const int offset = (2 + (sym & 1)) << extra;
  return offset + (int)read_bits(br, extra) + 1;
}

static int plane_to_distance(int xsize, int code) {  // PlaneCodeToDistance (constants.go:150-170)
  if (code > 120) return code - 120;
  const int d = kCodeToPlane[code - 1];
  const int dist = (d >> 4) * xsize + 8 - (d & 0xf);
  return dist < 1 ? 1 : dist;
}

/* decodeImageData (decode_image.go:451-713) */
static int decode_image_data(BitReader* br, const Level* L, uint32_t* data, int width, int height) {
  const int total = width * height;
  uint32_t* cache = L->cache_bits ? (uint32_t*)calloc((size_t)1 << L->cache_bits, sizeof(uint32_t)) : NULL;
  const int shift = 32 - L->cache_bits;
  int pos = 0, rc = 0;
#define CACHE_INSERT(v)                                      \
  do {                                                       \
    if (cache) cache[((uint32_t)(v)*0x1e35a7bdu) >> shift] = (v); \
  } while (0)
  while (pos < total) {
    const int x = pos % width, y = pos / width;
    const int g = L->meta_bits ? (int)L->meta[(y >> L->meta_bits) * L->meta_xsize + (x >> L->meta_bits)] : 0;
    const Huff* H = &L->groups[5 * g];
    const int code = huff_read(&H[0], br);
    if (code < NUM_LITERAL) {
      const uint32_t r = (uint32_t)huff_read(&H[1], br);
      const uint32_t b = (uint32_t)huff_read(&H[2], br);
      const uint32_t a = (uint32_t)huff_read(&H[3], br);
      const uint32_t v = a << 24 | r << 16 | (uint32_t)code << 8 | b;
      data[pos++] = v;
      CACHE_INSERT(v);
    } else if (code < NUM_LITERAL + NUM_LENGTH) {
      const int length = copy_value(code - NUM_LITERAL, br);
      const int dsym = huff_read(&H[4], br);
      const int dist = plane_to_distance(width, copy_value(dsym, br));
      if (dist > pos || pos + length > total) {
        rc = -1;
        break;
      }
      for (int i = 0; i < length; i++, pos++) {
        data[pos] = data[pos - dist];
        CACHE_INSERT(data[pos]);
      }
    } else {
      const int key = code - (NUM_LITERAL + NUM_LENGTH);
      if (!cache || key >= (1 << L->cache_bits)) {
        rc = -1;
        break;
      }
      const uint32_t v = cache[key];
      data[pos++] = v;
      CACHE_INSERT(v);
    }
    if (br->eos) {
      rc = -1;
      break;
    }
  }
#undef CACHE_INSERT
  free(cache);
  return rc;
}

/* expandColorMap (decode_transform.go:81-109): per-byte delta decoding into
 * 1 << (8 >> bits) entries, the rest zero. */
static void expand_color_map(const uint32_t* pal, int ncolors, int bits, uint32_t* out) {
  const int final_n = 1 << (8 >> bits);
  memset(out, 0, sizeof(uint32_t) * (size_t)final_n);
  out[0] = pal[0];
  for (int i = 1; i < ncolors; i++) {
    uint32_t v = 0;
    for (int c = 0; c < 4; c++) {
      const uint32_t s = ((pal[i] >> (8 * c)) + (out[i - 1] >> (8 * c))) & 0xff;
      v |= s << (8 * c);
    }
    out[i] = v;
  }
}

/* One call does the whole parse.  The VP8L payload (after the chunk header,
 * starting with the 0x2f signature byte) is decoded; info receives the size,
 * the transforms in bitstream order (type, bits, the width they apply to, the
 * word count of their data) and the working width.  When `pixels` is non-NULL
 * it receives the entropy-decoded image (tw x height words); tdata[k], when
 * non-NULL, transform k's data (predictor modes / cross-colour multipliers:
 * the sub-image; colour indexing: the expanded palette of 1 << (8 >> bits)
 * entries).  Returns 0, or -1 on a malformed stream. */
int or_vp8l_decode(const uint8_t* payload, size_t len, or_vp8l_info* info, uint32_t* pixels, uint32_t** tdata) {
  memset(info, 0, sizeof *info);
  if (len < 5 || payload[0] != 0x2f) return -1;
  BitReader br = {payload + 1, len - 1, 0, 0};
  info->width = (int)read_bits(&br, 14) + 1;  // decodeHeader (decode.go:199-222)
  info->height = (int)read_bits(&br, 14) + 1;
  info->has_alpha = (int)read_bits(&br, 1);
  if (read_bits(&br, 3) != 0) return -1;
  int xsize = info->width;
  const int ysize = info->height;
  uint32_t seen = 0;
  while (read_bits(&br, 1)) {  // readTransform (decode_transform.go:23-79)
    if (info->n_transforms >= 4) return -1;
    const int k = info->n_transforms++;
    const int type = (int)read_bits(&br, 2);
    if (seen & (1u << type)) return -1;
    seen |= 1u << type;
    info->type[k] = type;
    info->xsize[k] = xsize;
    if (type == 0 || type == 1) {
      info->bits[k] = 2 + (int)read_bits(&br, 3);
      const int sw = subsample(xsize, info->bits[k]), sh = subsample(ysize, info->bits[k]);
      Level L;
      uint32_t* d = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)sw * sh);
      int rc = read_level(&br, sw, sh, 0, &L);
      if (rc == 0) rc = decode_image_data(&br, &L, d, sw, sh);
      level_free(&L);
      if (rc == 0 && tdata && tdata[k]) memcpy(tdata[k], d, sizeof(uint32_t) * (size_t)sw * sh);
      free(d);
      if (rc < 0) return -1;
      info->dsize[k] = sw * sh;
    } else if (type == 3) {
      const int ncolors = (int)read_bits(&br, 8) + 1;
      const int bits = ncolors > 16 ? 0 : ncolors > 4 ? 1 : ncolors > 2 ? 2 : 3;
      info->bits[k] = bits;
      uint32_t pal[256];
      Level L;
      int rc = read_level(&br, ncolors, 1, 0, &L);
      if (rc == 0) rc = decode_image_data(&br, &L, pal, ncolors, 1);
      level_free(&L);
      if (rc < 0) return -1;
      info->dsize[k] = 1 << (8 >> bits);
      if (tdata && tdata[k]) expand_color_map(pal, ncolors, bits, tdata[k]);
      xsize = subsample(xsize, bits);
    }
  }
  info->tw = xsize;
  Level L;
  int rc = read_level(&br, xsize, ysize, 1, &L);
  if (rc == 0 && pixels) rc = decode_image_data(&br, &L, pixels, xsize, ysize);
  level_free(&L);
  return rc;
}
