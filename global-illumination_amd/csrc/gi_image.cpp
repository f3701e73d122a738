// gi_image.cpp -- gi_write_image: R2Image::Write (R2Image.cpp:316-339) for the renderer's 8-bit
// RGB output. rgb rows are R2Image rows (row 0 = bottom, R2Image.cpp:205-208); every format
// below stores the top row first except BMP and RAW, as the reference's writers do.
//   .png        R2Image::WritePNG  (:1389-1466)   zlib, 8-bit RGB
//   .ppm        R2Image::WritePPM(ascii = 1) (:767-846)  P3 text, four pixels per line
//   .pgm        R2Image::WritePPM(ascii = 0)       P5 bytes, (int)(0.30 r + 0.59 g + 0.11 b)
//   .bmp        R2Image::WriteBMP  (:541-620)    24-bit BI_RGB, bottom-up, BGR, rows padded to 4 B
//   .jpg/.jpeg  R2Image::WriteJPEG (:1094-1163)  the vendored IJG libjpeg with quality 75,
//               optimize_coding, JDCT_ISLOW and jpeg_set_defaults (JFIF 1.01, YCbCr 4:2:0):
//               restated below from that library's algorithms (jccolor.c, jcsample.c,
//               jcprepct.c, jfdctint.c, jcdctmgr.c, jcparam.c, jchuff.c, jcmarker.c)
//   .raw        R2Image::WriteRAW  (:1545-1604)  {54321, w, h, 3} header + planar f32 / 255
//   .tif/.tiff  the reference is built without RN_USE_TIFF: "TIFF not supported" -> error
#include <zlib.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>
#include "../../include/gi.h"

namespace {

// ---- JPEG -------------------------------------------------------------------------------------
// zig-zag scan position -> natural (row-major) coefficient index
const int kNatural[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                          12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                          35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                          58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// ITU T.81 Annex K.1 example tables (jcparam.c's std tables), natural order
const int kLumQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                       14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                       18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                       49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const int kChrQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                       24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                       99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                       99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

// jpeg_set_quality(q, force_baseline = TRUE): jpeg_quality_scaling + jpeg_add_quant_table
void quant_table(const int *basic, int quality, int *out) {
  int s = quality <= 0 ? 1 : (quality > 100 ? 100 : quality);
  s = s < 50 ? 5000 / s : 200 - 2 * s;
  for (int i = 0; i < 64; i++) {
    long t = ((long)basic[i] * s + 50L) / 100L;
    if (t <= 0) t = 1;
    if (t > 255) t = 255;
    out[i] = (int)t;
  }
}

// jfdctint.c jpeg_fdct_islow: LL&M integer DCT, CONST_BITS 13, PASS1_BITS 2; output scaled by 8
inline int32_t descale(int32_t x, int n) { return (x + (1 << (n - 1))) >> n; }
void fdct_islow(int32_t *d) {
  const int CB = 13, P1 = 2;
  const int32_t c0298 = 2446, c0390 = 3196, c0541 = 4433, c0765 = 6270, c0899 = 7373,
                c1175 = 9633, c1501 = 12299, c1847 = 15137, c1961 = 16069, c2053 = 16819,
                c2562 = 20995, c3072 = 25172;
  for (int pass = 0; pass < 2; pass++) {
    const int st = pass == 0 ? 1 : 8;    // element stride inside a row / column
    const int adv = pass == 0 ? 8 : 1;   // next row / column
    for (int k = 0; k < 8; k++) {
      int32_t *p = d + k * adv;
      int32_t t0 = p[0] + p[7 * st], t7 = p[0] - p[7 * st];
      int32_t t1 = p[st] + p[6 * st], t6 = p[st] - p[6 * st];
      int32_t t2 = p[2 * st] + p[5 * st], t5 = p[2 * st] - p[5 * st];
      int32_t t3 = p[3 * st] + p[4 * st], t4 = p[3 * st] - p[4 * st];
      int32_t t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
      if (pass == 0) {
        p[0] = (t10 + t11) << P1;
        p[4 * st] = (t10 - t11) << P1;
      } else {
        p[0] = descale(t10 + t11, P1);
        p[4 * st] = descale(t10 - t11, P1);
      }
      const int sh = pass == 0 ? CB - P1 : CB + P1;
      int32_t z1 = (t12 + t13) * c0541;
      p[2 * st] = descale(z1 + t13 * c0765, sh);
      p[6 * st] = descale(z1 + t12 * -c1847, sh);
      z1 = t4 + t7;
      int32_t z2 = t5 + t6, z3 = t4 + t6, z4 = t5 + t7;
      const int32_t z5 = (z3 + z4) * c1175;
      t4 *= c0298; t5 *= c2053; t6 *= c3072; t7 *= c1501;
      z1 *= -c0899; z2 *= -c2562; z3 *= -c1961; z4 *= -c0390;
      z3 += z5;
      z4 += z5;
      p[7 * st] = descale(t4 + z1 + z3, sh);
      p[5 * st] = descale(t5 + z2 + z4, sh);
      p[3 * st] = descale(t6 + z2 + z3, sh);
      p[st] = descale(t7 + z1 + z4, sh);
    }
  }
}

// one component plane, padded to whole MCUs by edge replication
struct Plane {
  int w = 0, h = 0;
  std::vector<uint8_t> v;
  uint8_t at(int x, int y) const { return v[(size_t)y * w + x]; }
};

struct HuffTable {
  uint8_t bits[17] = {0};
  std::vector<uint8_t> vals;
  uint32_t code[256] = {0};
  uint8_t size[256] = {0};
};

// jchuff.c jpeg_gen_optimal_table (ITU T.81 K.2), then the canonical codes
// (jpeg_make_c_derived_tbl)
void optimal_table(long *freq, HuffTable &t) {
  int codesize[257] = {0}, others[257];
  uint8_t bits[33] = {0};
  for (int i = 0; i < 257; i++) others[i] = -1;
  freq[256] = 1;
  for (;;) {
    int c1 = -1, c2 = -1;
    long v = 1000000000L;
    for (int i = 0; i <= 256; i++)
      if (freq[i] && freq[i] <= v) { v = freq[i]; c1 = i; }
    v = 1000000000L;
    for (int i = 0; i <= 256; i++)
      if (freq[i] && freq[i] <= v && i != c1) { v = freq[i]; c2 = i; }
    if (c2 < 0) break;
    freq[c1] += freq[c2];
    freq[c2] = 0;
    codesize[c1]++;
    while (others[c1] >= 0) { c1 = others[c1]; codesize[c1]++; }
    others[c1] = c2;
    codesize[c2]++;
    while (others[c2] >= 0) { c2 = others[c2]; codesize[c2]++; }
  }
  for (int i = 0; i <= 256; i++)
    if (codesize[i]) bits[codesize[i]]++;
  int i = 32;
  for (; i > 16; i--)
    while (bits[i] > 0) {
      int j = i - 2;
      while (bits[j] == 0) j--;
      bits[i] -= 2;
      bits[i - 1]++;
      bits[j + 1] += 2;
      bits[j]--;
    }
  while (bits[i] == 0) i--;
  bits[i]--;
  memcpy(t.bits, bits, 17);
  t.vals.clear();
  for (int l = 1; l <= 32; l++)
    for (int s = 0; s <= 255; s++)
      if (codesize[s] == l) t.vals.push_back((uint8_t)s);
  uint32_t code = 0;
  size_t k = 0;
  for (int l = 1; l <= 16; l++) {
    for (int n = 0; n < t.bits[l]; n++, k++) {
      t.code[t.vals[k]] = code++;
      t.size[t.vals[k]] = (uint8_t)l;
    }
    code <<= 1;
  }
}

inline int nbits(int v) {
  int n = 0;
  for (v = v < 0 ? -v : v; v; v >>= 1) n++;
  return n;
}

struct BitWriter {
  std::vector<uint8_t> out;
  uint32_t acc = 0;
  int n = 0;
  void put(uint32_t code, int size) {
    for (int b = size - 1; b >= 0; b--) {
      acc = (acc << 1) | ((code >> b) & 1u);
      if (++n == 8) {
        out.push_back((uint8_t)acc);
        if (acc == 0xff) out.push_back(0);  // byte stuffing
        acc = 0;
        n = 0;
      }
    }
  }
  void flush() {  // pad with 1 bits (jchuff.c flush_bits: emit_bits(0x7F, 7))
    if (n) put(0x7f, 8 - n);
  }
};

int write_jpeg(FILE *fp, int W, int H, const uint8_t *rgb) {
  // colour conversion (jccolor.c rgb_ycc_convert: 16-bit fixed point tables)
  auto fix = [](double x) { return (int32_t)(x * 65536.0 + 0.5); };
  const int32_t half = 1 << 15, cbcr = 128 << 16;
  const int W16 = (W + 15) / 16 * 16, H16 = (H + 15) / 16 * 16;
  Plane Y, Cb, Cr;
  Y.w = W16; Y.h = H16;
  Y.v.resize((size_t)W16 * H16);
  std::vector<uint8_t> cbf((size_t)W16 * H16), crf((size_t)W16 * H16);
  for (int y = 0; y < H16; y++) {
    // JPEG row y = image row from the top; past the image: the last row (jcprepct.c
    // expand_bottom_edge), past the right edge: the last column (jcsample.c expand_right_edge)
    const int ry = H - 1 - (y < H ? y : H - 1);
    for (int x = 0; x < W16; x++) {
      const uint8_t *p = rgb + ((size_t)ry * W + (x < W ? x : W - 1)) * 3;
      const int r = p[0], g = p[1], b = p[2];
      const size_t o = (size_t)y * W16 + x;
      Y.v[o] = (uint8_t)((fix(0.29900) * r + fix(0.58700) * g + fix(0.11400) * b + half) >> 16);
      cbf[o] = (uint8_t)((-fix(0.16874) * r - fix(0.33126) * g + fix(0.5) * b + cbcr + half - 1) >> 16);
      crf[o] = (uint8_t)((fix(0.5) * r - fix(0.41869) * g - fix(0.08131) * b + cbcr + half - 1) >> 16);
    }
  }
  // 2x2 downsampling with the alternating bias 1, 2, 1, ... per output row (jcsample.c
  // h2v2_downsample); the padded input makes every chroma sample of the MCU grid defined
  Cb.w = Cr.w = W16 / 2;
  Cb.h = Cr.h = H16 / 2;
  Cb.v.resize((size_t)Cb.w * Cb.h);
  Cr.v.resize((size_t)Cr.w * Cr.h);
  // rows: from the input rows (an odd last row paired with its copy) up to ceil(H/2), then
  // copies of the last computed row (jcprepct.c pads each component to the iMCU height by
  // repeating its last row); columns: from the input replicated out to W16 (jcsample.c
  // expand_right_edge before downsampling)
  const int ch = (H + 1) / 2;
  for (int y = 0; y < Cb.h; y++)
    for (int x = 0, bias = 1; x < Cb.w; x++, bias ^= 3) {
      const int ys = y < ch ? y : ch - 1;
      const size_t a = (size_t)(2 * ys) * W16 + 2 * x, b = a + W16;
      Cb.v[(size_t)y * Cb.w + x] = (uint8_t)((cbf[a] + cbf[a + 1] + cbf[b] + cbf[b + 1] + bias) >> 2);
      Cr.v[(size_t)y * Cr.w + x] = (uint8_t)((crf[a] + crf[a + 1] + crf[b] + crf[b + 1] + bias) >> 2);
    }
  int q[2][64];
  quant_table(kLumQ, 75, q[0]);
  quant_table(kChrQ, 75, q[1]);
  // forward DCT + quantisation (jcdctmgr.c forward_DCT: divisor = 8 q, rounded division of the
  // magnitude) of every block, in MCU order: Y00 Y01 Y10 Y11 Cb Cr
  const int mx = W16 / 16, my = H16 / 16;
  std::vector<int16_t> coef((size_t)mx * my * 6 * 64);
  auto block = [&](const Plane &P, int bx, int by, const int *qt, int16_t *outc) {
    int32_t d[64];
    for (int r = 0; r < 8; r++)
      for (int c = 0; c < 8; c++) d[r * 8 + c] = (int32_t)P.at(bx * 8 + c, by * 8 + r) - 128;
    fdct_islow(d);
    for (int i = 0; i < 64; i++) {
      const int32_t qv = qt[i] << 3;
      int32_t t = d[i];
      if (t < 0) {
        t = -t + (qv >> 1);
        t = t >= qv ? t / qv : 0;
        t = -t;
      } else {
        t += qv >> 1;
        t = t >= qv ? t / qv : 0;
      }
      outc[i] = (int16_t)t;
    }
  };
  // Y blocks past ceil(W/8) x ceil(H/8) are libjpeg's dummy blocks (jccoefct.c compress_data):
  // zero AC, the DC of the block before them (left neighbour at the right edge, the MCU's
  // previous block for a bottom row). The chroma MCU is one block: always real.
  const int ybw = (W + 7) / 8, ybh = (H + 7) / 8;
  auto dummy = [](int16_t *outc, int dc) {
    memset(outc, 0, 64 * sizeof(int16_t));
    outc[0] = (int16_t)dc;
  };
  for (int j = 0; j < my; j++)
    for (int i = 0; i < mx; i++) {
      int16_t *c = &coef[((size_t)j * mx + i) * 6 * 64];
      block(Y, 2 * i, 2 * j, q[0], c);
      if (2 * i + 1 < ybw) block(Y, 2 * i + 1, 2 * j, q[0], c + 64);
      else dummy(c + 64, c[0]);
      if (2 * j + 1 < ybh) {
        block(Y, 2 * i, 2 * j + 1, q[0], c + 128);
        if (2 * i + 1 < ybw) block(Y, 2 * i + 1, 2 * j + 1, q[0], c + 192);
        else dummy(c + 192, c[128]);
      } else {
        dummy(c + 128, c[64]);
        dummy(c + 192, c[64]);
      }
      block(Cb, i, j, q[1], c + 256);
      block(Cr, i, j, q[1], c + 320);
    }
  // symbol statistics (jchuff.c encode_mcu_gather) -> optimal tables, then the entropy pass
  auto walk = [&](auto &&emit_dc, auto &&emit_ac) {
    int last[3] = {0, 0, 0};
    for (size_t m = 0; m < (size_t)mx * my; m++)
      for (int b = 0; b < 6; b++) {
        const int ci = b < 4 ? 0 : b - 3;
        const int tb = ci == 0 ? 0 : 1;
        const int16_t *c = &coef[(m * 6 + b) * 64];
        const int diff = c[0] - last[ci];
        last[ci] = c[0];
        emit_dc(tb, diff);
        int run = 0;
        for (int k = 1; k < 64; k++) {
          const int v = c[kNatural[k]];
          if (v == 0) { run++; continue; }
          while (run > 15) { emit_ac(tb, 0xf0, 0); run -= 16; }
          emit_ac(tb, (run << 4) | nbits(v), v);
          run = 0;
        }
        if (run > 0) emit_ac(tb, 0x00, 0);
      }
  };
  long fdc[2][257] = {{0}}, fac[2][257] = {{0}};
  walk([&](int tb, int diff) { fdc[tb][nbits(diff)]++; },
       [&](int tb, int sym, int) { fac[tb][sym]++; });
  HuffTable hdc[2], hac[2];
  for (int t = 0; t < 2; t++) {
    optimal_table(fdc[t], hdc[t]);
    optimal_table(fac[t], hac[t]);
  }
  BitWriter bw;
  auto put_value = [&](int v, int n) {  // the low n bits of v, ones' complement when negative
    if (n) bw.put((uint32_t)(v < 0 ? v - 1 : v) & ((1u << n) - 1u), n);
  };
  walk([&](int tb, int diff) {
         const int n = nbits(diff);
         bw.put(hdc[tb].code[n], hdc[tb].size[n]);
         put_value(diff, n);
       },
       [&](int tb, int sym, int v) {
         bw.put(hac[tb].code[sym], hac[tb].size[sym]);
         put_value(v, sym & 15);
       });
  bw.flush();
  // markers (jcmarker.c): SOI, JFIF APP0 1.01, DQT x2, SOF0, DHT x4, SOS, data, EOI
  std::vector<uint8_t> o;
  auto b1 = [&](int v) { o.push_back((uint8_t)v); };
  auto b2 = [&](int v) { b1(v >> 8); b1(v & 255); };
  b2(0xffd8);
  b2(0xffe0); b2(16);
  b1('J'); b1('F'); b1('I'); b1('F'); b1(0);
  b1(1); b1(1); b1(0); b2(1); b2(1); b1(0); b1(0);
  for (int t = 0; t < 2; t++) {
    b2(0xffdb); b2(67); b1(t);
    for (int k = 0; k < 64; k++) b1(q[t][kNatural[k]]);
  }
  b2(0xffc0); b2(17); b1(8); b2(H); b2(W); b1(3);
  b1(1); b1(0x22); b1(0);
  b1(2); b1(0x11); b1(1);
  b1(3); b1(0x11); b1(1);
  auto dht = [&](const HuffTable &t, int cls_index) {
    b2(0xffc4);
    b2(2 + 1 + 16 + (int)t.vals.size());
    b1(cls_index);
    for (int l = 1; l <= 16; l++) b1(t.bits[l]);
    for (uint8_t v : t.vals) b1(v);
  };
  dht(hdc[0], 0x00); dht(hac[0], 0x10);
  dht(hdc[1], 0x01); dht(hac[1], 0x11);
  b2(0xffda); b2(12); b1(3);
  b1(1); b1(0x00);
  b1(2); b1(0x11);
  b1(3); b1(0x11);
  b1(0); b1(63); b1(0);
  o.insert(o.end(), bw.out.begin(), bw.out.end());
  b2(0xffd9);
  return fwrite(o.data(), 1, o.size(), fp) == o.size() ? GI_OK : GI_ERR_IO;
}

}  // namespace

extern "C" {

int gi_write_image(const char *path, int w, int h, const uint8_t *rgb) {
  if (!path || !rgb || w <= 0 || h <= 0) return GI_ERR_ARG;
  const char *ext = strrchr(path, '.');
  if (!ext) return GI_ERR_ARG;
  const std::string e(ext);
  if (e.compare(0, 4, ".tif") == 0) return GI_ERR_UNSUPPORTED;  // "TIFF not supported"
  const bool known = e.compare(0, 4, ".png") == 0 || e.compare(0, 4, ".ppm") == 0 ||
                     e.compare(0, 4, ".pgm") == 0 || e.compare(0, 4, ".bmp") == 0 ||
                     e.compare(0, 4, ".jpg") == 0 || e.compare(0, 5, ".jpeg") == 0 ||
                     e.compare(0, 4, ".raw") == 0;
  if (!known) return GI_ERR_UNSUPPORTED;
  FILE *fp = fopen(path, e.compare(0, 4, ".ppm") == 0 ? "w" : "wb");
  if (!fp) return GI_ERR_IO;
  int rc = GI_OK;
  auto row = [&](int r) { return rgb + (size_t)r * w * 3; };  // R2Image row r (0 = bottom)
  if (e.compare(0, 4, ".ppm") == 0) {
    fprintf(fp, "P3\n%d %d\n255\n", w, h);
    for (int j = h - 1; j >= 0; j--) {
      for (int i = 0; i < w; i++) {
        const uint8_t *p = row(j) + 3 * i;
        fprintf(fp, "%-3d %-3d %-3d  ", p[0], p[1], p[2]);
        if (((i + 1) % 4) == 0) fprintf(fp, "\n");
      }
      if ((w % 4) != 0) fprintf(fp, "\n");
    }
    fprintf(fp, "\n");
  } else if (e.compare(0, 4, ".pgm") == 0) {
    fprintf(fp, "P5\n%d %d\n255\n", w, h);
    for (int j = h - 1; j >= 0; j--)
      for (int i = 0; i < w; i++) {
        const uint8_t *p = row(j) + 3 * i;
        fputc((int)(0.30 * p[0] + 0.59 * p[1] + 0.11 * p[2]), fp);
      }
  } else if (e.compare(0, 4, ".bmp") == 0) {
    const int rowsize = (3 * w + 3) / 4 * 4;
    auto le = [&](uint32_t v, int n) { for (int k = 0; k < n; k++) fputc((v >> (8 * k)) & 255, fp); };
    const uint32_t off = 14 + 40;
    le(0x4d42, 2); le(off + (uint32_t)rowsize * h, 4); le(0, 2); le(0, 2); le(off, 4);
    le(40, 4); le((uint32_t)w, 4); le((uint32_t)h, 4); le(1, 2); le(24, 2); le(0, 4);
    le((uint32_t)rowsize * h, 4); le(2925, 4); le(2925, 4); le(0, 4); le(0, 4);
    for (int j = 0; j < h; j++) {
      for (int i = 0; i < w; i++) {
        const uint8_t *p = row(j) + 3 * i;
        fputc(p[2], fp); fputc(p[1], fp); fputc(p[0], fp);
      }
      for (int k = 3 * w; k < rowsize; k++) fputc(0, fp);
    }
  } else if (e.compare(0, 4, ".raw") == 0) {
    const uint32_t hd[4] = {54321u, (uint32_t)w, (uint32_t)h, 3u};
    fwrite(hd, 4, 4, fp);
    std::vector<float> buf(w);
    for (int c = 0; c < 3; c++)
      for (int j = 0; j < h; j++) {
        for (int i = 0; i < w; i++) buf[i] = row(j)[3 * i + c] / 255.0F;
        fwrite(buf.data(), 4, w, fp);
      }
  } else if (e.compare(0, 4, ".jpg") == 0 || e.compare(0, 5, ".jpeg") == 0) {
    rc = write_jpeg(fp, w, h, rgb);
  } else {  // .png (R2Image.cpp:1430: rows written top first)
    auto be32 = [](uint8_t *p, uint32_t v) { p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v; };
    auto chunk = [&](const char *type, const uint8_t *data, size_t n) {
      uint8_t hd[8];
      be32(hd, (uint32_t)n);
      memcpy(hd + 4, type, 4);
      fwrite(hd, 1, 8, fp);
      if (n) fwrite(data, 1, n, fp);
      uLong crc = crc32(0, (const Bytef *)type, 4);
      if (n) crc = crc32(crc, data, (uInt)n);
      uint8_t cb[4];
      be32(cb, (uint32_t)crc);
      fwrite(cb, 1, 4, fp);
    };
    const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    fwrite(sig, 1, 8, fp);
    uint8_t ihdr[13] = {0};
    be32(ihdr, w);
    be32(ihdr + 4, h);
    ihdr[8] = 8;
    ihdr[9] = 2;
    chunk("IHDR", ihdr, 13);
    std::vector<uint8_t> raw;
    raw.reserve((size_t)(w * 3 + 1) * h);
    for (int r = 0; r < h; r++) {
      raw.push_back(0);
      raw.insert(raw.end(), row(h - 1 - r), row(h - 1 - r) + (size_t)w * 3);
    }
    uLongf zl = compressBound(raw.size());
    std::vector<uint8_t> z(zl);
    compress2(z.data(), &zl, raw.data(), raw.size(), 6);
    chunk("IDAT", z.data(), zl);
    chunk("IEND", nullptr, 0);
  }
  if (fclose(fp) != 0 && rc == GI_OK) rc = GI_ERR_IO;
  return rc;
}

}  // extern "C"
