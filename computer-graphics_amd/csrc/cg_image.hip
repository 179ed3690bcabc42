// cg_image.hip -- texture loading: cv::imread(path, CV_LOAD_IMAGE_UNCHANGED)
// of the reference's JPEG maps (rasteriser/Source/skeleton.cpp:135-146).
//
// The reference's OpenCV 3.4 reads JPEGs through IJG libjpeg 9 with default
// parameters (islow IDCT, fancy upsampling).  libjpeg >= 7 then produces
// 2x-subsampled chroma by a 16x16 scaled IDCT instead of upsampling, so the
// decoded texels are a pure integer function of the coefficients; that is
// what this module computes (bit-identical to libjpeg 9, and pinned through
// rasteriser/screenshot.bmp, tests/test_rast_screenshot.py).
//
// Split: the entropy-coded segment is inherently sequential and is decoded
// on the host (baseline and progressive Huffman, ITU-T T.81 F.2 / G.1.2,
// restart markers) into one int16 coefficient plane per component; the
// coefficients go to the device in one copy and the sample work runs there:
//   jpeg_idct_kernel<S>  one 64-thread group per 4 (S = 2) or 8 (S = 1)
//                        blocks: dequantise + LL&M integer IDCT, 8x8 -> 8S x 8S,
//                        column pass into LDS, row pass to the plane
//   jpeg_colour_kernel   YCbCr -> BGR (libjpeg 9's fixed-point tables, computed
//                        inline), one thread per pixel
// Output is BGR bytes (gray for 1-component files), row-major, as imread
// returns them.  Unsupported inputs (arithmetic coding, 12-bit, lossless,
// sampling factors that libjpeg 9 would still upsample) return CG_E_INVALID.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "cg_internal.h"

namespace cg {
void *ctx_buf(cg_ctx *c, int which, size_t bytes, hipError_t *e);
hipStream_t ctx_stream(cg_ctx *c);
int ctx_invalid(cg_ctx *c, const char *what);
int ctx_fail(cg_ctx *c, hipError_t e, const char *what);
int ctx_device(cg_ctx *c);
}  // namespace cg

namespace {

using namespace cg;

// T.81 Figure A.6 zig-zag -> natural index, plus guard entries for runs past 63.
constexpr int kZigzag[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// ------------------------------------------------------------ host: entropy

struct HuffTable {
    bool present = false;
    bool dc_ok = false;   // every symbol <= 15: usable as a DC table (libjpeg jdhuff.c)
    // lookahead: the next 9 bits -> (length << 8 | symbol), 0 = longer code
    uint16_t fast[512];
    int32_t maxcode[18], valoff[17];
    uint8_t vals[256];
    // false for an over-subscribed code or one using an all-ones code word
    // (libjpeg jdhuff.c jpeg_make_d_derived_tbl: code >= 2^len is JERR_BAD_HUFF_TABLE)
    bool build(const uint8_t *counts, const uint8_t *symbols, int total)
    {
        present = false;
        memset(vals, 0, sizeof(vals));
        memcpy(vals, symbols, (size_t)total);
        memset(fast, 0, sizeof(fast));
        dc_ok = true;
        for (int i = 0; i < total; ++i) dc_ok &= symbols[i] <= 15;
        int code = 0, k = 0;
        for (int len = 1; len <= 16; ++len) {
            valoff[len] = k - code;
            if (counts[len - 1] && code + counts[len - 1] >= (1 << len)) return false;
            for (int i = 0; i < counts[len - 1]; ++i, ++code, ++k)
                if (len <= 9) {
                    int lo = code << (9 - len), hi = (code + 1) << (9 - len);
                    for (int b = lo; b < hi; ++b) fast[b] = (uint16_t)((len << 8) | vals[k]);
                }
            maxcode[len] = counts[len - 1] ? code - 1 : -1;
            code <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        present = true;
        return true;
    }
};

class BitReader {
  public:
    BitReader(const uint8_t *p, const uint8_t *end) : p_(p), end_(end) {}
    const uint8_t *pos() const { return p_; }
    // Skip to just after the next RSTn marker and reset (restart interval).
    void restart()
    {
        while (p_ + 1 < end_ && !(p_[0] == 0xFF && p_[1] >= 0xD0 && p_[1] <= 0xD7)) ++p_;
        if (p_ + 1 < end_) p_ += 2;
        acc_ = 0;
        n_ = 0;
        marker_ = false;
    }
    uint32_t peek(int k)
    {
        refill();
        return (uint32_t)(acc_ >> (64 - k));
    }
    void skip(int k)
    {
        acc_ <<= k;
        n_ -= k;
    }
    int bits(int k)
    {
        if (!k) return 0;
        int v = (int)peek(k);
        skip(k);
        return v;
    }
    int decode(const HuffTable &t)
    {
        uint16_t f = t.fast[peek(9)];
        if (f) {
            skip(f >> 8);
            return f & 0xFF;
        }
        uint32_t look = peek(16);
        for (int len = 10; len <= 16; ++len) {
            int code = (int)(look >> (16 - len));
            if (code <= t.maxcode[len]) {
                skip(len);
                return t.vals[t.valoff[len] + code];
            }
        }
        skip(16);
        return 0;   // corrupt data: libjpeg substitutes 0 as well
    }

  private:
    void refill()
    {
        while (n_ <= 56) {
            uint64_t byte = 0;
            if (!marker_ && p_ < end_) {
                if (p_[0] != 0xFF) {
                    byte = *p_++;
                } else if (p_ + 1 < end_ && p_[1] == 0x00) {
                    byte = 0xFF;
                    p_ += 2;
                } else {
                    marker_ = true;   // a marker ends the segment: zeros from here on
                }
            }
            acc_ |= byte << (56 - n_);
            n_ += 8;
        }
    }
    const uint8_t *p_, *end_;
    uint64_t acc_ = 0;
    int n_ = 0;
    bool marker_ = false;
};

inline int extend(int v, int s) { return (s && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v; }

struct Component {
    int id, h, v, tq;
    int blocks_x, blocks_y;   // coefficient plane, padded to whole MCUs
    int samp_w, samp_h;       // component size in samples
    int scale;                // IDCT output = 8 * scale per block side (1 or 2)
    bool latched = false;     // quantisation table copied at its first scan (libjpeg jdinput.c)
    uint16_t q[64] = {};
    std::vector<int16_t> coef;
    int pred = 0;
    int16_t *block(int bx, int by) { return coef.data() + ((size_t)by * blocks_x + bx) * 64; }
};

struct JpegFrame {
    int width = 0, height = 0, ncomp = 0;
    bool progressive = false, adobe_rgb = false;
    int hmax = 1, vmax = 1, mcus_x = 0, mcus_y = 0, restart = 0;
    uint16_t quant[4][64] = {};   // natural order
    bool quant_present[4] = {};
    HuffTable dc[4], ac[4];
    Component comp[3];
    int eobrun = 0;
};

inline int be16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

class JpegDecoder {
  public:
    explicit JpegDecoder(JpegFrame &f) : f_(f) {}
    // -> 0, or an error message
    const char *parse(const uint8_t *data, size_t n, bool header_only);

  private:
    const char *frame(const uint8_t *p, int len, int marker);
    const char *scan(const uint8_t *&p, const uint8_t *end);
    void block_seq(BitReader &br, Component &c, int16_t *b, const HuffTable &dct, const HuffTable &act);
    void block_dc(BitReader &br, Component &c, int16_t *b, const HuffTable &dct, int ah, int al);
    void block_ac_first(BitReader &br, int16_t *b, const HuffTable &act, int ss, int se, int al);
    void block_ac_refine(BitReader &br, int16_t *b, const HuffTable &act, int ss, int se, int al);
    JpegFrame &f_;
    bool have_frame_ = false;
};

const char *JpegDecoder::frame(const uint8_t *p, int len, int marker)
{
    if (have_frame_) return "duplicate JPEG frame header";
    if (len < 8) return "truncated JPEG frame header";
    if (p[2] != 8) return "only 8-bit JPEG is supported";
    f_.progressive = marker == 0xC2;
    f_.height = be16(p + 3);
    f_.width = be16(p + 5);
    f_.ncomp = p[7];
    if (f_.ncomp != 1 && f_.ncomp != 3) return "only 1- or 3-component JPEG is supported";
    if (len < 8 + 3 * f_.ncomp) return "truncated JPEG frame header";
    if (f_.width <= 0 || f_.height <= 0) return "bad JPEG dimensions";
    for (int i = 0; i < f_.ncomp; ++i) {
        Component &c = f_.comp[i];
        c.id = p[8 + 3 * i];
        c.h = p[9 + 3 * i] >> 4;
        c.v = p[9 + 3 * i] & 15;
        c.tq = p[10 + 3 * i];
        if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) return "bad JPEG component";
        f_.hmax = std::max(f_.hmax, c.h);
        f_.vmax = std::max(f_.vmax, c.v);
    }
    f_.mcus_x = (f_.width + 8 * f_.hmax - 1) / (8 * f_.hmax);
    f_.mcus_y = (f_.height + 8 * f_.vmax - 1) / (8 * f_.vmax);
    for (int i = 0; i < f_.ncomp; ++i) {
        Component &c = f_.comp[i];
        c.samp_w = (f_.width * c.h + f_.hmax - 1) / f_.hmax;
        c.samp_h = (f_.height * c.v + f_.vmax - 1) / f_.vmax;
        if (f_.ncomp == 1) {
            c.blocks_x = (c.samp_w + 7) / 8;
            c.blocks_y = (c.samp_h + 7) / 8;
        } else {
            c.blocks_x = f_.mcus_x * c.h;
            c.blocks_y = f_.mcus_y * c.v;
        }
        // libjpeg >= 7 (jdmaster.c): a 2:1 sampling ratio is absorbed by a 16-point IDCT
        int sx = (f_.hmax % (2 * c.h) == 0) ? 2 : 1, sy = (f_.vmax % (2 * c.v) == 0) ? 2 : 1;
        if (sx != sy || c.h * sx != f_.hmax || c.v * sy != f_.vmax)
            return "JPEG sampling factors need upsampling (unsupported)";
        c.scale = sx;
        c.coef.assign((size_t)c.blocks_x * c.blocks_y * 64, 0);
    }
    have_frame_ = true;
    return nullptr;
}

void JpegDecoder::block_seq(BitReader &br, Component &c, int16_t *b, const HuffTable &dct, const HuffTable &act)
{
    int s = br.decode(dct);
    c.pred += extend(br.bits(s), s);
    b[0] = (int16_t)c.pred;
    for (int k = 1; k < 64; ++k) {
        int rs = br.decode(act), r = rs >> 4;
        s = rs & 15;
        if (s) {
            k += r;
            b[kZigzag[k]] = (int16_t)extend(br.bits(s), s);
        } else if (r == 15) {
            k += 15;
        } else {
            break;
        }
    }
}

void JpegDecoder::block_dc(BitReader &br, Component &c, int16_t *b, const HuffTable &dct, int ah, int al)
{
    if (ah == 0) {
        int s = br.decode(dct);
        c.pred += extend(br.bits(s), s);
        b[0] = (int16_t)(c.pred * (1 << al));
    } else if (br.bits(1)) {
        b[0] = (int16_t)(b[0] | (1 << al));
    }
}

void JpegDecoder::block_ac_first(BitReader &br, int16_t *b, const HuffTable &act, int ss, int se, int al)
{
    if (f_.eobrun > 0) {
        --f_.eobrun;
        return;
    }
    for (int k = ss; k <= se; ++k) {
        int rs = br.decode(act), r = rs >> 4, s = rs & 15;
        if (s) {
            k += r;
            b[kZigzag[k]] = (int16_t)(extend(br.bits(s), s) * (1 << al));
        } else if (r == 15) {
            k += 15;
        } else {
            f_.eobrun = (1 << r) + br.bits(r) - 1;   // this block ends the band now
            break;
        }
    }
}

// T.81 G.1.2.3: correction bits for nonzero history, new +-1 coefficients.
void JpegDecoder::block_ac_refine(BitReader &br, int16_t *b, const HuffTable &act, int ss, int se, int al)
{
    const int p1 = 1 << al, m1 = -(1 << al);
    auto correct = [&](int16_t &cf) {
        if (br.bits(1) && (cf & p1) == 0) cf = (int16_t)(cf >= 0 ? cf + p1 : cf + m1);
    };
    int k = ss;
    if (f_.eobrun == 0) {
        for (; k <= se; ++k) {
            int rs = br.decode(act), r = rs >> 4, s = rs & 15, val = 0;
            if (s) {
                val = br.bits(1) ? p1 : m1;
            } else if (r != 15) {
                f_.eobrun = (1 << r) + br.bits(r);
                break;
            }
            // skip r zero-history coefficients (correcting the nonzero ones on the way)
            for (; k <= se; ++k) {
                int16_t &cf = b[kZigzag[k]];
                if (cf != 0) correct(cf);
                else if (r-- == 0) break;
            }
            if (val) b[kZigzag[k]] = (int16_t)val;
        }
    }
    if (f_.eobrun > 0) {
        for (; k <= se; ++k) {
            int16_t &cf = b[kZigzag[k]];
            if (cf != 0) correct(cf);
        }
        --f_.eobrun;
    }
}

const char *JpegDecoder::scan(const uint8_t *&p, const uint8_t *end)
{
    int len = be16(p);
    if (len < 3) return "bad JPEG scan header";
    int ns = p[2];
    if (ns < 1 || ns > f_.ncomp || len != 6 + 2 * ns) return "bad JPEG scan header";
    Component *sc[4];
    const HuffTable *dct[4], *act[4];
    for (int i = 0; i < ns; ++i) {
        int id = p[3 + 2 * i], t = p[4 + 2 * i];
        sc[i] = nullptr;
        for (int k = 0; k < f_.ncomp; ++k)
            if (f_.comp[k].id == id) sc[i] = &f_.comp[k];
        if (!sc[i] || (t >> 4) > 3 || (t & 15) > 3) return "bad JPEG scan component";
        dct[i] = &f_.dc[t >> 4];
        act[i] = &f_.ac[t & 15];
    }
    int ss = p[3 + 2 * ns], se = p[4 + 2 * ns], ah = p[5 + 2 * ns] >> 4, al = p[5 + 2 * ns] & 15;
    if (!f_.progressive) ss = 0, se = 63, ah = al = 0;
    else if (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1) || al > 13)
        return "bad progressive scan parameters";
    // the tables the scan decodes with must exist (libjpeg: JERR_NO_HUFF_TABLE,
    // JERR_NO_QUANT_TABLE); a DC table's symbols are magnitude categories <= 15
    for (int i = 0; i < ns; ++i) {
        const bool need_dc = ss == 0 && ah == 0, need_ac = se > 0;
        if (need_dc && (!dct[i]->present || !dct[i]->dc_ok)) return "JPEG scan uses an undefined DC table";
        if (need_ac && !act[i]->present) return "JPEG scan uses an undefined AC table";
        Component &c = *sc[i];
        if (!c.latched) {
            if (!f_.quant_present[c.tq]) return "JPEG component uses an undefined quantisation table";
            memcpy(c.q, f_.quant[c.tq], sizeof(c.q));
            c.latched = true;
        }
    }
    p += len;
    BitReader br(p, end);
    for (int i = 0; i < ns; ++i) sc[i]->pred = 0;
    f_.eobrun = 0;
    int todo = f_.restart;
    auto maybe_restart = [&]() {
        if (f_.restart && todo-- == 0) {
            br.restart();
            for (int i = 0; i < ns; ++i) sc[i]->pred = 0;
            f_.eobrun = 0;
            todo = f_.restart - 1;
        }
    };
    auto one = [&](int i, int16_t *b) {
        if (!f_.progressive) block_seq(br, *sc[i], b, *dct[i], *act[i]);
        else if (ss == 0) block_dc(br, *sc[i], b, *dct[i], ah, al);
        else if (ah == 0) block_ac_first(br, b, *act[i], ss, se, al);
        else block_ac_refine(br, b, *act[i], ss, se, al);
    };
    if (ns == 1) {
        Component &c = *sc[0];
        int nbx = (c.samp_w + 7) / 8, nby = (c.samp_h + 7) / 8;
        for (int by = 0; by < nby; ++by)
            for (int bx = 0; bx < nbx; ++bx) {
                maybe_restart();
                one(0, c.block(bx, by));
            }
    } else {
        for (int my = 0; my < f_.mcus_y; ++my)
            for (int mx = 0; mx < f_.mcus_x; ++mx) {
                maybe_restart();
                for (int i = 0; i < ns; ++i)
                    for (int v = 0; v < sc[i]->v; ++v)
                        for (int h = 0; h < sc[i]->h; ++h) one(i, sc[i]->block(mx * sc[i]->h + h, my * sc[i]->v + v));
            }
    }
    // continue after the entropy-coded segment: the next marker other than RSTn
    p = br.pos();
    while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0x00 && !(p[1] >= 0xD0 && p[1] <= 0xD7))) ++p;
    return nullptr;
}

const char *JpegDecoder::parse(const uint8_t *data, size_t n, bool header_only)
{
    const uint8_t *p = data, *end = data + n;
    if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) return "not a JPEG file";
    p += 2;
    while (p + 2 <= end) {
        if (p[0] != 0xFF) {
            ++p;
            continue;
        }
        int m = p[1];
        if (m == 0xFF) {
            ++p;
            continue;
        }
        p += 2;
        if (m == 0xD9) break;
        if (m >= 0xD0 && m <= 0xD7) continue;
        if (p + 2 > end) return "truncated JPEG";
        int len = be16(p);
        if (len < 2 || p + len > end) return "truncated JPEG segment";
        if (m == 0xDB) {
            for (const uint8_t *q = p + 2; q < p + len;) {
                int prec = q[0] >> 4, id = q[0] & 15;
                if (id > 3 || prec > 1) return "bad JPEG quantisation table";
                if (q + 1 + (prec ? 128 : 64) > p + len) return "truncated JPEG quantisation table";
                for (int k = 0; k < 64; ++k) f_.quant[id][kZigzag[k]] = (uint16_t)(prec ? be16(q + 1 + 2 * k) : q[1 + k]);
                f_.quant_present[id] = true;
                q += 1 + (prec ? 128 : 64);
            }
        } else if (m == 0xC4) {
            for (const uint8_t *q = p + 2; q < p + len;) {
                int cls = q[0] >> 4, id = q[0] & 15, total = 0;
                if (cls > 1 || id > 3) return "bad JPEG Huffman table";
                if (q + 17 > p + len) return "truncated JPEG Huffman table";
                for (int l = 0; l < 16; ++l) total += q[1 + l];
                if (total > 256) return "bad JPEG Huffman table";
                if (q + 17 + total > p + len) return "truncated JPEG Huffman table";
                if (!(cls ? f_.ac[id] : f_.dc[id]).build(q + 1, q + 17, total)) return "bad JPEG Huffman table";
                q += 17 + total;
            }
        } else if (m == 0xDD) {
            if (len < 4) return "truncated JPEG restart interval";
            f_.restart = be16(p + 2);
        } else if (m == 0xEE && len >= 14 && !memcmp(p + 2, "Adobe", 5)) {
            f_.adobe_rgb = p[13] == 0;
        } else if (m == 0xC0 || m == 0xC1 || m == 0xC2) {
            if (const char *e = frame(p, len, m)) return e;
            if (header_only) return nullptr;
        } else if (m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            return "lossless / arithmetic / hierarchical JPEG is not supported";
        } else if (m == 0xDA) {
            if (!have_frame_) return "JPEG scan before frame header";
            if (const char *e = scan(p, end)) return e;
            continue;
        }
        p += len;
    }
    return have_frame_ ? nullptr : "JPEG without a frame header";
}

// ---------------------------------------------------------- device: samples

constexpr int kConstBits = 13, kPass1Bits = 2;
constexpr int64_t fix13(double x) { return (int64_t)(x * (1 << kConstBits) + 0.5); }

struct QuantTables {
    uint16_t q[3][64];
};

// libjpeg 9's IDCT range limit: table index (v + 512) & 1023, clamped to 0..255
__device__ __forceinline__ uint32_t idct_limit(int64_t v)
{
    int s = (int)(v & 1023) - 384;
    return (uint32_t)min(max(s, 0), 255);
}

// 8-point LL&M kernel (jidctint.c jpeg_idct_islow); `even0` is the DC term
// already shifted up by CONST_BITS and carrying the pass's rounding/centre.
__device__ __forceinline__ void idct8(const int64_t x[8], int64_t even0, int64_t o[8])
{
    int64_t z1, z2, z3, t0, t1, t2, t3, t10, t11, t12, t13;
    z3 = x[4] * (1 << kConstBits);
    t0 = even0 + z3;
    t1 = even0 - z3;
    z2 = x[2];
    z3 = x[6];
    z1 = (z2 + z3) * fix13(0.541196100);
    t2 = z1 + z2 * fix13(0.765366865);
    t3 = z1 - z3 * fix13(1.847759065);
    t10 = t0 + t2;
    t13 = t0 - t2;
    t11 = t1 + t3;
    t12 = t1 - t3;
    t0 = x[7];
    t1 = x[5];
    t2 = x[3];
    t3 = x[1];
    z2 = t0 + t2;
    z3 = t1 + t3;
    z1 = (z2 + z3) * fix13(1.175875602);
    z2 = z2 * -fix13(1.961570560) + z1;
    z3 = z3 * -fix13(0.390180644) + z1;
    z1 = (t0 + t3) * -fix13(0.899976223);
    t0 = t0 * fix13(0.298631336) + z1 + z2;
    t3 = t3 * fix13(1.501321110) + z1 + z3;
    z1 = (t1 + t2) * -fix13(2.562915447);
    t1 = t1 * fix13(2.053119869) + z1 + z3;
    t2 = t2 * fix13(3.072711026) + z1 + z2;
    o[0] = t10 + t3; o[7] = t10 - t3;
    o[1] = t11 + t2; o[6] = t11 - t2;
    o[2] = t12 + t1; o[5] = t12 - t1;
    o[3] = t13 + t0; o[4] = t13 - t0;
}

// 16-point kernel of jpeg_idct_16x16 (cK = sqrt(2) cos(K pi / 32)).
__device__ __forceinline__ void idct16(const int64_t x[8], int64_t even0, int64_t o[16])
{
    int64_t t0, t1, t2, t3, t10, t11, t12, t13, t20, t21, t22, t23, t24, t25, t26, t27, z1, z2, z3, z4;
    t1 = x[4] * fix13(1.306562965);
    t2 = x[4] * fix13(0.541196100);
    t10 = even0 + t1;
    t11 = even0 - t1;
    t12 = even0 + t2;
    t13 = even0 - t2;
    z1 = x[2];
    z2 = x[6];
    z3 = z1 - z2;
    z4 = z3 * fix13(0.275899379);
    z3 = z3 * fix13(1.387039845);
    t0 = z3 + z2 * fix13(2.562915447);
    t1 = z4 + z1 * fix13(0.899976223);
    t2 = z3 - z1 * fix13(0.601344887);
    t3 = z4 - z2 * fix13(0.509795579);
    t20 = t10 + t0; t27 = t10 - t0;
    t21 = t12 + t1; t26 = t12 - t1;
    t22 = t13 + t2; t25 = t13 - t2;
    t23 = t11 + t3; t24 = t11 - t3;
    z1 = x[1];
    z2 = x[3];
    z3 = x[5];
    z4 = x[7];
    t11 = z1 + z3;
    t1 = (z1 + z2) * fix13(1.353318001);
    t2 = t11 * fix13(1.247225013);
    t3 = (z1 + z4) * fix13(1.093201867);
    t10 = (z1 - z4) * fix13(0.897167586);
    t11 = t11 * fix13(0.666655658);
    t12 = (z1 - z2) * fix13(0.410524528);
    t0 = t1 + t2 + t3 - z1 * fix13(2.286341144);
    t13 = t10 + t11 + t12 - z1 * fix13(1.835730603);
    int64_t w = (z2 + z3) * fix13(0.138617169);
    t1 += w + z2 * fix13(0.071888074);
    t2 += w - z3 * fix13(1.125726048);
    w = (z3 - z2) * fix13(1.407403738);
    t11 += w - z3 * fix13(0.766367282);
    t12 += w + z2 * fix13(1.971951411);
    z2 += z4;
    w = z2 * -fix13(0.666655658);
    t1 += w;
    t3 += w + z4 * fix13(1.065388962);
    w = z2 * -fix13(1.247225013);
    t10 += w + z4 * fix13(3.141271809);
    t12 += w;
    w = (z3 + z4) * -fix13(1.353318001);
    t2 += w;
    t3 += w;
    w = (z4 - z3) * fix13(0.410524528);
    t10 += w;
    t11 += w;
    o[0] = t20 + t0;  o[15] = t20 - t0;
    o[1] = t21 + t1;  o[14] = t21 - t1;
    o[2] = t22 + t2;  o[13] = t22 - t2;
    o[3] = t23 + t3;  o[12] = t23 - t3;
    o[4] = t24 + t10; o[11] = t24 - t10;
    o[5] = t25 + t11; o[10] = t25 - t11;
    o[6] = t26 + t12; o[9] = t26 - t12;
    o[7] = t27 + t13; o[8] = t27 - t13;
}

// Blocks of one component -> its sample plane (row stride `pitch`).  S = 1:
// 8x8 IDCT, 8 blocks per 64-thread group (8 threads per block); S = 2: the
// 16x16 scaled IDCT, 4 blocks per group (16 threads per block).  Pass 1
// (columns, 8 threads per block) goes through LDS to pass 2 (8S rows).
template <int S>
__global__ __launch_bounds__(64) void jpeg_idct_kernel(const int16_t *__restrict__ coef, int blocks_x, int blocks_y,
                                                       QuantTables qt, int comp, uint8_t *__restrict__ plane,
                                                       int pitch)
{
    constexpr int N = 8 * S, TPB = N, BPG = 64 / TPB;
    __shared__ int ws[BPG][N * 8];
    const int lane = threadIdx.x % TPB, slot = threadIdx.x / TPB;
    const long blk = (long)blockIdx.x * BPG + slot;
    const bool live = blk < (long)blocks_x * blocks_y;
    const int16_t *in = coef + (live ? blk : 0) * 64;
    const uint16_t *q = qt.q[comp];
    if (live && lane < 8) {
        int64_t x[8], o[N];
        for (int k = 0; k < 8; ++k) x[k] = (int64_t)in[k * 8 + lane] * q[k * 8 + lane];
        const int64_t even0 = x[0] * (1 << kConstBits) + (1 << (kConstBits - kPass1Bits - 1));
        if constexpr (S == 1) idct8(x, even0, o);
        else idct16(x, even0, o);
        for (int r = 0; r < N; ++r) ws[slot][r * 8 + lane] = (int)(o[r] >> (kConstBits - kPass1Bits));
    }
    __syncthreads();
    if (!live) return;
    int64_t x[8], o[N];
    for (int k = 0; k < 8; ++k) x[k] = ws[slot][lane * 8 + k];
    const int64_t even0 = (x[0] + ((512 << (kPass1Bits + 3)) + (1 << (kPass1Bits + 2)))) * (1 << kConstBits);
    if constexpr (S == 1) idct8(x, even0, o);
    else idct16(x, even0, o);
    const int bx = (int)(blk % blocks_x), by = (int)(blk / blocks_x);
    uint32_t *dst = reinterpret_cast<uint32_t *>(plane + (size_t)(by * N + lane) * pitch + (size_t)bx * N);
    for (int k = 0; k < N; k += 4) {
        const int sh = kConstBits + kPass1Bits + 3;
        dst[k / 4] = idct_limit(o[k] >> sh) | idct_limit(o[k + 1] >> sh) << 8 | idct_limit(o[k + 2] >> sh) << 16 |
                     idct_limit(o[k + 3] >> sh) << 24;
    }
}

constexpr int64_t fix16(double x) { return (int64_t)(x * 65536.0 + 0.5); }

__device__ __forceinline__ uint8_t clamp_u8(int v) { return (uint8_t)min(max(v, 0), 255); }

// jdcolor.c (libjpeg 9) ycc_rgb_convert, then OpenCV's RGB -> BGR order.
__global__ void jpeg_colour_kernel(const uint8_t *__restrict__ planes, int pitch, size_t plane_bytes, int w, int h,
                                   int ncomp, int adobe_rgb, uint8_t *__restrict__ out)
{
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)w * h) return;
    const int x = (int)(i % w), y = (int)(i / w);
    const size_t o = (size_t)y * pitch + x;
    const int Y = planes[o];
    if (ncomp == 1) {
        out[i] = (uint8_t)Y;
        return;
    }
    const int c1 = planes[plane_bytes + o], c2 = planes[2 * plane_bytes + o];
    int R, G, B;
    if (adobe_rgb) {
        R = Y, G = c1, B = c2;
    } else {
        const int64_t cb = c1 - 128, cr = c2 - 128, half = 1 << 15;
        R = Y + (int)((fix16(1.402) * cr + half) >> 16);
        G = Y + (int)((-fix16(0.344136286) * cb + half + -fix16(0.714136286) * cr) >> 16);
        B = Y + (int)((fix16(1.772) * cb + half) >> 16);
    }
    out[3 * i + 0] = clamp_u8(B);
    out[3 * i + 1] = clamp_u8(G);
    out[3 * i + 2] = clamp_u8(R);
}

int decode_into(cg_ctx *c, const uint8_t *data, size_t n, uint8_t *d_out, size_t cap, hipStream_t st,
                bool to_host, uint8_t *h_out)
{
    JpegFrame f;
    JpegDecoder dec(f);
    if (const char *e = dec.parse(data, n, false)) return ctx_invalid(c, e);
    const size_t out_bytes = (size_t)f.width * f.height * f.ncomp;
    if (cap < out_bytes) {
        (void)ctx_invalid(c, "jpeg: output capacity too small");
        return CG_E_CAPACITY;
    }
    // device layout: [coef comp 0 | comp 1 | comp 2][planes 0..2 (pitch x rows)][out if host]
    const int pitch = f.ncomp == 1 ? f.comp[0].blocks_x * 8 : f.mcus_x * f.hmax * 8;
    const int rows = f.ncomp == 1 ? f.comp[0].blocks_y * 8 : f.mcus_y * f.vmax * 8;
    const size_t plane_bytes = (size_t)pitch * rows;
    size_t coef_bytes = 0, coef_off[3];
    for (int i = 0; i < f.ncomp; ++i) {
        coef_off[i] = coef_bytes;
        coef_bytes += f.comp[i].coef.size() * sizeof(int16_t);
    }
    coef_bytes = (coef_bytes + 255) & ~(size_t)255;
    const size_t need = coef_bytes + plane_bytes * f.ncomp + (to_host ? out_bytes : 0);
    hipError_t e = hipSuccess;
    uint8_t *scratch = static_cast<uint8_t *>(ctx_buf(c, 17, need, &e));
    if (!scratch) return ctx_fail(c, e, "jpeg scratch");
    for (int i = 0; i < f.ncomp; ++i)
        if ((e = hipMemcpyAsync(scratch + coef_off[i], f.comp[i].coef.data(), f.comp[i].coef.size() * 2,
                                hipMemcpyHostToDevice, st)) != hipSuccess)
            return ctx_fail(c, e, "jpeg coefficient upload");
    QuantTables qt;
    // a component no scan reached keeps a zero table (libjpeg jddctmgr.c:
    // its multipliers stay zero, the samples mid-grey)
    for (int i = 0; i < f.ncomp; ++i) memcpy(qt.q[i], f.comp[i].q, sizeof(qt.q[i]));
    uint8_t *planes = scratch + coef_bytes;
    for (int i = 0; i < f.ncomp; ++i) {
        const Component &cp = f.comp[i];
        const long nb = (long)cp.blocks_x * cp.blocks_y;
        const int16_t *cf = reinterpret_cast<const int16_t *>(scratch + coef_off[i]);
        if (cp.scale == 1)
            hipLaunchKernelGGL(jpeg_idct_kernel<1>, dim3((unsigned)((nb + 7) / 8)), dim3(64), 0, st, cf,
                               cp.blocks_x, cp.blocks_y, qt, i, planes + i * plane_bytes, pitch);
        else
            hipLaunchKernelGGL(jpeg_idct_kernel<2>, dim3((unsigned)((nb + 3) / 4)), dim3(64), 0, st, cf,
                               cp.blocks_x, cp.blocks_y, qt, i, planes + i * plane_bytes, pitch);
    }
    uint8_t *dst = to_host ? planes + plane_bytes * f.ncomp : d_out;
    const long npx = (long)f.width * f.height;
    hipLaunchKernelGGL(jpeg_colour_kernel, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, st, planes, pitch,
                       plane_bytes, f.width, f.height, f.ncomp, f.adobe_rgb ? 1 : 0, dst);
    if ((e = hipGetLastError()) != hipSuccess) return ctx_fail(c, e, "jpeg kernels");
    if (to_host) {
        if ((e = hipMemcpyAsync(h_out, dst, out_bytes, hipMemcpyDeviceToHost, st)) != hipSuccess ||
            (e = hipStreamSynchronize(st)) != hipSuccess)
            return ctx_fail(c, e, "jpeg download");
    }
    return CG_OK;
}

}  // namespace

extern "C" int cg_image_jpeg_info(const uint8_t *data, size_t n, int *width, int *height, int *channels)
{
    if (!data || !width || !height || !channels) return CG_E_INVALID;
    JpegFrame f;
    JpegDecoder dec(f);
    if (dec.parse(data, n, true) || f.width == 0) return CG_E_INVALID;
    *width = f.width;
    *height = f.height;
    *channels = f.ncomp;
    return CG_OK;
}

extern "C" int cg_image_jpeg_check(const uint8_t *data, size_t n)
{
    if (!data) return CG_E_INVALID;
    JpegFrame f;
    JpegDecoder dec(f);
    return dec.parse(data, n, false) ? CG_E_INVALID : CG_OK;
}

extern "C" int cg_image_decode_jpeg(cg_ctx *ctx, const uint8_t *data, size_t n, uint8_t *out, size_t cap)
{
    if (!ctx || !data || !out) return CG_E_INVALID;
    hipError_t e = hipSetDevice(ctx_device(ctx));
    if (e != hipSuccess) return ctx_fail(ctx, e, "hipSetDevice");
    return decode_into(ctx, data, n, nullptr, cap, ctx_stream(ctx), true, out);
}

extern "C" int cg_image_decode_jpeg_device(cg_ctx *ctx, const uint8_t *data, size_t n, uint8_t *d_out, size_t cap,
                                           void *stream)
{
    if (!ctx || !data || !d_out) return CG_E_INVALID;
    hipError_t e = hipSetDevice(ctx_device(ctx));
    if (e != hipSuccess) return ctx_fail(ctx, e, "hipSetDevice");
    return decode_into(ctx, data, n, d_out, cap, stream ? (hipStream_t)stream : ctx_stream(ctx), false, nullptr);
}
