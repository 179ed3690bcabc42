/*
 * cg_oracle_jpeg.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Restatement of the texture loader the reference's rasteriser calls at
 * start-up: cv::imread(path, CV_LOAD_IMAGE_UNCHANGED)
 * (rasteriser/Source/skeleton.cpp:135-146).  The reference was built on macOS
 * against Homebrew OpenCV 3.4.1_5 (skeleton.cpp:9), whose JPEG reader is IJG
 * libjpeg 9 (third-party, not in /root/reference).  What OpenCV 3.4's
 * JpegDecoder does with it: default decompression parameters (JDCT_ISLOW,
 * fancy upsampling on, block smoothing on), out_color_space JCS_RGB, then an
 * RGB -> BGR byte swap.  What libjpeg 9 does with those parameters, restated
 * from its published algorithm:
 *
 *  - entropy decoding per ITU-T T.81 (baseline/extended Huffman, and
 *    progressive: DC first/refine, AC first/refine with EOB runs, the
 *    refinement-scan correction bits, restart markers);
 *  - IDCT scaling instead of upsampling: with fancy upsampling on, libjpeg >= 7
 *    picks each component's DCT output size as 8 * s, s = 2 when
 *    max_samp_factor % (2 * samp_factor) == 0 (else 1), per direction
 *    (jdmaster.c jpeg_core_output_dimensions).  For 4:2:0 chroma that is the
 *    16x16 scaled IDCT (jidctint.c jpeg_idct_16x16), so the chroma planes come
 *    out at full resolution and the upsampler is 1:1.  (libjpeg-turbo / 6b
 *    instead decode chroma 8x8 and triangle-upsample -- that is why Pillow's
 *    texels differ by +-1 from the reference's.)
 *  - the LL&M integer IDCT (CONST_BITS 13, PASS1_BITS 2, raw quantisation
 *    multipliers) and libjpeg 9's range limiting ((v + 512) & 1023 then clamp);
 *  - YCbCr -> RGB with libjpeg 9's tables (Cr->R 1.402, Cb->B 1.772,
 *    Cr->G -0.714136286, Cb->G -0.344136286, SCALEBITS 16).
 *
 * Pinning: decoding the reference's Metal_Grill_002_* maps with this code and
 * rendering the state that produced rasteriser/screenshot.bmp reproduces every
 * screenshot pixel that does not depend on the missing marble map, bit for
 * bit (tests/test_rast_screenshot.py).  Cross-checked against the system's
 * libjpeg 9 where one is installed (scripts/jpeg_xcheck.c).
 *
 * Scope: 8-bit, 1 or 3 components, sampling factors whose libjpeg 9 output
 * needs no further upsampling (4:4:4, 4:2:0, grayscale); anything else, and
 * arithmetic coding, returns an error.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "cg_oracle.h"

/* ITU-T T.81 Figure A.6: zig-zag index -> natural (row-major) index. */
static const int ZZ[80] = {
    0,  1,  8, 16,  9,  2,  3, 10, 17, 24, 32, 25, 18, 11,  4,  5,
   12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,  6,  7, 14, 21, 28,
   35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
   58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
   /* guard entries (a corrupt run past Se lands here, like libjpeg's) */
   63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

typedef struct {
    int present;
    uint8_t bits[17];
    uint8_t vals[256];
    int32_t mincode[17], maxcode[18], valptr[17];
} huff;

typedef struct {
    int id, h, v, tq;
    int bw, bh;            /* blocks per row / column, padded to whole MCUs */
    int cw, ch;            /* component size in samples (ceil) */
    int16_t *coef;         /* bw * bh * 64, natural order */
    int dc_pred;
} comp;

typedef struct {
    const uint8_t *p, *end;
    uint32_t buf;
    int nbits;
    int hit_marker;
} bits;

typedef struct {
    int w, h, nc, progressive, hmax, vmax, mcux, mcuy, restart, adobe, adobe_transform;
    uint16_t q[4][64];     /* natural order */
    huff dc[4], ac[4];
    comp c[4];
    int eobrun;
} dec;

/* jdhuff.c (libjpeg 9) jpeg_make_d_derived_tbl: the codes of length l must
 * fit in l bits and none may be all ones (code >= 2^l: JERR_BAD_HUFF_TABLE);
 * returns 0 for such a table. */
static int huff_build(huff *t)
{
    int code = 0, k = 0;
    for (int l = 1; l <= 16; ++l) {
        t->valptr[l] = k;
        t->mincode[l] = code;
        code += t->bits[l];
        k += t->bits[l];
        if (t->bits[l] && code >= (1 << l)) return 0;
        t->maxcode[l] = t->bits[l] ? code - 1 : -1;
        code <<= 1;
    }
    t->maxcode[17] = 0x7fffffff;
    return 1;
}

static void fill(bits *b)
{
    while (b->nbits <= 24) {
        uint32_t byte = 0;
        if (!b->hit_marker && b->p < b->end) {
            byte = *b->p;
            if (byte == 0xFF) {
                uint8_t nx = (b->p + 1 < b->end) ? b->p[1] : 0xD9;
                if (nx == 0x00) b->p += 2;
                else { b->hit_marker = 1; byte = 0; }   /* a marker: feed zeros (jdhuff.c) */
            } else {
                b->p++;
            }
        }
        b->buf |= byte << (24 - b->nbits);
        b->nbits += 8;
    }
}

static int get_bits(bits *b, int n)
{
    if (n == 0) return 0;
    fill(b);
    int v = (int)(b->buf >> (32 - n));
    b->buf <<= n;
    b->nbits -= n;
    return v;
}

static int get_bit(bits *b) { return get_bits(b, 1); }

static int decode(bits *b, const huff *t)
{
    int code = 0;
    for (int l = 1; l <= 16; ++l) {
        code = (code << 1) | get_bit(b);
        if (t->maxcode[l] >= 0 && code <= t->maxcode[l] && code >= t->mincode[l])
            return t->vals[t->valptr[l] + code - t->mincode[l]];
    }
    return 0;   /* corrupt: libjpeg warns and returns 0 */
}

/* T.81 F.2.2.1 EXTEND */
static int extend(int v, int s) { return (s && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v; }

static int16_t *blk(comp *c, int bx, int by) { return c->coef + ((size_t)by * c->bw + bx) * 64; }

/* One block of a scan.  Returns 0. */
static void decode_block(dec *d, bits *b, comp *c, int16_t *bl, int ss, int se, int ah, int al,
                         const huff *dct, const huff *act)
{
    if (!d->progressive) {
        int s = decode(b, dct);
        c->dc_pred += extend(get_bits(b, s), s);
        bl[0] = (int16_t)c->dc_pred;
        for (int k = 1; k < 64; ++k) {
            int rs = decode(b, act), r = rs >> 4;
            s = rs & 15;
            if (s) { k += r; bl[ZZ[k]] = (int16_t)extend(get_bits(b, s), s); }
            else if (r == 15) k += 15;
            else break;
        }
        return;
    }
    if (ss == 0) {                                   /* DC scans */
        if (ah == 0) {
            int s = decode(b, dct);
            c->dc_pred += extend(get_bits(b, s), s);
            bl[0] = (int16_t)(c->dc_pred * (1 << al));
        } else if (get_bit(b)) {
            bl[0] |= (int16_t)(1 << al);
        }
        return;
    }
    if (ah == 0) {                                   /* AC first */
        if (d->eobrun > 0) { d->eobrun--; return; }
        for (int k = ss; k <= se; ++k) {
            int rs = decode(b, act), r = rs >> 4, s = rs & 15;
            if (s) {
                k += r;
                bl[ZZ[k]] = (int16_t)(extend(get_bits(b, s), s) * (1 << al));
            } else if (r == 15) {
                k += 15;
            } else {
                d->eobrun = 1 << r;
                if (r) d->eobrun += get_bits(b, r);
                d->eobrun--;
                break;
            }
        }
        return;
    }
    /* AC refine (T.81 G.1.2.3; libjpeg jdhuff.c decode_mcu_AC_refine) */
    int p1 = 1 << al, m1 = -1 * (1 << al);
    int k = ss;
    if (d->eobrun == 0) {
        for (; k <= se; ++k) {
            int rs = decode(b, act), r = rs >> 4, s = rs & 15;
            if (s) {
                s = get_bit(b) ? p1 : m1;
            } else if (r != 15) {
                d->eobrun = 1 << r;
                if (r) d->eobrun += get_bits(b, r);
                break;
            }
            do {
                int16_t *cf = bl + ZZ[k];
                if (*cf != 0) {
                    if (get_bit(b) && (*cf & p1) == 0)
                        *cf = (int16_t)(*cf >= 0 ? *cf + p1 : *cf + m1);
                } else {
                    if (--r < 0) break;
                }
                k++;
            } while (k <= se);
            if (s) bl[ZZ[k]] = (int16_t)s;
        }
    }
    if (d->eobrun > 0) {
        for (; k <= se; ++k) {
            int16_t *cf = bl + ZZ[k];
            if (*cf != 0 && get_bit(b) && (*cf & p1) == 0)
                *cf = (int16_t)(*cf >= 0 ? *cf + p1 : *cf + m1);
        }
        d->eobrun--;
    }
}

static int u16(const uint8_t *p) { return (p[0] << 8) | p[1]; }

/* Scan: returns pointer after the entropy-coded segment. */
static const uint8_t *scan(dec *d, const uint8_t *p, const uint8_t *end, int *err)
{
    int len = u16(p), ns = p[2];
    if (ns < 1 || ns > 4 || len != 6 + 2 * ns) { *err = -3; return end; }
    comp *sc[4];
    int td[4], ta[4];
    for (int i = 0; i < ns; ++i) {
        int id = p[3 + 2 * i], t = p[4 + 2 * i];
        sc[i] = NULL;
        for (int k = 0; k < d->nc; ++k) if (d->c[k].id == id) sc[i] = &d->c[k];
        if (!sc[i]) { *err = -3; return end; }
        td[i] = t >> 4; ta[i] = t & 15;
        if (td[i] > 3 || ta[i] > 3) { *err = -3; return end; }
    }
    int ss = p[3 + 2 * ns], se = p[4 + 2 * ns], ah = p[5 + 2 * ns] >> 4, al = p[5 + 2 * ns] & 15;
    if (!d->progressive) { ss = 0; se = 63; ah = al = 0; }
    if (ss > se || se > 63 || (ss == 0 && se != 0 && d->progressive) || (ss > 0 && ns != 1)) {
        *err = -3; return end;
    }
    p += len;
    bits b = {p, end, 0, 0, 0};
    for (int i = 0; i < ns; ++i) sc[i]->dc_pred = 0;
    d->eobrun = 0;
    int restarts_left = d->restart;
    if (ns == 1) {
        comp *c = sc[0];
        int nbx = (c->cw + 7) / 8, nby = (c->ch + 7) / 8;
        for (int by = 0; by < nby; ++by)
            for (int bx = 0; bx < nbx; ++bx) {
                if (d->restart && restarts_left == 0) {
                    /* skip to the RSTn marker, reset state (jdhuff.c process_restart) */
                    while (b.p + 1 < end && !(b.p[0] == 0xFF && b.p[1] >= 0xD0 && b.p[1] <= 0xD7)) b.p++;
                    if (b.p + 1 < end) b.p += 2;
                    b.buf = 0; b.nbits = 0; b.hit_marker = 0;
                    c->dc_pred = 0; d->eobrun = 0;
                    restarts_left = d->restart;
                }
                const huff *dct = &d->dc[td[0]], *act = &d->ac[ta[0]];
                decode_block(d, &b, c, blk(c, bx, by), ss, se, ah, al, dct, act);
                if (d->restart) restarts_left--;
            }
    } else {
        for (int my = 0; my < d->mcuy; ++my)
            for (int mx = 0; mx < d->mcux; ++mx) {
                if (d->restart && restarts_left == 0) {
                    while (b.p + 1 < end && !(b.p[0] == 0xFF && b.p[1] >= 0xD0 && b.p[1] <= 0xD7)) b.p++;
                    if (b.p + 1 < end) b.p += 2;
                    b.buf = 0; b.nbits = 0; b.hit_marker = 0;
                    for (int i = 0; i < ns; ++i) sc[i]->dc_pred = 0;
                    d->eobrun = 0;
                    restarts_left = d->restart;
                }
                for (int i = 0; i < ns; ++i) {
                    comp *c = sc[i];
                    for (int v = 0; v < c->v; ++v)
                        for (int h = 0; h < c->h; ++h)
                            decode_block(d, &b, c, blk(c, mx * c->h + h, my * c->v + v), ss, se, ah, al,
                                         &d->dc[td[i]], &d->ac[ta[i]]);
                }
                if (d->restart) restarts_left--;
            }
    }
    /* resume after the entropy-coded data: next marker that is not RSTn / stuffing */
    const uint8_t *q = b.p;
    while (q + 1 < end && !(q[0] == 0xFF && q[1] != 0x00 && !(q[1] >= 0xD0 && q[1] <= 0xD7))) q++;
    return q;
}

/* ----------------------------- IDCT ------------------------------------ */
/* jidctint.c (IJG libjpeg 9): LL&M islow, CONST_BITS 13, PASS1_BITS 2.
 * Only the exact integer result matters: every output is the same integer
 * linear form of the dequantised inputs (products of FIX() constants), with
 * the rounding shifts after pass 1 and pass 2. */
#define CONST_BITS 13
#define PASS1_BITS 2
#define FIX(x) ((int64_t)((x) * (1 << CONST_BITS) + 0.5))
#define FIX_0_298631336 ((int64_t)2446)
#define FIX_0_390180644 ((int64_t)3196)
#define FIX_0_541196100 ((int64_t)4433)
#define FIX_0_765366865 ((int64_t)6270)
#define FIX_0_899976223 ((int64_t)7373)
#define FIX_1_175875602 ((int64_t)9633)
#define FIX_1_501321110 ((int64_t)12299)
#define FIX_1_847759065 ((int64_t)15137)
#define FIX_1_961570560 ((int64_t)16069)
#define FIX_2_053119869 ((int64_t)16819)
#define FIX_2_562915447 ((int64_t)20995)
#define FIX_3_072711026 ((int64_t)25172)

/* libjpeg 9 range limit: index (v + 512) & 1023, table clamps to [0, 255]. */
static inline uint8_t rlimit(int64_t descaled_centred)
{
    int s = (int)((descaled_centred) & 1023) - 384;
    return (uint8_t)(s < 0 ? 0 : s > 255 ? 255 : s);
}

static void idct_8x8(const int16_t *in, const uint16_t *q, uint8_t *out, int stride)
{
    int ws[64];
    for (int c = 0; c < 8; ++c) {
        int64_t z1, z2, z3, t0, t1, t2, t3, t10, t11, t12, t13;
        z2 = (int64_t)in[c] * q[c];
        z3 = (int64_t)in[32 + c] * q[32 + c];
        z2 = z2 * (1 << CONST_BITS);
        z3 = z3 * (1 << CONST_BITS);
        z2 += 1 << (CONST_BITS - PASS1_BITS - 1);
        t0 = z2 + z3;
        t1 = z2 - z3;
        z2 = (int64_t)in[16 + c] * q[16 + c];
        z3 = (int64_t)in[48 + c] * q[48 + c];
        z1 = (z2 + z3) * FIX_0_541196100;
        t2 = z1 + z2 * FIX_0_765366865;
        t3 = z1 - z3 * FIX_1_847759065;
        t10 = t0 + t2; t13 = t0 - t2; t11 = t1 + t3; t12 = t1 - t3;
        t0 = (int64_t)in[56 + c] * q[56 + c];
        t1 = (int64_t)in[40 + c] * q[40 + c];
        t2 = (int64_t)in[24 + c] * q[24 + c];
        t3 = (int64_t)in[8 + c] * q[8 + c];
        z2 = t0 + t2; z3 = t1 + t3;
        z1 = (z2 + z3) * FIX_1_175875602;
        z2 = z2 * -FIX_1_961570560;
        z3 = z3 * -FIX_0_390180644;
        z2 += z1; z3 += z1;
        z1 = (t0 + t3) * -FIX_0_899976223;
        t0 = t0 * FIX_0_298631336;
        t3 = t3 * FIX_1_501321110;
        t0 += z1 + z2; t3 += z1 + z3;
        z1 = (t1 + t2) * -FIX_2_562915447;
        t1 = t1 * FIX_2_053119869;
        t2 = t2 * FIX_3_072711026;
        t1 += z1 + z3; t2 += z1 + z2;
        const int sh = CONST_BITS - PASS1_BITS;
        ws[0 * 8 + c] = (int)((t10 + t3) >> sh); ws[7 * 8 + c] = (int)((t10 - t3) >> sh);
        ws[1 * 8 + c] = (int)((t11 + t2) >> sh); ws[6 * 8 + c] = (int)((t11 - t2) >> sh);
        ws[2 * 8 + c] = (int)((t12 + t1) >> sh); ws[5 * 8 + c] = (int)((t12 - t1) >> sh);
        ws[3 * 8 + c] = (int)((t13 + t0) >> sh); ws[4 * 8 + c] = (int)((t13 - t0) >> sh);
    }
    for (int r = 0; r < 8; ++r) {
        const int *w = ws + r * 8;
        int64_t z1, z2, z3, t0, t1, t2, t3, t10, t11, t12, t13;
        z2 = (int64_t)w[0] + ((512 << (PASS1_BITS + 3)) + (1 << (PASS1_BITS + 2)));
        z3 = w[4];
        t0 = (z2 + z3) * (1 << CONST_BITS);
        t1 = (z2 - z3) * (1 << CONST_BITS);
        z2 = w[2]; z3 = w[6];
        z1 = (z2 + z3) * FIX_0_541196100;
        t2 = z1 + z2 * FIX_0_765366865;
        t3 = z1 - z3 * FIX_1_847759065;
        t10 = t0 + t2; t13 = t0 - t2; t11 = t1 + t3; t12 = t1 - t3;
        t0 = w[7]; t1 = w[5]; t2 = w[3]; t3 = w[1];
        z2 = t0 + t2; z3 = t1 + t3;
        z1 = (z2 + z3) * FIX_1_175875602;
        z2 = z2 * -FIX_1_961570560;
        z3 = z3 * -FIX_0_390180644;
        z2 += z1; z3 += z1;
        z1 = (t0 + t3) * -FIX_0_899976223;
        t0 = t0 * FIX_0_298631336;
        t3 = t3 * FIX_1_501321110;
        t0 += z1 + z2; t3 += z1 + z3;
        z1 = (t1 + t2) * -FIX_2_562915447;
        t1 = t1 * FIX_2_053119869;
        t2 = t2 * FIX_3_072711026;
        t1 += z1 + z3; t2 += z1 + z2;
        const int sh = CONST_BITS + PASS1_BITS + 3;
        uint8_t *o = out + (size_t)r * stride;
        o[0] = rlimit((t10 + t3) >> sh); o[7] = rlimit((t10 - t3) >> sh);
        o[1] = rlimit((t11 + t2) >> sh); o[6] = rlimit((t11 - t2) >> sh);
        o[2] = rlimit((t12 + t1) >> sh); o[5] = rlimit((t12 - t1) >> sh);
        o[3] = rlimit((t13 + t0) >> sh); o[4] = rlimit((t13 - t0) >> sh);
    }
}

/* jpeg_idct_16x16: 8x8 coefficients -> 16x16 samples; 16-point kernel with
 * cK = sqrt(2) * cos(K * pi / 32).  The same even/odd decomposition is used in
 * both passes (columns of the input, then the 16 rows of the work array). */
static void idct16_1d(const int64_t x[8], int64_t even_dc, int64_t outv[16])
{
    int64_t t0, t1, t2, t3, t10, t11, t12, t13, t20, t21, t22, t23, t24, t25, t26, t27;
    int64_t z1, z2, z3, z4;
    t0 = even_dc;
    z1 = x[4];
    t1 = z1 * FIX(1.306562965);
    t2 = z1 * FIX_0_541196100;
    t10 = t0 + t1; t11 = t0 - t1; t12 = t0 + t2; t13 = t0 - t2;
    z1 = x[2]; z2 = x[6];
    z3 = z1 - z2;
    z4 = z3 * FIX(0.275899379);
    z3 = z3 * FIX(1.387039845);
    t0 = z3 + z2 * FIX_2_562915447;
    t1 = z4 + z1 * FIX_0_899976223;
    t2 = z3 - z1 * FIX(0.601344887);
    t3 = z4 - z2 * FIX(0.509795579);
    t20 = t10 + t0; t27 = t10 - t0;
    t21 = t12 + t1; t26 = t12 - t1;
    t22 = t13 + t2; t25 = t13 - t2;
    t23 = t11 + t3; t24 = t11 - t3;
    z1 = x[1]; z2 = x[3]; z3 = x[5]; z4 = x[7];
    t11 = z1 + z3;
    t1 = (z1 + z2) * FIX(1.353318001);
    t2 = t11 * FIX(1.247225013);
    t3 = (z1 + z4) * FIX(1.093201867);
    t10 = (z1 - z4) * FIX(0.897167586);
    t11 = t11 * FIX(0.666655658);
    t12 = (z1 - z2) * FIX(0.410524528);
    t0 = t1 + t2 + t3 - z1 * FIX(2.286341144);
    t13 = t10 + t11 + t12 - z1 * FIX(1.835730603);
    z1 = (z2 + z3) * FIX(0.138617169);
    t1 += z1 + z2 * FIX(0.071888074);
    t2 += z1 - z3 * FIX(1.125726048);
    z1 = (z3 - z2) * FIX(1.407403738);
    t11 += z1 - z3 * FIX(0.766367282);
    t12 += z1 + z2 * FIX(1.971951411);
    z2 += z4;
    z1 = z2 * -FIX(0.666655658);
    t1 += z1;
    t3 += z1 + z4 * FIX(1.065388962);
    z2 = z2 * -FIX(1.247225013);
    t10 += z2 + z4 * FIX(3.141271809);
    t12 += z2;
    z2 = (z3 + z4) * -FIX(1.353318001);
    t2 += z2;
    t3 += z2;
    z2 = (z4 - z3) * FIX(0.410524528);
    t10 += z2;
    t11 += z2;
    outv[0] = t20 + t0;  outv[15] = t20 - t0;
    outv[1] = t21 + t1;  outv[14] = t21 - t1;
    outv[2] = t22 + t2;  outv[13] = t22 - t2;
    outv[3] = t23 + t3;  outv[12] = t23 - t3;
    outv[4] = t24 + t10; outv[11] = t24 - t10;
    outv[5] = t25 + t11; outv[10] = t25 - t11;
    outv[6] = t26 + t12; outv[9]  = t26 - t12;
    outv[7] = t27 + t13; outv[8]  = t27 - t13;
}

static void idct_16x16(const int16_t *in, const uint16_t *q, uint8_t *out, int stride)
{
    int ws[8 * 16];
    for (int c = 0; c < 8; ++c) {
        int64_t x[8], o[16];
        for (int k = 0; k < 8; ++k) x[k] = (int64_t)in[k * 8 + c] * q[k * 8 + c];
        int64_t dc = x[0] * (1 << CONST_BITS) + (1 << (CONST_BITS - PASS1_BITS - 1));
        idct16_1d(x, dc, o);
        for (int r = 0; r < 16; ++r) ws[r * 8 + c] = (int)(o[r] >> (CONST_BITS - PASS1_BITS));
    }
    for (int r = 0; r < 16; ++r) {
        int64_t x[8], o[16];
        for (int k = 0; k < 8; ++k) x[k] = ws[r * 8 + k];
        int64_t dc = (x[0] + ((512 << (PASS1_BITS + 3)) + (1 << (PASS1_BITS + 2)))) * (1 << CONST_BITS);
        idct16_1d(x, dc, o);
        uint8_t *op = out + (size_t)r * stride;
        for (int k = 0; k < 16; ++k) op[k] = rlimit(o[k] >> (CONST_BITS + PASS1_BITS + 3));
    }
}

/* jdcolor.c (libjpeg 9) build_ycc_rgb_table, SCALEBITS 16 */
#define SCALEBITS 16
#define ONE_HALF ((int64_t)1 << (SCALEBITS - 1))
#define FIXC(x) ((int64_t)((x) * (1L << SCALEBITS) + 0.5))

static uint8_t clamp255(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

int cgo_jpeg_info(const uint8_t *data, size_t n, int *w, int *h, int *nc)
{
    const uint8_t *p = data, *end = data + n;
    if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) return -1;
    p += 2;
    while (p + 4 <= end) {
        if (p[0] != 0xFF) { p++; continue; }
        int m = p[1];
        if (m == 0xFF) { p++; continue; }
        int len = u16(p + 2);
        if (m >= 0xC0 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            if (p + 2 + 8 > end) return -1;
            *h = u16(p + 5); *w = u16(p + 7); *nc = p[9];
            return 0;
        }
        p += 2 + len;
    }
    return -1;
}

int cgo_jpeg_decode(const uint8_t *data, size_t n, uint8_t *out, size_t cap)
{
    dec *d = (dec *)calloc(1, sizeof(dec));
    if (!d) return -2;
    int err = 0, have_frame = 0;
    const uint8_t *p = data, *end = data + n;
    if (n < 4 || p[0] != 0xFF || p[1] != 0xD8) { free(d); return -1; }
    p += 2;
    while (p + 2 <= end && !err) {
        if (p[0] != 0xFF) { p++; continue; }
        int m = p[1];
        if (m == 0xFF) { p++; continue; }
        p += 2;
        if (m == 0xD9) break;                               /* EOI */
        if (m >= 0xD0 && m <= 0xD7) continue;
        if (p + 2 > end) { err = -1; break; }
        int len = u16(p);
        if (p + len > end) { err = -1; break; }
        if (m == 0xDB) {                                    /* DQT */
            const uint8_t *q = p + 2;
            while (q < p + len) {
                int pq = q[0] >> 4, tq = q[0] & 15;
                if (tq > 3) { err = -3; break; }
                for (int k = 0; k < 64; ++k)
                    d->q[tq][ZZ[k]] = (uint16_t)(pq ? u16(q + 1 + 2 * k) : q[1 + k]);
                q += 1 + (pq ? 128 : 64);
            }
        } else if (m == 0xC4) {                             /* DHT */
            const uint8_t *q = p + 2;
            while (q < p + len) {
                int tc = q[0] >> 4, th = q[0] & 15, tot = 0;
                if (th > 3 || tc > 1) { err = -3; break; }
                huff *t = tc ? &d->ac[th] : &d->dc[th];
                t->bits[0] = 0;
                for (int l = 1; l <= 16; ++l) { t->bits[l] = q[l]; tot += q[l]; }
                if (tot > 256) { err = -3; break; }
                memcpy(t->vals, q + 17, (size_t)tot);
                if (!huff_build(t)) { err = -3; break; }
                t->present = 1;
                q += 17 + tot;
            }
        } else if (m == 0xDD) {                             /* DRI */
            d->restart = u16(p + 2);
        } else if (m == 0xEE && len >= 12 && !memcmp(p + 2, "Adobe", 5)) {
            d->adobe = 1;
            d->adobe_transform = p[13];
        } else if (m == 0xC0 || m == 0xC1 || m == 0xC2) {  /* SOF0/1/2, Huffman */
            if (p[2] != 8) { err = -4; break; }
            d->progressive = (m == 0xC2);
            d->h = u16(p + 3); d->w = u16(p + 5); d->nc = p[7];
            if (d->nc != 1 && d->nc != 3) { err = -4; break; }
            if (d->w <= 0 || d->h <= 0) { err = -3; break; }
            d->hmax = d->vmax = 1;
            for (int i = 0; i < d->nc; ++i) {
                comp *c = &d->c[i];
                c->id = p[8 + 3 * i]; c->h = p[9 + 3 * i] >> 4; c->v = p[9 + 3 * i] & 15; c->tq = p[10 + 3 * i];
                if (c->h < 1 || c->h > 4 || c->v < 1 || c->v > 4 || c->tq > 3) { err = -3; break; }
                if (c->h > d->hmax) d->hmax = c->h;
                if (c->v > d->vmax) d->vmax = c->v;
            }
            if (err) break;
            d->mcux = (d->w + 8 * d->hmax - 1) / (8 * d->hmax);
            d->mcuy = (d->h + 8 * d->vmax - 1) / (8 * d->vmax);
            for (int i = 0; i < d->nc; ++i) {
                comp *c = &d->c[i];
                c->cw = (d->w * c->h + d->hmax - 1) / d->hmax;
                c->ch = (d->h * c->v + d->vmax - 1) / d->vmax;
                c->bw = d->mcux * c->h;
                c->bh = d->mcuy * c->v;
                if (d->nc == 1) { c->bw = (c->cw + 7) / 8; c->bh = (c->ch + 7) / 8; }
                c->coef = (int16_t *)calloc((size_t)c->bw * c->bh * 64, sizeof(int16_t));
                if (!c->coef) { err = -2; break; }
                /* libjpeg 9: IDCT scaling replaces upsampling when the ratio is 2 */
                int sh = (d->hmax % (2 * c->h) == 0) ? 2 : 1, sv = (d->vmax % (2 * c->v) == 0) ? 2 : 1;
                if (c->h * sh != d->hmax || c->v * sv != d->vmax || sh != sv) { err = -4; break; }
            }
            have_frame = 1;
        } else if ((m >= 0xC3 && m <= 0xCF) && m != 0xC4 && m != 0xC8 && m != 0xCC) {
            err = -4;                                       /* lossless / arithmetic / hierarchical */
            break;
        } else if (m == 0xDA) {                             /* SOS */
            if (!have_frame) { err = -3; break; }
            p = scan(d, p, end, &err);
            continue;
        }
        p += len;
    }
    if (!err && !have_frame) err = -3;
    if (!err && cap < (size_t)d->w * d->h * d->nc) err = -5;
    if (!err) {
        /* IDCT every component into a full-resolution plane */
        uint8_t *plane[3] = {0};
        int pw = d->mcux * d->hmax * 8, ph = d->mcuy * d->vmax * 8;
        if (d->nc == 1) { pw = d->c[0].bw * 8; ph = d->c[0].bh * 8; }
        for (int i = 0; i < d->nc && !err; ++i) {
            comp *c = &d->c[i];
            plane[i] = (uint8_t *)malloc((size_t)pw * ph);
            if (!plane[i]) { err = -2; break; }
            int scale = d->hmax / c->h;                   /* 1 or 2 (checked above) */
            const uint16_t *q = d->q[c->tq];
            for (int by = 0; by < c->bh; ++by)
                for (int bx = 0; bx < c->bw; ++bx) {
                    int ox = bx * 8 * scale, oy = by * 8 * scale;
                    if (ox >= pw || oy >= ph) continue;
                    uint8_t *o = plane[i] + (size_t)oy * pw + ox;
                    if (scale == 1) idct_8x8(blk(c, bx, by), q, o, pw);
                    else idct_16x16(blk(c, bx, by), q, o, pw);
                }
        }
        if (!err) {
            int rgb = d->adobe && d->adobe_transform == 0;
            for (int y = 0; y < d->h; ++y)
                for (int x = 0; x < d->w; ++x) {
                    size_t o = (size_t)y * pw + x, dst = ((size_t)y * d->w + x) * d->nc;
                    if (d->nc == 1) { out[dst] = plane[0][o]; continue; }
                    int Y = plane[0][o], cb = plane[1][o] - 128, cr = plane[2][o] - 128;
                    int R, G, B;
                    if (rgb) { R = Y; G = plane[1][o]; B = plane[2][o]; }
                    else {
                        int crr = (int)((FIXC(1.402) * cr + ONE_HALF) >> SCALEBITS);
                        int cbb = (int)((FIXC(1.772) * cb + ONE_HALF) >> SCALEBITS);
                        int64_t crg = -FIXC(0.714136286) * cr;
                        int64_t cbg = -FIXC(0.344136286) * cb + ONE_HALF;
                        R = Y + crr;
                        G = Y + (int)((cbg + crg) >> SCALEBITS);
                        B = Y + cbb;
                    }
                    out[dst + 0] = clamp255(B);                /* OpenCV: BGR */
                    out[dst + 1] = clamp255(G);
                    out[dst + 2] = clamp255(R);
                }
        }
        for (int i = 0; i < 3; ++i) free(plane[i]);
    }
    for (int i = 0; i < 4; ++i) free(d->c[i].coef);
    free(d);
    return err;
}
