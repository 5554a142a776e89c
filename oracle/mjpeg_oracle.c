/*
 * oracle/mjpeg_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the arithmetic that the reference's hot path runs inside the
 * external `ffmpeg` worker (ffmpeg_distributed.py:131-141 spawns
 * `ffmpeg -f matroska -i pipe: <remote_args> -f matroska pipe:`), restricted to the
 * north-star profile  [-vf scale=W:H:flags=bicubic] -c:v mjpeg -q:v N -dct int
 * -huffman default|optimal -bitexact  on yuv420p / yuvj420p frames, plus the 4:2:2 / 4:4:4
 * variants and the RST (slice-threaded) bitstream layout.
 *
 * The arithmetic lives in third-party FFmpeg (libavcodec mjpeg encoder, libswscale),
 * which is NOT vendored under /root/reference, not pinned by it (no requirements
 * file, README.md:1-39 names no version) and absent from this container and from the
 * GPU box (probed: no ffmpeg binary, no libavcodec/libswscale).  Each function below
 * restates the published FFmpeg algorithm and names the FFmpeg file/function it
 * follows; the reference-side call site is ffmpeg_distributed.py:131-141.
 *
 *   PARITY STATUS: unpinned against FFmpeg itself (no FFmpeg build or golden
 *   vectors exist in /root/reference or anywhere on this pool).  Pinned pieces:
 *   the Annex K Huffman BITS/HUFFVAL tables are checked against libjpeg-turbo's
 *   standard tables (Pillow, tests/test_oracle.py); decodability and PSNR are checked
 *   with Pillow; the dispatcher behaviour is pinned by fixtures captured from the
 *   real reference (tests/golden/).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 * Nothing on the product path links it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

/* ------------------------------------------------------------------ tables */

/* libavcodec/mathtables.c ff_zigzag_direct */
static const uint8_t or_zigzag[64] = {
    0,  1,  8, 16,  9,  2,  3, 10, 17, 24, 32, 25, 18, 11,  4,  5,
   12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,  6,  7, 14, 21, 28,
   35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
   58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63
};

/* libavcodec/mpeg12data.c ff_mpeg1_default_intra_matrix (raster order) */
static const uint16_t or_mpeg1_intra[64] = {
    8, 16, 19, 22, 26, 27, 29, 34,
   16, 16, 22, 24, 27, 29, 34, 37,
   19, 22, 26, 27, 29, 34, 34, 38,
   22, 22, 26, 27, 29, 34, 37, 40,
   22, 26, 27, 29, 32, 35, 40, 48,
   26, 27, 29, 32, 35, 40, 48, 58,
   26, 27, 29, 34, 38, 46, 56, 69,
   27, 29, 35, 38, 46, 56, 69, 83
};

/* libavcodec/jpegtables.c (ITU T.81 Annex K.3) */
static const uint8_t or_bits_dc_lum[17] = { 0, 0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0 };
static const uint8_t or_bits_dc_chr[17] = { 0, 0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0 };
static const uint8_t or_val_dc[12] = { 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11 };
static const uint8_t or_bits_ac_lum[17] = { 0, 0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d };
static const uint8_t or_val_ac_lum[162] = {
  0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
  0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0,
  0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28,
  0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
  0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
  0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
  0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
  0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5,
  0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
  0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
  0xf9, 0xfa
};
static const uint8_t or_bits_ac_chr[17] = { 0, 0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77 };
static const uint8_t or_val_ac_chr[162] = {
  0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
  0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0,
  0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26,
  0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48,
  0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68,
  0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87,
  0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5,
  0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
  0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
  0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
  0xf9, 0xfa
};

/* -------------------------------------------------------------- bit writer */
/* libavcodec/put_bits.h semantics: MSB-first. */
typedef struct {
    uint8_t *buf;
    size_t cap;       /* bytes */
    size_t nbits;     /* bits written */
    int overflow;
} or_pb;

static void pb_put(or_pb *pb, int n, uint32_t v)
{
    for (int i = n - 1; i >= 0; i--) {
        size_t byte = pb->nbits >> 3;
        if (byte >= pb->cap) { pb->overflow = 1; pb->nbits++; continue; }
        int bit = (v >> i) & 1;
        if ((pb->nbits & 7) == 0) pb->buf[byte] = 0;
        if (bit) pb->buf[byte] |= (uint8_t)(0x80 >> (pb->nbits & 7));
        pb->nbits++;
    }
}

/* ------------------------------------------------------ Huffman code tables */
/* libavcodec/mjpegenc_huffman.c / jpegtables.c ff_mjpeg_build_huffman_codes */
static void or_build_huff(uint8_t size[256], uint16_t code[256],
                          const uint8_t *bits, const uint8_t *vals)
{
    int k = 0, c = 0;
    memset(size, 0, 256);
    memset(code, 0, 256 * sizeof(uint16_t));
    for (int i = 1; i <= 16; i++) {
        for (int j = 0; j < bits[i]; j++) {
            int sym = vals[k++];
            size[sym] = (uint8_t)i;
            code[sym] = (uint16_t)c;
            c++;
        }
        c <<= 1;
    }
}

/* exported for tests: table id 0=DC lum, 1=DC chr, 2=AC lum, 3=AC chr */
int or_huff_table(int id, uint8_t size[256], uint16_t code[256])
{
    switch (id) {
    case 0: or_build_huff(size, code, or_bits_dc_lum, or_val_dc); return 0;
    case 1: or_build_huff(size, code, or_bits_dc_chr, or_val_dc); return 0;
    case 2: or_build_huff(size, code, or_bits_ac_lum, or_val_ac_lum); return 0;
    case 3: or_build_huff(size, code, or_bits_ac_chr, or_val_ac_chr); return 0;
    }
    return -1;
}

/* ----------------------------------------------------------------- FDCT */
/* libavcodec/jfdctint_template.c, ff_jpeg_fdct_islow_8 (BITS_IN_JSAMPLE 8):
 * CONST_BITS 13, PASS1_BITS 4, 32-bit MULTIPLY (PASS1_BITS > 2), int16 storage
 * between the passes.  Input is unshifted 0..255 samples (get_pixels, no -128). */
#define OR_CONST_BITS 13
#define OR_PASS1_BITS 4
#define OR_DESCALE(x, n) (((x) + (1 << ((n) - 1))) >> (n))
#define FIX_0_298631336  2446
#define FIX_0_390180644  3196
#define FIX_0_541196100  4433
#define FIX_0_765366865  6270
#define FIX_0_899976223  7373
#define FIX_1_175875602  9633
#define FIX_1_501321110  12299
#define FIX_1_847759065  15137
#define FIX_1_961570560  16069
#define FIX_2_053119869  16819
#define FIX_2_562915447  20995
#define FIX_3_072711026  25172

void or_fdct_islow(int16_t *data)
{
    int tmp0, tmp1, tmp2, tmp3, tmp4, tmp5, tmp6, tmp7;
    int tmp10, tmp11, tmp12, tmp13;
    int z1, z2, z3, z4, z5;
    int16_t *p;

    /* Pass 1: rows (row_fdct) */
    p = data;
    for (int ctr = 0; ctr < 8; ctr++, p += 8) {
        tmp0 = p[0] + p[7]; tmp7 = p[0] - p[7];
        tmp1 = p[1] + p[6]; tmp6 = p[1] - p[6];
        tmp2 = p[2] + p[5]; tmp5 = p[2] - p[5];
        tmp3 = p[3] + p[4]; tmp4 = p[3] - p[4];

        tmp10 = tmp0 + tmp3; tmp13 = tmp0 - tmp3;
        tmp11 = tmp1 + tmp2; tmp12 = tmp1 - tmp2;

        p[0] = (int16_t)((tmp10 + tmp11) * (1 << OR_PASS1_BITS));
        p[4] = (int16_t)((tmp10 - tmp11) * (1 << OR_PASS1_BITS));

        z1 = (tmp12 + tmp13) * FIX_0_541196100;
        p[2] = (int16_t)OR_DESCALE(z1 + tmp13 * FIX_0_765366865, OR_CONST_BITS - OR_PASS1_BITS);
        p[6] = (int16_t)OR_DESCALE(z1 + tmp12 * (-FIX_1_847759065), OR_CONST_BITS - OR_PASS1_BITS);

        z1 = tmp4 + tmp7; z2 = tmp5 + tmp6; z3 = tmp4 + tmp6; z4 = tmp5 + tmp7;
        z5 = (z3 + z4) * FIX_1_175875602;
        tmp4 = tmp4 * FIX_0_298631336; tmp5 = tmp5 * FIX_2_053119869;
        tmp6 = tmp6 * FIX_3_072711026; tmp7 = tmp7 * FIX_1_501321110;
        z1 = z1 * (-FIX_0_899976223); z2 = z2 * (-FIX_2_562915447);
        z3 = z3 * (-FIX_1_961570560); z4 = z4 * (-FIX_0_390180644);
        z3 += z5; z4 += z5;
        p[7] = (int16_t)OR_DESCALE(tmp4 + z1 + z3, OR_CONST_BITS - OR_PASS1_BITS);
        p[5] = (int16_t)OR_DESCALE(tmp5 + z2 + z4, OR_CONST_BITS - OR_PASS1_BITS);
        p[3] = (int16_t)OR_DESCALE(tmp6 + z2 + z3, OR_CONST_BITS - OR_PASS1_BITS);
        p[1] = (int16_t)OR_DESCALE(tmp7 + z1 + z4, OR_CONST_BITS - OR_PASS1_BITS);
    }

    /* Pass 2: columns */
    p = data;
    for (int ctr = 0; ctr < 8; ctr++, p++) {
        tmp0 = p[8 * 0] + p[8 * 7]; tmp7 = p[8 * 0] - p[8 * 7];
        tmp1 = p[8 * 1] + p[8 * 6]; tmp6 = p[8 * 1] - p[8 * 6];
        tmp2 = p[8 * 2] + p[8 * 5]; tmp5 = p[8 * 2] - p[8 * 5];
        tmp3 = p[8 * 3] + p[8 * 4]; tmp4 = p[8 * 3] - p[8 * 4];

        tmp10 = tmp0 + tmp3; tmp13 = tmp0 - tmp3;
        tmp11 = tmp1 + tmp2; tmp12 = tmp1 - tmp2;

        p[8 * 0] = (int16_t)OR_DESCALE(tmp10 + tmp11, OR_PASS1_BITS);
        p[8 * 4] = (int16_t)OR_DESCALE(tmp10 - tmp11, OR_PASS1_BITS);

        z1 = (tmp12 + tmp13) * FIX_0_541196100;
        p[8 * 2] = (int16_t)OR_DESCALE(z1 + tmp13 * FIX_0_765366865, OR_CONST_BITS + OR_PASS1_BITS);
        p[8 * 6] = (int16_t)OR_DESCALE(z1 + tmp12 * (-FIX_1_847759065), OR_CONST_BITS + OR_PASS1_BITS);

        z1 = tmp4 + tmp7; z2 = tmp5 + tmp6; z3 = tmp4 + tmp6; z4 = tmp5 + tmp7;
        z5 = (z3 + z4) * FIX_1_175875602;
        tmp4 = tmp4 * FIX_0_298631336; tmp5 = tmp5 * FIX_2_053119869;
        tmp6 = tmp6 * FIX_3_072711026; tmp7 = tmp7 * FIX_1_501321110;
        z1 = z1 * (-FIX_0_899976223); z2 = z2 * (-FIX_2_562915447);
        z3 = z3 * (-FIX_1_961570560); z4 = z4 * (-FIX_0_390180644);
        z3 += z5; z4 += z5;
        p[8 * 7] = (int16_t)OR_DESCALE(tmp4 + z1 + z3, OR_CONST_BITS + OR_PASS1_BITS);
        p[8 * 5] = (int16_t)OR_DESCALE(tmp5 + z2 + z4, OR_CONST_BITS + OR_PASS1_BITS);
        p[8 * 3] = (int16_t)OR_DESCALE(tmp6 + z2 + z3, OR_CONST_BITS + OR_PASS1_BITS);
        p[8 * 1] = (int16_t)OR_DESCALE(tmp7 + z1 + z4, OR_CONST_BITS + OR_PASS1_BITS);
    }
}

/* ----------------------------------------------------------- quantizer */
/* libavcodec/mpegvideo_enc.c update_qscale: lambda = q * FF_QP2LAMBDA(118),
 * qscale = (lambda*139 + 128*64) >> 14 clipped to [qmin=2, qmax=31]. */
int or_effective_qscale(double q)
{
    int lambda = (int)(q * 118.0);
    int qs = (lambda * 139 + 128 * 64) >> 14;
    if (qs < 2) qs = 2;
    if (qs > 31) qs = 31;
    return qs;
}

/* mpegvideo_enc.c encode_picture (FMT_MJPEG block): m'[i] = clip_u8((M[i]*qscale)>>3)
 * for i>=1, m'[0] = 8; then ff_convert_matrix with qscale forced to 8:
 * qmat[i] = (2<<QMAT_SHIFT) / (qscale2 * m'[i]), qscale2 = 8<<1 = 16. */
void or_build_matrix(int qscale, uint8_t mprime[64], int32_t qmat[64])
{
    for (int i = 0; i < 64; i++) {
        int v = (i == 0) ? 8 : ((or_mpeg1_intra[i] * qscale) >> 3);
        if (v > 255) v = 255;
        if (v < 0) v = 0;
        mprime[i] = (uint8_t)v;
        qmat[i] = (int32_t)(((uint64_t)2 << 21) / (uint64_t)(16 * (v ? v : 1)));
    }
}

/* mpegvideo_enc.c dct_quantize_c, intra, MJPEG: DC q = dc_scale(8)<<3 = 64,
 * bias = intra_quant_bias(3<<5) << (QMAT_SHIFT-QUANT_BIAS_SHIFT) = 3<<18,
 * QMAT_SHIFT 21; then clip_coeffs to [-1023,1023] if the OR'd max overflows.
 * Returns last_non_zero (zigzag index, 0 when only DC). */
int or_quantize(int16_t *block, const int32_t *qmat)
{
    const int QMAT_SHIFT = 21;
    const int bias = 3 << 18;
    const int threshold1 = (1 << QMAT_SHIFT) - bias - 1;
    const unsigned threshold2 = (unsigned)threshold1 << 1;
    int last_non_zero = 0, max = 0;

    block[0] = (int16_t)((block[0] + 32) / 64);
    for (int i = 63; i >= 1; i--) {
        int j = or_zigzag[i];
        int level = (int)((uint32_t)block[j] * (uint32_t)qmat[j]);
        if ((unsigned)(level + threshold1) > threshold2) { last_non_zero = i; break; }
        block[j] = 0;
    }
    for (int i = 1; i <= last_non_zero; i++) {
        int j = or_zigzag[i];
        int level = (int)((uint32_t)block[j] * (uint32_t)qmat[j]);
        if ((unsigned)(level + threshold1) > threshold2) {
            if (level > 0) { level = (bias + level) >> QMAT_SHIFT; block[j] = (int16_t)level; }
            else { level = (bias - level) >> QMAT_SHIFT; block[j] = (int16_t)-level; }
            max |= level;
        } else {
            block[j] = 0;
        }
    }
    if (max > 1023) { /* clip_coeffs, intra: skip DC */
        for (int i = 1; i <= last_non_zero; i++) {
            int j = or_zigzag[i];
            if (block[j] > 1023) block[j] = 1023;
            else if (block[j] < -1023) block[j] = -1023;
        }
    }
    return last_non_zero;
}

/* ------------------------------------------------------- entropy coding */
typedef struct {
    uint8_t dc_size[2][256]; uint16_t dc_code[2][256];
    uint8_t ac_size[2][256]; uint16_t ac_code[2][256];
} or_huff;

static void or_huff_init_tables(or_huff *h, const uint8_t *const bits[4], const uint8_t *const vals[4])
{
    or_build_huff(h->dc_size[0], h->dc_code[0], bits[0], vals[0]);
    or_build_huff(h->dc_size[1], h->dc_code[1], bits[1], vals[1]);
    or_build_huff(h->ac_size[0], h->ac_code[0], bits[2], vals[2]);
    or_build_huff(h->ac_size[1], h->ac_code[1], bits[3], vals[3]);
}


static int or_log2_16(int v) { int n = 0; while (v >> (n + 1)) n++; return n; }

/* mjpegenc_common.c ff_mjpeg_encode_dc */
static void or_encode_dc(or_pb *pb, int val, const uint8_t *size, const uint16_t *code)
{
    if (val == 0) {
        pb_put(pb, size[0], code[0]);
    } else {
        int mant = val;
        if (val < 0) { val = -val; mant--; }
        int nbits = or_log2_16(val) + 1;
        pb_put(pb, size[nbits], code[nbits]);
        pb_put(pb, nbits, (uint32_t)mant & ((1u << nbits) - 1));
    }
}

/* mjpegenc.c encode_block (HUFFMAN_TABLE_DEFAULT path) */
static void or_encode_block(or_pb *pb, const or_huff *h, const int16_t *block, int n,
                            int last_index, int *last_dc)
{
    int component = (n <= 3) ? 0 : (n & 1) + 1;
    int tab = (n <= 3) ? 0 : 1;
    int dc = block[0];
    or_encode_dc(pb, dc - last_dc[component], h->dc_size[tab], h->dc_code[tab]);
    last_dc[component] = dc;

    int run = 0;
    for (int i = 1; i <= last_index; i++) {
        int val = block[or_zigzag[i]];
        if (val == 0) { run++; continue; }
        while (run >= 16) { pb_put(pb, h->ac_size[tab][0xf0], h->ac_code[tab][0xf0]); run -= 16; }
        int mant = val;
        if (val < 0) { val = -val; mant--; }
        int nbits = or_log2_16(val) + 1;
        int code = (run << 4) | nbits;
        pb_put(pb, h->ac_size[tab][code], h->ac_code[tab][code]);
        pb_put(pb, nbits, (uint32_t)mant & ((1u << nbits) - 1));
        run = 0;
    }
    if (last_index < 63 || run != 0)
        pb_put(pb, h->ac_size[tab][0], h->ac_code[tab][0]);
}

/* mjpegenc.c record_block / ff_mjpeg_encode_coef / ff_mjpeg_encode_code (-huffman
 * optimal): the same symbols encode_block emits, counted per table (0 DC lum, 1 DC chr,
 * 2 AC lum, 3 AC chr) as mjpeg_build_optimal_huffman does over the picture's buffer. */
static void or_count_block(uint32_t counts[4][256], const int16_t *block, int n, int last_index,
                           int *last_dc)
{
    int component = (n <= 3) ? 0 : (n & 1) + 1;
    int tab = (n <= 3) ? 0 : 1;
    int dc = block[0], val = dc - last_dc[component];
    last_dc[component] = dc;
    counts[tab][val == 0 ? 0 : or_log2_16(val < 0 ? -val : val) + 1]++;
    int run = 0;
    for (int i = 1; i <= last_index; i++) {
        int v = block[or_zigzag[i]];
        if (v == 0) { run++; continue; }
        while (run >= 16) { counts[2 + tab][0xf0]++; run -= 16; }
        counts[2 + tab][(run << 4) | (or_log2_16(v < 0 ? -v : v) + 1)]++;
        run = 0;
    }
    if (last_index < 63 || run != 0) counts[2 + tab][0]++;
}

/* ---------------------------------------------------------------- header */
/* mjpegenc_common.c ff_mjpeg_encode_picture_header + jpeg_put_comments +
 * jpeg_table_header, for AV_CODEC_ID_MJPEG, -bitexact (no COM Lavc), equal luma/chroma
 * matrices (one DQT table); SOF0 sampling factors from ff_mjpeg_init_hvsample; DRI only
 * with slice threading (dri_interval > 0, written after DQT and before DHT).
 * com_itu601: the COM "CS=ITU601" segment for limited-range input. */
static void put16(or_pb *pb, int v) { pb_put(pb, 16, (uint32_t)v & 0xffff); }
static void put8(or_pb *pb, int v) { pb_put(pb, 8, (uint32_t)v & 0xff); }

static int put_huffman_table(or_pb *pb, int cls, int id, const uint8_t *bits, const uint8_t *vals)
{
    int n = 0;
    pb_put(pb, 4, cls); pb_put(pb, 4, id);
    for (int i = 1; i <= 16; i++) { n += bits[i]; put8(pb, bits[i]); }
    for (int i = 0; i < n; i++) put8(pb, vals[i]);
    return n + 17;
}

static void or_hvsample(int cfmt, int hs[3], int vs[3]);
static size_t or_header_fmt(int width, int height, int cfmt, int qscale, int sar_num, int sar_den,
                            int com_itu601, int dri_interval, const uint8_t *const bits[4],
                            const uint8_t *const vals[4], uint8_t *out, size_t cap)
{
    int hs[3], vs[3];
    or_hvsample(cfmt, hs, vs);
    or_pb pb = { out, cap, 0, 0 };
    uint8_t mprime[64]; int32_t qmat[64];
    or_build_matrix(qscale, mprime, qmat);

    put16(&pb, 0xFFD8);                                  /* SOI */
    if (sar_num > 0 && sar_den > 0) {                    /* APP0 JFIF */
        put16(&pb, 0xFFE0); put16(&pb, 16);
        put8(&pb, 'J'); put8(&pb, 'F'); put8(&pb, 'I'); put8(&pb, 'F'); put8(&pb, 0);
        put16(&pb, 0x0102); put8(&pb, 0);
        put16(&pb, sar_num); put16(&pb, sar_den);
        put8(&pb, 0); put8(&pb, 0);
    }
    if (com_itu601) {
        const char *s = "CS=ITU601";
        put16(&pb, 0xFFFE); put16(&pb, (int)strlen(s) + 3);
        for (const char *c = s; *c; c++) put8(&pb, *c);
        put8(&pb, 0);
    }
    put16(&pb, 0xFFDB); put16(&pb, 2 + 1 * (1 + 64));   /* DQT, one table */
    pb_put(&pb, 4, 0); pb_put(&pb, 4, 0);
    for (int i = 0; i < 64; i++) put8(&pb, mprime[or_zigzag[i]]);
    if (dri_interval > 0) { put16(&pb, 0xFFDD); put16(&pb, 4); put16(&pb, dri_interval); }
    put16(&pb, 0xFFC4);                                  /* DHT */
    size_t len_pos = pb.nbits >> 3;
    put16(&pb, 0);
    int size = 2;
    /* jpeg_table_header: one DHT, order DC0, DC1, AC0, AC1 (default or optimal tables) */
    size += put_huffman_table(&pb, 0, 0, bits[0], vals[0]);
    size += put_huffman_table(&pb, 0, 1, bits[1], vals[1]);
    size += put_huffman_table(&pb, 1, 0, bits[2], vals[2]);
    size += put_huffman_table(&pb, 1, 1, bits[3], vals[3]);
    if (len_pos + 1 < cap) { out[len_pos] = (uint8_t)(size >> 8); out[len_pos + 1] = (uint8_t)size; }
    put16(&pb, 0xFFC0); put16(&pb, 17); put8(&pb, 8);   /* SOF0 */
    put16(&pb, height); put16(&pb, width); put8(&pb, 3);
    for (int c = 0; c < 3; c++) {                        /* id, HxV, Tq 0 (one matrix) */
        put8(&pb, c + 1); pb_put(&pb, 4, hs[c]); pb_put(&pb, 4, vs[c]); put8(&pb, 0);
    }
    put16(&pb, 0xFFDA); put16(&pb, 6 + 2 * 3); put8(&pb, 3);  /* SOS */
    put8(&pb, 1); pb_put(&pb, 4, 0); pb_put(&pb, 4, 0);
    put8(&pb, 2); pb_put(&pb, 4, 1); pb_put(&pb, 4, 1);
    put8(&pb, 3); pb_put(&pb, 4, 1); pb_put(&pb, 4, 1);
    put8(&pb, 0); put8(&pb, 63); put8(&pb, 0);
    if (pb.overflow) return 0;
    return pb.nbits >> 3;
}

/* mjpegenc_common.c ff_mjpeg_init_hvsample: (h, v) sampling factors of Y, Cb, Cr.
 * cfmt 0 = 4:2:0, 1 = 4:2:2, 2 = 4:4:4 (the 4:4:4 special case: every component 1x2, so an
 * MCU is 8x16 pixels). */
static void or_hvsample(int cfmt, int hs[3], int vs[3])
{
    if (cfmt == 2) { hs[0] = hs[1] = hs[2] = 1; vs[0] = vs[1] = vs[2] = 2; return; }
    hs[0] = 2; vs[0] = 2;
    hs[1] = hs[2] = 1;
    vs[1] = vs[2] = cfmt == 1 ? 2 : 1;
}

static size_t or_header_tables(int width, int height, int qscale, int sar_num, int sar_den,
                               int com_itu601, int dri_interval, const uint8_t *const bits[4],
                               const uint8_t *const vals[4], uint8_t *out, size_t cap)
{
    return or_header_fmt(width, height, 0, qscale, sar_num, sar_den, com_itu601, dri_interval,
                         bits, vals, out, cap);
}

static const uint8_t *const or_default_bits[4] = { or_bits_dc_lum, or_bits_dc_chr, or_bits_ac_lum, or_bits_ac_chr };
static const uint8_t *const or_default_vals[4] = { or_val_dc, or_val_dc, or_val_ac_lum, or_val_ac_chr };

size_t or_header(int width, int height, int qscale, int sar_num, int sar_den, int com_itu601,
                 int dri_interval, uint8_t *out, size_t cap)
{
    return or_header_tables(width, height, qscale, sar_num, sar_den, com_itu601, dri_interval,
                            or_default_bits, or_default_vals, out, cap);
}

/* The header for chroma format cfmt; rst != 0 adds the DRI segment slice threading writes
 * (jpeg_table_header: interval (width - 1) / (8 * hsample[0]) + 1 = MCUs per MCU row). */
size_t or_header_cfmt(int width, int height, int cfmt, int qscale, int sar_num, int sar_den,
                      int com_itu601, int rst, uint8_t *out, size_t cap)
{
    int hs[3], vs[3];
    if (cfmt < 0 || cfmt > 2) return 0;
    or_hvsample(cfmt, hs, vs);
    return or_header_fmt(width, height, cfmt, qscale, sar_num, sar_den, com_itu601,
                         rst ? (width - 1) / (8 * hs[0]) + 1 : 0, or_default_bits, or_default_vals,
                         out, cap);
}

/* ------------------------------------------------- -huffman optimal tables */
/* libavutil/qsort.h AV_QSORT (the in-place median-of-3 quicksort with an explicit stack
 * and the "already sorted" early exit), restated over elements of `size` bytes.  The
 * tie order it leaves matters: mjpegenc_huffman.c sorts symbol counts with it before
 * package-merge, and equal counts can end up with different code lengths. */
typedef int (*or_cmp_fn)(const void *, const void *);
static void or_memswap(void *a, void *b, size_t size)
{
    uint8_t t[16], *x = (uint8_t *)a, *y = (uint8_t *)b;
    if (a == b) return;
    memcpy(t, x, size); memcpy(x, y, size); memcpy(y, t, size);
}
static void or_av_qsort(void *base, int num, size_t size, or_cmp_fn cmp)
{
#define E(i) ((uint8_t *)base + (size_t)(i) * size)
    int stack[64][2];
    int sp = 1;
    stack[0][0] = 0;
    stack[0][1] = num - 1;
    while (sp) {
        int start = stack[--sp][0];
        int end = stack[sp][1];
        while (start < end) {
            if (start < end - 1) {
                int checksort = 0;
                int right = end - 2;
                int left = start + 1;
                int mid = start + ((end - start) >> 1);
                if (cmp(E(start), E(end)) > 0) {
                    if (cmp(E(end), E(mid)) > 0) or_memswap(E(start), E(mid), size);
                    else                         or_memswap(E(start), E(end), size);
                } else {
                    if (cmp(E(start), E(mid)) > 0) or_memswap(E(start), E(mid), size);
                    else checksort = 1;
                }
                if (cmp(E(mid), E(end)) > 0) {
                    or_memswap(E(mid), E(end), size);
                    checksort = 0;
                }
                if (start == end - 2) break;
                or_memswap(E(end - 1), E(mid), size);
                while (left <= right) {
                    while (left <= right && cmp(E(left), E(end - 1)) < 0) left++;
                    while (left <= right && cmp(E(right), E(end - 1)) > 0) right--;
                    if (left <= right) {
                        or_memswap(E(left), E(right), size);
                        left++;
                        right--;
                    }
                }
                or_memswap(E(end - 1), E(left), size);
                if (checksort && (mid == left - 1 || mid == left)) {
                    mid = start;
                    while (mid < end && cmp(E(mid), E(mid + 1)) <= 0) mid++;
                    if (mid == end) break;
                }
                if (end - left < left - start) {
                    stack[sp][0] = start;
                    stack[sp++][1] = right;
                    start = left + 1;
                } else {
                    stack[sp][0] = left + 1;
                    stack[sp++][1] = end;
                    end = right;
                }
            } else {
                if (cmp(E(start), E(end)) > 0) or_memswap(E(start), E(end), size);
                break;
            }
        }
    }
#undef E
}

/* mjpegenc_huffman.h PTable / HuffTable */
typedef struct { int value; int prob; } or_ptable;
typedef struct { int code; int length; } or_hufftable;

static int or_cmp_prob(const void *a, const void *b)
{
    return ((const or_ptable *)a)->prob - ((const or_ptable *)b)->prob;
}
static int or_cmp_length(const void *a, const void *b)
{
    const or_hufftable *x = (const or_hufftable *)a, *y = (const or_hufftable *)b;
    if (x->length == y->length) return x->code - y->code;
    return x->length - y->length;
}

/* mjpegenc_huffman.c ff_mjpegenc_huffman_compute_bits: package-merge limited to
 * max_length bits over prob_table (sorted here with AV_QSORT). */
typedef struct {
    int nitems;
    int item_idx[515];
    int probability[514];
    int items[257 * 16];
} or_pm_list;

static void or_huffman_compute_bits(or_ptable *prob_table, or_hufftable *distincts, int size,
                                    int max_length, int *ndistinct)
{
    or_pm_list list_a, list_b;  /* ~41 KB of stack: every call owns its lists (thread-safe) */
    or_pm_list *to = &list_a, *from = &list_b, *temp;
    int times, i = 0, j, k;
    int nbits[257] = { 0 };
    int min;

    to->nitems = 0;
    from->nitems = 0;
    to->item_idx[0] = 0;
    from->item_idx[0] = 0;
    or_av_qsort(prob_table, size, sizeof(or_ptable), or_cmp_prob);

    for (times = 0; times <= max_length; times++) {
        to->nitems = 0;
        to->item_idx[0] = 0;
        j = 0;
        k = 0;
        if (times < max_length) i = 0;
        while (i < size || j + 1 < from->nitems) {
            to->nitems++;
            to->item_idx[to->nitems] = to->item_idx[to->nitems - 1];
            if (i < size &&
                (j + 1 >= from->nitems ||
                 prob_table[i].prob < from->probability[j] + from->probability[j + 1])) {
                to->items[to->item_idx[to->nitems]++] = prob_table[i].value;
                to->probability[to->nitems - 1] = prob_table[i].prob;
                i++;
            } else {
                for (k = from->item_idx[j]; k < from->item_idx[j + 2]; k++)
                    to->items[to->item_idx[to->nitems]++] = from->items[k];
                to->probability[to->nitems - 1] = from->probability[j] + from->probability[j + 1];
                j += 2;
            }
        }
        temp = to;
        to = from;
        from = temp;
    }

    min = (size - 1 < from->nitems) ? size - 1 : from->nitems;
    for (i = 0; i < from->item_idx[min]; i++) nbits[from->items[i]]++;
    /* the 256 entry only prevents an all-ones code; it is not returned */
    j = 0;
    for (i = 0; i < 256; i++) {
        if (nbits[i] > 0) {
            distincts[j].code = i;
            distincts[j].length = nbits[i];
            j++;
        }
    }
    *ndistinct = j;
}

/* mjpegenc_huffman.c ff_mjpeg_encode_huffman_close: BITS/HUFFVAL of the optimal code for
 * one table's symbol counts.  Returns the number of values. */
int or_huff_optimal(const uint32_t counts[256], uint8_t bits[17], uint8_t vals[256])
{
    or_ptable val_counts[257];
    or_hufftable distincts[256];
    int nval = 0, nd = 0;
    for (int i = 0; i < 256; i++) {
        if (counts[i]) {
            val_counts[nval].value = i;
            val_counts[nval].prob = (int)counts[i];
            nval++;
        }
    }
    val_counts[nval].value = 256;
    val_counts[nval].prob = 0;
    or_huffman_compute_bits(val_counts, distincts, nval + 1, 16, &nd);
    or_av_qsort(distincts, nval, sizeof(or_hufftable), or_cmp_length);
    memset(bits, 0, 17);
    for (int i = 0; i < nval; i++) {
        vals[i] = (uint8_t)distincts[i].code;
        bits[distincts[i].length]++;
    }
    return nval;
}

/* ------------------------------------------------------- block gathering */
/* mpegvideo_enc.c encode_mb_internal: get_pixels of 4 luma + Cb + Cr blocks of
 * MB (mb_x, mb_y); partial MBs go through emulated_edge_mc (edge replication,
 * i.e. coordinate clamping) with cw = (W+1)>>1, ch = (H+1)>>1. */
static void or_get_block(int16_t *blk, const uint8_t *plane, int stride, int pw, int ph,
                         int x0, int y0)
{
    for (int y = 0; y < 8; y++) {
        int sy = y0 + y; if (sy > ph - 1) sy = ph - 1;
        for (int x = 0; x < 8; x++) {
            int sx = x0 + x; if (sx > pw - 1) sx = pw - 1;
            blk[y * 8 + x] = plane[(size_t)sy * stride + sx];
        }
    }
}

/* MCU layouts per chroma format (cfmt 0 = 4:2:0, 1 = 4:2:2, 2 = 4:4:4).
 * mpegvideo_enc.c encode_mb_internal numbers a 16x16 macroblock's blocks 0-3 = Y TL TR BL
 * BR, 4/5 = Cb/Cr top (left), 6/7 = Cb/Cr bottom (4:2:2) or right (4:4:4), 8-11 = Cb/Cr
 * bottom-left, Cb/Cr bottom-right (4:4:4); mjpegenc.c ff_mjpeg_encode_mb codes them as
 *   4:2:0  0 1 2 3 4 5             (MCU 16x16: Y 2x2, Cb 1x1, Cr 1x1)
 *   4:2:2  0 1 2 3 4 6 5 7         (MCU 16x16: Y 2x2, Cb 1x2, Cr 1x2)
 *   4:4:4  0 2 4 8 5 9 | 1 3 6 10 7 11   (two 8x16 MCUs per macroblock, every component 1x2;
 *          the right one only when 16*mb_x + 8 < width)
 * so in MCU units every format is a raster of MCUs of `bpm` blocks whose (plane, dx, dy)
 * is fixed; `n` is FFmpeg's block number, which selects the component (n < 4: Y, else
 * (n & 1) + 1) and the Huffman table in encode_block. */
typedef struct { int n, plane, dx, dy; } or_blk;
typedef struct { int bpm, mcu_w[3], mcu_h[3], hshift, vshift; or_blk b[8]; } or_layout;
static const or_layout or_layouts[3] = {
    { 6, { 16, 8, 8 }, { 16, 8, 8 }, 1, 1,
      { { 0, 0, 0, 0 }, { 1, 0, 8, 0 }, { 2, 0, 0, 8 }, { 3, 0, 8, 8 }, { 4, 1, 0, 0 }, { 5, 2, 0, 0 } } },
    { 8, { 16, 8, 8 }, { 16, 16, 16 }, 1, 0,
      { { 0, 0, 0, 0 }, { 1, 0, 8, 0 }, { 2, 0, 0, 8 }, { 3, 0, 8, 8 }, { 4, 1, 0, 0 }, { 6, 1, 0, 8 },
        { 5, 2, 0, 0 }, { 7, 2, 0, 8 } } },
    { 6, { 8, 8, 8 }, { 16, 16, 16 }, 0, 0,
      { { 0, 0, 0, 0 }, { 2, 0, 0, 8 }, { 4, 1, 0, 0 }, { 8, 1, 0, 8 }, { 5, 2, 0, 0 }, { 9, 2, 0, 8 } } },
};

/* MCUs per row / per column of a w x h frame in chroma format cfmt. */
void or_mcu_grid(int cfmt, int w, int h, int *mcw, int *mch)
{
    const or_layout *L = &or_layouts[cfmt];
    *mcw = (w + L->mcu_w[0] - 1) / L->mcu_w[0];
    *mch = (h + 15) / 16;
}

/* Quantized coefficients of every block of one frame in chroma format cfmt, natural
 * order, in coding order (MCU raster, the layout's blocks per MCU), plus last_index per
 * block.  Chroma planes are ((w + hshift) >> hshift) x ((h + vshift) >> vshift); partial
 * MCUs replicate the plane's last row/column (emulated_edge_mc).  Exposed so the GPU's
 * intermediate products can be compared block by block. */
int or_frame_coeffs_cfmt(const uint8_t *y, int ys, const uint8_t *u, int us, const uint8_t *v, int vs,
                         int w, int h, int cfmt, int qscale, int16_t *coef_out, int8_t *last_out)
{
    if (cfmt < 0 || cfmt > 2) return -1;
    const or_layout *L = &or_layouts[cfmt];
    uint8_t mprime[64]; int32_t qmat[64];
    or_build_matrix(qscale, mprime, qmat);
    int mcw, mch;
    or_mcu_grid(cfmt, w, h, &mcw, &mch);
    const uint8_t *pl[3] = { y, u, v };
    const int st[3] = { ys, us, vs };
    const int pw[3] = { w, (w + L->hshift) >> L->hshift, (w + L->hshift) >> L->hshift };
    const int ph[3] = { h, (h + L->vshift) >> L->vshift, (h + L->vshift) >> L->vshift };
    size_t b = 0;
    for (int my = 0; my < mch; my++)
        for (int mx = 0; mx < mcw; mx++)
            for (int j = 0; j < L->bpm; j++, b++) {
                const or_blk *d = &L->b[j];
                int16_t *blk = coef_out + b * 64;
                or_get_block(blk, pl[d->plane], st[d->plane], pw[d->plane], ph[d->plane],
                             mx * L->mcu_w[d->plane] + d->dx, my * L->mcu_h[d->plane] + d->dy);
                or_fdct_islow(blk);
                last_out[b] = (int8_t)or_quantize(blk, qmat);
            }
    return 0;
}

int or_frame_coeffs(const uint8_t *y, int ys, const uint8_t *u, int us, const uint8_t *v, int vs,
                    int w, int h, int qscale, int16_t *coef_out, int8_t *last_out)
{
    return or_frame_coeffs_cfmt(y, ys, u, us, v, vs, w, h, 0, qscale, coef_out, last_out);
}

/* ----------------------------------------------------------- full frame */
/* mjpegenc_common.c ff_mjpeg_escape_FF (+ the 1-bit padding of ff_mjpeg_encode_stuffing):
 * pad the entropy-coded segment in seg to a byte boundary with 1-bits and append its bytes
 * to out[*pos] with a 0x00 after every 0xFF.  Returns 0, or -1 on overflow. */
static int or_flush_segment(or_pb *seg, uint8_t *out, size_t cap, size_t *pos)
{
    int pad = (int)((8 - (seg->nbits & 7)) & 7);
    if (pad) pb_put(seg, pad, (1u << pad) - 1);
    if (seg->overflow) return -1;
    size_t size = seg->nbits >> 3;
    for (size_t i = 0; i < size; i++) {
        if (*pos + 2 > cap) return -1;
        out[(*pos)++] = seg->buf[i];
        if (seg->buf[i] == 0xFF) out[(*pos)++] = 0x00;
    }
    seg->nbits = 0;
    return 0;
}

/* One frame in chroma format cfmt:
 *   header (ff_mjpeg_encode_picture_header), scan, EOI (ff_mjpeg_encode_picture_trailer).
 * rst = 0 (frame threading, the default): one entropy-coded segment, padded and escaped.
 * rst = 1 (slice threading: -slices N or -thread_type slice; mpegvideo_enc.c sets rtp_mode
 *   and encode_thread's MJPEG case starts a "GOB" at every mb_x == 0, mb_y != 0, i.e.
 *   write_slice_end -> ff_mjpeg_encode_stuffing at the end of every MCU row): each MCU row
 *   is its own segment -- padded with 1-bits, escaped, followed by RST0 + (row & 7) unless
 *   it is the last row -- and the DC predictors restart at 128 in every row.  Slice
 *   threading forces -huffman default (mjpegenc.c: slice_context_count > 1), so
 *   huff_optimal with rst is rejected here.
 * huff_optimal: mjpegenc.c ff_mjpeg_encode_stuffing -> mjpeg_build_optimal_huffman: the
 *   picture's symbols are buffered, counted, and the tables built before the header and
 *   the scan are written. */
size_t or_encode_planes_cfmt(const uint8_t *y, int ys, const uint8_t *u, int us, const uint8_t *v, int vs,
                             int w, int h, int cfmt, int qscale, int sar_num, int sar_den, int com_itu601,
                             int huff_optimal, int rst, uint8_t *out, size_t cap)
{
    if (cfmt < 0 || cfmt > 2 || (rst && huff_optimal)) return 0;
    const or_layout *L = &or_layouts[cfmt];
    int mcw, mch;
    or_mcu_grid(cfmt, w, h, &mcw, &mch);
    if (mch < 2) rst = 0;   /* mpegvideo: nb_slices is clipped to mb_height */
    const int bpm = L->bpm;
    size_t nblocks = (size_t)mcw * mch * bpm;
    int16_t *coef = (int16_t *)malloc(nblocks * 64 * sizeof(int16_t));
    int8_t *last = (int8_t *)malloc(nblocks);
    size_t seg_cap = nblocks * 210 + 64;     /* worst case ~1664 bits per block */
    uint8_t *segbuf = (uint8_t *)malloc(seg_cap);
    if (!coef || !last || !segbuf) { free(coef); free(last); free(segbuf); return 0; }
    or_frame_coeffs_cfmt(y, ys, u, us, v, vs, w, h, cfmt, qscale, coef, last);

    const uint8_t *bits[4], *vals[4];
    uint8_t obits[4][17], ovals[4][256];
    for (int t = 0; t < 4; t++) { bits[t] = or_default_bits[t]; vals[t] = or_default_vals[t]; }
    if (huff_optimal) {
        uint32_t counts[4][256];
        int last_dc[3] = { 128, 128, 128 };
        memset(counts, 0, sizeof counts);
        for (size_t b = 0; b < nblocks; b++)
            or_count_block(counts, coef + b * 64, L->b[b % bpm].n, last[b], last_dc);
        for (int t = 0; t < 4; t++) {
            or_huff_optimal(counts[t], obits[t], ovals[t]);
            bits[t] = obits[t];
            vals[t] = ovals[t];
        }
    }
    int hs[3], vs3[3];
    or_hvsample(cfmt, hs, vs3);
    size_t pos = or_header_fmt(w, h, cfmt, qscale, sar_num, sar_den, com_itu601,
                               rst ? (w - 1) / (8 * hs[0]) + 1 : 0, bits, vals, out, cap);
    int ok = pos != 0;

    or_huff hf; or_huff_init_tables(&hf, bits, vals);
    or_pb seg = { segbuf, seg_cap, 0, 0 };
    int last_dc[3] = { 128, 128, 128 };
    const size_t row_blocks = (size_t)mcw * bpm;
    for (size_t b = 0; ok && b < nblocks; b++) {
        or_encode_block(&seg, &hf, coef + b * 64, L->b[b % bpm].n, last[b], last_dc);
        if (rst && (b + 1) % row_blocks == 0 && b + 1 < nblocks) {
            const int row = (int)(b / row_blocks);
            ok = or_flush_segment(&seg, out, cap, &pos) == 0 && pos + 2 <= cap;
            if (ok) { out[pos++] = 0xFF; out[pos++] = (uint8_t)(0xD0 + (row & 7)); }
            last_dc[0] = last_dc[1] = last_dc[2] = 128;
        }
    }
    if (ok) ok = or_flush_segment(&seg, out, cap, &pos) == 0 && pos + 2 <= cap;
    free(coef); free(last); free(segbuf);
    if (!ok) return 0;
    out[pos++] = 0xFF; out[pos++] = 0xD9;             /* EOI */
    return pos;
}

size_t or_encode_planes_ex(const uint8_t *y, int ys, const uint8_t *u, int us, const uint8_t *v, int vs,
                           int w, int h, int qscale, int sar_num, int sar_den, int com_itu601,
                           int huff_optimal, uint8_t *out, size_t cap)
{
    return or_encode_planes_cfmt(y, ys, u, us, v, vs, w, h, 0, qscale, sar_num, sar_den, com_itu601,
                                 huff_optimal, 0, out, cap);
}

size_t or_encode_planes(const uint8_t *y, int ys, const uint8_t *u, int us, const uint8_t *v, int vs,
                        int w, int h, int qscale, int sar_num, int sar_den, int com_itu601,
                        uint8_t *out, size_t cap)
{
    return or_encode_planes_ex(y, ys, u, us, v, vs, w, h, qscale, sar_num, sar_den, com_itu601, 0,
                               out, cap);
}

/* ================================================================ swscale */
/* libswscale/utils.c initFilter for SWS_BICUBIC (B = 0, C = 0.6 defaults),
 * generic branch (xInc != 1<<16 or srcPos != dstPos) and the unscaled branch,
 * followed by the reduce / align / border-fix / normalise steps.
 *   one: 1<<14 (horizontal) or 1<<12 (vertical)
 *   filter_align: x86 MMX value (4 horizontal, 2 vertical)
 *   bitexact: SWS_BITEXACT (zero taps beyond minFilterSize)
 * Outputs: filter[dstW * (*out_size)] int16, pos[dstW] int32, *out_size.
 * Returns 0, or -1 if max_size is too small. */
#define OR_SWS_MAX_REDUCE_CUTOFF 0.002
static int or_av_log2(unsigned v) { int n = 0; while (v >>= 1) n++; return n; }

int or_sws_init_filter(int srcW, int dstW, int one, int filter_align, int bitexact,
                       int srcPos, int dstPos, int16_t *out_filter, int32_t *out_pos,
                       int *out_size, int max_size)
{
    int64_t xInc = (((int64_t)srcW << 16) + (dstW >> 1)) / dstW;
    const int64_t fone = 1LL << (54 - (or_av_log2((unsigned)(srcW / dstW)) < 8 ? or_av_log2((unsigned)(srcW / dstW)) : 8));
    int filterSize;
    int64_t *filter = NULL;
    int32_t *pos = out_pos;

    if (llabs(xInc - 0x10000) < 10 && srcPos == dstPos) {
        filterSize = 1;
        filter = (int64_t *)calloc((size_t)dstW * filterSize, sizeof(int64_t));
        for (int i = 0; i < dstW; i++) { filter[i] = fone; pos[i] = i; }
    } else {
        const int sizeFactor = 4; /* bicubic */
        if (xInc <= 1 << 16) filterSize = 1 + sizeFactor;
        else filterSize = 1 + (int)((sizeFactor * (int64_t)srcW + dstW - 1) / dstW);
        if (filterSize > srcW - 2) filterSize = srcW - 2;
        if (filterSize < 1) filterSize = 1;
        filter = (int64_t *)calloc((size_t)dstW * filterSize, sizeof(int64_t));
        int64_t xDstInSrc = ((dstPos * (int64_t)xInc) >> 7) - ((srcPos * 0x10000LL) >> 7);
        for (int i = 0; i < dstW; i++) {
            int xx = (int)((xDstInSrc - (filterSize - 2) * (1LL << 16)) / (1 << 17));
            pos[i] = xx;
            for (int j = 0; j < filterSize; j++) {
                int64_t d = (llabs(((int64_t)xx * (1 << 17)) - xDstInSrc)) << 13;
                int64_t coeff;
                if (xInc > 1 << 16) d = d * dstW / srcW;
                {
                    int64_t B = (int64_t)(0.0 * (1 << 24));
                    int64_t C = (int64_t)(0.6 * (1 << 24));
                    if (d >= 1LL << 31) {
                        coeff = 0;
                    } else {
                        int64_t dd = (d * d) >> 30;
                        int64_t ddd = (dd * d) >> 30;
                        if (d < 1LL << 30)
                            coeff = (12 * (1 << 24) - 9 * B - 6 * C) * ddd +
                                    (-18 * (1 << 24) + 12 * B + 6 * C) * dd +
                                    (6 * (1 << 24) - 2 * B) * (1 << 30);
                        else
                            coeff = (-B - 6 * C) * ddd +
                                    (6 * B + 30 * C) * dd +
                                    (-12 * B - 48 * C) * d +
                                    (8 * B + 24 * C) * (1 << 30);
                    }
                    coeff /= (1LL << 54) / fone;
                }
                filter[i * filterSize + j] = coeff;
                xx++;
            }
            xDstInSrc += 2LL * xInc;
        }
    }

    /* no src/dst vectors: filter2 = filter */
    int filter2Size = filterSize;
    int64_t *filter2 = filter;

    /* reduce step 1 */
    int minFilterSize = 0;
    for (int i = dstW - 1; i >= 0; i--) {
        int min = filter2Size;
        int64_t cutOff = 0;
        for (int j = 0; j < filter2Size; j++) {
            cutOff += llabs(filter2[i * filter2Size]);
            if (cutOff > OR_SWS_MAX_REDUCE_CUTOFF * fone) break;
            if (i < dstW - 1 && pos[i] >= pos[i + 1]) break;
            int k;
            for (k = 1; k < filter2Size; k++)
                filter2[i * filter2Size + k - 1] = filter2[i * filter2Size + k];
            filter2[i * filter2Size + k - 1] = 0;
            pos[i]++;
        }
        cutOff = 0;
        for (int j = filter2Size - 1; j > 0; j--) {
            cutOff += llabs(filter2[i * filter2Size + j]);
            if (cutOff > OR_SWS_MAX_REDUCE_CUTOFF * fone) break;
            min--;
        }
        if (min > minFilterSize) minFilterSize = min;
    }
    /* x86: special case for unscaled vertical filtering */
    if (minFilterSize == 1 && filter_align == 2) filter_align = 1;

    filterSize = (minFilterSize + (filter_align - 1)) & ~(filter_align - 1);
    if (filterSize > max_size) { free(filter); return -1; }
    int64_t *f = (int64_t *)calloc((size_t)dstW * filterSize, sizeof(int64_t));
    for (int i = 0; i < dstW; i++)
        for (int j = 0; j < filterSize; j++) {
            f[i * filterSize + j] = (j >= filter2Size) ? 0 : filter2[i * filter2Size + j];
            if (bitexact && j >= minFilterSize) f[i * filterSize + j] = 0;
        }
    free(filter);

    /* fix borders */
    for (int i = 0; i < dstW; i++) {
        if (pos[i] < 0) {
            for (int j = 1; j < filterSize; j++) {
                int left = j + pos[i] > 0 ? j + pos[i] : 0;
                f[i * filterSize + left] += f[i * filterSize + j];
                f[i * filterSize + j] = 0;
            }
            pos[i] = 0;
        }
        if (pos[i] + filterSize > srcW) {
            int shift = pos[i] + (filterSize - srcW < 0 ? filterSize - srcW : 0);
            int64_t acc = 0;
            for (int j = filterSize - 1; j >= 0; j--) {
                if (pos[i] + j >= srcW) { acc += f[i * filterSize + j]; f[i * filterSize + j] = 0; }
            }
            for (int j = filterSize - 1; j >= 0; j--) {
                if (j < shift) f[i * filterSize + j] = 0;
                else f[i * filterSize + j] = f[i * filterSize + j - shift];
            }
            pos[i] -= shift;
            f[i * filterSize + srcW - 1 - pos[i]] += acc;
        }
    }

    /* normalise with error diffusion */
    for (int i = 0; i < dstW; i++) {
        int64_t error = 0, sum = 0;
        for (int j = 0; j < filterSize; j++) sum += f[i * filterSize + j];
        sum = (sum + one / 2) / one;
        if (!sum) sum = 1;
        for (int j = 0; j < filterSize; j++) {
            int64_t v = f[i * filterSize + j] + error;
            int64_t intV = v >= 0 ? (v + (sum >> 1)) / sum : (v - (sum >> 1)) / sum; /* ROUNDED_DIV */
            out_filter[i * filterSize + j] = (int16_t)intV;
            error = v - intV * sum;
        }
    }
    free(f);
    *out_size = filterSize;
    return 0;
}

/* libswscale/hscale.c hScale8To15_c + swscale.c lumRangeToJpeg_c / chrRangeToJpeg_c
 * (FFmpeg <= 7.0 constants) + output.c yuv2planeX_8_c / yuv2plane1_8_c with the flat
 * 64 dither used for 8-bit sources.  range: 0 none, 1 luma tv->pc, 2 chroma tv->pc. */
static inline int16_t or_range(int v, int range)
{
    if (range == 1) { if (v > 30189) v = 30189; return (int16_t)((v * 19077 - 39057361) >> 14); }
    if (range == 2) { if (v > 30775) v = 30775; return (int16_t)((v * 4663 - 9289992) >> 12); }
    return (int16_t)v;
}

int or_scale_plane(const uint8_t *src, int sstride, int sw, int sh,
                   uint8_t *dst, int dstride, int dw, int dh, int range, int bitexact,
                   int src_pos_h, int dst_pos_h, int src_pos_v, int dst_pos_v)
{
    const int MAXF = 256;
    int16_t *hf = (int16_t *)malloc((size_t)dw * MAXF * sizeof(int16_t));
    int32_t *hp = (int32_t *)malloc((size_t)dw * sizeof(int32_t));
    int16_t *vf = (int16_t *)malloc((size_t)dh * MAXF * sizeof(int16_t));
    int32_t *vp = (int32_t *)malloc((size_t)dh * sizeof(int32_t));
    int hs, vs;
    if (or_sws_init_filter(sw, dw, 1 << 14, 4, bitexact, src_pos_h, dst_pos_h, hf, hp, &hs, MAXF) ||
        or_sws_init_filter(sh, dh, 1 << 12, 2, bitexact, src_pos_v, dst_pos_v, vf, vp, &vs, MAXF)) {
        free(hf); free(hp); free(vf); free(vp); return -1;
    }
    int16_t *rows = (int16_t *)malloc((size_t)sh * dw * sizeof(int16_t));
    for (int y = 0; y < sh; y++) {
        const uint8_t *s = src + (size_t)y * sstride;
        for (int i = 0; i < dw; i++) {
            int val = 0;
            for (int j = 0; j < hs; j++) val += (int)s[hp[i] + j] * hf[i * hs + j];
            val >>= 7;
            if (val > 32767) val = 32767;
            rows[(size_t)y * dw + i] = or_range(val, range);
        }
    }
    for (int y = 0; y < dh; y++) {
        for (int i = 0; i < dw; i++) {
            int val = 64 << 12;
            for (int j = 0; j < vs; j++) val += rows[(size_t)(vp[y] + j) * dw + i] * vf[y * vs + j];
            val >>= 19;
            dst[(size_t)y * dstride + i] = (uint8_t)(val < 0 ? 0 : val > 255 ? 255 : val);
        }
    }
    free(rows); free(hf); free(hp); free(vf); free(vp);
    return 0;
}

/* swscale: get_local_pos default siting (pos = -513 -> centred) for a plane with
 * chroma subsampling shift `sub`. */
int or_local_pos(int sub, int pos)
{
    if (pos == -1 || pos <= -513) pos = (128 << sub) - 128;
    pos += 128;
    return pos >> sub;
}

/* Full worker path for one frame of chroma format cfmt (yuv420p/422p/444p or their yuvj
 * variants): optional bicubic resize and the auto-inserted tv->pc conversion (swscale
 * context yuv4xxp -> yuvj4xxp), then the mjpeg encode.  in_full_range: 1 for yuvj input
 * (no conversion).  Chroma siting per direction: get_local_pos(shift, -513). */
size_t or_encode_frame_cfmt(const uint8_t *y, int ys, const uint8_t *u, int us, const uint8_t *v, int vs,
                            int sw, int sh, int dw, int dh, int cfmt, int in_full_range, int qscale,
                            int sar_num, int sar_den, int bitexact_sws, int huff_optimal, int rst,
                            uint8_t *out, size_t cap)
{
    if (cfmt < 0 || cfmt > 2) return 0;
    int need_sws = (sw != dw || sh != dh || !in_full_range);
    if (!need_sws)
        return or_encode_planes_cfmt(y, ys, u, us, v, vs, sw, sh, cfmt, qscale, sar_num, sar_den, 0,
                                     huff_optimal, rst, out, cap);
    const int hsh = or_layouts[cfmt].hshift, vsh = or_layouts[cfmt].vshift;
    int dcw = (dw + hsh) >> hsh, dch = (dh + vsh) >> vsh, scw = (sw + hsh) >> hsh, sch = (sh + vsh) >> vsh;
    uint8_t *Y = (uint8_t *)malloc((size_t)dw * dh);
    uint8_t *U = (uint8_t *)malloc((size_t)dcw * dch);
    uint8_t *V = (uint8_t *)malloc((size_t)dcw * dch);
    int rl = in_full_range ? 0 : 1, rc = in_full_range ? 0 : 2;
    int lp = or_local_pos(0, 0), cph = or_local_pos(hsh, -513), cpv = or_local_pos(vsh, -513);
    size_t n = 0;
    if (Y && U && V &&
        !or_scale_plane(y, ys, sw, sh, Y, dw, dw, dh, rl, bitexact_sws, lp, lp, lp, lp) &&
        !or_scale_plane(u, us, scw, sch, U, dcw, dcw, dch, rc, bitexact_sws, cph, cph, cpv, cpv) &&
        !or_scale_plane(v, vs, scw, sch, V, dcw, dcw, dch, rc, bitexact_sws, cph, cph, cpv, cpv))
        n = or_encode_planes_cfmt(Y, dw, U, dcw, V, dcw, dw, dh, cfmt, qscale, sar_num, sar_den, 0,
                                  huff_optimal, rst, out, cap);
    free(Y); free(U); free(V);
    return n;
}

size_t or_encode_frame_ex(const uint8_t *y, int ys, const uint8_t *u, int us, const uint8_t *v, int vs,
                          int sw, int sh, int dw, int dh, int in_full_range, int qscale,
                          int sar_num, int sar_den, int bitexact_sws, int huff_optimal,
                          uint8_t *out, size_t cap)
{
    return or_encode_frame_cfmt(y, ys, u, us, v, vs, sw, sh, dw, dh, 0, in_full_range, qscale, sar_num,
                                sar_den, bitexact_sws, huff_optimal, 0, out, cap);
}

size_t or_encode_frame(const uint8_t *y, int ys, const uint8_t *u, int us, const uint8_t *v, int vs,
                       int sw, int sh, int dw, int dh, int in_full_range, int qscale,
                       int sar_num, int sar_den, int bitexact_sws, uint8_t *out, size_t cap)
{
    return or_encode_frame_ex(y, ys, u, us, v, vs, sw, sh, dw, dh, in_full_range, qscale, sar_num,
                              sar_den, bitexact_sws, 0, out, cap);
}
