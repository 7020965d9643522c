/*
 * clahe.c -- CPU restatement of Tracking::preprocessing's image steps
 * (TEST INFRASTRUCTURE ONLY; see gvx_oracle.h).
 *
 *   orc_clahe       clahe_->apply(image, image) at
 *                   ic_gvins/ic_gvins/tracking/tracking.cc:139 with
 *                   clahe_ = cv::createCLAHE(3.0, cv::Size(21, 21)) (:63):
 *                   OpenCV 4.x CLAHE_Impl::apply (modules/imgproc/src/clahe.cpp,
 *                   un-vendored), 8-bit path:
 *                   - tile size: if w % tx == 0 and h % ty == 0, (w/tx, h/ty);
 *                     otherwise the LUT source is copyMakeBorder(src, 0,
 *                     ty - h%ty, 0, tx - w%tx, BORDER_REFLECT_101) (note: a full
 *                     extra tile of rows/columns when only the other side is
 *                     indivisible) and the tile size is its size / (tx, ty);
 *                   - clip = max(int(clipLimit * tw*th / 256), 1) when
 *                     clipLimit > 0; lutScale = float(255) / (tw*th);
 *                   - CLAHE_CalcLut_Body: tile histogram, clip, redistribute
 *                     clipped/256 to every bin, then the residual one by one
 *                     at bins 0, s, 2s, ... with s = max(256/residual, 1);
 *                     lut[i] = saturate_cast<uchar>(cumsum_i * lutScale);
 *                   - CLAHE_Interpolation_Body (scalar form): per pixel,
 *                     txf = x * (1.0f/tw) - 0.5f, tx1 = floor, xa = txf - tx1,
 *                     likewise y; clamp tile indices; res = (L11*xa1 + L12*xa)*ya1
 *                     + (L21*xa1 + L22*xa)*ya in float; dst = saturate_cast<uchar>
 *                     (round half to even).
 *   orc_hist_mean   Tracking::calculateHistigram (tracking.cc:88-105):
 *                   sum_k double(float(hist[k]) * float(k)) / 256.0, then / (w*h).
 *
 * Parity unpinned: OpenCV is not present here and the reference has no CLAHE
 * fixtures; pinned by the known answers in tests/test_oracle_clahe.py and an
 * independent numpy restatement of the same rules.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gvx_oracle.h"

static int reflect101(int i, int n) {
    if (n == 1) return 0;
    while (i < 0 || i >= n) i = i < 0 ? -i : 2 * (n - 1) - i;
    return i;
}

static uint8_t sat_round_u8(float v) {
    /* cv::saturate_cast<uchar>(float) = saturate(cvRound(v)), round half to even */
    int r = (int)lrintf(v);
    return (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

void orc_clahe_geometry(int w, int h, int tiles_x, int tiles_y, int* tw, int* th, int* ext_w, int* ext_h) {
    int ew = w, eh = h;
    if (!(w % tiles_x == 0 && h % tiles_y == 0)) {
        ew = w + tiles_x - (w % tiles_x);
        eh = h + tiles_y - (h % tiles_y);
    }
    *ext_w = ew;
    *ext_h = eh;
    *tw = ew / tiles_x;
    *th = eh / tiles_y;
}

void orc_clahe_luts(const uint8_t* src, int w, int h, int stride, double clip_limit, int tiles_x,
                    int tiles_y, uint8_t* lut /* tiles_y*tiles_x*256 */) {
    int tw, th, ew, eh;
    orc_clahe_geometry(w, h, tiles_x, tiles_y, &tw, &th, &ew, &eh);
    const int total = tw * th;
    const float lut_scale = (float)255 / total;
    int clip = 0;
    if (clip_limit > 0.0) {
        clip = (int)(clip_limit * total / 256);
        if (clip < 1) clip = 1;
    }
    for (int k = 0; k < tiles_x * tiles_y; ++k) {
        const int ty = k / tiles_x, tx = k % tiles_x;
        int hist[256];
        memset(hist, 0, sizeof hist);
        for (int y = ty * th; y < (ty + 1) * th; ++y) {
            const int sy = reflect101(y, h);
            for (int x = tx * tw; x < (tx + 1) * tw; ++x) hist[src[(size_t)sy * stride + reflect101(x, w)]]++;
        }
        if (clip > 0) {
            int clipped = 0;
            for (int i = 0; i < 256; ++i)
                if (hist[i] > clip) {
                    clipped += hist[i] - clip;
                    hist[i] = clip;
                }
            const int batch = clipped / 256;
            int residual = clipped - batch * 256;
            for (int i = 0; i < 256; ++i) hist[i] += batch;
            if (residual != 0) {
                int step = 256 / residual;
                if (step < 1) step = 1;
                for (int i = 0; i < 256 && residual > 0; i += step, residual--) hist[i]++;
            }
        }
        int sum = 0;
        for (int i = 0; i < 256; ++i) {
            sum += hist[i];
            lut[(size_t)k * 256 + i] = sat_round_u8((float)sum * lut_scale);
        }
    }
}

void orc_clahe(const uint8_t* src, int w, int h, int stride, double clip_limit, int tiles_x, int tiles_y,
               uint8_t* dst, int dst_stride) {
    int tw, th, ew, eh;
    orc_clahe_geometry(w, h, tiles_x, tiles_y, &tw, &th, &ew, &eh);
    uint8_t* lut = (uint8_t*)malloc((size_t)tiles_x * tiles_y * 256);
    orc_clahe_luts(src, w, h, stride, clip_limit, tiles_x, tiles_y, lut);
    const float inv_tw = 1.0f / tw, inv_th = 1.0f / th;
    for (int y = 0; y < h; ++y) {
        const float tyf = (float)y * inv_th - 0.5f;
        int ty1 = (int)floorf(tyf);
        int ty2 = ty1 + 1;
        const float ya = tyf - (float)ty1, ya1 = 1.0f - ya;
        if (ty1 < 0) ty1 = 0;
        if (ty2 > tiles_y - 1) ty2 = tiles_y - 1;
        const uint8_t* p1 = lut + (size_t)ty1 * tiles_x * 256;
        const uint8_t* p2 = lut + (size_t)ty2 * tiles_x * 256;
        for (int x = 0; x < w; ++x) {
            const float txf = (float)x * inv_tw - 0.5f;
            int tx1 = (int)floorf(txf);
            int tx2 = tx1 + 1;
            const float xa = txf - (float)tx1, xa1 = 1.0f - xa;
            if (tx1 < 0) tx1 = 0;
            if (tx2 > tiles_x - 1) tx2 = tiles_x - 1;
            const int v = src[(size_t)y * stride + x];
            const int i1 = tx1 * 256 + v, i2 = tx2 * 256 + v;
            const float res = ((float)p1[i1] * xa1 + (float)p1[i2] * xa) * ya1 +
                              ((float)p2[i1] * xa1 + (float)p2[i2] * xa) * ya;
            dst[(size_t)y * dst_stride + x] = sat_round_u8(res);
        }
    }
    free(lut);
}

double orc_hist_mean(const uint8_t* src, int w, int h, int stride) {
    int hist[256];
    memset(hist, 0, sizeof hist);
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) hist[src[(size_t)y * stride + x]]++;
    double m = 0;
    for (int k = 0; k < 256; ++k) m += (double)((float)hist[k] * (float)k) / 256.0;
    return m / (w * h);
}

/* RGB2Gray<uchar> (imgproc/src/color_rgb.simd.hpp, OpenCV 4.x) with blueIdx = 0:
   tab[i] = i*B2Y, tab[256+i] = i*G2Y, tab[512+i] = i*R2Y + (1 << 13), yuv_shift 14,
   R2Y = 4899, G2Y = 9617, B2Y = 1868 -- the integer sum, whatever the SIMD path. */
void orc_bgr2gray(const uint8_t* bgr, int w, int h, int stride, uint8_t* gray, int gray_stride) {
    for (int y = 0; y < h; y++) {
        const uint8_t* s = bgr + (size_t)y * stride;
        uint8_t* d = gray + (size_t)y * gray_stride;
        for (int x = 0; x < w; x++)
            d[x] = (uint8_t)((s[3 * x] * 1868 + s[3 * x + 1] * 9617 + s[3 * x + 2] * 4899 + (1 << 13)) >> 14);
    }
}
