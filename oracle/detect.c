/*
 * detect.c -- TEST INFRASTRUCTURE (parity oracle + CPU baseline), see gvx_oracle.h.
 *
 * Restates Tracking::featuresDetection (ic_gvins/ic_gvins/tracking/tracking.cc:576-688)
 * with its block grid (tracking.cc:65-85), the FILLED circle mask (:609-620),
 * and the OpenCV 4.x routines it calls per block: goodFeaturesToTrack
 * (cornerMinEigenVal, threshold TOZERO, 3x3 dilate, sorted candidates with the
 * address tie-break, grid suppression) and cornerSubPix/getRectSubPix.
 * Semantics: SURVEY.md Appendix A.4-A.6, OpenCV scalar paths, no FMA.
 * Parity vs. a real OpenCV binary is unpinned (see gvx_oracle.h).
 */
#include "gvx_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

static int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        if (p < 0)
            p = -p;
        else
            p = 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}
static int cv_round_f(float v) { return (int)lrintf(v); }
static int cv_round_d(double v) { return (int)lrint(v); }
static int cv_floor(float v) {
    int i = (int)v;
    return i - (i > v);
}

void orc_detect_params_default(orc_detect_params* p) {
    p->block_size = 200.0;
    p->max_features = 150;
    p->quality = 0.01;
    p->subpix_win = 5;
    p->subpix_iters = 20;
    p->subpix_eps = 0.01;
}

void orc_block_grid_make(int w, int h, const orc_detect_params* p, orc_block_grid* g) {
    g->block_cols = (int)lround(w / p->block_size);
    g->block_rows = (int)lround(h / p->block_size);
    g->block_cnts = g->block_cols * g->block_rows;
    g->row = h / g->block_rows;
    g->col = w / g->block_cols;
    g->max_block_features =
        (int)lround((double)p->max_features / (double)g->block_cnts);
    g->min_pixel_distance = (int)round(p->block_size / sqrt(g->max_block_features * 1.5));
}

/* cv::circle(..., FILLED, LINE_8, shift 0) -> Circle(img, center, r, color, fill=1)
   (imgproc/src/drawing.cpp), colour 0. */
void orc_mask_circles(uint8_t* mask, int w, int h, const float* xy, int n, int radius) {
    for (int i = 0; i < n; i++) {
        int cx = cv_round_f(xy[2 * i]), cy = cv_round_f(xy[2 * i + 1]);
        int err = 0, dx = radius, dy = 0, plus = 1, minus = (radius << 1) - 1;
        while (dx >= dy) {
            int spans[4][3] = {{cy - dy, cx - dx, cx + dx},
                               {cy + dy, cx - dx, cx + dx},
                               {cy - dx, cx - dy, cx + dy},
                               {cy + dx, cx - dy, cx + dy}};
            for (int s = 0; s < 4; s++) {
                int y = spans[s][0], x1 = spans[s][1], x2 = spans[s][2];
                if (y < 0 || y >= h) continue;
                if (x1 < 0) x1 = 0;
                if (x2 > w - 1) x2 = w - 1;
                for (int x = x1; x <= x2; x++) mask[(size_t)y * w + x] = 0;
            }
            dy++;
            err += plus;
            plus += 2;
            int m = (err <= 0) - 1;
            err -= minus & m;
            dx += m;
            minus -= m & 2;
        }
    }
}

/* cornerEigenValsVecs(MINEIGENVAL, blockSize 3, ksize 3) on an ROI. */
void orc_corner_min_eigen_val(const uint8_t* img, int w, int h, int stride, int x0, int y0, int rw,
                              int rh, float* eig) {
    double scale_d = (double)(1 << (3 - 1)) * 3;
    scale_d *= 255.0;
    scale_d = 1.0 / scale_d;
    const float sc = (float)scale_d;  /* kernels are CV_32F */
    const float sc2 = (float)(2.0 * scale_d);
    /* Sobel rows for ROI rows y-1..y+1 (parent pixels, REFLECT_101 at the
       whole-image border); then column pass. */
    size_t npx = (size_t)rw * rh;
    float* cov = (float*)malloc(sizeof(float) * 3 * npx);
    float* rdx = (float*)malloc(sizeof(float) * 3 * rw); /* row-filtered for Dx */
    float* rdy = (float*)malloc(sizeof(float) * 3 * rw); /* row-filtered for Dy */
    for (int y = 0; y < rh; y++) {
        for (int r = 0; r < 3; r++) {
            int py = reflect101(y0 + y + r - 1, h);
            const uint8_t* row = img + (size_t)py * stride;
            for (int x = 0; x < rw; x++) {
                int X = x0 + x;
                float s0 = (float)row[reflect101(X - 1, w)];
                float s1 = (float)row[reflect101(X, w)];
                float s2 = (float)row[reflect101(X + 1, w)];
                /* RowFilter<uchar,float>: s = k0*S0; s += k1*S1; s += k2*S2 */
                float a = -1.f * s0;
                a = a + 0.f * s1;
                a = a + 1.f * s2;
                rdx[r * rw + x] = a;
                float b = sc * s0;
                b = b + sc2 * s1;
                b = b + sc * s2;
                rdy[r * rw + x] = b;
            }
        }
        for (int x = 0; x < rw; x++) {
            /* SymmColumnSmallFilter (symmetric, not 1-2-1): (S0+S2)*f1 + S1*f0 + 0 */
            float dx = (rdx[x] + rdx[2 * rw + x]) * sc + rdx[rw + x] * sc2;
            dx = dx + 0.f;
            /* is_m1_0_1: S2 - S0 + 0 */
            float dy = rdy[2 * rw + x] - rdy[x];
            dy = dy + 0.f;
            float* c = cov + 3 * ((size_t)y * rw + x);
            c[0] = dx * dx;
            c[1] = dx * dy;
            c[2] = dy * dy;
        }
    }
    free(rdx);
    free(rdy);
    /* boxFilter 3x3, normalize=false, sums in double (exact for these values),
       REFLECT_101 inside the ROI (cov is a fresh Mat). */
    for (int y = 0; y < rh; y++) {
        for (int x = 0; x < rw; x++) {
            double s[3] = {0, 0, 0};
            for (int dyy = -1; dyy <= 1; dyy++) {
                int yy = reflect101(y + dyy, rh);
                for (int k = 0; k < 3; k++) {
                    double rs = (double)cov[3 * ((size_t)yy * rw + reflect101(x - 1, rw)) + k];
                    rs = rs + (double)cov[3 * ((size_t)yy * rw + x) + k];
                    rs = rs + (double)cov[3 * ((size_t)yy * rw + reflect101(x + 1, rw)) + k];
                    s[k] = s[k] + rs;
                }
            }
            /* calcMinEigenVal */
            float a = (float)s[0] * 0.5f;
            float b = (float)s[1];
            float c = (float)s[2] * 0.5f;
            eig[(size_t)y * rw + x] = (a + c) - sqrtf((a - c) * (a - c) + b * b);
        }
    }
    free(cov);
}

typedef struct {
    float v;
    int idx;
} cand_t;

static int cand_cmp(const void* pa, const void* pb) {
    const cand_t* a = (const cand_t*)pa;
    const cand_t* b = (const cand_t*)pb;
    /* greaterThanPtr: value descending, ties -> larger address first */
    if (a->v > b->v) return -1;
    if (a->v < b->v) return 1;
    return a->idx > b->idx ? -1 : (a->idx < b->idx ? 1 : 0);
}

int orc_good_features_to_track(const uint8_t* img, int w, int h, int stride, int x0, int y0, int rw,
                               int rh, const uint8_t* mask, int mask_stride, int max_corners,
                               double quality, double min_distance, float* out_xy) {
    size_t npx = (size_t)rw * rh;
    float* eig = (float*)malloc(sizeof(float) * npx);
    float* tmp = (float*)malloc(sizeof(float) * npx);
    orc_corner_min_eigen_val(img, w, h, stride, x0, y0, rw, rh, eig);
    /* minMaxLoc over the mask */
    double maxv = 0;
    int found = 0;
    for (int y = 0; y < rh; y++)
        for (int x = 0; x < rw; x++)
            if (!mask || mask[(size_t)y * mask_stride + x]) {
                double v = eig[(size_t)y * rw + x];
                if (!found || v > maxv) maxv = v;
                found = 1;
            }
    if (!found) maxv = 0;
    float thr = (float)(maxv * quality);
    for (size_t i = 0; i < npx; i++) eig[i] = eig[i] > thr ? eig[i] : 0.f;
    /* dilate 3x3, constant border -FLT_MAX */
    for (int y = 0; y < rh; y++)
        for (int x = 0; x < rw; x++) {
            float m = -FLT_MAX;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    int yy = y + dy, xx = x + dx;
                    if (yy < 0 || yy >= rh || xx < 0 || xx >= rw) continue;
                    float v = eig[(size_t)yy * rw + xx];
                    if (v > m) m = v;
                }
            tmp[(size_t)y * rw + x] = m;
        }
    cand_t* cands = (cand_t*)malloc(sizeof(cand_t) * npx);
    int total = 0;
    for (int y = 1; y < rh - 1; y++)
        for (int x = 1; x < rw - 1; x++) {
            float v = eig[(size_t)y * rw + x];
            if (v != 0 && v == tmp[(size_t)y * rw + x] && (!mask || mask[(size_t)y * mask_stride + x])) {
                cands[total].v = v;
                cands[total].idx = y * rw + x;
                total++;
            }
        }
    int ncorners = 0;
    if (total > 0) {
        qsort(cands, (size_t)total, sizeof(cand_t), cand_cmp);
        if (min_distance >= 1) {
            int cell = cv_round_d(min_distance);
            int gw = (rw + cell - 1) / cell, gh = (rh + cell - 1) / cell;
            double md2 = min_distance * min_distance;
            /* accepted points (at most max_corners or total) */
            int cap = max_corners > 0 ? max_corners : total;
            float* acc = (float*)malloc(sizeof(float) * 2 * (size_t)(cap > 0 ? cap : 1));
            for (int i = 0; i < total; i++) {
                int y = cands[i].idx / rw, x = cands[i].idx - (cands[i].idx / rw) * rw;
                int xc = x / cell, yc = y / cell;
                int good = 1;
                for (int j = 0; j < ncorners && good; j++) {
                    int axc = (int)acc[2 * j] / cell, ayc = (int)acc[2 * j + 1] / cell;
                    if (axc < xc - 1 || axc > xc + 1 || ayc < yc - 1 || ayc > yc + 1) continue;
                    float dx = x - acc[2 * j];
                    float dy = y - acc[2 * j + 1];
                    if (dx * dx + dy * dy < md2) good = 0;
                }
                (void)gw;
                (void)gh;
                if (good) {
                    acc[2 * ncorners] = (float)x;
                    acc[2 * ncorners + 1] = (float)y;
                    out_xy[2 * ncorners] = (float)x;
                    out_xy[2 * ncorners + 1] = (float)y;
                    ncorners++;
                    if (max_corners > 0 && ncorners == max_corners) break;
                }
            }
            free(acc);
        } else {
            for (int i = 0; i < total; i++) {
                out_xy[2 * ncorners] = (float)(cands[i].idx % rw);
                out_xy[2 * ncorners + 1] = (float)(cands[i].idx / rw);
                ncorners++;
                if (max_corners > 0 && ncorners == max_corners) break;
            }
        }
    }
    free(cands);
    free(eig);
    free(tmp);
    return ncorners;
}

/* getRectSubPix(src ROI, Size(ww, wh), center, CV_32F) (imgproc/src/samplers.cpp). */
static void get_rect_subpix(const uint8_t* src, int sstep, int sw, int sh, float* dst, int ww, int wh,
                            float cx0, float cy0) {
    float cx = cx0 - (ww - 1) * 0.5f;
    float cy = cy0 - (wh - 1) * 0.5f;
    int ipx = cv_floor(cx), ipy = cv_floor(cy);
    if (0 <= ipx && ipx + ww < sw && 0 <= ipy && ipy + wh < sh) {
        /* getRectSubPix_8u32f fast path */
        float a = cx - ipx, b = cy - ipy;
        a = a > 0.0001f ? a : 0.0001f;
        float a12 = a * (1.f - b), a22 = a * b, b1 = 1.f - b, b2 = b;
        double s = (1. - a) / a;
        const uint8_t* p = src + (size_t)ipy * sstep + ipx;
        for (int i = 0; i < wh; i++, p += sstep) {
            float prev = (1 - a) * (b1 * (float)p[0] + b2 * (float)p[sstep]);
            for (int j = 0; j < ww; j++) {
                float t = a12 * (float)p[j + 1] + a22 * (float)p[j + 1 + sstep];
                dst[i * ww + j] = prev + t;
                prev = (float)(t * s);
            }
        }
        return;
    }
    /* getRectSubPix_Cn_<uchar, float, float> border branch with adjustRect */
    float a = cx - ipx, b = cy - ipy;
    float a11 = (1.f - a) * (1.f - b), a12 = a * (1.f - b), a21 = (1.f - a) * b, a22 = a * b;
    float b1 = 1.f - b, b2 = b;
    /* adjustRect */
    long off = 0;
    int rx, rwid, ry, rhei;
    if (ipx >= 0) {
        off += ipx;
        rx = 0;
    } else {
        rx = -ipx;
        if (rx > ww) rx = ww;
    }
    if (ipx < sw - ww)
        rwid = ww;
    else {
        rwid = sw - ipx - 1;
        if (rwid < 0) {
            off += rwid;
            rwid = 0;
        }
    }
    if (ipy >= 0) {
        off += (long)ipy * sstep;
        ry = 0;
    } else
        ry = -ipy;
    if (ipy < sh - wh)
        rhei = wh;
    else {
        rhei = sh - ipy - 1;
        if (rhei < 0) {
            off += (long)rhei * sstep;
            rhei = 0;
        }
    }
    const uint8_t* s = src + off - rx;
    for (int i = 0; i < wh; i++) {
        const uint8_t* s2 = s + sstep;
        if (i < ry || i >= rhei) s2 -= sstep;
        float v = (float)s[rx] * b1 + (float)s2[rx] * b2;
        int j;
        for (j = 0; j < rx; j++) dst[i * ww + j] = v;
        v = (float)s[rwid] * b1 + (float)s2[rwid] * b2;
        for (j = rwid; j < ww; j++) dst[i * ww + j] = v;
        for (j = rx; j < rwid; j++) {
            float v0 = (float)s[j] * a11 + (float)s[j + 1] * a12 + (float)s2[j] * a21 +
                       (float)s2[j + 1] * a22;
            dst[i * ww + j] = v0;
        }
        if (i < rhei) s = s2;
    }
}

void orc_corner_subpix(const uint8_t* img, int stride, int x0, int y0, int rw, int rh, float* xy,
                       int n, int win, int max_iters, double eps) {
    const int MAX_ITERS = 100;
    int win_w = win * 2 + 1, win_h = win * 2 + 1;
    if (max_iters < 1) max_iters = 1;
    if (max_iters > MAX_ITERS) max_iters = MAX_ITERS;
    eps = eps > 0 ? eps : 0;
    eps *= eps;
    const uint8_t* src = img + (size_t)y0 * stride + x0;
    float* mask = (float*)malloc(sizeof(float) * win_w * win_h);
    for (int i = 0; i < win_h; i++) {
        float y = (float)(i - win) / win;
        float vy = expf(-y * y);
        for (int j = 0; j < win_w; j++) {
            float x = (float)(j - win) / win;
            mask[i * win_w + j] = (float)(vy * expf(-x * x));
        }
    }
    int bw = win_w + 2;
    float* buf = (float*)malloc(sizeof(float) * bw * (win_h + 2));
    for (int pi = 0; pi < n; pi++) {
        float cTx = xy[2 * pi], cTy = xy[2 * pi + 1];
        float cIx = cTx, cIy = cTy;
        int iter = 0;
        double err = 0;
        do {
            double a = 0, b = 0, c = 0, bb1 = 0, bb2 = 0;
            get_rect_subpix(src, stride, rw, rh, buf, bw, win_h + 2, cIx, cIy);
            const float* sp = buf + bw + 1;
            for (int i = 0, k = 0; i < win_h; i++, sp += bw) {
                double py = i - win;
                for (int j = 0; j < win_w; j++, k++) {
                    double m = mask[k];
                    double tgx = sp[j + 1] - sp[j - 1];
                    double tgy = sp[j + bw] - sp[j - bw];
                    double gxx = tgx * tgx * m;
                    double gxy = tgx * tgy * m;
                    double gyy = tgy * tgy * m;
                    double pxx = j - win;
                    a += gxx;
                    b += gxy;
                    c += gyy;
                    bb1 += gxx * pxx + gxy * py;
                    bb2 += gxy * pxx + gyy * py;
                }
            }
            double det = a * c - b * b;
            if (fabs(det) <= DBL_EPSILON * DBL_EPSILON) break;
            double scale = 1.0 / det;
            float nx = (float)(cIx + c * scale * bb1 - b * scale * bb2);
            float ny = (float)(cIy - b * scale * bb1 + a * scale * bb2);
            err = (nx - cIx) * (nx - cIx) + (ny - cIy) * (ny - cIy);
            cIx = nx;
            cIy = ny;
            if (cIx < 0 || cIx >= rw || cIy < 0 || cIy >= rh) break;
        } while (++iter < max_iters && err > eps);
        if (fabsf(cIx - cTx) > win || fabsf(cIy - cTy) > win) {
            cIx = cTx;
            cIy = cTy;
        }
        xy[2 * pi] = cIx;
        xy[2 * pi + 1] = cIy;
    }
    free(buf);
    free(mask);
}

int orc_features_detection(const uint8_t* img, int w, int h, int stride, const float* count_xy,
                           int n_count, const float* mask_xy, int n_mask, int ismask, int n_existing,
                           const orc_detect_params* p, float* out_xy, int* out_block_counts) {
    orc_block_grid g;
    orc_block_grid_make(w, h, p, &g);
    if (n_existing > (p->max_features - 5)) return -1;
    int* cnts = (int*)calloc((size_t)g.block_cnts, sizeof(int));
    for (int i = 0; i < n_count; i++) {
        int col = (int)(count_xy[2 * i] / (float)g.col);
        int row = (int)(count_xy[2 * i + 1] / (float)g.row);
        int idx = row * g.block_cols + col;
        /* the reference indexes a VLA here (tracking.cc:597-606); indices outside
           [0, block_cnts) are undefined behaviour there and are skipped here. */
        if (idx >= 0 && idx < g.block_cnts) cnts[idx]++;
    }
    uint8_t* mask = (uint8_t*)malloc((size_t)w * h);
    memset(mask, 255, (size_t)w * h);
    if (ismask) orc_mask_circles(mask, w, h, mask_xy, n_mask, g.min_pixel_distance);
    int total = 0;
    float* tmp = (float*)malloc(sizeof(float) * 2 * (size_t)(g.max_block_features > 0 ? g.max_block_features : 1));
    for (int k = 0; k < g.block_cnts; k++) {
        out_block_counts[k] = 0;
        int want = g.max_block_features - cnts[k];
        if (want <= 0) continue;
        int bc = k % g.block_cols, br = k / g.block_cols;
        int cs = bc * g.col, ce = cs + g.col, rs = br * g.row, re = rs + g.row;
        if (k != g.block_cnts - 1) {
            ce -= 5;
            re -= 5;
        }
        int rw = ce - cs, rh = re - rs;
        int nc = orc_good_features_to_track(img, w, h, stride, cs, rs, rw, rh, mask + (size_t)rs * w + cs,
                                            w, want, p->quality, (double)g.min_pixel_distance, tmp);
        if (nc > 0)
            orc_corner_subpix(img, stride, cs, rs, rw, rh, tmp, nc, p->subpix_win, p->subpix_iters,
                              p->subpix_eps);
        for (int i = 0; i < nc; i++) {
            out_xy[2 * (total + i)] = (float)(bc * g.col) + tmp[2 * i];
            out_xy[2 * (total + i) + 1] = (float)(br * g.row) + tmp[2 * i + 1];
        }
        out_block_counts[k] = nc;
        total += nc;
    }
    free(tmp);
    free(mask);
    free(cnts);
    return total;
}
