// detect.hip -- block-grid feature detection for gfx950: replaces
// Tracking::featuresDetection (/root/reference/ic_gvins/ic_gvins/tracking/tracking.cc:576-688):
// circle mask (:609-620), per-block cv::goodFeaturesToTrack (:647-648) and
// cv::cornerSubPix (:651), whose TBB fan-out over blocks (:656) becomes the grid.
//
// Kernels (two launches):
//  mask_eig_kernel  the first workgroups rasterise the circle mask (FILLED
//                 integer-midpoint circles, cv::circle LINE_8, as a per-row
//                 half-width table -> u8 255 / 0), the rest compute
//                 cornerMinEigenVal(blockSize 3, ksize 3) tiles per block ROI:
//                 the Sobel reads the parent image across the ROI edge (padded
//                 level 0 supplies REFLECT_101 at the image border), the 3x3 box
//                 of the covariance reflects inside the ROI; fp32 products and
//                 fp64 box sums in the CPU restatement's order.
//  select_kernel  one workgroup per block: max over the mask, TOZERO threshold,
//                 3x3 dilate, local-max candidates (keys = value, raster index),
//                 then the greedy minDistance suppression as <= maxCorners
//                 rounds of a block-wide argmax -- identical to sorting by
//                 (value desc, address desc) and scanning (goodFeaturesToTrack);
//                 then cornerSubPix, one wavefront per corner: getRectSubPix +
//                 gradient normal equations, the five fp64 sums sequentially in
//                 one lane each, in OpenCV's row-major order (bit-exact corners).
#include <hip/hip_runtime.h>

#include "gvx_internal.h"

namespace gvx {

namespace {

__device__ __forceinline__ int refl(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// ------------------------------------------------------------------ mask
// One workgroup per 64 x 4 tile.  The circle centres are taken 256 at a time,
// and only those whose (2r+1)^2 box meets the tile are kept (LDS append), so a
// pixel tests the few circles near it instead of all of them (the raster is a
// logical OR: the order of the tests does not matter).
__device__ void mask_tile(int bx, int by, int w, int h, const int2* __restrict__ centers, int n,
                          const int* __restrict__ hw, int r, uint8_t* __restrict__ mask,
                          const int* __restrict__ n_dev, const int* __restrict__ skip) {
    __shared__ int2 sc[256];
    __shared__ int s_n;
    if (skip && *skip) return;   // device-resident call: no detection this frame
    if (n_dev) n = *n_dev;
    const int tx0 = bx * 64, ty0 = by * 4;
    const int x = tx0 + (threadIdx.x & 63);
    const int y = ty0 + (threadIdx.x >> 6);
    bool hit = false;
    for (int base = 0; base < n; base += 256) {
        if (threadIdx.x == 0) s_n = 0;
        __syncthreads();
        const int i = base + (int)threadIdx.x;
        if (i < n) {
            const int2 cc = centers[i];
            const int ddx = cc.x < tx0 ? tx0 - cc.x : (cc.x > tx0 + 63 ? cc.x - tx0 - 63 : 0);
            const int ddy = cc.y < ty0 ? ty0 - cc.y : (cc.y > ty0 + 3 ? cc.y - ty0 - 3 : 0);
            if (ddx <= r && ddy <= r) sc[atomicAdd(&s_n, 1)] = cc;
        }
        __syncthreads();
        const int cnt = s_n;
        for (int k = 0; k < cnt && !hit; ++k) {
            const int dy = abs(y - sc[k].y);
            if (dy > r) continue;
            const int hwv = hw[dy];
            hit = hwv >= 0 && abs(x - sc[k].x) <= hwv;
        }
        __syncthreads();
    }
    if (x < w && y < h) mask[(int64_t)y * w + x] = hit ? 0 : 255;
}

// ------------------------------------------------------------------ eig
constexpr int ET_W = 64, ET_H = 16;

__device__ void eig_tile(int bx, int by, int bz, const uint8_t* __restrict__ img0, int pitch,
                         const int4* __restrict__ rois, const int* __restrict__ blk_ids, int64_t eig_stride,
                         float* __restrict__ eig, float sc, float sc2, const int* __restrict__ n_active_dev) {
    __shared__ uint8_t px[ET_H + 4][ET_W + 4];
    __shared__ float cov[3][ET_H + 2][ET_W + 2];
    if (n_active_dev && bz >= *n_active_dev) return;
    const int k = blk_ids ? blk_ids[bz] : bz;  // nullptr: every block, in order
    const int4 roi = rois[k];  // x0, y0, rw, rh
    const int rw = roi.z, rh = roi.w;
    const int tx0 = bx * ET_W, ty0 = by * ET_H;
    if (tx0 >= rw || ty0 >= rh) return;
    // parent pixels for ROI coords [tx0-2, tx0+ET_W+1] x [ty0-2, ty0+ET_H+1]
    // (ROI coords beyond rw+1 / rh+1 are never used; clamp them so the reads stay
    // inside the PAD ring of the padded level)
    for (int i = threadIdx.x; i < (ET_H + 4) * (ET_W + 4); i += 256) {
        const int r = i / (ET_W + 4), c = i - r * (ET_W + 4);
        const int yy = min(ty0 - 2 + r, rh + 1), xx = min(tx0 - 2 + c, rw + 1);
        px[r][c] = img0[(int64_t)(roi.y + yy) * pitch + roi.x + xx];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < (ET_H + 2) * (ET_W + 2); i += 256) {
        const int r = i / (ET_W + 2), c = i - r * (ET_W + 2);
        const int ry = refl(ty0 + r - 1, rh) - ty0 + 2;  // staged coords of the centre
        const int rx = refl(tx0 + c - 1, rw) - tx0 + 2;
        float dx = 0.f, dy = 0.f;
        if (ry >= 1 && ry <= ET_H + 2 && rx >= 1 && rx <= ET_W + 2) {
            float rdx[3], rdy[3];
            for (int q = 0; q < 3; ++q) {
                const float s0 = (float)px[ry - 1 + q][rx - 1];
                const float s1 = (float)px[ry - 1 + q][rx];
                const float s2 = (float)px[ry - 1 + q][rx + 1];
                float a = -1.f * s0;
                a = a + 0.f * s1;
                a = a + 1.f * s2;
                rdx[q] = a;
                float b = sc * s0;
                b = b + sc2 * s1;
                b = b + sc * s2;
                rdy[q] = b;
            }
            dx = (rdx[0] + rdx[2]) * sc + rdx[1] * sc2;
            dx = dx + 0.f;
            dy = rdy[2] - rdy[0];
            dy = dy + 0.f;
        }
        cov[0][r][c] = dx * dx;
        cov[1][r][c] = dx * dy;
        cov[2][r][c] = dy * dy;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < ET_H * ET_W; i += 256) {
        const int r = i / ET_W, c = i - r * ET_W;
        const int x = tx0 + c, y = ty0 + r;
        if (x >= rw || y >= rh) continue;
        double s[3];
        for (int q = 0; q < 3; ++q) {
            double acc = 0;
            for (int d = 0; d < 3; ++d) {
                double rs = (double)cov[q][r + d][c];
                rs = rs + (double)cov[q][r + d][c + 1];
                rs = rs + (double)cov[q][r + d][c + 2];
                acc = acc + rs;
            }
            s[q] = acc;
        }
        const float a = (float)s[0] * 0.5f;
        const float b = (float)s[1];
        const float cc = (float)s[2] * 0.5f;
        eig[k * eig_stride + (int64_t)y * rw + x] = (a + cc) - __fsqrt_rn((a - cc) * (a - cc) + b * b);
    }
}

// The circle mask and the eigenvalue tiles do not depend on each other: one
// launch, the first n_mask workgroups rasterise mask tiles (mx per row), the
// rest compute eig tiles (ex x ey per block).  One kernel node less per frame
// (a node costs ~4.5 us in the sequence replay's graph, however little it does).
__global__ void __launch_bounds__(256) mask_eig_kernel(int n_mask, int mx, int w, int h,
                                                       const int2* __restrict__ centers, int n_circles,
                                                       const int* __restrict__ hw, int radius,
                                                       uint8_t* __restrict__ mask, const int* __restrict__ n_dev,
                                                       const int* __restrict__ skip, int ex, int ey,
                                                       const uint8_t* __restrict__ img0, int pitch,
                                                       const int4* __restrict__ rois,
                                                       const int* __restrict__ blk_ids, int64_t eig_stride,
                                                       float* __restrict__ eig, float sc, float sc2,
                                                       const int* __restrict__ n_active_dev) {
    const int b = blockIdx.x;
    if (b < n_mask) {
        mask_tile(b % mx, b / mx, w, h, centers, n_circles, hw, radius, mask, n_dev, skip);
        return;
    }
    const int e = b - n_mask;
    const int per = ex * ey;
    const int bz = e / per, r = e - bz * per;
    eig_tile(r % ex, r / ex, bz, img0, pitch, rois, blk_ids, eig_stride, eig, sc, sc2, n_active_dev);
}

// ------------------------------------------------------------------ subpix
constexpr int SP_WIN = 5;
constexpr int SP_W = 2 * SP_WIN + 1;  // 11
constexpr int SP_B = SP_W + 2;        // 13

// The ROI pixels around a corner's start, staged in LDS once per corner: every
// iteration's 13x13 patch reads them from there while the centre stays inside
// (ROI pixel (x, y) at win[(y - oy) * SW_W + x - ox]); other reads go to memory.
constexpr int SW_W = 32;
struct SubpixWin {
    const uint8_t* win;
    int ox, oy, nx, ny;  // origin and extent (clipped to the ROI)
};
__device__ __forceinline__ float roi_px(const uint8_t* __restrict__ src, int pitch, const SubpixWin& sw, int x,
                                        int y) {
    const unsigned dx = (unsigned)(x - sw.ox), dy = (unsigned)(y - sw.oy);
    if (dx < (unsigned)sw.nx && dy < (unsigned)sw.ny) return (float)sw.win[dy * SW_W + dx];
    return (float)src[(int64_t)y * pitch + x];
}

// getRectSubPix(ROI, 13x13, centre, CV_32F): value of patch pixel (i, j).
__device__ float rect_subpix_px(const uint8_t* __restrict__ src, int pitch, int sw, int sh, float cx0,
                                float cy0, int i, int j, const SubpixWin& win) {
    const float cx = cx0 - (SP_B - 1) * 0.5f;
    const float cy = cy0 - (SP_B - 1) * 0.5f;
    const int ipx = (int)floorf(cx), ipy = (int)floorf(cy);
    if (0 <= ipx && ipx + SP_B < sw && 0 <= ipy && ipy + SP_B < sh) {
        float a = cx - ipx;
        const float b = cy - ipy;
        a = a > 0.0001f ? a : 0.0001f;
        const float a12 = a * (1.f - b), a22 = a * b, b1 = 1.f - b, b2 = b;
        const double s = (1. - a) / a;
        const int y0 = ipy + i, x0 = ipx;
        const float t = a12 * roi_px(src, pitch, win, x0 + j + 1, y0) + a22 * roi_px(src, pitch, win, x0 + j + 1, y0 + 1);
        float prev;
        if (j == 0) {
            prev = (1 - a) * (b1 * roi_px(src, pitch, win, x0, y0) + b2 * roi_px(src, pitch, win, x0, y0 + 1));
        } else {
            const float tp = a12 * roi_px(src, pitch, win, x0 + j, y0) + a22 * roi_px(src, pitch, win, x0 + j, y0 + 1);
            prev = (float)(tp * s);
        }
        return prev + t;
    }
    const float a = cx - ipx, b = cy - ipy;
    const float a11 = (1.f - a) * (1.f - b), a12 = a * (1.f - b), a21 = (1.f - a) * b, a22 = a * b;
    const float b1 = 1.f - b, b2 = b;
    // adjustRect
    int64_t off = 0;
    int rx, rwid, ry, rhei;
    if (ipx >= 0) {
        off += ipx;
        rx = 0;
    } else {
        rx = -ipx;
        if (rx > SP_B) rx = SP_B;
    }
    if (ipx < sw - SP_B)
        rwid = SP_B;
    else {
        rwid = sw - ipx - 1;
        if (rwid < 0) {
            off += rwid;
            rwid = 0;
        }
    }
    if (ipy >= 0) {
        off += (int64_t)ipy * pitch;
        ry = 0;
    } else
        ry = -ipy;
    if (ipy < sh - SP_B)
        rhei = SP_B;
    else {
        rhei = sh - ipy - 1;
        if (rhei < 0) {
            off += (int64_t)rhei * pitch;
            rhei = 0;
        }
    }
    const uint8_t* s = src + off - rx;
    for (int q = 0; q < i; ++q) {
        const uint8_t* s2 = s + pitch;
        if (q < ry || q >= rhei) s2 -= pitch;
        if (q < rhei) s = s2;
    }
    const uint8_t* s2 = s + pitch;
    if (i < ry || i >= rhei) s2 -= pitch;
    if (j < rx) return (float)s[rx] * b1 + (float)s2[rx] * b2;
    if (j >= rwid) return (float)s[rwid] * b1 + (float)s2[rwid] * b2;
    return (float)s[j] * a11 + (float)s[j + 1] * a12 + (float)s2[j] * a21 + (float)s2[j + 1] * a22;
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// cornerSubPix of one corner by one wavefront (per-wave LDS: the 13x13 patch,
// the five term arrays, their sums and the staged pixel window): getRectSubPix +
// gradient normal equations; the five fp64 sums run sequentially in one lane
// each, in OpenCV's row-major order, so corners are bit-exact.
struct SubpixLds {
    float patch[SP_B * SP_B];
    double terms[5][SP_W * SP_W];
    double sums[5];
    uint8_t win[SW_W * SW_W];
};
__device__ float2 subpix_corner(const uint8_t* __restrict__ src, int pitch, int4 roi, int2 c0,
                                const float* __restrict__ gmask, int max_iters, double eps2, int lane,
                                SubpixLds& L) {
    float* patch = L.patch;
    const float cTx = (float)c0.x, cTy = (float)c0.y;
    // stage the ROI pixels around the start (the patch of a centre within
    // about +-9 px of it): lane l copies 16 bytes of row l/2
    SubpixWin win;
    win.win = L.win;
    win.ox = max(0, min(c0.x - SW_W / 2 + 1, roi.z - SW_W));
    win.oy = max(0, min(c0.y - SW_W / 2 + 1, roi.w - SW_W));
    win.nx = min(SW_W, roi.z - win.ox);
    win.ny = min(SW_W, roi.w - win.oy);
    {
        const int r = lane >> 1, c = (lane & 1) * 16;
        if (r < win.ny) {
            const uint8_t* g = src + (int64_t)(win.oy + r) * pitch + win.ox + c;
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if (c + q < win.nx) L.win[r * SW_W + c + q] = g[q];
        }
    }
    wave_lds_sync();
    float cIx = cTx, cIy = cTy;
    int iter = 0;
    double err = 0;
    do {
        // getRectSubPix's per-call terms (one centre for the whole patch) once, then
        // the interior formula of rect_subpix_px per pixel (the same arithmetic)
        const float pcx = cIx - (SP_B - 1) * 0.5f, pcy = cIy - (SP_B - 1) * 0.5f;
        const int ipx = (int)floorf(pcx), ipy = (int)floorf(pcy);
        if (0 <= ipx && ipx + SP_B < roi.z && 0 <= ipy && ipy + SP_B < roi.w) {
            float pa = pcx - ipx;
            const float pb = pcy - ipy;
            pa = pa > 0.0001f ? pa : 0.0001f;
            const float a12 = pa * (1.f - pb), a22 = pa * pb, b1 = 1.f - pb, b2 = pb;
            const double ps = (1. - pa) / pa;
            auto patch_px = [&](auto px) {
                for (int e = lane; e < SP_B * SP_B; e += 64) {
                    const int i = e / SP_B, j = e - i * SP_B;
                    const int y0 = ipy + i, x0 = ipx;
                    const float t = a12 * px(x0 + j + 1, y0) + a22 * px(x0 + j + 1, y0 + 1);
                    float prev;
                    if (j == 0) {
                        prev = (1 - pa) * (b1 * px(x0, y0) + b2 * px(x0, y0 + 1));
                    } else {
                        const float tp = a12 * px(x0 + j, y0) + a22 * px(x0 + j, y0 + 1);
                        prev = (float)(tp * ps);
                    }
                    patch[e] = prev + t;
                }
            };
            // the patch's (SP_B + 1)^2 pixels inside the staged window: LDS reads
            // only (ds_read_u8, no flat loads); otherwise each pixel picks its source
            if (ipx >= win.ox && ipx + SP_B + 1 <= win.ox + win.nx && ipy >= win.oy &&
                ipy + SP_B + 1 <= win.oy + win.ny) {
                const uint8_t* lw = L.win + (ipy - win.oy) * SW_W + (ipx - win.ox);
                patch_px([&](int x, int y) -> float { return (float)lw[(y - ipy) * SW_W + (x - ipx)]; });
            } else {
                patch_px([&](int x, int y) -> float { return roi_px(src, pitch, win, x, y); });
            }
        } else {
            for (int e = lane; e < SP_B * SP_B; e += 64)
                patch[e] = rect_subpix_px(src, pitch, roi.z, roi.w, cIx, cIy, e / SP_B, e % SP_B, win);
        }
        wave_lds_sync();
        for (int e = lane; e < SP_W * SP_W; e += 64) {
            const int i = e / SP_W, j = e - i * SP_W;
            const float* sp = patch + (i + 1) * SP_B + 1;
            const double m = gmask[e];
            const double tgx = sp[j + 1] - sp[j - 1];
            const double tgy = sp[j + SP_B] - sp[j - SP_B];
            const double gxx = tgx * tgx * m;
            const double gxy = tgx * tgy * m;
            const double gyy = tgy * tgy * m;
            const double pxx = j - SP_WIN, py = i - SP_WIN;
            L.terms[0][e] = gxx;
            L.terms[1][e] = gxy;
            L.terms[2][e] = gyy;
            L.terms[3][e] = gxx * pxx + gxy * py;
            L.terms[4][e] = gxy * pxx + gyy * py;
        }
        wave_lds_sync();
        if (lane < 5) {
            // the sequential sum (OpenCV's order), its LDS reads a batch ahead of the adds
            const double* T = L.terms[lane];
            double acc = 0, cur[SP_W], nxt[SP_W];
#pragma unroll
            for (int q = 0; q < SP_W; ++q) cur[q] = T[q];
#pragma unroll
            for (int bt = 0; bt < SP_W; ++bt) {
                if (bt + 1 < SP_W) {
#pragma unroll
                    for (int q = 0; q < SP_W; ++q) nxt[q] = T[(bt + 1) * SP_W + q];
                }
#pragma unroll
                for (int q = 0; q < SP_W; ++q) acc += cur[q];
#pragma unroll
                for (int q = 0; q < SP_W; ++q) cur[q] = nxt[q];
            }
            L.sums[lane] = acc;
        }
        wave_lds_sync();
        const double a = L.sums[0], b = L.sums[1], c = L.sums[2], bb1 = L.sums[3], bb2 = L.sums[4];
        const double det = a * c - b * b;
        if (fabs(det) <= __DBL_EPSILON__ * __DBL_EPSILON__) break;
        const double scale = 1.0 / det;
        const float nx = (float)(cIx + c * scale * bb1 - b * scale * bb2);
        const float ny = (float)(cIy - b * scale * bb1 + a * scale * bb2);
        err = (nx - cIx) * (nx - cIx) + (ny - cIy) * (ny - cIy);
        cIx = nx;
        cIy = ny;
        if (cIx < 0 || cIx >= roi.z || cIy < 0 || cIy >= roi.w) break;
    } while (++iter < max_iters && err > eps2);
    if (fabsf(cIx - cTx) > SP_WIN || fabsf(cIy - cTy) > SP_WIN) {
        cIx = cTx;
        cIy = cTy;
    }
    return make_float2(cIx, cIy);
}

// ------------------------------------------------------------------ select
__device__ __forceinline__ uint32_t fkey(float v) {
    const uint32_t b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

// the inverse of fkey
__device__ __forceinline__ float funkey(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
    for (int o = 32; o >= 1; o >>= 1) {
        const unsigned long long t = __shfl_xor(v, o, 64);
        v = t > v ? t : v;
    }
    return v;
}

constexpr int SEL_T = 1024;

// goodFeaturesToTrack + cornerSubPix of block k (ROI roi, eigenvalues E in ROI
// raster order, maxCorners maxc) by one workgroup; allowed(x, y) is the mask at
// ROI pixel (x, y).  The caller's LDS: sub (one SubpixLds per wave).
struct SelectShared {
    float s_max[SEL_T / 64];
    int s_found[SEL_T / 64];
    unsigned long long s_key[SEL_T / 64];
    int s_ncand;
    float s_acc[64][2];
    int s_nacc;
};

// minMaxLoc over the mask, TOZERO threshold, 3x3 dilate and the local-max
// candidates of block k by one workgroup scanning its whole ROI
template <class Allowed>
__device__ __forceinline__ void scan_block(int4 roi, const float* __restrict__ E, Allowed allowed, double quality,
                                           unsigned long long* __restrict__ CK, SelectShared& S) {
    const int rw = roi.z, rh = roi.w;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int npx = rw * rh;
    // minMaxLoc(eig, 0, &maxVal, 0, 0, mask)
    float mx = -__FLT_MAX__;
    int found = 0;
    for (int i = t; i < npx; i += SEL_T) {
        const int y = i / rw, x = i - y * rw;
        if (allowed(x, y)) {
            mx = fmaxf(mx, E[i]);
            found = 1;
        }
    }
    for (int o = 32; o >= 1; o >>= 1) {
        mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        found |= __shfl_xor(found, o, 64);
    }
    if (lane == 0) {
        S.s_max[wv] = mx;
        S.s_found[wv] = found;
    }
    if (t == 0) {
        S.s_ncand = 0;
        S.s_nacc = 0;
    }
    __syncthreads();
    float mxa = -__FLT_MAX__;
    int fa = 0;
    for (int q = 0; q < SEL_T / 64; ++q) {
        mxa = fmaxf(mxa, S.s_max[q]);
        fa |= S.s_found[q];
    }
    const double maxv = fa ? (double)mxa : 0.0;
    const float thr = (float)(maxv * quality);
    // candidates: thresholded local maxima of the 3x3 dilation, inside the
    // 1-pixel ROI ring, on the mask
    for (int i = t; i < npx; i += SEL_T) {
        const int y = i / rw, x = i - y * rw;
        if (y < 1 || y > rh - 2 || x < 1 || x > rw - 2) continue;
        float v = E[i];
        v = v > thr ? v : 0.f;
        if (v == 0.f || !allowed(x, y)) continue;
        float d = -__FLT_MAX__;
        for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
                float u = E[(y + dy) * rw + x + dx];
                u = u > thr ? u : 0.f;
                d = fmaxf(d, u);
            }
        if (v == d) {
            const int slot = atomicAdd(&S.s_ncand, 1);
            CK[slot] = ((unsigned long long)fkey(v) << 32) | (unsigned)i;
        }
    }
    __syncthreads();
}

// goodFeaturesToTrack's greedy minDistance suppression over the S.s_ncand
// candidates in CK, then cornerSubPix of the accepted corners
__device__ __forceinline__ void select_corners(int k, int4 roi, int maxc, float min_dist,
                                               const unsigned long long* __restrict__ CK, int2* __restrict__ corners,
                                               int max_per_block, int* __restrict__ ncorner,
                                               const uint8_t* __restrict__ img0, int pitch,
                                               const float* __restrict__ gmask, int max_iters, double eps2,
                                               float2* __restrict__ out, SelectShared& S, SubpixLds* s_sub) {
    const int rw = roi.z;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) S.s_nacc = 0;
    __syncthreads();
    const int nc = S.s_ncand;
    const float md2 = min_dist * min_dist;
    for (int round = 0; round < maxc; ++round) {
        unsigned long long best = 0;
        const int na = S.s_nacc;
        for (int i = t; i < nc; i += SEL_T) {
            const unsigned long long key = CK[i];
            if (key <= best) continue;
            const int idx = (int)(key & 0xffffffffu);
            const int y = idx / rw, x = idx - y * rw;
            bool good = true;
            for (int j = 0; j < na && good; ++j) {
                const float dx = (float)x - S.s_acc[j][0];
                const float dy = (float)y - S.s_acc[j][1];
                if (dx * dx + dy * dy < md2) good = false;
            }
            if (good) best = key;
        }
        best = wave_max_u64(best);
        if (lane == 0) S.s_key[wv] = best;
        __syncthreads();
        if (t == 0) {
            unsigned long long b = 0;
            for (int q = 0; q < SEL_T / 64; ++q) b = S.s_key[q] > b ? S.s_key[q] : b;
            if (b != 0) {
                const int idx = (int)(b & 0xffffffffu);
                const int y = idx / rw, x = idx - y * rw;
                S.s_acc[S.s_nacc][0] = (float)x;
                S.s_acc[S.s_nacc][1] = (float)y;
                corners[k * max_per_block + S.s_nacc] = make_int2(x, y);
                S.s_nacc = S.s_nacc + 1;
            } else {
                S.s_key[0] = 0;  // signal: no more candidates
            }
        }
        __syncthreads();
        if (S.s_nacc == round) break;  // nothing accepted this round
    }
    if (t == 0) ncorner[k] = S.s_nacc;
    // cornerSubPix of the block's corners (the old separate launch), one wave
    // per corner: the block's ROI and corner list are already here
    __syncthreads();
    const int nacc = S.s_nacc;
    const uint8_t* src = img0 + (int64_t)roi.y * pitch + roi.x;
    for (int ci = wv; ci < nacc; ci += SEL_T / 64) {
        const int2 c0 = make_int2((int)S.s_acc[ci][0], (int)S.s_acc[ci][1]);
        const float2 r = subpix_corner(src, pitch, roi, c0, gmask, max_iters, eps2, lane, s_sub[wv]);
        if (lane == 0) out[k * max_per_block + ci] = r;
    }
}

__global__ void __launch_bounds__(SEL_T) select_kernel(const float* __restrict__ eig, int64_t eig_stride,
                                                       const uint8_t* __restrict__ mask, int w,
                                                       const int4* __restrict__ rois,
                                                       const int* __restrict__ blk_ids,
                                                       const int* __restrict__ want, double quality,
                                                       float min_dist, unsigned long long* __restrict__ cand,
                                                       int2* __restrict__ corners, int max_per_block,
                                                       int* __restrict__ ncorner, const int* __restrict__ n_active_dev,
                                                       const uint8_t* __restrict__ img0, int pitch,
                                                       const float* __restrict__ gmask, int max_iters, double eps2,
                                                       float2* __restrict__ out) {
    __shared__ SubpixLds s_sub[SEL_T / 64];
    __shared__ SelectShared S;
    if (n_active_dev && (int)blockIdx.x >= *n_active_dev) return;
    const int k = blk_ids[blockIdx.x];
    const int4 roi = rois[k];
    const uint8_t* M = mask + (int64_t)roi.y * w + roi.x;
    auto allowed = [&](int x, int y) -> bool { return M[(int64_t)y * w + x] != 0; };
    scan_block(roi, eig + k * eig_stride, allowed, quality, cand + k * eig_stride, S);
    select_corners(k, roi, want[k], min_dist, cand + k * eig_stride, corners, max_per_block, ncorner, img0, pitch,
                   gmask, max_iters, eps2, out, S, s_sub);
}

// featuresDetection's early exit and block k's maxCorners from the tracked points
// (the kept FB flags and positions of the frame's LK, or the point list of a
// first frame): a block-wide count by every workgroup that needs it, so no
// preparation launch precedes the tracking path's detection.  Returns maxCorners
// (<= 0: nothing to detect in block k).  The circle centres near roi (ROI
// coordinates) go to circ / *nc when circ != nullptr.
__device__ int block_want(const TrackSelect& a, int k, int4 roi, int* s_nk, int* s_cnt, int2* circ, int* s_nc) {
    const int t = threadIdx.x, r = a.radius;
    if (t == 0) {
        *s_nk = 0;
        *s_cnt = 0;
        if (circ) *s_nc = 0;
    }
    __syncthreads();
    const int n_in = min(*a.n, a.cap);
    for (int i = t; i < n_in; i += blockDim.x) {
        const bool kept = a.flags ? (a.flags[i] & 4) != 0 : true;
        if (!kept) continue;
        const float2 p = a.flags ? reinterpret_cast<const float2*>(a.next_xy)[i]
                                 : reinterpret_cast<const float2*>(a.pts)[i];
        atomicAdd(s_nk, 1);
        const int cc = (int)(p.x / (float)a.col), rr = (int)(p.y / (float)a.row);
        if (rr * a.bcols + cc == k) atomicAdd(s_cnt, 1);
        if (circ) {
            const int cx = (int)rintf(p.x), cy = (int)rintf(p.y);
            if (cx >= roi.x - r && cx <= roi.x + roi.z - 1 + r && cy >= roi.y - r && cy <= roi.y + roi.w - 1 + r)
                circ[atomicAdd(s_nc, 1)] = make_int2(cx - roi.x, cy - roi.y);
        }
    }
    __syncthreads();
    const int nk = *s_nk;
    const bool skip = !(nk < a.max_features) || nk > a.max_features - 5 || a.maxpb <= 0;
    return skip ? 0 : a.maxpb - *s_cnt;
}

// The eigenvalue tiles of the tracking path, for the blocks that detect this
// frame only (each workgroup counts the tracked points itself, as the selection
// does): one launch, no preparation launch before it.  Each tile is computed
// with a one-pixel halo of eigenvalues (the same arithmetic at every pixel, so
// the halo equals the neighbouring tiles' values), which lets the tile do the
// selection's two whole-ROI scans for its own pixels, spread over the grid
// instead of one workgroup per block:
//  * minMaxLoc over the mask: the tile's maximum over its allowed pixels (the
//    circle mask of the tracked points, cv::circle FILLED as in the selection's
//    bitmap) -> atomicMax of fkey(v) into sel[2k] (0: no allowed pixel yet);
//  * the candidates: for a threshold thr > 0, "v > thr and v equals the 3x3
//    dilation of the TOZERO-thresholded map" holds exactly when v > thr and v
//    is >= its 8 raw neighbours (a neighbour above v is above thr; one at or
//    below thr becomes 0 < v), so the tile appends its allowed raw local maxima
//    with v > 0 (ROI ring excluded) to the block's list, count sel[2k + 1]; the
//    selection keeps those above thr.  A block whose maximum is <= 0 (thr <= 0,
//    where that equivalence fails) falls back to the full scan.
// sel is zero at entry (the selection clears it after reading it).
constexpr int EH_W = ET_W + 2, EH_H = ET_H + 2;  // eigenvalues with the halo
__global__ void __launch_bounds__(256) eig_track_kernel(TrackSelect a, int ex, int ey, float sc, float sc2) {
    __shared__ int s_nk, s_cnt, s_nc, s_nt;
    __shared__ int2 s_circ[TS_MAX_POINTS], s_tc[TS_MAX_POINTS];
    __shared__ uint8_t px[EH_H + 4][EH_W + 4];
    __shared__ float cov[3][EH_H + 2][EH_W + 2];
    __shared__ float ev[EH_H][EH_W];
    __shared__ unsigned s_max;
    const int per = ex * ey;
    const int k = blockIdx.x / per, r = blockIdx.x - k * per;
    const int4 roi = a.rois[k];
    // the circles near the ROI (ROI coordinates), only when the candidates are wanted
    if (block_want(a, k, roi, &s_nk, &s_cnt, a.sel ? s_circ : nullptr, &s_nc) <= 0) return;  // uniform
    if (!a.sel) {
        eig_tile(r % ex, r / ex, k, a.img0, a.pitch, a.rois, nullptr, a.eig_stride, const_cast<float*>(a.eig), sc,
                 sc2, nullptr);
        return;
    }
    const int rw = roi.z, rh = roi.w;
    const int tx0 = (r % ex) * ET_W, ty0 = (r / ex) * ET_H;
    if (tx0 >= rw || ty0 >= rh) return;
    const int t = threadIdx.x;
    // the circles that reach the tile (a pixel then tests only those)
    if (t == 0) {
        s_nt = 0;
        s_max = 0u;
    }
    __syncthreads();
    const int rad = a.radius;
    for (int i = t; i < s_nc; i += 256) {
        const int2 c = s_circ[i];
        if (c.x + rad >= tx0 && c.x - rad <= tx0 + ET_W - 1 && c.y + rad >= ty0 && c.y - rad <= ty0 + ET_H - 1)
            s_tc[atomicAdd(&s_nt, 1)] = c;
    }
    // parent pixels for ROI coords [tx0-3, tx0+ET_W+2] x [ty0-3, ty0+ET_H+2]
    // (clamped past rw+1 / rh+1 as in eig_tile; the reads stay in the padded ring)
    for (int i = t; i < (EH_H + 4) * (EH_W + 4); i += 256) {
        const int rr = i / (EH_W + 4), c = i - rr * (EH_W + 4);
        const int yy = max(min(ty0 - 3 + rr, rh + 1), -2), xx = max(min(tx0 - 3 + c, rw + 1), -2);
        px[rr][c] = a.img0[(int64_t)(roi.y + yy) * a.pitch + roi.x + xx];
    }
    __syncthreads();
    // covariance at ROI coords [tx0-2, tx0+ET_W+1] x [ty0-2, ty0+ET_H+1]: the Sobel
    // at the REFLECT_101 position inside the ROI (staged row / col = roi - (t0 - 3))
    for (int i = t; i < (EH_H + 2) * (EH_W + 2); i += 256) {
        const int rr = i / (EH_W + 2), c = i - rr * (EH_W + 2);
        const int ry = refl(ty0 + rr - 2, rh) - ty0 + 3;
        const int rx = refl(tx0 + c - 2, rw) - tx0 + 3;
        float dx = 0.f, dy = 0.f;
        if (ry >= 1 && ry <= EH_H + 2 && rx >= 1 && rx <= EH_W + 2) {
            float rdx[3], rdy[3];
            for (int q = 0; q < 3; ++q) {
                const float s0 = (float)px[ry - 1 + q][rx - 1];
                const float s1 = (float)px[ry - 1 + q][rx];
                const float s2 = (float)px[ry - 1 + q][rx + 1];
                float aa = -1.f * s0;
                aa = aa + 0.f * s1;
                aa = aa + 1.f * s2;
                rdx[q] = aa;
                float b = sc * s0;
                b = b + sc2 * s1;
                b = b + sc * s2;
                rdy[q] = b;
            }
            dx = (rdx[0] + rdx[2]) * sc + rdx[1] * sc2;
            dx = dx + 0.f;
            dy = rdy[2] - rdy[0];
            dy = dy + 0.f;
        }
        cov[0][rr][c] = dx * dx;
        cov[1][rr][c] = dx * dy;
        cov[2][rr][c] = dy * dy;
    }
    __syncthreads();
    // eigenvalues at ROI coords [tx0-1, tx0+ET_W] x [ty0-1, ty0+ET_H]; the tile's own
    // pixels also go to the block's map (the fallback scan reads it)
    float* E = const_cast<float*>(a.eig) + k * a.eig_stride;
    for (int i = t; i < EH_H * EH_W; i += 256) {
        const int rr = i / EH_W, c = i - rr * EH_W;
        const int x = tx0 + c - 1, y = ty0 + rr - 1;
        if (x < 0 || y < 0 || x >= rw || y >= rh) continue;
        double sacc[3];
        for (int q = 0; q < 3; ++q) {
            double acc = 0;
            for (int d = 0; d < 3; ++d) {
                double rs = (double)cov[q][rr + d][c];
                rs = rs + (double)cov[q][rr + d][c + 1];
                rs = rs + (double)cov[q][rr + d][c + 2];
                acc = acc + rs;
            }
            sacc[q] = acc;
        }
        const float aa = (float)sacc[0] * 0.5f;
        const float b = (float)sacc[1];
        const float cc = (float)sacc[2] * 0.5f;
        const float v = (aa + cc) - __fsqrt_rn((aa - cc) * (aa - cc) + b * b);
        ev[rr][c] = v;
        if (rr >= 1 && rr <= ET_H && c >= 1 && c <= ET_W) E[(int64_t)y * rw + x] = v;
    }
    __syncthreads();
    const int nt = s_nt;
    unsigned kmax = 0u;
    unsigned* sel = a.sel + 2 * k;
    unsigned long long* CK = a.cand + k * a.eig_stride;
    for (int i = t; i < ET_H * ET_W; i += 256) {
        const int rr = i / ET_W + 1, c = i % ET_W + 1;
        const int x = tx0 + c - 1, y = ty0 + rr - 1;
        if (x >= rw || y >= rh) continue;
        bool allowed = true;
        for (int q = 0; q < nt && allowed; ++q) {
            const int2 cc = s_tc[q];
            const int dyy = abs(y - cc.y);
            if (dyy > rad) continue;
            const int hwv = a.hw[dyy];
            allowed = !(hwv >= 0 && abs(x - cc.x) <= hwv);
        }
        if (!allowed) continue;
        const float v = ev[rr][c];
        kmax = max(kmax, fkey(v));
        if (v > 0.f && y >= 1 && y <= rh - 2 && x >= 1 && x <= rw - 2) {
            bool lm = true;
#pragma unroll
            for (int q = 0; q < 9; ++q) lm = lm && !(ev[rr + q / 3 - 1][c + q % 3 - 1] > v);
            if (lm) CK[atomicAdd(&sel[1], 1u)] = ((unsigned long long)fkey(v) << 32) | (unsigned)(y * rw + x);
        }
    }
    if (kmax) atomicMax(&s_max, kmax);
    __syncthreads();
    if (t == 0 && s_max) atomicMax(&sel[0], s_max);
}

// The tracking path's detection (gvx_track_frame_dev), one workgroup per block
// and no preparation launch: each workgroup counts the tracked points itself
// (the kept FB flags and tracked positions of the frame's LK, or the point list
// of a first frame), takes featuresDetection's early exit and the block's
// maxCorners from them, and rasterises the circle mask of the points near its
// ROI into an LDS bitmap (cv::circle FILLED, radius minDistance, at the
// cvRound centres: the same per-row half-widths as mask_tile) instead of
// reading a full-frame mask.  The eigenvalue map is the frame's, computed
// beforehand (gvx_frame_eig_dev on the preprocessing branch, or a launch of
// eig tiles right before this one).  Inactive blocks write ncorner = 0.
__global__ void __launch_bounds__(SEL_T) select_track_kernel(TrackSelect a) {
    __shared__ SubpixLds s_sub[SEL_T / 64];
    __shared__ SelectShared S;
    __shared__ int s_nk, s_cnt, s_nc;
    __shared__ int2 s_circ[TS_MAX_POINTS];
    extern __shared__ uint32_t bm[];  // ROI bitmap, 1 = allowed, wpr words per row
    const int k = blockIdx.x, t = threadIdx.x;
    const int4 roi = a.rois[k];
    const int rw = roi.z, rh = roi.w, r = a.radius;
    const int want = block_want(a, k, roi, &s_nk, &s_cnt, s_circ, &s_nc);
    // the tile scan's results (eig_track_kernel): read, then cleared for the next frame
    unsigned smax = 0u, sncand = 0u;
    if (a.sel) {
        smax = a.sel[2 * k];
        sncand = a.sel[2 * k + 1];
        __syncthreads();  // every thread has read them
        if (t == 0) {
            a.sel[2 * k] = 0u;
            a.sel[2 * k + 1] = 0u;
        }
    }
    if (want <= 0) {  // uniform over the workgroup
        if (t == 0) a.ncorner[k] = 0;
        return;
    }
    unsigned long long* CK = a.cand + k * a.eig_stride;
    // the tile scan applies when the block's maximum over the mask is > 0
    const float tmax = smax ? funkey(smax) : 0.f;
    if (a.sel && tmax > 0.f) {
        const float thr = (float)((double)tmax * a.quality);
        if (t == 0) S.s_ncand = 0;
        __syncthreads();
        // keep the local maxima above thr, compacted in place a chunk at a time
        // (every key of a chunk is read before any slot of it is written)
        for (int c0 = 0; c0 < (int)sncand; c0 += SEL_T) {
            const int i = c0 + t;
            const unsigned long long key = i < (int)sncand ? CK[i] : 0ull;
            __syncthreads();
            if (i < (int)sncand && funkey((unsigned)(key >> 32)) > thr) CK[atomicAdd(&S.s_ncand, 1)] = key;
            __syncthreads();
        }
        select_corners(k, roi, want, a.min_dist, CK, a.corners, a.max_per_block, a.ncorner, a.img0, a.pitch, a.gmask,
                       a.max_iters, a.eps2, a.out, S, s_sub);
        return;
    }
    const int wpr = (rw + 31) >> 5;
    for (int i = t; i < wpr * rh; i += SEL_T) bm[i] = ~0u;
    __syncthreads();
    const int span = 2 * r + 1, nrow = s_nc * span;
    for (int it = t; it < nrow; it += SEL_T) {
        const int ci = it / span, dy = it - ci * span - r;
        const int2 c = s_circ[ci];
        const int y = c.y + dy;
        const int hwv = a.hw[dy < 0 ? -dy : dy];
        if (y < 0 || y >= rh || hwv < 0) continue;
        const int x0 = max(c.x - hwv, 0), x1 = min(c.x + hwv, rw - 1);
        for (int x = x0; x <= x1;) {  // clear bits x0..x1 of row y, a word at a time
            const int wi = x >> 5, b0 = x & 31, b1 = min(31, b0 + (x1 - x));
            const uint32_t m = (b1 == 31 ? ~0u : ((1u << (b1 + 1)) - 1u)) & ~((1u << b0) - 1u);
            atomicAnd(&bm[y * wpr + wi], ~m);
            x += b1 - b0 + 1;
        }
    }
    __syncthreads();
    auto allowed = [&](int x, int y) -> bool { return (bm[y * wpr + (x >> 5)] >> (x & 31)) & 1u; };
    scan_block(roi, a.eig + k * a.eig_stride, allowed, a.quality, CK, S);
    select_corners(k, roi, want, a.min_dist, CK, a.corners, a.max_per_block, a.ncorner, a.img0, a.pitch, a.gmask,
                   a.max_iters, a.eps2, a.out, S, s_sub);
}

}  // namespace

hipError_t launch_eig_all(gvx_ctx* c, int n_blocks, int max_rw, int max_rh, const uint8_t* img0, int pitch,
                          const int4* rois, int64_t eig_stride, float* eig, float sc, float sc2) {
    if (n_blocks <= 0) return hipSuccess;
    const int ex = (max_rw + ET_W - 1) / ET_W, ey = (max_rh + ET_H - 1) / ET_H;
    hipLaunchKernelGGL(mask_eig_kernel, dim3(ex * ey * n_blocks), dim3(256), 0, c->stream, 0, 1, 0, 0, nullptr, 0,
                       nullptr, 0, nullptr, nullptr, nullptr, ex, ey, img0, pitch, rois, nullptr, eig_stride, eig, sc,
                       sc2, nullptr);
    return hipGetLastError();
}

hipError_t launch_eig_track(gvx_ctx* c, int n_blocks, int max_rw, int max_rh, const TrackSelect& a, float sc,
                            float sc2) {
    if (n_blocks <= 0) return hipSuccess;
    if (a.cap > TS_MAX_POINTS) return hipErrorInvalidValue;
    const int ex = (max_rw + ET_W - 1) / ET_W, ey = (max_rh + ET_H - 1) / ET_H;
    hipLaunchKernelGGL(eig_track_kernel, dim3(ex * ey * n_blocks), dim3(256), 0, c->stream, a, ex, ey, sc, sc2);
    return hipGetLastError();
}

size_t select_track_lds(int max_rw, int max_rh) { return (size_t)((max_rw + 31) / 32) * max_rh * 4; }

hipError_t launch_select_track(gvx_ctx* c, int n_blocks, int max_rw, int max_rh, const TrackSelect& a) {
    if (n_blocks <= 0) return hipSuccess;
    if (a.cap > TS_MAX_POINTS || select_track_lds(max_rw, max_rh) > TS_MAX_BITMAP) return hipErrorInvalidValue;
    hipLaunchKernelGGL(select_track_kernel, dim3(n_blocks), dim3(SEL_T), select_track_lds(max_rw, max_rh), c->stream,
                       a);
    return hipGetLastError();
}

hipError_t launch_detect(gvx_ctx* c, const DetectLaunch& d) {
    // device-resident counts (n_active_dev): every launch is sized for all blocks
    // / the capacity and the kernels read the counts, so the topology is fixed
    const bool dev_counts = d.n_active_dev != nullptr;
    const bool with_mask = d.n_circles > 0 || d.fill_mask || dev_counts;
    const int n_act = dev_counts ? d.n_blocks : d.n_active;
    const int mx = (d.w + 63) / 64, my = (d.h + 3) / 4;
    const int n_mask = with_mask ? mx * my : 0;
    const int ex = (d.max_rw + ET_W - 1) / ET_W, ey = (d.max_rh + ET_H - 1) / ET_H;
    const int n_eig = n_act > 0 ? ex * ey * n_act : 0;
    if (n_mask + n_eig > 0)
        hipLaunchKernelGGL(mask_eig_kernel, dim3(n_mask + n_eig), dim3(256), 0, c->stream, n_mask, mx, d.w, d.h,
                           d.centers, d.n_circles, d.hw, d.radius, d.mask, d.n_circles_dev, d.skip_dev, ex, ey,
                           d.img0, d.pitch, d.rois, d.blk_ids, d.eig_stride, d.eig, d.sc, d.sc2, d.n_active_dev);
    if (n_act <= 0) return hipGetLastError();
    hipLaunchKernelGGL(select_kernel, dim3(n_act), dim3(SEL_T), 0, c->stream, d.eig, d.eig_stride, d.mask,
                       d.w, d.rois, d.blk_ids, d.want, d.quality, d.min_dist, d.cand, d.corners,
                       d.max_per_block, d.ncorner, d.n_active_dev, d.img0, d.pitch, d.gmask, d.max_iters, d.eps2,
                       d.out);
    return hipGetLastError();
}

}  // namespace gvx
