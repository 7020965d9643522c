// clahe.hip -- Tracking::preprocessing's image steps for gfx950:
// clahe_->apply(image, image) (/root/reference/ic_gvins/ic_gvins/tracking/tracking.cc:139,
// clahe_ = cv::createCLAHE(3.0, cv::Size(21, 21)) at :63) and calculateHistigram
// (:88-105), batched over images resident in HBM.  The rules (OpenCV 4.x
// CLAHE_Impl::apply, 8-bit) are written down in oracle/clahe.c.
//
// Kernels:
//  lut_kernel    one 256-thread workgroup per (image, tile): LDS histogram of
//                the tile (REFLECT_101 source for the bottom/right pad tiles),
//                clip, redistribute, cumulative sum and the 256-byte LUT by
//                wave 0 (4 bins per lane, shuffle scan).  When the histogram
//                check is on, the in-image part of each tile's histogram is
//                added to the image histogram first (global atomics, non-zero
//                bins only).
//  apply_kernel  one workgroup per (image, band of rows): the <= 3 LUT rows of
//                tiles the band touches are staged in LDS, then every pixel is
//                the bilinear blend of 4 LUT entries in fp32 (OpenCV's scalar
//                CLAHE_Interpolation_Body order, no FMA) rounded half to even.
//                4 pixels per thread and step, dword loads/stores when aligned.
//  mean_kernel   Tracking::calculateHistigram from the image histogram.
#include <hip/hip_runtime.h>

#include "gvx_internal.h"

namespace gvx {

namespace {

__device__ __forceinline__ int refl101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

__device__ __forceinline__ uint32_t sat_round_u8(float v) {
    const int r = (int)__builtin_rintf(v);  // cvRound: half to even
    return (uint32_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

__global__ void __launch_bounds__(256) lut_kernel(const uint8_t* __restrict__ src, int64_t img_stride,
                                                  int stride, ClaheGeom g, uint8_t* __restrict__ lut,
                                                  uint32_t* __restrict__ hist_img) {
    __shared__ uint32_t hist[256];
    const int ntiles = g.tiles_x * g.tiles_y;
    const int img = blockIdx.x / ntiles, k = blockIdx.x - img * ntiles;
    const int ty = k / g.tiles_x, tx = k - ty * g.tiles_x;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    hist[t] = 0;
    __syncthreads();
    const uint8_t* s = src + img * img_stride;
    const int x0 = tx * g.tw, y0 = ty * g.th;
    const int xe = min(x0 + g.tw, g.w), ye = min(y0 + g.th, g.h);
    for (int y = y0 + wave; y < ye; y += 4) {
        const uint8_t* row = s + (int64_t)y * stride;
        for (int x = x0 + lane; x < xe; x += 64) atomicAdd(&hist[row[x]], 1u);
    }
    if (hist_img) {
        __syncthreads();
        const uint32_t v = hist[t];
        if (v) atomicAdd(&hist_img[img * 256 + t], v);
    }
    if (x0 + g.tw > g.w || y0 + g.th > g.h) {
        // the copyMakeBorder(..., BORDER_REFLECT_101) part of the LUT source
        for (int y = y0 + wave; y < y0 + g.th; y += 4) {
            const uint8_t* row = s + (int64_t)refl101(y, g.h) * stride;
            const bool yin = y < g.h;
            for (int x = x0 + lane; x < x0 + g.tw; x += 64)
                if (!yin || x >= g.w) atomicAdd(&hist[row[refl101(x, g.w)]], 1u);
        }
    }
    __syncthreads();
    if (wave != 0) return;
    uint32_t h4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) h4[i] = hist[4 * lane + i];
    if (g.clip > 0) {
        const uint32_t clip = (uint32_t)g.clip;
        uint32_t cl = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (h4[i] > clip) {
                cl += h4[i] - clip;
                h4[i] = clip;
            }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) cl += __shfl_xor(cl, o, 64);
        const uint32_t batch = cl / 256, residual = cl - batch * 256;
        const uint32_t step = residual ? max(256u / residual, 1u) : 1u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t b = 4 * lane + i;
            h4[i] += batch + ((residual && b % step == 0 && b / step < residual) ? 1u : 0u);
        }
    }
    uint32_t c4[4];
    c4[0] = h4[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) c4[i] = c4[i - 1] + h4[i];
    uint32_t incl = c4[3];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    const uint32_t base = incl - c4[3];
    uint32_t packed = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) packed |= sat_round_u8((float)(base + c4[i]) * g.lut_scale) << (8 * i);
    reinterpret_cast<uint32_t*>(lut + ((int64_t)img * ntiles + k) * 256)[lane] = packed;
}

constexpr int MAX_LUT_ROWS = 3;

// src may equal dst (in place, like the reference's apply(image, image)): each
// thread reads its 4 pixels before it writes them, and no other thread reads them.
__global__ void __launch_bounds__(256) apply_kernel(const uint8_t* src, int64_t img_stride,
                                                    int stride, uint8_t* dst, int64_t dst_img_stride,
                                                    int dst_stride, ClaheGeom g, const uint8_t* __restrict__ lut,
                                                    int band_rows, int nbands, int aligned) {
    extern __shared__ uint4 sl4[];  // MAX_LUT_ROWS * tiles_x * 256 bytes
    uint8_t* sl = reinterpret_cast<uint8_t*>(sl4);
    const int img = blockIdx.x / nbands, band = blockIdx.x - img * nbands;
    const int y0 = band * band_rows, y1 = min(y0 + band_rows, g.h);
    const float inv_th = 1.0f / g.th, inv_tw = 1.0f / g.tw;
    const int tyA = max((int)floorf((float)y0 * inv_th - 0.5f), 0);
    const int tyB = min((int)floorf((float)(y1 - 1) * inv_th - 0.5f) + 1, g.tiles_y - 1);
    const int ntiles = g.tiles_x * g.tiles_y;
    {
        const uint4* lsrc = reinterpret_cast<const uint4*>(lut + ((int64_t)img * ntiles + tyA * g.tiles_x) * 256);
        const int n16 = (tyB - tyA + 1) * g.tiles_x * 16;
        for (int i = threadIdx.x; i < n16; i += 256) sl4[i] = lsrc[i];
    }
    __syncthreads();
    const uint8_t* s = src + img * img_stride;
    uint8_t* d = dst + img * dst_img_stride;
    const int nq = (g.w + 3) >> 2;
    const int total = (y1 - y0) * nq;
    const int lrow = g.tiles_x * 256;
    for (int idx = threadIdx.x; idx < total; idx += 256) {
        const int r = idx / nq, q = idx - r * nq;
        const int y = y0 + r, x = 4 * q;
        const float tyf = (float)y * inv_th - 0.5f;
        const int ty1r = (int)floorf(tyf);
        const float ya = tyf - (float)ty1r, ya1 = 1.0f - ya;
        const uint8_t* p1 = sl + (max(ty1r, 0) - tyA) * lrow;
        const uint8_t* p2 = sl + (min(ty1r + 1, g.tiles_y - 1) - tyA) * lrow;
        const uint8_t* srow = s + (int64_t)y * stride;
        uint8_t* drow = d + (int64_t)y * dst_stride;
        const int nv = min(4, g.w - x);
        uint32_t pix;
        if (aligned && nv == 4)
            pix = *reinterpret_cast<const uint32_t*>(srow + x);
        else {
            pix = 0;
            for (int j = 0; j < nv; ++j) pix |= (uint32_t)srow[x + j] << (8 * j);
        }
        uint32_t out = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float txf = (float)(x + j) * inv_tw - 0.5f;
            const int tx1r = (int)floorf(txf);
            const float xa = txf - (float)tx1r, xa1 = 1.0f - xa;
            const int v = (pix >> (8 * j)) & 255;
            const int i1 = max(tx1r, 0) * 256 + v, i2 = min(tx1r + 1, g.tiles_x - 1) * 256 + v;
            const float res = ((float)p1[i1] * xa1 + (float)p1[i2] * xa) * ya1 +
                              ((float)p2[i1] * xa1 + (float)p2[i2] * xa) * ya;
            out |= sat_round_u8(res) << (8 * j);
        }
        if (aligned && nv == 4)
            *reinterpret_cast<uint32_t*>(drow + x) = out;
        else
            for (int j = 0; j < nv; ++j) drow[x + j] = (uint8_t)(out >> (8 * j));
    }
}

__global__ void __launch_bounds__(64) mean_kernel(const uint32_t* __restrict__ hist_img, int n, int w, int h,
                                                  double* __restrict__ mean) {
    const int img = blockIdx.x * 64 + threadIdx.x;
    if (img >= n) return;
    const uint32_t* hs = hist_img + img * 256;
    double m = 0;
    for (int k = 0; k < 256; ++k) m += (double)((float)hs[k] * (float)k) / 256.0;
    mean[img] = m / (double)(w * h);
}

}  // namespace

ClaheGeom clahe_geometry(int w, int h, double clip_limit, int tiles_x, int tiles_y) {
    ClaheGeom g{};
    g.w = w;
    g.h = h;
    g.tiles_x = tiles_x;
    g.tiles_y = tiles_y;
    int ew = w, eh = h;
    if (!(w % tiles_x == 0 && h % tiles_y == 0)) {
        ew = w + tiles_x - (w % tiles_x);
        eh = h + tiles_y - (h % tiles_y);
    }
    g.tw = ew / tiles_x;
    g.th = eh / tiles_y;
    const int total = g.tw * g.th;
    g.lut_scale = (float)255 / total;
    g.clip = 0;
    if (clip_limit > 0.0) g.clip = std::max((int)(clip_limit * total / 256), 1);
    return g;
}

hipError_t launch_clahe(gvx_ctx* c, int n, const ClaheGeom& g, const uint8_t* src, int64_t img_stride,
                        int stride, uint8_t* dst, int64_t dst_img_stride, int dst_stride, uint8_t* lut,
                        uint32_t* hist_img, double* hist_mean) {
    if (n <= 0) return hipSuccess;
    const int ntiles = g.tiles_x * g.tiles_y;
    if (hist_img) {
        hipError_t e = hipMemsetAsync(hist_img, 0, (size_t)n * 256 * sizeof(uint32_t), c->stream);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(lut_kernel, dim3(n * ntiles), dim3(256), 0, c->stream, src, img_stride, stride, g, lut,
                       hist_img);
    // bands: <= th rows (so <= 3 LUT rows), and enough workgroups to fill the chip
    int band = (int)std::min<int64_t>(g.th, 32);
    const int64_t want = 4LL * c->n_cu;
    while (band > 1 && (int64_t)n * ((g.h + band - 1) / band) < want) band = (band + 1) / 2;
    const int nbands = (g.h + band - 1) / band;
    const int aligned = ((uintptr_t)src % 4 == 0) && ((uintptr_t)dst % 4 == 0) && stride % 4 == 0 &&
                        dst_stride % 4 == 0 && img_stride % 4 == 0 && dst_img_stride % 4 == 0;
    const size_t lds = (size_t)MAX_LUT_ROWS * g.tiles_x * 256;
    hipLaunchKernelGGL(apply_kernel, dim3(n * nbands), dim3(256), lds, c->stream, src, img_stride, stride, dst,
                       dst_img_stride, dst_stride, g, (const uint8_t*)lut, band, nbands, aligned);
    if (hist_img && hist_mean)
        hipLaunchKernelGGL(mean_kernel, dim3((n + 63) / 64), dim3(64), 0, c->stream, (const uint32_t*)hist_img, n,
                           g.w, g.h, hist_mean);
    return hipGetLastError();
}

}  // namespace gvx
