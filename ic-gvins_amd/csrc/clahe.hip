// clahe.hip -- Tracking::preprocessing's image steps for gfx950:
// clahe_->apply(image, image) (/root/reference/ic_gvins/ic_gvins/tracking/tracking.cc:139,
// clahe_ = cv::createCLAHE(3.0, cv::Size(21, 21)) at :63) and calculateHistigram
// (:88-105), batched over images resident in HBM.  The rules (OpenCV 4.x
// CLAHE_Impl::apply, 8-bit) are written down in oracle/clahe.c.
//
// Kernels:
//  lut_kernel    one 256-thread workgroup per (image, row of tiles, group of
//                tiles -- the whole row for batches, a few tiles for a single
//                frame): every pixel of the group is read once (8 bytes per load, 8 loads
//                in flight per thread) into per-tile LDS histograms, the
//                REFLECT_101 pad pixels (copyMakeBorder of the LUT source)
//                are added, and each wave then turns tiles into LUTs: clip,
//                redistribute, cumulative sum (4 bins per lane, shuffle scan)
//                and the 256-byte LUT.  When the histogram check is on, the
//                in-image counts of the tile row go to the image histogram
//                (one global atomic per non-zero bin) before the pads are added.
//  apply_kernel  one workgroup per (image, band of rows with the same upper
//                tile row, part of the band): the band's two LUT rows are
//                interleaved in LDS so one ds_read_b32 returns a pixel's four
//                LUT values; each thread owns 8 columns for the whole band --
//                their table offsets and fp32 weights are computed once -- and
//                walks the band 8 rows at a time, loads first.  Every pixel is
//                the bilinear blend of the 4 LUT values in fp32 (OpenCV's
//                scalar CLAHE_Interpolation_Body order, no FMA), rounded half
//                to even.
//  mean_kernel   Tracking::calculateHistigram from the image histogram.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

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

typedef float f2 __attribute__((ext_vector_type(2)));

// a * {b.lo, b.lo} and a * {b.hi, b.hi}: one v_pk_mul_f32 each, the half of b
// broadcast through op_sel (no register pair per multiplier)
__device__ __forceinline__ f2 pk_mul_lo(f2 a, f2 b) {
    f2 r;
    __asm__("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f2 pk_mul_hi(f2 a, f2 b) {
    f2 r;
    __asm__("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ uint32_t sat_round_u8(float v) {
    const int r = (int)__builtin_rintf(v);  // cvRound: half to even
    return (uint32_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

// x / d for 0 <= x < 2^20, d >= 1 (fp32 estimate, corrected to exact)
__device__ __forceinline__ int div_small(int x, int d, float inv_d) {
    int q = (int)((float)x * inv_d);
    q += (q + 1) * d <= x ? 1 : 0;
    q -= q * d > x ? 1 : 0;
    return q;
}

constexpr int LUT_THREADS = 256;
constexpr int HROW = 257;  // histogram stride: one value in neighbouring tiles -> different banks
constexpr int LUT_UNROLL = 8;

// Inclusive prefix sum of v over the wave's 64 lanes: row_shr DPP steps within
// each 16-lane row (no LDS round trip, unlike a shuffle), then the totals of
// the lower rows by readlane.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31),
                   r2 = __builtin_amdgcn_readlane(v, 47);
    const int row = lane >> 4;
    return v + (row > 0 ? r0 : 0u) + (row > 1 ? r1 : 0u) + (row > 2 ? r2 : 0u);
}

// CLAHE_CalcLut_Body for one tile, by one wavefront: h4 = the lane's bins
// 4*lane .. 4*lane+3 of the tile's histogram.
__device__ __forceinline__ void tile_lut4(uint32_t (&h4)[4], const ClaheGeom& g, int lane, uint8_t* out) {
    if (g.clip > 0) {
        const uint32_t clip = (uint32_t)g.clip;
        uint32_t cl = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (h4[i] > clip) {
                cl += h4[i] - clip;
                h4[i] = clip;
            }
        cl = __builtin_amdgcn_readlane(wave_incl_scan(cl, lane), 63);  // the tile's clipped total
        const uint32_t batch = cl / 256, residual = cl - batch * 256;
        // integer quotients through the fp32 reciprocal, corrected to exact
        // (div_small: no integer division sequence)
        const uint32_t step =
            residual ? (uint32_t)max(div_small(256, (int)residual, __builtin_amdgcn_rcpf((float)residual)), 1) : 1u;
        // bin b gets one more where b % step == 0 and b / step < residual: one
        // division for the lane's first bin, then carried over its four bins
        uint32_t q = (uint32_t)div_small(4 * lane, (int)step, __builtin_amdgcn_rcpf((float)step)),
                 r = 4u * lane - q * step;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            h4[i] += batch + ((residual && r == 0 && q < residual) ? 1u : 0u);
            if (++r == step) {
                r = 0;
                ++q;
            }
        }
    }
    uint32_t c4[4];
    c4[0] = h4[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) c4[i] = c4[i - 1] + h4[i];
    const uint32_t base = wave_incl_scan(c4[3], lane) - c4[3];
    uint32_t packed = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) packed |= sat_round_u8((float)(base + c4[i]) * g.lut_scale) << (8 * i);
    reinterpret_cast<uint32_t*>(out)[lane] = packed;
}
// the same from the tile's 256 bins h (one dword each)
__device__ __forceinline__ void tile_lut(const uint32_t* h, const ClaheGeom& g, int lane, uint8_t* out) {
    uint32_t h4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) h4[i] = h[4 * lane + i];
    tile_lut4(h4, g, lane, out);
}

// fused_kernel's tile histograms (an A/B build switch):
// CLAHE_PACK 0 = one dword per bin; 1 / 2 = two 16-bit bins per dword (a tile
// holds at most 1,647 + pad pixels), in 1 / 2 copies (lanes 0-31 / 32-63)
#ifndef CLAHE_PACK
#define CLAHE_PACK 0
#endif
constexpr int HPK = CLAHE_PACK;
constexpr int HSTR = HPK ? 129 : HROW;  // dwords per tile histogram
constexpr int HCOPY = HPK ? HPK : 1;

// cv::cvtColor(COLOR_BGR2GRAY), 8-bit (OpenCV 4.x RGB2Gray<uchar>, tracking.cc:111-113)
__device__ __forceinline__ uint32_t bgr_gray(uint32_t b, uint32_t g, uint32_t r) {
    return (b * 1868u + g * 9617u + r * 4899u + 8192u) >> 14;
}
// byte k of the 24-byte value {c:b:a} (k constant after unrolling)
__device__ __forceinline__ uint32_t byte24(const uint2& a, const uint2& b, const uint2& c, int k) {
    const uint32_t d[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
    return (d[k >> 2] >> (8 * (k & 3))) & 255u;
}

// chan 3: the source is BGR8 (3 bytes per pixel, strides in bytes); each pixel
// is converted to gray as it is read, and the in-image gray pixels are written
// to gray (image i at gray + i*gray_img, rows gray_pitch apart) for the apply pass.
__global__ void __launch_bounds__(LUT_THREADS) lut_kernel(const uint8_t* __restrict__ src, int64_t img_stride,
                                                          int stride, ClaheGeom g, int vec8, int tpw,
                                                          uint8_t* __restrict__ lut,
                                                          uint32_t* __restrict__ hist_img,
                                                          const int32_t* __restrict__ src_index, int n_src, int chan,
                                                          uint8_t* __restrict__ gray, int64_t gray_img,
                                                          int gray_pitch) {
    extern __shared__ uint32_t hs[];  // tpw histograms of 256 bins, HROW dwords apart
    const int ngrp = (g.tiles_x + tpw - 1) / tpw;
    const int img = blockIdx.x / (g.tiles_y * ngrp);
    const int rem = blockIdx.x - img * g.tiles_y * ngrp;
    const int ty = rem / ngrp, grp = rem - ty * ngrp;
    const int txa0 = grp * tpw, txa1 = min(txa0 + tpw, g.tiles_x);  // this workgroup's tiles
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
    const int nbins = (txa1 - txa0) * HROW;
    for (int i = t; i < nbins; i += LUT_THREADS) hs[i] = 0;
    __syncthreads();
    // src_index (one image): the source image is picked on the device
    const uint8_t* s = src + (src_index ? (int64_t)min(max(*src_index, 0), n_src - 1) : (int64_t)img) * img_stride;
    const int y0 = ty * g.th;
    const int rows_in = max(0, min(y0 + g.th, g.h) - y0);
    const float inv_tw = 1.0f / g.tw;
    const int xlo = txa0 * g.tw, xhi_ext = txa1 * g.tw, xhi = min(xhi_ext, g.w);  // in-image columns [xlo, xhi)
    // the gray value of in-image pixel (x, y)
    auto pixel = [&](int y, int x) -> uint32_t {
        const uint8_t* p = s + (int64_t)y * stride;
        return chan == 3 ? bgr_gray(p[3 * x], p[3 * x + 1], p[3 * x + 2]) : p[x];
    };
    uint8_t* gimg = chan == 3 ? gray + img * gray_img : nullptr;
    // ---- in-image pixels ----
    if (vec8 && chan == 3) {
        // 8 pixels = 24 bytes per chunk; the chunk's gray bytes are stored whole (a
        // chunk shared with the neighbouring group is written with the same bytes)
        const int c8lo = xlo >> 3, n8 = ((xhi + 7) >> 3) - c8lo;
        const int total = rows_in * max(n8, 0);
        for (int base = t; base < total; base += LUT_UNROLL * LUT_THREADS) {
            uint2 v[LUT_UNROLL][3];
            int x0[LUT_UNROLL], yr[LUT_UNROLL];
#pragma unroll
            for (int k = 0; k < LUT_UNROLL; ++k) {
                const int i = base + k * LUT_THREADS;
                const int r = i / n8, c8 = c8lo + (i - r * n8);
                x0[k] = 8 * c8;
                yr[k] = y0 + r;
                const uint2* p = reinterpret_cast<const uint2*>(s + (int64_t)(y0 + r) * stride + 24 * c8);
#pragma unroll
                for (int q = 0; q < 3; ++q) v[k][q] = i < total ? p[q] : uint2{0, 0};
            }
#pragma unroll
            for (int k = 0; k < LUT_UNROLL; ++k) {
                if (base + k * LUT_THREADS >= total) break;
                const int txa = div_small(max(x0[k], xlo), g.tw, inv_tw);
                const int xb = (txa + 1) * g.tw;
                uint32_t gw[2] = {0, 0};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t b = bgr_gray(byte24(v[k][0], v[k][1], v[k][2], 3 * j),
                                                byte24(v[k][0], v[k][1], v[k][2], 3 * j + 1),
                                                byte24(v[k][0], v[k][1], v[k][2], 3 * j + 2));
                    gw[j >> 2] |= b << (8 * (j & 3));
                    const int x = x0[k] + j;
                    const int tx = x < xb ? txa : (x < xb + g.tw ? txa + 1 : div_small(x, g.tw, inv_tw));
                    if (x >= xlo && x < xhi) atomicAdd(&hs[(tx - txa0) * HROW + b], 1u);
                }
                *reinterpret_cast<uint2*>(gimg + (int64_t)yr[k] * gray_pitch + x0[k]) = uint2{gw[0], gw[1]};
            }
        }
    } else if (vec8) {
        const int c8lo = xlo >> 3, n8 = ((xhi + 7) >> 3) - c8lo;  // w % 8 == 0: chunks stay in the row
        const int total = rows_in * max(n8, 0);
        for (int base = t; base < total; base += LUT_UNROLL * LUT_THREADS) {
            uint2 v[LUT_UNROLL];
            int x0[LUT_UNROLL];
#pragma unroll
            for (int k = 0; k < LUT_UNROLL; ++k) {
                const int i = base + k * LUT_THREADS;
                const int r = i / n8, c8 = c8lo + (i - r * n8);
                x0[k] = 8 * c8;
                v[k] = i < total ? *reinterpret_cast<const uint2*>(s + (int64_t)(y0 + r) * stride + 8 * c8)
                                 : uint2{0, 0};
            }
#pragma unroll
            for (int k = 0; k < LUT_UNROLL; ++k) {
                if (base + k * LUT_THREADS >= total) break;
                const int txa = div_small(max(x0[k], xlo), g.tw, inv_tw);
                const int xb = (txa + 1) * g.tw;  // first column of the next tile
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t b = ((j < 4 ? v[k].x : v[k].y) >> (8 * (j & 3))) & 255u;
                    const int x = x0[k] + j;
                    const int tx = x < xb ? txa : (x < xb + g.tw ? txa + 1 : div_small(x, g.tw, inv_tw));
                    if (x >= xlo && x < xhi) atomicAdd(&hs[(tx - txa0) * HROW + b], 1u);
                }
            }
        }
    } else {
        const int cw = xhi - xlo;
        const int total = rows_in * max(cw, 0);
        for (int i = t; i < total; i += LUT_THREADS) {
            const int r = i / cw, x = xlo + (i - r * cw);
            const uint32_t b = pixel(y0 + r, x);
            if (gimg) gimg[(int64_t)(y0 + r) * gray_pitch + x] = (uint8_t)b;
            atomicAdd(&hs[(div_small(x, g.tw, inv_tw) - txa0) * HROW + b], 1u);
        }
    }
    if (hist_img) {
        __syncthreads();
        for (int b = t; b < 256; b += LUT_THREADS) {
            uint32_t sum = 0;
            for (int tx = 0; tx < txa1 - txa0; ++tx) sum += hs[tx * HROW + b];
            if (sum) atomicAdd(&hist_img[img * 256 + b], sum);
        }
    }
    // ---- the copyMakeBorder(..., BORDER_REFLECT_101) part of the LUT source ----
    if (xhi_ext > g.w) {  // pad columns of the in-image rows (this group's share)
        const int pxlo = max(g.w, xlo), pc = xhi_ext - pxlo;
        for (int i = t; i < rows_in * pc; i += LUT_THREADS) {
            const int r = i / pc, x = pxlo + (i - r * pc);
            atomicAdd(&hs[(div_small(x, g.tw, inv_tw) - txa0) * HROW + pixel(y0 + r, refl101(x, g.w))], 1u);
        }
    }
    const int pr = g.th - rows_in, ecw = xhi_ext - xlo;  // pad rows (reflected source rows), this group's columns
    for (int i = t; i < pr * ecw; i += LUT_THREADS) {
        const int r = i / ecw, x = xlo + (i - r * ecw);
        const int sy = refl101(y0 + rows_in + r, g.h);
        atomicAdd(&hs[(div_small(x, g.tw, inv_tw) - txa0) * HROW + pixel(sy, refl101(x, g.w))], 1u);
    }
    __syncthreads();
    for (int tx = txa0 + wave; tx < txa1; tx += LUT_THREADS / 64)
        tile_lut(hs + (tx - txa0) * HROW, g, lane,
                 lut + ((int64_t)img * g.tiles_x * g.tiles_y + ty * g.tiles_x + tx) * 256);
}

constexpr int TROW = 260;  // LDS dwords per table row (16-B aligned, bank skew between tiles)
constexpr int PPT = 8;     // pixels (columns) per thread
constexpr int ROWS_UNROLL = 8;
constexpr int TAB_UNROLL = 8;

// First row y with floor(y/th - 0.5) >= k in fp32 (CLAHE_Interpolation_Body's
// row mapping), y in [0, h].
__device__ __forceinline__ int first_row(int k, const ClaheGeom& g, float inv_th) {
    int y = max(0, min(g.h, (int)((k + 0.5f) * g.th)));
    while (y > 0 && (int)floorf((float)(y - 1) * inv_th - 0.5f) >= k) --y;
    while (y < g.h && (int)floorf((float)y * inv_th - 0.5f) < k) ++y;
    return y;
}

// src may equal dst (in place, like the reference's apply(image, image)): each
// thread reads its pixels before it writes them, and no other thread reads them.
//
// Band b = the rows whose upper tile row is ty1 = b - 1 (b = 0 .. tiles_y), so a
// band blends one pair of LUT rows (ty1, ty2 clamped); the band is split over
// `nsplit` workgroups.  LDS table: entry (k, v), k = tx1 + 1 in [0, tiles_x],
// is one dword {L[ty1][tx1c][v], L[ty1][tx2c][v], L[ty2][tx1c][v],
// L[ty2][tx2c][v]} (tile indices clamped as the reference does), so each pixel
// takes one ds_read_b32 for its four LUT values.
// ring: dst is pixel (0,0) of a level with a PAD-pixel ring (a frame's padded
// level-0 slot); every output pixel is also stored where the REFLECT_101 ring
// copies it -- the mirrored ring row (top / bottom) and the mirrored side-band
// column (left / right), both for the corners -- so the pyramid pass and the
// detection read the equalised frame with its ring and no copy pass runs.
__global__ void __launch_bounds__(1024) apply_kernel(const uint8_t* src, int64_t img_stride, int stride,
                                                     uint8_t* dst, int64_t dst_img_stride, int dst_stride,
                                                     ClaheGeom g, const uint8_t* __restrict__ lut, int nsplit,
                                                     int vec8, const int32_t* __restrict__ src_index, int n_src, int ring) {
    extern __shared__ uint32_t tab[];  // (tiles_x + 1) * TROW dwords
    const int nb = g.tiles_y + 1;
    const int img = blockIdx.x / (nb * nsplit);
    const int rem = blockIdx.x - img * nb * nsplit;
    const int b = rem / nsplit, part = rem - b * nsplit;
    const float inv_th = 1.0f / g.th, inv_tw = 1.0f / g.tw;
    const int ys = b == 0 ? 0 : first_row(b - 1, g, inv_th);
    const int ye = b == g.tiles_y ? g.h : first_row(b, g, inv_th);
    const int per = (ye - ys + nsplit - 1) / nsplit;
    const int y0 = ys + part * per, y1 = min(ye, y0 + per);
    if (y0 >= y1) return;  // whole workgroup: no barrier below is skipped by part of it
    const int ty1 = max(b - 1, 0), ty2 = min(b, g.tiles_y - 1);
    {
        // all loads of a thread's table entries first (L2 hits; one round trip)
        const uint32_t* L = reinterpret_cast<const uint32_t*>(lut + (int64_t)img * g.tiles_x * g.tiles_y * 256);
        const int items = (g.tiles_x + 1) * 64;
        for (int i0 = threadIdx.x; i0 < items; i0 += TAB_UNROLL * blockDim.x) {
            uint32_t a[TAB_UNROLL], bb[TAB_UNROLL], c[TAB_UNROLL], d[TAB_UNROLL];
#pragma unroll
            for (int u = 0; u < TAB_UNROLL; ++u) {
                const int i = min(i0 + u * (int)blockDim.x, items - 1);
                const int k = i >> 6, q = i & 63;
                const int ta = max(k - 1, 0), tb = min(k, g.tiles_x - 1);
                a[u] = L[(ty1 * g.tiles_x + ta) * 64 + q];
                bb[u] = L[(ty1 * g.tiles_x + tb) * 64 + q];
                c[u] = L[(ty2 * g.tiles_x + ta) * 64 + q];
                d[u] = L[(ty2 * g.tiles_x + tb) * 64 + q];
            }
#pragma unroll
            for (int u = 0; u < TAB_UNROLL; ++u) {
                const int i = i0 + u * (int)blockDim.x;
                if (i >= items) break;
                const int k = i >> 6, q = i & 63;
                // byte j of (a, bb, c, d) -> dword for value 4q + j
                const uint32_t ab_lo = __builtin_amdgcn_perm(bb[u], a[u], 0x05010400u);  // a0 b0 a1 b1
                const uint32_t ab_hi = __builtin_amdgcn_perm(bb[u], a[u], 0x07030602u);  // a2 b2 a3 b3
                const uint32_t cd_lo = __builtin_amdgcn_perm(d[u], c[u], 0x05010400u);
                const uint32_t cd_hi = __builtin_amdgcn_perm(d[u], c[u], 0x07030602u);
                uint32_t* o = tab + k * TROW + 4 * q;
                o[0] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u);  // a0 b0 c0 d0
                o[1] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u);  // a1 b1 c1 d1
                o[2] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u);
                o[3] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u);
            }
        }
    }
    __syncthreads();
    const uint8_t* s = src + (src_index ? (int64_t)min(max(*src_index, 0), n_src - 1) : (int64_t)img) * img_stride;
    uint8_t* dd = dst + img * dst_img_stride;
    for (int x0 = PPT * threadIdx.x; x0 < g.w; x0 += PPT * blockDim.x) {
        // column terms of CLAHE_Interpolation_Body's constructor, once per thread
        int ko[PPT];
        float xa[PPT], xa1[PPT];
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const float txf = (float)(x0 + j) * inv_tw - 0.5f;
            const int tx1 = (int)floorf(txf);
            xa[j] = txf - (float)tx1;
            xa1[j] = 1.0f - xa[j];
            ko[j] = (min(tx1, g.tiles_x - 1) + 1) * TROW;
        }
        const int nv = min(PPT, g.w - x0);
        const bool fast = vec8 && nv == PPT;
        for (int yb = y0; yb < y1; yb += ROWS_UNROLL) {
            uint2 pix[ROWS_UNROLL];
#pragma unroll
            for (int k = 0; k < ROWS_UNROLL; ++k) {
                const int y = min(yb + k, y1 - 1);
                const uint8_t* srow = s + (int64_t)y * stride + x0;
                if (fast) {
                    pix[k] = *reinterpret_cast<const uint2*>(srow);
                } else {
                    uint32_t lo = 0, hi = 0;
                    for (int j = 0; j < nv; ++j) {
                        const uint32_t bv = srow[j];
                        if (j < 4)
                            lo |= bv << (8 * j);
                        else
                            hi |= bv << (8 * (j - 4));
                    }
                    pix[k] = uint2{lo, hi};
                }
            }
#pragma unroll
            for (int k = 0; k < ROWS_UNROLL; ++k) {
                const int y = yb + k;
                if (y >= y1) break;
                const float tyf = (float)y * inv_th - 0.5f;
                const float ya = tyf - floorf(tyf), ya1 = 1.0f - ya;
                uint32_t out[2] = {0, 0};
#pragma unroll
                for (int j = 0; j < PPT; ++j) {
                    const uint32_t v = ((j < 4 ? pix[k].x : pix[k].y) >> (8 * (j & 3))) & 255u;
                    const uint32_t e = tab[ko[j] + v];
                    const float l11 = (float)(e & 255u), l12 = (float)((e >> 8) & 255u);
                    const float l21 = (float)((e >> 16) & 255u), l22 = (float)(e >> 24);
                    const float res = (l11 * xa1[j] + l12 * xa[j]) * ya1 + (l21 * xa1[j] + l22 * xa[j]) * ya;
                    // cvRound + saturate_cast<uchar> in one instruction (tools/cvt_pk_u8_probe.hip)
                    out[j >> 2] = __builtin_amdgcn_cvt_pk_u8_f32(res, j & 3, out[j >> 2]);
                }
                uint8_t* drow = dd + (int64_t)y * dst_stride + x0;
                if (fast) {
                    *reinterpret_cast<uint2*>(drow) = uint2{out[0], out[1]};
                } else {
                    for (int j = 0; j < nv; ++j) drow[j] = (uint8_t)(out[j >> 2] >> (8 * (j & 3)));
                }
                if (ring) {
                    // REFLECT_101 ring: row y is copied to ring row -y (1 <= y <= PAD) or
                    // 2h-2-y (h-1-PAD <= y <= h-2); column x to -x or 2w-2-x likewise
                    const int my = (y >= 1 && y <= PAD) ? -y : ((y >= g.h - 1 - PAD && y <= g.h - 2) ? 2 * g.h - 2 - y : y);
                    uint8_t* mrow = dd + (int64_t)my * dst_stride + x0;
                    if (my != y) {
                        if (fast)
                            *reinterpret_cast<uint2*>(mrow) = uint2{out[0], out[1]};
                        else
                            for (int j = 0; j < nv; ++j) mrow[j] = (uint8_t)(out[j >> 2] >> (8 * (j & 3)));
                    }
                    if (x0 <= PAD || x0 + PPT >= g.w - 1 - PAD) {
                        for (int j = 0; j < nv; ++j) {
                            const int x = x0 + j;
                            const int mx = (x >= 1 && x <= PAD) ? -x : ((x >= g.w - 1 - PAD && x <= g.w - 2) ? 2 * g.w - 2 - x : x);
                            if (mx == x) continue;
                            const uint8_t v8 = (uint8_t)(out[j >> 2] >> (8 * (j & 3)));
                            drow[mx - x0] = v8;
                            if (my != y) mrow[mx - x0] = v8;
                        }
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// fused_kernel: both passes in one workgroup per (image, segment of bands), for
// batches.  The workgroup walks its bands top to bottom; each thread owns one
// 8-pixel column chunk and the rows ph, ph + nph, ... of every tile row, and
// holds the pixels of the three tile rows in use in registers: while band b is
// blended from tile rows b-1 and b, tile row b+1 is loaded, its histograms are
// built and turned into LUT row b+1 (two LUT-row buffers, by parity), and the
// band's table is rebuilt from LUT rows b and b+1.  Every source pixel is read
// from HBM once and every output pixel written once (2 B/px against 3 B/px for
// lut_kernel + apply_kernel), and BGR8 frames are converted in registers (no
// gray scratch).  The table holds the four LUT values of an entry as bytes (one
// ds_read_b32 per pixel, converted by v_cvt_f32_ubyte0..3): the LDS, not the
// VALU, bounds this kernel (r04: LDS-array cycles ~60 % of the launch, two thirds
// of them bank conflicts), and the fp32 table's ds_read_b128 took four LDS
// cycles per pixel group and four times the table stores -- 0.236 -> 0.223 ms per
// 256 frames (r04 v9).  The result is rounded and packed by v_cvt_pk_u8_f32
// (round half to even, saturating: cvRound + saturate_cast,
// tools/cvt_pk_u8_probe.hip).  The
// arithmetic is that of lut_kernel / apply_kernel (same tile_lut, same fp32
// blend order), so the two paths are bit-identical.  Segments > 1 recompute the
// LUT row at each seam, so src must not overlap dst (the host keeps in-place
// calls on the two-kernel path).
template <int RMAX, int CHAN, bool VEC8>
__global__ void __launch_bounds__(1024) fused_kernel(const uint8_t* __restrict__ src, int64_t img_stride,
                                                     int stride, uint8_t* __restrict__ dst, int64_t dst_img_stride,
                                                     int dst_stride, ClaheGeom g, int nseg, int cpr, int nph,
                                                     uint32_t* __restrict__ hist_img) {
    extern __shared__ float4 smf[];
    uint32_t* tab = reinterpret_cast<uint32_t*>(smf);                      // (tiles_x + 1) * TROW entries
    uint32_t* hs = tab + (g.tiles_x + 1) * TROW;  // tiles_x (+1 scratch) histograms, HSTR apart, HCOPY copies
    const int hcs = (g.tiles_x + 1) * HSTR;        // dwords per copy
    uint32_t* lrb = hs + hcs * HCOPY;              // 2 x tiles_x * 64 dwords: LUT rows by parity
    uint32_t* ih = lrb + 2 * g.tiles_x * 64;       // 256: in-image counts (histogram check)
    const int nb = g.tiles_y + 1;
    const int img = blockIdx.x / nseg, seg = blockIdx.x - img * nseg;
    const int b0 = seg * nb / nseg, b1 = (seg + 1) * nb / nseg;
    const int t = threadIdx.x, nthr = blockDim.x, wave = t >> 6, lane = t & 63, nwave = nthr >> 6;
    const int c8 = t % cpr, ph = t / cpr;
    const bool act = ph < nph;
    const int x0 = 8 * c8, nv = min(8, g.w - x0);
    const bool fast = VEC8;  // 8-byte aligned rows, w % 8 == 0: every chunk is whole
    const uint8_t* s = src + (int64_t)img * img_stride;
    uint8_t* dd = dst + (int64_t)img * dst_img_stride;
    const float inv_th = 1.0f / g.th, inv_tw = 1.0f / g.tw;
    const int ew = g.tiles_x * g.tw;
    for (int i = t; i < hcs * HCOPY; i += nthr) hs[i] = 0;
    // this lane's histogram copy; one bin count of value v into tile offset ho
    uint32_t* const hmine = hs + ((HPK == 2 && (lane & 32)) ? hcs : 0);
    auto hadd = [&](uint32_t* h, int ho, uint32_t v) {
        if constexpr (HPK)
            atomicAdd(&h[ho + (int)(v >> 1)], 1u << ((v & 1u) << 4));
        else
            atomicAdd(&h[ho + (int)v], 1u);
    };
    auto hget = [&](int tx, int b) -> uint32_t {  // bin b of tile tx, all copies
        uint32_t n = 0;
#pragma unroll
        for (int c = 0; c < HCOPY; ++c) {
            const uint32_t d = hs[c * hcs + tx * HSTR + (HPK ? (b >> 1) : b)];
            n += HPK ? ((d >> ((b & 1) << 4)) & 0xffffu) : d;
        }
        return n;
    };
    if (hist_img)
        for (int i = t; i < 256; i += nthr) ih[i] = 0;
    // column terms: the histogram bin offset (-1 past the image) and the blend terms
    // kh[j]: the table entry of (tx1 + 1, value 0) in the low half, the histogram
    // offset of column x in the high half (past the image: a scratch histogram
    // that is never read), one register per column
    uint32_t kh[8];
    f2 xw[8];  // {xa1, xa} of column j
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int x = x0 + j;
        const int hoff = (x < g.w ? div_small(x, g.tw, inv_tw) : g.tiles_x) * HSTR;
        const float txf = (float)x * inv_tw - 0.5f;
        const int tx1 = (int)floorf(txf);
        const float xa = txf - (float)tx1;
        xw[j] = f2{1.0f - xa, xa};
        kh[j] = (uint32_t)((min(tx1, g.tiles_x - 1) + 1) * TROW) | ((uint32_t)hoff << 16);
    }
    auto pixel = [&](int y, int x) -> uint32_t {
        const uint8_t* p = s + (int64_t)y * stride;
        return CHAN == 3 ? bgr_gray(p[3 * x], p[3 * x + 1], p[3 * x + 2]) : p[x];
    };
    // row slot i of tile row k: y = k*th + ph + nph*i (valid when inside the tile row and the image)
    auto slot_row = [&](int k, int i) -> int {
        const int yr = ph + nph * i;
        return (act && yr < g.th) ? k * g.th + yr : -1;
    };
    // raw loads of tile row k (CHAN 3: 24 bytes per chunk, converted in gray_of)
    auto load = [&](int k, uint2 (&raw)[RMAX][CHAN]) {
        if (fast) {
            // branch-free: a slot outside the tile row or the image reads row 0
            // (its value is never used), so the loads issue back to back
#pragma unroll
            for (int i = 0; i < RMAX; ++i) {
                const int y0 = slot_row(k, i);
                const int y = (y0 >= 0 && y0 < g.h) ? y0 : 0;
                const uint64_t* p = reinterpret_cast<const uint64_t*>(s + (int64_t)y * stride + CHAN * x0);
#pragma unroll
                for (int q = 0; q < CHAN; ++q) {
                    const uint64_t v = __builtin_nontemporal_load(p + q);
                    raw[i][q] = uint2{(uint32_t)v, (uint32_t)(v >> 32)};
                }
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < RMAX; ++i) {
            const int y = slot_row(k, i);
            if (y >= 0 && y < g.h) {
                const uint8_t* p = s + (int64_t)y * stride + CHAN * x0;
                if (fast) {
#pragma unroll
                    for (int q = 0; q < CHAN; ++q) raw[i][q] = reinterpret_cast<const uint2*>(p)[q];
                } else {
                    uint32_t lo = 0, hi = 0;
                    for (int j = 0; j < nv; ++j) {
                        const uint32_t v = pixel(y, x0 + j);
                        if (j < 4)
                            lo |= v << (8 * j);
                        else
                            hi |= v << (8 * (j - 4));
                    }
                    raw[i][0] = uint2{lo, hi};  // already gray (gray_of passes it through)
                }
            }
        }
    };
    auto gray_of = [&](const uint2 (&r)[CHAN]) -> uint2 {
        if (CHAN == 1 || !fast) return r[0];
        uint32_t gw[2] = {0, 0};
#pragma unroll
        for (int j = 0; j < 8; ++j)
            gw[j >> 2] |= bgr_gray(byte24(r[0], r[CHAN / 2], r[CHAN - 1], 3 * j),
                                   byte24(r[0], r[CHAN / 2], r[CHAN - 1], 3 * j + 1),
                                   byte24(r[0], r[CHAN / 2], r[CHAN - 1], 3 * j + 2))
                          << (8 * (j & 3));
        return uint2{gw[0], gw[1]};
    };
    // histograms of tile row k: in-image pixels (from registers), the image
    // histogram, then the REFLECT_101 pad pixels of copyMakeBorder; LUT row -> lr
    auto build_lut_row = [&](int k, const uint2 (&px)[RMAX], bool count_img) {
#pragma unroll
        for (int i = 0; i < RMAX; ++i) {
            const int y = slot_row(k, i);
            if (y < 0 || y >= g.h) continue;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t v = ((j < 4 ? px[i].x : px[i].y) >> (8 * (j & 3))) & 255u;
                hadd(hmine, (int)(kh[j] >> 16), v);
            }
        }
        if (hist_img && count_img) {
            __syncthreads();
            for (int b = t; b < 256; b += nthr) {
                uint32_t sum = 0;
                for (int tx = 0; tx < g.tiles_x; ++tx) sum += hget(tx, b);
                ih[b] += sum;
            }
            __syncthreads();
        }
        const int y0 = k * g.th, rows_in = max(0, min(y0 + g.th, g.h) - y0);
        if (ew > g.w) {
            const int pc = ew - g.w;
            for (int i = t; i < rows_in * pc; i += nthr) {
                const int r = i / pc, x = g.w + (i - r * pc);
                hadd(hs, div_small(x, g.tw, inv_tw) * HSTR, pixel(y0 + r, refl101(x, g.w)));
            }
        }
        const int pr = g.th - rows_in;
        for (int i = t; i < pr * ew; i += nthr) {
            const int r = i / ew, x = i - r * ew;
            const int sy = refl101(y0 + rows_in + r, g.h);
            hadd(hs, div_small(x, g.tw, inv_tw) * HSTR, pixel(sy, refl101(x, g.w)));
        }
        __syncthreads();
        uint32_t* lr = lrb + (k & 1) * g.tiles_x * 64;
        for (int tx = wave; tx < g.tiles_x; tx += nwave) {
            if constexpr (HPK) {
                uint32_t h4[4] = {0, 0, 0, 0};
#pragma unroll
                for (int c = 0; c < HCOPY; ++c) {
                    uint32_t* h = hs + c * hcs + tx * HSTR + 2 * lane;
                    const uint32_t d0 = h[0], d1 = h[1];
                    h4[0] += d0 & 0xffffu;
                    h4[1] += d0 >> 16;
                    h4[2] += d1 & 0xffffu;
                    h4[3] += d1 >> 16;
                    h[0] = 0;
                    h[1] = 0;
                }
                tile_lut4(h4, g, lane, reinterpret_cast<uint8_t*>(lr + tx * 64));
            } else {
                tile_lut(hs + tx * HROW, g, lane, reinterpret_cast<uint8_t*>(lr + tx * 64));
#pragma unroll
                for (int q = 0; q < 4; ++q) hs[tx * HROW + 4 * lane + q] = 0;
            }
        }
        __syncthreads();
    };
    // the band's table from LUT rows p (ty1) and q (ty2): entry (k, v) =
    // {L[p][tx1c][v], L[q][tx1c][v], L[p][tx2c][v], L[q][tx2c][v]} as fp32,
    // tx1c = max(k - 1, 0), tx2c = min(k, tiles_x - 1) (the reference's clamps);
    // the two rows of one column are adjacent, so the blend's two rows run as
    // packed pairs (v_pk_mul_f32 / v_pk_add_f32)
    auto table = [&](int p, int q) {
        const uint32_t* P = lrb + (p & 1) * g.tiles_x * 64;
        const uint32_t* Q = lrb + (q & 1) * g.tiles_x * 64;
        const int items = (g.tiles_x + 1) * 64;
        for (int i = t; i < items; i += nthr) {
            const int k = i >> 6, qd = i & 63;
            const int ta = max(k - 1, 0) * 64 + qd, tb = min(k, g.tiles_x - 1) * 64 + qd;
            const uint32_t a = P[ta], bb = P[tb], c = Q[ta], d = Q[tb];
            // byte j of (a, c, bb, d) -> dword for value 4qd + j: {a_j, c_j, bb_j, d_j}
            const uint32_t ac_lo = __builtin_amdgcn_perm(c, a, 0x05010400u);   // a0 c0 a1 c1
            const uint32_t ac_hi = __builtin_amdgcn_perm(c, a, 0x07030602u);   // a2 c2 a3 c3
            const uint32_t bd_lo = __builtin_amdgcn_perm(d, bb, 0x05010400u);
            const uint32_t bd_hi = __builtin_amdgcn_perm(d, bb, 0x07030602u);
            uint4* o = reinterpret_cast<uint4*>(tab + k * TROW + 4 * qd);
            *o = uint4{__builtin_amdgcn_perm(bd_lo, ac_lo, 0x05040100u), __builtin_amdgcn_perm(bd_lo, ac_lo, 0x07060302u),
                       __builtin_amdgcn_perm(bd_hi, ac_hi, 0x05040100u), __builtin_amdgcn_perm(bd_hi, ac_hi, 0x07060302u)};
        }
    };
    // CLAHE_Interpolation_Body for the rows of tile row k in [ys, ye) held in px
    auto apply = [&](int k, const uint2 (&px)[RMAX], int ys, int ye) {
#pragma unroll
        for (int i = 0; i < RMAX; ++i) {
            const int y = slot_row(k, i);
            if (y < ys || y >= ye) continue;
            const float tyf = (float)y * inv_th - 0.5f;
            const float ya = tyf - floorf(tyf), ya1 = 1.0f - ya;
            const f2 yv = {ya1, ya};
            uint32_t out[2] = {0, 0};
            uint32_t ev[8];  // the 8 gathers first, then the blends
#pragma unroll
            for (int j = 0; j < 8; ++j)
                ev[j] = tab[(kh[j] & 0xffffu) + (((j < 4 ? px[i].x : px[i].y) >> (8 * (j & 3))) & 255u)];
            __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);  // the scheduler keeps the 8 reads together
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float4 e = float4{(float)(ev[j] & 255u), (float)((ev[j] >> 8) & 255u),
                                        (float)((ev[j] >> 16) & 255u), (float)(ev[j] >> 24)};
                // {top, bot} = {L[p][tx1], L[q][tx1]} * xa1 + {L[p][tx2], L[q][tx2]} * xa, then
                // res = top * ya1 + bot * ya: the reference's products and sums, each rounded
                const f2 tb = pk_mul_lo(f2{e.x, e.y}, xw[j]) + pk_mul_hi(f2{e.z, e.w}, xw[j]);
                const f2 u = tb * yv;
                const float res = u.x + u.y;
                out[j >> 2] = __builtin_amdgcn_cvt_pk_u8_f32(res, j & 3, out[j >> 2]);
            }
            uint8_t* drow = dd + (int64_t)y * dst_stride + x0;
            if (fast)
                *reinterpret_cast<uint2*>(drow) = uint2{out[0], out[1]};
            else
                for (int j = 0; j < nv; ++j) drow[j] = (uint8_t)(out[j >> 2] >> (8 * (j & 3)));
        }
    };
    uint2 raw[RMAX][CHAN], prv[RMAX], cur[RMAX];
#pragma unroll
    for (int i = 0; i < RMAX; ++i) prv[i] = cur[i] = uint2{0, 0};
    // prologue: the table of band b0 (LUT rows max(b0-1, 0) and min(b0, tiles_y-1));
    // tile row k enters the image histogram in the segment with b0 <= k < b1
    {
        const int r1 = max(b0 - 1, 0);
        load(r1, raw);
#pragma unroll
        for (int i = 0; i < RMAX; ++i) cur[i] = gray_of(raw[i]);
        build_lut_row(r1, cur, r1 >= b0);
        if (b0 >= 1 && b0 < g.tiles_y) {
#pragma unroll
            for (int i = 0; i < RMAX; ++i) prv[i] = cur[i];
            load(b0, raw);
#pragma unroll
            for (int i = 0; i < RMAX; ++i) cur[i] = gray_of(raw[i]);
            build_lut_row(b0, cur, true);
        } else if (b0 >= 1) {
#pragma unroll
            for (int i = 0; i < RMAX; ++i) prv[i] = cur[i];
        }
        table(r1, min(b0, g.tiles_y - 1));
        __syncthreads();
    }
    for (int b = b0; b < b1; ++b) {
        const bool more = b + 1 < b1;                // band b+1 is this segment's too
        const bool nrow = more && b + 1 < g.tiles_y;  // ... and brings tile row b+1
        if (nrow) load(b + 1, raw);                  // in flight while band b is blended
        const int ys = b == 0 ? 0 : first_row(b - 1, g, inv_th);
        const int ye = b == g.tiles_y ? g.h : first_row(b, g, inv_th);
        if (b >= 1) apply(b - 1, prv, ys, ye);
        if (b < g.tiles_y) apply(b, cur, ys, ye);
        if (!more) break;
#pragma unroll
        for (int i = 0; i < RMAX; ++i) prv[i] = cur[i];
        if (nrow) {
#pragma unroll
            for (int i = 0; i < RMAX; ++i) cur[i] = gray_of(raw[i]);
            build_lut_row(b + 1, cur, true);  // its first barrier also ends band b's table reads
            table(b, b + 1);
        } else {
            __syncthreads();
            table(b, b);  // the last band: ty1 = ty2 = tiles_y - 1
        }
        __syncthreads();
    }
    if (hist_img) {
        __syncthreads();
        for (int b = t; b < 256; b += nthr)
            if (ih[b]) atomicAdd(&hist_img[img * 256 + b], ih[b]);
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

namespace {

// Batches of at least this many images take fused_kernel; smaller calls (the
// live path's single frame, picked on the device by src_index) keep the
// two-kernel form, whose LUT pass spreads one frame over hundreds of workgroups.
constexpr int FUSED_MIN_BATCH = 8;

// fused_kernel's LDS: the fp32 table, the histograms, two LUT rows, the image histogram
size_t fused_lds(const ClaheGeom& g) {
    return (size_t)(g.tiles_x + 1) * TROW * 4 + ((size_t)(g.tiles_x + 1) * HSTR * HCOPY + 2 * g.tiles_x * 64 + 256) * 4;
}

struct FusedPlan {
    int rmax = 0;  // 0: two-kernel path
    int nseg = 1, cpr = 0, nph = 0, threads = 0;
};

FusedPlan clahe_fused_plan(const gvx_ctx* c, int n, const ClaheGeom& g, const uint8_t* src, int64_t img_stride,
                           int stride, int chan, const uint8_t* dst, int64_t dst_img_stride, int dst_stride,
                           const int32_t* src_index, int ring) {
    FusedPlan p;
    if (n < FUSED_MIN_BATCH || src_index || ring) return p;
    // source and destination must not overlap: segment seams re-read rows
    const int r = 0;
    const uintptr_t s0 = (uintptr_t)src, s1 = s0 + (uintptr_t)((n - 1) * img_stride + (int64_t)(g.h - 1) * stride + chan * g.w);
    const uintptr_t d0 = (uintptr_t)dst - (uintptr_t)((int64_t)r * dst_stride + r);
    const uintptr_t d1 = (uintptr_t)dst + (uintptr_t)((n - 1) * dst_img_stride + (int64_t)(g.h - 1 + r) * dst_stride + g.w + r);
    if (s0 < d1 && d0 < s1) return p;
    p.cpr = (g.w + 7) / 8;
    if (p.cpr > 1024 || fused_lds(g) > 160 * 1024) return p;
    p.nph = std::min(1024 / p.cpr, g.th);
    const int rows = (g.th + p.nph - 1) / p.nph;  // row slots per thread and tile row
    if (rows > 8) return p;
    p.rmax = rows <= 2 ? 2 : (rows == 7 ? 8 : rows);  // the instantiated slot counts
    p.threads = (p.nph * p.cpr + 63) / 64 * 64;
    const int nb = g.tiles_y + 1;
    while ((int64_t)n * p.nseg < c->n_cu && p.nseg < nb) ++p.nseg;
    return p;
}

}  // namespace

hipError_t launch_clahe(gvx_ctx* c, int n, const ClaheGeom& g, const uint8_t* src, int64_t img_stride,
                        int stride, uint8_t* dst, int64_t dst_img_stride, int dst_stride, uint8_t* lut,
                        uint32_t* hist_img, double* hist_mean, const int32_t* src_index, int n_src, int ring,
                        int chan, uint8_t* gray) {
    if (n <= 0) return hipSuccess;
    if (chan == 3 && !gray) return hipErrorInvalidValue;
    const int gray_pitch = (g.w + 63) & ~63;
    if (hist_img) {
        hipError_t e = hipMemsetAsync(hist_img, 0, (size_t)n * 256 * sizeof(uint32_t), c->stream);
        if (e != hipSuccess) return e;
    }
    const bool src8 = (uintptr_t)src % 8 == 0 && stride % 8 == 0 && img_stride % 8 == 0;
    const bool dst8 = (uintptr_t)dst % 8 == 0 && dst_stride % 8 == 0 && dst_img_stride % 8 == 0;
    const FusedPlan fp = clahe_fused_plan(c, n, g, src, img_stride, stride, chan, dst, dst_img_stride, dst_stride,
                                          src_index, ring);
    if (fp.rmax) {
        const bool vec8 = src8 && dst8 && g.w % 8 == 0;
        const size_t lds = fused_lds(g);
        const dim3 grid(n * fp.nseg), block(fp.threads);
        auto go = [&](auto k8, auto k1) {
            hipLaunchKernelGGL(vec8 ? k8 : k1, grid, block, lds, c->stream, src, img_stride, stride, dst,
                               dst_img_stride, dst_stride, g, fp.nseg, fp.cpr, fp.nph, hist_img);
        };
        auto pick = [&](auto chan_tag) {
            constexpr int C = decltype(chan_tag)::value;
            switch (fp.rmax) {
                case 2: go(fused_kernel<2, C, true>, fused_kernel<2, C, false>); break;
                case 3: go(fused_kernel<3, C, true>, fused_kernel<3, C, false>); break;
                case 4: go(fused_kernel<4, C, true>, fused_kernel<4, C, false>); break;
                case 5: go(fused_kernel<5, C, true>, fused_kernel<5, C, false>); break;
                case 6: go(fused_kernel<6, C, true>, fused_kernel<6, C, false>); break;
                default: go(fused_kernel<8, C, true>, fused_kernel<8, C, false>); break;
            }
        };
        if (chan == 3)
            pick(std::integral_constant<int, 3>{});
        else
            pick(std::integral_constant<int, 1>{});
        if (hist_img && hist_mean)
            hipLaunchKernelGGL(mean_kernel, dim3((n + 63) / 64), dim3(64), 0, c->stream, (const uint32_t*)hist_img, n,
                               g.w, g.h, hist_mean);
        return hipGetLastError();
    }
    const int lut_vec8 = src8 && g.w % 8 == 0;
    // tiles per workgroup: a whole tile row for batches, fewer for single frames
    int ngrp = 1;
    while ((int64_t)n * g.tiles_y * ngrp < 2LL * c->n_cu && ngrp < g.tiles_x) ++ngrp;
    const int tpw = (g.tiles_x + ngrp - 1) / ngrp;
    ngrp = (g.tiles_x + tpw - 1) / tpw;
    hipLaunchKernelGGL(lut_kernel, dim3(n * g.tiles_y * ngrp), dim3(LUT_THREADS), (size_t)tpw * HROW * 4, c->stream,
                       src, img_stride, stride, g, lut_vec8, tpw, lut, hist_img, src_index, n_src, chan, gray,
                       (int64_t)gray_pitch * g.h, gray_pitch);
    if (chan == 3) {
        // the apply pass reads the gray frames the LUT pass wrote
        src = gray;
        img_stride = (int64_t)gray_pitch * g.h;
        stride = gray_pitch;
        src_index = nullptr;
    }
    const bool asrc8 = (uintptr_t)src % 8 == 0 && stride % 8 == 0 && img_stride % 8 == 0;
    // bands of rows sharing one pair of LUT rows, split to fill the chip
    const int nb = g.tiles_y + 1;
    // workgroups wanted for the apply pass (the sequence replay's single frames
    // measured 17.5 us at 1,024 against 19.9 at 128, r02 v16)
    const int64_t want_wg = 4LL * c->n_cu;
    int nsplit = 1;
    while ((int64_t)n * nb * nsplit < want_wg && nsplit < g.th) nsplit *= 2;
    const int cols = (g.w + PPT - 1) / PPT;
    const int threads = std::min(1024, (cols + 63) / 64 * 64);
    const size_t lds = (size_t)(g.tiles_x + 1) * TROW * 4;
    hipLaunchKernelGGL(apply_kernel, dim3(n * nb * nsplit), dim3(threads), lds, c->stream, src, img_stride, stride,
                       dst, dst_img_stride, dst_stride, g, (const uint8_t*)lut, nsplit, (int)(asrc8 && dst8), src_index,
                       n_src, ring);
    if (hist_img && hist_mean)
        hipLaunchKernelGGL(mean_kernel, dim3((n + 63) / 64), dim3(64), 0, c->stream, (const uint32_t*)hist_img, n,
                           g.w, g.h, hist_mean);
    return hipGetLastError();
}

}  // namespace gvx
