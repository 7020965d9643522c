// pyramid.hip -- image pyramid build for gfx950, replacing the per-call
// buildOpticalFlowPyramid / pyrDown inside each cv::calcOpticalFlowPyrLK of
// /root/reference/ic_gvins/ic_gvins/tracking/tracking.cc:385,390,487,493
// (each image's pyramid is built once here and reused by every LK direction).
//
// Layout (gvx::PyrLayout): level l is stored with a PAD-pixel ring; the
// interior is the exact pyrDown result, the ring replicates OpenCV's
// copyMakeBorder(BORDER_REFLECT_101) padding.
//   level0_kernel  padded copy of the source image, 16 bytes per thread
//                  (16-byte loads/stores in the interior, reflect map in the ring)
//   down_kernel    pyrDown interior: 64x32-output tiles; coalesced dword loads of
//                  the 131x67 input tile into LDS, horizontal [1 4 6 4 1] pass on
//                  8-byte LDS reads into an int16 LDS tile, vertical pass in
//                  registers, one dword store per 4 outputs
//   ring_kernel    the PAD ring of a level, only ring pixels are launched
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

// ------------------------------------------------------------------ level 0
__global__ void __launch_bounds__(256) level0_kernel(const uint8_t* __restrict__ src, int64_t img_stride,
                                                     int stride, int w, int h, int pitch, int64_t pyr_bytes,
                                                     uint8_t* __restrict__ dst) {
    // flat (padded row, 16-byte column group) index over one image
    const int img = blockIdx.y;
    const int groups = (w + 2 * PAD + 15) >> 4;
    const int item = blockIdx.x * 256 + threadIdx.x;
    const int prow = item / groups, q = item - prow * groups;
    if (prow >= h + 2 * PAD) return;
    const int X = q * 16 - PAD;                        // first source column
    const int sy = refl(prow - PAD, h);
    const uint8_t* s = src + img * img_stride + (int64_t)sy * stride;
    uint8_t* d = dst + img * pyr_bytes + (int64_t)prow * pitch + q * 16;
    uint4 v;
    const uintptr_t sa = reinterpret_cast<uintptr_t>(s + X);
    if (X >= 0 && X + 16 <= w && (sa & 15) == 0) {
        v = *reinterpret_cast<const uint4*>(s + X);
    } else {
        uint32_t wv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t acc = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int x = X + 4 * k + b;
                const uint32_t byte = x < w + PAD ? s[refl(x, w)] : 0u;
                acc |= byte << (8 * b);
            }
            wv[k] = acc;
        }
        v = make_uint4(wv[0], wv[1], wv[2], wv[3]);
    }
    *reinterpret_cast<uint4*>(d) = v;
}

// ------------------------------------------------------------------ pyrDown
constexpr int TW = 64, TH = 32;             // output tile
constexpr int IN_ROWS = 2 * TH + 3;         // 67
constexpr int IN_DW = 34;                   // 136 bytes >= 2 + 2*TW + 3
constexpr int HS_STRIDE = TW + 4;           // int16 per hsum row (8-byte aligned rows)

__global__ void __launch_bounds__(256) down_kernel(uint8_t* __restrict__ pyr, int64_t pyr_bytes, int64_t off_src,
                                                   int pitch_src, int h_src, int64_t off_dst, int pitch_dst,
                                                   int w_dst, int h_dst) {
    __shared__ uint32_t tile[IN_ROWS * IN_DW];
    __shared__ short hs[IN_ROWS * HS_STRIDE];
    const int img = blockIdx.z;
    uint8_t* base = pyr + img * pyr_bytes;
    const int x0 = blockIdx.x * TW, y0 = blockIdx.y * TH;
    // input pixels X in [2*x0-2, 2*x0+2*TW+1), Y in [2*y0-2, 2*y0+2*TH+1); the
    // byte column of X = 2*x0-2 is 2*x0+PAD-2 = 2 (mod 4): load from 2 earlier.
    const int col0 = 2 * x0 + PAD - 4;   // dword aligned
    const int row0 = 2 * y0 - 2 + PAD;   // padded row of the first input row
    const int last_row = h_src + 2 * PAD - 1;
    const uint8_t* src = base + off_src;
    for (int i = threadIdx.x; i < IN_ROWS * IN_DW; i += 256) {
        const int r = i / IN_DW, c = i - r * IN_DW;
        const int prow = row0 + r, pcol = col0 + 4 * c;
        uint32_t v = 0;
        if (prow <= last_row && pcol + 4 <= pitch_src)
            v = *reinterpret_cast<const uint32_t*>(src + (int64_t)prow * pitch_src + pcol);
        tile[i] = v;
    }
    __syncthreads();
    // horizontal pass: item = (row r, group g of 4 output columns)
    for (int i = threadIdx.x; i < IN_ROWS * (TW / 4); i += 256) {
        const int r = i / (TW / 4), g = i - r * (TW / 4);
        // input bytes for outputs 4g..4g+3 start at tile byte 2 + 8g: read dwords 2g..2g+3
        const uint2 lo = *reinterpret_cast<const uint2*>(&tile[r * IN_DW + 2 * g]);
        const uint2 hi = *reinterpret_cast<const uint2*>(&tile[r * IN_DW + 2 * g + 2]);
        const uint32_t d0 = __builtin_amdgcn_alignbyte(lo.y, lo.x, 2);
        const uint32_t d1 = __builtin_amdgcn_alignbyte(hi.x, lo.y, 2);
        const uint32_t d2 = __builtin_amdgcn_alignbyte(hi.y, hi.x, 2);
        int p[12];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            p[k] = (d0 >> (8 * k)) & 255;
            p[4 + k] = (d1 >> (8 * k)) & 255;
            p[8 + k] = (d2 >> (8 * k)) & 255;
        }
        short o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = (short)(p[2 * k] + 4 * p[2 * k + 1] + 6 * p[2 * k + 2] + 4 * p[2 * k + 3] + p[2 * k + 4]);
        uint2 packed;
        packed.x = (uint32_t)(uint16_t)o[0] | ((uint32_t)(uint16_t)o[1] << 16);
        packed.y = (uint32_t)(uint16_t)o[2] | ((uint32_t)(uint16_t)o[3] << 16);
        *reinterpret_cast<uint2*>(&hs[r * HS_STRIDE + 4 * g]) = packed;
    }
    __syncthreads();
    // vertical pass: thread = (row pair rp, group g); 16 row pairs x 16 groups
    {
        const int g = threadIdx.x & 15, rp = threadIdx.x >> 4;
        const int y = y0 + 2 * rp;
        int v[7][4];
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const uint2 u = *reinterpret_cast<const uint2*>(&hs[(4 * rp + k) * HS_STRIDE + 4 * g]);
            v[k][0] = (short)(u.x & 0xffff);
            v[k][1] = (short)(u.x >> 16);
            v[k][2] = (short)(u.y & 0xffff);
            v[k][3] = (short)(u.y >> 16);
        }
        const int x = x0 + 4 * g;
        if (x < w_dst) {
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                if (y + rr >= h_dst) break;
                uint32_t out = 0;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int s = v[2 * rr][k] + 4 * v[2 * rr + 1][k] + 6 * v[2 * rr + 2][k] +
                                  4 * v[2 * rr + 3][k] + v[2 * rr + 4][k];
                    out |= (uint32_t)((s + 128) >> 8) << (8 * k);
                }
                // bytes past w_dst land in the ring, which ring_kernel rewrites
                *reinterpret_cast<uint32_t*>(base + off_dst + (int64_t)(y + rr + PAD) * pitch_dst + x + PAD) = out;
            }
        }
    }
}

// ------------------------------------------------------------------ ring
// Ring pixels only: the top/bottom PAD rows over the full padded width, plus the
// left/right PAD columns of the interior rows.
__global__ void __launch_bounds__(256) ring_kernel(uint8_t* __restrict__ pyr, int64_t pyr_bytes, int64_t off,
                                                   int pitch, int w, int h) {
    const int img = blockIdx.y;
    uint8_t* base = pyr + img * pyr_bytes + off;
    const int wp = w + 2 * PAD;
    const int n_band = 2 * PAD * wp;      // top + bottom bands
    const int n_side = h * 2 * PAD;       // side bands of interior rows
    const int i = blockIdx.x * 256 + threadIdx.x;
    int x, y;
    if (i < n_band) {
        const int r = i / wp, c = i - r * wp;
        y = r < PAD ? r - PAD : h + (r - PAD);
        x = c - PAD;
    } else if (i < n_band + n_side) {
        const int j = i - n_band;
        const int r = j / (2 * PAD), c = j - r * (2 * PAD);
        y = r;
        x = c < PAD ? c - PAD : w + (c - PAD);
    } else {
        return;
    }
    const int sy = refl(y, h), sx = refl(x, w);
    base[(int64_t)(y + PAD) * pitch + x + PAD] = base[(int64_t)(sy + PAD) * pitch + sx + PAD];
}

}  // namespace

PyrLayout make_layout(int w, int h, int max_level, int win) {
    PyrLayout L{};
    int64_t off = 0;
    int sw = w, sh = h;
    L.nlev = 0;
    for (int level = 0; level <= max_level && level < MAX_LEVELS; ++level) {
        L.w[level] = sw;
        L.h[level] = sh;
        L.pitch[level] = ((sw + 2 * PAD) + 63) / 64 * 64;
        L.off[level] = off;
        off += (int64_t)L.pitch[level] * (sh + 2 * PAD);
        off = (off + 255) / 256 * 256;
        L.nlev = level + 1;
        // buildOpticalFlowPyramid stops when the next level would be <= winSize
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= win || sh <= win) break;
    }
    L.bytes = off;
    return L;
}

hipError_t launch_build_pyramids(gvx_ctx* c, const uint8_t* src, int64_t img_stride, int stride, int n_img,
                                 const PyrLayout& lay, uint8_t* dst) {
    if (n_img <= 0) return hipSuccess;
    {
        const int groups = (lay.w[0] + 2 * PAD + 15) / 16;
        const int items = groups * (lay.h[0] + 2 * PAD);
        dim3 grid((items + 255) / 256, n_img);
        hipLaunchKernelGGL(level0_kernel, grid, dim3(256), 0, c->stream, src, img_stride, stride, lay.w[0],
                           lay.h[0], lay.pitch[0], lay.bytes, dst);
    }
    for (int l = 1; l < lay.nlev; ++l) {
        dim3 g1((lay.w[l] + TW - 1) / TW, (lay.h[l] + TH - 1) / TH, n_img);
        hipLaunchKernelGGL(down_kernel, g1, dim3(256), 0, c->stream, dst, lay.bytes, lay.off[l - 1],
                           lay.pitch[l - 1], lay.h[l - 1], lay.off[l], lay.pitch[l], lay.w[l], lay.h[l]);
        const int n_ring = 2 * PAD * (lay.w[l] + 2 * PAD) + lay.h[l] * 2 * PAD;
        dim3 g2((n_ring + 255) / 256, n_img);
        hipLaunchKernelGGL(ring_kernel, g2, dim3(256), 0, c->stream, dst, lay.bytes, lay.off[l], lay.pitch[l],
                           lay.w[l], lay.h[l]);
    }
    return hipGetLastError();
}

}  // namespace gvx
