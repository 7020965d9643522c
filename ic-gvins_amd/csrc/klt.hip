// klt.hip -- pyramid build, pyramidal LK (fwd / fwd+bwd+FB) and compaction
// kernels for gfx950.  Replaces the four cv::calcOpticalFlowPyrLK calls per
// frame at /root/reference/ic_gvins/ic_gvins/tracking/tracking.cc:385,390,487,493
// and the status/reduceVector logic at tracking.cc:396-408, :831-849.
//
// Design (DESIGN.md "KLT"):
//  * pyramids are built once per image into a padded layout (gvx::PAD ring,
//    BORDER_REFLECT_101) -- the reference rebuilds them in each of its 4 calls;
//  * the Scharr derivative planes are never materialised: each LK wavefront
//    computes the derivative of its 22x22 window from the padded pyramid in
//    registers (zero outside the image, as OpenCV's BORDER_CONSTANT deriv pad);
//  * one 64-lane wavefront per point; lane = 3*row + segment owns 7 consecutive
//    window pixels of one of the 21 rows, loaded as aligned dwords and realigned
//    with v_alignbyte; window sums are exact integer wave reductions, so the
//    fp32 2x2 solve sees bit-identical inputs to the CPU restatement.
#include <hip/hip_runtime.h>

#include "gvx_internal.h"

namespace gvx {

namespace {

__device__ __forceinline__ int reflect101(int p, int len) {
    if ((unsigned)p < (unsigned)len) return p;
    if (len == 1) return 0;
    do {
        p = p < 0 ? -p : 2 * len - 2 - p;
    } while ((unsigned)p >= (unsigned)len);
    return p;
}

// ----------------------------------------------------------------- pyramid

// Level 0: padded copy of the source image (copyMakeBorder REFLECT_101).
// One thread per output dword; the source is read through the reflect map.
__global__ void __launch_bounds__(256) pyr_level0_kernel(const uint8_t* __restrict__ src,
                                                         int64_t img_stride, int stride, int w,
                                                         int h, int pitch, int64_t pyr_bytes,
                                                         uint8_t* __restrict__ dst) {
    const int img = blockIdx.z;
    const int row = blockIdx.y;           // padded row 0 .. h+2P-1
    const int dw = blockIdx.x * 256 + threadIdx.x;  // dword column
    const int x0 = dw * 4 - PAD;
    if (dw * 4 >= w + 2 * PAD) return;
    const int y = reflect101(row - PAD, h);
    const uint8_t* s = src + img * img_stride + (int64_t)y * stride;
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int x = x0 + k;
        uint32_t b = (x < w + PAD) ? s[reflect101(x, w)] : 0u;
        v |= b << (8 * k);
    }
    uint8_t* d = dst + img * pyr_bytes + (int64_t)row * pitch + dw * 4;
    *reinterpret_cast<uint32_t*>(d) = v;
}

// pyrDown interior of level l+1 from padded level l (pyramids.cpp pyrDown_):
// out(y,x) = (sum k_i k_j in(2y+i-2, 2x+j-2) + 128) >> 8, k = [1 4 6 4 1].
// LDS tile: 16 output rows x 64 output cols <- 35 x 131 input bytes.
constexpr int PD_TW = 64, PD_TH = 16;
constexpr int PD_IN_ROWS = 2 * PD_TH + 3;     // 35
constexpr int PD_IN_DW = (2 * PD_TW + 3 + 3 + 3) / 4 + 1;  // dwords per input row (36)

__global__ void __launch_bounds__(256) pyr_down_kernel(uint8_t* __restrict__ pyr, int64_t pyr_bytes,
                                                       int64_t off_src, int pitch_src, int w_src,
                                                       int h_src, int64_t off_dst, int pitch_dst,
                                                       int w_dst, int h_dst) {
    __shared__ uint32_t tile[PD_IN_ROWS][PD_IN_DW];
    __shared__ int hsum[PD_IN_ROWS][PD_TW + 1];
    const int img = blockIdx.z;
    uint8_t* base = pyr + img * pyr_bytes;
    const int x0 = blockIdx.x * PD_TW, y0 = blockIdx.y * PD_TH;
    // input region: X in [2*x0-2, 2*x0+2*PD_TW+1), Y in [2*y0-2, 2*y0+2*PD_TH+1)
    const int64_t row0 = off_src + (int64_t)(2 * y0 - 2 + PAD) * pitch_src;
    const int xb = 2 * x0 - 2 + PAD;   // byte column of the first input pixel
    const int xa = xb & ~3, sh = xb - xa;
    const int max_y = h_src + PAD - 1 + PAD;  // last valid padded row index (inclusive)
    for (int i = threadIdx.x; i < PD_IN_ROWS * PD_IN_DW; i += 256) {
        int r = i / PD_IN_DW, c = i - r * PD_IN_DW;
        int prow = 2 * y0 - 2 + PAD + r;
        int pcol = xa + 4 * c;
        uint32_t v = 0;
        if (prow <= max_y && pcol + 3 < pitch_src)
            v = *reinterpret_cast<const uint32_t*>(base + row0 + (int64_t)r * pitch_src + pcol);
        tile[r][c] = v;
    }
    __syncthreads();
    const uint8_t* tb = reinterpret_cast<const uint8_t*>(&tile[0][0]);
    // horizontal pass
    for (int i = threadIdx.x; i < PD_IN_ROWS * PD_TW; i += 256) {
        int r = i / PD_TW, c = i - r * PD_TW;
        const uint8_t* p = tb + r * (PD_IN_DW * 4) + sh + 2 * c;
        hsum[r][c] = (int)p[0] + 4 * (int)p[1] + 6 * (int)p[2] + 4 * (int)p[3] + (int)p[4];
    }
    __syncthreads();
    // vertical pass + store
    for (int i = threadIdx.x; i < PD_TH * PD_TW; i += 256) {
        int r = i / PD_TW, c = i - r * PD_TW;
        int x = x0 + c, y = y0 + r;
        if (x >= w_dst || y >= h_dst) continue;
        int s = hsum[2 * r][c] + 4 * hsum[2 * r + 1][c] + 6 * hsum[2 * r + 2][c] +
                4 * hsum[2 * r + 3][c] + hsum[2 * r + 4][c];
        base[off_dst + (int64_t)(y + PAD) * pitch_dst + x + PAD] = (uint8_t)((s + 128) >> 8);
    }
}

// Fill the PAD ring of a level from its interior (copyMakeBorder REFLECT_101).
__global__ void __launch_bounds__(256) pyr_ring_kernel(uint8_t* __restrict__ pyr, int64_t pyr_bytes,
                                                       int64_t off, int pitch, int w, int h) {
    const int img = blockIdx.z;
    const int prow = blockIdx.y;  // 0 .. h+2P-1
    const int y = prow - PAD;
    const int x = blockIdx.x * 256 + threadIdx.x - PAD;
    if (x >= w + PAD) return;
    const bool inside_row = (unsigned)y < (unsigned)h;
    if (inside_row && (unsigned)x < (unsigned)w) return;
    uint8_t* base = pyr + img * pyr_bytes + off;
    const int sy = reflect101(y, h), sx = reflect101(x, w);
    base[(int64_t)prow * pitch + x + PAD] = base[(int64_t)(sy + PAD) * pitch + sx + PAD];
}

// ----------------------------------------------------------------- LK

constexpr int W_BITS = 14;
constexpr float FLT_SCALE = 1.f / (1 << 20);

__device__ __forceinline__ int descale(int x, int n) { return (x + (1 << (n - 1))) >> n; }

__device__ __forceinline__ long long wave_sum(long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Load 16 bytes around p from dword-aligned addresses and realign so that the
// returned d[k] holds bytes p[4k .. 4k+3].
template <int NDW>
__device__ __forceinline__ void load_aligned(const uint8_t* p, uint32_t (&d)[NDW]) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t w[NDW + 1];
#pragma unroll
    for (int k = 0; k <= NDW; ++k) w[k] = q[k];
#pragma unroll
    for (int k = 0; k < NDW; ++k) d[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
}

template <int NDW>
__device__ __forceinline__ int byte_at(const uint32_t (&d)[NDW], int c) {
    return (int)((d[c >> 2] >> (8 * (c & 3))) & 0xffu);
}

__device__ __forceinline__ void bilinear_weights(float a, float b, int& w00, int& w01, int& w10,
                                                 int& w11) {
    w00 = __float2int_rn((1.f - a) * (1.f - b) * (float)(1 << W_BITS));
    w01 = __float2int_rn(a * (1.f - b) * (float)(1 << W_BITS));
    w10 = __float2int_rn((1.f - a) * b * (float)(1 << W_BITS));
    w11 = (1 << W_BITS) - w00 - w01 - w10;
}

struct LkCfg {
    int max_iter;
    double crit_eps;
    float min_eig;
    int use_initial_flow;
};

// LKTrackerInvoker::operator() for one point across all levels (coarse to fine),
// executed by one wavefront.  I/J are the padded pyramids of prev/next image.
__device__ void lk_point(const uint8_t* __restrict__ I, const uint8_t* __restrict__ J,
                         const PyrLayout& lay, const LkCfg& cfg, float p0x, float p0y, float& nx,
                         float& ny, int& status, float& err, int lane) {
    const bool valid = lane < 63;
    const int wy = valid ? lane / 3 : 20;   // window row owned by this lane
    const int ws = valid ? lane - 3 * (lane / 3) : 2;  // 7-pixel segment
    const float halfw = (float)((WIN - 1) * 0.5f);
    const int max_level = lay.nlev - 1;
    status = 1;
    err = 0.f;
    for (int l = max_level; l >= 0; --l) {
        const int W = lay.w[l], H = lay.h[l], pitch = lay.pitch[l];
        const uint8_t* Il = I + lay.off[l] + (int64_t)PAD * pitch + PAD;  // (0,0)
        const uint8_t* Jl = J + lay.off[l] + (int64_t)PAD * pitch + PAD;
        const float sc = (float)(1. / (1 << l));
        float prevx = p0x * sc, prevy = p0y * sc;
        float nextx, nexty;
        if (l == max_level) {
            if (cfg.use_initial_flow) {
                nextx = nx * sc;
                nexty = ny * sc;
            } else {
                nextx = prevx;
                nexty = prevy;
            }
        } else {
            nextx = nx * 2.f;
            nexty = ny * 2.f;
        }
        nx = nextx;
        ny = nexty;
        prevx -= halfw;
        prevy -= halfw;
        const int ipx = (int)floorf(prevx), ipy = (int)floorf(prevy);
        if (ipx < -WIN || ipx >= W || ipy < -WIN || ipy >= H) {
            if (l == 0) {
                status = 0;
                err = 0.f;
            }
            continue;
        }
        int iw00, iw01, iw10, iw11;
        bilinear_weights(prevx - ipx, prevy - ipy, iw00, iw01, iw10, iw11);

        // ---- window of I and its Scharr derivative (rows wy-1 .. wy+2) ----
        int P[4][10];
        {
            const int X = ipx + 7 * ws - 1;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                uint32_t d[3];
                load_aligned<3>(Il + (int64_t)(ipy + wy - 1 + r) * pitch + X, d);
#pragma unroll
                for (int c = 0; c < 10; ++c) P[r][c] = byte_at<3>(d, c);
            }
        }
        int Iv[7], Ix[7], Iy[7];
        int dxv[2][8], dyv[2][8];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const int r = rr + 1;
            const int Yd = ipy + wy + rr;
            const bool row_in = (unsigned)Yd < (unsigned)H;
            int t0[10], t1[10];
#pragma unroll
            for (int c = 0; c < 10; ++c) {
                t0[c] = (P[r - 1][c] + P[r + 1][c]) * 3 + P[r][c] * 10;
                t1[c] = P[r + 1][c] - P[r - 1][c];
            }
#pragma unroll
            for (int c = 1; c <= 8; ++c) {
                const int Xd = ipx + 7 * ws + c - 1;
                const bool in = row_in && (unsigned)Xd < (unsigned)W;
                dxv[rr][c - 1] = in ? (t0[c + 1] - t0[c - 1]) : 0;
                dyv[rr][c - 1] = in ? ((t1[c + 1] + t1[c - 1]) * 3 + t1[c] * 10) : 0;
            }
        }
        int a11 = 0, a12 = 0, a22 = 0;
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            Iv[t] = descale(P[1][t + 1] * iw00 + P[1][t + 2] * iw01 + P[2][t + 1] * iw10 +
                                P[2][t + 2] * iw11,
                            W_BITS - 5);
            Ix[t] = descale(dxv[0][t] * iw00 + dxv[0][t + 1] * iw01 + dxv[1][t] * iw10 +
                                dxv[1][t + 1] * iw11,
                            W_BITS);
            Iy[t] = descale(dyv[0][t] * iw00 + dyv[0][t + 1] * iw01 + dyv[1][t] * iw10 +
                                dyv[1][t + 1] * iw11,
                            W_BITS);
            a11 += Ix[t] * Ix[t];
            a12 += Ix[t] * Iy[t];
            a22 += Iy[t] * Iy[t];
        }
        if (!valid) a11 = a12 = a22 = 0;
        const long long iA11 = wave_sum((long long)a11);
        const long long iA12 = wave_sum((long long)a12);
        const long long iA22 = wave_sum((long long)a22);
        const float A11 = (float)iA11 * FLT_SCALE;
        const float A12 = (float)iA12 * FLT_SCALE;
        const float A22 = (float)iA22 * FLT_SCALE;
        float D = A11 * A22 - A12 * A12;
        const float minEig =
            __fdiv_rn(A22 + A11 - __fsqrt_rn((A11 - A22) * (A11 - A22) + 4.f * A12 * A12),
                      (float)(2 * WIN * WIN));
        if (minEig < cfg.min_eig || D < __FLT_EPSILON__) {
            if (l == 0) {
                status = 0;
                err = 0.f;
            }
            continue;
        }
        D = __fdiv_rn(1.f, D);

        nextx -= halfw;
        nexty -= halfw;
        float pdx = 0.f, pdy = 0.f;
        for (int j = 0; j < cfg.max_iter; ++j) {
            const int inx = (int)floorf(nextx), iny = (int)floorf(nexty);
            if (inx < -WIN || inx >= W || iny < -WIN || iny >= H) {
                if (l == 0) status = 0;
                break;
            }
            int jw00, jw01, jw10, jw11;
            bilinear_weights(nextx - inx, nexty - iny, jw00, jw01, jw10, jw11);
            const uint8_t* jp = Jl + (int64_t)(iny + wy) * pitch + inx + 7 * ws;
            uint32_t d0[2], d1[2];
            load_aligned<2>(jp, d0);
            load_aligned<2>(jp + pitch, d1);
            int b1 = 0, b2 = 0;
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                const int jv = descale(byte_at<2>(d0, t) * jw00 + byte_at<2>(d0, t + 1) * jw01 +
                                           byte_at<2>(d1, t) * jw10 + byte_at<2>(d1, t + 1) * jw11,
                                       W_BITS - 5);
                const int diff = jv - Iv[t];
                b1 += diff * Ix[t];
                b2 += diff * Iy[t];
            }
            if (!valid) b1 = b2 = 0;
            const float fb1 = (float)wave_sum((long long)b1) * FLT_SCALE;
            const float fb2 = (float)wave_sum((long long)b2) * FLT_SCALE;
            const float dx = (A12 * fb2 - A22 * fb1) * D;
            const float dy = (A12 * fb1 - A11 * fb2) * D;
            nextx += dx;
            nexty += dy;
            nx = nextx + halfw;
            ny = nexty + halfw;
            if ((double)dx * (double)dx + (double)dy * (double)dy <= cfg.crit_eps) break;
            if (j > 0 && fabsf(dx + pdx) < 0.01f && fabsf(dy + pdy) < 0.01f) {
                nx -= dx * 0.5f;
                ny -= dy * 0.5f;
                break;
            }
            pdx = dx;
            pdy = dy;
        }
        if (status && l == 0) {
            const float ex = nx - halfw, ey = ny - halfw;
            const int inx = (int)floorf(ex), iny = (int)floorf(ey);
            if (inx < -WIN || inx >= W || iny < -WIN || iny >= H) {
                status = 0;
                continue;
            }
            int jw00, jw01, jw10, jw11;
            bilinear_weights(ex - inx, ey - iny, jw00, jw01, jw10, jw11);
            const uint8_t* jp = Jl + (int64_t)(iny + wy) * pitch + inx + 7 * ws;
            uint32_t d0[2], d1[2];
            load_aligned<2>(jp, d0);
            load_aligned<2>(jp + pitch, d1);
            int es = 0;
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                const int jv = descale(byte_at<2>(d0, t) * jw00 + byte_at<2>(d0, t + 1) * jw01 +
                                           byte_at<2>(d1, t) * jw10 + byte_at<2>(d1, t + 1) * jw11,
                                       W_BITS - 5);
                const int diff = jv - Iv[t];
                es += diff < 0 ? -diff : diff;
            }
            if (!valid) es = 0;
            err = __fdiv_rn((float)wave_sum_i(es) * 1.f, (float)(32 * WIN * WIN));
        }
    }
}

__global__ void __launch_bounds__(256) klt_kernel(KltArgs a, PyrLayout lay,
                                                  const uint8_t* __restrict__ pyr_prev,
                                                  const uint8_t* __restrict__ pyr_next,
                                                  int64_t prev_stride, int64_t next_stride,
                                                  const float* __restrict__ prev_xy,
                                                  float* __restrict__ next_xy,
                                                  float* __restrict__ back_xy,
                                                  uint8_t* __restrict__ flags,
                                                  float* __restrict__ err_out) {
    const int lane = threadIdx.x & 63;
    const int64_t gp = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t total = (int64_t)a.n_pairs * a.n_pts;
    if (gp >= total) return;
    const int64_t pair = gp / a.n_pts;
    const uint8_t* I = pyr_prev + pair * prev_stride;
    const uint8_t* J = pyr_next + pair * next_stride;
    LkCfg cfg{a.max_iter, a.crit_eps, a.min_eig, a.use_initial_flow};
    const float p0x = prev_xy[2 * gp], p0y = prev_xy[2 * gp + 1];
    float nx = next_xy[2 * gp], ny = next_xy[2 * gp + 1];
    int st = 1;
    float e = 0.f;
    lk_point(I, J, lay, cfg, p0x, p0y, nx, ny, st, e, lane);
    if (a.mode == 0) {
        if (lane == 0) {
            next_xy[2 * gp] = nx;
            next_xy[2 * gp + 1] = ny;
            flags[gp] = (uint8_t)st;
            if (err_out) err_out[gp] = e;
        }
        return;
    }
    // backward: prevPts = forward result, initial flow = original prev points
    float bx = p0x, by = p0y;
    int st2 = 1;
    float e2 = 0.f;
    cfg.use_initial_flow = 1;
    lk_point(J, I, lay, cfg, nx, ny, bx, by, st2, e2, lane);
    if (lane == 0) {
        const double B = a.border;
        const bool on_border = nx < B || ny < B || nx > (a.cam_w - B) || ny > (a.cam_h - B);
        const double ddx = (double)(bx - p0x), ddy = (double)(by - p0y);
        const double dist = __dsqrt_rn(ddx * ddx + ddy * ddy);
        const bool keep = st && st2 && !on_border && dist < a.fb_thresh;
        next_xy[2 * gp] = nx;
        next_xy[2 * gp + 1] = ny;
        if (back_xy) {
            back_xy[2 * gp] = bx;
            back_xy[2 * gp + 1] = by;
        }
        flags[gp] = (uint8_t)((st ? 1 : 0) | (st2 ? 2 : 0) | (keep ? 4 : 0));
        if (err_out) err_out[gp] = e;
    }
}

// reduceVector (tracking.cc:831-839): order-preserving index compaction of the
// keep bit, one workgroup per pair.
__global__ void __launch_bounds__(256) compact_kernel(int n_pts, const uint8_t* __restrict__ flags,
                                                      int32_t* __restrict__ kept_idx,
                                                      int32_t* __restrict__ n_kept) {
    __shared__ int wsum[4];
    const int pair = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint8_t* f = flags + (int64_t)pair * n_pts;
    int32_t* out = kept_idx + (int64_t)pair * n_pts;
    int base = 0;
    for (int start = 0; start < n_pts; start += 256) {
        const int i = start + tid;
        const bool k = i < n_pts && (f[i] & 4);
        const unsigned long long m = __ballot(k);
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wv] = __popcll(m);
        __syncthreads();
        int off = base;
        for (int q = 0; q < wv; ++q) off += wsum[q];
        if (k) out[off + before] = i;
        const int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
        base += tot;
    }
    if (tid == 0) n_kept[pair] = base;
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
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= win || sh <= win) break;
    }
    L.bytes = off;
    return L;
}

hipError_t launch_build_pyramids(gvx_ctx* c, const uint8_t* src, int64_t img_stride, int stride,
                                 int n_img, const PyrLayout& lay, uint8_t* dst) {
    if (n_img <= 0) return hipSuccess;
    {
        dim3 grid((lay.w[0] + 2 * PAD + 1023) / 1024, lay.h[0] + 2 * PAD, n_img);
        hipLaunchKernelGGL(pyr_level0_kernel, grid, dim3(256), 0, c->stream, src, img_stride, stride,
                           lay.w[0], lay.h[0], lay.pitch[0], lay.bytes, dst);
    }
    for (int l = 1; l < lay.nlev; ++l) {
        dim3 g1((lay.w[l] + PD_TW - 1) / PD_TW, (lay.h[l] + PD_TH - 1) / PD_TH, n_img);
        hipLaunchKernelGGL(pyr_down_kernel, g1, dim3(256), 0, c->stream, dst, lay.bytes,
                           lay.off[l - 1], lay.pitch[l - 1], lay.w[l - 1], lay.h[l - 1], lay.off[l],
                           lay.pitch[l], lay.w[l], lay.h[l]);
        dim3 g2((lay.w[l] + 2 * PAD + 255) / 256, lay.h[l] + 2 * PAD, n_img);
        hipLaunchKernelGGL(pyr_ring_kernel, g2, dim3(256), 0, c->stream, dst, lay.bytes, lay.off[l],
                           lay.pitch[l], lay.w[l], lay.h[l]);
    }
    return hipGetLastError();
}

hipError_t launch_klt(gvx_ctx* c, const KltArgs& a, const PyrLayout& lay, const uint8_t* pyr_prev,
                      const uint8_t* pyr_next, int64_t prev_pair_stride, int64_t next_pair_stride,
                      const float* prev_xy, float* next_xy, float* back_xy, uint8_t* flags,
                      float* err) {
    const int64_t total = (int64_t)a.n_pairs * a.n_pts;
    if (total <= 0) return hipSuccess;
    dim3 grid((unsigned)((total + 3) / 4));
    hipLaunchKernelGGL(klt_kernel, grid, dim3(256), 0, c->stream, a, lay, pyr_prev, pyr_next,
                       prev_pair_stride, next_pair_stride, prev_xy, next_xy, back_xy, flags, err);
    return hipGetLastError();
}

hipError_t launch_compact(gvx_ctx* c, int n_pairs, int n_pts, const uint8_t* flags, int32_t* kept_idx,
                          int32_t* n_kept) {
    if (n_pairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(compact_kernel, dim3(n_pairs), dim3(256), 0, c->stream, n_pts, flags, kept_idx,
                       n_kept);
    return hipGetLastError();
}

}  // namespace gvx
