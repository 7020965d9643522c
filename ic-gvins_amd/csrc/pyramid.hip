// pyramid.hip -- image pyramid build for gfx950, replacing the per-call
// buildOpticalFlowPyramid / pyrDown inside each cv::calcOpticalFlowPyrLK of
// /root/reference/ic_gvins/ic_gvins/tracking/tracking.cc:385,390,487,493
// (each image's pyramid is built once here and reused by every LK direction).
//
// Layout (gvx::PyrLayout): level l >= 1 is stored with a PAD-pixel ring; the
// interior is the exact pyrDown result ((sum of [1 4 6 4 1]^T[1 4 6 4 1] + 128)
// >> 8 over the REFLECT_101-extended source), the ring replicates OpenCV's
// copyMakeBorder(BORDER_REFLECT_101) padding.  Level 0 is either read in place
// from the caller's image (batched path; the LK kernel handles its border) or
// copied into the padded slot of the layout (frame cache, whose detection pass
// reads across ROI edges).
//
//   level0_kernel   padded copy of level 0 (frame cache only)
//   edge_kernel     REFLECT_101 edge bands of level 0 (batched path)
//   stream_kernel<NL> NL pyrDown levels in one streaming pass per band
//   ring_kernel     the PAD rings of all built levels >= 1, one launch
#include <hip/hip_runtime.h>

#include <type_traits>

#include "gvx_internal.h"

namespace gvx {

namespace {

// BORDER_REFLECT_101 index, branchless: exact for -(2*len-2) <= p <= 3*len-3
// (two bounces), which covers every position these kernels read (halo and ring
// overshoot <= 32 < 2*len-2 since levels are > 21 px); the final clamp keeps
// addresses of unused positions in range.
__device__ __forceinline__ int refl(int p, int len) {
    int a = abs(p);
    a = min(a, 2 * len - 2 - a);
    a = abs(a);
    return min(a, len - 1);
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
    const int X = q * 16 - PAD;  // first source column
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

// ------------------------------------------------------------ pyrDown helpers
struct DownLevels {
    int64_t off[3];  // padded-level offsets (bytes) inside one pyramid
    int32_t pitch[3], w[3], h[3];
};

// Horizontal [1 4 6 4 1] taps of one source row into four u16 outputs: outputs
// 4g..4g+3 read source bytes 8g .. 8g+10 of the row (`sh` = byte shift of the row
// start inside its first dword, 0 or 2).
template <int SH>
__device__ __forceinline__ uint2 hsum4(const uint32_t* row, int g) {
    const uint32_t* p = row + 2 * g;
    const uint32_t w0 = p[0], w1 = p[1], w2 = p[2];
    uint32_t d0, d1, d2;
    if (SH == 0) {
        d0 = w0;
        d1 = w1;
        d2 = w2;
    } else {
        const uint32_t w3 = p[3];
        d0 = __builtin_amdgcn_alignbyte(w1, w0, SH);
        d1 = __builtin_amdgcn_alignbyte(w2, w1, SH);
        d2 = __builtin_amdgcn_alignbyte(w3, w2, SH);
    }
    constexpr uint32_t K = 0x04060401u;  // taps 1 4 6 4 on bytes 0..3
    const uint32_t e1 = __builtin_amdgcn_alignbyte(d1, d0, 2), e3 = __builtin_amdgcn_alignbyte(d2, d1, 2);
    const uint32_t o0 = __builtin_amdgcn_udot4(d0, K, d1 & 0xffu, false);
    const uint32_t o1 = __builtin_amdgcn_udot4(e1, K, (d1 >> 16) & 0xffu, false);
    const uint32_t o2 = __builtin_amdgcn_udot4(d1, K, d2 & 0xffu, false);
    const uint32_t o3 = __builtin_amdgcn_udot4(e3, K, (d2 >> 16) & 0xffu, false);
    return make_uint2(o0 | (o1 << 16), o2 | (o3 << 16));
}

// Vertical taps on packed u16 pairs: (a + 4b + 6c + 4d + e + 128) per half.
// Every partial sum stays < 2^16 (inputs <= 4080, result <= 65408), so the two
// halves never interact.
__device__ __forceinline__ uint32_t vsum2(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e) {
    typedef unsigned short v2u __attribute__((ext_vector_type(2)));
    const v2u A = __builtin_bit_cast(v2u, a), B = __builtin_bit_cast(v2u, b), C = __builtin_bit_cast(v2u, c),
              D = __builtin_bit_cast(v2u, d), E = __builtin_bit_cast(v2u, e);
    const v2u r = A + E + (B + D) * (unsigned short)4 + C * (unsigned short)6 + (unsigned short)128;
    return __builtin_bit_cast(uint32_t, r);
}
// high bytes of the four u16 lanes of (lo, hi) = the (s + 128) >> 8 results
__device__ __forceinline__ uint32_t hibytes(uint32_t lo, uint32_t hi) {
    return __builtin_amdgcn_perm(hi, lo, 0x07050301u);
}


// ------------------------------------------------------- streaming pyrDown
// Row-streaming build of NL levels (the production path).  One wavefront owns
// a column strip of the source level and a band of rows, and walks the rows
// with rolling registers: no LDS, no barriers.
//   lane L loads 16 source bytes per row at x0 = 480*strip + 8L - 20 and makes
//   the four level-1 outputs at columns 240*strip + 4(L-2) + {0..3} (horizontal
//   [1 4 6 4 1] on v_dot4_u32_u8, vertical on packed u16);
//   level 2 (two outputs per lane) and level 3 (one) take their horizontal
//   neighbours from lanes L-1 / L+1 with DPP wave shifts, so valid results
//   shrink by one lane per level and lanes 2..61 own the strip (480 source
//   columns per strip, 7 % overlap).
// Band b owns level-1 rows [BAND*b, BAND*(b+1)) (level k: the same >> (k-1)).
// Borders: source rows / columns are REFLECT_101-extended at load.  Because the
// filter is symmetric, the extension of a level computed from an extended
// source IS the REFLECT_101 extension of that level at the left / top edges;
// at the right / bottom edges it is not when the level size is even, so the
// columns >= w are re-gathered from their mirror lanes (ds_bpermute) and the
// rows >= h are taken from their mirror rows in the rolling registers.
constexpr int ST_COLS = 480;  // source columns owned per strip
#ifndef STREAM_BAND
#define STREAM_BAND 32
#endif
constexpr int BAND = STREAM_BAND;  // level-1 rows owned per band (level k: BAND >> (k-1))

// Levels of at least RING_MIRROR_H rows get their top / bottom ring rows from
// the streaming pass (each ring row is a single-bounce REFLECT_101 copy of one
// interior row); shorter levels get the whole ring from ring_kernel.
constexpr int RING_MIRROR_H = 2 * PAD + 2;
// The top / bottom ring row that is the REFLECT_101 copy of row r (rows 1..PAD
// -> -r, rows h-1-PAD..h-2 -> 2h-2-r), or r itself when none is.
__device__ __forceinline__ int mirror_row(int r, int h) {
    if (h < RING_MIRROR_H) return r;
    if (r >= 1 && r <= PAD) return -r;
    if (r >= h - 1 - PAD && r <= h - 2) return 2 * h - 2 - r;
    return r;
}

__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {  // lane L <- lane L-1
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v) {  // lane L <- lane L+1
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}

// Edge bands: for every source row, the REFLECT_101-extended columns
// [-32, 16) and [w-16, w+32) are stored in a padded plane (the pyramid's unused
// level-0 slot on the batched path, the padded level 0 itself in the frame
// cache).  Lanes whose 16-byte window leaves [48, w-48) read the band instead
// of the source, so the streaming loop never gathers bytes: every row is one
// 16-byte load per lane and the prefetched rows stay in flight.
struct EdgePlane {
    const uint8_t* base;  // pixel (0,0) of image 0
    int64_t img_stride;
    int pitch;
};
constexpr int EDGE_L = 16, EDGE_R = 16;  // band extents inside the image

__device__ __forceinline__ uint4 src_row16(const uint8_t* __restrict__ S, int pitch, const uint8_t* __restrict__ E,
                                           int epitch, int w, int h, int x, int y) {
    const int ry = refl(y, h);
    const bool edge = x < EDGE_L - 16 || x + 16 > w - (EDGE_R - 16);
    const int xc = min(x, w + 16);  // lanes past the band are never used: keep them in range
    const uint8_t* p = edge ? E + (int64_t)ry * epitch + xc : S + (int64_t)ry * pitch + x;
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);  // 4-byte aligned
    return make_uint4(q[0], q[1], q[2], q[3]);
}

// Fill the edge bands of n_img source images into the padded plane E: per row
// three 16-byte chunks on each side.  Inside and outside chunks are separate
// item ranges, so waves never mix paths: the chunk inside the image ([0, 16),
// [w-16, w)) is a vector copy; the two outside chunks per side are the
// byte-reversed mirror ranges, built from aligned dword loads and v_perm.
// Requires w % 4 == 0 and 4-byte aligned rows (other inputs take the padded
// level-0 copy instead); vec16: 16-byte aligned rows and w % 16 == 0.
__global__ void __launch_bounds__(256) edge_kernel(const uint8_t* __restrict__ src, const uint8_t* __restrict__ src_b,
                                                   int n_a, int64_t img_stride, int pitch, int w, int h,
                                                   uint8_t* __restrict__ E, int64_t e_img_stride, int epitch,
                                                   int vec16) {
    const int img = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= h * 6) return;
    // items [0, 2h): the chunk inside the image on each side; [2h, 6h): the 4
    // mirrored chunks of a row
    int q, y;
    if (i < 2 * h) {
        y = i >> 1;
        q = 2 + (i & 1);
    } else {
        const int j = i - 2 * h;
        y = j >> 2;
        q = (j & 3) < 2 ? (j & 3) : (j & 3) + 2;
    }
    const int x = q < 3 ? -32 + 16 * q : w - EDGE_R + 16 * (q - 3);
    const uint8_t* row = (img < n_a ? src + img * img_stride : src_b + (img - n_a) * img_stride) + (int64_t)y * pitch;
    const uint32_t* rw = reinterpret_cast<const uint32_t*>(row);  // 4-byte aligned rows
    uint32_t* o = reinterpret_cast<uint32_t*>(E + img * e_img_stride + (int64_t)y * epitch + x);
    uint32_t d[4];
    if (x >= 0 && x + 16 <= w) {
        if (vec16) {
            *reinterpret_cast<uint4*>(o) = *reinterpret_cast<const uint4*>(row + x);
            return;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = rw[(x >> 2) + k];
    } else if (x < 0 && w >= 40) {
        // columns x..x+15 mirror to -x .. -x-15 (descending): output dword k
        // holds source bytes m-4k .. m-4k-3 with m = -x, a multiple of 16
        const int m4 = (-x) >> 2;
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = __builtin_amdgcn_perm(rw[m4 - k], rw[m4 - k - 1], 0x01020304u);
    } else if (x >= w && (w & 3) == 0 && w >= 40) {
        // columns x..x+15 mirror to 2w-2-x .. 2w-17-x (descending)
        const int m4 = (2 * w - 2 - x) >> 2;  // dword holding the first source byte (its byte 2)
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = __builtin_amdgcn_perm(rw[m4 - k], rw[m4 - k - 1], 0x03040506u);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t t = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) t |= (uint32_t)row[refl(x + 4 * k + b, w)] << (8 * b);
            d[k] = t;
        }
    }
    if (vec16) {
        *reinterpret_cast<uint4*>(o) = make_uint4(d[0], d[1], d[2], d[3]);
        return;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = d[k];
}

// four level-1 horizontal sums (u16 pairs) from the lane's 16 bytes (outputs
// read bytes 2+2j .. 6+2j)
__device__ __forceinline__ uint2 hsum_row(uint4 r) {
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
    return hsum4<2>(w, 0);
}
// Right-edge fix-up.  The next level's taps read this level at most two
// columns past its width w (columns w and w+1); their REFLECT_101 values are
// columns w-2 and w-3, which lie in this lane or the one / two lanes to the
// left.  The pass gathers them with DPP wave shifts and one v_perm whose
// per-lane selector is fixed for the whole strip.  Columns further out are
// never read and may hold anything.
// Level 1 (4 bytes per lane, lane column base c1 + 4(L-2)): window = the lane
// to the left (perm bytes 0..3) and this lane (4..7).
__device__ __forceinline__ uint32_t fix_sel4(int lane, int c0, int w) {
    const int base = c0 + 4 * (lane - 2);
    uint32_t sel = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int c = base + b;
        const int idx = c < w ? 4 + b : min(max(2 * w - 2 - c - base + 4, 0), 7);
        sel |= (uint32_t)idx << (8 * b);
    }
    return sel;
}
// Level 2 (2 bytes per lane in the low half): window = lanes L-2 (perm bytes
// 0,1), L-1 (2,3) and this lane (4,5).
__device__ __forceinline__ uint32_t fix_sel2(int lane, int c0, int w) {
    const int base = c0 + 2 * (lane - 2);
    uint32_t sel = 0x0c0c0000u;  // bytes 2,3 of the result: zero
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int c = base + b;
        const int idx = c < w ? 4 + b : min(max(2 * w - 2 - c - base + 4, 0), 5);
        sel |= (uint32_t)idx << (8 * b);
    }
    return sel;
}

// SKIP (tools/pyr_micro.hip only): bit k-1 set = level-k outputs are folded
// into a register instead of stored (to time the store traffic).
#ifndef STREAM_OCC
#define STREAM_OCC 4
#endif
template <int NL, int SKIP = 0>
__global__ void __launch_bounds__(256, STREAM_OCC) stream_kernel(const uint8_t* __restrict__ src,
                                                     const uint8_t* __restrict__ src_b, int n_a, int64_t src_img_stride,
                                                     int src_pitch, int w0, int h0, EdgePlane ep,
                                                     uint8_t* __restrict__ pyr, int64_t pyr_bytes, DownLevels L,
                                                     int n_strips, int n_bands, int n_units, int band,
                                                     uint8_t* __restrict__ trash) {
    const int lane = threadIdx.x & 63;
    const int nblk = (n_units + 3) / 4;
    const int unit = xcd_swizzle(blockIdx.x, nblk) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (unit >= n_units) return;
    const int st = unit % n_strips, rest = unit / n_strips;
    const int bd = rest % n_bands, img = rest / n_bands;
    // images [0, n_a) from src, the rest from src_b (prev and next frames of a
    // batch in one launch); the edge plane and the pyramids are contiguous
    const uint8_t* S = img < n_a ? src + img * src_img_stride : src_b + (img - n_a) * src_img_stride;
    const uint8_t* E = ep.base + img * ep.img_stride;
    uint8_t* P = pyr + img * pyr_bytes;
    const int x0 = ST_COLS * st + 8 * lane - 20;  // this lane's 16 source bytes
    const bool own_lane = lane >= 2 && lane < 62;
    const int w1 = L.w[0], h1 = L.h[0], p1 = L.pitch[0];
    const int c1 = (ST_COLS / 2) * st;            // level-1 column of lane 2, byte 0
    const bool fix1 = NL > 1 && c1 + 4 * 62 > w1;  // strip reaches past the right edge
    int w2 = 0, h2 = 0, p2 = 0, c2 = 0, w3 = 0, h3 = 0, p3 = 0, c3 = 0;
    bool fix2 = false;
    if (NL > 1) {
        w2 = L.w[1], h2 = L.h[1], p2 = L.pitch[1], c2 = (ST_COLS / 4) * st;
        fix2 = NL > 2 && c2 + 2 * 62 > w2;
    }
    if (NL > 2) w3 = L.w[2], h3 = L.h[2], p3 = L.pitch[2], c3 = (ST_COLS / 8) * st;
    const uint32_t sel1 = fix1 ? fix_sel4(lane, c1, w1) : 0u;
    const uint32_t sel2 = fix2 ? fix_sel2(lane, c2, w2) : 0u;
    // level-1 rows walked: everything the band's deepest owned rows depend on
    // (band: a multiple of 4, so r1s = 2 mod 4 and the level-2 / level-3 schedule below holds)
    const int r1s = band * bd - (NL == 3 ? 6 : NL == 2 ? 2 : 0);
    const int n1 = band + (NL == 3 ? 9 : NL == 2 ? 3 : 0);  // rows r1s .. r1s+n1-1
    const int o1lo = band * bd, o1hi = min(band * bd + band, h1);
    const int o2lo = (band >> 1) * bd, o2hi = NL > 1 ? min((band >> 1) * (bd + 1), h2) : 0;
    const int o3lo = (band >> 2) * bd, o3hi = NL > 2 ? min((band >> 2) * (bd + 1), h3) : 0;

    // rolling state: horizontal sums of source rows 2r1-2 .. 2r1+2 (hr[0..4]),
    // level-2 horizontal sums of level-1 rows (g2[0..4], newest last), level-3
    // horizontal sums of level-2 rows (g3[0..4])
    uint2 hr[5];
    uint32_t g2[5] = {0, 0, 0, 0, 0}, g3[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 3; ++k) hr[k] = hsum_row(src_row16(S, src_pitch, E, ep.pitch, w0, h0, x0, 2 * r1s - 2 + k));
    // source rows 2r1+1, 2r1+2 of level-1 row r1 = r1s+k live in slot k % RS;
    // they are fetched PF iterations ahead (2*PF rows x 1 KB in flight per wave).
    // PF = 4 at 4 waves per SIMD (99 VGPRs) measured 0.230 ms per 512 images
    // against 0.244 for PF = 2 at 8 (63 VGPRs) and 0.234 / 0.231 for PF = 3 / 5
    // (tools/ab.sh, r01 v21); 5 waves per SIMD spill.
#ifndef STREAM_PF
#define STREAM_PF 4
#endif
    constexpr int PF = STREAM_PF;
    constexpr int RS = PF <= 2 ? 4 : 8;  // ring slots (a multiple of 4: the level-3 schedule)
    static_assert(PF >= 1 && PF <= 6, "prefetch depth must fit the 8-slot ring");
    uint4 pa[RS], pb[RS];
#pragma unroll
    for (int k = 0; k < PF; ++k) {
        pa[k] = src_row16(S, src_pitch, E, ep.pitch, w0, h0, x0, 2 * (r1s + k) + 1);
        pb[k] = src_row16(S, src_pitch, E, ep.pitch, w0, h0, x0, 2 * (r1s + k) + 2);
    }
    // Loads are issued unconditionally and stores branch only on wave-uniform
    // row conditions (rows of the band, mirrored ring rows): on gfx9 stores and
    // loads share vmcnt, and a store under a lane-divergent branch would make the
    // compiler wait for all earlier stores before using a prefetched row; a
    // uniform branch costs at most one extra counted op at the join.  Lanes that
    // own no output (lanes 0/1/62/63, columns past the level) store to this
    // lane's dword of a trash line.
    uint8_t* const tl = trash + (int64_t)unit * 256 + 4 * lane;  // this wave's own line (no sharing)
    uint32_t nsink = 0;
    auto body = [&](int k, auto slot_c) {
        constexpr int slot = decltype(slot_c)::value;
        const int r1 = r1s + k;
        hr[3] = hsum_row(pa[slot]);
        hr[4] = hsum_row(pb[slot]);
        pa[(slot + PF) % RS] = src_row16(S, src_pitch, E, ep.pitch, w0, h0, x0, 2 * (r1 + PF) + 1);
        pb[(slot + PF) % RS] = src_row16(S, src_pitch, E, ep.pitch, w0, h0, x0, 2 * (r1 + PF) + 2);
        // level-1 row r1
        uint32_t l1 = hibytes(vsum2(hr[0].x, hr[1].x, hr[2].x, hr[3].x, hr[4].x),
                              vsum2(hr[0].y, hr[1].y, hr[2].y, hr[3].y, hr[4].y));
        hr[0] = hr[2];
        hr[1] = hr[3];
        hr[2] = hr[4];
        if (fix1) l1 = __builtin_amdgcn_perm(l1, wave_shr1(l1), sel1);
        if (r1 >= o1lo && r1 < o1hi) {  // wave-uniform: rows of the band
            const bool ok = own_lane && c1 + 4 * (lane - 2) < w1;
            uint8_t* q = P + L.off[0] + c1 + 4 * (lane - 2) + PAD;
            const int mr = mirror_row(r1, h1);  // the ring row holding this row's REFLECT_101 copy
            if constexpr ((SKIP & 1) != 0) {
                nsink ^= l1;
            } else {
                *reinterpret_cast<uint32_t*>(ok ? q + (int64_t)(r1 + PAD) * p1 : tl) = l1;
                if (mr != r1) *reinterpret_cast<uint32_t*>(ok ? q + (int64_t)(mr + PAD) * p1 : tl) = l1;
            }
        }
        if constexpr (NL > 1) {
            // level-2 horizontal sums of level-1 row r1 (rows >= h1 mirror rows
            // 2h1-2-r1, which are 2 / 4 rows back)
            uint32_t g;
            if (r1 < h1) {
                const uint32_t pv = wave_shr1(l1), nx = wave_shl1(l1);
                const uint32_t a = __builtin_amdgcn_perm(l1, pv, 0x05040302u);  // prev.b2 prev.b3 l1.b0 l1.b1
                const uint32_t o0 = __builtin_amdgcn_udot4(a, 0x04060401u, (l1 >> 16) & 0xffu, false);
                const uint32_t o1 = __builtin_amdgcn_udot4(l1, 0x04060401u, nx & 0xffu, false);
                g = o0 | (o1 << 16);
            } else {
                g = r1 == h1 ? g2[3] : g2[1];
            }
            g2[0] = g2[1];
            g2[1] = g2[2];
            g2[2] = g2[3];
            g2[3] = g2[4];
            g2[4] = g;
            // level-2 row r2 = (r1-2)/2 at every even k (rows before k = 4 are
            // warm-up garbage and go to the trash line)
            if constexpr ((slot & 1) == 0) {
                const int r2 = (r1 - 2) >> 1;
                const uint32_t v = vsum2(g2[0], g2[1], g2[2], g2[3], g2[4]);
                uint32_t l2 = __builtin_amdgcn_perm(0u, v, 0x0c0c0301u);  // (s+128)>>8 of both halves
                if (fix2) {
                    const uint32_t a1 = wave_shr1(l2), a2 = wave_shr1(a1);
                    l2 = __builtin_amdgcn_perm(l2, (a2 & 0xffffu) | (a1 << 16), sel2);
                }
                if (k >= 4 && r2 >= o2lo && r2 < o2hi) {
                    const bool ok = own_lane && c2 + 2 * (lane - 2) < w2;
                    uint8_t* q = P + L.off[1] + c2 + 2 * (lane - 2) + PAD;
                    const int mr = mirror_row(r2, h2);
                    if constexpr ((SKIP & 2) != 0) {
                        nsink ^= l2 << 7;
                    } else {
                        *reinterpret_cast<uint16_t*>(ok ? q + (int64_t)(r2 + PAD) * p2 : tl) = (uint16_t)l2;
                        if (mr != r2)
                            *reinterpret_cast<uint16_t*>(ok ? q + (int64_t)(mr + PAD) * p2 : tl) = (uint16_t)l2;
                    }
                }
                if constexpr (NL > 2) {
                    uint32_t g;
                    if (r2 < h2) {
                        const uint32_t pv = wave_shr1(l2), nx = wave_shl1(l2);
                        const uint32_t a = __builtin_amdgcn_perm(l2, pv, 0x05040100u);  // prev.b0 prev.b1 l2.b0 l2.b1
                        g = __builtin_amdgcn_udot4(a, 0x04060401u, nx & 0xffu, false);
                    } else {
                        g = r2 == h2 ? g3[3] : g3[1];
                    }
                    g3[0] = g3[1];
                    g3[1] = g3[2];
                    g3[2] = g3[3];
                    g3[3] = g3[4];
                    g3[4] = g;
                    // level-3 row r3 = (r2-2)/2 at every k = 0 (mod 4); valid from
                    // k = 12, when level-2 rows r2-4 .. r2 (k = 4..12) are in
                    if constexpr ((slot & 3) == 0) {
                        const int r3 = (r2 - 2) >> 1;
                        const uint32_t s3 = g3[0] + g3[4] + 4 * (g3[1] + g3[3]) + 6 * g3[2] + 128;
                        const bool ok = own_lane && c3 + (lane - 2) < w3;
                        uint8_t* q = P + L.off[2] + c3 + (lane - 2) + PAD;
                        const int mr = mirror_row(r3, h3);
                        if constexpr ((SKIP & 4) != 0) {
                            nsink ^= s3 << 13;
                        } else if (k >= 12 && r3 >= o3lo && r3 < o3hi) {
                            *(ok ? q + (int64_t)(r3 + PAD) * p3 : tl) = (uint8_t)(s3 >> 8);
                            if (mr != r3) *(ok ? q + (int64_t)(mr + PAD) * p3 : tl) = (uint8_t)(s3 >> 8);
                        }
                    }
                }
            }
        }
    };
    // r1s is even and the slot tracks k % RS, so the level-2 / level-3 schedule
    // (k % 2, k % 4) is static; the trip count is rounded up to whole groups of
    // four rows
    for (int k = 0; k < n1; k += RS) {
        body(k, std::integral_constant<int, 0>{});
        body(k + 1, std::integral_constant<int, 1>{});
        body(k + 2, std::integral_constant<int, 2>{});
        body(k + 3, std::integral_constant<int, 3>{});
        if constexpr (RS == 8) {
            if (k + 4 >= n1) break;  // wave-uniform
            body(k + 4, std::integral_constant<int, 4 % RS>{});
            body(k + 5, std::integral_constant<int, 5 % RS>{});
            body(k + 6, std::integral_constant<int, 6 % RS>{});
            body(k + 7, std::integral_constant<int, 7 % RS>{});
        }
    }
    if constexpr (SKIP != 0) *reinterpret_cast<uint32_t*>(tl) = nsink;
}

template <int NL>
void launch_stream(gvx_ctx* c, const uint8_t* src, const uint8_t* src_b, int n_a, int64_t src_img_stride,
                   int src_pitch, int src_w, int src_h, const EdgePlane& ep, int n_img, const PyrLayout& lay, int l0,
                   uint8_t* dst) {
    DownLevels D{};
    for (int k = 0; k < NL; ++k) {
        D.off[k] = lay.off[l0 + 1 + k];
        D.pitch[k] = lay.pitch[l0 + 1 + k];
        D.w[k] = lay.w[l0 + 1 + k];
        D.h[k] = lay.h[l0 + 1 + k];
    }
    const int n_strips = (D.w[0] + ST_COLS / 2 - 1) / (ST_COLS / 2);
    // BAND level-1 rows per wave when the batch fills the chip; a small batch
    // (the live tracker's single frame or pair) takes narrower bands down to 4
    // rows: more waves, each walking band + 9 rows instead of BAND + 9 -- less
    // latency for more halo work on an otherwise idle GPU
    int band = BAND;
    while (band > 4 && n_strips * ((D.h[0] + band - 1) / band) * n_img < 4 * c->n_cu) band >>= 1;
    const int n_bands = (D.h[0] + band - 1) / band;
    const int n_units = n_strips * n_bands * n_img;
    const int nblk = (n_units + 3) / 4;
    uint8_t* trash = (uint8_t*)scratch(c, "pyr_trash", (size_t)n_units * 256);
    hipLaunchKernelGGL(stream_kernel<NL>, dim3(N_XCD * xcd_per(nblk)), dim3(256), 0, c->stream, src, src_b, n_a,
                       src_img_stride, src_pitch, src_w, src_h, ep, dst, lay.bytes, D, n_strips, n_bands, n_units,
                       band, trash);
}


// ------------------------------------------------------------------ rings
// REFLECT_101 rings of levels lo..hi of every image in one launch.  Item = one
// dword of ring: the top / bottom PAD rows over the padded width, then per
// interior row the left PAD columns and the right columns [w, w+PAD) (dword
// aligned; bytes of the last interior dword rewrite their own value).
struct RingLevels {
    int32_t n;                  // levels
    int64_t off[MAX_LEVELS];
    int32_t pitch[MAX_LEVELS], w[MAX_LEVELS], h[MAX_LEVELS];
    int32_t dw[MAX_LEVELS];     // dwords per padded row (top/bottom bands)
    int32_t rd0[MAX_LEVELS];    // first dword (padded col / 4) of the right band
    int32_t rdn[MAX_LEVELS];    // dwords of the right band
    int32_t sides[MAX_LEVELS];  // 1: top/bottom rows already written (side bands only)
    int32_t items[MAX_LEVELS];  // ring dwords of the level
};

// One ring dword at padded byte column pcol of padded row prow.  Inside the
// level it is a plain copy (last interior dword of a row: its own bytes); outside,
// the four REFLECT_101 source columns span at most 4 consecutive bytes
// (descending, or folded at the right edge), so two aligned dwords and one
// v_perm with a computed selector build it.
__device__ __forceinline__ uint32_t ring_dword(const uint32_t* rw, int pcol, int w) {
    const int x0 = pcol - PAD;
    if (x0 >= 0 && x0 + 4 <= w) return rw[pcol >> 2];
    int sx[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) sx[b] = refl(min(x0 + b, w + PAD - 1), w) + PAD;
    const int lo = min(min(sx[0], sx[1]), min(sx[2], sx[3])) & ~3;
    uint32_t sel = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) sel |= (uint32_t)(sx[b] - lo) << (8 * b);
    return __builtin_amdgcn_perm(rw[(lo >> 2) + 1], rw[lo >> 2], sel);
}

// Item = one ring dword.  Full ring: the top / bottom PAD rows over the
// padded width, then the side bands of the interior rows.  Side-bands-only
// levels: the left PAD columns and the right columns [w, w+PAD) of every padded
// row (ring rows included: their sources are interior pixels).  Bytes of the
// last interior dword of a row rewrite their own value.
__global__ void __launch_bounds__(256) ring_kernel(uint8_t* __restrict__ pyr, int64_t pyr_bytes, RingLevels R) {
    const int l = blockIdx.z;  // level slot (wave-uniform)
    int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= R.items[l]) return;
    const int w = R.w[l], h = R.h[l], pitch = R.pitch[l];
    uint8_t* base = pyr + (int64_t)blockIdx.y * pyr_bytes + R.off[l];
    int prow, pcol;  // padded row, padded byte column of the dword
    const int nb = R.sides[l] ? 0 : 2 * PAD * R.dw[l];
    if (j < nb) {
        const int r = j / R.dw[l];
        prow = r < PAD ? r : h + r;
        pcol = 4 * (j - r * R.dw[l]);
    } else {
        j -= nb;
        const int per = PAD / 4 + R.rdn[l];
        const int r = j / per, c = j - r * per;
        prow = R.sides[l] ? r : PAD + r;
        pcol = c < PAD / 4 ? 4 * c : 4 * (R.rd0[l] + c - PAD / 4);
    }
    const uint32_t* rw = reinterpret_cast<const uint32_t*>(base + (int64_t)(refl(prow - PAD, h) + PAD) * pitch);
    *reinterpret_cast<uint32_t*>(base + (int64_t)prow * pitch + pcol) = ring_dword(rw, pcol, w);
}

// Rings of levels lo..hi.  sides_only: the streaming pass already wrote the
// top / bottom ring rows of every level tall enough (RING_MIRROR_H).
void launch_rings(gvx_ctx* c, int n_img, const PyrLayout& lay, int lo, int hi, uint8_t* dst, bool sides_only) {
    RingLevels R{};
    R.n = hi - lo + 1;
    int most = 0;
    for (int k = 0; k < R.n; ++k) {
        const int lv = lo + k, w = lay.w[lv];
        R.off[k] = lay.off[lv];
        R.pitch[k] = lay.pitch[lv];
        R.w[k] = w;
        R.h[k] = lay.h[lv];
        R.dw[k] = (w + 2 * PAD + 3) / 4;
        R.rd0[k] = (w + PAD) / 4;
        R.rdn[k] = (w + 2 * PAD + 3) / 4 - R.rd0[k];
        R.sides[k] = sides_only && lay.h[lv] >= RING_MIRROR_H;
        R.items[k] = R.sides[k] ? (lay.h[lv] + 2 * PAD) * (PAD / 4 + R.rdn[k])
                                : 2 * PAD * R.dw[k] + lay.h[lv] * (PAD / 4 + R.rdn[k]);
        most = R.items[k] > most ? R.items[k] : most;
    }
    dim3 grid((most + 255) / 256, n_img, R.n);
    hipLaunchKernelGGL(ring_kernel, grid, dim3(256), 0, c->stream, dst, lay.bytes, R);
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
                                 const PyrLayout& lay, uint8_t* dst, bool write_l0, const uint8_t* src_b, int n_a) {
    if (n_img <= 0) return hipSuccess;
    if (!src_b) n_a = n_img;
    // level-0 slot of the pyramid: pixel (0,0) of image 0
    uint8_t* slot0 = dst + lay.off[0] + (int64_t)PAD * lay.pitch[0] + PAD;
    const bool aligned = stride % 4 == 0 && img_stride % 4 == 0 && reinterpret_cast<uintptr_t>(src) % 4 == 0 &&
                         lay.w[0] % 4 == 0;
    const uint8_t* s0 = src;
    int64_t s0_img = img_stride;
    int s0_pitch = stride;
    if (n_a < n_img && (write_l0 || !aligned || reinterpret_cast<uintptr_t>(src_b) % 4 != 0)) {
        // two sources on the level-0-copy path: one build per source
        hipError_t e = launch_build_pyramids(c, src, img_stride, stride, n_a, lay, dst, write_l0, nullptr, 0);
        if (e != hipSuccess) return e;
        return launch_build_pyramids(c, src_b, img_stride, stride, n_img - n_a, lay, dst + (int64_t)n_a * lay.bytes,
                                     write_l0, nullptr, 0);
    }
    if (write_l0 || !aligned) {
        // full padded level-0 copy: the source of the build and its own edge plane
        const int groups = (lay.w[0] + 2 * PAD + 15) / 16;
        const int items = groups * (lay.h[0] + 2 * PAD);
        dim3 grid((items + 255) / 256, n_img);
        hipLaunchKernelGGL(level0_kernel, grid, dim3(256), 0, c->stream, src, img_stride, stride, lay.w[0],
                           lay.h[0], lay.pitch[0], lay.bytes, dst);
        s0 = slot0;
        s0_img = lay.bytes;
        s0_pitch = lay.pitch[0];
    } else {
        // read level 0 in place; only its edge bands go to the (otherwise unused) slot
        const int vec16 = stride % 16 == 0 && img_stride % 16 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0 &&
                          (n_a == n_img || reinterpret_cast<uintptr_t>(src_b) % 16 == 0) &&
                          lay.w[0] % 16 == 0 && reinterpret_cast<uintptr_t>(slot0) % 16 == 0 && lay.pitch[0] % 16 == 0;
        dim3 grid((lay.h[0] * 6 + 255) / 256, n_img);
        hipLaunchKernelGGL(edge_kernel, grid, dim3(256), 0, c->stream, src, src_b, n_a, img_stride, stride, lay.w[0],
                           lay.h[0], slot0, lay.bytes, lay.pitch[0], vec16);
    }
    // levels 1.. in streaming passes of up to 3 levels; a later pass reads the
    // previous pass's deepest level (padded, its ring built first)
    int l = 0;
    while (l + 1 < lay.nlev) {
        const int nl = lay.nlev - 1 - l >= 3 ? 3 : lay.nlev - 1 - l;
        const uint8_t* s = l == 0 ? s0 : dst + lay.off[l] + (int64_t)PAD * lay.pitch[l] + PAD;
        const uint8_t* sb = l == 0 ? src_b : nullptr;  // the level-0 copy path never has two sources here
        const int na = l == 0 ? n_a : n_img;
        const int64_t si = l == 0 ? s0_img : lay.bytes;
        const int sp = l == 0 ? s0_pitch : lay.pitch[l];
        const EdgePlane ep = l == 0 ? EdgePlane{slot0, lay.bytes, lay.pitch[0]} : EdgePlane{s, lay.bytes, sp};
        if (nl == 3)
            launch_stream<3>(c, s, sb, na, si, sp, lay.w[l], lay.h[l], ep, n_img, lay, l, dst);
        else if (nl == 2)
            launch_stream<2>(c, s, sb, na, si, sp, lay.w[l], lay.h[l], ep, n_img, lay, l, dst);
        else
            launch_stream<1>(c, s, sb, na, si, sp, lay.w[l], lay.h[l], ep, n_img, lay, l, dst);
        launch_rings(c, n_img, lay, l + 1, l + nl, dst, true);
        l += nl;
    }
    return hipGetLastError();
}

}  // namespace gvx
