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
//   stream_kernel<NL> NL pyrDown levels and their PAD rings in one streaming
//                   pass (level 0 read in place, REFLECT_101 gathered at its edges)
//   ring_kernel     the rings of levels too small for the pass (< RING_MIN)
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
// Horizontal [1 4 6 4 1] taps of one source row into four u16 outputs: outputs
// 4g..4g+3 read source bytes 8g .. 8g+10 of the row (`sh` = byte shift of the row
// start inside its first dword, 0 or 2).
template <int SH>
__device__ __forceinline__ uint2 hsum4(const uint32_t* row, int g) {
    static_assert(SH == 0 || SH == 2, "row starts at byte 0 or 2 of its first dword");
    const uint32_t* p = row + 2 * g;
    const uint32_t w0 = p[0], w1 = p[1], w2 = p[2];
    constexpr uint32_t K = 0x04060401u;  // taps 1 4 6 4 on bytes 0..3, the fifth tap added
    uint32_t a0, a1, a2, a3, t0, t1, t2, t3;  // the four outputs' first four bytes and fifth byte
    if constexpr (SH == 0) {
        // outputs read bytes 0..4, 2..6, 4..8, 6..10
        a0 = w0;
        a1 = __builtin_amdgcn_alignbyte(w1, w0, 2);
        a2 = w1;
        a3 = __builtin_amdgcn_alignbyte(w2, w1, 2);
        t0 = w1 & 0xffu;
        t1 = (w1 >> 16) & 0xffu;
        t2 = w2 & 0xffu;
        t3 = (w2 >> 16) & 0xffu;
    } else {
        // outputs read bytes 2..6, 4..8, 6..10, 8..12: the odd outputs' windows are
        // whole loaded dwords, so only the even ones realign (2 alignbytes a row,
        // not 5)
        const uint32_t w3 = p[3];
        a0 = __builtin_amdgcn_alignbyte(w1, w0, 2);
        a1 = w1;
        a2 = __builtin_amdgcn_alignbyte(w2, w1, 2);
        a3 = w2;
        t0 = (w1 >> 16) & 0xffu;
        t1 = w2 & 0xffu;
        t2 = (w2 >> 16) & 0xffu;
        t3 = w3 & 0xffu;
    }
    const uint32_t o0 = __builtin_amdgcn_udot4(a0, K, t0, false);
    const uint32_t o1 = __builtin_amdgcn_udot4(a1, K, t1, false);
    const uint32_t o2 = __builtin_amdgcn_udot4(a2, K, t2, false);
    const uint32_t o3 = __builtin_amdgcn_udot4(a3, K, t3, false);
    return make_uint2(o0 | (o1 << 16), o2 | (o3 << 16));
}

// Vertical taps on packed u16 pairs: (a + 4b + 6c + 4d + e + 128) per half.
// Every partial sum stays < 2^16 (inputs <= 4080, result <= 65408), so the two
// halves never interact.
// Five packed ops: the compiler's own form of the same sum takes six (it turns
// the multiply by 4 into a shift and an add), so the two multiply-adds are
// written out.
__device__ __forceinline__ uint32_t vsum2(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e) {
    typedef unsigned short v2u __attribute__((ext_vector_type(2)));
    const uint32_t ae = __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2u, a) + __builtin_bit_cast(v2u, e));
    const uint32_t bd = __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2u, b) + __builtin_bit_cast(v2u, d));
    uint32_t t, r;
    asm("v_pk_mad_u16 %0, %1, 4, %2 op_sel_hi:[1,0,1]" : "=v"(t) : "v"(bd), "v"(ae));
    asm("v_pk_mad_u16 %0, %1, 6, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(c), "v"(t));
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2u, r) + (unsigned short)128);
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
// Band b owns level-1 rows [band*b, band*(b+1)) (level k: the same >> (k-1)).
// Borders, all inside this one pass:
//  * source columns are REFLECT_101-extended at load: the strips that touch an
//    edge of an unpadded level 0 gather each output dword with one v_perm of an
//    aligned dword pair at a per-lane offset (fixed for the strip); a padded
//    source is read through its ring;
//  * because the filter is symmetric, a level computed from an extended source
//    IS the REFLECT_101 extension of that level at the left / top edges; at the
//    right / bottom edges it is not when the level size is even, so the columns
//    >= w are re-gathered from their mirror lanes (DPP + v_perm) and the rows
//    >= h are taken from their mirror rows in the rolling registers;
//  * the PAD ring of each level is written by the lanes that hold its source
//    pixels: the top / bottom ring rows are extra stores of the mirrored rows,
//    the side bands extra stores of the mirrored columns (level 1: one dword per
//    lane, built with a DPP neighbour and a v_perm; levels 2 and 3: bytes).
//    Levels narrower or shorter than RING_MIN take their ring from ring_kernel.
constexpr int ST_COLS = 480;  // source columns owned per strip
// Level-1 rows per band when the batch fills the chip.  72 (r06, profiles/r06_bd):
// beside LK in the three-stream step, 72-96-row bands beat 40 by 1-2 % (fewer
// warm-up rows, 6,144 instead of 10,752 waves at configs[1]), though the pass
// alone is 5 % slower (0.169 against 0.161 ms); 140 loses (its long waves hold
// LK out of the SIMDs).
#ifndef STREAM_BAND
#define STREAM_BAND 72
#endif
constexpr int BAND = STREAM_BAND;  // level-1 rows owned per band (level k: BAND >> (k-1))

// Levels at least RING_MIN pixels wide and tall get their whole PAD ring from
// the streaming pass (every ring pixel is then a single-bounce REFLECT_101 copy
// of an interior pixel); smaller levels get it from ring_kernel.
constexpr int RING_MIN = 2 * PAD + 2;
// The top / bottom ring row that is the REFLECT_101 copy of row r (rows 1..PAD
// -> -r, rows h-1-PAD..h-2 -> 2h-2-r), or r itself when none is.
__device__ __forceinline__ int mirror_row(int r, int h) {
    if (h < RING_MIN) return r;
    if (r >= 1 && r <= PAD) return -r;
    if (r >= h - 1 - PAD && r <= h - 2) return 2 * h - 2 - r;
    return r;
}
// The side-band column that is the REFLECT_101 copy of column c (1..PAD -> -c,
// w-1-PAD..w-2 -> 2w-2-c), or 0 when none is (column 0 is never a ring column).
__device__ __forceinline__ int ring_col(int c, int w) {
    return (c >= 1 && c <= PAD) ? -c : (c >= w - 1 - PAD && c <= w - 2) ? 2 * w - 2 - c : 0;
}

// (bound_ctrl: a lane without a source lane reads 0, so no `old` operand has to
// be zeroed first -- one v_mov_b32_dpp instead of two moves; every lane of the
// pass is active)
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {  // lane L <- lane L-1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x138, 0xf, 0xf, true);
}
__device__ __forceinline__ uint32_t wave_shl1(uint32_t v) {  // lane L <- lane L+1
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x130, 0xf, 0xf, true);
}

// Source of a pass: images [0, n_a) at a + i*img_stride, the rest at
// b + (i - n_a)*img_stride (the prev and next frames of a batch in one launch);
// pointers at pixel (0,0).  raw: the caller's unpadded level 0 (w % 4 == 0,
// 4-byte aligned rows), read in place; otherwise a padded level, whose ring
// the edge lanes read directly.
struct StreamSrc {
    const uint8_t* a;
    const uint8_t* b;
    int n_a;
    int64_t img_stride;
    int pitch, w, h;
    int raw;
};

// Edge strips of an unpadded source.  Every lane loads its 16 bytes at a
// column clamped into the image, xc = clamp(x0, 0, w-16), and shifts them back
// by r = (x0 - xc)/4 dwords.  The dwords past the ends that a level-1 output
// inside the image still reads are REFLECT_101 copies of the first / last
// loaded dword (one v_perm): lane 2 of strip 0 (x0 = -4, r = -1) needs columns
// -2, -1 (= 2, 1) and the lane holding level-1 column w1-1 (r = 1 or 2) needs
// column w (= w-2).  Lanes 0 and 1 of strip 0 (r < -1) and the lanes past the
// right edge (r > 2) compute unused values, and their level-1 columns are
// replaced afterwards (left: the mirrored level-1 pixels of lanes 2..4, right:
// the fix-up below).  r is fixed for the strip, so the three per-lane choices
// are lane masks in SGPRs.
struct Gather {
    int dx;                    // xc - x0
    uint64_t m_left, m_1, m_2;  // lanes with r = -1 / 1 / 2 (the others: r = 0)
};
__device__ __forceinline__ Gather make_gather(int x0, int w) {
    Gather g;
    const int xc = min(max(x0, 0), w - 16);
    const int r = (x0 - xc) >> 2;
    g.dx = xc - x0;
    g.m_left = __ballot(r == -1);
    g.m_1 = __ballot(r == 1);
    g.m_2 = __ballot(r >= 2);
    return g;
}
__device__ __forceinline__ bool lane_in(uint64_t m) { return (m >> __lane_id()) & 1u; }
// 16 source bytes of row y (REFLECT_101) for this lane
// Interior strips load through a buffer view of the source whose base sits
// SRC_BIAS bytes before pixel (0,0) (padded sources are read up to 20 bytes
// left of it, in their ring): the lane's column is a fixed voffset and the row a
// wave-uniform soffset, so a row load costs no VALU address arithmetic.
constexpr int SRC_BIAS = 64;
typedef uint32_t v4u_t __attribute__((ext_vector_type(4)));
// GATHER: 0 = interior strip; 1 / 2 = the strip holds the left / right edge of an
// unpadded source; 3 = both (a source narrower than a strip).  Every lane loads
// through the buffer view (edge strips at their clamped column x = xc, so no
// per-row address arithmetic), and an edge strip then shifts the dwords of the
// lanes the Gather masks name: the left edge has only r = -1 lanes, the right
// edge only r = 1 / 2 lanes (r06_pp: the three-way selects of every row of
// both edge strips were a fifth of their instructions).
template <int GATHER>
__device__ __forceinline__ uint4 src_row16(int pitch, int h, int x, const Gather& g, int y,
                                           const __amdgpu_buffer_rsrc_t& srs) {
    const v4u_t w = __builtin_amdgcn_raw_buffer_load_b128(srs, x + SRC_BIAS, refl(y, h) * pitch, 0);
    if constexpr (GATHER == 0) return make_uint4(w.x, w.y, w.z, w.w);
    const uint32_t d0 = w.x, d1 = w.y, d2 = w.z, d3 = w.w;
    if constexpr (GATHER == 1) {
        const uint32_t el = __builtin_amdgcn_perm(d0, d0, 0x01020303u);  // columns -4..-1 <- (3,) 3, 2, 1
        const bool L = lane_in(g.m_left);
        return make_uint4(L ? el : d0, L ? d0 : d1, L ? d1 : d2, L ? d2 : d3);
    }
    const uint32_t er = __builtin_amdgcn_perm(d3, d3, 0x00000102u);  // columns +16.. <- +14, +13, +12
    const bool R1 = lane_in(g.m_1), R2 = lane_in(g.m_2);
    if constexpr (GATHER == 2)
        return make_uint4(R1 ? d1 : R2 ? d2 : d0, R1 ? d2 : R2 ? d3 : d1, R1 ? d3 : R2 ? er : d2,
                          R1 || R2 ? er : d3);
    const uint32_t el = __builtin_amdgcn_perm(d0, d0, 0x01020303u);
    const bool L = lane_in(g.m_left);
    return make_uint4(L ? el : R1 ? d1 : R2 ? d2 : d0, L ? d0 : R1 ? d2 : R2 ? d3 : d1,
                      L ? d1 : R1 ? d3 : R2 ? er : d2, L ? d2 : R1 ? er : R2 ? er : d3);
}
// Strip 0 of an unpadded source: level-1 columns -8..-1 (lanes 0, 1) are the
// REFLECT_101 copies of columns 8..1 (lanes 2..4), taken with DPP row shifts.
__device__ __forceinline__ uint32_t left_mirror_l1(uint32_t l1, int lane) {
    const uint32_t s1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)l1, 0x101, 0xf, 0xf, true);  // row_shl:1
    const uint32_t s2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)l1, 0x102, 0xf, 0xf, true);  // row_shl:2
    const uint32_t v = __builtin_amdgcn_perm(s2, s1, 0x01020304u);  // lane L: columns of lanes L+1, L+2 reversed
    const uint32_t v2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x102, 0xf, 0xf, true);
    return lane == 1 ? v : lane == 0 ? v2 : l1;
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

// the levels a pass writes (offsets of the padded (-PAD,-PAD) corners)
struct DownLevels {
    int64_t off[3];
    int32_t pitch[3], w[3], h[3];
    int32_t sides[3];  // SIDES passes: 1 = the pass writes the level's side bands (w, h >= RING_MIN)
};

// SKIP (tools/pyr_probe.hip only): bit k-1 set = level-k outputs are folded
// into a register instead of stored (to time the store traffic).
#ifndef STREAM_OCC
#define STREAM_OCC 4
#endif
// One wave's walk over its (strip, band).  GATHER (wave-uniform, one instance
// each): 0 = an interior strip, 1 / 2 / 3 = the strip holds the left / right /
// both edges of an unpadded source (src_row16).  The loop has no per-row path
// choice (loads stay in flight across iterations).
// Side bands.  A batch that fills the chip (the default, SIDES = false): the
// pass writes each level's rows and their top / bottom REFLECT_101 ring rows,
// and ring_kernel the side bands (r06: written here they took the edge strips'
// waves to ~2x the interior strips' instructions, 64-bit flat stores that the
// buffer form would have spilled; pass + sides 0.179 -> 0.166 ms at configs[1],
// profiles/r06_sb1).  A small launch (SIDES = true: the live tracker's pair or
// frame, whose pass is latency-bound and where another launch costs ~1 us) also
// writes the side bands here, from the lanes that hold their source pixels.
// Stores: pixel column `col` of padded row `row` of a level whose column 0 of
// padded row 0 is d.ptr (byte d.off of the image's pyramid).  Lanes that own no
// output (own == false) must not write the level: BUF stores through a buffer
// view at an offset past the pyramid, which the bounds check drops (a 32-bit
// offset per store, r04_v24); the SIDES instances keep the flat form, those
// lanes writing the wave's trash line.
struct PyrDst {
    __amdgpu_buffer_rsrc_t rs;
    uint8_t* ptr;
    int off;
    uint8_t* tl;
};
constexpr int PYR_OOB = 0x7fffffff;
template <bool BUF, typename T>
__device__ __forceinline__ void pyr_store(const PyrDst& d, bool own, int col, int row, int pitch, T v) {
    if constexpr (BUF) {
        const int o = own ? d.off + col + row * pitch : PYR_OOB;
        if constexpr (sizeof(T) == 4)
            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, d.rs, o, 0, 0);
        else if constexpr (sizeof(T) == 2)
            __builtin_amdgcn_raw_buffer_store_b16((unsigned short)v, d.rs, o, 0, 0);
        else
            __builtin_amdgcn_raw_buffer_store_b8((unsigned char)v, d.rs, o, 0, 0);
    } else {
        *reinterpret_cast<T*>(own ? d.ptr + col + (int64_t)row * pitch : d.tl) = v;
    }
}

template <int NL, int GATHER, bool SIDES, int SKIP>
__device__ __forceinline__ void stream_walk(const StreamSrc& src, uint8_t* __restrict__ pyr, int64_t pyr_bytes,
                                            const DownLevels& L, int st, int bd, int img, int band, int lane,
                                            uint8_t* __restrict__ tl, bool side1, bool side2, bool side3) {
    const uint8_t* S = img < src.n_a ? src.a + img * src.img_stride : src.b + (img - src.n_a) * src.img_stride;
    uint8_t* P = pyr + img * pyr_bytes;
    // stores go through a buffer view of the image's pyramid (pyr_store)
    constexpr bool BUF = !SIDES;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(P, (short)0, (int)pyr_bytes, 0x00020000);
    const int w0 = src.w, h0 = src.h, sp = src.pitch;
    const int x0 = ST_COLS * st + 8 * lane - 20;  // this lane's 16 source bytes
    // padded sources: lanes past the ring read inside it (their outputs are unused);
    // edge strips of an unpadded source load at the clamped column xc = x0 + dx
    Gather g{};
    if constexpr (GATHER != 0) g = make_gather(x0, w0);
    const int xs = GATHER != 0 ? x0 + g.dx : src.raw ? x0 : min(x0, w0 + 16);
    const __amdgpu_buffer_rsrc_t srs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(S - SRC_BIAS), (short)0, 0x7fffffff, 0x00020000);
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
    // level-1 side bands as dwords: the left band always (ring dword [-a-4, -a-1]
    // from lanes a, a+4), the right one when w1 % 4 == 0 ([2w1-4-a, 2w1-1-a] from
    // lanes a-4, a); otherwise the right band byte by byte
    const bool r1dw = (w1 & 3) == 0;
    // level-1 rows walked: everything the band's deepest owned rows depend on
    // (band: a multiple of 4, so r1s = 2 mod 4 and the level-2 / level-3 schedule below holds)
    const int r1s = band * bd - (NL == 3 ? 6 : NL == 2 ? 2 : 0);
    const int n1 = band + (NL == 3 ? 9 : NL == 2 ? 3 : 0);  // rows r1s .. r1s+n1-1
    const int o1lo = band * bd, o1hi = min(band * bd + band, h1);
    const int o2lo = (band >> 1) * bd, o2hi = NL > 1 ? min((band >> 1) * (bd + 1), h2) : 0;
    const int o3lo = (band >> 2) * bd, o3hi = NL > 2 ? min((band >> 2) * (bd + 1), h3) : 0;
    // the last source row the walk needs: the prefetch and the trip count's
    // round-up re-read it (a cache hit) instead of fetching rows past the band
    const int ylast = 2 * (r1s + n1 - 1) + 2;

    // rolling state: horizontal sums of source rows 2r1-2 .. 2r1+2 (hr[0..4]),
    // level-2 horizontal sums of level-1 rows (g2[0..4], newest last), level-3
    // horizontal sums of level-2 rows (g3[0..4])
    uint2 hr[5];
    uint32_t g2[5] = {0, 0, 0, 0, 0}, g3[5] = {0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 3; ++k) hr[k] = hsum_row(src_row16<GATHER>(sp, h0, xs, g, 2 * r1s - 2 + k, srs));
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
        pa[k] = src_row16<GATHER>(sp, h0, xs, g, min(2 * (r1s + k) + 1, ylast), srs);
        pb[k] = src_row16<GATHER>(sp, h0, xs, g, min(2 * (r1s + k) + 2, ylast), srs);
    }
    // Loads are issued unconditionally and stores branch only on wave-uniform
    // row conditions (rows of the band, mirrored ring rows): on gfx9 stores and
    // loads share vmcnt, and a store under a lane-divergent branch would make the
    // compiler wait for all earlier stores before using a prefetched row; a
    // uniform branch costs at most one extra counted op at the join.  Lanes that
    // own no output (lanes 0/1/62/63, columns past the level, no ring column)
    // store out of bounds (BUF) or to this lane's dword of the wave's trash line.
    uint32_t nsink = 0;
    auto body = [&](int k, auto slot_c) {
        constexpr int slot = decltype(slot_c)::value;
        const int r1 = r1s + k;
        hr[3] = hsum_row(pa[slot]);
        hr[4] = hsum_row(pb[slot]);
        pa[(slot + PF) % RS] = src_row16<GATHER>(sp, h0, xs, g, min(2 * (r1 + PF) + 1, ylast), srs);
        pb[(slot + PF) % RS] = src_row16<GATHER>(sp, h0, xs, g, min(2 * (r1 + PF) + 2, ylast), srs);
        // level-1 row r1
        uint32_t l1 = hibytes(vsum2(hr[0].x, hr[1].x, hr[2].x, hr[3].x, hr[4].x),
                              vsum2(hr[0].y, hr[1].y, hr[2].y, hr[3].y, hr[4].y));
        hr[0] = hr[2];
        hr[1] = hr[3];
        hr[2] = hr[4];
        if constexpr (GATHER == 1 || GATHER == 3) {
            if (st == 0) l1 = left_mirror_l1(l1, lane);  // wave-uniform
        }
        if (fix1) l1 = __builtin_amdgcn_perm(l1, wave_shr1(l1), sel1);
        if (r1 >= o1lo && r1 < o1hi) {  // wave-uniform: rows of the band
            const int a = c1 + 4 * (lane - 2);
            const bool ok = own_lane && a < w1;
            const PyrDst rb{rs, P + L.off[0] + PAD, (int)L.off[0] + PAD, tl};  // column 0 of padded row 0
            const int mr = mirror_row(r1, h1);  // the ring row holding this row's REFLECT_101 copy
            if constexpr ((SKIP & 1) != 0) {
                nsink ^= l1;
            } else {
                pyr_store<BUF, uint32_t>(rb, ok, a, r1 + PAD, p1, l1);
                if (mr != r1) pyr_store<BUF, uint32_t>(rb, ok, a, mr + PAD, p1, l1);
                if constexpr (SIDES) {
                    if (side1) {  // wave-uniform
                        const uint32_t nx = wave_shl1(l1), pv = wave_shr1(l1);
                        const bool lw = own_lane && a <= PAD - 4;
                        const bool rw = r1dw && own_lane && a >= w1 - PAD && a <= w1 - 4;
                        const uint32_t v = lw ? __builtin_amdgcn_perm(nx, l1, 0x01020304u)
                                              : __builtin_amdgcn_perm(l1, pv, 0x03040506u);
                        const int col = lw ? -a - 4 : 2 * w1 - 4 - a;
                        pyr_store<BUF, uint32_t>(rb, lw || rw, col, r1 + PAD, p1, v);
                        if (mr != r1)
                            pyr_store<BUF, uint32_t>(rb, lw || rw, col, mr + PAD, p1, v);
                        if (!r1dw) {  // odd widths: the right band byte by byte
#pragma unroll
                            for (int b = 0; b < 4; ++b) {
                                const int c = a + b, rc = ring_col(c, w1);
                                const bool wb = own_lane && rc > 0;
                                pyr_store<BUF, uint8_t>(rb, wb, rc, r1 + PAD, p1, (uint8_t)(l1 >> (8 * b)));
                                if (mr != r1) pyr_store<BUF, uint8_t>(rb, wb, rc, mr + PAD, p1, (uint8_t)(l1 >> (8 * b)));
                            }
                        }
                    }
                }
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
                    const int a = c2 + 2 * (lane - 2);
                    const bool ok = own_lane && a < w2;
                    const PyrDst rb{rs, P + L.off[1] + PAD, (int)L.off[1] + PAD, tl};
                    const int mr = mirror_row(r2, h2);
                    if constexpr ((SKIP & 2) != 0) {
                        nsink ^= l2 << 7;
                    } else {
                        pyr_store<BUF, uint16_t>(rb, ok, a, r2 + PAD, p2, (uint16_t)l2);
                        if (mr != r2)
                            pyr_store<BUF, uint16_t>(rb, ok, a, mr + PAD, p2, (uint16_t)l2);
                        if constexpr (SIDES) {
                            if (side2) {  // wave-uniform
#pragma unroll
                                for (int b = 0; b < 2; ++b) {
                                    const int rc = ring_col(a + b, w2);
                                    const bool wb = own_lane && rc != 0;
                                    const uint8_t v8 = (uint8_t)(l2 >> (8 * b));
                                    pyr_store<BUF, uint8_t>(rb, wb, rc, r2 + PAD, p2, v8);
                                    if (mr != r2) pyr_store<BUF, uint8_t>(rb, wb, rc, mr + PAD, p2, v8);
                                }
                            }
                        }
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
                        const int a = c3 + (lane - 2);
                        const bool ok = own_lane && a < w3;
                        const PyrDst rb{rs, P + L.off[2] + PAD, (int)L.off[2] + PAD, tl};
                        const int mr = mirror_row(r3, h3);
                        const uint8_t v8 = (uint8_t)(s3 >> 8);
                        if constexpr ((SKIP & 4) != 0) {
                            nsink ^= s3 << 13;
                        } else if (k >= 12 && r3 >= o3lo && r3 < o3hi) {
                            pyr_store<BUF, uint8_t>(rb, ok, a, r3 + PAD, p3, v8);
                            if (mr != r3) pyr_store<BUF, uint8_t>(rb, ok, a, mr + PAD, p3, v8);
                            if constexpr (SIDES) {
                                if (side3) {  // wave-uniform
                                    const int rc = ring_col(a, w3);
                                    const bool wb = own_lane && rc != 0;
                                    pyr_store<BUF, uint8_t>(rb, wb, rc, r3 + PAD, p3, v8);
                                    if (mr != r3) pyr_store<BUF, uint8_t>(rb, wb, rc, mr + PAD, p3, v8);
                                }
                            }
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

#ifdef GVX_KLT_TRACE
__device__ uint64_t* gvx_pyr_trace_buf;  // diagnostic build only (tools/pyr_residency.py)
#endif

// Work order (edge_first, r06): the edge strips (REFLECT_101 gathers, side
// bands) take ~52 us per wave at configs[1], an interior strip ~38 us
// (profiles/r06_l2/res_pyr).  Units are dispatched edge strips first, each
// strip's units image by image and band by band (vertical neighbours, which
// share their warm-up rows, in one XCD's L2), so the launch drains on the short
// interior waves.  edge_first = 0: strip-major within a band, the r05 order.
// WPB waves per workgroup: 1 frees a finished wave's slot at once (a 4-wave
// workgroup held its slots until its slowest wave ended, 17 us apart on average).
template <int NL, int SKIP = 0, int WPB = 1, bool SIDES = false>
__global__ void __launch_bounds__(64 * WPB, STREAM_OCC) stream_kernel(StreamSrc src, uint8_t* __restrict__ pyr,
                                                                  int64_t pyr_bytes, DownLevels L, int n_strips,
                                                                  int n_bands, int n_units, int band,
                                                                  uint8_t* __restrict__ trash, int edge_first) {
#ifdef GVX_KLT_TRACE
    WaveStamp wave_stamp_(gvx_pyr_trace_buf);
#endif
#ifdef PYR_PRIO
    __builtin_amdgcn_s_setprio(PYR_PRIO);  // A/B: the pass's waves issue first on a shared SIMD
#endif
    const int lane = threadIdx.x & 63;
    const int nblk = (n_units + WPB - 1) / WPB;
    const int unit = xcd_swizzle(blockIdx.x, nblk) * WPB + (WPB > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0);
    if (unit >= n_units) return;
    int st, bd, img;
    if (edge_first) {
        const int per = n_units / n_strips, k = unit / per, rest = unit - k * per;
        st = k == 0 ? 0 : k == 1 ? n_strips - 1 : k - 1;
        img = rest / n_bands;
        bd = rest - img * n_bands;
    } else {
        st = unit % n_strips;
        const int rest = unit / n_strips;
        bd = rest % n_bands;
        img = rest / n_bands;
    }
    uint8_t* const tl = trash + (int64_t)unit * 256 + 4 * lane;  // this wave's own line (no sharing)
    // wave-uniform strip classes: source columns past an edge of an unpadded
    // level 0 (lanes 0 / 63 read x0 = 480*st - 20 / 480*st + 484, 16 bytes), and
    // (SIDES) owned columns (240 / 120 / 60 per strip) that some side band copies
    const bool gl = src.raw && st == 0, gr = src.raw && ST_COLS * st + 8 * 63 - 20 + 16 > src.w;
    if constexpr (SIDES) {
        const int c1 = (ST_COLS / 2) * st;
        const bool side1 = L.sides[0] && (st == 0 || c1 + ST_COLS / 2 > L.w[0] - 1 - PAD);
        const bool side2 = NL > 1 && L.sides[1] && (st == 0 || c1 / 2 + ST_COLS / 4 > L.w[1] - 1 - PAD);
        const bool side3 = NL > 2 && L.sides[2] && (st == 0 || c1 / 4 + ST_COLS / 8 > L.w[2] - 1 - PAD);
        // one edge instance for both sides (fewer instances, fewer SGPRs spilled)
        if (gl || gr)
            stream_walk<NL, 3, true, SKIP>(src, pyr, pyr_bytes, L, st, bd, img, band, lane, tl, side1, side2, side3);
        else if (side1 || side2 || side3)
            stream_walk<NL, 0, true, SKIP>(src, pyr, pyr_bytes, L, st, bd, img, band, lane, tl, side1, side2, side3);
        else
            stream_walk<NL, 0, false, SKIP>(src, pyr, pyr_bytes, L, st, bd, img, band, lane, tl, false, false, false);
    } else {
        if (gl && gr)
            stream_walk<NL, 3, false, SKIP>(src, pyr, pyr_bytes, L, st, bd, img, band, lane, tl, false, false, false);
        else if (gl)
            stream_walk<NL, 1, false, SKIP>(src, pyr, pyr_bytes, L, st, bd, img, band, lane, tl, false, false, false);
        else if (gr)
            stream_walk<NL, 2, false, SKIP>(src, pyr, pyr_bytes, L, st, bd, img, band, lane, tl, false, false, false);
        else
            stream_walk<NL, 0, false, SKIP>(src, pyr, pyr_bytes, L, st, bd, img, band, lane, tl, false, false, false);
    }
}

// Levels whose top / bottom ring rows the pass writes (mirror_row): tall enough
// that every ring row is a single-bounce copy.  ring_kernel then writes only
// their side bands (every padded row); shorter levels get their whole ring there.
__host__ __device__ inline bool pass_writes_rows(int h) { return h >= RING_MIN; }
// SIDES passes also write the side bands of levels wide and tall enough
__host__ __device__ inline bool pass_writes_sides(int w, int h) { return w >= RING_MIN && h >= RING_MIN; }
// Launches smaller than the chip's wave slots (4 per SIMD) are latency-bound:
// their pass writes the side bands itself (one launch fewer); larger ones leave
// them to ring_kernel
inline bool stream_sides(int n_units, int n_cu) { return n_units < 16 * n_cu; }

// band height: BAND level-1 rows per wave when the batch fills the chip; a
// small batch (the live tracker's single frame or pair) takes narrower bands
// down to 4 rows: more waves, each walking band + 9 rows instead of BAND + 9 --
// less latency for more halo work on an otherwise idle GPU
inline int stream_band(int n_strips, int h1, int n_img, int n_cu) {
    int band = BAND;
    while (band > 4 && n_strips * ((h1 + band - 1) / band) * n_img < 4 * n_cu) band = std::max(4, (band >> 1) & ~3);
    // the same number of bands, balanced (a multiple of 4 rows each)
    const int n_bands = (h1 + band - 1) / band;
    return std::min(band, ((h1 + n_bands - 1) / n_bands + 3) / 4 * 4);
}

// *sides: whether the pass wrote the side bands of the levels pass_writes_sides names
template <int NL>
hipError_t launch_stream(gvx_ctx* c, const StreamSrc& src, int n_img, const PyrLayout& lay, int l0, uint8_t* dst,
                         bool* sides) {
    DownLevels D{};
    for (int k = 0; k < NL; ++k) {
        D.off[k] = lay.off[l0 + 1 + k];
        D.pitch[k] = lay.pitch[l0 + 1 + k];
        D.w[k] = lay.w[l0 + 1 + k];
        D.h[k] = lay.h[l0 + 1 + k];
        D.sides[k] = pass_writes_sides(D.w[k], D.h[k]);
    }
    const int n_strips = (D.w[0] + ST_COLS / 2 - 1) / (ST_COLS / 2);
    const int band = stream_band(n_strips, D.h[0], n_img, c->n_cu);
    const int n_bands = (D.h[0] + band - 1) / band;
    const int n_units = n_strips * n_bands * n_img;
    *sides = stream_sides(n_units, c->n_cu);
    // the SIDES instances' lanes without an output store to their wave's trash
    // line: the kernel must not run without it (a scratch buffer cannot grow
    // inside a capture)
    uint8_t* trash = (uint8_t*)scratch(c, "pyr_trash", (size_t)n_units * 256);
    if (!trash) return hipErrorOutOfMemory;
    if (*sides)
        return launch_timed(c, "pyramid", stream_kernel<NL, 0, 1, true>, dim3(N_XCD * xcd_per(n_units)), dim3(64),
                            0, src, dst, lay.bytes, D, n_strips, n_bands, n_units, band, trash, c->pyr_order);
    if (c->pyr_wpb == 4)
        return launch_timed(c, "pyramid", stream_kernel<NL, 0, 4>, dim3(N_XCD * xcd_per((n_units + 3) / 4)),
                            dim3(256), 0, src, dst, lay.bytes, D, n_strips, n_bands, n_units, band, trash,
                            c->pyr_order);
    return launch_timed(c, "pyramid", stream_kernel<NL, 0, 1>, dim3(N_XCD * xcd_per(n_units)), dim3(64), 0, src,
                        dst, lay.bytes, D, n_strips, n_bands, n_units, band, trash, c->pyr_order);
}


// ------------------------------------------------------------------ rings
// REFLECT_101 rings the streaming pass does not write, all images in one
// launch: for levels the pass writes the top / bottom ring rows of
// (pass_writes_rows), the side bands of every padded row; for shorter levels
// (the ring reflects more than once) the whole ring.  Item = one ring dword:
// [whole ring only: the top / bottom PAD rows over the padded width, then] per
// padded row the left PAD columns and the right columns [w, w+PAD) (dword
// aligned; bytes of the last interior dword rewrite their own value).
struct RingLevels {
    int32_t n;                  // levels
    int64_t off[MAX_LEVELS];
    int32_t pitch[MAX_LEVELS], w[MAX_LEVELS], h[MAX_LEVELS];
    int32_t dw[MAX_LEVELS];     // dwords per padded row (top/bottom bands)
    int32_t rd0[MAX_LEVELS];    // first dword (padded col / 4) of the right band
    int32_t rdn[MAX_LEVELS];    // dwords of the right band
    int32_t sides[MAX_LEVELS];  // 1: side bands only, over all h + 2*PAD padded rows
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

// Side bands of levels whose rows (ring rows included) the pass wrote, w a
// multiple of 4 and >= 36 (every side byte a single-bounce copy of an interior
// byte): the 32 ring bytes of a (padded row, side) are the 32 interior bytes next
// to the edge, reversed.  Eight lanes per (row, side), one output dword each: a
// dword pair of the mirrored row and one v_perm with a fixed selector, so a wave
// reads and writes 32-byte runs.  (ring_kernel's generic one-dword items took
// 33 us for configs[1]'s 512 images, profiles/r06_m8; one lane per (row, side)
// with 16-byte accesses was slower still, 64 rows per wave instruction.)
struct SideLevels {
    int32_t n;
    int64_t off[3];
    int32_t pitch[3], w[3], h[3];
};
__host__ __device__ inline bool side_fast(int w) { return (w & 3) == 0 && w >= 36; }
// Grid (items, images, levels): the level is wave-uniform, so the buffer view is
// an SGPR operand (a per-lane level would make every access a waterfall loop).
__global__ void __launch_bounds__(256) side_kernel(uint8_t* __restrict__ pyr, int64_t pyr_bytes, SideLevels S) {
    // a wave: 8 padded rows x 8 dwords of one side (the branch below is wave-uniform)
    const int k = blockIdx.z;
    const int t = blockIdx.x * 256 + threadIdx.x, q = t & 7, side = (t >> 6) & 1;
    const int prow = (t >> 7) * 8 + ((t >> 3) & 7), w = S.w[k], h = S.h[k], pitch = S.pitch[k];
    if (prow >= h + 2 * PAD) return;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        pyr + (int64_t)blockIdx.y * pyr_bytes + S.off[k], (short)0, (h + 2 * PAD) * pitch, 0x00020000);
    const int so = (refl(prow - PAD, h) + PAD) * pitch, dof = prow * pitch;
    typedef uint32_t v2u_t __attribute__((ext_vector_type(2)));
    if (side == 0) {
        // left: padded col 4q+b <- col 64-4q-b (D[t] = cols 32+4t .. 35+4t: D[8-q] byte 0,
        // D[7-q] bytes 3, 2, 1)
        const v2u_t d = __builtin_amdgcn_raw_buffer_load_b64(rs, so + PAD + 4 * (7 - q), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(d.y, d.x, 0x01020304u), rs, dof + 4 * q, 0, 0);
    } else {
        // right: padded col e+4q+b <- col e-2-4q-b, e = PAD + w (D[t] = dword (e-36)/4 + t:
        // D[8-q] bytes 2, 1, 0, D[7-q] byte 3)
        const int e = PAD + w;
        const v2u_t d = __builtin_amdgcn_raw_buffer_load_b64(rs, so + e - 36 + 4 * (7 - q), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_amdgcn_perm(d.x, d.y, 0x07000102u), rs, dof + e + 4 * q, 0,
                                              0);
    }
}

// The rings of levels lo..hi the streaming pass left (side_kernel, ring_kernel);
// pass_sides: the pass wrote the side bands of the levels pass_writes_sides
// names (none left).
hipError_t launch_rings(gvx_ctx* c, int n_img, const PyrLayout& lay, int lo, int hi, uint8_t* dst,
                        bool pass_sides) {
    RingLevels R{};
    SideLevels S{};
    int most = 0;
    for (int lv = lo; lv <= hi; ++lv) {
        const int w = lay.w[lv];
        if (pass_sides && pass_writes_sides(w, lay.h[lv])) continue;
        if (pass_writes_rows(lay.h[lv]) && side_fast(w) && S.n < 3) {
            const int k = S.n++;
            S.off[k] = lay.off[lv];
            S.pitch[k] = lay.pitch[lv];
            S.w[k] = w;
            S.h[k] = lay.h[lv];
            continue;
        }
        const int k = R.n++;
        R.off[k] = lay.off[lv];
        R.pitch[k] = lay.pitch[lv];
        R.w[k] = w;
        R.h[k] = lay.h[lv];
        R.dw[k] = (w + 2 * PAD + 3) / 4;
        R.rd0[k] = (w + PAD) / 4;
        R.rdn[k] = (w + 2 * PAD + 3) / 4 - R.rd0[k];
        R.sides[k] = pass_writes_rows(lay.h[lv]);
        R.items[k] = R.sides[k] ? (lay.h[lv] + 2 * PAD) * (PAD / 4 + R.rdn[k])
                                : 2 * PAD * R.dw[k] + lay.h[lv] * (PAD / 4 + R.rdn[k]);
        most = R.items[k] > most ? R.items[k] : most;
    }
    if (S.n > 0) {
        int most_s = 0;  // padded rows of the tallest level
        for (int k = 0; k < S.n; ++k) most_s = std::max(most_s, S.h[k] + 2 * PAD);
        const hipError_t e = launch_timed(c, "pyramid", side_kernel, dim3((128 * ((most_s + 7) / 8) + 255) / 256, n_img, S.n),
                                          dim3(256), 0, dst, lay.bytes, S);
        if (e != hipSuccess) return e;
    }
    if (R.n == 0) return hipSuccess;
    dim3 grid((most + 255) / 256, n_img, R.n);
    return launch_timed(c, "pyramid", ring_kernel, grid, dim3(256), 0, dst, lay.bytes, R);
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
                                 const PyrLayout& lay, uint8_t* dst, bool write_l0, const uint8_t* src_b, int n_a,
                                 bool l0_in_slot) {
    if (n_img <= 0) return hipSuccess;
    if (!src_b) n_a = n_img;
    // level-0 slot of the pyramid: pixel (0,0) of image 0
    uint8_t* slot0 = dst + lay.off[0] + (int64_t)PAD * lay.pitch[0] + PAD;
    if (l0_in_slot) {
        // the padded slot is the source of the first pass (ring included)
        src = slot0;
        img_stride = lay.bytes;
        stride = lay.pitch[0];
        src_b = nullptr;
        n_a = n_img;
        write_l0 = false;
    }
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
    const bool raw = !(write_l0 || !aligned) && !l0_in_slot;
    if (!raw && !l0_in_slot) {
        // full padded level-0 copy (ring included): the source of the build
        const int groups = (lay.w[0] + 2 * PAD + 15) / 16;
        const int items = groups * (lay.h[0] + 2 * PAD);
        dim3 grid((items + 255) / 256, n_img);
        const hipError_t e = launch_timed(c, "pyramid", level0_kernel, grid, dim3(256), 0, src, img_stride, stride,
                                          lay.w[0], lay.h[0], lay.pitch[0], lay.bytes, dst);
        if (e != hipSuccess) return e;
        s0 = slot0;
        s0_img = lay.bytes;
        s0_pitch = lay.pitch[0];
    }
    // levels 1.. in streaming passes of up to 3 levels; a later pass reads the
    // previous pass's deepest level (padded, its ring complete)
    int l = 0;
    while (l + 1 < lay.nlev) {
        const int nl = lay.nlev - 1 - l >= 3 ? 3 : lay.nlev - 1 - l;
        StreamSrc s{};
        s.a = l == 0 ? s0 : dst + lay.off[l] + (int64_t)PAD * lay.pitch[l] + PAD;
        s.b = l == 0 ? src_b : nullptr;  // the level-0 copy path never has two sources here
        s.n_a = l == 0 ? n_a : n_img;
        s.img_stride = l == 0 ? s0_img : lay.bytes;
        s.pitch = l == 0 ? s0_pitch : lay.pitch[l];
        s.w = lay.w[l];
        s.h = lay.h[l];
        s.raw = l == 0 && raw;
        bool sides = false;
        const hipError_t e = nl == 3   ? launch_stream<3>(c, s, n_img, lay, l, dst, &sides)
                             : nl == 2 ? launch_stream<2>(c, s, n_img, lay, l, dst, &sides)
                                       : launch_stream<1>(c, s, n_img, lay, l, dst, &sides);
        if (e != hipSuccess) return e;
        const hipError_t er = launch_rings(c, n_img, lay, l + 1, l + nl, dst, sides);
        if (er != hipSuccess) return er;
        l += nl;
    }
    return hipGetLastError();
}

}  // namespace gvx

#ifdef GVX_KLT_TRACE
// diagnostic build only: the wave-stamp buffer of stream_kernel (nullptr: off)
extern "C" int gvx_pyr_trace_set(void* buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(gvx::gvx_pyr_trace_buf), &buf, sizeof(buf));
}
#endif
