// klt.hip -- pyramidal Lucas-Kanade (fwd / fwd+bwd+FB) and compaction kernels
// for gfx950.  Replaces the four cv::calcOpticalFlowPyrLK calls per frame at
// /root/reference/ic_gvins/ic_gvins/tracking/tracking.cc:385,390,487,493 and the
// status / reduceVector logic at tracking.cc:396-408, :831-849.
//
// Design (DESIGN.md "KLT"):
//  * pyramids are built once per image (pyramid.hip) into a padded layout;
//  * the Scharr derivative planes are never materialised: each window's
//    derivative is computed in registers from the padded pyramid (zero outside
//    the image, as OpenCV's BORDER_CONSTANT derivative padding);
//  * the 21x21 window is 63 seven-pixel "units" (window row k/3, segment k%3):
//    one point per 64-lane wavefront (lane k owns unit k) for launches of up to
//    4,096 points, three per wave for larger ones in the exact order (21 lanes a
//    point, three vertically adjacent units a lane: lk_group3), two per wave in
//    the fp32 orders; window rows are read with aligned dword loads and
//    realigned with v_alignbyte;
//  * window values are kept as packed int16 pairs and the bilinear weights,
//    gradients and mismatch products run on v_dot2_i32_i16; every per-pixel
//    quantity is an exact integer, and the window sums are exact (int32 DPP
//    reductions, or a split fp64 route when a lane's partial could overflow) --
//    so the fp32 2x2 solve sees bit-identical inputs to
//    the CPU restatement (oracle/klt.c), whose LK outputs are matched bit-exactly.
#include <hip/hip_runtime.h>

#include <climits>

#include "gvx_internal.h"

namespace gvx {

namespace {

constexpr int W_BITS = 14;
constexpr float FLT_SCALE = 1.f / (1 << 20);

typedef short v2s __attribute__((ext_vector_type(2)));

typedef uint32_t v3u __attribute__((ext_vector_type(3)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// a.lo*b.lo + a.hi*b.hi + c on signed int16 halves (v_dot2_i32_i16)
__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, a), __builtin_bit_cast(v2s, b), c, false);
}
// the same with a wave-uniform addend taken straight from an SGPR (the VOP3P
// form: no per-accumulator v_mov of the rounding constant)
__device__ __forceinline__ int dot2k(uint32_t a, uint32_t b, int k) {
    int r;
    __asm__("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}
typedef unsigned short v2us __attribute__((ext_vector_type(2)));
// a.lo*b.lo + a.hi*b.hi + c on unsigned int16 halves (v_dot2_u32_u16)
__device__ __forceinline__ uint32_t udot2(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(v2us, a), __builtin_bit_cast(v2us, b), c, false);
}
__device__ __forceinline__ uint32_t udot2k(uint32_t a, uint32_t b, uint32_t k) {
    uint32_t r;
    __asm__("v_dot2_u32_u16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}
// (lo & 0xffff) | (hi << 16)
__device__ __forceinline__ uint32_t pack16(int lo, int hi) {
    return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u);
}
// signed int16 half `hi` of a packed pair
__device__ __forceinline__ int half16(uint32_t v, int hi) { return hi ? ((int)v >> 16) : (int)(short)(v & 0xffffu); }
// bytes (b[t], b[t+1]) of the 8-byte value {d1:d0} zero-extended to int16 halves
template <int T>
__device__ __forceinline__ uint32_t byte_pair(uint32_t d0, uint32_t d1) {
    return __builtin_amdgcn_perm(d1, d0, 0x0c000c00u | ((uint32_t)(T + 1) << 16) | (uint32_t)T);
}
// the same for byte T of a 12-byte row held in three dwords (T <= 10)
template <int T>
__device__ __forceinline__ uint32_t byte_pair3(const uint32_t (&d)[3]) {
    return byte_pair<(T & 3)>(d[T >> 2], d[(T >> 2) + 1 < 3 ? (T >> 2) + 1 : 2]);
}
__device__ __forceinline__ uint32_t psub16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2s, a) - __builtin_bit_cast(v2s, b));
}
__device__ __forceinline__ uint32_t padd16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2s, a) + __builtin_bit_cast(v2s, b));
}
// a*k + c on int16 halves (k small)
__device__ __forceinline__ uint32_t pmad16(uint32_t a, short k, uint32_t c) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2s, a) * k + __builtin_bit_cast(v2s, c));
}
__device__ __forceinline__ uint32_t pmul16(uint32_t a, short k) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2s, a) * k);
}
// (hi half of a, lo half of b): the pair starting one column later
__device__ __forceinline__ uint32_t shift_pair(uint32_t a, uint32_t b) {
    return __builtin_amdgcn_alignbit(b, a, 16);
}

// A pyramid level (or level-0 image) as a buffer resource: pixel (x, y) is at
// byte o0 + y*pitch + x (every offset the LK loop produces is non-negative).
struct Plane {
    __amdgpu_buffer_rsrc_t rs;
    int o0, pitch;
};
__device__ __forceinline__ Plane make_plane(const uint8_t* base, int o0, int pitch) {
    Plane p;
    p.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, 0x7fffffff, 0x00020000);
    p.o0 = o0;
    p.pitch = pitch;
    return p;
}
// NDW realigned dwords of a row starting at byte `off` (any alignment), the row
// `soff` bytes further (soff wave-uniform, in the SGPR soffset).
template <int NDW>
__device__ __forceinline__ void brow(const Plane& P, int off_al, uint32_t sh, int soff, uint32_t (&d)[NDW]) {
    if constexpr (NDW == 3) {
        const v4u w = __builtin_amdgcn_raw_buffer_load_b128(P.rs, off_al, soff, 0);
        d[0] = __builtin_amdgcn_alignbyte(w.y, w.x, sh);
        d[1] = __builtin_amdgcn_alignbyte(w.z, w.y, sh);
        d[2] = __builtin_amdgcn_alignbyte(w.w, w.z, sh);
    } else {
        const v3u w = __builtin_amdgcn_raw_buffer_load_b96(P.rs, off_al, soff, 0);
        d[0] = __builtin_amdgcn_alignbyte(w.y, w.x, sh);
        d[1] = __builtin_amdgcn_alignbyte(w.z, w.y, sh);
    }
}

// BORDER_REFLECT_101 index, branchless: exact for -(2*len-2) <= p <= 3*len-3;
// LK windows overshoot a level (> 21 px) by at most 26 px.
__device__ __forceinline__ int refl(int p, int len) {
    int a = abs(p);
    a = min(a, 2 * len - 2 - a);
    a = abs(a);
    return min(a, len - 1);
}
// Border windows of an unpadded plane (level 0 read in place): a point's lane
// group gathers its window -- rows y0 .. y0+rows-1, bytes x0 .. x0+31,
// REFLECT_101 outside the image (the values the padded ring of OpenCV's
// pyramid level holds there) -- into its own LDS tile once (byte buffer loads
// off the wave-uniform plane base), then every lane reads its rows from LDS
// like the aligned global path.
constexpr int WIN_DW = 8;  // dwords per LDS tile row
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int G>
__device__ __forceinline__ void fill_win(uint32_t* win, const Plane& P, int W, int H, int x0, int y0, int rows,
                                         int gl) {
    wave_lds_sync();  // earlier reads of the tile are done
#pragma unroll 1
    for (int i = gl; i < rows * WIN_DW; i += G) {
        const int r = i >> 3, q = i & 7;
        const int ro = P.o0 + refl(y0 + r, H) * P.pitch;
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
            v |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(P.rs, ro + refl(x0 + 4 * q + b, W), 0, 0) << (8 * b);
        win[i] = v;
    }
    wave_lds_sync();
}
template <int NDW>
__device__ __forceinline__ void read_win(const uint32_t* win, int row, int byteoff, uint32_t (&d)[NDW]) {
    const uint32_t* p = win + row * WIN_DW + (byteoff >> 2);
    const uint32_t sh = (uint32_t)(byteoff & 3);
    uint32_t w[NDW + 1];
#pragma unroll
    for (int k = 0; k <= NDW; ++k) w[k] = p[k];
#pragma unroll
    for (int k = 0; k < NDW; ++k) d[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
}

// The lane id, recomputed where it is used (volatile: never hoisted or kept
// live): everything lane-derived (the lane group, the window units, LDS slots,
// the point index) is rebuilt from it inside each LK pass, so nothing per-lane
// stays live across the forward and backward passes (where the register
// allocator spilled such values to scratch: 45 MB of writes per 256 pairs, r02).
__device__ __forceinline__ int lane_v() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// cvRound((1-a)(1-b) 2^14) ... in fp32 (LKTrackerInvoker), packed as int16 pairs
// W0 = (w00, w01), W1 = (w10, w11).  p*2^14 is exact, so fma(p, 2^14, 1.5*2^23)
// is 1.5*2^23 + cvRound(p*2^14) (round to nearest even, 0 <= p*2^14 <= 2^14)
// with the integer in the low mantissa bits; the packs read those bits and
// w11 = 2^14 - w00 - w01 - w10 is taken on the raw bit patterns (mod 2^32).
__device__ __forceinline__ void weights(float a, float b, uint32_t& W0, uint32_t& W1) {
    constexpr float M = 12582912.0f;  // 1.5 * 2^23, bit pattern 0x4B400000
    const float ra = 1.f - a, rb = 1.f - b;
    const uint32_t f00 = __float_as_uint(__builtin_fmaf(ra * rb, (float)(1 << W_BITS), M));
    const uint32_t f01 = __float_as_uint(__builtin_fmaf(a * rb, (float)(1 << W_BITS), M));
    const uint32_t f10 = __float_as_uint(__builtin_fmaf(ra * b, (float)(1 << W_BITS), M));
    const uint32_t f11 = ((1u << W_BITS) + 3u * 0x4B400000u) - (f00 + f01 + f10);
    W0 = __builtin_amdgcn_perm(f01, f00, 0x05040100u);
    W1 = __builtin_amdgcn_perm(f11, f10, 0x05040100u);
}


struct LkCfg {
    int max_iter;
    double crit_eps;
    float min_eig;
    int use_initial_flow;
    int want_err;  // compute the level-0 error (the status checks run regardless)
};

// One window unit: 7 pixels (cols 7*seg .. 7*seg+6 of window row `row`).
struct Unit {
    int row, seg;
    bool valid;
    uint32_t iv[4], ix[4], iy[4];  // packed int16 pairs (pixel 2k, 2k+1); pair 3 high = 0
};
// A lane's extracted window values live in LDS between the extraction and the
// iterations (registers hold only the unit being matched): slot (s, q) of lane
// `lane` at ust[(3*s + q)*64], ust = wave base + lane (16-B per lane, linear).
__device__ __forceinline__ void unit_put(v4u* ust, int s, const Unit& u) {
    ust[(3 * s + 0) * 64] = v4u{u.iv[0], u.iv[1], u.iv[2], u.iv[3]};
    ust[(3 * s + 1) * 64] = v4u{u.ix[0], u.ix[1], u.ix[2], u.ix[3]};
    ust[(3 * s + 2) * 64] = v4u{u.iy[0], u.iy[1], u.iy[2], u.iy[3]};
}
__device__ __forceinline__ void unit_get(const v4u* ust, int s, Unit& u) {
    const v4u a = ust[(3 * s + 0) * 64], b = ust[(3 * s + 1) * 64], c = ust[(3 * s + 2) * 64];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        u.iv[k] = a[k];
        u.ix[k] = b[k];
        u.iy[k] = c[k];
    }
}

// byte pair (T, T+1) of a 12-byte row in three dwords, as int16 halves (T <= 9;
// T is a constant after unrolling)
__device__ __forceinline__ uint32_t bpair(const uint32_t (&d)[3], int T) {
    const int q = T >> 2, r = T & 3;
    const uint32_t lo = d[q], hi = d[q + 1 < 3 ? q + 1 : 2];
    return __builtin_amdgcn_perm(hi, lo, 0x0c000c00u | ((uint32_t)(r + 1) << 16) | (uint32_t)r);
}

// Extract I (5 fractional bits) and the Scharr gradient at the bilinear
// window positions of one unit (LKTrackerInvoker window extraction), and
// accumulate its structure-tensor partial sums.
// d[r]: bytes X .. X+11 (X = ipx + 7*seg - 1) of rows ipy+row-1+r, r = 0..3.
// The Scharr taps run on int16 column pairs (v_pk_*): t0 = 3(a+e)+10b and
// t1 = e-a per column, dx = t0[c+1]-t0[c-1], dy = 3(t1[c+1]+t1[c-1])+10 t1[c],
// every value an exact integer of at most 13 bits.  `interior`: the whole
// window of every unit is inside the image (no derivative masking).
__device__ __forceinline__ void extract_unit(Unit& u, const uint32_t (&d)[4][3], int W, int H, int ipx,
                                             int ipy, bool interior, uint32_t W0, uint32_t W1, int& a11,
                                             int& a12, int& a22) {
    const int X = ipx + 7 * u.seg - 1;
    constexpr int RNDV = 1 << (W_BITS - 6), RNDD = 1 << (W_BITS - 1);
    // even-aligned column pairs (2k, 2k+1), k = 0..4, of the four rows
    uint32_t E[4][5];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int k = 0; k < 5; ++k) E[r][k] = bpair(d[r], 2 * k);
    int iv[7], ix[7], iy[7];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const uint32_t Wr = rr ? W1 : W0;
        // the derivatives are formed times 4 (|4 dI| <= 16320 fits int16; the
        // constants absorb the factor): the interpolated 4 (sum + 2^13) then
        // holds CV_DESCALE(sum, 14) in its high half, and one perm packs two
        // pixels' Ix (or Iy) without the two shifts
        uint32_t T0[5], T1[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            T0[k] = pmad16(padd16(E[rr][k], E[rr + 2][k]), 12, pmul16(E[rr + 1][k], 40));
            T1[k] = psub16(E[rr + 2][k], E[rr][k]);
        }
        // derivative pairs at columns (2k+1, 2k+2), k = 0..3
        uint32_t DX[4], DY[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            DX[k] = psub16(T0[k + 1], T0[k]);
            DY[k] = pmad16(padd16(T1[k + 1], T1[k]), 12, pmul16(shift_pair(T1[k], T1[k + 1]), 40));
        }
        if (!interior) {
            // derivatives are zero outside the image (BORDER_CONSTANT padding of
            // OpenCV's derivative pyramid)
            const bool row_in = (unsigned)(ipy + u.row + rr) < (unsigned)H;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const bool lo = row_in && (unsigned)(X + 2 * k + 1) < (unsigned)W;
                const bool hi = row_in && (unsigned)(X + 2 * k + 2) < (unsigned)W;
                const uint32_t m = (lo ? 0xffffu : 0u) | (hi ? 0xffff0000u : 0u);
                DX[k] &= m;
                DY[k] &= m;
            }
        }
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            // pixel pair (t+1, t+2): CV_DESCALE(sum, 9) for I, (sum, 14) for dI
            const int k = t >> 1;
            const uint32_t pv = (t & 1) ? E[rr + 1][k + 1] : bpair(d[rr + 1], t + 1);
            const uint32_t px = (t & 1) ? shift_pair(DX[k], DX[k + 1]) : DX[k];
            const uint32_t py = (t & 1) ? shift_pair(DY[k], DY[k + 1]) : DY[k];
            if (rr == 0) {
                iv[t] = dot2k(pv, Wr, RNDV);
                ix[t] = dot2k(px, Wr, 4 * RNDD);
                iy[t] = dot2k(py, Wr, 4 * RNDD);
            } else {
                iv[t] = dot2(pv, Wr, iv[t]);
                ix[t] = dot2(px, Wr, ix[t]);
                iy[t] = dot2(py, Wr, iy[t]);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int h = 2 * k + 1 < 7 ? 2 * k + 1 : 0;
        u.iv[k] = pack16(iv[2 * k] >> (W_BITS - 5), 2 * k + 1 < 7 ? iv[h] >> (W_BITS - 5) : 0);
        // (4 sum) >> 16 = sum >> 14 (arithmetic), the high halves of the two
        // pixels; the missing 8th pixel of the last pair is 0
        u.ix[k] = 2 * k + 1 < 7 ? __builtin_amdgcn_perm((uint32_t)ix[h], (uint32_t)ix[2 * k], 0x07060302u)
                                : __builtin_amdgcn_perm(0u, (uint32_t)ix[2 * k], 0x07060302u);
        u.iy[k] = 2 * k + 1 < 7 ? __builtin_amdgcn_perm((uint32_t)iy[h], (uint32_t)iy[2 * k], 0x07060302u)
                                : __builtin_amdgcn_perm(0u, (uint32_t)iy[2 * k], 0x07060302u);
    }
    int s11 = dot2k(u.ix[0], u.ix[0], 0), s12 = dot2k(u.ix[0], u.iy[0], 0), s22 = dot2k(u.iy[0], u.iy[0], 0);
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        s11 = dot2(u.ix[k], u.ix[k], s11);
        s12 = dot2(u.ix[k], u.iy[k], s12);
        s22 = dot2(u.iy[k], u.iy[k], s22);
    }
    // an invalid unit (k >= 63: lane 31's second unit) gets zero gradients, so its
    // products vanish in every iteration without a per-iteration select
    if (!u.valid) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            u.ix[k] = 0u;
            u.iy[k] = 0u;
        }
    }
    a11 = u.valid ? s11 : 0;
    a12 = u.valid ? s12 : 0;
    a22 = u.valid ? s22 : 0;
}

// The J window values of a unit from its two raw J rows r0 / r1 (bytes
// jx+7*seg .. +7 of rows jy+row and jy+row+1) as packed int16 pairs (pixel 2k,
// 2k+1; pair 3 high = 0): CV_DESCALE(w00 J00 + w01 J01 + w10 J10 + w11 J11,
// W_BITS - 5) on the signed v_dot2_i32_i16 (any w11, also the -1 / -2 that three
// separately rounded weights can leave it at).  The iterations use the spread
// rows below; this form serves the level-0 error.
__device__ __forceinline__ void j_pairs_signed(const uint32_t (&r0)[2], const uint32_t (&r1)[2], uint32_t W0,
                                               uint32_t W1, uint32_t (&jp)[4]) {
    constexpr int RND = 1 << (W_BITS - 6);
    int jv[8];
    jv[0] = dot2(byte_pair<0>(r1[0], r1[1]), W1, dot2k(byte_pair<0>(r0[0], r0[1]), W0, RND));
    jv[1] = dot2(byte_pair<1>(r1[0], r1[1]), W1, dot2k(byte_pair<1>(r0[0], r0[1]), W0, RND));
    jv[2] = dot2(byte_pair<2>(r1[0], r1[1]), W1, dot2k(byte_pair<2>(r0[0], r0[1]), W0, RND));
    jv[3] = dot2(byte_pair<3>(r1[0], r1[1]), W1, dot2k(byte_pair<3>(r0[0], r0[1]), W0, RND));
    jv[4] = dot2(byte_pair<4>(r1[0], r1[1]), W1, dot2k(byte_pair<4>(r0[0], r0[1]), W0, RND));
    jv[5] = dot2(byte_pair<5>(r1[0], r1[1]), W1, dot2k(byte_pair<5>(r0[0], r0[1]), W0, RND));
    jv[6] = dot2(byte_pair<6>(r1[0], r1[1]), W1, dot2k(byte_pair<6>(r0[0], r0[1]), W0, RND));
#pragma unroll
    for (int t = 0; t < 7; ++t) jv[t] >>= (W_BITS - 5);
    jv[7] = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) jp[k] = pack16(jv[2 * k], jv[2 * k + 1]);
}
// A J row of a unit cached between iterations as its even byte pairs, each byte
// times 128 in a uint16 half ("spread": h[k] = (b[2k], b[2k+1]) * 128, k = 0..3):
// the even pairs of an iteration are then free and each odd pair is one
// alignbit of two neighbours (3 operations a row, not 7 perms; the spread
// itself is formed once per reload, by 4 perms with run-time selectors straight
// from the loaded dwords and a packed shift).  Iterations mostly reuse the rows
// (sub-pixel steps).  With the bytes at 128 the bilinear sum is
// X = 128 (sum + 2^8), so the descaled value (sum + 2^8) >> 9 is X >> 16: one
// perm takes it for two pixels, no shift (the unsigned v_dot2_u32_u16: w11 >= 0).
__device__ __forceinline__ uint32_t spread_pair(const uint32_t (&h)[4], int t) {
    return (t & 1) ? shift_pair(h[t >> 1], h[(t >> 1) + 1]) : h[t >> 1];
}
// h from 12 loaded bytes {z:y:x} at byte offset sh (0..3): bytes sh .. sh+7
__device__ __forceinline__ void spread_row(uint32_t x, uint32_t y, uint32_t z, uint32_t sh, uint32_t (&h)[4]) {
    const uint32_t d = sh * 0x01000100u;
    const auto half = [](uint32_t v) {
        return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2us, v) >> (unsigned short)1);
    };
    h[0] = half(__builtin_amdgcn_perm(y, x, 0x010c000cu + d));
    h[1] = half(__builtin_amdgcn_perm(y, x, 0x030c020cu + d));
    h[2] = half(__builtin_amdgcn_perm(z, y, 0x010c000cu + d));
    h[3] = half(__builtin_amdgcn_perm(z, y, 0x030c020cu + d));
}
// the same from an 8-byte row already aligned
__device__ __forceinline__ void spread_row2(const uint32_t (&r)[2], uint32_t (&h)[4]) {
    spread_row(r[0], r[1], r[1], 0, h);
}
// the seven pixel pairs of a spread row (the odd ones are shifted pairs)
__device__ __forceinline__ void spread7(const uint32_t (&h)[4], uint32_t (&p)[7]) {
#pragma unroll
    for (int t = 0; t < 7; ++t) p[t] = spread_pair(h, t);
}
__device__ __forceinline__ void j_pairs_p(const uint32_t (&p0)[7], const uint32_t (&p1)[7], uint32_t W0, uint32_t W1,
                                          uint32_t (&jp)[4]) {
    constexpr uint32_t RND = 1u << (W_BITS - 6 + 7);
    uint32_t X[8];
#pragma unroll
    for (int t = 0; t < 7; ++t) X[t] = udot2(p1[t], W1, udot2k(p0[t], W0, RND));
    X[7] = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) jp[k] = __builtin_amdgcn_perm(X[2 * k + 1], X[2 * k], 0x07060302u);  // (X0 >> 16, X1 >> 16)
}
// the signed form (w11 < 0) from the spread pairs: plain bytes are the pairs >> 7
__device__ __forceinline__ void j_pairs_p_signed(const uint32_t (&p0)[7], const uint32_t (&p1)[7], uint32_t W0,
                                                 uint32_t W1, uint32_t (&jp)[4]) {
    constexpr int RND = 1 << (W_BITS - 6);
    const auto plain = [](uint32_t v) {
        return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2us, v) >> (unsigned short)7);
    };
    int jv[8];
#pragma unroll
    for (int t = 0; t < 7; ++t) jv[t] = dot2(plain(p1[t]), W1, dot2k(plain(p0[t]), W0, RND)) >> (W_BITS - 5);
    jv[7] = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) jp[k] = pack16(jv[2 * k], jv[2 * k + 1]);
}
__device__ __forceinline__ void j_pairs_h(const uint32_t (&h0)[4], const uint32_t (&h1)[4], uint32_t W0, uint32_t W1,
                                          uint32_t (&jp)[4]) {
    uint32_t p0[7], p1[7];
    spread7(h0, p0);
    spread7(h1, p1);
    j_pairs_p(p0, p1, W0, W1, jp);
}
__device__ __forceinline__ void j_pairs_h_signed(const uint32_t (&h0)[4], const uint32_t (&h1)[4], uint32_t W0,
                                                 uint32_t W1, uint32_t (&jp)[4]) {
    uint32_t p0[7], p1[7];
    spread7(h0, p0);
    spread7(h1, p1);
    j_pairs_p_signed(p0, p1, W0, W1, jp);
}
// an iteration's products of one unit: b1 += sum J Ix, b2 += sum J Iy (the I
// side of b = sum (J - I) I' is the level's constant, subtracted once)
template <bool SIGNED>
__device__ __forceinline__ void match_grad_u(const Unit& u, const uint32_t (&h0)[4], const uint32_t (&h1)[4],
                                             uint32_t W0, uint32_t W1, int& b1, int& b2) {
    uint32_t jp[4];
    if constexpr (SIGNED)
        j_pairs_h_signed(h0, h1, W0, W1, jp);
    else
        j_pairs_h(h0, h1, W0, W1, jp);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        b1 = dot2(jp[k], u.ix[k], b1);
        b2 = dot2(jp[k], u.iy[k], b2);
    }
}
// the level-0 error's part of one unit: es += sum |J - I| over its pixels
__device__ __forceinline__ void unit_abs_err(const Unit& u, const uint32_t (&r0)[2], const uint32_t (&r1)[2],
                                             uint32_t W0, uint32_t W1, bool valid, int& es) {
    uint32_t jp[4];
    j_pairs_signed(r0, r1, W0, W1, jp);
    int e = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t d = psub16(jp[k], u.iv[k]);  // diff pair
        const int dlo = (int)(short)(d & 0xffff), dhi = (int)(short)(d >> 16);
        e += (dlo < 0 ? -dlo : dlo) + (k < 3 ? (dhi < 0 ? -dhi : dhi) : 0);
    }
    es += valid ? e : 0;
}

// a unit's products for the fp32 orders: p1[t] = (float)(diff*Ix),
// p2[t] = (float)(diff*Iy) of the unit's 7 pixels (OpenCV converts the int32
// products, `ib1 += (itemtype)(diff*dIptr[0])`; |diff*Ix| < 2^25, round to
// nearest even like the CPU's int -> float conversion).
__device__ __forceinline__ uint32_t bp2(const uint32_t (&r)[2], int T) {
    return __builtin_amdgcn_perm(r[1], r[0], 0x0c000c00u | ((uint32_t)(T + 1) << 16) | (uint32_t)T);
}
__device__ __forceinline__ void match_unit_f32(const Unit& u, const uint32_t (&r0)[2], const uint32_t (&r1)[2],
                                               uint32_t W0, uint32_t W1, float (&p1)[7], float (&p2)[7]) {
    constexpr int RND = 1 << (W_BITS - 6);
#pragma unroll
    for (int t = 0; t < 7; ++t) {
        const int jv = dot2(bp2(r1, t), W1, dot2k(bp2(r0, t), W0, RND)) >> (W_BITS - 5);
        const int d = jv - half16(u.iv[t >> 1], t & 1);
        p1[t] = (float)__mul24(d, half16(u.ix[t >> 1], t & 1));
        p2[t] = (float)__mul24(d, half16(u.iy[t >> 1], t & 1));
    }
}

// Exact sums over a point's lane group (G = 16, 32 or 64 lanes, aligned):
// a butterfly, so every lane of the group ends with the group total --
// DPP quad / row mirrors inside 16-lane rows, then v_permlane16_swap /
// v_permlane32_swap across rows (CDNA4).
template <int G>
__device__ __forceinline__ int group_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false);   // quad_perm 1,0,3,2
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xf, 0xf, false);   // quad_perm 2,3,0,1
    v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xf, 0xf, false);  // row_half_mirror
    v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xf, 0xf, false);  // row_mirror
    if constexpr (G >= 32) {
        const auto r = __builtin_amdgcn_permlane16_swap((uint32_t)v, (uint32_t)v, false, false);
        v = (int)(r[0] + r[1]);
    }
    if constexpr (G >= 64) {
        const auto r = __builtin_amdgcn_permlane32_swap((uint32_t)v, (uint32_t)v, false, false);
        v = (int)(r[0] + r[1]);
    }
    return v;
}
// (float) of the exact group sums of per-lane values |v| < 2^31, round to
// nearest even: v = hi*2^10 + lo with lo in [0, 1024); the hi sums stay below
// 2^27 and two lo sums (< 2^16 each) share one packed chain; hi*2^10 + lo is
// exact in fp64 (|sum| < 2^37) and the fp64 -> fp32 conversion rounds once.
template <int G>
__device__ __forceinline__ void group_sums_f32(int v0, int v1, float& f0, float& f1) {
    const int h0 = group_sum<G>(v0 >> 10), h1 = group_sum<G>(v1 >> 10);
    const uint32_t l = (uint32_t)group_sum<G>((int)(((uint32_t)v0 & 1023u) | (((uint32_t)v1 & 1023u) << 16)));
    f0 = (float)__builtin_fma((double)h0, 1024.0, (double)(l & 0xffffu));
    f1 = (float)__builtin_fma((double)h1, 1024.0, (double)(l >> 16));
}
// The same sums when no lane's value reaches 2^31 / G in magnitude (2^26 for a
// 32-lane group; the usual case: the mismatch shrinks as the iterations
// converge): the group sum then stays below 2^31, so one int32 chain per sum
// and the int -> fp32 conversion (round to nearest even, as the fp64 route) give
// the same bits with 2 chains instead of 3 and no fp64 (wave-uniform choice)
template <int G>
__device__ __forceinline__ void group_sums_f32_fast(int v0, int v1, float& f0, float& f1) {
    constexpr int LIM = (int)((1u << 31) / G);
    const bool big = (v0 >= LIM || v0 <= -LIM) || (v1 >= LIM || v1 <= -LIM);
    if (__builtin_amdgcn_ballot_w64(big) == 0) {
        f0 = (float)group_sum<G>(v0);
        f1 = (float)group_sum<G>(v1);
    } else {
        group_sums_f32<G>(v0, v1, f0, f1);
    }
}
template <int G>
__device__ __forceinline__ float group_sum_f32(int v) {
    const int h = group_sum<G>(v >> 10), l = group_sum<G>(v & 1023);
    return (float)__builtin_fma((double)h, 1024.0, (double)l);
}

// ---- OpenCV's fp32 window-sum orders (gvx_klt_params.accum, oracle/klt.c
// ORC_ACC_F32 / ORC_ACC_F32X4) ----
// The products of one window sum are computed lane-parallel like the exact
// path, staged in the point group's LDS region, and summed in OpenCV's order
// by one lane per fp32 accumulator (a dependent chain: 441 adds for the scalar
// loop, at most 105 for the CV_SIMD128 lanes and the scalar tail); the finished
// accumulators are combined in OpenCV's reduction order by every lane.
// Region layout (floats), two arrays k = 0, 1 (two sums at once):
//  ACC 1 (scalar): array k at 512k; unit q's 7 pixels at 8q .. 8q+6 (window
//    pixel (y, x) is unit 3y + x/7, slot x%7: row-major order is unit order);
//    accumulator lane gl = k walks q = 0..62.
//  ACC 2 (SIMD4): array k at 540k; lane m = 0..3 (pixels x = m, m+4, m+8, m+12
//    of every row, index 4y + x/4) at 108m, the scalar tail (x = 16..20, index
//    5y + x - 16) at 432; zero padded to 108 per accumulator (adding +0 is
//    exact: no partial sum is -0); accumulator lane gl = 5k + m.
//  Accumulator results at ACC_RES + gl.
constexpr int ACC_RES = 1080, ACC_FLOATS = 1092;
template <int ACC>
constexpr int acc_chains() {
    return ACC == 1 ? 2 : 10;
}

// unit q's 7 values into array k
template <int ACC>
__device__ __forceinline__ void acc_put(float* scr, int k, int q, const float (&v)[7]) {
    if constexpr (ACC == 1) {
        float4* p = reinterpret_cast<float4*>(scr + 512 * k + 8 * q);
        p[0] = float4{v[0], v[1], v[2], v[3]};
        p[1] = float4{v[4], v[5], v[6], 0.f};
    } else {
        const int y = q / 3, x0 = 7 * (q - 3 * y);
        float* a = scr + 540 * k;
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            const int x = x0 + t;
            const int idx = x < 16 ? (x & 3) * 108 + 4 * y + (x >> 2) : 432 + 5 * y + (x - 16);
            a[idx] = v[t];
        }
    }
}
// zero the region once per wave (the SIMD4 pads are never written again)
template <int ACC, int G>
__device__ __forceinline__ void acc_clear(float* scr, int gl) {
    if constexpr (ACC != 0) {
        float4* p = reinterpret_cast<float4*>(scr);
        for (int i = gl; i < ACC_FLOATS / 4; i += G) p[i] = float4{0.f, 0.f, 0.f, 0.f};
    }
}
// the accumulator lanes' sequential sums; every lane of the group ends with
// the region's accumulators published at ACC_RES
template <int ACC>
__device__ __forceinline__ void acc_chains_run(float* scr, int gl) {
    wave_lds_sync();  // the products are in place
    float s = 0.f;
    if constexpr (ACC == 1) {
        const float4* p = reinterpret_cast<const float4*>(scr + 512 * (gl & 1));
#pragma unroll 9
        for (int q = 0; q < 63; ++q) {
            const float4 a = p[2 * q], b = p[2 * q + 1];
            s += a.x;
            s += a.y;
            s += a.z;
            s += a.w;
            s += b.x;
            s += b.y;
            s += b.z;
        }
    } else {
        const int c = gl < 10 ? gl : 9, k = c >= 5 ? 1 : 0, m = c - 5 * k;
        const float4* p = reinterpret_cast<const float4*>(scr + 540 * k + 108 * m);
#pragma unroll 9
        for (int i = 0; i < 27; ++i) {
            const float4 a = p[i];
            s += a.x;
            s += a.y;
            s += a.z;
            s += a.w;
        }
    }
    if (gl < acc_chains<ACC>()) scr[ACC_RES + gl] = s;
    wave_lds_sync();
}
// sum k of the region in OpenCV's reduction order (after acc_chains_run).
// A (qA..: lane x mod 4): tail + ((l0 + l1) + (l2 + l3)) (v_reduce_sum);
// b (qb0 = (b1, b2) of x%4 = 0, 1; qb1 of x%4 = 2, 3): tail + ((l0 + l2) + (l1 + l3))
// (v_interleave_pairs(qb0 + qb1), then the two-lane v_reduce_sum).
template <int ACC, bool B>
__device__ __forceinline__ float acc_result(const float* scr, int k) {
    if constexpr (ACC == 1) {
        return scr[ACC_RES + k];
    } else {
        const float* r = scr + ACC_RES + 5 * k;
        return B ? r[4] + ((r[0] + r[2]) + (r[1] + r[3])) : r[4] + ((r[0] + r[1]) + (r[2] + r[3]));
    }
}

// Window rows of a point's units: 4 rows x 12 bytes of I per unit for the
// extraction, 2 rows x 8 bytes of J for a match.  `raw` planes (level 0 read in
// place from the caller's image) take the aligned-load path only when every
// byte the window touches is inside the image, and gather with REFLECT_101
// otherwise; padded levels always take the aligned path (their PAD ring covers
// every window the LK loop admits).  lane_off[s] = row*pitch + 7*seg of unit s.
__device__ __forceinline__ void load_i_unit(const Unit& u, const Plane& P, int lane_off, int ipx, int ipy, bool fast,
                                            const uint32_t* win, uint32_t (&d)[4][3]) {
    if (fast) {
        const int off = lane_off + (P.o0 + (ipy - 1) * P.pitch + ipx - 1);
        const int al = off & ~3;
        const uint32_t sh = (uint32_t)off & 3u;
        brow<3>(P, al, sh, 0, d[0]);
        brow<3>(P, al, sh, P.pitch, d[1]);
        brow<3>(P, al, sh, 2 * P.pitch, d[2]);
        brow<3>(P, al, sh, 3 * P.pitch, d[3]);
    } else {
        // tile: rows ipy-1 .., bytes ipx-1 ..; the unit reads 4 rows x 12 bytes
#pragma unroll
        for (int r = 0; r < 4; ++r) read_win<3>(win, u.row + r, 7 * u.seg, d[r]);
    }
}
__device__ __forceinline__ void load_j_unit(const Unit& u, const Plane& P, int lane_off, int jx, int jy, bool fast,
                                            const uint32_t* win, uint32_t (&r0)[2], uint32_t (&r1)[2]) {
    if (fast) {
        const int off = lane_off + (P.o0 + jy * P.pitch + jx);
        const int al = off & ~3;
        const uint32_t sh = (uint32_t)off & 3u;
        brow<2>(P, al, sh, 0, r0);
        brow<2>(P, al, sh, P.pitch, r1);
    } else {
        // tile: rows jy .., bytes jx ..; the unit reads 2 rows x 8 bytes
        read_win<2>(win, u.row, 7 * u.seg, r0);
        read_win<2>(win, u.row + 1, 7 * u.seg, r1);
    }
}

// Level-0 planes of one pair: pointers to pixel (0,0), row pitch, and whether
// they are the caller's unpadded images.
struct L0Planes {
    const uint8_t* i;  // plane bases; pixel (0,0) at byte o0
    const uint8_t* j;
    int o0, pitch;
    bool raw;
};

// LKTrackerInvoker::operator() for one point across all levels (coarse to
// fine).  PPW points share a wavefront: each point has a group of G = 64/PPW
// lanes and lane gl of the group owns the PPW 7-pixel window units
// gl, gl+G, .. (unit k = window row k/3, segment k%3; unit 63 does not exist).
// The per-point scalar work (weights, sums, 2x2 solve, convergence) is thus
// issued once for PPW points.  I/J: padded pyramids of the prev / next image
// (levels >= 1); level 0 from `p0`.  Every per-point value below is uniform
// over the point's group; control flow diverges only between groups.
// ACC: the window-sum order (0 exact, 1 / 2 OpenCV's fp32 scalar / SIMD4
// orders through the group's LDS region `acc`).
// wins / units / accs: the wave's LDS bases (wave-uniform); the lane's slots
// are derived from lane_v() here.
template <int PPW, int ACC>
__device__ __forceinline__ void lk_group(const uint8_t* __restrict__ I, const uint8_t* __restrict__ J,
                                         const L0Planes& p0, const PyrLayout& lay, const LkCfg& cfg, float p0x,
                                         float p0y, float& nx, float& ny, int& status, float& err,
                                         uint32_t (*wins)[(WIN + 3) * WIN_DW], v4u* units, float (*accs)[ACC_FLOATS]) {
    constexpr int G = 64 / PPW, U = PPW;
    const int lane = lane_v(), grp = lane / G, gl = lane & (G - 1);
    uint32_t* win = wins[grp];
    v4u* ust = units + lane;
    float* acc = ACC ? accs[grp] : nullptr;
    Unit u[U];
#pragma unroll
    for (int s = 0; s < U; ++s) {
        const int k = gl + s * G;
        u[s].valid = k < 63;
        const int kc = k < 63 ? k : 62;
        u[s].row = kc / 3;
        u[s].seg = kc - 3 * u[s].row;
    }
    const float halfw = (float)((WIN - 1) * 0.5f);
    const int max_level = lay.nlev - 1;
    status = 1;
    err = 0.f;
    for (int l = max_level; l >= 0; --l) {
        const int W = lay.w[l], H = lay.h[l];
        const bool raw = l == 0 && p0.raw;
        const int pitch = l == 0 ? p0.pitch : lay.pitch[l];
        const int o0 = l == 0 ? p0.o0 : PAD * pitch + PAD;
        const Plane PI = make_plane(l == 0 ? p0.i : I + lay.off[l], o0, pitch);
        const Plane PJ = make_plane(l == 0 ? p0.j : J + lay.off[l], o0, pitch);
        int lane_off[U];
#pragma unroll
        for (int s = 0; s < U; ++s) lane_off[s] = __mul24(u[s].row, pitch) + 7 * u[s].seg;
        const float sc = ldexpf(1.f, -l);  // == (float)(1./(1 << l)), exact
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
        const float fpx = floorf(prevx), fpy = floorf(prevy);
        const int ipx = (int)fpx, ipy = (int)fpy;
        if (ipx < -WIN || ipx >= W || ipy < -WIN || ipy >= H) {
            if (l == 0) {
                status = 0;
                err = 0.f;
            }
            continue;
        }
        uint32_t W0, W1;
        weights(prevx - fpx, prevy - fpy, W0, W1);
        int a11 = 0, a12 = 0, a22 = 0;
        int c1 = 0, c2 = 0;  // the exact order's per-level I side of b (see lk_group3)
        {
            const bool fast = !raw || (ipx >= 4 && ipx + 30 <= W && ipy >= 1 && ipy + 23 <= H);
            if (!fast) fill_win<G>(win, PI, W, H, ipx - 1, ipy - 1, WIN + 3, gl);
            // every unit's derivative columns / rows inside the image
            const bool interior = ipx >= 0 && ipx + WIN + 1 <= W && ipy >= 0 && ipy + WIN + 1 <= H;
#pragma unroll
            for (int s = 0; s < U; ++s) {
                uint32_t d[4][3];
                load_i_unit(u[s], PI, lane_off[s], ipx, ipy, fast, win, d);
                int t11, t12, t22;
                extract_unit(u[s], d, W, H, ipx, ipy, interior, W0, W1, t11, t12, t22);
                a11 += t11;
                a12 += t12;
                a22 += t22;
                if constexpr (ACC == 0) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {  // invalid units: Ix = Iy = 0
                        c1 = dot2(u[s].iv[k], u[s].ix[k], c1);
                        c2 = dot2(u[s].iv[k], u[s].iy[k], c2);
                    }
                }
                // one unit per lane, or the fp32 orders (their occupancy is set by LDS, not
                // registers): kept in registers
                if constexpr (PPW > 1 && ACC == 0) unit_put(ust, s, u[s]);
            }
        }
        float A11, A12, A22;
        if constexpr (ACC == 0) {
            // the structure tensor: three int32 chains when every lane's partial
            // is below 2^31 / G (same bits as the split fp64 route, as for b)
            constexpr int LIM = (int)((1u << 31) / G);
            const bool big = (a11 >= LIM) || (a22 >= LIM) || (a12 >= LIM || a12 <= -LIM);  // a11, a22 >= 0
            if (__builtin_amdgcn_ballot_w64(big) == 0) {
                A11 = (float)group_sum<G>(a11);
                A12 = (float)group_sum<G>(a12);
                A22 = (float)group_sum<G>(a22);
            } else {
                group_sums_f32<G>(a11, a12, A11, A12);
                A22 = group_sum_f32<G>(a22);
            }
        } else {
            // Ix*Ix and Ix*Iy first, then Iy*Iy (exact int products < 2^24: the
            // float conversion is exact, as OpenCV's fx*fx of converted values)
            wave_lds_sync();  // the previous readers of the region are done
#pragma unroll
            for (int s = 0; s < U; ++s) {
                if (!u[s].valid) continue;
                float v0[7], v1[7];
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    const int x = half16(u[s].ix[t >> 1], t & 1), y = half16(u[s].iy[t >> 1], t & 1);
                    v0[t] = (float)__mul24(x, x);
                    v1[t] = (float)__mul24(x, y);
                }
                acc_put<ACC>(acc, 0, gl + s * G, v0);
                acc_put<ACC>(acc, 1, gl + s * G, v1);
            }
            acc_chains_run<ACC>(acc, gl);
            A11 = acc_result<ACC, false>(acc, 0);
            A12 = acc_result<ACC, false>(acc, 1);
#pragma unroll
            for (int s = 0; s < U; ++s) {
                if (!u[s].valid) continue;
                float v0[7];
#pragma unroll
                for (int t = 0; t < 7; ++t) {
                    const int y = half16(u[s].iy[t >> 1], t & 1);
                    v0[t] = (float)__mul24(y, y);
                }
                acc_put<ACC>(acc, 0, gl + s * G, v0);
            }
            acc_chains_run<ACC>(acc, gl);
            A22 = acc_result<ACC, false>(acc, 0);
        }
        A11 *= FLT_SCALE;
        A12 *= FLT_SCALE;
        A22 *= FLT_SCALE;
        float D = A11 * A22 - A12 * A12;
        const float minEig =
            __fdiv_rn(A22 + A11 - __fsqrt_rn((A11 - A22) * (A11 - A22) + 4.f * A12 * A12), (float)(2 * WIN * WIN));
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
        // the J rows of the last integer position: once the steps fall below a
        // pixel the window stays on the same pixel grid and only the bilinear
        // weights change, so the rows are reused instead of loaded again
        int cinx = INT_MIN, ciny = INT_MIN;
        // the exact path keeps the spread form (jh), the fp32 orders the bytes (jr)
        constexpr int JW = ACC == 0 ? 4 : 2;
        uint32_t jr0[U][JW], jr1[U][JW];
        // one exit, at the bottom: every loop-carried value is updated in place
        // (with the early exits the register allocator copied all of them -- the
        // cached J rows, the position, the previous step -- on every iteration)
        bool more = cfg.max_iter > 0;
        int j = 0;
        while (more) {
            const float fnx = floorf(nextx), fny = floorf(nexty);
            // a window off the level ends the point's iterations (status 0 at level
            // 0) with its position as it was.  The body still runs (no divergent
            // branch around it: see the reloads below) at a position clamped into
            // the padded level, and its result is discarded by the selects.
            const int fxi = (int)fnx, fyi = (int)fny;
            const int inx = min(max(fxi, -WIN), W - 1), iny = min(max(fyi, -WIN), H - 1);
            const bool oob = inx != fxi || iny != fyi;  // the clamp moved it: off the level
            uint32_t J0, J1;
            weights(nextx - fnx, nexty - fny, J0, J1);
            int b1 = -c1, b2 = -c2;  // b = sum J I' - sum I I' (exact order; c = 0 otherwise)
            // reload decisions are wave-uniform (ballots): a group whose position did
            // not move reloads the same rows, and a border window of either group
            // sends both groups through their LDS tiles (the tile path is correct for
            // any window).  Branches on a group's own conditions made the compiler
            // copy every cached row in and out of a second register set each
            // iteration, to keep the other group's values.
            if (__builtin_amdgcn_ballot_w64(inx != cinx || iny != ciny)) {
                const bool fast =
                    !__builtin_amdgcn_ballot_w64(raw && !(inx >= 3 && inx + 26 <= W && iny >= 0 && iny + 22 <= H));
                if (!fast) fill_win<G>(win, PJ, W, H, inx, iny, WIN + 1, gl);
                if (U > 1 && fast) {
                    // every unit's two rows in flight before the first is realigned
                    // (one memory round trip per reload, not one per unit; the
                    // compiler otherwise reuses one unit's load registers and waits
                    // in between: batch LK 0.449 -> 0.443 ms, r03 v39)
                    const int base = PJ.o0 + iny * PJ.pitch + inx;
                    v3u w0[U], w1[U];
                    uint32_t sh[U];
                    int al[U];
#pragma unroll
                    for (int s = 0; s < U; ++s) {
                        const int off = lane_off[s] + base;
                        al[s] = off & ~3;
                        sh[s] = (uint32_t)off & 3u;
                        w0[s] = __builtin_amdgcn_raw_buffer_load_b96(PJ.rs, al[s], 0, 0);
                        w1[s] = __builtin_amdgcn_raw_buffer_load_b96(PJ.rs, al[s], PJ.pitch, 0);
                    }
#pragma unroll
                    for (int s = 0; s < U; ++s) {
                        if constexpr (ACC == 0) {
                            spread_row(w0[s].x, w0[s].y, w0[s].z, sh[s], jr0[s]);
                            spread_row(w1[s].x, w1[s].y, w1[s].z, sh[s], jr1[s]);
                        } else {
                            jr0[s][0] = __builtin_amdgcn_alignbyte(w0[s].y, w0[s].x, sh[s]);
                            jr0[s][1] = __builtin_amdgcn_alignbyte(w0[s].z, w0[s].y, sh[s]);
                            jr1[s][0] = __builtin_amdgcn_alignbyte(w1[s].y, w1[s].x, sh[s]);
                            jr1[s][1] = __builtin_amdgcn_alignbyte(w1[s].z, w1[s].y, sh[s]);
                        }
                    }
                } else {
#pragma unroll
                    for (int s = 0; s < U; ++s) {
                        if constexpr (ACC == 0) {
                            uint32_t r0[2], r1[2];
                            load_j_unit(u[s], PJ, lane_off[s], inx, iny, fast, win, r0, r1);
                            spread_row2(r0, jr0[s]);
                            spread_row2(r1, jr1[s]);
                        } else {
                            load_j_unit(u[s], PJ, lane_off[s], inx, iny, fast, win, jr0[s], jr1[s]);
                        }
                    }
                }
                cinx = inx;
                ciny = iny;
            }
            float fb1, fb2;
            if constexpr (ACC == 0) {
                // a negative w11 anywhere in the wave (rare): the signed form (uniform branch)
                if (__builtin_amdgcn_ballot_w64((int)J1 < 0)) {
#pragma unroll
                    for (int s = 0; s < U; ++s) {
                        if constexpr (PPW > 1) unit_get(ust, s, u[s]);
                        match_grad_u<true>(u[s], jr0[s], jr1[s], J0, J1, b1, b2);  // invalid: Ix = Iy = 0
                    }
                } else {
#pragma unroll
                    for (int s = 0; s < U; ++s) {
                        if constexpr (PPW > 1) unit_get(ust, s, u[s]);
                        match_grad_u<false>(u[s], jr0[s], jr1[s], J0, J1, b1, b2);
                    }
                }
                group_sums_f32_fast<G>(b1, b2, fb1, fb2);
            } else {
                wave_lds_sync();  // the previous readers of the region are done
#pragma unroll
                for (int s = 0; s < U; ++s) {
                    float p1[7], p2[7];
                    match_unit_f32(u[s], jr0[s], jr1[s], J0, J1, p1, p2);
                    if (u[s].valid) {
                        acc_put<ACC>(acc, 0, gl + s * G, p1);
                        acc_put<ACC>(acc, 1, gl + s * G, p2);
                    }
                }
                acc_chains_run<ACC>(acc, gl);
                fb1 = acc_result<ACC, true>(acc, 0);
                fb2 = acc_result<ACC, true>(acc, 1);
            }
            fb1 *= FLT_SCALE;
            fb2 *= FLT_SCALE;
            const float dx = (A12 * fb2 - A22 * fb1) * D;
            const float dy = (A12 * fb1 - A11 * fb2) * D;
            const float tx = nextx + dx, ty = nexty + dy;
            // delta.ddot(delta) <= eps^2 in double: dx*dx is exact in fp64, so the fma rounds once like the sum
            const bool conv = __builtin_fma((double)dx, (double)dx, (double)dy * (double)dy) <= cfg.crit_eps;
            const bool osc = !conv && j > 0 && fabsf(dx + pdx) < 0.01f && fabsf(dy + pdy) < 0.01f;
            // (tx + halfw) - dx*0.5 in that order: next_pts = nextPt + halfWin, then -= delta*0.5
            const float ux = osc ? (tx + halfw) - dx * 0.5f : tx + halfw;
            const float uy = osc ? (ty + halfw) - dy * 0.5f : ty + halfw;
            nx = oob ? nx : ux;
            ny = oob ? ny : uy;
            nextx = oob ? nextx : tx;
            nexty = oob ? nexty : ty;
            status = (oob && l == 0) ? 0 : status;
            pdx = dx;
            pdy = dy;
            more = !oob && !conv && !osc && ++j < cfg.max_iter;
        }
        if (status && l == 0) {
            // final error (OPTFLOW_LK_GET_MIN_EIGENVALS not set)
            const float exf = nx - halfw, eyf = ny - halfw;
            const float fex = floorf(exf), fey = floorf(eyf);
            const int inx = (int)fex, iny = (int)fey;
            if (inx < -WIN || inx >= W || iny < -WIN || iny >= H) {
                status = 0;
                continue;
            }
            if (!cfg.want_err) continue;
            uint32_t J0, J1;
            weights(exf - fex, eyf - fey, J0, J1);
            int es = 0;
            {
                const bool fast = !raw || (inx >= 3 && inx + 26 <= W && iny >= 0 && iny + 22 <= H);
                if (!fast) fill_win<G>(win, PJ, W, H, inx, iny, WIN + 1, gl);
#pragma unroll
                for (int s = 0; s < U; ++s) {
                    uint32_t r0[2], r1[2];
                    load_j_unit(u[s], PJ, lane_off[s], inx, iny, fast, win, r0, r1);
                    if constexpr (PPW > 1 && ACC == 0) unit_get(ust, s, u[s]);
                    unit_abs_err(u[s], r0, r1, J0, J1, s < U - 1 || u[s].valid, es);
                }
            }
            err = __fdiv_rn((float)group_sum<G>(es) * 1.f, (float)(32 * WIN * WIN));
        }
    }
}

// ---- three points per wave (PPW 3, exact order) ----
// Point group g holds lanes 21g .. 21g+20 (lane 63 shadows lane 62 and belongs to
// no sum).  Lane gl of a group owns three vertically adjacent units: window
// rows 3(gl/3) .. 3(gl/3)+2 of segment gl%3.  Three units share their
// derivative rows (4 instead of 6) and their J rows (4 instead of 6), and the
// per-point scalar work is issued once for three points.
constexpr int G3 = 21;
__device__ __forceinline__ int grp3(int lane) { return lane < G3 ? 0 : lane < 2 * G3 ? 1 : 2; }

// inclusive prefix sum over the wave, modulo 2^32 (DPP row shifts, then the row
// broadcasts of lanes 15 and 31).  Groups that have left the loop are disabled
// lanes: a DPP read of a disabled lane is invalid, so the write is skipped and
// the add takes `old` = 0.  Such lanes contribute nothing, and a group is a
// contiguous run of lanes, so the difference gsum3 takes inside an active group
// is exact whatever the other groups are doing (checked by a lane-level model
// of the scan over random activity patterns).
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 (rows 1, 3)
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 (rows 2, 3)
    return v;
}
// the total of v over the lane's point group: the inclusive scan at the group's
// last lane minus the exclusive scan at its first, both read by ds_bpermute
// (ga = 4 * first lane).  Modulo 2^32, so exact whenever the total fits int32.
__device__ __forceinline__ int gsum3(int v, int ga) {
    const uint32_t s = wave_scan((uint32_t)v);
    const uint32_t e = (uint32_t)__builtin_amdgcn_ds_bpermute(ga + 4 * (G3 - 1), (int)s);
    const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(ga, (int)(s - (uint32_t)v));
    return (int)(e - b);
}
// group_sums_f32 / group_sums_f32_fast / group_sum_f32 over the 21-lane groups
// (the packed lo halves stay below 2^16 over the whole wave: 63 * 1023)
__device__ __forceinline__ void gsums_f32_3(int v0, int v1, float& f0, float& f1, int ga) {
    const int h0 = gsum3(v0 >> 10, ga), h1 = gsum3(v1 >> 10, ga);
    const uint32_t l = (uint32_t)gsum3((int)(((uint32_t)v0 & 1023u) | (((uint32_t)v1 & 1023u) << 16)), ga);
    f0 = (float)__builtin_fma((double)h0, 1024.0, (double)(l & 0xffffu));
    f1 = (float)__builtin_fma((double)h1, 1024.0, (double)(l >> 16));
}
constexpr int LIM3 = (int)((1u << 31) / G3);
__device__ __forceinline__ void gsums_f32_fast3(int v0, int v1, float& f0, float& f1, int ga) {
    const bool big = (v0 >= LIM3 || v0 <= -LIM3) || (v1 >= LIM3 || v1 <= -LIM3);
    if (__builtin_amdgcn_ballot_w64(big) == 0) {
        f0 = (float)gsum3(v0, ga);
        f1 = (float)gsum3(v1, ga);
    } else {
        gsums_f32_3(v0, v1, f0, f1, ga);
    }
}
__device__ __forceinline__ float gsum_f32_3(int v, int ga) {
    const int h = gsum3(v >> 10, ga), l = gsum3(v & 1023, ga);
    return (float)__builtin_fma((double)h, 1024.0, (double)l);
}

// fill_win by the wave's active lanes (the groups still on this level): the one
// tile of the wave serves the groups in turn
__device__ __forceinline__ void fill_win_active(uint32_t* win, const Plane& P, int W, int H, int x0, int y0,
                                                int rows) {
    const uint64_t ex = __builtin_amdgcn_read_exec();
    const int n = __builtin_popcountll(ex);
    const int first = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(ex >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ex, 0u));
    wave_lds_sync();  // earlier reads of the tile are done
#pragma unroll 1
    for (int i = first; i < rows * WIN_DW; i += n) {
        const int r = i >> 3, q = i & 7;
        const int ro = P.o0 + refl(y0 + r, H) * P.pitch;
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b)
            v |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(P.rs, ro + refl(x0 + 4 * q + b, W), 0, 0) << (8 * b);
        win[i] = v;
    }
    wave_lds_sync();
}

// The J side of match_unit_h for unit slot s: b1 += sum J Ix, b2 += sum J Iy over
// its pixels (the gradients read from the slot; I is not needed)
template <bool SIGNED>
__device__ __forceinline__ void match_grad_p(const v4u* ust, int s, const uint32_t (&p0)[7], const uint32_t (&p1)[7],
                                             uint32_t W0, uint32_t W1, int& b1, int& b2) {
    const v4u gx = ust[(3 * s + 1) * 64], gy = ust[(3 * s + 2) * 64];
    uint32_t jp[4];
    if constexpr (SIGNED)
        j_pairs_p_signed(p0, p1, W0, W1, jp);
    else
        j_pairs_p(p0, p1, W0, W1, jp);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        b1 = dot2(jp[k], gx[k], b1);
        b2 = dot2(jp[k], gy[k], b2);
    }
}
template <bool SIGNED>
__device__ __forceinline__ void match_grad_h(const v4u* ust, int s, const uint32_t (&h0)[4], const uint32_t (&h1)[4],
                                             uint32_t W0, uint32_t W1, int& b1, int& b2) {
    uint32_t p0[7], p1[7];
    spread7(h0, p0);
    spread7(h1, p1);
    match_grad_p<SIGNED>(ust, s, p0, p1, W0, W1, b1, b2);
}

// A lane's three units from its six source rows d[r] (bytes X .. X+11, X =
// ipx + 7 seg - 1, of rows y0 - 1 + r, y0 = ipy + 3 rb): the Scharr rows at
// window rows 3rb .. 3rb+3 are formed once each; unit j takes derivative rows j
// (weights W0) and j+1 (W1), exactly as extract_unit does for one unit.  Each
// finished unit goes to its LDS slot; the structure-tensor partials of the
// three are summed into a11 / a12 / a22.
__device__ __forceinline__ void extract_triple(const uint32_t (&d)[6][3], int X, int y0, int W, int H,
                                               bool interior, uint32_t W0, uint32_t W1, v4u* ust, int& a11,
                                               int& a12, int& a22, int& c1, int& c2) {
    constexpr int RNDV = 1 << (W_BITS - 6), RNDD = 1 << (W_BITS - 1);
    uint32_t E[6][5];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int k = 0; k < 5; ++k) E[r][k] = bpair(d[r], 2 * k);
    // column masks for border windows, formed only when the wave holds one
    uint32_t cm[4] = {~0u, ~0u, ~0u, ~0u};
    if (__builtin_amdgcn_ballot_w64(!interior)) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool lo = (unsigned)(X + 2 * k + 1) < (unsigned)W;
            const bool hi = (unsigned)(X + 2 * k + 2) < (unsigned)W;
            cm[k] = (lo ? 0xffffu : 0u) | (hi ? 0xffff0000u : 0u);
        }
    }
    int iv[7], ix[7], iy[7];
    a11 = a12 = a22 = 0;
    c1 = c2 = 0;
#pragma unroll
    for (int dd = 0; dd < 4; ++dd) {
        // derivative row dd (times 4, as extract_unit)
        uint32_t T0[5], T1[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            T0[k] = pmad16(padd16(E[dd][k], E[dd + 2][k]), 12, pmul16(E[dd + 1][k], 40));
            T1[k] = psub16(E[dd + 2][k], E[dd][k]);
        }
        uint32_t DX[4], DY[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            DX[k] = psub16(T0[k + 1], T0[k]);
            DY[k] = pmad16(padd16(T1[k + 1], T1[k]), 12, pmul16(shift_pair(T1[k], T1[k + 1]), 40));
        }
        if (!interior) {
            const bool row_in = (unsigned)(y0 + dd) < (unsigned)H;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t m = row_in ? cm[k] : 0u;
                DX[k] &= m;
                DY[k] &= m;
            }
        }
        // both output rows that use derivative row dd read I from source row dd+1
#pragma unroll
        for (int rr = 1; rr >= 0; --rr) {
            // rr = 1: the second half of unit dd-1 (W1); rr = 0: the first half of unit dd (W0)
            if (rr == 1 && dd == 0) continue;
            if (rr == 0 && dd == 3) continue;
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                const int k = t >> 1;
                const uint32_t pv = (t & 1) ? E[dd + 1][k + 1] : bpair(d[dd + 1], t + 1);
                const uint32_t px = (t & 1) ? shift_pair(DX[k], DX[k + 1]) : DX[k];
                const uint32_t py = (t & 1) ? shift_pair(DY[k], DY[k + 1]) : DY[k];
                if (rr == 0) {
                    iv[t] = dot2k(pv, W0, RNDV);
                    ix[t] = dot2k(px, W0, 4 * RNDD);
                    iy[t] = dot2k(py, W0, 4 * RNDD);
                } else {
                    iv[t] = dot2(pv, W1, iv[t]);
                    ix[t] = dot2(px, W1, ix[t]);
                    iy[t] = dot2(py, W1, iy[t]);
                }
            }
            if (rr == 1) {
                // unit dd-1 is complete
                Unit u;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int h = 2 * k + 1 < 7 ? 2 * k + 1 : 0;
                    u.iv[k] = pack16(iv[2 * k] >> (W_BITS - 5), 2 * k + 1 < 7 ? iv[h] >> (W_BITS - 5) : 0);
                    u.ix[k] = 2 * k + 1 < 7 ? __builtin_amdgcn_perm((uint32_t)ix[h], (uint32_t)ix[2 * k], 0x07060302u)
                                            : __builtin_amdgcn_perm(0u, (uint32_t)ix[2 * k], 0x07060302u);
                    u.iy[k] = 2 * k + 1 < 7 ? __builtin_amdgcn_perm((uint32_t)iy[h], (uint32_t)iy[2 * k], 0x07060302u)
                                            : __builtin_amdgcn_perm(0u, (uint32_t)iy[2 * k], 0x07060302u);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    a11 = dot2(u.ix[k], u.ix[k], a11);
                    a12 = dot2(u.ix[k], u.iy[k], a12);
                    a22 = dot2(u.iy[k], u.iy[k], a22);
                    c1 = dot2(u.iv[k], u.ix[k], c1);
                    c2 = dot2(u.iv[k], u.iy[k], c2);
                }
                unit_put(ust, dd - 1, u);
            }
        }
    }
}

// lk_group for three points per wave (exact order only): the same algorithm and
// the same selects, with the units, rows and sums of the triple layout.
// klt_phase_kernel: the flow a phase starts from arrives from the previous
// phase's wave; `resolve(nx, ny)` supplies it before the first level.  (Resolving
// it after the top level's extraction, to hide the load behind the extraction's
// own, costs 5 spilled VGPRs at 128.)  A whole-chain call resolves nothing.
// KLT_LONE: when one group of the three is left iterating a level, the wave
// finishes that point with one unit per lane over all 64 lanes (lone mode, in
// lk_group3) instead of 21 lanes doing three units each.  Bit-identical (the
// parity suite passes on it), but slower on the configs[1] headline: 0.455-0.457
// against 0.427-0.431 ms per step (profiles/r06_ab, r06_a11).  The switch, the
// J-row reload and the state hand-off cost more than the 17 % of wave-iterations
// that run one group save.  Off.
#ifndef KLT_LONE
#define KLT_LONE 0
#endif
#if KLT_LONE
__device__ __forceinline__ uint64_t gmask3(int g) {
    return g == 0 ? (1ull << G3) - 1 : g == 1 ? ((1ull << G3) - 1) << G3 : ~0ull << (2 * G3);
}
#endif
struct NoResolve {
    __device__ void operator()(float&, float&) const {}
};
template <typename Resolve = NoResolve>
__device__ __forceinline__ void lk_group3(const uint8_t* __restrict__ I, const uint8_t* __restrict__ J,
                                          const L0Planes& p0, const PyrLayout& lay, const LkCfg& cfg, float p0x,
                                          float p0y, float& nx, float& ny, int& status, float& err, uint32_t* win,
                                          v4u* units, int l_top = 99, int l_bot = 0,
                                          const Resolve& resolve = Resolve()) {
    int rb, seg, ga;
    {
        const int lane = lane_v(), g = grp3(lane), gl = min(lane - G3 * g, G3 - 1);  // lane 63 shadows lane 62
        rb = gl / 3;
        seg = gl - 3 * rb;
        ga = 4 * G3 * g;
    }
    v4u* ust = units + lane_v();
    const float halfw = (float)((WIN - 1) * 0.5f);
    const int max_level = lay.nlev - 1;
    status = 1;  // only level 0 clears it: a phase of levels > 0 (klt_phase_kernel) leaves it
    err = 0.f;
    // levels l_top .. l_bot (the whole pyramid by default); nx, ny carry the
    // flow between levels, in level-(l+1) pixels when l_top < max_level
    resolve(nx, ny);
    for (int l = min(l_top, max_level); l >= l_bot; --l) {
        const int W = lay.w[l], H = lay.h[l];
        const bool raw = l == 0 && p0.raw;
        const int pitch = l == 0 ? p0.pitch : lay.pitch[l];
        const int o0 = l == 0 ? p0.o0 : PAD * pitch + PAD;
        const Plane PI = make_plane(l == 0 ? p0.i : I + lay.off[l], o0, pitch);
        const Plane PJ = make_plane(l == 0 ? p0.j : J + lay.off[l], o0, pitch);
        const int lane_off = __mul24(3 * rb, pitch) + 7 * seg;
        const float sc = ldexpf(1.f, -l);
        const float psx = p0x * sc, psy = p0y * sc;
        float prevx = psx, prevy = psy;
        float nextx, nexty;
        // the level's starting flow (nx, ny become it)
        auto start_flow = [&]() {
            if (l == max_level) {
                if (cfg.use_initial_flow) {
                    nextx = nx * sc;
                    nexty = ny * sc;
                } else {
                    nextx = psx;
                    nexty = psy;
                }
            } else {
                nextx = nx * 2.f;
                nexty = ny * 2.f;
            }
            nx = nextx;
            ny = nexty;
        };
        start_flow();
        prevx -= halfw;
        prevy -= halfw;
        const float fpx = floorf(prevx), fpy = floorf(prevy);
        const int ipx = (int)fpx, ipy = (int)fpy;
        if (ipx < -WIN || ipx >= W || ipy < -WIN || ipy >= H) {
            if (l == 0) {
                status = 0;
                err = 0.f;
            }
            continue;
        }
        uint32_t W0, W1;
        weights(prevx - fpx, prevy - fpy, W0, W1);
        int a11, a12, a22, c1, c2;
        {
            uint32_t d[6][3];
            const bool fast = !raw || (ipx >= 4 && ipx + 30 <= W && ipy >= 1 && ipy + 23 <= H);
            if (__builtin_amdgcn_ballot_w64(!fast) == 0) {
                const int off = lane_off + (PI.o0 + (ipy - 1) * PI.pitch + ipx - 1);
                const int al = off & ~3;
                const uint32_t sh = (uint32_t)off & 3u;
#pragma unroll
                for (int r = 0; r < 6; ++r) brow<3>(PI, al, sh, r * PI.pitch, d[r]);
            } else {
                // a border window in the wave: every group's rows from the tile, one group at a time
                // (d defined before the selects: a select against an undefined value may fold away)
                const int g = grp3(lane_v());
#pragma unroll
                for (int r = 0; r < 6; ++r) d[r][0] = d[r][1] = d[r][2] = 0u;
#pragma unroll
                for (int gs = 0; gs < 3; ++gs) {
                    if (__builtin_amdgcn_ballot_w64(g == gs) == 0) continue;  // group gs is off this level
                    const int gx = __builtin_amdgcn_readlane(ipx, G3 * gs), gy = __builtin_amdgcn_readlane(ipy, G3 * gs);
                    fill_win_active(win, PI, W, H, gx - 1, gy - 1, WIN + 3);
#pragma unroll
                    for (int r = 0; r < 6; ++r) {
                        uint32_t t[3];
                        read_win<3>(win, 3 * rb + r, 7 * seg, t);
#pragma unroll
                        for (int q = 0; q < 3; ++q) d[r][q] = g == gs ? t[q] : d[r][q];
                    }
                }
            }
            const bool interior = ipx >= 0 && ipx + WIN + 1 <= W && ipy >= 0 && ipy + WIN + 1 <= H;
            extract_triple(d, ipx + 7 * seg - 1, ipy + 3 * rb, W, H, interior, W0, W1, ust, a11, a12, a22, c1, c2);
        }
        float A11, A12, A22;
        {
            const bool big = (a11 >= LIM3) || (a22 >= LIM3) || (a12 >= LIM3 || a12 <= -LIM3);  // a11, a22 >= 0
            if (__builtin_amdgcn_ballot_w64(big) == 0) {
                A11 = (float)gsum3(a11, ga);
                A12 = (float)gsum3(a12, ga);
                A22 = (float)gsum3(a22, ga);
            } else {
                gsums_f32_3(a11, a12, A11, A12, ga);
                A22 = gsum_f32_3(a22, ga);
            }
        }
        A11 *= FLT_SCALE;
        A12 *= FLT_SCALE;
        A22 *= FLT_SCALE;
        float D = A11 * A22 - A12 * A12;
        const float minEig =
            __fdiv_rn(A22 + A11 - __fsqrt_rn((A11 - A22) * (A11 - A22) + 4.f * A12 * A12), (float)(2 * WIN * WIN));
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
        int cinx = INT_MIN, ciny = INT_MIN;
        // the lane's four J rows as their seven spread pixel pairs, formed once per
        // reload.  Defined here by an empty asm: an undefined start lets the rows live
        // across the levels (spills at 128 VGPRs), and zeros cost a move per register
        uint32_t jr[4][7];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < 7; ++t) asm volatile("" : "=v"(jr[r][t]));
        bool more = cfg.max_iter > 0;
        int j = 0;
#if KLT_LONE
        // lone mode needs every lane: all three groups start the level's iterations
        const bool lone_ok = __builtin_amdgcn_ballot_w64(true) == ~0ull;
#endif
        while (more) {
#if KLT_LONE
            if (lone_ok) {
                const uint64_t m = __builtin_amdgcn_ballot_w64(true);
                const int g = grp3(__builtin_ctzll(m));
                if ((m & ~gmask3(g)) == 0) {
                    // one group left: its state goes through the (idle) tile, not
                    // through registers live out of the loop
                    const int k = lane_v() - G3 * g;
                    if (k == 0) {
                        win[0] = __builtin_bit_cast(uint32_t, nextx);
                        win[1] = __builtin_bit_cast(uint32_t, nexty);
                        win[2] = __builtin_bit_cast(uint32_t, pdx);
                        win[3] = __builtin_bit_cast(uint32_t, pdy);
                        win[4] = (uint32_t)j;
                        win[5] = __builtin_bit_cast(uint32_t, A11);
                        win[6] = __builtin_bit_cast(uint32_t, A12);
                        win[7] = __builtin_bit_cast(uint32_t, A22);
                        win[8] = __builtin_bit_cast(uint32_t, D);
                    }
                    if (k < G3) {
                        win[32 + k] = (uint32_t)c1;
                        win[64 + k] = (uint32_t)c2;
                    }
                    break;
                }
            }
#endif
            const float fnx = floorf(nextx), fny = floorf(nexty);
            const int fxi = (int)fnx, fyi = (int)fny;
            const int inx = min(max(fxi, -WIN), W - 1), iny = min(max(fyi, -WIN), H - 1);
            const bool oob = inx != fxi || iny != fyi;  // the clamp moved it: off the level
            uint32_t J0, J1;
            weights(nextx - fnx, nexty - fny, J0, J1);
            if (__builtin_amdgcn_ballot_w64(inx != cinx || iny != ciny)) {
                const bool fast = !raw || (inx >= 3 && inx + 26 <= W && iny >= 0 && iny + 22 <= H);
                if (__builtin_amdgcn_ballot_w64(!fast) == 0) {
                    const int off = lane_off + (PJ.o0 + iny * PJ.pitch + inx);
                    const int al = off & ~3;
                    const uint32_t sh = (uint32_t)off & 3u;
                    v3u w[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) w[r] = __builtin_amdgcn_raw_buffer_load_b96(PJ.rs, al, r * PJ.pitch, 0);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        uint32_t h[4];
                        spread_row(w[r].x, w[r].y, w[r].z, sh, h);
                        spread7(h, jr[r]);
                    }
                } else {
                    const int g = grp3(lane_v());
                    uint32_t nj[4][4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) nj[r][0] = nj[r][1] = nj[r][2] = nj[r][3] = 0u;
#pragma unroll
                    for (int gs = 0; gs < 3; ++gs) {
                        if (__builtin_amdgcn_ballot_w64(g == gs) == 0) continue;
                        const int gx = __builtin_amdgcn_readlane(inx, G3 * gs), gy = __builtin_amdgcn_readlane(iny, G3 * gs);
                        fill_win_active(win, PJ, W, H, gx, gy, WIN + 1);
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            uint32_t t[2], h[4];
                            read_win<2>(win, 3 * rb + r, 7 * seg, t);
                            spread_row2(t, h);
#pragma unroll
                            for (int q = 0; q < 4; ++q) nj[r][q] = g == gs ? h[q] : nj[r][q];
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) spread7(nj[r], jr[r]);
                }
                cinx = inx;
                ciny = iny;
            }
            // b = sum (J - I) I' = sum J I' - sum I I': the second sum is the level's
            // constant (c1, c2), so an iteration forms only the J products (exact
            // integers either way; the lane partial is the same value)
            int b1 = -c1, b2 = -c2;
            if (__builtin_amdgcn_ballot_w64((int)J1 < 0)) {
#pragma unroll
                for (int s = 0; s < 3; ++s) match_grad_p<true>(ust, s, jr[s], jr[s + 1], J0, J1, b1, b2);
            } else {
#pragma unroll
                for (int s = 0; s < 3; ++s) match_grad_p<false>(ust, s, jr[s], jr[s + 1], J0, J1, b1, b2);
            }
            float fb1, fb2;
            gsums_f32_fast3(b1, b2, fb1, fb2, ga);
            fb1 *= FLT_SCALE;
            fb2 *= FLT_SCALE;
            const float dx = (A12 * fb2 - A22 * fb1) * D;
            const float dy = (A12 * fb1 - A11 * fb2) * D;
            const float tx = nextx + dx, ty = nexty + dy;
            const bool conv = __builtin_fma((double)dx, (double)dx, (double)dy * (double)dy) <= cfg.crit_eps;
            const bool osc = !conv && j > 0 && fabsf(dx + pdx) < 0.01f && fabsf(dy + pdy) < 0.01f;
            const float ux = osc ? (tx + halfw) - dx * 0.5f : tx + halfw;
            const float uy = osc ? (ty + halfw) - dy * 0.5f : ty + halfw;
            nx = oob ? nx : ux;
            ny = oob ? ny : uy;
            nextx = oob ? nextx : tx;
            nexty = oob ? nexty : ty;
            status = (oob && l == 0) ? 0 : status;
            pdx = dx;
            pdy = dy;
            more = !oob && !conv && !osc && ++j < cfg.max_iter;
        }
#if KLT_LONE
        if (lone_ok && __builtin_amdgcn_ballot_w64(more)) {
            // Lone mode: group lg's point, unit k = lane (window rows k / 3,
            // segment k % 3; lane 63 has none) read from its owner lane's slot.
            // The same integer partials in another arrangement, so the same exact
            // sums and the same fp32 steps; every lane carries the point's state.
            const int lg = grp3(__builtin_ctzll(__builtin_amdgcn_ballot_w64(more))), sl = G3 * lg;
            const int k = min(lane_v(), 62), lr = k / 3, ls = k - 3 * lr;
            const bool live = lane_v() < 63;
            const v4u* uo = units + (sl + 3 * (lr / 3) + ls);
            const int slot = lr - 3 * (lr / 3);
            const int loff = __mul24(lr, pitch) + 7 * ls;
            const auto rdf = [&](float v) {
                return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), sl));
            };
            const auto wf = [&](int i) { return __builtin_bit_cast(float, win[i]); };
            wave_lds_sync();
            const int lc1 = lane_v() < G3 ? (int)win[32 + min(lane_v(), G3 - 1)] : 0;
            const int lc2 = lane_v() < G3 ? (int)win[64 + min(lane_v(), G3 - 1)] : 0;
            const float LA11 = wf(5), LA12 = wf(6), LA22 = wf(7), LD = wf(8);
            float lx = wf(0), ly = wf(1), lpdx = wf(2), lpdy = wf(3);
            int lj = (int)win[4];
            float lnx = rdf(nx), lny = rdf(ny);
            int lst = __builtin_amdgcn_readlane(status, sl);
            int lcx = INT_MIN, lcy = INT_MIN;
            uint32_t h0[4], h1[4];
            bool lmore = true;
            while (lmore) {
                const float fnx = floorf(lx), fny = floorf(ly);
                const int fxi = (int)fnx, fyi = (int)fny;
                const int inx = min(max(fxi, -WIN), W - 1), iny = min(max(fyi, -WIN), H - 1);
                const bool oob = inx != fxi || iny != fyi;
                uint32_t J0, J1;
                weights(lx - fnx, ly - fny, J0, J1);
                if (inx != lcx || iny != lcy) {
                    const bool fast = !raw || (inx >= 3 && inx + 26 <= W && iny >= 0 && iny + 22 <= H);
                    if (fast) {
                        const int off = loff + (PJ.o0 + iny * PJ.pitch + inx);
                        const int al = off & ~3;
                        const uint32_t sh = (uint32_t)off & 3u;
                        const v3u w0 = __builtin_amdgcn_raw_buffer_load_b96(PJ.rs, al, 0, 0);
                        const v3u w1 = __builtin_amdgcn_raw_buffer_load_b96(PJ.rs, al, PJ.pitch, 0);
                        spread_row(w0.x, w0.y, w0.z, sh, h0);
                        spread_row(w1.x, w1.y, w1.z, sh, h1);
                    } else {
                        fill_win_active(win, PJ, W, H, inx, iny, WIN + 1);
                        uint32_t t[2];
                        read_win<2>(win, lr, 7 * ls, t);
                        spread_row2(t, h0);
                        read_win<2>(win, lr + 1, 7 * ls, t);
                        spread_row2(t, h1);
                    }
                    lcx = inx;
                    lcy = iny;
                }
                int b1 = -lc1, b2 = -lc2;
                const v4u* ul = uo;
                asm volatile("" : "+v"(ul));  // the slot reads stay in the loop (registers)
                if ((int)J1 < 0)
                    match_grad_h<true>(ul, slot, h0, h1, J0, J1, b1, b2);
                else
                    match_grad_h<false>(ul, slot, h0, h1, J0, J1, b1, b2);
                b1 = live ? b1 : 0;
                b2 = live ? b2 : 0;
                float fb1, fb2;
                group_sums_f32_fast<64>(b1, b2, fb1, fb2);
                fb1 *= FLT_SCALE;
                fb2 *= FLT_SCALE;
                const float dx = (LA12 * fb2 - LA22 * fb1) * LD;
                const float dy = (LA12 * fb1 - LA11 * fb2) * LD;
                const float tx = lx + dx, ty = ly + dy;
                const bool conv = __builtin_fma((double)dx, (double)dx, (double)dy * (double)dy) <= cfg.crit_eps;
                const bool osc = !conv && lj > 0 && fabsf(dx + lpdx) < 0.01f && fabsf(dy + lpdy) < 0.01f;
                const float ux = osc ? (tx + halfw) - dx * 0.5f : tx + halfw;
                const float uy = osc ? (ty + halfw) - dy * 0.5f : ty + halfw;
                lnx = oob ? lnx : ux;
                lny = oob ? lny : uy;
                lx = oob ? lx : tx;
                ly = oob ? ly : ty;
                lst = (oob && l == 0) ? 0 : lst;
                lpdx = dx;
                lpdy = dy;
                lmore = !oob && !conv && !osc && ++lj < cfg.max_iter;
            }
            const bool mine = grp3(lane_v()) == lg;
            nx = mine ? lnx : nx;
            ny = mine ? lny : ny;
            status = mine ? lst : status;
        }
#endif
        if (status && l == 0) {
            const float exf = nx - halfw, eyf = ny - halfw;
            const float fex = floorf(exf), fey = floorf(eyf);
            const int inx = (int)fex, iny = (int)fey;
            if (inx < -WIN || inx >= W || iny < -WIN || iny >= H) {
                status = 0;
                continue;
            }
            if (!cfg.want_err) continue;
            uint32_t J0, J1;
            weights(exf - fex, eyf - fey, J0, J1);
            int es = 0;
            {
                uint32_t r[4][2];
                const bool fast = !raw || (inx >= 3 && inx + 26 <= W && iny >= 0 && iny + 22 <= H);
                if (__builtin_amdgcn_ballot_w64(!fast) == 0) {
                    const int off = lane_off + (PJ.o0 + iny * PJ.pitch + inx);
                    const int al = off & ~3;
                    const uint32_t sh = (uint32_t)off & 3u;
#pragma unroll
                    for (int q = 0; q < 4; ++q) brow<2>(PJ, al, sh, q * PJ.pitch, r[q]);
                } else {
                    const int g = grp3(lane_v());
#pragma unroll
                    for (int q = 0; q < 4; ++q) r[q][0] = r[q][1] = 0u;
#pragma unroll
                    for (int gs = 0; gs < 3; ++gs) {
                        if (__builtin_amdgcn_ballot_w64(g == gs) == 0) continue;
                        const int gx = __builtin_amdgcn_readlane(inx, G3 * gs), gy = __builtin_amdgcn_readlane(iny, G3 * gs);
                        fill_win_active(win, PJ, W, H, gx, gy, WIN + 1);
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            uint32_t t[2];
                            read_win<2>(win, 3 * rb + q, 7 * seg, t);
                            r[q][0] = g == gs ? t[0] : r[q][0];
                            r[q][1] = g == gs ? t[1] : r[q][1];
                        }
                    }
                }
#pragma unroll
                for (int s = 0; s < 3; ++s) {
                    Unit u;
                    unit_get(ust, s, u);
                    unit_abs_err(u, r[s], r[s + 1], J0, J1, true, es);
                }
            }
            err = __fdiv_rn((float)gsum3(es, ga) * 1.f, (float)(32 * WIN * WIN));
        }
    }
}

// One launch for a batch of pairs: PPW points per wavefront, the points of a
// wave always from one pair (wave-uniform plane bases); ceil(n_pts / PPW)
// waves per pair, the spare groups of a pair's last wave recompute its last
// point and store nothing.
// Waves per workgroup.  One: a finished wave's slot (and its LDS) is refilled
// at once instead of idling until the slowest wave of its workgroup is done
// (per-point iteration counts differ).
#ifndef KLT_WPB
#define KLT_WPB 1
#endif
// minimum waves per SIMD the register allocation must allow.  The fp32-order
// instances are bound by their chains' latency, so by occupancy: their units stay
// in registers (10 KB of LDS per two-point wave instead of 16), for 3 waves per
// SIMD instead of 2
#ifndef KLT_ACC_OCC
#define KLT_ACC_OCC 3
#endif
template <int PPW, int ACC>
constexpr int klt_occupancy() {
    return PPW == 1 ? 4 : ACC ? KLT_ACC_OCC : 4;
}
// border tiles per wave: one per point group; the three-point layout shares one
// (its groups take turns), so its LDS stays within 160 KB / 16 waves
template <int PPW>
constexpr int klt_tiles() {
    return PPW == 3 ? 1 : PPW;
}
// reduceVector (tracking.cc:831-839) inside the LK launch, one point per wave
// (the live tracker's pair: 150 waves, where a compact_kernel launch of its own
// cost ~4 us of a ~43 us pair).  Lane 0 ORs the wave's keep bit into its pair's
// words, then counts the wave in.  Both are returning agent-scope atomics,
// performed where every XCD sees them, and the count is issued only after the
// OR has returned, so the wave that counts the pair's n_pts-th arrival sees
// every bit.  That wave lists the set bits in point order (compact_kernel's
// kept_idx / n_kept) and zeroes the words and the count for the next launch
// (graph replays included).  No release fence: the other outputs are not read
// inside the launch.
__device__ __forceinline__ void fused_compact(const KltArgs& a, int pair, int pt, bool keep) {
    const int nw = (a.n_pts + 63) >> 6;
    unsigned long long* m = a.cmask + (int64_t)pair * (nw + 1);
    bool last = false;
    if (lane_v() == 0) {
        if (keep) {
            const unsigned long long o = __hip_atomic_fetch_or(m + (pt >> 6), 1ull << (pt & 63), __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("; keep bit in: %0" ::"v"(o) : "memory");  // its return before the count
        }
        last = __hip_atomic_fetch_add(m + nw, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (unsigned long long)(a.n_pts - 1);
    }
    if (__builtin_amdgcn_ballot_w64(last) == 0) return;
    const int lane = lane_v();
    // the words read by read-modify-write atomics like the ones that set them (an
    // OR of a literal 0 would compile to an atomic load)
    unsigned long long zero = 0, mine = 0;
    asm volatile("" : "+v"(zero));
    if (lane < nw) mine = __hip_atomic_fetch_or(m + lane, zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int32_t* out = a.kept_idx + (int64_t)pair * a.n_pts;
    int base = 0;
    for (int w = 0; w < nw; ++w) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)mine, w);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(mine >> 32), w);
        const unsigned long long word = ((unsigned long long)hi << 32) | lo;
        if ((word >> lane) & 1ull) out[base + __popcll(word & ((1ull << lane) - 1ull))] = 64 * w + lane;
        base += __popcll(word);
    }
    if (lane == 0) a.n_kept[pair] = base;
    if (lane <= nw) __hip_atomic_exchange(m + lane, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#ifdef GVX_KLT_TRACE
// Diagnostic build only (tools/lk_residency.py): every wave of the batch
// layout stamps itself (gvx_internal.h WaveStamp) into gvx_klt_trace_buf.
__device__ uint64_t* gvx_klt_trace_buf;
#define KLT_WAVE_STAMP WaveStamp wave_stamp_(gvx_klt_trace_buf)
#else
#define KLT_WAVE_STAMP
#endif

template <int PPW, int ACC>
__global__ void __launch_bounds__(64 * KLT_WPB, (klt_occupancy<PPW, ACC>())) klt_kernel(KltArgs a, PyrLayout lay, const uint8_t* __restrict__ pyr_prev,
                                                  const uint8_t* __restrict__ pyr_next, int64_t prev_stride,
                                                  int64_t next_stride, Level0 l0, const float* __restrict__ prev_xy,
                                                  float* __restrict__ next_xy, float* __restrict__ back_xy,
                                                  uint8_t* __restrict__ flags, float* __restrict__ err_out) {
    static_assert(PPW == 3 ? ACC == 0 : (PPW == 1 || PPW == 2), "three points per wave: exact order only");
    __shared__ uint32_t wins[KLT_WPB * klt_tiles<PPW>()][(WIN + 3) * WIN_DW];  // border tiles
    __shared__ v4u units[KLT_WPB][ACC ? 1 : 3 * PPW * 64];        // per-lane window values (exact order)
    // fp32-order window sums: one region per point group
    __shared__ __attribute__((aligned(16))) float accs[ACC ? KLT_WPB * PPW : 1][ACC_FLOATS];
    KLT_WAVE_STAMP;
#ifdef KLT_PRIO
    __builtin_amdgcn_s_setprio(KLT_PRIO);  // A/B
#endif
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wpp = (a.n_pts + PPW - 1) / PPW;  // waves per pair (launch capacity)
    const int n_waves = a.n_pairs * wpp;
    const int nb = (n_waves + KLT_WPB - 1) / KLT_WPB;
    const int wg = xcd_swizzle(blockIdx.x, nb) * KLT_WPB + wv;
    if (wg >= n_waves) return;
    const int pair = wg / wpp;
    // device-resident count (the per-frame loop without host round trips)
    const int npt = a.n_dev ? min(a.n_pts, *a.n_dev) : a.n_pts;
    if ((wg - pair * wpp) * PPW >= npt) return;  // the whole wave is past the count
    // the group's point (a spare group of a pair's last wave recomputes the last
    // point); rebuilt from the lane id where needed
    auto point = [&](bool& writer) -> int64_t {
        const int lane = lane_v();
        int grp, gl;
        if constexpr (PPW == 3) {
            grp = grp3(lane);
            gl = lane - G3 * grp;  // 21 on lane 63: no group's writer
        } else {
            grp = lane / (64 / PPW);
            gl = lane & (64 / PPW - 1);
        }
        const int pt_raw = (wg - pair * wpp) * PPW + grp;
        writer = pt_raw < npt && gl == 0;
        return (int64_t)pair * a.n_pts + (pt_raw < npt ? pt_raw : npt - 1);
    };
    uint32_t(*wv_wins)[(WIN + 3) * WIN_DW] = wins + wv * klt_tiles<PPW>();
    v4u* wv_units = units[wv];
    float(*wv_accs)[ACC_FLOATS] = accs + (ACC ? wv * PPW : 0);
    const uint8_t* I = pyr_prev + pair * prev_stride;
    const uint8_t* J = pyr_next + pair * next_stride;
    const L0Planes pf{l0.prev + pair * l0.prev_stride, l0.next + pair * l0.next_stride, l0.o0, l0.pitch,
                      l0.raw != 0};
    const L0Planes pb{pf.j, pf.i, pf.o0, pf.pitch, pf.raw};
    LkCfg cfg{a.max_iter, a.crit_eps, a.min_eig, a.use_initial_flow, err_out != nullptr};
    bool writer;
    int64_t gp = point(writer);
    float nx = 0.f, ny = 0.f;
    int st = 1;
    float e = 0.f;
    {
        const float p0x = prev_xy[2 * gp], p0y = prev_xy[2 * gp + 1];
        const float* init_xy = a.init_xy ? a.init_xy : next_xy;
        nx = init_xy[2 * gp];
        ny = init_xy[2 * gp + 1];
        if constexpr (ACC != 0) {
            constexpr int G = 64 / PPW;
            const int lane = lane_v();
            acc_clear<ACC, G>(wv_accs[lane / G], lane & (G - 1));
        }
        if constexpr (PPW == 3)
            lk_group3(I, J, pf, lay, cfg, p0x, p0y, nx, ny, st, e, wv_wins[0], wv_units);
        else
            lk_group<PPW, ACC>(I, J, pf, lay, cfg, p0x, p0y, nx, ny, st, e, wv_wins, wv_units, wv_accs);
    }
    if (a.mode == 0) {
        gp = point(writer);
        if (writer) {
            next_xy[2 * gp] = nx;
            next_xy[2 * gp + 1] = ny;
            flags[gp] = (uint8_t)st;
            if (err_out) err_out[gp] = e;
        }
        return;
    }
    // backward: prevPts = forward result, initial flow = original prev points
    // (re-read: an opaque copy of the pointer keeps the compiler from holding
    // the first load's values live across the forward pass)
    const float* pxy = prev_xy;
    asm volatile("" : "+s"(pxy));
    gp = point(writer);
    float bx = pxy[2 * gp], by = pxy[2 * gp + 1];
    int st2 = 1;
    float e2 = 0.f;
    cfg.use_initial_flow = 1;
    cfg.want_err = 0;  // the backward error is not reported
    if constexpr (PPW == 3)
        lk_group3(J, I, pb, lay, cfg, nx, ny, bx, by, st2, e2, wv_wins[0], wv_units);
    else
        lk_group<PPW, ACC>(J, I, pb, lay, cfg, nx, ny, bx, by, st2, e2, wv_wins, wv_units, wv_accs);
    gp = point(writer);
    bool keep = false;
    if (writer) {
        const float p0x = pxy[2 * gp], p0y = pxy[2 * gp + 1];
        const double B = a.border;
        const bool on_border = nx < B || ny < B || nx > (a.cam_w - B) || ny > (a.cam_h - B);
        const double ddx = (double)(bx - p0x), ddy = (double)(by - p0y);
        const double dist = __dsqrt_rn(ddx * ddx + ddy * ddy);
        keep = st && st2 && !on_border && dist < a.fb_thresh;
        next_xy[2 * gp] = nx;
        next_xy[2 * gp + 1] = ny;
        if (back_xy) {
            back_xy[2 * gp] = bx;
            back_xy[2 * gp + 1] = by;
        }
        flags[gp] = (uint8_t)((st ? 1 : 0) | (st2 ? 2 : 0) | (keep ? 4 : 0));
        if (err_out) err_out[gp] = e;
    }
    if constexpr (PPW == 1) {
        if (a.cmask) fused_compact(a, pair, wg - pair * wpp, keep);
    }
}


// ---- the batch LK as a chain of phases (r06) ----
// klt_kernel runs a point group's whole chain -- forward levels L..0, then
// backward L..0 -- in one wave of ~84 us.  Its launch ends in a drain: the last
// waves start ~100 us before the end, and the SIMDs hold 1.5 waves on average
// from then on, against 3.9 before (profiles/r06_d1/res: one configs[1] launch,
// per-wave s_memrealtime stamps).  Here the chain is cut into phases of `lpp`
// levels of one direction, each a wave of its own, dispatched phase-major: all
// groups' phase 0, then all groups' phase 1, ...  The drain is then as long as
// one phase.  Measured (profiles/r06_l2, r06_l3): it is, but a phase wave costs
// more than its share of the chain (+15-18 % wave time in all: its start-up, the
// hand-off, level-0 windows re-read from HBM by the backward phases), so the net
// is -1.7 % at 4 levels per phase (forward / backward) and a loss at 1-2; beside
// the next batch's pyramid pass (bench.py's default) the whole-chain kernel wins,
// because the pyramid waves fill its drain.  So gvx_set_klt_phases defaults to 0.
// Hand-off: every value a phase passes on is one 64-bit word, the float in the
// low half and a tag (the phase that wrote it, plus one) in the high half,
// stored and loaded as single-copy-atomic dwordx2 accesses.  A reader waits for
// the tag it expects, so no ordering between words is needed and a wave ends
// without waiting for its stores.  Per point (PH_WORDS words): the running flow
// x, y; the forward result fx, fy and status.  The last phase sets every tag back
// to 0, so a launch leaves the words as it found them (graph replays included).
// Coherence: the dispatcher sends workgroup b to XCD b % 8 and a phase's block
// count is a multiple of 8, so the phases of a group run on one XCD and meet in
// its L2; the accesses are agent-scope relaxed atomics (sc1: past the CU's L1).
// Progress: workgroups of one XCD are dispatched in id order, so a phase's
// predecessor has been dispatched before it waits; the wait is also bounded
// (2^22 polls, about a second), so a broken assumption shows as wrong results,
// not a hang.
constexpr int PH_WORDS = 8;  // per point: x, y, fx, fy, st (64 B)
enum { PH_X = 0, PH_Y = 1, PH_FX = 2, PH_FY = 3, PH_ST = 4 };
__device__ __forceinline__ uint64_t ph_ld(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ph_st(uint64_t* p, uint32_t tag, uint32_t bits) {
    __hip_atomic_store(p, ((uint64_t)tag << 32) | bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// the words `a` and `b` as written by phase tag-1 (va, vb: their first loads)
__device__ __forceinline__ void ph_wait2(const uint64_t* a, const uint64_t* b, uint64_t& va, uint64_t& vb,
                                         uint32_t tag) {
    int guard = 0;
    while (((uint32_t)(va >> 32) != tag || (uint32_t)(vb >> 32) != tag) && ++guard < (1 << 22)) {
        __builtin_amdgcn_s_sleep(4);
        va = ph_ld(a);
        vb = ph_ld(b);
    }
}
struct PhResolve {  // lk_group3's hook: the running flow of the previous phase
    const uint64_t* hs;
    uint32_t gi;   // the point (a 32-bit index: one VGPR live across the chain)
    uint32_t tag;  // 0: the phase starts the chain (nothing to wait for)
    __device__ void operator()(float& x, float& y) const {
        if (tag == 0) return;
        const uint64_t* w = hs + (size_t)PH_WORDS * gi;
        uint64_t a = ph_ld(w + PH_X), b = ph_ld(w + PH_Y);
        ph_wait2(w + PH_X, w + PH_Y, a, b, tag);
        x = __uint_as_float((uint32_t)a);
        y = __uint_as_float((uint32_t)b);
    }
};

__global__ void __launch_bounds__(64, 4) klt_phase_kernel(KltArgs a, PyrLayout lay, const uint8_t* __restrict__ pyr_prev,
                                                          const uint8_t* __restrict__ pyr_next, int64_t prev_stride,
                                                          int64_t next_stride, Level0 l0, const float* __restrict__ prev_xy,
                                                          float* next_xy, float* __restrict__ back_xy,
                                                          uint8_t* __restrict__ flags, float* __restrict__ err_out,
                                                          uint64_t* hs, int sc, int lpp) {
    __shared__ uint32_t win[(WIN + 3) * WIN_DW];  // border tile
    __shared__ v4u units[3 * 3 * 64];             // per-lane window values
    KLT_WAVE_STAMP;
    const int wpp = (a.n_pts + 2) / 3;
    const int n_groups = a.n_pairs * wpp;
    const int pd = (lay.nlev + lpp - 1) / lpp;  // phases per direction
    const int n_ph = a.mode == 0 ? pd : 2 * pd;
    // superchunks of sc groups, each dispatched phase-major; the last one holds
    // the remaining groups on 8 * xcd_per(remainder) blocks per phase
    const int span = n_ph * sc, n_full = n_groups / sc;
    int q = blockIdx.x / span, r = blockIdx.x - q * span, blk = sc;
    if (q >= n_full) {
        q = n_full;
        r = blockIdx.x - n_full * span;
        blk = N_XCD * xcd_per(n_groups - n_full * sc);
    }
    const int ph = r / blk;
    const int g0 = q * sc, gs = min(sc, n_groups - g0);
    const int lg = xcd_swizzle(r - ph * blk, gs);  // block b runs on XCD b % 8 in every phase
    if (lg >= gs) return;
    const int wg = g0 + lg;
    const int pair = wg / wpp;
    const int npt = a.n_dev ? min(a.n_pts, *a.n_dev) : a.n_pts;
    if ((wg - pair * wpp) * 3 >= npt) return;  // every phase of this group leaves here
    const bool bwd = ph >= pd;
    const int c = bwd ? ph - pd : ph;
    const int l_top = lay.nlev - 1 - c * lpp, l_bot = max(l_top - lpp + 1, 0);
    const bool last = ph == (a.mode == 0 ? pd : 2 * pd) - 1;
    const int lane = lane_v(), grp = grp3(lane), gl = lane - G3 * grp;
    const int pt_raw = (wg - pair * wpp) * 3 + grp;
    const bool writer = pt_raw < npt && gl == 0;
    const int64_t gp = (int64_t)pair * a.n_pts + (pt_raw < npt ? pt_raw : npt - 1);
    uint64_t* w = hs + PH_WORDS * gp;
    // one LK call for either direction (one inlined copy of the chain): the
    // backward call tracks the forward result back from J to I, from the
    // original prev points as its initial flow
    const uint8_t* Ip = pyr_prev + pair * prev_stride;
    const uint8_t* Jp = pyr_next + pair * next_stride;
    const uint8_t* l0i = l0.prev + pair * l0.prev_stride;
    const uint8_t* l0j = l0.next + pair * l0.next_stride;
    const L0Planes pl{bwd ? l0j : l0i, bwd ? l0i : l0j, l0.o0, l0.pitch, l0.raw != 0};
    const LkCfg cfg{a.max_iter, a.crit_eps, a.min_eig, bwd ? 1 : a.use_initial_flow,
                    !bwd && err_out != nullptr && l_bot == 0};
    float px, py, nx, ny;
    // the running flow of the previous phase, read where the chain needs it (PhResolve)
    const PhResolve res{hs, (uint32_t)gp, ph > 0 && ph != pd ? (uint32_t)ph : 0u};
    if (!bwd) {
        px = prev_xy[2 * gp];
        py = prev_xy[2 * gp + 1];
        nx = ny = 0.f;
        if (ph == 0) {
            const float* init_xy = a.init_xy ? a.init_xy : next_xy;
            nx = init_xy[2 * gp];
            ny = init_xy[2 * gp + 1];
        }
    } else {
        uint64_t fx = ph_ld(w + PH_FX), fy = ph_ld(w + PH_FY);
        ph_wait2(w + PH_FX, w + PH_FY, fx, fy, (uint32_t)pd);
        px = __uint_as_float((uint32_t)fx);
        py = __uint_as_float((uint32_t)fy);
        nx = prev_xy[2 * gp];
        ny = prev_xy[2 * gp + 1];
    }
    int st = 1;
    float e = 0.f;
    lk_group3(bwd ? Jp : Ip, bwd ? Ip : Jp, pl, lay, cfg, px, py, nx, ny, st, e, win, units, l_top, l_bot, res);
    if (!writer) return;
    const int64_t gq = res.gi;  // gp again, from the one VGPR the chain kept
    w = hs + (size_t)PH_WORDS * res.gi;
    const uint32_t tag = (uint32_t)ph + 1;
    if (!bwd && l_bot != 0) {
        ph_st(w + PH_X, tag, __float_as_uint(nx));
        ph_st(w + PH_Y, tag, __float_as_uint(ny));
    } else if (!bwd) {  // the forward result
        next_xy[2 * gq] = nx;
        next_xy[2 * gq + 1] = ny;
        if (err_out) err_out[gq] = e;
        if (a.mode == 0) {
            flags[gq] = (uint8_t)st;
            ph_st(w + PH_X, 0, 0);  // the last phase: tags back to 0
            ph_st(w + PH_Y, 0, 0);
        } else {
            ph_st(w + PH_FX, tag, __float_as_uint(nx));
            ph_st(w + PH_FY, tag, __float_as_uint(ny));
            ph_st(w + PH_ST, tag, (uint32_t)st);
        }
    } else if (!last) {
        ph_st(w + PH_X, tag, __float_as_uint(nx));
        ph_st(w + PH_Y, tag, __float_as_uint(ny));
    } else {
        // tracking.cc:396-408 / :831-849 on the forward result (px, py), the
        // backward result (nx, ny) and the original prev points
        uint64_t s1 = ph_ld(w + PH_ST), dummy = (uint64_t)pd << 32;
        ph_wait2(w + PH_ST, w + PH_ST, s1, dummy, (uint32_t)pd);
        const int st1 = (int)(uint32_t)s1;
        const float p0x = prev_xy[2 * gq], p0y = prev_xy[2 * gq + 1];
        const double B = a.border;
        const bool on_border = px < B || py < B || px > (a.cam_w - B) || py > (a.cam_h - B);
        const double ddx = (double)(nx - p0x), ddy = (double)(ny - p0y);
        const double dist = __dsqrt_rn(ddx * ddx + ddy * ddy);
        const bool keep = st1 && st && !on_border && dist < a.fb_thresh;
        if (back_xy) {
            back_xy[2 * gq] = nx;
            back_xy[2 * gq + 1] = ny;
        }
        flags[gq] = (uint8_t)((st1 ? 1 : 0) | (st ? 2 : 0) | (keep ? 4 : 0));
#pragma unroll
        for (int k = 0; k < 5; ++k) ph_st(w + k, 0, 0);  // tags back to 0
    }
}

// reduceVector (tracking.cc:831-839): order-preserving index compaction of the
// keep bit, one workgroup per pair.
__global__ void __launch_bounds__(256) compact_kernel(int n_pts, const uint8_t* __restrict__ flags,
                                                      int32_t* __restrict__ kept_idx, int32_t* __restrict__ n_kept) {
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

// Points per wavefront of the LK launch.  Batches that fill the chip take 2
// (the per-point scalar work is shared; 0.47 vs 0.61 ms per 256 pairs); small
// ones (one frame of a sequence: 150 points) take 1, which halves the work of
// the slowest wave (41 vs 54 us per frame), built for 4 waves per SIMD (no
// spills; at most 4 waves per SIMD below the threshold: 36.8 -> 35.8 us per
// sequence frame, 50.3 -> 49.0 us per pair, r02 v18).
// KLT_PPW_BATCH 3: batches in the three-point layout (exact order only; the
// fp32 orders keep two).
#ifndef KLT_PPW_BATCH
#define KLT_PPW_BATCH 3
#endif
static int klt_ppw(int64_t total_points) { return total_points <= 4096 ? 1 : 2; }

template <int PPW, int ACC>
static void launch_klt_ppw(gvx_ctx* c, const KltArgs& a, const PyrLayout& lay, const uint8_t* pyr_prev,
                           const uint8_t* pyr_next, int64_t prev_pair_stride, int64_t next_pair_stride,
                           const Level0& l0, const float* prev_xy, float* next_xy, float* back_xy, uint8_t* flags,
                           float* err) {
    const int n_waves = a.n_pairs * ((a.n_pts + PPW - 1) / PPW);
    dim3 grid((unsigned)(N_XCD * xcd_per((n_waves + KLT_WPB - 1) / KLT_WPB)));
    launch_timed(c, "klt", klt_kernel<PPW, ACC>, grid, dim3(64 * KLT_WPB), 0, a, lay, pyr_prev, pyr_next,
                 prev_pair_stride, next_pair_stride, l0, prev_xy, next_xy, back_xy, flags, err);
}

// The batch LK as phases of c->klt_lpp levels (klt_phase_kernel); false when
// the hand-off buffers cannot be had (a capture that would grow them): the
// caller then runs the single-wave chain, which gives the same bits.
static bool launch_klt_phases(gvx_ctx* c, const KltArgs& a, const PyrLayout& lay, const uint8_t* pyr_prev,
                              const uint8_t* pyr_next, int64_t prev_pair_stride, int64_t next_pair_stride,
                              const Level0& l0, const float* prev_xy, float* next_xy, float* back_xy,
                              uint8_t* flags, float* err) {
    const int lpp = c->klt_lpp;
    if (lpp <= 0) return false;
    const int n_groups = a.n_pairs * ((a.n_pts + 2) / 3);
    // one set per stream: a launch on the branch stream must not share them
    const std::string tag = c->stream == c->main ? "" : "_side";
    const bool failed_before = c->capture_failed;
    const std::string name = "klt_phase_state" + tag;
    uint64_t* hs = (uint64_t*)scratch(c, name, sizeof(uint64_t) * PH_WORDS * (size_t)a.n_pairs * a.n_pts);
    if (!hs) {
        c->capture_failed = failed_before;  // not a failure: the fallback needs no buffer
        return false;
    }
    DevBuf& db = c->dev[name];
    if (db.fresh) {  // tags start at 0; every launch leaves them at 0
        if (hipMemsetAsync(db.p, 0, db.bytes, c->stream) != hipSuccess) return false;
        db.fresh = false;
    }
    // superchunks of sc groups (a multiple of 8), each run phase-major: a group's
    // phases are sc waves apart in dispatch order, so its level-0 windows are
    // still near in the caches when its backward pass reads them again
    const int sc = std::min(std::max(8, c->klt_super / 8 * 8), N_XCD * xcd_per(n_groups));
    const int pd = (lay.nlev + lpp - 1) / lpp;
    const int n_ph = a.mode == 0 ? pd : 2 * pd;
    const int n_full = n_groups / sc, rem = n_groups - n_full * sc;
    const int64_t grid = (int64_t)n_ph * ((int64_t)n_full * sc + (rem ? N_XCD * xcd_per(rem) : 0));
    launch_timed(c, "klt", klt_phase_kernel, dim3((unsigned)grid), dim3(64), 0, a, lay, pyr_prev, pyr_next,
                 prev_pair_stride, next_pair_stride, l0, prev_xy, next_xy, back_xy, flags, err, hs, sc, lpp);
    return true;
}

template <int ACC>
static void launch_klt_acc(gvx_ctx* c, const KltArgs& a, const PyrLayout& lay, const uint8_t* pyr_prev,
                           const uint8_t* pyr_next, int64_t prev_pair_stride, int64_t next_pair_stride,
                           const Level0& l0, const float* prev_xy, float* next_xy, float* back_xy, uint8_t* flags,
                           float* err) {
    if (klt_ppw((int64_t)a.n_pairs * a.n_pts) == 1)
        launch_klt_ppw<1, ACC>(c, a, lay, pyr_prev, pyr_next, prev_pair_stride, next_pair_stride, l0, prev_xy,
                               next_xy, back_xy, flags, err);
    else if (ACC == 0 && KLT_PPW_BATCH == 3) {
        if (!launch_klt_phases(c, a, lay, pyr_prev, pyr_next, prev_pair_stride, next_pair_stride, l0, prev_xy,
                               next_xy, back_xy, flags, err))
            launch_klt_ppw<3, 0>(c, a, lay, pyr_prev, pyr_next, prev_pair_stride, next_pair_stride, l0, prev_xy,
                                 next_xy, back_xy, flags, err);
    }
    else
        launch_klt_ppw<2, ACC>(c, a, lay, pyr_prev, pyr_next, prev_pair_stride, next_pair_stride, l0, prev_xy,
                               next_xy, back_xy, flags, err);
}

hipError_t launch_klt(gvx_ctx* c, const KltArgs& a, const PyrLayout& lay, const uint8_t* pyr_prev,
                      const uint8_t* pyr_next, int64_t prev_pair_stride, int64_t next_pair_stride,
                      const Level0& l0, const float* prev_xy, float* next_xy, float* back_xy, uint8_t* flags,
                      float* err) {
    const int64_t total = (int64_t)a.n_pairs * a.n_pts;
    if (total <= 0) return hipSuccess;
    if (total > (int64_t)1 << 30) return hipErrorInvalidValue;  // wave indices are int32
    switch (a.accum) {
        case GVX_LK_ACCUM_EXACT:
            launch_klt_acc<0>(c, a, lay, pyr_prev, pyr_next, prev_pair_stride, next_pair_stride, l0, prev_xy, next_xy,
                              back_xy, flags, err);
            break;
        case GVX_LK_ACCUM_F32_SCALAR:
            launch_klt_acc<1>(c, a, lay, pyr_prev, pyr_next, prev_pair_stride, next_pair_stride, l0, prev_xy, next_xy,
                              back_xy, flags, err);
            break;
        case GVX_LK_ACCUM_F32_SIMD4:
            launch_klt_acc<2>(c, a, lay, pyr_prev, pyr_next, prev_pair_stride, next_pair_stride, l0, prev_xy, next_xy,
                              back_xy, flags, err);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_compact(gvx_ctx* c, int n_pairs, int n_pts, const uint8_t* flags, int32_t* kept_idx,
                          int32_t* n_kept) {
    if (n_pairs <= 0) return hipSuccess;
    return launch_timed(c, "compact", compact_kernel, dim3(n_pairs), dim3(256), 0, n_pts, flags, kept_idx, n_kept);
}

hipError_t launch_klt_compact(gvx_ctx* c, KltArgs a, const PyrLayout& lay, const uint8_t* pyr_prev,
                              const uint8_t* pyr_next, int64_t prev_pair_stride, int64_t next_pair_stride,
                              const Level0& l0, const float* prev_xy, float* next_xy, float* back_xy,
                              uint8_t* flags, float* err, int32_t* kept_idx, int32_t* n_kept) {
    a.mode = 1;
    const int64_t total = (int64_t)a.n_pairs * a.n_pts;
    if (c->fused_compact && total > 0 && klt_ppw(total) == 1 && !a.n_dev) {
        // one set of words per stream: a launch on the branch stream must not share them
        const std::string name = std::string("klt_cmask") + (c->stream == c->main ? "" : "_side");
        const size_t bytes = sizeof(unsigned long long) * (size_t)a.n_pairs * ((a.n_pts + 63) / 64 + 1);
        const bool failed_before = c->capture_failed;
        unsigned long long* m = (unsigned long long*)scratch(c, name, bytes);
        if (m) {
            DevBuf& db = c->dev[name];
            if (db.fresh) {  // zero once; every launch leaves them zero
                const hipError_t e = hipMemsetAsync(db.p, 0, db.bytes, c->stream);
                if (e != hipSuccess) return e;
                db.fresh = false;
            }
            a.cmask = m;
            a.kept_idx = kept_idx;
            a.n_kept = n_kept;
            return launch_klt(c, a, lay, pyr_prev, pyr_next, prev_pair_stride, next_pair_stride, l0, prev_xy,
                              next_xy, back_xy, flags, err);
        }
        c->capture_failed = failed_before;  // not a failure: the two-launch form needs no buffer
    }
    const hipError_t e = launch_klt(c, a, lay, pyr_prev, pyr_next, prev_pair_stride, next_pair_stride, l0, prev_xy,
                                    next_xy, back_xy, flags, err);
    if (e != hipSuccess) return e;
    return launch_compact(c, a.n_pairs, a.n_pts, flags, kept_idx, n_kept);
}

}  // namespace gvx

#ifdef GVX_KLT_TRACE
// diagnostic build only: the wave-stamp buffer of klt_kernel (4 uint64 per wave
// of the launch; nullptr turns the stamps off)
extern "C" int gvx_klt_trace_set(void* buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(gvx::gvx_klt_trace_buf), &buf, sizeof(buf));
}
#endif
