/*
 * klt.c -- TEST INFRASTRUCTURE (parity oracle + CPU baseline), see gvx_oracle.h.
 *
 * Restates OpenCV 4.x calcOpticalFlowPyrLK as the reference calls it at
 * ic_gvins/ic_gvins/tracking/tracking.cc:385-393 and :487-496
 * (winSize 21x21, maxLevel 3, TermCriteria(COUNT+EPS, 30, 0.01),
 * OPTFLOW_USE_INITIAL_FLOW, minEigThreshold 1e-4), plus the FB/border status
 * and reduceVector compaction of tracking.cc:396-408 / :831-849.
 * The OpenCV sources are not in this environment; the semantics follow
 * SURVEY.md Appendix A.1-A.3 (modules/video/src/lkpyramid.cpp scalar path).
 * Parity vs. a real OpenCV binary is unpinned (see gvx_oracle.h).
 */
#include "gvx_oracle.h"

#include <float.h>
#include <math.h>
#include "orc_pool.h"
#include <stdlib.h>
#include <string.h>

#ifdef ORC_ITER_STATS
/* LK iterations per (level, point) -- diagnostic builds (-DORC_ITER_STATS, one thread) */
long orc_iter_hist[8][64];
#endif
#ifdef ORC_ACC_STATS
/* window sums whose absolute sum stays <= 2^24 (every fp32 partial sum exact) --
   diagnostic builds (-DORC_ACC_STATS, one thread): [0] A sets, [1] A sets with
   all three small, [2] b pairs, [3] b pairs with both small */
long orc_acc_stats[16];
#endif

#define DESCALE(x, n) (((x) + (1 << ((n)-1))) >> (n))

void orc_klt_params_default(orc_klt_params* p) {
    p->win = 21;
    p->max_level = 3;
    p->max_iter = 30;
    p->eps = 0.01;
    p->use_initial_flow = 1;
    p->min_eig = 1e-4f;
}

/* cv::borderInterpolate(p, len, BORDER_REFLECT_101) */
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

/* cvRound: round half to even (lrintf in the default rounding mode). */
static int cv_round(float v) { return (int)lrintf(v); }
/* cvFloor */
static int cv_floor(float v) {
    int i = (int)v;
    return i - (i > v);
}

static uint8_t* px(const orc_u8plane* p, int x, int y) {
    return p->buf + (size_t)(y + p->pad) * p->pitch + (x + p->pad);
}

static void alloc_plane(orc_u8plane* p, int w, int h, int pad) {
    p->w = w;
    p->h = h;
    p->pad = pad;
    p->pitch = w + 2 * pad;
    p->buf = (uint8_t*)malloc((size_t)p->pitch * (h + 2 * pad));
}

/* copyMakeBorder(..., BORDER_REFLECT_101) of the interior into the pad ring. */
static void fill_border_reflect101(orc_u8plane* p) {
    for (int y = -p->pad; y < p->h + p->pad; y++) {
        int sy = reflect101(y, p->h);
        for (int x = -p->pad; x < p->w + p->pad; x++) {
            if (y >= 0 && y < p->h && x >= 0 && x < p->w) continue;
            *px(p, x, y) = *px(p, reflect101(x, p->w), sy);
        }
    }
}

/* pyrDown (imgproc/src/pyramids.cpp pyrDown_ with FixPtCast<uchar,8>):
   dst(y,x) = (sum_ij k_i k_j src(refl(2y+i-2), refl(2x+j-2)) + 128) >> 8,
   k = [1 4 6 4 1].  Integer arithmetic: evaluation order is irrelevant, so the
   separable form (horizontal taps per source row, then vertical) and any row
   split over threads give the identical result. */
typedef struct {
    const orc_u8plane* src;
    orc_u8plane* dst;
    const int* xtab; /* 5 reflected source columns per destination column */
} pyr_job;

static void pyr_rows(void* vctx, int y0, int y1) {
    const pyr_job* jb = (const pyr_job*)vctx;
    const orc_u8plane* src = jb->src;
    orc_u8plane* dst = jb->dst;
    int* rows = (int*)malloc(sizeof(int) * 5 * (size_t)dst->w);
    for (int y = y0; y < y1; y++) {
        for (int i = 0; i < 5; i++) {
            const uint8_t* s = px(src, 0, reflect101(2 * y + i - 2, src->h));
            int* r = rows + (size_t)i * dst->w;
            for (int x = 0; x < dst->w; x++) {
                const int* t = jb->xtab + 5 * x;
                r[x] = s[t[0]] + 4 * s[t[1]] + 6 * s[t[2]] + 4 * s[t[3]] + s[t[4]];
            }
        }
        uint8_t* d = px(dst, 0, y);
        for (int x = 0; x < dst->w; x++) {
            int v = rows[x] + 4 * rows[dst->w + x] + 6 * rows[2 * dst->w + x] + 4 * rows[3 * dst->w + x] +
                    rows[4 * dst->w + x];
            d[x] = (uint8_t)((v + 128) >> 8);
        }
    }
    free(rows);
}

static void pyr_down(const orc_u8plane* src, orc_u8plane* dst, int nthreads) {
    int* xtab = (int*)malloc(sizeof(int) * 5 * (size_t)dst->w);
    for (int x = 0; x < dst->w; x++)
        for (int j = 0; j < 5; j++) xtab[5 * x + j] = reflect101(2 * x + j - 2, src->w);
    pyr_job jb = {src, dst, xtab};
    orc_parallel_for(dst->h, nthreads, pyr_rows, &jb);
    free(xtab);
}

static int build_pyramid_mt(const uint8_t* img, int w, int h, int stride, int win, int max_level,
                            orc_pyramid* pyr, int nthreads);

int orc_build_pyramid(const uint8_t* img, int w, int h, int stride, int win, int max_level,
                      orc_pyramid* pyr) {
    return build_pyramid_mt(img, w, h, stride, win, max_level, pyr, 1);
}

static int build_pyramid_mt(const uint8_t* img, int w, int h, int stride, int win, int max_level,
                            orc_pyramid* pyr, int nthreads) {
    memset(pyr, 0, sizeof(*pyr));
    orc_u8plane* l0 = &pyr->lv[0];
    alloc_plane(l0, w, h, win);
    for (int y = 0; y < h; y++) memcpy(px(l0, 0, y), img + (size_t)y * stride, (size_t)w);
    fill_border_reflect101(l0);
    int sw = w, sh = h;
    for (int level = 0; level <= max_level; level++) {
        if (level != 0) {
            alloc_plane(&pyr->lv[level], sw, sh, win);
            pyr_down(&pyr->lv[level - 1], &pyr->lv[level], nthreads);
            fill_border_reflect101(&pyr->lv[level]);
        }
        pyr->nlevels = level + 1;
        sw = (sw + 1) / 2;
        sh = (sh + 1) / 2;
        if (sw <= win || sh <= win) return level;
    }
    return max_level;
}

void orc_free_pyramid(orc_pyramid* pyr) {
    for (int i = 0; i < pyr->nlevels; i++) free(pyr->lv[i].buf);
    memset(pyr, 0, sizeof(*pyr));
}

/* calcSharrDeriv (lkpyramid.cpp): vertical [3 10 3] / [-1 0 1] pass with
   REFLECT_101 rows, then horizontal [-1 0 1] / [3 10 3] with REFLECT_101
   columns.  Rows are independent (integer arithmetic): split over threads. */
typedef struct {
    const orc_u8plane* src;
    int16_t* out;
    int out_pitch; /* int16 pairs per output row */
} scharr_job;

static void scharr_rows(void* vctx, int ya, int yb) {
    const scharr_job* jb = (const scharr_job*)vctx;
    const orc_u8plane* src = jb->src;
    int w = src->w, h = src->h;
    int* t0 = (int*)malloc(sizeof(int) * (w + 2));
    int* t1 = (int*)malloc(sizeof(int) * (w + 2));
    for (int y = ya; y < yb; y++) {
        int y0 = y > 0 ? y - 1 : (h > 1 ? 1 : 0);
        int y2 = y < h - 1 ? y + 1 : (h > 1 ? h - 2 : 0);
        for (int x = 0; x < w; x++) {
            int a = *px(src, x, y0), b = *px(src, x, y), c = *px(src, x, y2);
            t0[x + 1] = (a + c) * 3 + b * 10;
            t1[x + 1] = c - a;
        }
        int x0 = w > 1 ? 1 : 0, x1 = w > 1 ? w - 2 : 0;
        t0[0] = t0[x0 + 1];
        t0[w + 1] = t0[x1 + 1];
        t1[0] = t1[x0 + 1];
        t1[w + 1] = t1[x1 + 1];
        int16_t* o = jb->out + 2 * (size_t)y * jb->out_pitch;
        for (int x = 0; x < w; x++) {
            o[2 * x + 0] = (int16_t)(t0[x + 2] - t0[x]);
            o[2 * x + 1] = (int16_t)((t1[x + 2] + t1[x]) * 3 + t1[x + 1] * 10);
        }
    }
    free(t0);
    free(t1);
}

static void scharr_mt(const orc_u8plane* src, int16_t* out, int out_pitch, int nthreads) {
    scharr_job jb = {src, out, out_pitch};
    orc_parallel_for(src->h, nthreads, scharr_rows, &jb);
}

void orc_scharr(const orc_u8plane* src, int16_t* out) { scharr_mt(src, out, src->w, 1); }

/* derivI buffer: Scharr of the level, padded by `win` with zeros
   (copyMakeBorder BORDER_CONSTANT|BORDER_ISOLATED). */
static void make_deriv(const orc_u8plane* lv, int win, orc_s16plane* d, int nthreads) {
    d->w = lv->w;
    d->h = lv->h;
    d->pad = win;
    d->pitch = lv->w + 2 * win;
    size_t n = (size_t)d->pitch * (lv->h + 2 * win);
    d->buf = (int16_t*)calloc(n * 2, sizeof(int16_t));
    scharr_mt(lv, d->buf + 2 * ((size_t)win * d->pitch + win), d->pitch, nthreads);
}

typedef struct {
    const orc_u8plane* I;
    const orc_s16plane* dI;
    const orc_u8plane* J;
    const float* prev_pts;
    float* next_pts;
    uint8_t* status;
    float* err;
    int level, max_level, begin, end;
    const orc_klt_params* p;
} lk_job;

/* Accumulation order of the window sums A11/A12/A22 and b1/b2 (a parity
 * experiment switch; the default is the one the GPU matches):
 *   ORC_ACC_EXACT   exact int64 sums, rounded once to fp32 (the restatement's
 *                   documented choice: machine-independent, bit-exact on the GPU)
 *   ORC_ACC_F32     OpenCV 4.x's scalar loop: float accumulators, each int32
 *                   product converted to float and added in row-major order
 *                   (`iA11 += (itemtype)(ixval*ixval)`, itemtype = float)
 *   ORC_ACC_F32X4   OpenCV 4.x's CV_SIMD128 path: pixels 0..15 of each 21-pixel
 *                   row in 4-lane float accumulators (A: lane = x mod 4, fx*fx
 *                   then add, no FMA; b: int32 products of (dx,dy)x(diff,diff)
 *                   pairs, lanes (b1,b2,b1,b2) split over two accumulators),
 *                   pixels 16..20 in the scalar float accumulator, the lanes
 *                   reduced ((l0+l1)+(l2+l3)) and added last.
 * Not thread-safe to change while an LK call runs. */
static int lk_accum = ORC_ACC_EXACT;
void orc_set_lk_accum(int mode) { lk_accum = mode; }

typedef struct {
    float l[4];
} f4;
static float f4_sum(f4 v) { return (v.l[0] + v.l[1]) + (v.l[2] + v.l[3]); }

/* LKTrackerInvoker::operator() for points [begin, end) at one level. */
static void lk_level(const lk_job* jb) {
    const orc_u8plane* I = jb->I;
    const orc_s16plane* dI = jb->dI;
    const orc_u8plane* J = jb->J;
    const int win = jb->p->win;
    const int level = jb->level;
    const float halfw = (float)((win - 1) * 0.5f);
    const int W_BITS = 14, W_BITS1 = 14;
    const float FLT_SCALE = 1.f / (1 << 20);
    const double crit_eps = jb->p->eps * jb->p->eps;
    int16_t* Iwin = (int16_t*)malloc(sizeof(int16_t) * win * win);
    int16_t* dIwin = (int16_t*)malloc(sizeof(int16_t) * win * win * 2);
    const int dstep = dI->pitch * 2; /* in int16 elements */

    for (int pt = jb->begin; pt < jb->end; pt++) {
        float scale = (float)(1. / (1 << level));
        float prevx = jb->prev_pts[2 * pt] * scale;
        float prevy = jb->prev_pts[2 * pt + 1] * scale;
        float nextx, nexty;
        if (level == jb->max_level) {
            if (jb->p->use_initial_flow) {
                nextx = jb->next_pts[2 * pt] * scale;
                nexty = jb->next_pts[2 * pt + 1] * scale;
            } else {
                nextx = prevx;
                nexty = prevy;
            }
        } else {
            nextx = jb->next_pts[2 * pt] * 2.f;
            nexty = jb->next_pts[2 * pt + 1] * 2.f;
        }
        jb->next_pts[2 * pt] = nextx;
        jb->next_pts[2 * pt + 1] = nexty;

        prevx -= halfw;
        prevy -= halfw;
        int ipx = cv_floor(prevx), ipy = cv_floor(prevy);
        if (ipx < -win || ipx >= dI->w || ipy < -win || ipy >= dI->h) {
            if (level == 0) {
                jb->status[pt] = 0;
                jb->err[pt] = 0;
            }
            continue;
        }
        float a = prevx - ipx;
        float b = prevy - ipy;
        int iw00 = cv_round((1.f - a) * (1.f - b) * (1 << W_BITS));
        int iw01 = cv_round(a * (1.f - b) * (1 << W_BITS));
        int iw10 = cv_round((1.f - a) * b * (1 << W_BITS));
        int iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;

        int64_t iA11 = 0, iA12 = 0, iA22 = 0;
#ifdef ORC_ACC_STATS
        int64_t aA12 = 0, cA[3][5] = {{0}};
        double gx2[3] = {0, 0, 0}, gy2[3] = {0, 0, 0}, gax[3] = {0, 0, 0}, gay[3] = {0, 0, 0};
#endif
        float fA11 = 0.f, fA12 = 0.f, fA22 = 0.f;
        f4 qA11 = {{0}}, qA12 = {{0}}, qA22 = {{0}};
        const int simd_w = lk_accum == ORC_ACC_F32X4 ? win / 8 * 8 : 0;
        for (int y = 0; y < win; y++) {
            const uint8_t* src = px(I, ipx, ipy + y);
            const int16_t* dsrc = dI->buf + 2 * ((size_t)(ipy + y + dI->pad) * dI->pitch + ipx + dI->pad);
            int stepI = I->pitch;
            for (int x = 0; x < win; x++, dsrc += 2) {
                int ival = DESCALE(src[x] * iw00 + src[x + 1] * iw01 + src[x + stepI] * iw10 +
                                       src[x + stepI + 1] * iw11,
                                   W_BITS1 - 5);
                int ixval = DESCALE(dsrc[0] * iw00 + dsrc[2] * iw01 + dsrc[dstep] * iw10 +
                                        dsrc[dstep + 2] * iw11,
                                    W_BITS1);
                int iyval = DESCALE(dsrc[1] * iw00 + dsrc[3] * iw01 + dsrc[dstep + 1] * iw10 +
                                        dsrc[dstep + 3] * iw11,
                                    W_BITS1);
                Iwin[y * win + x] = (int16_t)ival;
                dIwin[(y * win + x) * 2] = (int16_t)ixval;
                dIwin[(y * win + x) * 2 + 1] = (int16_t)iyval;
                iA11 += (int64_t)ixval * ixval;
                iA12 += (int64_t)ixval * iyval;
                iA22 += (int64_t)iyval * iyval;
#ifdef ORC_ACC_STATS
                aA12 += llabs((int64_t)ixval * iyval);
                cA[0][x < 16 ? (x & 3) : 4] += (int64_t)ixval * ixval;
                cA[1][x < 16 ? (x & 3) : 4] += llabs((int64_t)ixval * iyval);
                cA[2][x < 16 ? (x & 3) : 4] += (int64_t)iyval * iyval;
                gx2[x >= 16 ? 2 : (x & 1)] += (double)ixval * ixval;
                gy2[x >= 16 ? 2 : (x & 1)] += (double)iyval * iyval;
                gax[x >= 16 ? 2 : (x & 1)] += abs(ixval);
                gay[x >= 16 ? 2 : (x & 1)] += abs(iyval);
#endif
                if (x < simd_w) {
                    const float fx = (float)ixval, fy = (float)iyval;
                    volatile float t11 = fx * fx, t12 = fx * fy, t22 = fy * fy;  /* no contraction */
                    qA22.l[x & 3] += t22;
                    qA12.l[x & 3] += t12;
                    qA11.l[x & 3] += t11;
                } else {
                    fA11 += (float)(ixval * ixval);
                    fA12 += (float)(ixval * iyval);
                    fA22 += (float)(iyval * iyval);
                }
            }
        }
#ifdef ORC_ACC_STATS
        orc_acc_stats[0]++;
        orc_acc_stats[1] += iA11 <= (1 << 24) && iA22 <= (1 << 24) && aA12 <= (1 << 24);
        {
            int ok = 1;
            for (int k = 0; k < 3; k++)
                for (int c = 0; c < 5; c++) ok &= cA[k][c] <= (1 << 24);
            orc_acc_stats[5] += ok;
        }
#endif
        float A11, A12, A22;
        if (lk_accum == ORC_ACC_EXACT) {
            A11 = (float)iA11 * FLT_SCALE;
            A12 = (float)iA12 * FLT_SCALE;
            A22 = (float)iA22 * FLT_SCALE;
        } else {
            if (lk_accum == ORC_ACC_F32X4) {
                fA11 += f4_sum(qA11);
                fA12 += f4_sum(qA12);
                fA22 += f4_sum(qA22);
            }
            A11 = fA11 * FLT_SCALE;
            A12 = fA12 * FLT_SCALE;
            A22 = fA22 * FLT_SCALE;
        }
        float D = A11 * A22 - A12 * A12;
        float minEig = (A22 + A11 - sqrtf((A11 - A22) * (A11 - A22) + 4.f * A12 * A12)) /
                       (float)(2 * win * win);
        if (minEig < jb->p->min_eig || D < FLT_EPSILON) {
            if (level == 0) {
                jb->status[pt] = 0;
                jb->err[pt] = 0;
            }
            continue;
        }
        D = 1.f / D;

        nextx -= halfw;
        nexty -= halfw;
        float pdx = 0.f, pdy = 0.f;
#ifdef ORC_ITER_STATS
        int j_used = 0;
#endif
        for (int j = 0; j < jb->p->max_iter; j++) {
#ifdef ORC_ITER_STATS
            j_used = j + 1;
#endif
            int inx = cv_floor(nextx), iny = cv_floor(nexty);
            if (inx < -win || inx >= J->w || iny < -win || iny >= J->h) {
                if (level == 0) jb->status[pt] = 0;
                break;
            }
            a = nextx - inx;
            b = nexty - iny;
            iw00 = cv_round((1.f - a) * (1.f - b) * (1 << W_BITS));
            iw01 = cv_round(a * (1.f - b) * (1 << W_BITS));
            iw10 = cv_round((1.f - a) * b * (1 << W_BITS));
            iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
            int64_t ib1 = 0, ib2 = 0;
#ifdef ORC_ACC_STATS
            int64_t ab1 = 0, ab2 = 0, cb[2][5] = {{0}};
            int64_t cls[2][3] = {{0}};           /* |p| by class: even x<16, odd x<16, x>=16 */
            int64_t lane[32][2][3];              /* per lane (unit k -> lane k % 32) */
            int maxd[32];
            double d2c[3] = {0, 0, 0};
            int mdc[3] = {0, 0, 0};
            memset(lane, 0, sizeof lane);
            memset(maxd, 0, sizeof maxd);
#endif
            float fb1 = 0.f, fb2 = 0.f;
            f4 qb0 = {{0}}, qb1 = {{0}};
            for (int y = 0; y < win; y++) {
                const uint8_t* Jp = px(J, inx, iny + y);
                int stepJ = J->pitch;
                for (int x = 0; x < win; x++) {
                    int diff = DESCALE(Jp[x] * iw00 + Jp[x + 1] * iw01 + Jp[x + stepJ] * iw10 +
                                           Jp[x + stepJ + 1] * iw11,
                                       W_BITS1 - 5) -
                               Iwin[y * win + x];
                    const int p1 = diff * dIwin[(y * win + x) * 2], p2 = diff * dIwin[(y * win + x) * 2 + 1];
                    ib1 += p1;
                    ib2 += p2;
#ifdef ORC_ACC_STATS
                    ab1 += p1 < 0 ? -p1 : p1;
                    ab2 += p2 < 0 ? -p2 : p2;
                    cb[0][x < 16 ? (x & 3) : 4] += p1 < 0 ? -p1 : p1;
                    cb[1][x < 16 ? (x & 3) : 4] += p2 < 0 ? -p2 : p2;
                    {
                        const int c = x >= 16 ? 2 : (x & 1), ln = (3 * y + x / 7) % 32;
                        cls[0][c] += p1 < 0 ? -p1 : p1;
                        cls[1][c] += p2 < 0 ? -p2 : p2;
                        lane[ln][0][c] += p1 < 0 ? -p1 : p1;
                        lane[ln][1][c] += p2 < 0 ? -p2 : p2;
                        d2c[c] += (double)diff * diff;
                        if ((diff < 0 ? -diff : diff) > mdc[c]) mdc[c] = diff < 0 ? -diff : diff;
                        const int ad = diff < 0 ? -diff : diff;
                        if (ad > maxd[ln]) maxd[ln] = ad;
                    }
#endif
                    if (x < simd_w) {
                        /* v_mul_expand of (dx,dy) pairs by (diff,diff): pixels x%4 in {0,1}
                           feed qb0 lanes (2(x%2), 2(x%2)+1), pixels x%4 in {2,3} feed qb1 */
                        f4* q = (x & 2) ? &qb1 : &qb0;
                        q->l[2 * (x & 1)] += (float)p1;
                        q->l[2 * (x & 1) + 1] += (float)p2;
                    } else {
                        fb1 += (float)p1;
                        fb2 += (float)p2;
                    }
                }
            }
#ifdef ORC_ACC_STATS
            orc_acc_stats[2]++;
            orc_acc_stats[3] += ab1 <= (1 << 24) && ab2 <= (1 << 24);
            {
                int ok = 1;
                for (int k = 0; k < 2; k++)
                    for (int c = 0; c < 5; c++) ok &= cb[k][c] <= (1 << 24);
                orc_acc_stats[4] += ok;
                int ok1 = 1, ok2 = 1;
                for (int k = 0; k < 2; k++)
                    for (int c = 0; c < 3; c++) ok1 &= cls[k][c] <= (1 << 24);
                for (int ln = 0; ln < 32; ln++)
                    for (int k = 0; k < 2; k++)
                        for (int c = 0; c < 3; c++) ok2 &= lane[ln][k][c] <= (1 << 19);
                orc_acc_stats[6] += ok1;
                orc_acc_stats[7] += ok2;
                {
                    /* Cauchy-Schwarz bounds: per class D2_c, and D2 total */
                    int ok3 = 1, ok4 = 1;
                    const double d2t = d2c[0] + d2c[1] + d2c[2];
                    for (int c = 0; c < 3; c++) {
                        ok3 &= d2c[c] * gx2[c] <= 281474976710656.0 && d2c[c] * gy2[c] <= 281474976710656.0;
                        ok4 &= d2t * gx2[c] <= 281474976710656.0 && d2t * gy2[c] <= 281474976710656.0;
                    }
                    orc_acc_stats[8] += ok3;
                    int ok5 = 1, ok6 = 1;
                    const int mdt = mdc[0] > mdc[1] ? (mdc[0] > mdc[2] ? mdc[0] : mdc[2]) : (mdc[1] > mdc[2] ? mdc[1] : mdc[2]);
                    for (int c = 0; c < 3; c++) {
                        ok5 &= (double)mdc[c] * gax[c] <= 16777216.0 && (double)mdc[c] * gay[c] <= 16777216.0;
                        ok6 &= (double)mdt * gax[c] <= 16777216.0 && (double)mdt * gay[c] <= 16777216.0;
                    }
                    orc_acc_stats[10] += ok5;
                    orc_acc_stats[11] += ok6;
                    orc_acc_stats[9] += ok4;
                }
            }
#endif
            float b1, b2;
            if (lk_accum == ORC_ACC_EXACT) {
                b1 = (float)ib1 * FLT_SCALE;
                b2 = (float)ib2 * FLT_SCALE;
            } else {
                if (lk_accum == ORC_ACC_F32X4) {
                    /* v_recombine(v_interleave_pairs(qb0 + qb1), 0): (l0, l2) -> b1, (l1, l3) -> b2 */
                    f4 s4;
                    for (int k = 0; k < 4; k++) s4.l[k] = qb0.l[k] + qb1.l[k];
                    fb1 += (s4.l[0] + s4.l[2]);
                    fb2 += (s4.l[1] + s4.l[3]);
                }
                b1 = fb1 * FLT_SCALE;
                b2 = fb2 * FLT_SCALE;
            }
            float dx = (A12 * b2 - A22 * b1) * D;
            float dy = (A12 * b1 - A11 * b2) * D;
            nextx += dx;
            nexty += dy;
            jb->next_pts[2 * pt] = nextx + halfw;
            jb->next_pts[2 * pt + 1] = nexty + halfw;
            if ((double)dx * dx + (double)dy * dy <= crit_eps) break;
            if (j > 0 && fabsf(dx + pdx) < 0.01f && fabsf(dy + pdy) < 0.01f) {
                jb->next_pts[2 * pt] -= dx * 0.5f;
                jb->next_pts[2 * pt + 1] -= dy * 0.5f;
                break;
            }
            pdx = dx;
            pdy = dy;
        }
#ifdef ORC_ITER_STATS
        orc_iter_hist[level][j_used]++;  /* single-threaded diagnostic build only */
#endif

        if (jb->status[pt] && level == 0) {
            float nx = jb->next_pts[2 * pt] - halfw;
            float ny = jb->next_pts[2 * pt + 1] - halfw;
            int inx = cv_floor(nx), iny = cv_floor(ny);
            if (inx < -win || inx >= J->w || iny < -win || iny >= J->h) {
                jb->status[pt] = 0;
                continue;
            }
            float aa = nx - inx, bb = ny - iny;
            iw00 = cv_round((1.f - aa) * (1.f - bb) * (1 << W_BITS));
            iw01 = cv_round(aa * (1.f - bb) * (1 << W_BITS));
            iw10 = cv_round((1.f - aa) * bb * (1 << W_BITS));
            iw11 = (1 << W_BITS) - iw00 - iw01 - iw10;
            /* sum of |diff| < 2^24: the float accumulation of OpenCV is exact. */
            int64_t errsum = 0;
            for (int y = 0; y < win; y++) {
                const uint8_t* Jp = px(J, inx, iny + y);
                int stepJ = J->pitch;
                for (int x = 0; x < win; x++) {
                    int diff = DESCALE(Jp[x] * iw00 + Jp[x + 1] * iw01 + Jp[x + stepJ] * iw10 +
                                           Jp[x + stepJ + 1] * iw11,
                                       W_BITS1 - 5) -
                               Iwin[y * win + x];
                    errsum += diff < 0 ? -diff : diff;
                }
            }
            /* errval * 1.f/(32*win*win): (errval*1.f) / 14112 by C precedence */
            jb->err[pt] = (float)errsum * 1.f / (float)(32 * win * win);
        }
    }
    free(Iwin);
    free(dIwin);
}

static void lk_range(void* vctx, int begin, int end) {
    lk_job jb = *(const lk_job*)vctx;
    jb.begin = begin;
    jb.end = end;
    lk_level(&jb);
}

static void run_level(lk_job* base, int n, int nthreads) { orc_parallel_for(n, nthreads, lk_range, base); }

void orc_lk_on_pyramids(const orc_pyramid* prev, const orc_pyramid* next, const float* prev_xy,
                        float* next_xy, uint8_t* status, float* err, int n, const orc_klt_params* p,
                        int nthreads) {
    int max_level = prev->nlevels - 1;
    if (next->nlevels - 1 < max_level) max_level = next->nlevels - 1;
    if (!p->use_initial_flow) memcpy(next_xy, prev_xy, sizeof(float) * 2 * n);
    for (int i = 0; i < n; i++) {
        status[i] = 1;
        err[i] = 0.f;
    }
    for (int level = max_level; level >= 0; level--) {
        orc_s16plane d;
        make_deriv(&prev->lv[level], p->win, &d, nthreads);
        lk_job jb;
        jb.I = &prev->lv[level];
        jb.dI = &d;
        jb.J = &next->lv[level];
        jb.prev_pts = prev_xy;
        jb.next_pts = next_xy;
        jb.status = status;
        jb.err = err;
        jb.level = level;
        jb.max_level = max_level;
        jb.p = p;
        run_level(&jb, n, nthreads);
        free(d.buf);
    }
}

void orc_calc_optical_flow_pyr_lk(const uint8_t* prev, const uint8_t* next, int w, int h, int stride,
                                  const float* prev_xy, float* next_xy, uint8_t* status, float* err,
                                  int n, const orc_klt_params* p, int nthreads) {
    if (n <= 0) return;
    orc_pyramid pp, pn;
    build_pyramid_mt(prev, w, h, stride, p->win, p->max_level, &pp, nthreads);
    build_pyramid_mt(next, w, h, stride, p->win, p->max_level, &pn, nthreads);
    orc_lk_on_pyramids(&pp, &pn, prev_xy, next_xy, status, err, n, p, nthreads);
    orc_free_pyramid(&pp);
    orc_free_pyramid(&pn);
}

/* Tracking::isOnBorder (tracking.cc:847-849). */
static int is_on_border(float x, float y, double border, int cam_w, int cam_h) {
    return x < border || y < border || (x > (cam_w - border)) || (y > (cam_h - border));
}

/* Tracking::ptsDistance (tracking.cc:841-845): float subtraction, double sqrt. */
static double pts_distance(const float* a, const float* b) {
    double dx = a[0] - b[0];
    double dy = a[1] - b[1];
    return sqrt(dx * dx + dy * dy);
}

int orc_klt_fb(const uint8_t* prev, const uint8_t* next, int w, int h, int stride,
               const float* prev_xy, float* next_xy, float* back_xy, uint8_t* st_f, uint8_t* st_b,
               uint8_t* keep, int* kept_idx, int n, double fb_thresh, double border, int cam_w,
               int cam_h, const orc_klt_params* p, int reuse_pyramids, int nthreads) {
    if (n <= 0) return 0;
    float* err = (float*)malloc(sizeof(float) * n);
    /* pts2d_reverse = pts2d_map (tracking.cc:383) */
    memcpy(back_xy, prev_xy, sizeof(float) * 2 * n);
    if (reuse_pyramids) {
        orc_pyramid pp, pn;
        build_pyramid_mt(prev, w, h, stride, p->win, p->max_level, &pp, nthreads);
        build_pyramid_mt(next, w, h, stride, p->win, p->max_level, &pn, nthreads);
        orc_lk_on_pyramids(&pp, &pn, prev_xy, next_xy, st_f, err, n, p, nthreads);
        orc_lk_on_pyramids(&pn, &pp, next_xy, back_xy, st_b, err, n, p, nthreads);
        orc_free_pyramid(&pp);
        orc_free_pyramid(&pn);
    } else {
        orc_calc_optical_flow_pyr_lk(prev, next, w, h, stride, prev_xy, next_xy, st_f, err, n, p,
                                     nthreads);
        orc_calc_optical_flow_pyr_lk(next, prev, w, h, stride, next_xy, back_xy, st_b, err, n, p,
                                     nthreads);
    }
    int kept = 0;
    for (int k = 0; k < n; k++) {
        int ok = st_f[k] && st_b[k] && !is_on_border(next_xy[2 * k], next_xy[2 * k + 1], border, cam_w, cam_h) &&
                 (pts_distance(&back_xy[2 * k], &prev_xy[2 * k]) < fb_thresh);
        keep[k] = (uint8_t)ok;
        if (ok) kept_idx[kept++] = k;
    }
    free(err);
    return kept;
}
