/* orc_pool.h -- minimal persistent thread pool for the CPU restatement
 * (test infrastructure).  Mirrors OpenCV's parallel_for_ over row / point
 * ranges so the multi-core CPU baseline parallelises the same stages the
 * reference's OpenCV build does (pyrDown, calcSharrDeriv, LKTrackerInvoker).
 * Results never depend on the thread count: every range writes disjoint
 * outputs with integer or per-item arithmetic. */
#ifndef ORC_POOL_H
#define ORC_POOL_H

typedef void (*orc_range_fn)(void* ctx, int begin, int end);

/* Run fn over [0, n) split into at most nthreads contiguous chunks (the caller
   takes part).  nthreads <= 1 runs inline. */
void orc_parallel_for(int n, int nthreads, orc_range_fn fn, void* ctx);

#endif
