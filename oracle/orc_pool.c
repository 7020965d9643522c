/* orc_pool.c -- see orc_pool.h (test infrastructure). */
#include "orc_pool.h"

#include <pthread.h>

#define ORC_MAX_WORKERS 63

static pthread_mutex_t g_call = PTHREAD_MUTEX_INITIALIZER; /* one parallel_for at a time */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_work = PTHREAD_COND_INITIALIZER;
static pthread_cond_t g_done = PTHREAD_COND_INITIALIZER;
static int g_workers = 0;
static pthread_t g_th[ORC_MAX_WORKERS];
/* current job (guarded by g_mu) */
static orc_range_fn g_fn;
static void* g_ctx;
static int g_n, g_chunks, g_next, g_finished;
static unsigned g_gen;

static void run_chunk(int c) {
    int b = (int)((long)g_n * c / g_chunks), e = (int)((long)g_n * (c + 1) / g_chunks);
    if (b < e) g_fn(g_ctx, b, e);
}

static void* worker(void* arg) {
    (void)arg;
    unsigned seen = 0;
    pthread_mutex_lock(&g_mu);
    for (;;) {
        while (g_gen == seen) pthread_cond_wait(&g_work, &g_mu);
        seen = g_gen;
        while (g_next < g_chunks) {
            int c = g_next++;
            pthread_mutex_unlock(&g_mu);
            run_chunk(c);
            pthread_mutex_lock(&g_mu);
            if (++g_finished == g_chunks) pthread_cond_signal(&g_done);
        }
    }
    return 0;
}

void orc_parallel_for(int n, int nthreads, orc_range_fn fn, void* ctx) {
    if (n <= 0) return;
    if (nthreads > n) nthreads = n;
    if (nthreads > ORC_MAX_WORKERS + 1) nthreads = ORC_MAX_WORKERS + 1;
    if (nthreads <= 1) {
        fn(ctx, 0, n);
        return;
    }
    pthread_mutex_lock(&g_call);
    pthread_mutex_lock(&g_mu);
    while (g_workers < nthreads - 1) {
        pthread_create(&g_th[g_workers], 0, worker, 0);
        pthread_detach(g_th[g_workers]);
        g_workers++;
    }
    g_fn = fn;
    g_ctx = ctx;
    g_n = n;
    g_chunks = nthreads;
    g_next = 0;
    g_finished = 0;
    g_gen++;
    pthread_cond_broadcast(&g_work);
    while (g_next < g_chunks) {
        int c = g_next++;
        pthread_mutex_unlock(&g_mu);
        run_chunk(c);
        pthread_mutex_lock(&g_mu);
        ++g_finished;
    }
    while (g_finished < g_chunks) pthread_cond_wait(&g_done, &g_mu);
    pthread_mutex_unlock(&g_mu);
    pthread_mutex_unlock(&g_call);
}
