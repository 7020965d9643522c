// api_graph.cpp -- C ABI of the hipGraph capture (include/gvx.h): one frame
// pair per graph launch.  The *_dev entry points only
// enqueue on the context stream and never synchronise or allocate once their
// scratch buffers are sized, so a stream capture of them replays the same
// kernels on the same buffers.
#include <hip/hip_runtime.h>

#include <new>

#include "gvx_internal.h"

using namespace gvx;

struct gvx_graph {
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    const gvx_ctx* ctx = nullptr;
    uint64_t mem_gen = 0;  // the context's memory generation the graph's pointers belong to
};

gvx_status gvx_capture_begin(gvx_ctx* c) {
    if (!c) return GVX_ERR_INVALID;
    if (c->in_branch || c->branch_open) return set_err(c, GVX_ERR_INVALID, "join the open branch before capturing");
    // the profiling brackets record and query events on the host: not capturable
    if (c->prof) return set_err(c, GVX_ERR_INVALID, "disable profiling before capturing a graph");
    if (c->capturing) return set_err(c, GVX_ERR_INVALID, "a capture is already open");
    hipSetDevice(c->device);
    gvx_status s = hip_err(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
    if (s == GVX_OK) {
        c->capturing = true;
        c->capture_failed = false;
        c->capture_gen = c->mem_gen;
    }
    return s;
}

gvx_status gvx_capture_abort(gvx_ctx* c) {
    if (!c) return GVX_ERR_INVALID;
    if (!c->capturing) return GVX_OK;
    hipSetDevice(c->device);
    // close an open branch first: the capture cannot end with the side stream unjoined
    if (c->in_branch) gvx_branch_end(c);
    if (c->branch_open) gvx_branch_join(c);
    c->capturing = false;
    c->capture_failed = false;
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(c->stream, &g);
    if (g) hipGraphDestroy(g);
    (void)hipGetLastError();
    return e == hipSuccess ? GVX_OK : hip_err(c, e, "hipStreamEndCapture (abort)");
}

gvx_status gvx_capture_end(gvx_ctx* c, gvx_graph** out) {
    if (!c || !out) return GVX_ERR_INVALID;
    *out = nullptr;
    hipSetDevice(c->device);
    if (!c->capturing) return set_err(c, GVX_ERR_INVALID, "no capture is open");
    if (c->in_branch || c->branch_open) return set_err(c, GVX_ERR_INVALID, "join the open branch before ending the capture");
    c->capturing = false;
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(c->stream, &g);
    if (e != hipSuccess) return hip_err(c, e, "hipStreamEndCapture");
    if (c->mem_gen != c->capture_gen) {
        hipGraphDestroy(g);
        return set_err(c, GVX_ERR_INVALID, "device buffers moved during the capture");
    }
    if (c->capture_failed) {
        c->capture_failed = false;
        hipGraphDestroy(g);
        return set_err(c, GVX_ERR_INVALID, "a call inside the capture needed a device allocation; run it once "
                                           "uncaptured first");
    }
    hipGraphExec_t x = nullptr;
    e = hipGraphInstantiate(&x, g, nullptr, nullptr, 0);
    if (e != hipSuccess) {
        hipGraphDestroy(g);
        return hip_err(c, e, "hipGraphInstantiate");
    }
    gvx_graph* h = new (std::nothrow) gvx_graph;
    if (!h) {
        hipGraphExecDestroy(x);
        hipGraphDestroy(g);
        return set_err(c, GVX_ERR_OOM, "graph handle");
    }
    h->graph = g;
    h->exec = x;
    h->ctx = c;
    h->mem_gen = c->mem_gen;
    *out = h;
    return GVX_OK;
}

gvx_status gvx_graph_launch(gvx_ctx* c, const gvx_graph* g) {
    if (!c || !g || !g->exec) return GVX_ERR_INVALID;
    if (g->ctx != c) return set_err(c, GVX_ERR_INVALID, "graph captured on another context");
    if (g->mem_gen != c->mem_gen)
        return set_err(c, GVX_ERR_INVALID, "stale graph: scratch or frame memory was reallocated after capture");
    hipSetDevice(c->device);
    return hip_err(c, hipGraphLaunch(g->exec, c->stream), "hipGraphLaunch");
}

void gvx_graph_destroy(gvx_graph* g) {
    if (!g) return;
    if (g->exec) hipGraphExecDestroy(g->exec);
    if (g->graph) hipGraphDestroy(g->graph);
    delete g;
}

gvx_status gvx_copy_dev(gvx_ctx* c, void* d_dst, const void* d_src, size_t bytes) {
    if (!c) return GVX_ERR_INVALID;
    if (bytes == 0) return GVX_OK;
    if (!d_dst || !d_src) return set_err(c, GVX_ERR_INVALID, "null device pointer");
    hipSetDevice(c->device);
    // a kernel, not hipMemcpyAsync: in a captured graph a memcpy node made the
    // one-pair replay slower than the eager calls (67 vs 60 us, r01)
    return hip_err(c, launch_copy(c, d_dst, d_src, bytes), "copy kernel");
}

// One side branch of the context (include/gvx.h): the calls between
// gvx_branch_begin and gvx_branch_end run on a second stream that first waits
// for everything enqueued before the branch; gvx_branch_join makes the context
// stream wait for the branch.  Under a capture the event record / wait pairs
// become graph edges, so the branch is a parallel path of the graph.
gvx_status gvx_branch_begin(gvx_ctx* c) {
    if (!c) return GVX_ERR_INVALID;
    if (c->in_branch || c->branch_open) return set_err(c, GVX_ERR_INVALID, "a branch is already open");
    if (c->prof && c->capturing) return set_err(c, GVX_ERR_INVALID, "disable profiling before branching");
    hipSetDevice(c->device);
    if (!c->side) {
        if (c->capturing) return set_err(c, GVX_ERR_INVALID, "open a first branch outside a capture");
        hipError_t e;
        if (c->side_low_prio) {  // the branch yields to the context stream (GVX_SIDE_LOW_PRIO)
            int least = 0, greatest = 0;
            e = hipDeviceGetStreamPriorityRange(&least, &greatest);
            if (e == hipSuccess)
                e = hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, c->side_low_prio == 2 ? greatest : least);
        } else {
            e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
        }
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming);
        if (e != hipSuccess) return hip_err(c, e, "branch stream");
    }
    hipError_t e = hipEventRecord(c->fork_ev, c->main);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->side, c->fork_ev, 0);
    if (e != hipSuccess) return hip_err(c, e, "branch fork");
    c->stream = c->side;
    c->in_branch = true;
    return GVX_OK;
}

gvx_status gvx_branch_end(gvx_ctx* c) {
    if (!c) return GVX_ERR_INVALID;
    if (!c->in_branch) return set_err(c, GVX_ERR_INVALID, "no branch is open");
    hipSetDevice(c->device);
    c->stream = c->main;
    c->in_branch = false;
    c->branch_open = true;
    return hip_err(c, hipEventRecord(c->join_ev, c->side), "branch end");
}

gvx_status gvx_branch_join(gvx_ctx* c) {
    if (!c) return GVX_ERR_INVALID;
    if (c->in_branch) return set_err(c, GVX_ERR_INVALID, "end the branch before joining it");
    if (!c->branch_open) return GVX_OK;
    hipSetDevice(c->device);
    c->branch_open = false;
    return hip_err(c, hipStreamWaitEvent(c->main, c->join_ev, 0), "branch join");
}
