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
};

gvx_status gvx_capture_begin(gvx_ctx* c) {
    if (!c) return GVX_ERR_INVALID;
    // the profiling brackets record and query events on the host: not capturable
    if (c->prof) return set_err(c, GVX_ERR_INVALID, "disable profiling before capturing a graph");
    hipSetDevice(c->device);
    return hip_err(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
}

gvx_status gvx_capture_end(gvx_ctx* c, gvx_graph** out) {
    if (!c || !out) return GVX_ERR_INVALID;
    *out = nullptr;
    hipSetDevice(c->device);
    hipGraph_t g = nullptr;
    hipError_t e = hipStreamEndCapture(c->stream, &g);
    if (e != hipSuccess) return hip_err(c, e, "hipStreamEndCapture");
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
    *out = h;
    return GVX_OK;
}

gvx_status gvx_graph_launch(gvx_ctx* c, const gvx_graph* g) {
    if (!c || !g || !g->exec) return GVX_ERR_INVALID;
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
    return hip_err(c, hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, c->stream), "hipMemcpyAsync D2D");
}
