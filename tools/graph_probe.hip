// graph_probe.hip -- how ROCm runs the shapes the sequence replay could take
// (timing probe for DESIGN §4, not product code).  Busy-wait kernels of fixed
// length stand in for the per-frame work:
//   A  two independent 30 us nodes in ONE graph (concurrent ~30 us, serial ~60)
//   B  per frame: node1 33 us -> node 5 -> node 5 -> node 4 (the tracking chain),
//      K frames in one graph (graph launch cost amortised over K)
//   C  the pipelined shape of gvx's tracker: per frame a 4-node tracking graph on
//      stream 1 and a 30 us preprocessing graph on stream 2, event fork / join
//   D  the same chain as B launched one graph per frame on one stream
// Build: hipcc --offload-arch=gfx950 -O2 tools/graph_probe.hip -o tools/graph_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// one workgroup per CU-ish, each spinning `us` microseconds on the 100 MHz clock
__global__ void spin(int us, int* sink) {
    const uint64_t t0 = wall_clock64();
    const uint64_t n = (uint64_t)us * 100;
    uint64_t t = t0;
    while (t - t0 < n) t = wall_clock64();
    if (threadIdx.x == 0 && blockIdx.x == 0 && sink) sink[0] = (int)(t - t0);
}

static void node(hipGraph_t g, hipGraphNode_t* out, const hipGraphNode_t* deps, int nd, int us, int blocks,
                 int* sink) {
    hipKernelNodeParams p{};
    void* args[] = {&us, &sink};
    p.func = (void*)spin;
    p.gridDim = dim3(blocks);
    p.blockDim = dim3(64);
    p.kernelParams = args;
    CK(hipGraphAddKernelNode(out, g, deps, nd, &p));
}

static float time_launches(hipGraphExec_t ge, hipStream_t s, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1000.f / reps;
}

int main(int argc, char** argv) {
    int* sink;
    CK(hipMalloc(&sink, 64));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const int reps = 200;
    // A: two parallel 30 us nodes
    {
        hipGraph_t g;
        CK(hipGraphCreate(&g, 0));
        hipGraphNode_t n1, n2;
        node(g, &n1, nullptr, 0, 30, 64, sink);
        node(g, &n2, nullptr, 0, 30, 64, sink);
        hipGraphExec_t ge;
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        printf("A two parallel 30us nodes: %.2f us per graph\n", time_launches(ge, s1, reps));
        hipGraphExec_t ge1;
        hipGraph_t g1;
        CK(hipGraphCreate(&g1, 0));
        node(g1, &n1, nullptr, 0, 30, 64, sink);
        CK(hipGraphInstantiate(&ge1, g1, nullptr, nullptr, 0));
        printf("A one 30us node: %.2f us per graph\n", time_launches(ge1, s1, reps));
    }
    // B / B+pre: K frames per graph, chain 33 -> 5 -> 5 -> 4 (+ a parallel 30 us branch per frame)
    for (int pre = 0; pre < 2; ++pre)
        for (int K : {1, 4, 16}) {
            hipGraph_t g;
            CK(hipGraphCreate(&g, 0));
            hipGraphNode_t last{};
            bool have = false;
            for (int f = 0; f < K; ++f) {
                hipGraphNode_t a, b, c, d, p;
                node(g, &a, have ? &last : nullptr, have ? 1 : 0, 33, 150, sink);
                if (pre) node(g, &p, have ? &last : nullptr, have ? 1 : 0, 30, 256, sink);
                node(g, &b, &a, 1, 5, 64, sink);
                node(g, &c, &b, 1, 5, 18, sink);
                hipGraphNode_t dd[2] = {c, p};
                node(g, &d, dd, pre ? 2 : 1, 4, 1, sink);
                last = d;
                have = true;
            }
            hipGraphExec_t ge;
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            const float us = time_launches(ge, s1, reps / K + 1);
            printf("B chain 33/5/5/4%s, %2d frames per graph: %.2f us per frame\n", pre ? " + parallel 30" : "", K,
                   us / K);
        }
    // C: the two-stream pipelined form (tracking graph on s1, preprocessing graph on s2)
    {
        hipGraph_t gt, gp;
        CK(hipGraphCreate(&gt, 0));
        CK(hipGraphCreate(&gp, 0));
        hipGraphNode_t a, b, c, d, p;
        node(gt, &a, nullptr, 0, 33, 150, sink);
        node(gt, &b, &a, 1, 5, 64, sink);
        node(gt, &c, &b, 1, 5, 18, sink);
        node(gt, &d, &c, 1, 4, 1, sink);
        node(gp, &p, nullptr, 0, 30, 256, sink);
        hipGraphExec_t et, ep;
        CK(hipGraphInstantiate(&et, gt, nullptr, nullptr, 0));
        CK(hipGraphInstantiate(&ep, gp, nullptr, nullptr, 0));
        hipEvent_t fork, join;
        CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
        hipEvent_t a0, b0;
        CK(hipEventCreate(&a0));
        CK(hipEventCreate(&b0));
        for (int pass = 0; pass < 2; ++pass) {
            CK(hipEventRecord(join, s2));
            CK(hipStreamSynchronize(s1));
            CK(hipEventRecord(a0, s1));
            for (int i = 0; i < reps; ++i) {
                CK(hipStreamWaitEvent(s1, join, 0));
                CK(hipEventRecord(fork, s1));
                CK(hipStreamWaitEvent(s2, fork, 0));
                CK(hipGraphLaunch(ep, s2));
                CK(hipEventRecord(join, s2));
                CK(hipGraphLaunch(et, s1));
            }
            CK(hipStreamWaitEvent(s1, join, 0));
            CK(hipEventRecord(b0, s1));
            CK(hipEventSynchronize(b0));
            float ms;
            CK(hipEventElapsedTime(&ms, a0, b0));
            if (pass) printf("C two-stream pipelined (graphs + event fork/join): %.2f us per frame\n", ms * 1000 / reps);
        }
        // D: the tracking graph alone, back to back on one stream
        printf("D tracking graph alone, one per frame: %.2f us per frame\n", time_launches(et, s1, reps));
        // E: C without the join on s1 (fork only)
        CK(hipStreamSynchronize(s2));
        CK(hipEventRecord(a0, s1));
        for (int i = 0; i < reps; ++i) {
            CK(hipEventRecord(fork, s1));
            CK(hipStreamWaitEvent(s2, fork, 0));
            CK(hipGraphLaunch(ep, s2));
            CK(hipGraphLaunch(et, s1));
        }
        CK(hipEventRecord(b0, s1));
        CK(hipEventSynchronize(b0));
        CK(hipStreamSynchronize(s2));
        float ms;
        CK(hipEventElapsedTime(&ms, a0, b0));
        printf("E two streams, fork only (no join wait on s1): %.2f us per frame\n", ms * 1000 / reps);
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
