// Phase timing of the fused pyramid pass (diagnostics, not part of libgvx):
// 256 random 1280x560 images, fused_kernel<3, STOP> for every truncation point.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off
//        -I include -I ic-gvins_amd/csrc tools/pyr_micro.hip -o tools/pyr_micro
#include "../ic-gvins_amd/csrc/pyramid.hip"

#include <cstdio>
#include <vector>

using namespace gvx;

__global__ void read_all(const uint4* __restrict__ p, size_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

float time_read(const uint8_t* src, size_t bytes, uint32_t* sink, int blocks, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    read_all<<<blocks, 256>>>((const uint4*)src, bytes / 16, sink);
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) read_all<<<blocks, 256>>>((const uint4*)src, bytes / 16, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return 1000.f * ms / reps;
}

template <int STOP>
float run(const uint8_t* src, uint8_t* dst, const PyrLayout& lay, int n_img, int n_cu, int reps) {
    DownLevels D{};
    for (int k = 0; k < 3; ++k) {
        D.off[k] = lay.off[1 + k];
        D.pitch[k] = lay.pitch[1 + k];
        D.w[k] = lay.w[1 + k];
        D.h[k] = lay.h[1 + k];
    }
    const int w = lay.w[0], h = lay.h[0];
    const int tiles_x = (w + 127) / 128, tiles_y = (h + 63) / 64, n_tiles = tiles_x * tiles_y * n_img;
    const int slots = n_cu * 5, per_wg = (n_tiles + slots - 1) / slots, n_wg = (n_tiles + per_wg - 1) / per_wg;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i)
        hipLaunchKernelGGL((fused_kernel<3, STOP>), dim3(N_XCD * xcd_per(n_wg)), dim3(256), 0, 0, src, (int64_t)w * h, w, w, h, 1,
                           dst, lay.bytes, D, tiles_x, tiles_y, n_tiles, per_wg);
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((fused_kernel<3, STOP>), dim3(N_XCD * xcd_per(n_wg)), dim3(256), 0, 0, src, (int64_t)w * h, w, w, h, 1,
                           dst, lay.bytes, D, tiles_x, tiles_y, n_tiles, per_wg);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return 1000.f * ms / reps;
}

int main() {
    const int w = 1280, h = 560, n = 256, reps = 20;
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    PyrLayout lay = make_layout(w, h, 3, 21);
    std::vector<uint8_t> img((size_t)w * h * n);
    uint32_t x = 12345;
    for (auto& v : img) v = (uint8_t)((x = x * 1664525u + 1013904223u) >> 24);
    uint8_t *src, *dst;
    hipMalloc(&src, img.size());
    hipMalloc(&dst, (size_t)lay.bytes * n);
    hipMemcpy(src, img.data(), img.size(), hipMemcpyHostToDevice);
    const int cu = prop.multiProcessorCount;
    for (int blocks : {cu * 4, cu * 8, cu * 16, cu * 32}) {
        const float us = time_read(src, img.size(), (uint32_t*)dst, blocks, reps);
        printf("read_all %5d blocks  %8.1f us  %6.2f TB/s\n", blocks, us, img.size() / us / 1e6);
    }
    printf("stage0 (staging)      %8.1f us\n", run<0>(src, dst, lay, n, cu, reps));
    printf("stage1 (+h L1)        %8.1f us\n", run<1>(src, dst, lay, n, cu, reps));
    printf("stage2 (+v L1)        %8.1f us\n", run<2>(src, dst, lay, n, cu, reps));
    printf("stage3 (+own/fix L1)  %8.1f us\n", run<3>(src, dst, lay, n, cu, reps));
    printf("stage6 (+L2)          %8.1f us\n", run<6>(src, dst, lay, n, cu, reps));
    printf("full                  %8.1f us\n", run<99>(src, dst, lay, n, cu, reps));
    printf("bytes in %.1f MB\n", img.size() / 1e6);
    return 0;
}
