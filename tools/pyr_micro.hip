// Phase timing of the pyramid passes (diagnostics, not part of libgvx):
// 256 random 1280x560 images; the streaming pass (levels 1-3 and their rings)
// with and without its stores, and a plain streaming read of the same bytes.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off
//        -Wno-unused-result -I include -I ic-gvins_amd/csrc tools/pyr_micro.hip -o tools/pyr_micro
#include "../ic-gvins_amd/csrc/pyramid.hip"

#include <cstdio>
#include <vector>

using namespace gvx;

namespace gvx {
void* scratch(gvx_ctx*, const std::string&, size_t) { return nullptr; }
}

__global__ void read_all(const uint4* __restrict__ p, size_t n16, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

template <class F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) f();
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return 1000.f * ms / reps;
}

int main() {
    const int w = 1280, h = 560, n = 256, reps = 20;
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    PyrLayout lay = make_layout(w, h, 3, 21);
    std::vector<uint8_t> img((size_t)w * h * n);
    uint32_t x = 12345;
    for (auto& v : img) v = (uint8_t)((x = x * 1664525u + 1013904223u) >> 24);
    uint8_t *src, *dst, *trash;
    hipMalloc(&src, img.size());
    hipMalloc(&dst, (size_t)lay.bytes * n);
    hipMalloc(&trash, 1 << 24);
    hipMemcpy(src, img.data(), img.size(), hipMemcpyHostToDevice);
    DownLevels D{};
    for (int k = 0; k < 3; ++k) {
        D.off[k] = lay.off[1 + k];
        D.pitch[k] = lay.pitch[1 + k];
        D.w[k] = lay.w[1 + k];
        D.h[k] = lay.h[1 + k];
    }
    for (int k = 0; k < 3; ++k) D.sides[k] = pass_writes_sides(D.w[k], D.h[k]);
    const StreamSrc ss{src, src, n, (int64_t)w * h, w, w, h, 1};
    const int n_strips = (D.w[0] + ST_COLS / 2 - 1) / (ST_COLS / 2), n_bands = (D.h[0] + BAND - 1) / BAND;
    const int n_units = n_strips * n_bands * n;
    const int nblk = (n_units + 3) / 4;
    const dim3 grid(N_XCD * xcd_per(nblk));
    const int cu = prop.multiProcessorCount;
    for (int blocks : {cu * 8, cu * 32}) {
        const float us = timeit([&] { read_all<<<blocks, 256>>>((const uint4*)src, img.size() / 16, (uint32_t*)trash); }, reps);
        printf("read_all %5d blocks  %8.1f us  %6.2f TB/s\n", blocks, us, img.size() / us / 1e6);
    }
    auto run3 = [&](auto skip_c, const char* what) {
        constexpr int SK = decltype(skip_c)::value;
        printf("stream_kernel<3> %-28s %7.1f us\n", what, timeit([&] {
            hipLaunchKernelGGL((stream_kernel<3, SK>), grid, dim3(256), 0, 0, ss, dst, lay.bytes, D, n_strips, n_bands,
                               n_units, BAND, trash);
        }, reps));
    };
    run3(std::integral_constant<int, 0>{}, "all stores");
    run3(std::integral_constant<int, 6>{}, "level-1 stores only");
    run3(std::integral_constant<int, 5>{}, "level-2 stores only");
    run3(std::integral_constant<int, 3>{}, "level-3 stores only");
    run3(std::integral_constant<int, 7>{}, "no stores");
    printf("units %d (waves), %d per SIMD\n", n_units, n_units / (cu * 4));
    return 0;
}
