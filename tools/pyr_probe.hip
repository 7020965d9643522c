// pyr_probe.hip -- what bounds the pyramid pass (r06 probe, not product code).
// Times, on the configs[1] batch (512 frames of 1280x560 u8):
//  * stream_kernel<3, SKIP> itself (SKIP 0: the product; 7: every level store
//    folded into a register), included from csrc/pyramid.hip;
//  * load-only walks of the same (strip, band) units: each wave streams its
//    band's source rows with PF row pairs in flight, in three load shapes:
//      mode 0  16 B per lane at an 8-B lane stride (the pass's own shape: a wave
//              instruction covers 520 distinct bytes),
//      mode 1  8 B per lane at an 8-B stride, the left 8 B from lane L-1 by DPP
//              (the same bytes per wave in half the registers),
//      mode 2  16 B per lane at a 16-B stride (1 KiB distinct per instruction).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I ic-gvins_amd/csrc \
//          tools/pyr_probe.hip -L ic-gvins_amd/gvx -lgvx -Wl,-rpath,$PWD/ic-gvins_amd/gvx -o tools/pyr_probe
#ifndef PYR_SRC
#define PYR_SRC "../ic-gvins_amd/csrc/pyramid.hip"
#endif
#include PYR_SRC

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace gvx;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef uint32_t p4u __attribute__((ext_vector_type(4)));
typedef uint32_t p2u __attribute__((ext_vector_type(2)));

template <int MODE, int PF, int OCC>
__global__ void __launch_bounds__(64, OCC) load_walk(const uint8_t* __restrict__ src, int64_t img_stride, int pitch,
                                                     int w, int h, int n_strips, int n_bands, int band_rows,
                                                     int warm, int n_units, uint32_t* __restrict__ out) {
    const int unit = xcd_swizzle(blockIdx.x, n_units);
    if (unit >= n_units) return;
    const int lane = threadIdx.x;
    const int st = unit % n_strips, rest = unit / n_strips, bd = rest % n_bands, img = rest / n_bands;
    const int scols = MODE == 2 ? 960 : 480;
    int x = scols * st + (MODE == 2 ? 16 : 8) * lane - 20;
    x = min(max(x, 0), w - 16);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src + img * img_stride), (short)0, 0x7fffffff, 0x00020000);
    const int y0 = band_rows * bd - warm, n = band_rows + warm, ylast = min(y0 + n - 1, h - 1);
    auto row = [&](int y) { return min(max(y, 0), ylast) * pitch; };
    constexpr int RS = 16;
    p4u ring[RS];
    auto ld = [&](int y) -> p4u {
        if constexpr (MODE == 1) {
            const p2u v = __builtin_amdgcn_raw_buffer_load_b64(rs, x + 8, row(y), 0);
            return p4u{v.x, v.y, 0u, 0u};
        } else {
            return __builtin_amdgcn_raw_buffer_load_b128(rs, x, row(y), 0);
        }
    };
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 2 * PF; ++k) ring[k] = ld(y0 + k);
    for (int k = 0; k < n; k += RS) {
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            p4u v = ring[s];
            if constexpr (MODE == 1) {
                v.z = v.x;
                v.w = v.y;
                v.x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.z, 0x138, 0xf, 0xf, false);
                v.y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v.w, 0x138, 0xf, 0xf, false);
            }
            acc += __builtin_amdgcn_udot4(v.x ^ v.z, 0x01010101u, v.y ^ v.w, false);
            ring[(s + 2 * PF) % RS] = ld(y0 + k + s + 2 * PF);
        }
    }
    out[unit * 64 + lane] = acc;
}

// store-only walks of the pass's output pattern, one wave per (strip, band):
// level-1 rows as one dword per lane (lanes 2..61), level-2 rows every second
// row as a u16, level-3 rows every fourth as a byte.  ALIGN 0: the pass's own
// column offsets (PAD + 240 st: strips share cache lines); 1: each strip's row
// segment inside its own 256 / 128 / 64-byte span (no line shared by two waves).
// LEVELS: 1 = level 1 only, 3 = all three.  NT: nontemporal stores.
template <int ALIGN, int LEVELS, int NT>
__global__ void __launch_bounds__(64, 4) store_walk(uint8_t* __restrict__ pyr, int64_t pyr_bytes, DownLevels L,
                                                    int n_strips, int n_bands, int band, int n_units) {
    const int unit = xcd_swizzle(blockIdx.x, n_units);
    if (unit >= n_units) return;
    const int lane = threadIdx.x;
    const int st = unit % n_strips, rest = unit / n_strips, bd = rest % n_bands, img = rest / n_bands;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(pyr + img * pyr_bytes, (short)0, (int)pyr_bytes, 0x00020000);
    const bool own = lane >= 2 && lane < 62;
    const int c1 = 240 * st + 4 * (lane - 2), c2 = 120 * st + 2 * (lane - 2), c3 = 60 * st + (lane - 2);
    // ALIGN: the row's start rounded down to the span, strip st at span * st
    // (ALIGN rows are 3 spans long, in the unused level-0 slot of the layout)
    const auto at = [&](int lev, int r, int span, int c, int cst) {
        return ALIGN ? 300000 * lev + (r + PAD) * 3 * span + span * st + (c - cst)
                     : (int)L.off[lev] + (r + PAD) * L.pitch[lev] + PAD + c;
    };
    uint32_t v = lane * 0x01010101u;
    constexpr int AUX = NT ? 2 : 0;  // slc
    for (int k = 0; k < band; ++k) {
        const int r1 = band * bd + k;
        if (r1 >= L.h[0]) break;
        const int o1 = own && c1 < L.w[0] ? at(0, r1, 256, c1, 240 * st) : PYR_OOB;
        __builtin_amdgcn_raw_buffer_store_b32(v + k, rs, o1, 0, AUX);
        if (LEVELS > 1 && (k & 1) == 0) {
            const int r2 = r1 >> 1;
            const int o2 = own && c2 < L.w[1] ? at(1, r2, 128, c2, 120 * st) : PYR_OOB;
            __builtin_amdgcn_raw_buffer_store_b16((unsigned short)(v + k), rs, o2, 0, AUX);
            if ((k & 3) == 0) {
                const int r3 = r2 >> 1;
                const int o3 = own && c3 < L.w[2] ? at(2, r3, 64, c3, 60 * st) : PYR_OOB;
                __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(v + k), rs, o3, 0, AUX);
            }
        }
    }
}

// the load walk (mode 0, PF 4) with the pass's stores in it: per level-1 row one
// dword per lane, every second row a u16, every fourth a byte.  SM 0: stores
// after the row's loads (the pass's order); 1: stores before them; 2: no level-2 /
// level-3 stores; 3: every store a dword (level 2 / 3 rows as dwords of a wider
// span); 4: stores only every 4th row, 4 rows at once (4 level-1 dwords).
template <int SM>
__global__ void __launch_bounds__(64, 4) mix_walk(const uint8_t* __restrict__ src, int64_t img_stride, int pitch, int w,
                                                  int h, int n_strips, int n_bands, int band, int n_units,
                                                  uint8_t* __restrict__ pyr, int64_t pyr_bytes, DownLevels L) {
    const int unit = xcd_swizzle(blockIdx.x, n_units);
    if (unit >= n_units) return;
    const int lane = threadIdx.x;
    const int st = unit % n_strips, rest = unit / n_strips, bd = rest % n_bands, img = rest / n_bands;
    int x = 480 * st + 8 * lane - 20;
    x = min(max(x, 0), w - 16);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src + img * img_stride), (short)0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t ds =
        __builtin_amdgcn_make_buffer_rsrc(pyr + img * pyr_bytes, (short)0, (int)pyr_bytes, 0x00020000);
    const bool own = lane >= 2 && lane < 62;
    const int c1 = 240 * st + 4 * (lane - 2), c2 = 120 * st + 2 * (lane - 2), c3 = 60 * st + (lane - 2);
    const int y0 = 2 * band * bd - 18, ylast = min(2 * band * bd + 2 * band - 1, h - 1);
    const int n1 = band + 9;
    auto row = [&](int y) { return min(max(y, 0), ylast) * pitch; };
    constexpr int PF = 4, RS = 8;
    p4u ra[RS], rb[RS];
    auto ld = [&](int k, p4u& a, p4u& b) {
        a = __builtin_amdgcn_raw_buffer_load_b128(rs, x, row(y0 + 2 * k), 0);
        b = __builtin_amdgcn_raw_buffer_load_b128(rs, x, row(y0 + 2 * k + 1), 0);
    };
    uint32_t acc = lane;
    auto stores = [&](int k) {
        const int r1 = band * bd + k - 9;
        if (r1 < band * bd || r1 >= min(band * bd + band, L.h[0])) return;
        if constexpr (SM == 4) {
            if ((k & 3) != 3) return;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int o1 = own && c1 < L.w[0] ? (int)L.off[0] + (r1 - 3 + q + PAD) * L.pitch[0] + PAD + c1 : PYR_OOB;
                __builtin_amdgcn_raw_buffer_store_b32(acc + q, ds, o1, 0, 0);
            }
            return;
        }
        const int o1 = own && c1 < L.w[0] ? (int)L.off[0] + (r1 + PAD) * L.pitch[0] + PAD + c1 : PYR_OOB;
        __builtin_amdgcn_raw_buffer_store_b32(acc, ds, o1, 0, 0);
        if (SM != 2 && (k & 1) == 0) {
            const int r2 = r1 >> 1;
            const int o2 = own && c2 < L.w[1] ? (int)L.off[1] + (r2 + PAD) * L.pitch[1] + PAD + c2 : PYR_OOB;
            if (SM == 3)
                __builtin_amdgcn_raw_buffer_store_b32(acc, ds, o2 & ~3, 0, 0);
            else
                __builtin_amdgcn_raw_buffer_store_b16((unsigned short)acc, ds, o2, 0, 0);
            if ((k & 3) == 0) {
                const int r3 = r2 >> 1;
                const int o3 = own && c3 < L.w[2] ? (int)L.off[2] + (r3 + PAD) * L.pitch[2] + PAD + c3 : PYR_OOB;
                if (SM == 3)
                    __builtin_amdgcn_raw_buffer_store_b32(acc, ds, o3 & ~3, 0, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b8((unsigned char)acc, ds, o3, 0, 0);
            }
        }
    };
#pragma unroll
    for (int k = 0; k < PF; ++k) ld(k, ra[k], rb[k]);
    for (int k = 0; k < n1; k += RS) {
#pragma unroll
        for (int s = 0; s < RS; ++s) {
            if (SM == 1) stores(k + s);
            const p4u a = ra[s], b = rb[s];
            ld(k + s + PF, ra[(s + PF) % RS], rb[(s + PF) % RS]);
            acc += __builtin_amdgcn_udot4(a.x ^ b.z, 0x01010101u, a.y ^ b.w, false) ^ (a.z + b.x) ^ (a.w + b.y);
            if (SM != 1) stores(k + s);
        }
    }
}

struct Timer {
    hipEvent_t a, b;
    Timer() {
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
    }
};

template <typename F>
static float time_it(F f, int reps) {
    Timer t;
    for (int i = 0; i < 3; ++i) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(t.a, 0));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(t.b, 0));
    CK(hipEventSynchronize(t.b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, t.a, t.b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int W = 1280, H = 560, NIMG = 512, REPS = argc > 1 ? atoi(argv[1]) : 40;
    const int64_t img_bytes = (int64_t)W * H;
    uint8_t* src;
    CK(hipMalloc(&src, img_bytes * NIMG));
    {
        std::vector<uint8_t> hbuf(img_bytes * NIMG);
        uint32_t s = 12345;
        for (auto& v : hbuf) {
            s = s * 1664525u + 1013904223u;
            v = (uint8_t)(s >> 24);
        }
        CK(hipMemcpy(src, hbuf.data(), hbuf.size(), hipMemcpyHostToDevice));
    }
    const PyrLayout lay = make_layout(W, H, 3, 21);
    uint8_t* pyr;
    CK(hipMalloc(&pyr, lay.bytes * NIMG));
    DownLevels D{};
    for (int k = 0; k < 3; ++k) {
        D.off[k] = lay.off[1 + k];
        D.pitch[k] = lay.pitch[1 + k];
        D.w[k] = lay.w[1 + k];
        D.h[k] = lay.h[1 + k];
    }
    const int n_strips = (D.w[0] + ST_COLS / 2 - 1) / (ST_COLS / 2);
    const int band = stream_band(n_strips, D.h[0], NIMG, 256);
    const int n_bands = (D.h[0] + band - 1) / band;
    const int n_units = n_strips * n_bands * NIMG;
    uint8_t* trash;
    CK(hipMalloc(&trash, (size_t)n_units * 256));
    uint32_t* out;
    CK(hipMalloc(&out, (size_t)n_units * 2 * 64 * 4));
    StreamSrc s{};
    s.a = src;
    s.b = nullptr;
    s.n_a = NIMG;
    s.img_stride = img_bytes;
    s.pitch = W;
    s.w = W;
    s.h = H;
    s.raw = 1;
    const double src_gb = (double)img_bytes * NIMG / 1e9;
    printf("layout bytes %lld  strips %d bands %d band %d units %d\n", (long long)lay.bytes, n_strips, n_bands, band,
           n_units);
    const dim3 g1(N_XCD * xcd_per(n_units));
    auto pass = [&](auto kern) {
        return time_it([&] { hipLaunchKernelGGL(kern, g1, dim3(64), 0, 0, s, pyr, lay.bytes, D, n_strips, n_bands,
                                                n_units, band, trash, 0); },
                       REPS);
    };
    const bool full = argc <= 2;
    if (argc > 2 && argv[2][0] == 'b') {
        // band sweep of the product kernel: band heights (level-1 rows per wave)
        for (int round = 0; round < 2; ++round)
            for (int bh : {40, 56, 72, 96, 140, 280}) {
                const int nb = (D.h[0] + bh - 1) / bh;
                const int b = std::min(bh, ((D.h[0] + nb - 1) / nb + 3) / 4 * 4);
                const int nu = n_strips * nb * NIMG;
                const float t = time_it([&] { hipLaunchKernelGGL((stream_kernel<3, 0, 1>), dim3(N_XCD * xcd_per(nu)),
                                                                 dim3(64), 0, 0, s, pyr, lay.bytes, D, n_strips, nb, nu,
                                                                 b, trash, 0); },
                                        REPS);
                printf("band %3d (%d bands, %5d waves) %.4f ms\n", b, nb, nu, t);
            }
        return 0;
    }
    for (int round = 0; round < 2; ++round) {
        const float t0 = pass(stream_kernel<3, 0, 1>);
        const float t7 = pass(stream_kernel<3, 7, 1>);
        const float t6 = pass(stream_kernel<3, 6, 1>);
        printf("stream_kernel       %.4f ms  (src %.2f TB/s)\n", t0, src_gb / t0);
        printf("stream_kernel skip7 %.4f ms  (no level stores)\n", t7);
        printf("stream_kernel skip6 %.4f ms  (level-1 stores only)\n", t6);
        auto mw = [&](auto kern, const char* name) {
            const float t = time_it([&] { hipLaunchKernelGGL(kern, g1, dim3(64), 0, 0, src, img_bytes, W, W, H,
                                                             n_strips, n_bands, band, n_units, pyr, lay.bytes, D); },
                                    REPS);
            printf("%-28s %.4f ms\n", name, t);
        };
        mw(mix_walk<0>, "mix: stores after loads");
        mw(mix_walk<1>, "mix: stores before loads");
        mw(mix_walk<2>, "mix: level-1 stores only");
        mw(mix_walk<3>, "mix: all stores dwords");
        mw(mix_walk<4>, "mix: L1 stores x4 bursts");
        if (!full) continue;
        // load-only walks: 2*band source rows owned + 18 warm-up rows per unit
        auto walk = [&](auto kern, int strips, const char* name) {
            const int nu = strips * n_bands * NIMG;
            const float t = time_it([&] { hipLaunchKernelGGL(kern, dim3(N_XCD * xcd_per(nu)), dim3(64), 0, 0, src,
                                                             img_bytes, W, W, H, strips, n_bands, 2 * band, 18, nu,
                                                             out); },
                                    REPS);
            printf("%-28s %.4f ms  (src %.2f TB/s)\n", name, t, src_gb / t);
        };
        walk(load_walk<0, 4, 4>, n_strips, "load b128/8B  PF4 occ4");
        walk(load_walk<0, 2, 8>, n_strips, "load b128/8B  PF2 occ8");
        walk(load_walk<0, 6, 4>, n_strips, "load b128/8B  PF6 occ4");
        walk(load_walk<1, 4, 4>, n_strips, "load b64+dpp  PF4 occ4");
        walk(load_walk<1, 8, 4>, n_strips, "load b64+dpp  PF8 occ4");
        walk(load_walk<1, 4, 8>, n_strips, "load b64+dpp  PF4 occ8");
        walk(load_walk<2, 4, 4>, 2, "load b128/16B PF4 occ4 (2 strips)");
        walk(load_walk<2, 2, 8>, 2, "load b128/16B PF2 occ8 (2 strips)");
        auto sw = [&](auto kern, const char* name) {
            const float t = time_it([&] { hipLaunchKernelGGL(kern, g1, dim3(64), 0, 0, pyr, lay.bytes, D, n_strips,
                                                             n_bands, band, n_units); },
                                    REPS);
            printf("%-28s %.4f ms\n", name, t);
        };
        sw(store_walk<0, 1, 0>, "store L1 shared lines");
        sw(store_walk<1, 1, 0>, "store L1 aligned strips");
        sw(store_walk<0, 3, 0>, "store L1-3 shared lines");
        sw(store_walk<1, 3, 0>, "store L1-3 aligned strips");
        sw(store_walk<0, 3, 1>, "store L1-3 shared, slc");
    }
    CK(hipDeviceSynchronize());
    return 0;
}
