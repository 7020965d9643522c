// Instruction-cost probe (diagnostics, r05): shader cycles (s_memtime) per
// wave64 fp64 FMA issued back to back (8 independent accumulators) and in one
// dependent chain, per 64-bit DPP row_newbcast move and per v_fmac_f64_dpp,
// and the ds_read_b64 round trip, at 1..4 waves per SIMD (one workgroup).
#include <hip/hip_runtime.h>
#include <cstdio>
#define R8(x) x x x x x x x x
#define R16(x) R8(x) R8(x)
__global__ void probe(long long* out, double* sink, int mode) {
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    double b = 1.0000001, c = 0.5;
    __shared__ double lds[1024];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    long long t0 = __builtin_amdgcn_s_memtime();
    if (mode == 0) {  // 128 independent fp64 FMAs (8 chains)
        for (int i = 0; i < 16; ++i)
            asm volatile(R8("v_fma_f64 %0, %8, %9, %0\n v_fma_f64 %1, %8, %9, %1\n v_fma_f64 %2, %8, %9, %2\n v_fma_f64 %3, %8, %9, %3\n v_fma_f64 %4, %8, %9, %4\n v_fma_f64 %5, %8, %9, %5\n v_fma_f64 %6, %8, %9, %6\n v_fma_f64 %7, %8, %9, %7\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
    } else if (mode == 1) {  // 1024 dependent fp64 FMAs
        for (int i = 0; i < 16; ++i)
            asm volatile(R16(R8("v_fma_f64 %0, %1, %2, %0\n")) : "+v"(a0) : "v"(b), "v"(c));
    } else if (mode == 2) {  // 1024 v_mov_b64_dpp row_newbcast (independent)
        for (int i = 0; i < 16; ++i)
            asm volatile(R16(R8("v_mov_b64_dpp %0, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_mov_b64_dpp %1, %3 row_newbcast:5 row_mask:0xf bank_mask:0xf\n"))
                         : "=&v"(a0), "=&v"(a1) : "v"(b), "v"(c));
    } else if (mode == 3) {  // 1024 v_fmac_f64_dpp (8 accumulators)
        for (int i = 0; i < 16; ++i)
            asm volatile("s_nop 1\n" R16("v_fmac_f64_dpp %0, %8, %9 row_newbcast:1 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %1, %8, %9 row_newbcast:2 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %2, %8, %9 row_newbcast:3 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %3, %8, %9 row_newbcast:4 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %4, %8, %9 row_newbcast:5 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %5, %8, %9 row_newbcast:6 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %6, %8, %9 row_newbcast:7 row_mask:0xf bank_mask:0xf\n v_fmac_f64_dpp %7, %8, %9 row_newbcast:8 row_mask:0xf bank_mask:0xf\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
    } else if (mode == 4) {  // 256 dependent ds_read_b64 round trips
        unsigned addr = threadIdx.x * 8;
        for (int i = 0; i < 256; ++i) {
            double v;
            asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)\n v_cvt_u32_f64 %1, %0\n v_lshlrev_b32 %1, 3, %1" : "=&v"(v), "+v"(addr));
            a0 += v;
        }
    } else if (mode == 5) {  // 1024 independent v_mul_f64 (f64 mul, 8 chains)
        for (int i = 0; i < 16; ++i)
            asm volatile(R8("v_mul_f64 %0, %8, %0\n v_mul_f64 %1, %8, %1\n v_mul_f64 %2, %8, %2\n v_mul_f64 %3, %8, %3\n v_mul_f64 %4, %8, %4\n v_mul_f64 %5, %8, %5\n v_mul_f64 %6, %8, %6\n v_mul_f64 %7, %8, %7\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
int main() {
    long long* d;
    double* s;
    hipMalloc(&d, 16 * 16 * sizeof(long long));
    hipMalloc(&s, 16 * 1024 * sizeof(double));
    const char* names[] = {"fma_f64 indep x1024", "fma_f64 dep x1024", "mov_b64_dpp x2048", "fmac_f64_dpp x1024",
                           "ds_read_b64 roundtrip x256", "mul_f64 indep x1024"};
    for (int mode = 0; mode < 6; ++mode)
        for (int threads : {64, 256, 512, 1024}) {
            probe<<<1, threads>>>(d, s, mode);
            probe<<<1, threads>>>(d, s, mode);
            long long h[16];
            hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
            long long mx = 0;
            for (int w = 0; w < threads / 64; ++w) mx = h[w] > mx ? h[w] : mx;
            printf("%-28s waves/SIMD %.2f: %lld cycles (max over waves)\n", names[mode], threads / 256.0, mx);
        }
    return 0;
}
