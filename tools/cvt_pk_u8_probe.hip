// Probe: does v_cvt_pk_u8_f32 equal cvRound + saturate_cast<uchar> (round half
// to even, clamp to [0, 255]) for every fp32 value in [-2, 258]?  Prints the
// number of mismatches and the first few.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdint>

__global__ void probe(uint32_t lo_bits, uint32_t n, unsigned long long* bad, uint32_t* first) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = __uint_as_float(lo_bits + i);
    const int r = (int)__builtin_rintf(v);
    const uint32_t want = (uint32_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
    const uint32_t got = __builtin_amdgcn_cvt_pk_u8_f32(v, 0, 0u) & 255u;
    if (got != want) {
        const unsigned long long k = atomicAdd(bad, 1ull);
        if (k < 8) first[k] = lo_bits + i;
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    hipMalloc(&bad, 8);
    hipMalloc(&first, 32);
    hipMemset(bad, 0, 8);
    // positive floats 0 .. 258 (bits 0 .. bits(258)), then negatives down to -2
    const float hi = 258.0f, neg = -2.0f;
    uint32_t hb, nb;
    memcpy(&hb, &hi, 4);
    memcpy(&nb, &neg, 4);
    probe<<<(hb + 255) / 256, 256>>>(0u, hb, bad, first);
    probe<<<((nb - 0x80000000u) + 255) / 256, 256>>>(0x80000000u, nb - 0x80000000u, bad, first);
    unsigned long long hbad;
    uint32_t f[8];
    hipMemcpy(&hbad, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
    printf("mismatches %llu of %u values\n", hbad, hb + (nb - 0x80000000u));
    for (unsigned k = 0; k < hbad && k < 8; ++k) {
        float x;
        memcpy(&x, &f[k], 4);
        printf("  %a (%.9g)\n", x, x);
    }
    return hbad ? 1 : 0;
}
