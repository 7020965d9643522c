// Layout probe of v_mfma_f64_16x16x4f64 (diagnostics): A(i,k) = i + 100 k,
// B(k,j) = (k == 0 && j == 0) ? 1 : 0 etc.; prints which (row, col) each
// lane's four accumulator doubles hold.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
__global__ void probe(double* out, int mode) {
    const int l = threadIdx.x, lr = l & 15, lk = l >> 4;
    // mode 0: A(i,k) = 1 if k == 0 (else 0), B(k,j) = j + 1000*k -> D(i,j) = j  (col id)
    // mode 1: A(i,k) = i + 1 if k == 0, B(k,j) = 1 if k == 0 -> D(i,j) = i + 1 (row id)
    double a, b;
    if (mode == 0) { a = lk == 0 ? 1.0 : 0.0; b = lk == 0 ? (double)lr : 0.0; }
    else { a = lk == 0 ? (double)(lr + 1) : 0.0; b = lk == 0 ? 1.0 : 0.0; }
    v4d acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    for (int i = 0; i < 4; ++i) out[l * 4 + i] = acc[i];
}
int main() {
    double* d;
    hipMalloc(&d, 64 * 4 * sizeof(double));
    double h[256];
    for (int mode = 0; mode < 2; ++mode) {
        probe<<<1, 64>>>(d, mode);
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        printf("mode %d (%s):\n", mode, mode ? "row+1" : "col");
        for (int l = 0; l < 64; l += 1) printf("l%02d: %g %g %g %g%s", l, h[4*l], h[4*l+1], h[4*l+2], h[4*l+3], (l % 4 == 3) ? "\n" : " | ");
    }
    return 0;
}
