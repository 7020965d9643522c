// api_aux.cpp -- C ABI of the remaining window factors (include/gvx.h):
// GnssFactor, ImuErrorFactor, ImuPosePriorFactor, ImuMixPriorFactor and
// MarginalizationFactor evaluation (kernels in aux_factors.hip).
#include <hip/hip_runtime.h>

#include <cstring>

#include "gvx_internal.h"

using namespace gvx;

namespace {

constexpr int MARG_MAX_R = 8192;  // dx staged in LDS (64 KB)

}  // namespace

gvx_status gvx_small_factor_eval_dev(gvx_ctx* c, int32_t kind, int32_t n, const double* d_consts,
                                     const double* d_params, const int32_t* d_offs, double* d_residuals,
                                     double* d_jacobians) {
    if (!c) return GVX_ERR_INVALID;
    int P = 0, NC = 0;
    if (small_factor_dims(kind, &P, &NC) == 0) return set_err(c, GVX_ERR_INVALID, "unknown factor kind %d", kind);
    if (n < 0) return set_err(c, GVX_ERR_INVALID, "n < 0");
    if (n == 0) return GVX_OK;
    if ((NC && !d_consts) || !d_params || !d_offs || !d_residuals)
        return set_err(c, GVX_ERR_INVALID, "null device pointer");
    hipSetDevice(c->device);
    hipError_t e = launch_small_factor(c, kind, n, d_consts, d_params, d_offs, d_residuals, d_jacobians);  // timed
    return hip_err(c, e, "small factor kernel");
}

gvx_status gvx_small_factor_eval(gvx_ctx* c, int32_t kind, int32_t n, const double* consts, const double* params,
                                 int32_t n_params, const int32_t* offs, double* residuals, double* jacobians) {
    if (!c) return GVX_ERR_INVALID;
    int P = 0, NC = 0;
    const int R = small_factor_dims(kind, &P, &NC);
    if (R == 0) return set_err(c, GVX_ERR_INVALID, "unknown factor kind %d", kind);
    if (n < 0 || n_params < 0) return set_err(c, GVX_ERR_INVALID, "negative size");
    if (n == 0) return GVX_OK;
    if ((NC && !consts) || !params || !offs || !residuals) return set_err(c, GVX_ERR_INVALID, "null pointer");
    for (int i = 0; i < n; ++i)
        if (offs[i] < 0 || offs[i] + P > n_params)
            return set_err(c, GVX_ERR_INVALID, "factor %d: parameter block [%d, %d) outside %d values", i, offs[i],
                           offs[i] + P, n_params);
    hipSetDevice(c->device);
    const size_t nc = (size_t)n * NC, nr = (size_t)n * R, nj = jacobians ? (size_t)n * R * P : 0;
    // pinned arena laid out like the device one: one upload, one download
    double *d_c, *h_c, *d_p, *h_p, *d_r, *h_r, *d_j, *h_j;
    int32_t *d_o, *h_o;
    Staging st;
    st.add(nc, &d_c, &h_c);
    st.add((size_t)n_params, &d_p, &h_p);
    st.add((size_t)n, &d_o, &h_o);
    st.add(nr, &d_r, &h_r);
    st.add(nj, &d_j, &h_j);
    void* db = scratch(c, "aux_factor", st.bytes());
    void* hb = pinned(c, "aux_factor", st.bytes());
    if (!db || !hb) return set_err(c, GVX_ERR_OOM, "factor staging");
    st.bind(db, hb);
    if (nc) std::memcpy(h_c, consts, sizeof(double) * nc);
    std::memcpy(h_p, params, sizeof(double) * n_params);
    std::memcpy(h_o, offs, sizeof(int32_t) * n);
    hipError_t e = hipMemcpyAsync(d_c, h_c, (size_t)((char*)d_r - (char*)d_c), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "factor upload");
    gvx_status s = gvx_small_factor_eval_dev(c, kind, n, d_c, d_p, d_o, d_r, nj ? d_j : nullptr);
    if (s) return s;
    const size_t out = (size_t)((char*)d_j - (char*)d_r) + sizeof(double) * nj;
    e = hipMemcpyAsync(h_r, d_r, out, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "factor download");
    std::memcpy(residuals, h_r, sizeof(double) * nr);
    if (nj) std::memcpy(jacobians, h_j, sizeof(double) * nj);
    return GVX_OK;
}

gvx_status gvx_marg_factor_eval(gvx_ctx* c, int32_t r, int32_t nb, const int32_t* size, const int32_t* index,
                                const int32_t* xoff, int32_t n_x, const double* x0, const double* params,
                                const double* J0, const double* e0, double* residuals, double* jacobians) {
    if (!c) return GVX_ERR_INVALID;
    if (r < 0 || nb < 0 || n_x < 0) return set_err(c, GVX_ERR_INVALID, "negative size");
    if (r > MARG_MAX_R) return set_err(c, GVX_ERR_UNSUPPORTED, "remained size %d > %d", r, MARG_MAX_R);
    if (r == 0) return GVX_OK;
    if (!size || !index || !xoff || !x0 || !params || !J0 || !e0 || !residuals)
        return set_err(c, GVX_ERR_INVALID, "null pointer");
    // every block inside dx and inside the parameter vectors (the kernel trusts them)
    int64_t jac_total = 0;
    for (int b = 0; b < nb; ++b) {
        const int local = size[b] == 7 ? 6 : size[b];
        if (size[b] <= 0 || index[b] < 0 || index[b] + local > r || xoff[b] < 0 || xoff[b] + size[b] > n_x)
            return set_err(c, GVX_ERR_INVALID, "remained block %d out of range", b);
        jac_total = std::max<int64_t>(jac_total, (int64_t)r * (xoff[b] + size[b]));
    }
    hipSetDevice(c->device);
    const size_t nj = jacobians ? (size_t)jac_total : 0;
    // one pinned staging arena laid out like the device one: the inputs are its
    // prefix (one upload), the outputs its suffix (one download)
    int32_t *d_blk, *h_blk;
    double *d_x0, *h_x0, *d_x, *h_x, *d_J, *h_J, *d_e, *h_e, *d_r, *h_r, *d_j, *h_j;
    Staging st;
    st.add(3 * (size_t)nb, &d_blk, &h_blk);
    st.add((size_t)n_x, &d_x0, &h_x0);
    st.add((size_t)n_x, &d_x, &h_x);
    st.add((size_t)r * r, &d_J, &h_J);
    st.add((size_t)r, &d_e, &h_e);
    st.add((size_t)r, &d_r, &h_r);
    st.add(nj, &d_j, &h_j);
    void* db = scratch(c, "marg_factor", st.bytes());
    void* hb = pinned(c, "marg_factor", st.bytes());
    if (!db || !hb) return set_err(c, GVX_ERR_OOM, "marginalisation staging");
    st.bind(db, hb);
    if (nb) {
        std::memcpy(h_blk, size, sizeof(int32_t) * nb);
        std::memcpy(h_blk + nb, index, sizeof(int32_t) * nb);
        std::memcpy(h_blk + 2 * nb, xoff, sizeof(int32_t) * nb);
    }
    if (n_x) {
        std::memcpy(h_x0, x0, sizeof(double) * n_x);
        std::memcpy(h_x, params, sizeof(double) * n_x);
    }
    std::memcpy(h_J, J0, sizeof(double) * r * r);
    std::memcpy(h_e, e0, sizeof(double) * r);
    hipError_t e = hipMemcpyAsync(d_blk, h_blk, (size_t)((char*)d_r - (char*)d_blk), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "marginalisation upload");
    hipEvent_t ev{};
    prof_begin(c, "marg_factor", &ev);
    e = launch_marg_factor(c, r, nb, d_blk, d_x0, d_x, d_J, d_e, d_r, nj ? d_j : nullptr);
    prof_end(c, "marg_factor", ev);
    if (e != hipSuccess) return hip_err(c, e, "marginalisation kernel");
    const size_t out = (size_t)((char*)d_j - (char*)d_r) + sizeof(double) * (nj ? nj : 0);
    e = hipMemcpyAsync(h_r, d_r, out, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "marginalisation download");
    std::memcpy(residuals, h_r, sizeof(double) * r);
    if (nj) std::memcpy(jacobians, h_j, sizeof(double) * nj);
    return GVX_OK;
}
