// api_factorset.cpp -- the two-phase factor evaluation of include/gvx.h
// (gvx_factor_set_*, gvx_factors_prepare, gvx_factor_read_*): the Ceres
// EvaluationCallback pattern of SURVEY.md 8b.  PrepareForEvaluation gathers
// the registered parameter blocks into one packed vector, uploads it, runs the
// reprojection and preintegration factor kernels over the whole window and
// copies residuals and Jacobians back into pinned host buffers owned by the set;
// every CostFunction::Evaluate reads its slice from those buffers.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "gvx_internal.h"

using namespace gvx;

struct gvx_factor_set {
    gvx_ctx* ctx = nullptr;
    // registered parameter blocks and their packed offsets
    std::vector<const double*> blocks;
    std::vector<int32_t> sizes, packed_off;
    int32_t n_params = 0, n_reproj = 0, n_preint = 0;
    // device: constants, packed offsets, parameter vector, results
    void* dev = nullptr;
    gvx_reproj_const* d_rc = nullptr;
    int32_t* d_roffs = nullptr;
    gvx_preint_result* d_pre = nullptr;
    double* d_pn = nullptr;
    int32_t* d_pn_off = nullptr;
    int32_t* d_poffs = nullptr;
    double* d_params = nullptr;
    double* d_out = nullptr;  // reproj res | reproj jac | preint res | preint jac
    // pinned host: gathered parameters and the results of the last prepare.
    // h_out is mapped into the device's address space (dh_out): the kernels
    // store the results straight into it over PCIe while they run, so a
    // prepare has no device-to-host copy to wait for (out_mode 1; 0 = a device
    // buffer and one D2H copy, the r04 form, kept for A/B: GVX_FACTORSET_D2H=1)
    double* h_params = nullptr;
    double* h_out = nullptr;
    double* dh_out = nullptr;
    int out_mode = 1;
    size_t out_doubles = 0;
    bool have_jac = false, prepared = false;
};

namespace {

constexpr int RP_RES = 2, RP_JAC = 46, PF_RES = 15, PF_JAC = 480;
const int RP_SIZES[5] = {7, 7, 7, 1, 1};
const int PF_SIZES[4] = {7, 9, 7, 9};

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

void destroy(gvx_factor_set* s) {
    if (!s) return;
    if (s->dev) hipFree(s->dev);
    if (s->h_params) hipHostFree(s->h_params);
    if (s->h_out) hipHostFree(s->h_out);
    delete s;
}

// copies rows x cols of a packed Jacobian block into a Ceres block
void put_block(const double* src, double* dst, int rows, int cols) {
    if (dst) std::memcpy(dst, src, sizeof(double) * rows * cols);
}

}  // namespace

extern "C" {

gvx_status gvx_factor_set_create(gvx_ctx* c, int32_t n_blocks, const double* const* blocks,
                                 const int32_t* block_sizes, int32_t n_reproj, const gvx_reproj_const* rc,
                                 const int32_t* r_blocks, int32_t n_preint, const gvx_preint_result* pre,
                                 const double* pn, int32_t n_pn, const int32_t* pn_off, const int32_t* p_blocks,
                                 gvx_factor_set** out) {
    if (!c || !out) return GVX_ERR_INVALID;
    *out = nullptr;
    if (n_blocks <= 0 || !blocks || !block_sizes || n_reproj < 0 || n_preint < 0)
        return set_err(c, GVX_ERR_INVALID, "bad factor set");
    if ((n_reproj > 0 && (!rc || !r_blocks)) || (n_preint > 0 && (!pre || !p_blocks)))
        return set_err(c, GVX_ERR_INVALID, "null factor arrays");
    auto* s = new gvx_factor_set;
    s->ctx = c;
    s->n_reproj = n_reproj;
    s->n_preint = n_preint;
    s->blocks.assign(blocks, blocks + n_blocks);
    s->sizes.assign(block_sizes, block_sizes + n_blocks);
    s->packed_off.resize(n_blocks);
    for (int b = 0; b < n_blocks; ++b) {
        if (!blocks[b] || block_sizes[b] <= 0) {
            destroy(s);
            return set_err(c, GVX_ERR_INVALID, "parameter block %d", b);
        }
        s->packed_off[b] = s->n_params;
        s->n_params += block_sizes[b];
    }
    // factor -> packed offsets, checking every block's size against the factor
    std::vector<int32_t> roffs(5 * (size_t)n_reproj), poffs(4 * (size_t)n_preint);
    for (int64_t i = 0; i < 5 * (int64_t)n_reproj; ++i) {
        const int b = r_blocks[i];
        if (b < 0 || b >= n_blocks || s->sizes[b] != RP_SIZES[i % 5]) {
            destroy(s);
            return set_err(c, GVX_ERR_INVALID, "reprojection factor %lld block %d", (long long)(i / 5), (int)(i % 5));
        }
        roffs[i] = s->packed_off[b];
    }
    bool any_earth = false;
    for (int i = 0; i < n_preint; ++i) {
        if (pre[i].variant != GVX_PREINT_NORMAL && pre[i].variant != GVX_PREINT_EARTH) {
            destroy(s);
            return set_err(c, GVX_ERR_UNSUPPORTED, "preintegration variant %d", pre[i].variant);
        }
        if (pre[i].variant == GVX_PREINT_EARTH) {
            any_earth = true;
            if (!pn || !pn_off || pn_off[i] < 0 || pn_off[i] + pre[i].m - 1 > n_pn) {
                destroy(s);
                return set_err(c, GVX_ERR_INVALID, "preintegration factor %d: pn list out of range", i);
            }
        }
        for (int k = 0; k < 4; ++k) {
            const int b = p_blocks[4 * i + k];
            if (b < 0 || b >= n_blocks || s->sizes[b] != PF_SIZES[k]) {
                destroy(s);
                return set_err(c, GVX_ERR_INVALID, "preintegration factor %d block %d", i, k);
            }
            poffs[4 * i + k] = s->packed_off[b];
        }
    }
    const size_t npn = any_earth ? (size_t)n_pn : 0;
    s->out_doubles = (size_t)n_reproj * (RP_RES + RP_JAC) + (size_t)n_preint * (PF_RES + PF_JAC);
    const size_t sz[8] = {sizeof(gvx_reproj_const) * n_reproj, sizeof(int32_t) * 5 * n_reproj,
                          sizeof(gvx_preint_result) * n_preint, sizeof(double) * 4 * (npn + 1),
                          sizeof(int32_t) * (n_preint + 1), sizeof(int32_t) * 4 * n_preint,
                          sizeof(double) * s->n_params, sizeof(double) * (s->out_doubles + 1)};
    size_t total = 0;
    for (size_t b : sz) total += align256(b);
    hipSetDevice(c->device);
    s->out_mode = c->factorset_d2h ? 0 : 1;
    if (hipMalloc(&s->dev, total) != hipSuccess || hipHostMalloc(&s->h_params, sizeof(double) * s->n_params) != hipSuccess ||
        hipHostMalloc(&s->h_out, sizeof(double) * (s->out_doubles + 1), hipHostMallocMapped) != hipSuccess ||
        hipHostGetDevicePointer((void**)&s->dh_out, s->h_out, 0) != hipSuccess) {
        destroy(s);
        return set_err(c, GVX_ERR_OOM, "factor set (%zu bytes)", total);
    }
    char* p = (char*)s->dev;
    void* ptr[8];
    for (int k = 0; k < 8; ++k) {
        ptr[k] = p;
        p += align256(sz[k]);
    }
    s->d_rc = (gvx_reproj_const*)ptr[0];
    s->d_roffs = (int32_t*)ptr[1];
    s->d_pre = (gvx_preint_result*)ptr[2];
    s->d_pn = (double*)ptr[3];
    s->d_pn_off = (int32_t*)ptr[4];
    s->d_poffs = (int32_t*)ptr[5];
    s->d_params = (double*)ptr[6];
    s->d_out = (double*)ptr[7];
    hipError_t e = hipSuccess;
    if (n_reproj > 0) {
        e = hipMemcpyAsync(s->d_rc, rc, sz[0], hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(s->d_roffs, roffs.data(), sz[1], hipMemcpyHostToDevice, c->stream);
    }
    if (e == hipSuccess && n_preint > 0) {
        e = hipMemcpyAsync(s->d_pre, pre, sz[2], hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess && any_earth) {
            e = hipMemcpyAsync(s->d_pn, pn, sizeof(double) * 4 * npn, hipMemcpyHostToDevice, c->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(s->d_pn_off, pn_off, sizeof(int32_t) * n_preint, hipMemcpyHostToDevice, c->stream);
        } else if (e == hipSuccess) {
            e = hipMemsetAsync(s->d_pn_off, 0, sizeof(int32_t) * n_preint, c->stream);
        }
        if (e == hipSuccess) e = hipMemcpyAsync(s->d_poffs, poffs.data(), sz[5], hipMemcpyHostToDevice, c->stream);
        // sqrt_information_ once per factor for the set's lifetime (the
        // reference recomputes it in every Evaluate; same bits)
        if (e == hipSuccess) e = launch_sqrt_info(c, n_preint, s->d_pre);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        destroy(s);
        return hip_err(c, e, "factor set upload");
    }
    *out = s;
    return GVX_OK;
}

void gvx_factor_set_destroy(gvx_factor_set* s) {
    if (s && s->ctx) hipStreamSynchronize(s->ctx->stream);
    destroy(s);
}

gvx_status gvx_factors_prepare(gvx_factor_set* s, int32_t with_jacobians) {
    if (!s) return GVX_ERR_INVALID;
    gvx_ctx* c = s->ctx;
    hipSetDevice(c->device);
    s->prepared = false;
    for (size_t b = 0; b < s->blocks.size(); ++b)
        std::memcpy(s->h_params + s->packed_off[b], s->blocks[b], sizeof(double) * s->sizes[b]);
    hipError_t e = hipMemcpyAsync(s->d_params, s->h_params, sizeof(double) * s->n_params, hipMemcpyHostToDevice,
                                  c->stream);
    if (e != hipSuccess) return hip_err(c, e, "factor parameters H2D");
    double* rres = s->out_mode == 1 ? s->dh_out : s->d_out;
    double* rjac = rres + (size_t)RP_RES * s->n_reproj;
    double* pres = rjac + (size_t)RP_JAC * s->n_reproj;
    double* pjac = pres + (size_t)PF_RES * s->n_preint;
    const bool jac = with_jacobians != 0;
    // both kinds in one call (gvx_factor_batch_eval_dev)
    gvx_status st = gvx_factor_batch_eval_dev(c, s->n_reproj, s->d_rc, s->d_roffs, rres, jac ? rjac : nullptr,
                                              s->n_preint, s->d_pre, s->d_pn, s->d_pn_off, s->d_poffs, pres,
                                              jac ? pjac : nullptr, s->d_params);
    if (st) return st;
    // one D2H of everything evaluated (the Jacobian regions only when computed),
    // unless the kernels wrote it to the mapped host buffer themselves
    if (s->out_mode == 1) {
        e = hipSuccess;
    } else if (jac) {
        e = hipMemcpyAsync(s->h_out, s->d_out, sizeof(double) * s->out_doubles, hipMemcpyDeviceToHost, c->stream);
    } else {
        e = hipMemcpyAsync(s->h_out, rres, sizeof(double) * RP_RES * s->n_reproj, hipMemcpyDeviceToHost, c->stream);
        const size_t po = (size_t)(RP_RES + RP_JAC) * s->n_reproj;
        if (e == hipSuccess && s->n_preint > 0)
            e = hipMemcpyAsync(s->h_out + po, pres, sizeof(double) * PF_RES * s->n_preint, hipMemcpyDeviceToHost,
                               c->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "factor results D2H");
    s->have_jac = jac;
    s->prepared = true;
    return GVX_OK;
}

gvx_status gvx_factor_read_reproj(const gvx_factor_set* s, int32_t i, double* residuals, double** jacobians) {
    if (!s || !s->prepared || i < 0 || i >= s->n_reproj || !residuals) return GVX_ERR_INVALID;
    const double* res = s->h_out + (size_t)RP_RES * i;
    std::memcpy(residuals, res, sizeof(double) * RP_RES);
    if (!jacobians) return GVX_OK;
    if (!s->have_jac) return GVX_ERR_INVALID;
    const double* J = s->h_out + (size_t)RP_RES * s->n_reproj + (size_t)RP_JAC * i;
    put_block(J, jacobians[0], 2, 7);
    put_block(J + 14, jacobians[1], 2, 7);
    put_block(J + 28, jacobians[2], 2, 7);
    put_block(J + 42, jacobians[3], 2, 1);
    put_block(J + 44, jacobians[4], 2, 1);
    return GVX_OK;
}

gvx_status gvx_factor_read_preint(const gvx_factor_set* s, int32_t i, double* residuals, double** jacobians) {
    if (!s || !s->prepared || i < 0 || i >= s->n_preint || !residuals) return GVX_ERR_INVALID;
    const double* base = s->h_out + (size_t)(RP_RES + RP_JAC) * s->n_reproj;
    std::memcpy(residuals, base + (size_t)PF_RES * i, sizeof(double) * PF_RES);
    if (!jacobians) return GVX_OK;
    if (!s->have_jac) return GVX_ERR_INVALID;
    const double* J = base + (size_t)PF_RES * s->n_preint + (size_t)PF_JAC * i;
    put_block(J, jacobians[0], 15, 7);
    put_block(J + 105, jacobians[1], 15, 9);
    put_block(J + 240, jacobians[2], 15, 7);
    put_block(J + 345, jacobians[3], 15, 9);
    return GVX_OK;
}

}  // extern "C"
