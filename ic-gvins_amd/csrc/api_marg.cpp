// api_marg.cpp -- C ABI of the device marginalisation (include/gvx.h):
// MarginalizationInfo::constructEquation / schurElimination / linearization
// (factors/marginalization_info.h:153-230) and the SelfAdjointEigenSolver they
// use (kernels in marg.hip).
//
// The host turns the residual blocks' structure into per-block-pair contribution
// lists (factor order, so every H0 entry is summed in the reference's order);
// the numbers themselves never leave the device in the _dev variant.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "gvx_internal.h"

using namespace gvx;

namespace {

constexpr int DENSE_PAIR_TABLE_MAX = 2048;  // block counts above this use a hash map

int local_size(int s) { return s == 7 ? 6 : s; }

struct Lists {
    std::vector<MargPairRec> recs;  // H0 pairs, then b0 blocks
    std::vector<int4> contrib;
    int n_pairs = 0, n_bvec = 0;
    // contribution chunks of at most H0_CHUNK (chunked H0 build, MargLaunch)
    std::vector<int4> chunks;
    std::vector<int2> recpart;
    int64_t n_part = 0;
};
constexpr int H0_CHUNK = 32;

void make_chunks(Lists& ls) {
    ls.chunks.clear();
    ls.recpart.resize(ls.recs.size());
    int64_t part = 0;
    for (size_t k = 0; k < ls.recs.size(); ++k) {
        const MargPairRec& r = ls.recs[k];
        const int n_ent = r.lp * r.lq;
        int nch = 0;
        int c0 = r.c0;
        do {  // at least one chunk per record (an empty one sums to 0)
            ls.chunks.push_back(make_int4((int)k, c0, std::min(c0 + H0_CHUNK, r.c1), (int)(part + (int64_t)nch * n_ent)));
            ++nch;
            c0 += H0_CHUNK;
        } while (c0 < r.c1);
        ls.recpart[k] = make_int2((int)part, nch);
        part += (int64_t)nch * n_ent;
    }
    ls.n_part = part;
}

// Validates the problem and builds the contribution lists.  Returns GVX_OK or
// an error with the message set.
// m_max: the largest eliminated set the caller's solver takes (the dense
// eigen / Cholesky kernels: GVX_EIG_MAX_N; the LM step with a diagonal Hee: any)
gvx_status build_lists(gvx_ctx* c, int n_fac, const int32_t* nres, const int32_t* blk_off, const int32_t* blk,
                       const int64_t* res_off, const int64_t* jac_off, int64_t n_data, int nb, const int32_t* size,
                       const int32_t* index, int m, int L, Lists& out, int m_max = GVX_EIG_MAX_N) {
    if (n_fac < 0 || nb < 0 || n_data < 0) return set_err(c, GVX_ERR_INVALID, "negative size");
    if (m <= 0) return set_err(c, GVX_ERR_INVALID, "nothing to marginalize (m = %d)", m);
    if (L < m) return set_err(c, GVX_ERR_INVALID, "local size %d < marginalized size %d", L, m);
    if (m > m_max || L - m > GVX_EIG_MAX_N)
        return set_err(c, GVX_ERR_UNSUPPORTED, "marginalized %d / remained %d above %d / %d", m, L - m, m_max,
                       GVX_EIG_MAX_N);
    if (n_fac && (!nres || !blk_off || !blk || !res_off || !jac_off)) return set_err(c, GVX_ERR_INVALID, "null pointer");
    if (nb && (!size || !index)) return set_err(c, GVX_ERR_INVALID, "null block table");
    for (int b = 0; b < nb; ++b)
        if (size[b] <= 0 || size[b] > 255 || index[b] < 0 || index[b] + local_size(size[b]) > L)
            return set_err(c, GVX_ERR_INVALID, "block %d: size %d at local index %d outside %d", b, size[b], index[b], L);
    if (n_fac && blk_off[0] != 0) return set_err(c, GVX_ERR_INVALID, "blk_off[0] != 0");
    // pair table: block pair -> record id
    const bool dense = nb <= DENSE_PAIR_TABLE_MAX;
    std::vector<int32_t> table(dense ? (size_t)nb * nb : 0, -1);
    std::unordered_map<int64_t, int32_t> hmap;
    std::vector<int32_t> bvec(nb, -1);
    std::vector<int32_t> cnt;          // contributions per record
    std::vector<MargPairRec> recs;
    auto rec_of = [&](int p, int q) -> int32_t& {
        if (dense) return table[(size_t)p * nb + q];
        auto it = hmap.find((int64_t)p * nb + q);
        if (it == hmap.end()) it = hmap.emplace((int64_t)p * nb + q, -1).first;
        return it->second;
    };
    // pass 1: records and counts
    for (int f = 0; f < n_fac; ++f) {
        const int R = nres[f], b0 = blk_off[f], b1 = blk_off[f + 1];
        if (R <= 0 || R > 32767 || b1 < b0) return set_err(c, GVX_ERR_INVALID, "factor %d: bad residual/block count", f);
        int64_t jt = 0;
        for (int i = b0; i < b1; ++i) {
            if (blk[i] < 0 || blk[i] >= nb) return set_err(c, GVX_ERR_INVALID, "factor %d: block id %d", f, blk[i]);
            jt += (int64_t)R * size[blk[i]];
        }
        if (res_off[f] < 0 || res_off[f] + R > n_data || res_off[f] + R > INT32_MAX || jac_off[f] < 0 || jac_off[f] + jt > n_data ||
            jac_off[f] + jt > INT32_MAX)
            return set_err(c, GVX_ERR_INVALID, "factor %d: data range outside %lld values", f, (long long)n_data);
        for (int i = b0; i < b1; ++i)
            for (int j = i; j < b1; ++j) {
                int p = blk[i], q = blk[j];
                if (i != j && p == q) return set_err(c, GVX_ERR_INVALID, "factor %d: block %d twice", f, p);
                if (index[p] < index[q]) std::swap(p, q);  // row block P: the larger local index
                int32_t& id = rec_of(p, q);
                if (id < 0) {
                    id = (int32_t)recs.size();
                    recs.push_back({index[p], index[q], local_size(size[p]), local_size(size[q]), 0, 0});
                    cnt.push_back(0);
                }
                cnt[id]++;
            }
    }
    out.n_pairs = (int)recs.size();
    for (int f = 0; f < n_fac; ++f)
        for (int i = blk_off[f]; i < blk_off[f + 1]; ++i) {
            const int p = blk[i];
            if (bvec[p] < 0) {
                bvec[p] = (int32_t)recs.size();
                recs.push_back({index[p], -1, local_size(size[p]), 1, 0, 0});
                cnt.push_back(0);
            }
            cnt[bvec[p]]++;
        }
    out.n_bvec = (int)recs.size() - out.n_pairs;
    int64_t total = 0;
    for (size_t k = 0; k < recs.size(); ++k) {
        recs[k].c0 = (int32_t)total;
        total += cnt[k];
        recs[k].c1 = recs[k].c0;
    }
    if (total > INT32_MAX) return set_err(c, GVX_ERR_UNSUPPORTED, "too many contributions");
    out.contrib.resize((size_t)total);
    // pass 2: fill in factor order
    int64_t joff[256];
    for (int f = 0; f < n_fac; ++f) {
        const int R = nres[f], b0 = blk_off[f], nbf = blk_off[f + 1] - b0;
        if (nbf > 256) return set_err(c, GVX_ERR_UNSUPPORTED, "factor %d: %d blocks", f, nbf);
        int64_t o = jac_off[f];
        for (int i = 0; i < nbf; ++i) {
            joff[i] = o;
            o += (int64_t)R * size[blk[b0 + i]];
        }
        for (int i = 0; i < nbf; ++i) {
            for (int j = i; j < nbf; ++j) {
                int p = blk[b0 + i], q = blk[b0 + j];
                int64_t op = joff[i], oq = joff[j];
                if (index[p] < index[q]) {
                    std::swap(p, q);
                    std::swap(op, oq);
                }
                MargPairRec& r = recs[rec_of(p, q)];
                out.contrib[r.c1++] = make_int4((int)op, (int)oq, size[p] | (size[q] << 8) | (R << 16), f);
            }
            const int p = blk[b0 + i];
            MargPairRec& r = recs[bvec[p]];
            out.contrib[r.c1++] = make_int4((int)joff[i], (int)res_off[f], size[p] | (1 << 8) | (R << 16), f);
        }
    }
    out.recs = std::move(recs);
    return GVX_OK;
}

// Hee (the first m local parameters) is diagonal: every block below m has one
// local parameter and no H0 record couples two different such blocks -- the
// reference's DENSE_SCHUR window, one inverse depth per landmark, each
// reprojection factor touching one landmark (ic_gvins.cc:1170-1180).
bool diagonal_e(const Lists& ls, int m) {
    for (int k = 0; k < ls.n_pairs; ++k) {
        const MargPairRec& r = ls.recs[k];  // row0 >= col0
        if (r.row0 >= m) continue;          // not an (eliminated, eliminated) pair
        if (r.row0 != r.col0 || r.lp != 1) return false;
    }
    return true;
}

struct DevOut {
    double *J0, *e0, *Hp, *bp, *eval;
    int32_t* info;
};

// Stages the lists (pinned -> device, one copy) and enqueues the pipeline.
gvx_status run(gvx_ctx* c, const Lists& ls, int n_fac, const int32_t* nres, const int64_t* res_off,
               const double* d_data, const double* d_loss, int m, int L, const DevOut& o) {
    const int r = L - m;
    MargPairRec *d_rec, *h_rec;
    int4 *d_con, *h_con;
    int32_t *d_nres, *h_nres;
    int64_t *d_roff, *h_roff;
    Staging lists;
    lists.add(ls.recs.size(), &d_rec, &h_rec);
    lists.add(ls.contrib.size(), &d_con, &h_con);
    const size_t nl = d_loss ? (size_t)n_fac : 0;
    lists.add(nl, &d_nres, &h_nres);
    lists.add(nl, &d_roff, &h_roff);
    const bool fast = c->marg_solver == GVX_MARG_SOLVER_FAST;
    int4 *d_chk = nullptr, *h_chk = nullptr;
    int2 *d_rpart = nullptr, *h_rpart = nullptr;
    if (fast) {
        lists.add(ls.chunks.size(), &d_chk, &h_chk);
        lists.add(ls.recpart.size(), &d_rpart, &h_rpart);
    }
    double *H0, *b0, *V1, *w1, *Hi, *T, *Hp, *bp, *V2, *w2, *hc, *sr, *J0, *e0, *Lm, *Lp, *X;
    int32_t *info, *chol;
    Staging work;
    work.add((size_t)L * L, &H0);
    work.add((size_t)L, &b0);
    work.add((size_t)m * m, &V1);
    work.add((size_t)m, &w1);
    work.add((size_t)m * m, &Hi);
    work.add((size_t)r * m, &T);
    work.add((size_t)r * r, &Hp);
    work.add((size_t)r, &bp);
    work.add((size_t)r * r, &V2);
    work.add((size_t)r, &w2);
    work.add((size_t)(m > r ? m : r), &hc);
    work.add((size_t)n_fac, &sr);
    work.add((size_t)r * r, &J0);
    work.add((size_t)r, &e0);
    work.add(2, &info);
    double* part = nullptr;
    if (fast) work.add((size_t)ls.n_part, &part);
    work.add(fast ? (size_t)m * m : 0, &Lm);
    work.add(fast ? (size_t)r * r : 0, &Lp);
    work.add(fast ? (size_t)m * (r + 1) : 0, &X);
    work.add(2, &chol);
    // the pinned list buffer may still feed an earlier call's upload
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "marginalisation: stream");
    void* hb = pinned(c, "marg_lists", lists.bytes());
    void* db = scratch(c, "marg_lists", lists.bytes());
    void* wb = scratch(c, "marg_work", work.bytes());
    if (!hb || !db || !wb) return set_err(c, GVX_ERR_OOM, "marginalisation staging");
    lists.bind(db, hb);
    work.bind(wb);
    if (!ls.recs.empty()) std::memcpy(h_rec, ls.recs.data(), sizeof(MargPairRec) * ls.recs.size());
    if (!ls.contrib.empty()) std::memcpy(h_con, ls.contrib.data(), sizeof(int4) * ls.contrib.size());
    if (nl) {
        std::memcpy(h_nres, nres, sizeof(int32_t) * nl);
        std::memcpy(h_roff, res_off, sizeof(int64_t) * nl);
    }
    if (fast) {
        std::memcpy(h_chk, ls.chunks.data(), sizeof(int4) * ls.chunks.size());
        std::memcpy(h_rpart, ls.recpart.data(), sizeof(int2) * ls.recpart.size());
    }
    e = hipMemcpyAsync(db, hb, lists.bytes(), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "marginalisation: list upload");
    if ((e = hipMemsetAsync(info, 0, 2 * sizeof(int32_t), c->stream)) != hipSuccess)
        return hip_err(c, e, "marginalisation: info");
    if ((e = hipMemsetAsync(chol, 0, 2 * sizeof(int32_t), c->stream)) != hipSuccess)
        return hip_err(c, e, "marginalisation: flags");
    MargLaunch p{};
    p.n_pairs = ls.n_pairs;
    p.n_bvec = ls.n_bvec;
    p.pairs = d_rec;
    p.contrib = d_con;
    p.n_fac = n_fac;
    p.nres = d_nres;
    p.res_off = d_roff;
    p.loss = d_loss;
    p.sr = sr;
    p.data = d_data;
    p.L = L;
    p.m = m;
    p.H0 = H0;
    p.b0 = b0;
    p.V1 = V1;
    p.w1 = w1;
    p.Hinv = Hi;
    p.T = T;
    p.Hp = o.Hp ? o.Hp : Hp;
    p.bp = o.bp ? o.bp : bp;
    p.V2 = V2;
    p.w2 = o.eval ? o.eval : w2;
    p.hc = hc;
    p.info = o.info ? o.info : info;
    p.J0 = o.J0 ? o.J0 : J0;
    p.e0 = o.e0 ? o.e0 : e0;
    p.solver = c->marg_solver;
    p.Lm = Lm;
    p.Lp = Lp;
    p.X = X;
    p.chol = chol;
    p.n_chunks = fast ? (int)ls.chunks.size() : 0;
    p.chunks = d_chk;
    p.recpart = d_rpart;
    p.part = part;
    if (o.info) {
        if ((e = hipMemsetAsync(o.info, 0, 2 * sizeof(int32_t), c->stream)) != hipSuccess)
            return hip_err(c, e, "marginalisation: info");
    }
    hipEvent_t ev{};
    prof_begin(c, "marg", &ev);
    e = launch_marginalize(c, p);
    prof_end(c, "marg", ev);
    return hip_err(c, e, "marginalisation kernels");
}

}  // namespace

gvx_status gvx_marginalize_dev(gvx_ctx* c, int32_t n_fac, const int32_t* nres, const int32_t* blk_off,
                               const int32_t* blk, const int64_t* res_off, const int64_t* jac_off,
                               const double* d_data, int64_t n_data, const double* d_loss, int32_t nb,
                               const int32_t* size, const int32_t* index, int32_t m, int32_t L, double* d_J0,
                               double* d_e0, double* d_Hp, double* d_bp, double* d_eval, int32_t* d_info) {
    if (!c) return GVX_ERR_INVALID;
    if (!d_J0 || !d_e0 || (n_fac && !d_data)) return set_err(c, GVX_ERR_INVALID, "null device pointer");
    hipSetDevice(c->device);
    Lists ls;
    gvx_status s = build_lists(c, n_fac, nres, blk_off, blk, res_off, jac_off, n_data, nb, size, index, m, L, ls);
    if (s) return s;
    if (c->marg_solver == GVX_MARG_SOLVER_FAST) make_chunks(ls);
    return run(c, ls, n_fac, nres, res_off, d_data, d_loss, m, L, DevOut{d_J0, d_e0, d_Hp, d_bp, d_eval, d_info});
}

gvx_status gvx_marginalize(gvx_ctx* c, int32_t n_fac, const int32_t* nres, const int32_t* blk_off, const int32_t* blk,
                           const int64_t* res_off, const int64_t* jac_off, const double* data, int64_t n_data,
                           const double* loss, int32_t nb, const int32_t* size, const int32_t* index, int32_t m,
                           int32_t L, double* J0, double* e0, double* Hp, double* bp, double* eval, int32_t* info) {
    if (!c) return GVX_ERR_INVALID;
    if (!J0 || !e0 || (n_fac && !data)) return set_err(c, GVX_ERR_INVALID, "null pointer");
    hipSetDevice(c->device);
    Lists ls;
    gvx_status s = build_lists(c, n_fac, nres, blk_off, blk, res_off, jac_off, n_data, nb, size, index, m, L, ls);
    if (s) return s;
    if (c->marg_solver == GVX_MARG_SOLVER_FAST) make_chunks(ls);
    const int r = L - m;
    // inputs and outputs through one pinned arena laid out like the device one
    double *d_in, *h_in, *d_loss, *h_loss, *d_J0, *h_J0, *d_e0, *h_e0, *d_Hp, *h_Hp, *d_bp, *h_bp, *d_ev, *h_ev;
    int32_t *d_info, *h_info;
    Staging st;
    st.add((size_t)n_data, &d_in, &h_in);
    st.add(loss ? (size_t)n_fac : 0, &d_loss, &h_loss);
    st.add((size_t)r * r, &d_J0, &h_J0);
    st.add((size_t)r, &d_e0, &h_e0);
    st.add((size_t)r * r, &d_Hp, &h_Hp);
    st.add((size_t)r, &d_bp, &h_bp);
    st.add((size_t)r, &d_ev, &h_ev);
    st.add(2, &d_info, &h_info);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "marginalisation: stream");
    void* hb = pinned(c, "marg_io", st.bytes());
    void* db = scratch(c, "marg_io", st.bytes());
    if (!hb || !db) return set_err(c, GVX_ERR_OOM, "marginalisation staging");
    st.bind(db, hb);
    if (n_data) std::memcpy(h_in, data, sizeof(double) * (size_t)n_data);
    if (loss) std::memcpy(h_loss, loss, sizeof(double) * (size_t)n_fac);
    e = hipMemcpyAsync(d_in, h_in, (size_t)((char*)d_J0 - (char*)d_in), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "marginalisation upload");
    s = run(c, ls, n_fac, nres, res_off, d_in, loss ? d_loss : nullptr, m, L,
            DevOut{d_J0, d_e0, d_Hp, d_bp, d_ev, d_info});
    if (s) return s;
    e = hipMemcpyAsync(h_J0, d_J0, (size_t)((char*)(d_info + 2) - (char*)d_J0), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "marginalisation download");
    std::memcpy(J0, h_J0, sizeof(double) * (size_t)r * r);
    std::memcpy(e0, h_e0, sizeof(double) * (size_t)r);
    if (Hp) std::memcpy(Hp, h_Hp, sizeof(double) * (size_t)r * r);
    if (bp) std::memcpy(bp, h_bp, sizeof(double) * (size_t)r);
    if (eval) std::memcpy(eval, h_ev, sizeof(double) * (size_t)r);
    if (info) std::memcpy(info, h_info, sizeof(int32_t) * 2);
    return GVX_OK;
}

// ---------------------------------------------------- LM step (DENSE_SCHUR)
namespace {

gvx_status run_lm(gvx_ctx* c, Lists& ls, const double* d_data, const double* d_D, int m, int L, double* d_delta,
                  double* d_S, int32_t* d_info) {
    const int r = L - m;
    // the dense L x L H0 (and the 32-bit indexing of the H0 kernels) bound the
    // window: GVX_SCHUR_MAX_L parameters, 2 GiB of H0
    if (L > GVX_SCHUR_MAX_L)
        return set_err(c, GVX_ERR_UNSUPPORTED, "schur solve: %d parameters (max %d)", L, GVX_SCHUR_MAX_L);
    const bool diag = diagonal_e(ls, m);
    if (!diag && m > GVX_EIG_MAX_N)
        return set_err(c, GVX_ERR_UNSUPPORTED, "schur solve: %d eliminated parameters with a non-diagonal Hee (max %d)",
                       m, GVX_EIG_MAX_N);
    make_chunks(ls);
    MargPairRec *d_rec, *h_rec;
    int4 *d_con, *h_con, *d_chk, *h_chk;
    int2 *d_rpart, *h_rpart;
    Staging lists;
    lists.add(ls.recs.size(), &d_rec, &h_rec);
    lists.add(ls.contrib.size(), &d_con, &h_con);
    lists.add(ls.chunks.size(), &d_chk, &h_chk);
    lists.add(ls.recpart.size(), &d_rpart, &h_rpart);
    double *H0, *b0, *Lm, *Lp, *X, *part, *S, *bs, *tmp;
    int32_t* chol;
    Staging work;
    work.add((size_t)L * L, &H0);
    work.add((size_t)L, &b0);
    work.add(diag ? (size_t)m : (size_t)m * m, &Lm);
    work.add((size_t)r * r, &Lp);
    work.add((size_t)m * (r + 1), &X);
    work.add((size_t)ls.n_part, &part);
    work.add((size_t)r * r, &S);
    work.add((size_t)r, &bs);
    work.add((size_t)(2 * m + r), &tmp);
    work.add(2, &chol);
    hipError_t e = hipStreamSynchronize(c->stream);  // the pinned list staging may feed an earlier call
    if (e != hipSuccess) return hip_err(c, e, "schur solve: stream");
    void* hb = pinned(c, "lm_lists", lists.bytes());
    void* db = scratch(c, "lm_lists", lists.bytes());
    void* wb = scratch(c, "lm_work", work.bytes());
    if (!hb || !db || !wb) return set_err(c, GVX_ERR_OOM, "schur solve staging");
    lists.bind(db, hb);
    work.bind(wb);
    std::memcpy(h_rec, ls.recs.data(), sizeof(MargPairRec) * ls.recs.size());
    if (!ls.contrib.empty()) std::memcpy(h_con, ls.contrib.data(), sizeof(int4) * ls.contrib.size());
    std::memcpy(h_chk, ls.chunks.data(), sizeof(int4) * ls.chunks.size());
    std::memcpy(h_rpart, ls.recpart.data(), sizeof(int2) * ls.recpart.size());
    e = hipMemcpyAsync(db, hb, lists.bytes(), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(chol, 0, 2 * sizeof(int32_t), c->stream);
    if (e != hipSuccess) return hip_err(c, e, "schur solve: upload");
    MargLaunch p{};
    p.n_pairs = ls.n_pairs;
    p.n_bvec = ls.n_bvec;
    p.pairs = d_rec;
    p.contrib = d_con;
    p.data = d_data;
    p.L = L;
    p.m = m;
    p.H0 = H0;
    p.b0 = b0;
    p.Lm = Lm;
    p.Lp = Lp;
    p.X = X;
    p.chol = chol;
    p.n_chunks = (int)ls.chunks.size();
    p.chunks = d_chk;
    p.recpart = d_rpart;
    p.part = part;
    p.diag_e = diag ? 1 : 0;
    hipEvent_t ev{};
    prof_begin(c, "lm_step", &ev);
    e = launch_lm_step(c, p, d_D, d_delta, d_S ? d_S : S, bs, tmp);
    if (e == hipSuccess && d_info) e = hipMemcpyAsync(d_info, chol, 2 * sizeof(int32_t), hipMemcpyDeviceToDevice, c->stream);
    prof_end(c, "lm_step", ev);
    return hip_err(c, e, "schur solve kernels");
}

}  // namespace

gvx_status gvx_schur_solve_dev(gvx_ctx* c, int32_t n_fac, const int32_t* nres, const int32_t* blk_off,
                               const int32_t* blk, const int64_t* res_off, const int64_t* jac_off,
                               const double* d_data, int64_t n_data, int32_t nb, const int32_t* size,
                               const int32_t* index, int32_t m, int32_t L, const double* d_D, double* d_delta,
                               double* d_S, int32_t* d_info) {
    if (!c) return GVX_ERR_INVALID;
    if (!d_delta || (n_fac && !d_data)) return set_err(c, GVX_ERR_INVALID, "null device pointer");
    if (L > GVX_SCHUR_MAX_L)  // before any list or staging is sized
        return set_err(c, GVX_ERR_UNSUPPORTED, "schur solve: %d parameters (max %d)", L, GVX_SCHUR_MAX_L);
    hipSetDevice(c->device);
    Lists ls;
    gvx_status s =
        build_lists(c, n_fac, nres, blk_off, blk, res_off, jac_off, n_data, nb, size, index, m, L, ls, INT32_MAX);
    if (s) return s;
    return run_lm(c, ls, d_data, d_D, m, L, d_delta, d_S, d_info);
}

gvx_status gvx_schur_solve(gvx_ctx* c, int32_t n_fac, const int32_t* nres, const int32_t* blk_off, const int32_t* blk,
                           const int64_t* res_off, const int64_t* jac_off, const double* data, int64_t n_data,
                           int32_t nb, const int32_t* size, const int32_t* index, int32_t m, int32_t L,
                           const double* D, double* delta, double* S, int32_t* info) {
    if (!c) return GVX_ERR_INVALID;
    if (!delta || (n_fac && !data)) return set_err(c, GVX_ERR_INVALID, "null pointer");
    if (L > GVX_SCHUR_MAX_L)  // before the r x r pinned / device staging is sized
        return set_err(c, GVX_ERR_UNSUPPORTED, "schur solve: %d parameters (max %d)", L, GVX_SCHUR_MAX_L);
    hipSetDevice(c->device);
    Lists ls;
    gvx_status s =
        build_lists(c, n_fac, nres, blk_off, blk, res_off, jac_off, n_data, nb, size, index, m, L, ls, INT32_MAX);
    if (s) return s;
    const int r = L - m;
    double *d_in, *h_in, *d_D, *h_D, *d_delta, *h_delta, *d_S, *h_S;
    int32_t *d_info, *h_info;
    Staging st;
    st.add((size_t)n_data, &d_in, &h_in);
    st.add(D ? (size_t)L : 0, &d_D, &h_D);
    st.add((size_t)L, &d_delta, &h_delta);
    st.add((size_t)r * r, &d_S, &h_S);
    st.add(2, &d_info, &h_info);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "schur solve: stream");
    void* hb = pinned(c, "lm_io", st.bytes());
    void* db = scratch(c, "lm_io", st.bytes());
    if (!hb || !db) return set_err(c, GVX_ERR_OOM, "schur solve staging");
    st.bind(db, hb);
    if (n_data) std::memcpy(h_in, data, sizeof(double) * (size_t)n_data);
    if (D) std::memcpy(h_D, D, sizeof(double) * (size_t)L);
    e = hipMemcpyAsync(d_in, h_in, (size_t)((char*)d_delta - (char*)d_in), hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "schur solve upload");
    s = run_lm(c, ls, d_in, D ? d_D : nullptr, m, L, d_delta, d_S, d_info);
    if (s) return s;
    e = hipMemcpyAsync(h_delta, d_delta, (size_t)((char*)(d_info + 2) - (char*)d_delta), hipMemcpyDeviceToHost,
                       c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "schur solve download");
    std::memcpy(delta, h_delta, sizeof(double) * (size_t)L);
    if (S) std::memcpy(S, h_S, sizeof(double) * (size_t)r * r);
    if (info) std::memcpy(info, h_info, sizeof(int32_t) * 2);
    if (h_info[0] || h_info[1])
        return set_err(c, GVX_ERR_NUMERIC, "schur solve: %s not positive definite (delta is NaN)",
                       h_info[0] ? "Hee + D" : "the reduced system S");
    return GVX_OK;
}

gvx_status gvx_set_marg_solver(gvx_ctx* c, int32_t solver) {
    if (!c) return GVX_ERR_INVALID;
    if (solver != GVX_MARG_SOLVER_EXACT && solver != GVX_MARG_SOLVER_FAST)
        return set_err(c, GVX_ERR_INVALID, "unknown marginalisation solver %d", solver);
    c->marg_solver = solver;
    return GVX_OK;
}

gvx_status gvx_sym_eigen(gvx_ctx* c, int32_t n, const double* A, int32_t lda, double* w, double* V, int32_t* info) {
    if (!c) return GVX_ERR_INVALID;
    if (n < 0 || lda < n) return set_err(c, GVX_ERR_INVALID, "bad size n = %d, lda = %d", n, lda);
    if (n > GVX_EIG_MAX_N) return set_err(c, GVX_ERR_UNSUPPORTED, "n = %d above %d", n, GVX_EIG_MAX_N);
    if (n == 0) return GVX_OK;
    if (!A || !w || !V) return set_err(c, GVX_ERR_INVALID, "null pointer");
    hipSetDevice(c->device);
    double *d_A, *h_A, *d_V, *h_V, *d_w, *h_w, *d_hc;
    int32_t *d_info, *h_info;
    unsigned long long *d_ts, *h_ts;
    Staging st;
    st.add((size_t)n * n, &d_A, &h_A);
    st.add((size_t)n * n, &d_V, &h_V);
    st.add((size_t)n, &d_w, &h_w);
    st.add(1, &d_info, &h_info);
    st.add(8, &d_ts, &h_ts);
    st.add((size_t)n, &d_hc);
    // GVX_EIG_TIMING=1: the solver's phase times to stderr (diagnostics)
    static const bool timing = getenv("GVX_EIG_TIMING") && *getenv("GVX_EIG_TIMING") == '1';
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "eigen: stream");
    void* hb = pinned(c, "eigen", st.bytes());
    void* db = scratch(c, "eigen", st.bytes());
    if (!hb || !db) return set_err(c, GVX_ERR_OOM, "eigen staging");
    st.bind(db, hb);
    for (int j = 0; j < n; ++j) std::memcpy(h_A + (size_t)j * n, A + (size_t)j * lda, sizeof(double) * n);
    e = hipMemcpyAsync(d_A, h_A, sizeof(double) * (size_t)n * n, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) return hip_err(c, e, "eigen upload");
    hipEvent_t ev{};
    prof_begin(c, "eigen", &ev);
    e = launch_sym_eigen(c, n, d_A, n, d_V, d_w, d_hc, d_info, timing ? d_ts : nullptr);
    prof_end(c, "eigen", ev);
    if (e != hipSuccess) return hip_err(c, e, "eigen kernel");
    e = hipMemcpyAsync(h_V, d_V, (size_t)((char*)(d_ts + 8) - (char*)d_V), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_err(c, e, "eigen download");
    std::memcpy(V, h_V, sizeof(double) * (size_t)n * n);
    std::memcpy(w, h_w, sizeof(double) * n);
    if (info) *info = *h_info;
    if (timing && n > 1)
        fprintf(stderr, "gvx eigen n=%d us: scale %.1f tridiag %.1f Q %.1f QR %.1f (%llu sweeps, %llu rotations) sort %.1f\n",
                n, (h_ts[1] - h_ts[0]) * 0.01, (h_ts[2] - h_ts[1]) * 0.01, (h_ts[3] - h_ts[2]) * 0.01,
                (h_ts[4] - h_ts[3]) * 0.01, h_ts[6], h_ts[7], (h_ts[5] - h_ts[4]) * 0.01);
    return GVX_OK;
}
