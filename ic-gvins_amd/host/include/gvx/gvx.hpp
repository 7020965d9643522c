// gvx.hpp -- C++ host mirror of the reference interfaces on the accelerated
// path, layered on the C ABI (include/gvx.h).  Header-only, C++17, no OpenCV /
// Eigen / Ceres dependency: the types are layout- and meaning-compatible stand-ins
// so the reference's call sites change only in the object they call.
//
//   reference (paths under /root/reference/ic_gvins/ic_gvins/)      here
//   cv::calcOpticalFlowPyrLK (tracking/tracking.cc:385,390,487,493)  gvx::calcOpticalFlowPyrLK
//   fwd/bwd/FB/reduceVector (tracking/tracking.cc:380-408, :831-849) gvx::trackFB, gvx::reduceVector
//   Tracking::featuresDetection (tracking/tracking.cc:576-688)       gvx::featuresDetection
//   PreintegrationBase / Earth / Normal (preintegration/*.h)          gvx::Preintegration
//   PreintegrationFactor::Evaluate (preintegration_factor.h:45-69)    gvx::PreintegrationFactor
//   ReprojectionFactor::Evaluate (factors/reprojection_factor.h:61)   gvx::ReprojectionFactor
//   cv::findFundamentalMat(FM_RANSAC) (tracking/tracking.cc:548)      gvx::findFundamentalMat
//   ResidualBlockInfo (factors/residual_block_info.h)                 gvx::ResidualBlockInfo
//   MarginalizationInfo (factors/marginalization_info.h)              gvx::MarginalizationInfo
//   MarginalizationFactor::Evaluate (marginalization_factor.h:54)     gvx::MarginalizationFactor
//
// Errors: the C ABI never throws; this layer converts a non-OK status into
// gvx::Error (the role cv::Exception plays for bad arguments in the reference).
// There is no CPU fallback: without a gfx950 device gvx::Context throws.
#pragma once

#include <gvx.h>

#include <array>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <unordered_map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace gvx {

class Error : public std::runtime_error {
public:
    Error(gvx_status s, const std::string& what) : std::runtime_error(what), status_(s) {}
    gvx_status status() const { return status_; }

private:
    gvx_status status_;
};

inline void check(gvx_status s, const gvx_ctx* c, const char* what) {
    if (s == GVX_OK) return;
    std::string msg = std::string(what) + ": " + gvx_status_string(s);
    if (c && gvx_last_error(c) && *gvx_last_error(c)) msg += std::string(" (") + gvx_last_error(c) + ")";
    throw Error(s, msg);
}

// One device context (stream, frame cache, scratch).  One per host thread, as
// the reference's tracking thread / Ceres workers would hold.
class Context {
public:
    explicit Context(int device = 0) { check(gvx_create(device, &c_), nullptr, "gvx_create"); }
    ~Context() { gvx_destroy(c_); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    gvx_ctx* get() const { return c_; }
    void sync() const { check(gvx_sync(c_), c_, "gvx_sync"); }

private:
    gvx_ctx* c_ = nullptr;
};

// ------------------------------------------------------------------ KLT
// OpenCV-shaped value types (layout of cv::Point2f / cv::Size / cv::TermCriteria).
struct Point2f {
    float x = 0.f, y = 0.f;
};
static_assert(sizeof(Point2f) == 8, "Point2f must be two packed floats");
struct Size {
    int width = 21, height = 21;
};
struct TermCriteria {
    enum { COUNT = 1, MAX_ITER = 1, EPS = 2 };
    int type = COUNT + EPS;
    int maxCount = 30;
    double epsilon = 0.01;
};
enum { OPTFLOW_USE_INITIAL_FLOW = 4, OPTFLOW_LK_GET_MIN_EIGENVALS = 8 };

// A gray frame (Frame::image() after CLAHE, tracking/frame.h:62-64) resident on
// the device with its pyramid built once; replaces the per-call
// buildOpticalFlowPyramid of every cv::calcOpticalFlowPyrLK on that image.
class GpuFrame {
public:
    GpuFrame(Context& ctx, const uint8_t* gray, int w, int h, int stride, int maxLevel = 3)
        : ctx_(&ctx), id_(next_id()), w_(w), h_(h), max_level_(maxLevel) {
        gvx_klt_params p;
        gvx_klt_params_default(&p);
        p.max_level = maxLevel;
        check(gvx_frame_put(ctx.get(), id_, gray, w, h, stride, &p), ctx.get(), "gvx_frame_put");
    }
    // The raw frame through Tracking::preprocessing's CLAHE first (see preprocessFrame).
    GpuFrame(Context& ctx, const uint8_t* gray, int w, int h, int stride, int maxLevel, const gvx_clahe_params* cp,
             uint8_t* equalized, double* histMean)
        : ctx_(&ctx), id_(next_id()), w_(w), h_(h), max_level_(maxLevel) {
        gvx_klt_params p;
        gvx_klt_params_default(&p);
        p.max_level = maxLevel;
        check(gvx_frame_preprocess(ctx.get(), id_, gray, w, h, stride, cp, &p, histMean, equalized), ctx.get(),
              "gvx_frame_preprocess");
    }
    ~GpuFrame() {
        if (ctx_) gvx_frame_drop(ctx_->get(), id_);
    }
    GpuFrame(GpuFrame&& o) noexcept : ctx_(o.ctx_), id_(o.id_), w_(o.w_), h_(o.h_), max_level_(o.max_level_) {
        o.ctx_ = nullptr;
    }
    GpuFrame(const GpuFrame&) = delete;
    GpuFrame& operator=(const GpuFrame&) = delete;
    uint64_t id() const { return id_; }
    int width() const { return w_; }
    int height() const { return h_; }
    int maxLevel() const { return max_level_; }
    Context& context() const { return *ctx_; }

private:
    static uint64_t next_id() {
        static std::atomic<uint64_t> n{1ull << 40};
        return n++;
    }
    Context* ctx_;
    uint64_t id_;
    int w_, h_, max_level_;
};

namespace detail {
// cv::calcOpticalFlowPyrLK's criteria handling (lkpyramid.cpp): COUNT clamped
// to [0, 100] (default 30), EPS clamped to [0, 10] (default 0.01).
inline gvx_klt_params klt_params(Size win, int maxLevel, TermCriteria c, int flags, double minEig) {
    if (win.width != 21 || win.height != 21)
        throw Error(GVX_ERR_UNSUPPORTED, "calcOpticalFlowPyrLK: the device path is specialised for 21x21");
    if (flags & OPTFLOW_LK_GET_MIN_EIGENVALS)
        throw Error(GVX_ERR_UNSUPPORTED, "calcOpticalFlowPyrLK: OPTFLOW_LK_GET_MIN_EIGENVALS is not on the path");
    gvx_klt_params p;
    gvx_klt_params_default(&p);
    p.win = 21;
    p.max_level = maxLevel;
    p.max_iter = (c.type & TermCriteria::COUNT) ? (c.maxCount < 0 ? 0 : c.maxCount > 100 ? 100 : c.maxCount) : 30;
    p.eps = (c.type & TermCriteria::EPS) ? (c.epsilon < 0 ? 0 : c.epsilon > 10 ? 10 : c.epsilon) : 0.01;
    p.use_initial_flow = (flags & OPTFLOW_USE_INITIAL_FLOW) ? 1 : 0;
    p.min_eig = (float)minEig;
    return p;
}
}  // namespace detail

// cv::calcOpticalFlowPyrLK(prevImg, nextImg, prevPts, nextPts, status, err,
// winSize, maxLevel, criteria, flags, minEigThreshold) on device-resident frames.
inline void calcOpticalFlowPyrLK(const GpuFrame& prev, const GpuFrame& next, const std::vector<Point2f>& prevPts,
                                 std::vector<Point2f>& nextPts, std::vector<uint8_t>& status,
                                 std::vector<float>& err, Size winSize = Size(), int maxLevel = 3,
                                 TermCriteria criteria = TermCriteria(), int flags = 0,
                                 double minEigThreshold = 1e-4) {
    gvx_klt_params p = detail::klt_params(winSize, maxLevel, criteria, flags, minEigThreshold);
    const size_t n = prevPts.size();
    if (p.use_initial_flow) {
        if (nextPts.size() != n) throw Error(GVX_ERR_INVALID, "calcOpticalFlowPyrLK: nextPts size != prevPts size");
    } else {
        nextPts = prevPts;
    }
    status.assign(n, 0);
    err.assign(n, 0.f);
    gvx_ctx* c = prev.context().get();
    check(gvx_klt(c, prev.id(), next.id(), reinterpret_cast<const float*>(prevPts.data()),
                  reinterpret_cast<float*>(nextPts.data()), status.data(), err.data(), (int32_t)n, &p),
          c, "gvx_klt");
}

// Fused tracking/tracking.cc:380-408: forward LK with initial flow, backward LK
// seeded with prevPts, keep = st_f && st_b && !isOnBorder(next) &&
// ptsDistance(back, prev) < fbThresh, plus the reduceVector index list.
struct TrackFB {
    std::vector<Point2f> next, back;
    std::vector<uint8_t> statusFwd, statusBwd, keep;
    std::vector<int32_t> kept;  // order-preserving indices with keep == 1
};
inline TrackFB trackFB(const GpuFrame& prev, const GpuFrame& next, const std::vector<Point2f>& prevPts,
                       const std::vector<Point2f>& initPts, int camWidth, int camHeight, double fbThresh = 0.5,
                       double border = 5.0, int maxLevel = 3) {
    const size_t n = prevPts.size();
    if (initPts.size() != n) throw Error(GVX_ERR_INVALID, "trackFB: initPts size != prevPts size");
    gvx_klt_params p = detail::klt_params(Size(), maxLevel, TermCriteria(), OPTFLOW_USE_INITIAL_FLOW, 1e-4);
    TrackFB r;
    r.next = initPts;
    r.back.resize(n);
    r.statusFwd.resize(n);
    r.statusBwd.resize(n);
    r.keep.resize(n);
    r.kept.resize(n);
    int32_t nk = 0;
    gvx_ctx* c = prev.context().get();
    check(gvx_klt_fb(c, prev.id(), next.id(), reinterpret_cast<const float*>(prevPts.data()),
                     reinterpret_cast<float*>(r.next.data()), reinterpret_cast<float*>(r.back.data()),
                     r.statusFwd.data(), r.statusBwd.data(), r.keep.data(), r.kept.data(), &nk, (int32_t)n,
                     fbThresh, border, camWidth, camHeight, &p),
          c, "gvx_klt_fb");
    r.kept.resize((size_t)nk);
    return r;
}

// Tracking::reduceVector (tracking/tracking.cc:831-839): keep the entries whose
// status is non-zero, in order.
template <class T>
void reduceVector(std::vector<T>& vec, const std::vector<uint8_t>& status) {
    size_t j = 0;
    for (size_t i = 0; i < vec.size(); ++i)
        if (status[i]) vec[j++] = vec[i];
    vec.resize(j);
}

enum { FM_RANSAC = 8 };  // cv::FM_RANSAC
// cv::findFundamentalMat(points1, points2, FM_RANSAC, ransacReprojThreshold,
// confidence, mask) as tracking/tracking.cc:548 calls it (>= 15 points); the mask
// is resized to the point count.  Returns false when no model was found (the mask
// is then all zero).  F (optional): the best model, row-major.
inline bool findFundamentalMat(Context& ctx, const std::vector<Point2f>& points1, const std::vector<Point2f>& points2,
                               int method, double ransacReprojThreshold, double confidence,
                               std::vector<uint8_t>& mask, double* F = nullptr, int maxIters = 1000) {
    if (method != FM_RANSAC) throw Error(GVX_ERR_UNSUPPORTED, "findFundamentalMat: only FM_RANSAC is on the path");
    if (points1.size() != points2.size()) throw Error(GVX_ERR_INVALID, "findFundamentalMat: point count mismatch");
    const int32_t off[2] = {0, (int32_t)points1.size()};
    mask.resize(points1.size());
    int32_t result = 0;
    double f[9];
    check(gvx_find_fundamental_ransac(ctx.get(), 1, off, reinterpret_cast<const float*>(points1.data()),
                                      reinterpret_cast<const float*>(points2.data()), ransacReprojThreshold,
                                      confidence, maxIters, mask.data(), f, &result),
          ctx.get(), "findFundamentalMat");
    if (F && result == 1) std::memcpy(F, f, sizeof f);
    return result != 0;
}

// Tracking::featuresDetection (tracking/tracking.cc:576-688) on a device frame:
// block grid of the Tracking ctor, circle mask around maskPts (when ismask),
// per-block goodFeaturesToTrack + cornerSubPix.  countPts are the points counted
// per block (frame->features() + pts2d_new_), nExisting = features + pts2d_ref_
// for the early exit.  Returns false when the early exit triggers.
struct DetectParams {
    gvx_detect_params p;
    DetectParams() { gvx_detect_params_default(&p); }
};
inline bool featuresDetection(const GpuFrame& frame, const std::vector<Point2f>& countPts,
                              const std::vector<Point2f>& maskPts, bool ismask, int nExisting,
                              const DetectParams& prm, std::vector<Point2f>& corners,
                              std::vector<int32_t>* blockCounts = nullptr) {
    // upper bound of block_cnts * track_max_block_features_
    const double bs = prm.p.block_size;
    const int cols = (int)(frame.width() / bs + 1.5), rows = (int)(frame.height() / bs + 1.5);
    const size_t cap = (size_t)(cols + 1) * (rows + 1) * (size_t)(prm.p.max_features + 1);
    std::vector<Point2f> out(cap);
    std::vector<int32_t> blk((size_t)(cols + 1) * (rows + 1));
    int32_t n = 0;
    gvx_ctx* c = frame.context().get();
    check(gvx_detect(c, frame.id(), reinterpret_cast<const float*>(countPts.data()), (int32_t)countPts.size(),
                     reinterpret_cast<const float*>(maskPts.data()), (int32_t)maskPts.size(), ismask ? 1 : 0,
                     nExisting, &prm.p, reinterpret_cast<float*>(out.data()), blk.data(), &n),
          c, "gvx_detect");
    if (n < 0) {
        corners.clear();
        return false;
    }
    out.resize((size_t)n);
    corners = std::move(out);
    if (blockCounts) *blockCounts = blk;
    return true;
}

// ------------------------------------------------------- preprocessing
// cv::CLAHE stand-in: createCLAHE(clipLimit, tileGridSize) then apply (in place
// allowed), as Tracking builds it at tracking.cc:63 and applies it at :139.
class CLAHE {
public:
    CLAHE(Context& ctx, double clipLimit = 40.0, Size tileGridSize = Size{8, 8}) : ctx_(&ctx) {
        gvx_clahe_params_default(&p_);  // MONO8 source (cv::CLAHE::apply takes CV_8UC1)
        p_.clip_limit = clipLimit;
        p_.tiles_x = tileGridSize.width;
        p_.tiles_y = tileGridSize.height;
    }
    void apply(const uint8_t* src, int w, int h, int srcStride, uint8_t* dst, int dstStride) const {
        check(gvx_clahe(ctx_->get(), w, h, src, srcStride, dst, dstStride, &p_, nullptr), ctx_->get(), "gvx_clahe");
    }
    const gvx_clahe_params& params() const { return p_; }
    Context& context() const { return *ctx_; }

private:
    Context* ctx_;
    gvx_clahe_params p_;
};
inline CLAHE createCLAHE(Context& ctx, double clipLimit = 40.0, Size tileGridSize = Size{8, 8}) {
    return CLAHE(ctx, clipLimit, tileGridSize);
}

// Tracking::preprocessing (tracking.cc:107-141) + the frame upload in one call:
// CLAHE of the raw gray frame on the device, then its pyramid (a GpuFrame of the
// equalised image).  equalized (nullable, w*h bytes) receives frame->image()
// after :139; histMean (nullable) calculateHistigram of the raw frame (:88-105).
inline GpuFrame preprocessFrame(const CLAHE& clahe, const uint8_t* gray, int w, int h, int stride,
                                uint8_t* equalized = nullptr, double* histMean = nullptr, int maxLevel = 3) {
    return GpuFrame(clahe.context(), gray, w, h, stride, maxLevel, &clahe.params(), equalized, histMean);
}

// ---------------------------------------------------------- camera ops
// Camera (tracking/camera.h) point operations on the device; vectors in/out like
// the reference's std::vector<cv::Point2f> calls.
class Camera {
public:
    Camera(Context& ctx, const gvx_camera& c) : ctx_(&ctx), c_(c) {}
    // Camera::undistortPoints / distortPoints (camera.cc:72-89), in place
    void undistortPoints(std::vector<Point2f>& pts) const { run(gvx_undistort_points, pts); }
    void distortPoints(std::vector<Point2f>& pts) const { run(gvx_distort_points, pts); }
    // trackReferenceFrame's initial flow (tracking.cc:465-478)
    std::vector<Point2f> predictRotated(const std::array<double, 9>& r_cur_pre, const std::vector<Point2f>& pts) const {
        std::vector<Point2f> out(pts.size());
        check(gvx_predict_rotated(ctx_->get(), &c_, r_cur_pre.data(), (int32_t)pts.size(), fp(pts), fp(out)),
              ctx_->get(), "gvx_predict_rotated");
        return out;
    }
    // trackMappoint's prediction: world2pixel + distortPoints (tracking.cc:366-377); pw n x 3
    std::vector<Point2f> projectPoints(const std::array<double, 9>& R, const std::array<double, 3>& t,
                                       const std::vector<double>& pw) const {
        std::vector<Point2f> out(pw.size() / 3);
        check(gvx_project_points(ctx_->get(), &c_, R.data(), t.data(), (int32_t)out.size(), pw.data(), fp(out)),
              ctx_->get(), "gvx_project_points");
        return out;
    }
    // (pixel2cam(cur) - pixel2cam(pre)) / dt (tracking.cc:433, :530), n x 2
    std::vector<double> velocity(const std::vector<Point2f>& pre, const std::vector<Point2f>& cur, double dt) const {
        if (pre.size() != cur.size()) throw Error(GVX_ERR_INVALID, "velocity: size mismatch");
        std::vector<double> v(2 * pre.size());
        check(gvx_point_velocity(ctx_->get(), &c_, (int32_t)pre.size(), fp(pre), fp(cur), dt, v.data()),
              ctx_->get(), "gvx_point_velocity");
        return v;
    }
    // Tracking::keyPointParallax (tracking.cc:861-871) per pair
    std::vector<double> keyPointParallax(const std::array<double, 9>& R0, const std::array<double, 9>& R1,
                                         const std::vector<Point2f>& ref, const std::vector<Point2f>& cur) const {
        if (ref.size() != cur.size()) throw Error(GVX_ERR_INVALID, "keyPointParallax: size mismatch");
        std::vector<double> out(ref.size());
        check(gvx_keypoint_parallax(ctx_->get(), &c_, R0.data(), R1.data(), (int32_t)ref.size(), fp(ref), fp(cur),
                                    out.data()),
              ctx_->get(), "gvx_keypoint_parallax");
        return out;
    }
    double focalLength() const { return (c_.fx + c_.fy) * 0.5; }  // camera.h:82-84

private:
    static const float* fp(const std::vector<Point2f>& v) { return reinterpret_cast<const float*>(v.data()); }
    static float* fp(std::vector<Point2f>& v) { return reinterpret_cast<float*>(v.data()); }
    template <class F>
    void run(F f, std::vector<Point2f>& pts) const {
        std::vector<Point2f> out(pts.size());
        check(f(ctx_->get(), &c_, (int32_t)pts.size(), fp(pts), fp(out)), ctx_->get(), "camera op");
        pts.swap(out);
    }
    Context* ctx_;
    gvx_camera c_;
};

// ------------------------------------------------------ preintegration
using IMU = gvx_imu;  // common/types.h:50-58 {time, dt, dtheta[3], dvel[3], odovel}

// IntegrationParameters (preintegration/integration_state.h:68-89): the
// fields the NORMAL / EARTH variants read.  station stays zero unless set, as
// in the reference (resetState computes iewn from it).
struct IntegrationParameters {
    double acc_vrw = 0, gyr_arw = 0, gyr_bias_std = 0, acc_bias_std = 0, corr_time = 0, gravity = 9.8;
    std::array<double, 3> station{0, 0, 0};
};

// IntegrationState core (integration_state.h:35-51); q = (x, y, z, w).
struct IntegrationState {
    double time = 0;
    std::array<double, 3> p{0, 0, 0};
    std::array<double, 4> q{0, 0, 0, 1};
    std::array<double, 3> v{0, 0, 0}, bg{0, 0, 0}, ba{0, 0, 0};
};

namespace detail {
inline gvx_state to_c(const IntegrationState& s) {
    gvx_state o;
    o.time = s.time;
    std::memcpy(o.p, s.p.data(), sizeof o.p);
    std::memcpy(o.q, s.q.data(), sizeof o.q);
    std::memcpy(o.v, s.v.data(), sizeof o.v);
    std::memcpy(o.bg, s.bg.data(), sizeof o.bg);
    std::memcpy(o.ba, s.ba.data(), sizeof o.ba);
    return o;
}
inline IntegrationState from_c(const gvx_state& s) {
    IntegrationState o;
    o.time = s.time;
    std::memcpy(o.p.data(), s.p, sizeof s.p);
    std::memcpy(o.q.data(), s.q, sizeof s.q);
    std::memcpy(o.v.data(), s.v, sizeof s.v);
    std::memcpy(o.bg.data(), s.bg, sizeof s.bg);
    std::memcpy(o.ba.data(), s.ba, sizeof s.ba);
    return o;
}
}  // namespace detail

// PreintegrationBase with the NORMAL or EARTH variant
// (preintegration/preintegration_base.h:38-70, preintegration_earth.h,
// preintegration_normal.h): same constructor arguments, addNewImu /
// reintegration / getters, and the factor-side evaluate + Jacobian blocks.
// The IMU buffer lives on the host; the integration runs on the device (one
// wavefront) when a result is first needed after a change -- integrating the
// whole buffer at once is the same arithmetic, step by step, as the
// reference's per-sample integrationProcess.
class Preintegration {
public:
    enum Variant { NORMAL = GVX_PREINT_NORMAL, EARTH = GVX_PREINT_EARTH };

    Preintegration(Context& ctx, Variant variant, const IntegrationParameters& prm, const IMU& imu0,
                   const IntegrationState& state)
        : ctx_(&ctx), variant_(variant), prm_(prm), state0_(state) {
        imu_buffer_.push_back(imu0);
    }

    void addNewImu(const IMU& imu) {
        imu_buffer_.push_back(imu);
        dirty_ = true;
    }
    // preintegration_base.cc:77-84: restart from `state`, re-integrate the buffer
    void reintegration(IntegrationState& state) {
        state0_ = state;
        dirty_ = true;
    }

    IntegrationState currentState() { return detail::from_c(result().current); }
    IntegrationState deltaState() { return detail::from_c(result().delta); }
    double deltaTime() { return result().delta_time; }
    double startTime() { return result().start_time; }
    double endTime() { return result().end_time; }
    std::array<double, 3> gravity() { return {result().gravity[0], result().gravity[1], result().gravity[2]}; }
    const std::vector<IMU>& imuBuffer() const { return imu_buffer_; }
    const gvx_preint_result& raw() { return result(); }
    const std::vector<double>& pn() {
        result();
        return pn_;
    }

    static constexpr int numResiduals() { return 15; }
    static std::vector<int> numBlocksParameters() { return {7, 9, 7, 9}; }
    int numMixParametersBlocks() const { return 9; }

    // constructState (preintegration_earth.cc:186-203): pose[7] = p, q(x,y,z,w);
    // mix[9] = v, bg, ba
    static void constructState(const double* const* parameters, IntegrationState& s0, IntegrationState& s1) {
        auto fill = [](const double* pose, const double* mix, IntegrationState& s) {
            s.p = {pose[0], pose[1], pose[2]};
            s.q = {pose[3], pose[4], pose[5], pose[6]};
            s.v = {mix[0], mix[1], mix[2]};
            s.bg = {mix[3], mix[4], mix[5]};
            s.ba = {mix[6], mix[7], mix[8]};
        };
        fill(parameters[0], parameters[1], s0);
        fill(parameters[2], parameters[3], s1);
    }

    // PreintegrationFactor::Evaluate semantics on one parameter set: residuals
    // (15) and, for every non-null jacobians[k], the Ceres row-major block
    // (15x7, 15x9, 15x7, 15x9), each already multiplied by sqrt_info.
    void evaluateAll(const double* const* parameters, double* residuals, double** jacobians) {
        const gvx_preint_result& r = result();
        double params[32];
        std::memcpy(params, parameters[0], 7 * sizeof(double));
        std::memcpy(params + 7, parameters[1], 9 * sizeof(double));
        std::memcpy(params + 16, parameters[2], 7 * sizeof(double));
        std::memcpy(params + 23, parameters[3], 9 * sizeof(double));
        const int32_t offs[4] = {0, 7, 16, 23};
        const int32_t pn_off = 0;
        double res[15];
        std::vector<double> jac(jacobians ? 480 : 0);
        const bool earth = variant_ == EARTH;
        check(gvx_preint_factor_eval(ctx_->get(), 1, &r, earth ? pn_.data() : nullptr,
                                     earth ? (int32_t)(pn_.size() / 4) : 0, earth ? &pn_off : nullptr, params, 32,
                                     offs, res, jacobians ? jac.data() : nullptr),
              ctx_->get(), "gvx_preint_factor_eval");
        if (residuals) std::memcpy(residuals, res, sizeof res);
        if (jacobians) {
            static const int cols[4] = {7, 9, 7, 9}, start[4] = {0, 105, 240, 345};
            for (int k = 0; k < 4; ++k)
                if (jacobians[k]) std::memcpy(jacobians[k], jac.data() + start[k], sizeof(double) * 15 * cols[k]);
        }
    }

private:
    const gvx_preint_result& result() {
        if (!dirty_) return res_;
        const int32_t m = (int32_t)imu_buffer_.size();
        const int32_t seg_off[2] = {0, m};
        const gvx_state s0 = detail::to_c(state0_);
        double iewn[3] = {0, 0, 0};
        if (variant_ == EARTH) gvx_earth_iewn(prm_.station.data(), state0_.p.data(), iewn);
        gvx_imu_params p{prm_.acc_vrw, prm_.gyr_arw, prm_.gyr_bias_std, prm_.acc_bias_std, prm_.corr_time,
                         prm_.gravity};
        pn_.assign((size_t)(m > 1 ? m - 1 : 0) * 4 + 4, 0.0);
        check(gvx_preint_integrate(ctx_->get(), (int32_t)variant_, &p, 1, imu_buffer_.data(), seg_off, &s0, iewn,
                                   &res_, variant_ == EARTH ? pn_.data() : nullptr),
              ctx_->get(), "gvx_preint_integrate");
        pn_.resize((size_t)(m > 1 ? m - 1 : 0) * 4);
        dirty_ = false;
        return res_;
    }

    Context* ctx_;
    Variant variant_;
    IntegrationParameters prm_;
    IntegrationState state0_;
    std::vector<IMU> imu_buffer_;
    std::vector<double> pn_;
    gvx_preint_result res_{};
    bool dirty_ = true;
};

// ceres::CostFunction-shaped wrappers: Evaluate(parameters, residuals,
// jacobians) with the reference's block sizes.  A ceres::CostFunction subclass
// forwarding to these is all the integration needs.
// ------------------------------------------------------- INS mechanization
// The fields of IntegrationConfiguration that MISC::insMechanization reads
// (integration_state.h:91-99).
struct IntegrationConfiguration {
    bool iswithearth = false;
    std::array<double, 3> gravity{0, 0, 9.8}, iewn{0, 0, 0};
};

namespace MISC {
namespace detail {
inline gvx_ins_config to_c(const IntegrationConfiguration& c) {
    gvx_ins_config o;
    o.iswithearth = c.iswithearth ? 1 : 0;
    std::memcpy(o.gravity, c.gravity.data(), sizeof o.gravity);
    std::memcpy(o.iewn, c.iewn.data(), sizeof o.iewn);
    return o;
}
}  // namespace detail

// MISC::insMechanization(config, imu_pre, imu_cur, state) (misc.cc:174-229)
inline void insMechanization(Context& ctx, const IntegrationConfiguration& config, const IMU& imu_pre,
                             const IMU& imu_cur, IntegrationState& state) {
    const gvx_ins_config cfg = detail::to_c(config);
    const gvx_imu imu[2] = {imu_pre, imu_cur};
    const int32_t off[2] = {0, 2};
    const gvx_state s0 = gvx::detail::to_c(state);
    gvx_state out[2];
    check(gvx_ins_propagate(ctx.get(), &cfg, 1, imu, off, &s0, out), ctx.get(), "insMechanization");
    state = gvx::detail::from_c(out[1]);
}

// MISC::redoInsMechanization (misc.cc:231-284): same arguments and effect on the
// window, including the pop_front of the expired epochs.
inline void redoInsMechanization(Context& ctx, const IntegrationConfiguration& config,
                                 const IntegrationState& updated_state, size_t reserved_ins_num,
                                 std::deque<std::pair<IMU, IntegrationState>>& ins_windows) {
    std::vector<gvx_imu> imu;
    std::vector<gvx_state> st;
    imu.reserve(ins_windows.size());
    st.reserve(ins_windows.size());
    for (const auto& w : ins_windows) {
        imu.push_back(w.first);
        st.push_back(gvx::detail::to_c(w.second));
    }
    const gvx_ins_config cfg = detail::to_c(config);
    const gvx_state u = gvx::detail::to_c(updated_state);
    int32_t index = 0;
    check(gvx_redo_ins_mechanization(ctx.get(), &cfg, &u, (int32_t)imu.size(), imu.data(), st.data(), &index),
          ctx.get(), "redoInsMechanization");
    if (index == 0) return;  // "Failed to get right index in mechanization"
    for (size_t k = (size_t)index; k < ins_windows.size(); ++k) ins_windows[k].second = gvx::detail::from_c(st[k]);
    if ((size_t)index < reserved_ins_num) return;
    for (size_t k = 0; k < (size_t)index - reserved_ins_num; ++k) ins_windows.pop_front();
}

// MISC::getImuSeriesFromTo (misc.cc:330-384)
inline bool getImuSeriesFromTo(const std::deque<std::pair<IMU, IntegrationState>>& ins_windows, double start,
                               double end, std::vector<IMU>& series) {
    std::vector<gvx_imu> imu;
    imu.reserve(ins_windows.size());
    for (const auto& w : ins_windows) imu.push_back(w.first);
    series.assign(imu.size() + 2, IMU{});
    int32_t n = 0;
    const gvx_status s = gvx_imu_series_from_to(imu.data(), (int32_t)imu.size(), start, end, series.data(), &n);
    if (s == GVX_ERR_NOT_FOUND) {
        series.clear();
        return false;
    }
    check(s, nullptr, "getImuSeriesFromTo");
    series.resize((size_t)n);
    return true;
}
}  // namespace MISC

// GnssFactor (factors/gnss_factor.h:36-100): Evaluate with Ceres' signature;
// one factor per call here, gvx_small_factor_eval batches many.
class GnssFactor {
public:
    GnssFactor(Context& ctx, const std::array<double, 3>& blh, const std::array<double, 3>& std,
               const std::array<double, 3>& lever)
        : ctx_(ctx) {
        std::memcpy(c_, blh.data(), sizeof(double) * 3);
        std::memcpy(c_ + 3, std.data(), sizeof(double) * 3);
        std::memcpy(c_ + 6, lever.data(), sizeof(double) * 3);
    }
    bool Evaluate(double const* const* parameters, double* residuals, double** jacobians) const {
        const int32_t off = 0;
        double* jac = jacobians ? jacobians[0] : nullptr;
        check(gvx_small_factor_eval(ctx_.get(), GVX_FACTOR_GNSS, 1, c_, parameters[0], 7, &off, residuals, jac),
              ctx_.get(), "GnssFactor::Evaluate");
        return true;
    }

private:
    Context& ctx_;
    double c_[9];
};

class PreintegrationFactor {
public:
    explicit PreintegrationFactor(Preintegration& pre) : pre_(&pre) {}
    std::vector<int> parameter_block_sizes() const { return Preintegration::numBlocksParameters(); }
    int num_residuals() const { return Preintegration::numResiduals(); }
    bool Evaluate(const double* const* parameters, double* residuals, double** jacobians) const {
        pre_->evaluateAll(parameters, residuals, jacobians);
        return true;
    }

private:
    Preintegration* pre_;
};

// ReprojectionFactor (factors/reprojection_factor.h:35-161): SizedCostFunction
// <2, 7, 7, 7, 1, 1>, constructed from the two normalized points, their pixel
// velocities, time delays and the normalized-plane std.
class ReprojectionFactor {
public:
    using Vec3 = std::array<double, 3>;
    ReprojectionFactor(Context& ctx, const Vec3& pts0, const Vec3& pts1, const Vec3& vel0, const Vec3& vel1,
                       double td0, double td1, double std)
        : ctx_(&ctx) {
        std::memcpy(c_.pts0, pts0.data(), sizeof c_.pts0);
        std::memcpy(c_.pts1, pts1.data(), sizeof c_.pts1);
        std::memcpy(c_.vel0, vel0.data(), sizeof c_.vel0);
        std::memcpy(c_.vel1, vel1.data(), sizeof c_.vel1);
        c_.td0 = td0;
        c_.td1 = td1;
        c_.std = std;
    }
    std::vector<int> parameter_block_sizes() const { return {7, 7, 7, 1, 1}; }
    int num_residuals() const { return 2; }
    bool Evaluate(const double* const* parameters, double* residuals, double** jacobians) const {
        double params[23];
        std::memcpy(params, parameters[0], 7 * sizeof(double));
        std::memcpy(params + 7, parameters[1], 7 * sizeof(double));
        std::memcpy(params + 14, parameters[2], 7 * sizeof(double));
        params[21] = parameters[3][0];
        params[22] = parameters[4][0];
        const int32_t offs[5] = {0, 7, 14, 21, 22};
        double res[2], jac[46];
        check(gvx_reproj_eval(ctx_->get(), 1, &c_, params, 23, offs, res, jacobians ? jac : nullptr), ctx_->get(),
              "gvx_reproj_eval");
        if (residuals) std::memcpy(residuals, res, sizeof res);
        if (jacobians) {
            static const int cols[5] = {7, 7, 7, 1, 1}, start[5] = {0, 14, 28, 42, 44};
            for (int k = 0; k < 5; ++k)
                if (jacobians[k]) std::memcpy(jacobians[k], jac + start[k], sizeof(double) * 2 * cols[k]);
        }
        return true;
    }
    const gvx_reproj_const& constants() const { return c_; }

private:
    Context* ctx_;
    gvx_reproj_const c_{};
};

// ------------------------------------------------- two-phase factor set
// The EvaluationCallback pattern: register the window's
// parameter blocks and factors once; prepare() from
// ceres::EvaluationCallback::PrepareForEvaluation evaluates everything on the
// device; each CostFunction::Evaluate reads its slice (reentrant).
class FactorSet {
public:
    struct ReprojFactor {
        gvx_reproj_const c;
        int32_t blocks[5];  // pose_ref, pose_obs, ext, invdepth, td (indices into the block table)
    };
    struct PreintFactor {
        Preintegration* pre;  // integrated segment (its result and pn list are copied at construction)
        int32_t blocks[4];    // pose0, mix0, pose1, mix1
    };
    FactorSet(Context& ctx, const std::vector<double*>& blocks, const std::vector<int32_t>& sizes,
              const std::vector<ReprojFactor>& reproj, const std::vector<PreintFactor>& preint)
        : ctx_(&ctx) {
        std::vector<gvx_reproj_const> rc;
        std::vector<int32_t> rb, pb, pn_off;
        for (const auto& f : reproj) {
            rc.push_back(f.c);
            rb.insert(rb.end(), f.blocks, f.blocks + 5);
        }
        std::vector<gvx_preint_result> pre;
        std::vector<double> pn;
        for (const auto& f : preint) {
            pre.push_back(f.pre->raw());
            pn_off.push_back((int32_t)(pn.size() / 4));
            const std::vector<double>& l = f.pre->pn();
            pn.insert(pn.end(), l.begin(), l.end());
            pb.insert(pb.end(), f.blocks, f.blocks + 4);
        }
        std::vector<const double*> cb(blocks.begin(), blocks.end());
        check(gvx_factor_set_create(ctx.get(), (int32_t)cb.size(), cb.data(), sizes.data(), (int32_t)rc.size(),
                                    rc.data(), rb.data(), (int32_t)pre.size(), pre.data(), pn.data(),
                                    (int32_t)(pn.size() / 4), pn_off.data(), pb.data(), &set_),
              ctx.get(), "gvx_factor_set_create");
    }
    ~FactorSet() { gvx_factor_set_destroy(set_); }
    FactorSet(const FactorSet&) = delete;
    FactorSet& operator=(const FactorSet&) = delete;

    void prepare(bool jacobians) { check(gvx_factors_prepare(set_, jacobians ? 1 : 0), ctx_->get(), "prepare"); }
    bool readReprojection(int i, double* residuals, double** jacobians) const {
        return gvx_factor_read_reproj(set_, i, residuals, jacobians) == GVX_OK;
    }
    bool readPreintegration(int i, double* residuals, double** jacobians) const {
        return gvx_factor_read_preint(set_, i, residuals, jacobians) == GVX_OK;
    }

private:
    Context* ctx_;
    gvx_factor_set* set_ = nullptr;
};

// ------------------------------------------------------- marginalisation
constexpr int POSE_LOCAL_SIZE = 6, POSE_GLOBAL_SIZE = 7;  // factors/residual_block_info.h:26-27

// ResidualBlockInfo (factors/residual_block_info.h:32-120): a cost function with
// Ceres' Evaluate signature, its parameter blocks and which of them are
// marginalized.  huber > 0 stands for a ceres::HuberLoss(huber) (the reference
// passes nullptr; the device applies ResidualBlockInfo::Evaluate's corrector).
class ResidualBlockInfo {
public:
    using CostFunction = std::function<bool(double const* const*, double*, double**)>;
    ResidualBlockInfo(CostFunction cost_function, int num_residuals, std::vector<int> block_sizes, double huber,
                      std::vector<double*> parameter_blocks, std::vector<int> marg_para_index)
        : cost_(std::move(cost_function)), nres_(num_residuals), sizes_(std::move(block_sizes)), huber_(huber),
          blocks_(std::move(parameter_blocks)), marg_(std::move(marg_para_index)) {}
    // residuals then the row-major Jacobian blocks, contiguous (the gvx_marginalize layout)
    void Evaluate() {
        size_t total = (size_t)nres_;
        for (int s : sizes_) total += (size_t)nres_ * s;
        data_.assign(total, 0.0);
        std::vector<double*> jac(sizes_.size());
        size_t o = (size_t)nres_;
        for (size_t i = 0; i < sizes_.size(); ++i) {
            jac[i] = data_.data() + o;
            o += (size_t)nres_ * sizes_[i];
        }
        if (!cost_(blocks_.data(), data_.data(), jac.data()))
            throw Error(GVX_ERR_INVALID, "ResidualBlockInfo::Evaluate: cost function failed");
    }
    const std::vector<int>& parameterBlockSizes() const { return sizes_; }
    const std::vector<double*>& parameterBlocks() const { return blocks_; }
    const std::vector<int>& marginalizationParametersIndex() const { return marg_; }
    int numResiduals() const { return nres_; }
    double huber() const { return huber_; }
    const std::vector<double>& data() const { return data_; }

private:
    CostFunction cost_;
    int nres_;
    std::vector<int> sizes_;
    double huber_;
    std::vector<double*> blocks_;
    std::vector<int> marg_;
    std::vector<double> data_;
};

// MarginalizationInfo (factors/marginalization_info.h:31-316): the same calls
// and the same std::unordered_map bookkeeping (so the block order that
// updateParameterBlocksIndex derives from the map iteration is the reference's);
// constructEquation / schurElimination / linearization run on the device
// through gvx_marginalize.  linearizedJacobians() is column-major r x r.
class MarginalizationInfo {
public:
    explicit MarginalizationInfo(Context& ctx) : ctx_(&ctx) {}
    MarginalizationInfo(const MarginalizationInfo&) = delete;
    MarginalizationInfo& operator=(const MarginalizationInfo&) = delete;

    bool isValid() const { return isvalid_; }
    static int localSize(int size) { return size == POSE_GLOBAL_SIZE ? POSE_LOCAL_SIZE : size; }
    static int globalSize(int size) { return size == POSE_LOCAL_SIZE ? POSE_GLOBAL_SIZE : size; }

    void addResidualBlockInfo(const std::shared_ptr<ResidualBlockInfo>& blockinfo) {
        factors_.push_back(blockinfo);
        const auto& parameter_blocks = blockinfo->parameterBlocks();
        const auto& block_sizes = blockinfo->parameterBlockSizes();
        for (size_t k = 0; k < parameter_blocks.size(); k++)
            parameter_block_size_[parameters_ids_[reinterpret_cast<long>(parameter_blocks[k])]] = block_sizes[k];
        for (int index : blockinfo->marginalizationParametersIndex())
            parameter_block_index_[parameters_ids_[reinterpret_cast<long>(parameter_blocks[index])]] = 0;
    }
    void updateParamtersIds(const std::unordered_map<long, long>& parameters_ids) { parameters_ids_ = parameters_ids; }

    bool marginalization() {
        if (!updateParameterBlocksIndex()) {
            isvalid_ = false;
            factors_.clear();
            return false;
        }
        preMarginalization();
        // the residual blocks in the gvx_marginalize layout, blocks numbered by id
        std::unordered_map<long, int32_t> slot;
        std::vector<int32_t> size, index;
        for (const auto& b : parameter_block_index_) {
            slot[b.first] = (int32_t)size.size();
            size.push_back(parameter_block_size_[b.first]);
            index.push_back(b.second);
        }
        std::vector<int32_t> nres, blk_off{0}, blk;
        std::vector<int64_t> res_off, jac_off;
        std::vector<double> data, loss;
        bool any_loss = false;
        for (const auto& f : factors_) {
            nres.push_back(f->numResiduals());
            for (double* p : f->parameterBlocks()) blk.push_back(slot.at(parameters_ids_[reinterpret_cast<long>(p)]));
            blk_off.push_back((int32_t)blk.size());
            res_off.push_back((int64_t)data.size());
            jac_off.push_back((int64_t)data.size() + f->numResiduals());
            data.insert(data.end(), f->data().begin(), f->data().end());
            loss.push_back(f->huber());
            any_loss |= f->huber() > 0;
        }
        const int r = remained_size_;
        linearized_jacobians_.assign((size_t)r * r, 0.0);
        linearized_residuals_.assign((size_t)r, 0.0);
        int32_t info[2] = {0, 0};
        check(gvx_marginalize(ctx_->get(), (int32_t)factors_.size(), nres.data(), blk_off.data(), blk.data(),
                              res_off.data(), jac_off.data(), data.data(), (int64_t)data.size(),
                              any_loss ? loss.data() : nullptr, (int32_t)size.size(), size.data(), index.data(),
                              marginalized_size_, local_size_, linearized_jacobians_.data(),
                              linearized_residuals_.data(), nullptr, nullptr, nullptr, info),
              ctx_->get(), "MarginalizationInfo::marginalization");
        factors_.clear();
        return true;
    }

    std::vector<double*> getParamterBlocks(std::unordered_map<long, double*>& address) {
        std::vector<double*> remained_block_addr;
        remained_block_data_.clear();
        remained_block_index_.clear();
        remained_block_size_.clear();
        for (const auto& block : parameter_block_index_) {
            if (block.second >= marginalized_size_) {
                remained_block_data_.push_back(parameter_block_data_[block.first].data());
                remained_block_size_.push_back(parameter_block_size_[block.first]);
                remained_block_index_.push_back(parameter_block_index_[block.first]);
                remained_block_addr.push_back(address[block.first]);
            }
        }
        return remained_block_addr;
    }
    const std::vector<double>& linearizedJacobians() const { return linearized_jacobians_; }
    const std::vector<double>& linearizedResiduals() const { return linearized_residuals_; }
    int marginalizedSize() const { return marginalized_size_; }
    int remainedSize() const { return remained_size_; }
    const std::vector<int>& remainedBlockSize() const { return remained_block_size_; }
    const std::vector<int>& remainedBlockIndex() const { return remained_block_index_; }
    const std::vector<double*>& remainedBlockData() const { return remained_block_data_; }
    // the local index updateParameterBlocksIndex gave the block with this id (-1: none)
    int blockIndex(long id) const {
        auto it = parameter_block_index_.find(id);
        return it == parameter_block_index_.end() ? -1 : it->second;
    }

private:
    bool updateParameterBlocksIndex() {
        int index = 0;
        for (auto& block : parameter_block_index_) {
            block.second = index;
            index += localSize(parameter_block_size_[block.first]);
        }
        marginalized_size_ = index;
        for (const auto& block : parameter_block_size_) {
            if (parameter_block_index_.find(block.first) == parameter_block_index_.end()) {
                parameter_block_index_[block.first] = index;
                index += localSize(block.second);
            }
        }
        remained_size_ = index - marginalized_size_;
        local_size_ = index;
        return marginalized_size_ > 0;
    }
    void preMarginalization() {
        for (const auto& factor : factors_) {
            factor->Evaluate();
            const auto& block_sizes = factor->parameterBlockSizes();
            for (size_t k = 0; k < block_sizes.size(); k++) {
                const long id = parameters_ids_[reinterpret_cast<long>(factor->parameterBlocks()[k])];
                if (parameter_block_data_.find(id) == parameter_block_data_.end()) {
                    const double* p = factor->parameterBlocks()[k];
                    parameter_block_data_[id].assign(p, p + block_sizes[k]);
                }
            }
        }
    }

    Context* ctx_;
    std::unordered_map<long, long> parameters_ids_;
    std::unordered_map<long, int> parameter_block_size_;
    std::unordered_map<long, int> parameter_block_index_;
    std::unordered_map<long, std::vector<double>> parameter_block_data_;
    std::vector<int> remained_block_size_, remained_block_index_;
    std::vector<double*> remained_block_data_;
    int marginalized_size_ = 0, remained_size_ = 0, local_size_ = 0;
    std::vector<std::shared_ptr<ResidualBlockInfo>> factors_;
    std::vector<double> linearized_jacobians_, linearized_residuals_;
    bool isvalid_ = true;
};

// MarginalizationFactor::Evaluate (factors/marginalization_factor.h:54-110) on
// the device from the previous MarginalizationInfo's J0 / e0 / x0.
class MarginalizationFactor {
public:
    MarginalizationFactor(Context& ctx, std::shared_ptr<MarginalizationInfo> info) : ctx_(&ctx), info_(std::move(info)) {
        const auto& sz = info_->remainedBlockSize();
        int32_t o = 0;
        for (size_t b = 0; b < sz.size(); ++b) {
            size_.push_back(sz[b]);
            index_.push_back(info_->remainedBlockIndex()[b] - info_->marginalizedSize());
            xoff_.push_back(o);
            x0_.insert(x0_.end(), info_->remainedBlockData()[b], info_->remainedBlockData()[b] + sz[b]);
            o += sz[b];
        }
    }
    std::vector<int> parameter_block_sizes() const { return std::vector<int>(size_.begin(), size_.end()); }
    int num_residuals() const { return info_->remainedSize(); }
    bool Evaluate(double const* const* parameters, double* residuals, double** jacobians) const {
        const int r = info_->remainedSize();
        std::vector<double> x;
        for (size_t b = 0; b < size_.size(); ++b) x.insert(x.end(), parameters[b], parameters[b] + size_[b]);
        std::vector<double> jac(jacobians ? (size_t)r * x.size() : 0);
        check(gvx_marg_factor_eval(ctx_->get(), r, (int32_t)size_.size(), size_.data(), index_.data(), xoff_.data(),
                                   (int32_t)x.size(), x0_.data(), x.data(), info_->linearizedJacobians().data(),
                                   info_->linearizedResiduals().data(), residuals, jacobians ? jac.data() : nullptr),
              ctx_->get(), "MarginalizationFactor::Evaluate");
        if (jacobians)
            for (size_t b = 0; b < size_.size(); ++b)
                if (jacobians[b])
                    std::memcpy(jacobians[b], jac.data() + (size_t)r * xoff_[b], sizeof(double) * r * size_[b]);
        return true;
    }

private:
    Context* ctx_;
    std::shared_ptr<MarginalizationInfo> info_;
    std::vector<int32_t> size_, index_, xoff_;
    std::vector<double> x0_;
};

}  // namespace gvx
