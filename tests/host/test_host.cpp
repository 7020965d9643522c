// C++ host-mirror check (tests/test_host_cpp.py builds and drives this).
//   test_host nodev       -> constructing gvx::Context without a device must throw
//                            gvx::Error(GVX_ERR_NO_DEVICE) (no CPU fallback)
//   test_host run <dir>   -> reads inputs written by the test, runs the reference-
//                            shaped calls through include/gvx/gvx.hpp, writes outputs
#include <gvx/gvx.hpp>

#include <cstdio>
#include <fstream>
#include <string>
#include <deque>
#include <vector>

template <class T>
static std::vector<T> readf(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw std::runtime_error("cannot read " + path);
    const size_t bytes = (size_t)f.tellg();
    std::vector<T> v(bytes / sizeof(T));
    f.seekg(0);
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
    return v;
}
template <class T>
static void writef(const std::string& path, const T* p, size_t n) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), (std::streamsize)(n * sizeof(T)));
}

static gvx::IntegrationState state_from(const double* d) {
    gvx::IntegrationState s;
    s.time = d[0];
    for (int k = 0; k < 3; ++k) s.p[k] = d[1 + k];
    for (int k = 0; k < 4; ++k) s.q[k] = d[4 + k];
    for (int k = 0; k < 3; ++k) s.v[k] = d[8 + k], s.bg[k] = d[11 + k], s.ba[k] = d[14 + k];
    return s;
}
static void state_to(const gvx::IntegrationState& s, double* d) {
    d[0] = s.time;
    for (int k = 0; k < 3; ++k) d[1 + k] = s.p[k];
    for (int k = 0; k < 4; ++k) d[4 + k] = s.q[k];
    for (int k = 0; k < 3; ++k) d[8 + k] = s.v[k], d[11 + k] = s.bg[k], d[14 + k] = s.ba[k];
}

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "";
    if (mode == "nodev") {
        try {
            gvx::Context c(0);
            std::printf("HAVE_DEVICE\n");
            return 0;
        } catch (const gvx::Error& e) {
            std::printf("ERROR %d %s\n", (int)e.status(), e.what());
            return e.status() == GVX_ERR_NO_DEVICE ? 0 : 1;
        }
    }
    if (mode != "run" || argc < 3) {
        std::fprintf(stderr, "usage: test_host nodev | run <dir>\n");
        return 2;
    }
    const std::string d = std::string(argv[2]) + "/";
    const auto meta = readf<int32_t>(d + "meta.bin");  // w h n variant
    const int w = meta[0], h = meta[1], n = meta[2];
    const auto I = readf<uint8_t>(d + "I.bin"), J = readf<uint8_t>(d + "J.bin");
    const auto prev = readf<gvx::Point2f>(d + "prev.bin"), init = readf<gvx::Point2f>(d + "init.bin");
    if ((int)prev.size() != n || (int)init.size() != n) throw std::runtime_error("point count mismatch");
    gvx::Context ctx(0);
    gvx::GpuFrame fI(ctx, I.data(), w, h, w), fJ(ctx, J.data(), w, h, w);

    // cv::calcOpticalFlowPyrLK as called at tracking.cc:385
    std::vector<gvx::Point2f> next = init;
    std::vector<uint8_t> status;
    std::vector<float> err;
    gvx::calcOpticalFlowPyrLK(fI, fJ, prev, next, status, err, gvx::Size{21, 21}, 3,
                              gvx::TermCriteria{gvx::TermCriteria::COUNT + gvx::TermCriteria::EPS, 30, 0.01},
                              gvx::OPTFLOW_USE_INITIAL_FLOW);
    writef(d + "lk_next.bin", next.data(), next.size());
    writef(d + "lk_status.bin", status.data(), status.size());
    writef(d + "lk_err.bin", err.data(), err.size());

    // fused fwd/bwd/FB + reduceVector (tracking.cc:380-408)
    gvx::TrackFB fb = gvx::trackFB(fI, fJ, prev, init, w, h);
    writef(d + "fb_next.bin", fb.next.data(), fb.next.size());
    writef(d + "fb_back.bin", fb.back.data(), fb.back.size());
    writef(d + "fb_keep.bin", fb.keep.data(), fb.keep.size());
    writef(d + "fb_kept.bin", fb.kept.data(), fb.kept.size());
    std::vector<gvx::Point2f> reduced = fb.next;
    gvx::reduceVector(reduced, fb.keep);
    writef(d + "fb_reduced.bin", reduced.data(), reduced.size());

    // featuresDetection on the first frame, no tracked points
    std::vector<gvx::Point2f> corners;
    gvx::DetectParams dp;
    const bool ran = gvx::featuresDetection(fI, {}, {}, false, 0, dp, corners);
    if (!ran) corners.clear();
    writef(d + "det.bin", corners.data(), corners.size());

    // Tracking::preprocessing: clahe_ = cv::createCLAHE(3.0, Size(21, 21)) (tracking.cc:63),
    // apply (:139); the one-call form must give the same equalised frame
    gvx::CLAHE clahe = gvx::createCLAHE(ctx, 3.0, gvx::Size{21, 21});
    std::vector<uint8_t> eq(I.size()), eq2(I.size());
    clahe.apply(I.data(), w, h, w, eq.data(), w);
    double hmean = 0;
    gvx::GpuFrame fP = gvx::preprocessFrame(clahe, I.data(), w, h, w, eq2.data(), &hmean);
    if (eq != eq2 || fP.width() != w) {
        std::printf("FAIL preprocessFrame\n");
        return 1;
    }
    writef(d + "clahe.bin", eq.data(), eq.size());
    writef(d + "hist_mean.bin", &hmean, 1);

    // Camera point operations (camera.cc, tracking.cc:366-544, :861-871)
    const auto cv = readf<double>(d + "cam.bin");  // fx fy cx cy skew k1 k2 p1 p2 k3
    const gvx_camera gc{cv[0], cv[1], cv[2], cv[3], cv[4], cv[5], cv[6], cv[7], cv[8], cv[9], w, h};
    gvx::Camera cam(ctx, gc);
    std::vector<gvx::Point2f> und = prev, dis = prev;
    cam.undistortPoints(und);
    cam.distortPoints(dis);
    const auto rot = readf<double>(d + "rot.bin");  // r_cur_pre, R0, R1
    std::array<double, 9> Rc, R0, R1;
    for (int k = 0; k < 9; ++k) Rc[k] = rot[k], R0[k] = rot[9 + k], R1[k] = rot[18 + k];
    const auto pred = cam.predictRotated(Rc, prev);
    const auto vel = cam.velocity(prev, init, 0.05);
    const auto par = cam.keyPointParallax(R0, R1, prev, init);
    writef(d + "cam_undist.bin", und.data(), und.size());
    writef(d + "cam_dist.bin", dis.data(), dis.size());
    writef(d + "cam_pred.bin", pred.data(), pred.size());
    writef(d + "cam_vel.bin", vel.data(), vel.size());
    writef(d + "cam_par.bin", par.data(), par.size());

    // preintegration: constructor(imu0) + addNewImu per sample, then reintegration
    const auto imu = readf<gvx::IMU>(d + "imu.bin");
    const auto st = readf<double>(d + "state.bin");
    const auto prm = readf<double>(d + "prm.bin");
    gvx::IntegrationParameters ip;
    ip.acc_vrw = prm[0], ip.gyr_arw = prm[1], ip.gyr_bias_std = prm[2], ip.acc_bias_std = prm[3];
    ip.corr_time = prm[4], ip.gravity = prm[5];
    gvx::Preintegration pre(ctx, (gvx::Preintegration::Variant)meta[3], ip, imu[0], state_from(st.data()));
    for (size_t k = 1; k < imu.size(); ++k) pre.addNewImu(imu[k]);
    double out[2 * 17 + 1];
    state_to(pre.deltaState(), out);
    state_to(pre.currentState(), out + 17);
    out[34] = pre.deltaTime();
    writef(d + "pre_state.bin", out, 35);
    writef(d + "pre_pn.bin", pre.pn().data(), pre.pn().size());

    // PreintegrationFactor::Evaluate with all four Jacobian blocks
    const auto fp = readf<double>(d + "fparams.bin");
    const double* blocks[4] = {fp.data(), fp.data() + 7, fp.data() + 16, fp.data() + 23};
    std::vector<double> res(15), j0(105), j1(135), j2(105), j3(135);
    double* jac[4] = {j0.data(), j1.data(), j2.data(), j3.data()};
    gvx::PreintegrationFactor pf(pre);
    pf.Evaluate(blocks, res.data(), jac);
    std::vector<double> all(res);
    for (auto* v : {&j0, &j1, &j2, &j3}) all.insert(all.end(), v->begin(), v->end());
    writef(d + "pf.bin", all.data(), all.size());

    // reintegration from a modified state (bias step, as after an LM update)
    gvx::IntegrationState s2 = state_from(st.data());
    s2.bg[0] += 1e-3;
    s2.ba[2] -= 2e-3;
    pre.reintegration(s2);
    state_to(pre.deltaState(), out);
    state_to(pre.currentState(), out + 17);
    out[34] = pre.deltaTime();
    writef(d + "pre_state2.bin", out, 35);

    // ReprojectionFactor::Evaluate
    const auto rc = readf<double>(d + "rconst.bin");
    const auto rp = readf<double>(d + "rparams.bin");
    gvx::ReprojectionFactor rf(ctx, {rc[0], rc[1], rc[2]}, {rc[3], rc[4], rc[5]}, {rc[6], rc[7], rc[8]},
                               {rc[9], rc[10], rc[11]}, rc[12], rc[13], rc[14]);
    const double* rb[5] = {rp.data(), rp.data() + 7, rp.data() + 14, rp.data() + 21, rp.data() + 22};
    std::vector<double> rr(2 + 46);
    double* rj[5] = {rr.data() + 2, rr.data() + 16, rr.data() + 30, rr.data() + 44, rr.data() + 46};
    rf.Evaluate(rb, rr.data(), rj);
    writef(d + "rf.bin", rr.data(), rr.size());

    // two-phase FactorSet over the same blocks (EvaluationCallback pattern): the
    // reprojection factor and the (reintegrated) preintegration factor; every
    // slice must equal the single-factor Evaluate
    std::vector<double> b_pose_ref(rp.begin(), rp.begin() + 7), b_pose_obs(rp.begin() + 7, rp.begin() + 14),
        b_ext(rp.begin() + 14, rp.begin() + 21), b_inv(1, rp[21]), b_td(1, rp[22]);
    std::vector<double> b_p0(fp.begin(), fp.begin() + 7), b_m0(fp.begin() + 7, fp.begin() + 16),
        b_p1(fp.begin() + 16, fp.begin() + 23), b_m1(fp.begin() + 23, fp.begin() + 32);
    std::vector<double*> tbl = {b_pose_ref.data(), b_pose_obs.data(), b_ext.data(), b_inv.data(), b_td.data(),
                                b_p0.data(), b_m0.data(), b_p1.data(), b_m1.data()};
    std::vector<int32_t> tsz = {7, 7, 7, 1, 1, 7, 9, 7, 9};
    gvx::FactorSet::ReprojFactor frp{rf.constants(), {0, 1, 2, 3, 4}};
    gvx::FactorSet::PreintFactor fpf{&pre, {5, 6, 7, 8}};
    gvx::FactorSet fs(ctx, tbl, tsz, {frp}, {fpf});
    fs.prepare(true);
    std::vector<double> sr(2 + 46);
    double* sj[5] = {sr.data() + 2, sr.data() + 16, sr.data() + 30, sr.data() + 44, sr.data() + 46};
    if (!fs.readReprojection(0, sr.data(), sj) || sr != rr) {
        std::printf("FAIL factor set reprojection\n");
        return 1;
    }
    gvx::PreintegrationFactor pf2(pre);
    std::vector<double> r2(15), k0(105), k1(135), k2(105), k3(135), q(15), q0(105), q1(135), q2(105), q3(135);
    double* kj[4] = {k0.data(), k1.data(), k2.data(), k3.data()};
    double* qj[4] = {q0.data(), nullptr, q2.data(), q3.data()};  // a null block is skipped
    pf2.Evaluate(blocks, r2.data(), kj);
    if (!fs.readPreintegration(0, q.data(), qj) || q != r2 || q0 != k0 || q2 != k2 || q3 != k3) {
        std::printf("FAIL factor set preintegration\n");
        return 1;
    }
    // MISC::redoInsMechanization on a window of the IMU records with the state as
    // its states, updated at imu[20].time + 0.0021 (interpolation split)
    {
        gvx::IntegrationConfiguration cfg;
        cfg.iswithearth = meta[3] == GVX_PREINT_EARTH;
        cfg.gravity = {0, 0, prm[5]};
        cfg.iewn = {1e-5, 2e-5, 6e-5};
        std::deque<std::pair<gvx::IMU, gvx::IntegrationState>> win;
        for (const auto& m : imu) win.emplace_back(m, state_from(st.data()));
        gvx::IntegrationState upd = state_from(st.data());
        upd.time = imu[20].time + 0.0021;
        gvx::MISC::redoInsMechanization(ctx, cfg, upd, 8, win);
        std::vector<double> o;
        o.push_back((double)win.size());
        for (const auto& w : win) {
            double t[17];
            state_to(w.second, t);
            o.insert(o.end(), t, t + 17);
        }
        writef(d + "ins_redo.bin", o.data(), o.size());
        std::vector<gvx::IMU> series;
        if (!gvx::MISC::getImuSeriesFromTo(win, imu[25].time + 0.001, imu[40].time + 0.003, series)) {
            std::printf("FAIL getImuSeriesFromTo\n");
            return 1;
        }
        writef(d + "ins_series.bin", series.data(), series.size());
        gvx::GnssFactor gf(ctx, {1.0, 2.0, 3.0}, {0.02, 0.03, 0.05}, {0.1, -0.2, 0.3});
        const double* pp[1] = {fp.data()};
        double gres[3], gjac[21];
        double* gj[1] = {gjac};
        gf.Evaluate(pp, gres, gj);
        writef(d + "gnss.bin", gres, 3);
        writef(d + "gnss_jac.bin", gjac, 21);
    }
    std::printf("OK\n");
    return 0;
}
