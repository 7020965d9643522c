"""Synthetic inputs for the KLT path.

The KAIST urban38/39 bags are not available offline, so frame pairs of the same
geometry are synthesised: band-limited noise (Gaussian-blurred uniform noise,
sigma 1.5 px, contrast-stretched to 0..255) plus random rectangles; the second
frame is the first warped by a sub-pixel similarity (tx, ty ~ U(-6, 6) px,
rotation ~ U(-1, 1) deg, scale 1 +- 0.01) with bilinear resampling plus +-2 LSB
noise.  Points are picked from a min-eigenvalue score on the reference block grid
(numpy only -- no dependency on the oracle) and topped up with random interior
points; the initial flow is the true warp plus U(-1, 1) px.
"""
from __future__ import annotations

import numpy as np

SEED = 20261015


def _gauss_kernel(sigma: float) -> np.ndarray:
    r = int(np.ceil(3 * sigma))
    x = np.arange(-r, r + 1, dtype=np.float64)
    k = np.exp(-0.5 * (x / sigma) ** 2)
    return k / k.sum()


def _blur(img: np.ndarray, sigma: float) -> np.ndarray:
    k = _gauss_kernel(sigma)
    r = len(k) // 2
    p = np.pad(img, ((0, 0), (r, r)), mode="reflect")
    out = np.zeros_like(img)
    for i, kv in enumerate(k):
        out += kv * p[:, i:i + img.shape[1]]
    p = np.pad(out, ((r, r), (0, 0)), mode="reflect")
    out2 = np.zeros_like(img)
    for i, kv in enumerate(k):
        out2 += kv * p[i:i + img.shape[0], :]
    return out2


def make_image(w: int, h: int, rng: np.random.Generator) -> np.ndarray:
    """Band-limited noise plus random rectangles, u8 h x w."""
    base = _blur(rng.uniform(0.0, 1.0, size=(h, w)), 1.5)
    lo, hi = np.percentile(base, [1, 99])
    img = np.clip((base - lo) / max(hi - lo, 1e-9), 0, 1) * 255.0
    nrect = max(4, (w * h) // 40000)
    for _ in range(nrect):
        rw, rh = rng.integers(8, max(9, w // 8)), rng.integers(8, max(9, h // 8))
        x0, y0 = rng.integers(0, w - rw), rng.integers(0, h - rh)
        val = rng.uniform(0, 255)
        img[y0:y0 + rh, x0:x0 + rw] = 0.6 * img[y0:y0 + rh, x0:x0 + rw] + 0.4 * val
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def similarity(rng: np.random.Generator, w: int, h: int):
    tx, ty = rng.uniform(-6, 6, size=2)
    th = np.deg2rad(rng.uniform(-1, 1))
    s = 1.0 + rng.uniform(-0.01, 0.01)
    cx, cy = w / 2.0, h / 2.0
    c, sn = s * np.cos(th), s * np.sin(th)
    # x' = A (x - c) + c + t
    A = np.array([[c, -sn], [sn, c]])
    t = np.array([cx + tx, cy + ty]) - A @ np.array([cx, cy])
    return A, t


def warp(img: np.ndarray, A: np.ndarray, t: np.ndarray, rng: np.random.Generator) -> np.ndarray:
    """J(x') = I(A^-1 (x' - t)) bilinear, +-2 LSB noise."""
    h, w = img.shape
    Ai = np.linalg.inv(A)
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float64)
    sx = Ai[0, 0] * (xs - t[0]) + Ai[0, 1] * (ys - t[1])
    sy = Ai[1, 0] * (xs - t[0]) + Ai[1, 1] * (ys - t[1])
    sx = np.clip(sx, 0, w - 1.001)
    sy = np.clip(sy, 0, h - 1.001)
    x0 = np.floor(sx).astype(np.int64)
    y0 = np.floor(sy).astype(np.int64)
    fx, fy = sx - x0, sy - y0
    f = img.astype(np.float64)
    v = (f[y0, x0] * (1 - fx) * (1 - fy) + f[y0, x0 + 1] * fx * (1 - fy) +
         f[y0 + 1, x0] * (1 - fx) * fy + f[y0 + 1, x0 + 1] * fx * fy)
    v += rng.integers(-2, 3, size=v.shape)
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def min_eig_score(img: np.ndarray) -> np.ndarray:
    f = img.astype(np.float64)
    gx = np.zeros_like(f)
    gy = np.zeros_like(f)
    gx[:, 1:-1] = f[:, 2:] - f[:, :-2]
    gy[1:-1, :] = f[2:, :] - f[:-2, :]
    a, b, c = _blur(gx * gx, 1.0), _blur(gx * gy, 1.0), _blur(gy * gy, 1.0)
    return 0.5 * (a + c) - np.sqrt(0.25 * (a - c) ** 2 + b * b)


def pick_points(img: np.ndarray, n: int, rng: np.random.Generator, block: float = 200.0,
                margin: int = 12) -> np.ndarray:
    """Up to ceil(n / blocks) strongest well-separated corners per block of the
    reference grid (tracking.cc:65-85), topped up with random interior points."""
    h, w = img.shape
    score = min_eig_score(img)
    bc, br = max(1, int(round(w / block))), max(1, int(round(h / block)))
    per = int(np.ceil(n / (bc * br)))
    cw, ch = w // bc, h // br
    pts = []
    for r in range(br):
        for c in range(bc):
            x0, y0 = c * cw, r * ch
            sub = score[y0:y0 + ch, x0:x0 + cw].copy()
            sub[:margin, :] = -1
            sub[-margin:, :] = -1
            sub[:, :margin] = -1
            sub[:, -margin:] = -1
            for _ in range(per):
                k = int(np.argmax(sub))
                yy, xx = divmod(k, sub.shape[1])
                if sub[yy, xx] <= 0:
                    break
                pts.append((x0 + xx + rng.uniform(-0.5, 0.5), y0 + yy + rng.uniform(-0.5, 0.5)))
                sub[max(0, yy - 20):yy + 21, max(0, xx - 20):xx + 21] = -1
    pts = pts[:n]
    while len(pts) < n:
        pts.append((rng.uniform(margin, w - margin), rng.uniform(margin, h - margin)))
    return np.asarray(pts, dtype=np.float32)


def make_pair(w: int, h: int, n: int, seed: int = SEED):
    """One synthetic frame pair: (I, J, prev_xy[n,2] f32, init_xy[n,2] f32, truth[n,2])."""
    rng = np.random.default_rng(seed)
    I = make_image(w, h, rng)
    A, t = similarity(rng, w, h)
    J = warp(I, A, t, rng)
    prev = pick_points(I, n, rng)
    truth = (prev.astype(np.float64) @ A.T + t).astype(np.float32)
    init = (truth + rng.uniform(-1, 1, size=truth.shape)).astype(np.float32)
    return I, J, prev, init, truth


def make_batch(n_pairs: int, w: int, h: int, n: int, seed: int = SEED, distinct: int | None = None):
    """n_pairs pairs with per-pair seeds seed+i.  If `distinct` is given only that
    many distinct pairs are synthesised and tiled (keeps generation time bounded
    for large benchmark batches; every pair is still processed in full)."""
    m = n_pairs if distinct is None else max(1, min(distinct, n_pairs))
    I = np.empty((m, h, w), np.uint8)
    J = np.empty((m, h, w), np.uint8)
    P = np.empty((m, n, 2), np.float32)
    Q = np.empty((m, n, 2), np.float32)
    for i in range(m):
        I[i], J[i], P[i], Q[i], _ = make_pair(w, h, n, seed + i)
    if m != n_pairs:
        idx = np.arange(n_pairs) % m
        I, J, P, Q = I[idx], J[idx], P[idx], Q[idx]
    return I, J, P, Q


SEQ_VEL = (1.6, 0.5)  # px / frame


def camera_path(t: int):
    """Similarity of frame t of a synthetic sequence: the camera drifts over a
    textured plane at SEQ_VEL px/frame with a slow roll (+-1.2 deg) and zoom
    (+-2 %).  Returns (A, c): texture point = A @ (x - centre) + c."""
    th = np.deg2rad(1.2) * np.sin(2 * np.pi * t / 700.0)
    s = 1.0 + 0.02 * np.sin(2 * np.pi * t / 900.0 + 1.0)
    A = s * np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    return A, np.array([SEQ_VEL[0] * t, SEQ_VEL[1] * t])


def make_sequence(w: int, h: int, n_frames: int, device, seed: int = SEED, tex=None):
    """configs[4]: n_frames u8 frames [F, h, w] of a moving camera
    over one band-limited texture, rendered on `device` with bilinear resampling
    (torch.nn.functional.grid_sample) plus +-2 LSB noise.  Returns the frame
    tensor and the texture (numpy) it was rendered from."""
    import torch
    import torch.nn.functional as F
    rng = np.random.default_rng(seed)
    tw, th_ = int(w + SEQ_VEL[0] * n_frames) + 1000, int(h + SEQ_VEL[1] * n_frames) + 600
    if tex is None:
        tex = make_image(tw, th_, rng)
    T = torch.from_numpy(tex).to(device=device, dtype=torch.float32)[None, None]
    out = torch.empty((n_frames, h, w), dtype=torch.uint8, device=device)
    ys, xs = torch.meshgrid(torch.arange(h, device=device, dtype=torch.float64),
                            torch.arange(w, device=device, dtype=torch.float64), indexing="ij")
    xc, yc = xs - (w - 1) / 2.0, ys - (h - 1) / 2.0
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    origin = np.array([(w - 1) / 2.0 + 500.0, (h - 1) / 2.0 + 300.0])
    for t in range(n_frames):
        A, c = camera_path(t)
        c = c + origin
        tx = A[0, 0] * xc + A[0, 1] * yc + c[0]
        ty = A[1, 0] * xc + A[1, 1] * yc + c[1]
        grid = torch.stack([2 * tx / (tw - 1) - 1, 2 * ty / (th_ - 1) - 1], dim=-1)[None].to(torch.float32)
        v = F.grid_sample(T, grid, mode="bilinear", padding_mode="border", align_corners=True)[0, 0]
        v = v + torch.randint(-2, 3, v.shape, device=device, generator=gen, dtype=torch.int32).to(v.dtype)
        out[t] = v.round().clamp(0, 255).to(torch.uint8)
        if (t & 63) == 63 and out.is_cuda:
            # bound the un-synchronised dispatch backlog (about 15 kernels a frame):
            # rocprofv3's counter collection fails on tens of thousands of queued
            # dispatches (a queue abort in r05_m1, a host SIGSEGV in r06_d1)
            torch.cuda.synchronize(out.device)
    return out, tex


def two_view_scene(n, outlier_frac=0.2, noise_px=0.3, seed=20261015, w=1280, h=560, f=787.0):
    """Undistorted pixel correspondences of a static scene seen from two camera
    poses (the reference points Tracking::trackReferenceFrame passes to
    findFundamentalMat, tracking.cc:547), with Gaussian pixel noise and a fraction
    of gross outliers.  -> (p1 f32 [n, 2], p2 f32 [n, 2], true-inlier bool [n])."""
    rng = np.random.default_rng(seed)
    K = np.array([[f, 0, w / 2], [0, f, h / 2], [0, 0, 1.0]])
    X = np.c_[rng.uniform(-10, 10, n), rng.uniform(-4, 4, n), rng.uniform(5, 50, n)]
    r = rng.normal(0, 0.02, 3)
    th = np.linalg.norm(r)
    kx = np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]]) / max(th, 1e-12)
    R = np.eye(3) + np.sin(th) * kx + (1 - np.cos(th)) * kx @ kx
    t = np.array([0.5, 0.02, 0.1]) + rng.normal(0, 0.05, 3)
    x1 = (K @ X.T).T
    x2 = (K @ (R @ X.T + t[:, None])).T
    x1 = x1[:, :2] / x1[:, 2:]
    x2 = x2[:, :2] / x2[:, 2:]
    x1 += rng.normal(0, noise_px, x1.shape)
    x2 += rng.normal(0, noise_px, x2.shape)
    out = rng.random(n) < outlier_frac
    x2[out] += rng.uniform(-30, 30, (int(out.sum()), 2))
    return (np.ascontiguousarray(x1, np.float32), np.ascontiguousarray(x2, np.float32), ~out)
