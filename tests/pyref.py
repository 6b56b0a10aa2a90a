"""Independent numpy restatement of the reference's CPU SGM path.

Written separately from oracle/sgm_oracle.c (different loop structure:
vectorised over disparities and over the independent pixels of each sweep
front) so that the two restatements check each other at small sizes.  Every
float32 operation is an explicit numpy float32 op in the reference's
association order.  Tests only; small inputs only.
"""
from __future__ import annotations

from collections import deque

import numpy as np

f32 = np.float32
FLT_MAX = np.finfo(np.float32).max


def blur(img):
    """Pinned cv::GaussianBlur(3x3, 2, 1) on CV_8U (src/Solver.cpp:124-125)."""
    a = img.astype(np.int64)
    H, W = a.shape

    def refl(idx, n):
        idx = np.where(idx < 0, -idx, idx)
        return np.where(idx >= n, 2 * n - 2 - idx, idx) if n > 1 else np.zeros_like(idx)

    cols = np.arange(W)
    rows = np.arange(H)
    hsum = 82 * a[:, refl(cols - 1, W)] + 93 * a + 82 * a[:, refl(cols + 1, W)]
    acc = 70 * hsum[refl(rows - 1, H)] + 116 * hsum + 70 * hsum[refl(rows + 1, H)]
    return np.minimum((acc + 32768) >> 16, 255).astype(np.uint8)


def census(img, scale=1):
    """CT_pts (src/cost.cpp:99-129) via shifted, edge-clamped copies."""
    H, W = img.shape
    wh, ww = 7 // scale, 9 // scale
    out = np.zeros((H, W), np.uint64)
    ctr = img
    ys = np.arange(H)
    xs = np.arange(W)
    for di in range(-(wh // 2), wh // 2 + 1):
        yy = np.clip(ys + di, 0, H - 1)
        for dj in range(-(ww // 2), ww // 2 + 1):
            if di == 0 and dj == 0:
                continue
            xx = np.clip(xs + dj, 0, W - 1)
            nb = img[yy][:, xx]
            out = (out << np.uint64(1)) | (nb > ctr).astype(np.uint64)
    return out


def _popcount(x):
    x = x.astype(np.uint64)
    c = np.zeros(x.shape, np.int64)
    for b in range(64):
        c += ((x >> np.uint64(b)) & np.uint64(1)).astype(np.int64)
    return c


def dsi(ctl, ctr, D, scale=1, view=0, sky=None):
    H, W = ctl.shape
    j = np.arange(W)[:, None]
    d = np.arange(D)[None, :]
    if view == 0:
        idx = np.maximum(j - d // scale, 0)
        c = _popcount(ctl[:, :, None] ^ ctr[:, idx])
    else:
        idx = np.minimum(j + d // scale, W - 1)
        c = _popcount(ctl[:, idx] ^ ctr[:, :, None])
    c = c.astype(np.float32)
    if sky is not None:
        m = sky == 255
        c[m] = f32(999999)
        c[m, 0] = f32(0)
    return c


def _iir_along(a, win):
    """In-place literal IIR along axis 0 of a (n, ...) float32 array
    (src/Solver.cpp:296-330 and :333-368 share this body)."""
    n = a.shape[0]
    s = np.zeros(a.shape[1:], np.float32)
    idx = 0
    for _ in range(win):
        s = s + a[idx]
        idx += 1
    h = win // 2
    j = h
    while j < n - h:
        a[idx - (h + 1)] = s / f32(win)
        if j == n - h - 1:
            break
        s = s + a[idx]
        s = s - a[idx - win]
        idx += 1
        j += 1
    return a


def hfilter(cost, win):
    c = np.array(cost, np.float32, copy=True)
    return np.ascontiguousarray(np.swapaxes(_iir_along(np.swapaxes(c, 0, 1), win), 0, 1))


def vfilter(cost, win):
    c = np.array(cost, np.float32, copy=True)
    return _iir_along(c, win)


def _dp(prev, min_prev, c, P1, P2):
    D = c.shape[-1]
    dm = np.maximum(np.arange(D) - 1, 0)
    dp = np.minimum(np.arange(D) + 1, D - 1)
    v = np.minimum(prev, prev[..., dm] + f32(P1))
    v = np.minimum(v, prev[..., dp] + f32(P1))
    v = np.minimum(v, (min_prev + f32(P2))[..., None])
    v = v + (c - min_prev[..., None])
    return v


# (di, dj): the step from predecessor to pixel along the path.
DIRS = [(0, 1), (0, -1), (1, 0), (-1, 0), (1, 1), (1, -1), (-1, 1), (-1, -1)]


def path(cost, direction, P1=10, P2=100):
    """src/SGM.cpp:81-369; sweeps one front at a time."""
    H, W, D = cost.shape
    di, dj = DIRS[direction]
    L = np.empty_like(cost)
    if di == 0:
        cols = range(W) if dj > 0 else range(W - 1, -1, -1)
        first = True
        for j in cols:
            if first:
                L[:, j] = cost[:, j]
                first = False
            else:
                p = L[:, j - dj]
                L[:, j] = _dp(p, p.min(axis=-1), cost[:, j], P1, P2)
    else:
        rows = range(H) if di > 0 else range(H - 1, -1, -1)
        first = True
        for i in rows:
            if first:
                L[i] = cost[i]
                first = False
                continue
            p_row = L[i - di]
            out = np.empty((W, D), np.float32)
            for j in range(W):
                pj = j - dj
                if pj < 0 or pj >= W:
                    out[j] = cost[i, j]
                else:
                    p = p_row[pj]
                    out[j] = _dp(p, p.min(), cost[i, j], P1, P2)
            L[i] = out
    return L, L.min(axis=-1)


def aggregate(Ls):
    s = ((Ls[0] + Ls[1]) + Ls[2]) + Ls[3]
    return s + (((Ls[4] + Ls[5]) + Ls[6]) + Ls[7])


def wta(S, uniq=0.7):
    H, W, D = S.shape
    out = np.empty((H, W), np.int32)
    u = f32(uniq)
    for i in range(H):
        for j in range(W):
            s = S[i, j]
            m = s.min()
            md = int(np.argmax(s == m))
            rest = s[s != m]
            if rest.size == 0:
                out[i, j] = md
                continue
            sm = rest.min()
            sd = int(np.argmax(s == sm))
            out[i, j] = D + 1 if (f32(m) / f32(sm) > u and abs(md - sd) > 1) else md
    return out


def subpixel(disp, S):
    H, W, D = S.shape
    out = np.empty((H, W), np.float32)
    for i in range(H):
        for j in range(W):
            d = int(disp[i, j])
            if d > D - 1:
                out[i, j] = D + 1
            elif d == 0 or d == D - 1:
                out[i, j] = d
            else:
                a, b, c = S[i, j, d - 1], S[i, j, d + 1], S[i, j, d]
                x = f32(d) + (a - b) / (f32(2) * ((a + b) - f32(2) * c))
                out[i, j] = f32(D - 1) if f32(D - 1) < x else x
    return out


def lr_check(FL, FR, D, scale=1, lr_dis=1.0):
    FL = np.array(FL, np.float32, copy=True)
    H, W = FL.shape
    for i in range(H):
        for j in range(W):
            dl = FL[i, j]
            if f32(j) >= dl:
                # clamped column (the build's choice where SGM.cpp:812 would read
                # outside the row; never acts on maps compute_subpixel produces)
                x = f32(j) - dl / f32(scale)
                jr = 0 if x < 0 else (W - 1 if x > W - 1 else int(x))
                if abs(dl - FR[i, jr]) > f32(lr_dis):
                    FL[i, j] = D + 1
    return FL


def post_filter(F, D, scale=1):
    F = np.array(F, np.float32, copy=True)
    H, W = F.shape
    for i in range(2, H - 2):
        for j in range(2, W - 2):
            if F[i, j] <= D - 1:
                continue
            win = F[i - 2:i + 3, j - 2:j + 3].ravel()
            v = sorted(int(x) for x in win if x <= D - 1)
            if len(v) > 12:
                F[i, j] = v[len(v) // 2]
    seen = np.zeros((H, W), bool)
    max_size = 1000 // scale
    for i in range(H):
        for j in range(W):
            if seen[i, j]:
                continue
            comp = [(i, j)]
            seen[i, j] = True
            q = deque(comp)
            while q:
                a, b = q.popleft()
                for na, nb in ((a - 1, b), (a + 1, b), (a, b - 1), (a, b + 1)):
                    if 0 <= na < H and 0 <= nb < W and not seen[na, nb] and \
                            abs(F[a, b] - F[na, nb]) < 2:
                        seen[na, nb] = True
                        comp.append((na, nb))
                        q.append((na, nb))
            if len(comp) <= max_size:
                for a, b in comp:
                    F[a, b] = D + 1
    return F


def lk_refine(L, R, disp, D):
    """LKRefineCore (LKRefine/LKSubPixelImpl.cpp:56-235), pure numpy float32
    scalars, with the fp32 evaluation order pinned in oracle/sgm_oracle.c."""
    L = np.asarray(L, np.int64)
    R = np.asarray(R, np.int64)
    F = np.array(disp, np.float32, copy=True)
    H, W = F.shape
    hw = 3
    Ix = np.zeros((H, W), np.float32)
    dt = F.copy()
    nd = F.copy()
    for i in range(hw, H - hw):
        for j in range(hw, W - hw):
            Ix[i, j] = f32(L[i, j + 1] - L[i, j - 1]) * f32(0.5)
            nd[i, j] = f32(int(F[i, j]))
            dt[i, j] = f32(int(F[i, j]))
    wcorner = f32(np.exp(-1.0))
    for i in range(hw, H - hw):
        for j in range(hw, W - hw):
            if not Ix[i, j] > 2:
                continue
            d0 = dt[i, j]
            if not (d0 > 0 and d0 < D):
                continue
            last_disp, last_doff, last_diff = d0, f32(0), f32(np.finfo(np.float32).max)
            for _ in range(10):
                w, jx, res = [], [], []
                valid = 0
                for v in range(-hw, hw + 1):
                    for u in range(-hw, hw + 1):
                        m, n = i + v, j + u
                        dm = dt[m, n]
                        dw = dm + last_doff
                        ok = (Ix[m, n] > 2 and dm > 0 and dm < D and abs(d0 - dm) <= 2
                              and not (f32(n) - dw < 0 or f32(n) - dw > f32(W - 1)))
                        if not ok:
                            w.append(f32(0)); jx.append(f32(0)); res.append(f32(0))
                            continue
                        w.append(wcorner if v * v + u * u >= 18 else f32(1))
                        res.append(f32(R[m, int(f32(n) - dw)] - L[m, n]))
                        jx.append(Ix[m, n])
                        valid += 1
                if valid < 4.9:
                    break
                s2 = f32(0)
                for x in w:
                    s2 = f32(s2 + x * x)
                nrm = np.sqrt(s2)
                w = [x / nrm for x in w]
                hs = f32(0)
                for a, b in zip(jx, w):
                    hs = f32(hs + (a * b) * a)
                if float(hs) < 1e-3:
                    break
                hinv = f32(1) / hs
                doff = f32(0)
                for a, b, r in zip(jx, w, res):
                    doff = f32(doff + ((hinv * a) * b) * r)
                if abs(doff - last_doff) > last_diff:
                    break
                if not (d0 + doff > 0 and d0 + doff < D):
                    break
                last_disp = d0 + doff
                last_diff = abs(doff - last_doff)
                last_doff = doff
                if float(last_diff) < 1e-6:
                    break
            nd[i, j] = last_disp
    return nd


def sky_detect(img, scale=1):
    """SkyAreaDetector::detect (sky_detector/imageSkyDetector.cpp:166-208),
    numpy restatement with the numerics pinned in oracle/sgm_oracle.c."""
    img = np.asarray(img, np.int64)
    if scale > 1:
        h, w = img.shape[0] // 2 * 2, img.shape[1] // 2 * 2
        G = (img[0:h:2, 0:w:2] + img[0:h:2, 1:w:2] + img[1:h:2, 0:w:2] + img[1:h:2, 1:w:2] + 2) >> 2
    else:
        G = img.copy()
    H, W = G.shape
    P = np.pad(G, 1, mode="reflect") if H > 1 and W > 1 else np.pad(G, 1, mode="edge")
    dx = (P[:-2, 2:] + 2 * P[1:-1, 2:] + P[2:, 2:]) - (P[:-2, :-2] + 2 * P[1:-1, :-2] + P[2:, :-2])
    dy = (P[2:, :-2] + 2 * P[2:, 1:-1] + P[2:, 2:]) - (P[:-2, :-2] + 2 * P[:-2, 1:-1] + P[:-2, 2:])
    a = dx * dx + dy * dy
    flat = G.ravel()
    nz = G != 0
    N, S1, S2 = int(nz.sum()), int(G[nz].sum()), int((G[nz] ** 2).sum())
    half = H // 2
    rows = np.arange(H)[:, None]
    best = np.full(W, H - 1)
    jn_max = 0.0
    for k in range(1, 121):
        t = 5 + 3 * (k - 1)
        b = np.full(W, -1)
        for c in range(W):
            hit = np.flatnonzero(a[:half + 1, c] > t * t)
            if hit.size == 0:
                continue
            r = int(hit[0])
            if r >= half or r <= 5:
                continue
            up, dn = (r - 1) * W + c, (r + 1) * W + c
            gy = (2 * flat[dn] + flat[dn + 1] + flat[dn - 1]) - (2 * flat[up] + flat[up + 1] + flat[up - 1])
            b[c] = -1 if gy > 0 else r
        sky = (rows < b[None, :]) & nz
        ns, s1, s2 = int(sky.sum()), int(G[sky].sum()), int((G[sky] ** 2).sum())
        ng, g1, g2 = N - ns, S1 - s1, S2 - s2
        if ng == 0 or ns == 0:
            jn = np.finfo(np.float64).tiny
        else:
            vs = float(ns * s2 - s1 * s1) / (float(ns) * float(ns))
            vg = float(ng * g2 - g1 * g1) / (float(ng) * float(ng))
            jn = 1 / ((2 * 0.0 + 0.0) + (2 * (3 * vs) + (3 * vg)))
        if jn > jn_max:
            jn_max, best = jn, b.copy()
    for i in range(W):
        border = best[i]
        if border > 0 and (G[:border, i] < 128).any():
            best[i] = -1
        if border != -1 and (i > 1 and best[i - 1] == -1) and (i < W - 1 and best[i + 1] == -1):
            best[i] = -1
    i = 0
    while i < W:
        if best[i] != -1:
            p = i
            q = W if i == W - 1 else -1
            for j in range(i + 1, W):
                if best[j] == -1 or j == W - 1:
                    q = W if j == W - 1 else j
                    break
            if q > p and q - p < 30:
                best[p:q] = -1
            i = q
        i += 1
    return np.where(rows <= best[None, :], 255, 0).astype(np.uint8)


def bm_process(left, right, D, scale=1, sky=None, uniq=0.7, blur_on=True):
    """BM::process (src/BM.cpp:9-97): rows not strided by the scale (:24-25),
    cost + filters, WTA with |min_d - sec_min_d| > 2."""
    left = np.asarray(left, np.uint8)
    right = np.asarray(right, np.uint8)
    h, w = left.shape
    H, W = h // scale, w // scale
    L = left[:H, 0:W * scale:scale][:, :W]
    R = right[:H, 0:W * scale:scale][:, :W]
    if blur_on:
        L, R = blur(L), blur(R)
    C = dsi(census(L, scale), census(R, scale), D, scale, 0, sky)
    C = vfilter(hfilter(C, 5 // scale), 3 // scale)
    disp = np.empty((H, W), np.int32)
    for i in range(H):
        for j in range(W):
            c = C[i, j]
            m = c.min()
            d = int(np.argmax(c == m))
            rest = c[c != m]
            if rest.size:
                s = rest.min()
                sd = int(np.argmax(c == s))
                if m / s > f32(uniq) and abs(d - sd) > 2:
                    d = D + 1
            disp[i, j] = d
    return disp


def colormap(F, D):
    """Solver::colormap (src/Solver.cpp:652-707): BGR u8, float32 arithmetic,
    float -> uchar conversions truncating, the last two bands in double."""
    F = np.asarray(F, np.float32)
    H, W = F.shape
    out = np.zeros((H, W, 3), np.uint8)
    for i in range(H):
        for j in range(W):
            v = F[i, j]
            if v > D - 1:
                continue
            v = f32(v * f32(256 // D))
            if v <= 51:
                out[i, j] = (255, int(f32(v * f32(5))), 0)
            elif v <= 102:
                v = f32(v - f32(51))
                out[i, j] = (int(f32(f32(255) - f32(v * f32(5)))), 255, 0)
            elif v <= 153:
                v = f32(v - f32(102))
                out[i, j] = (0, 255, int(f32(v * f32(5))))
            elif v <= 204:
                v = f32(v - f32(153))
                out[i, j] = (0, 255 - int(128.0 * float(v) / 51.0 + 0.5), 255)
            else:
                v = f32(v - f32(204))
                out[i, j] = (0, 127 - int(127.0 * float(v) / 51.0 + 0.5), 255)
    return out


def point_cloud(F, img, D, scale, fx, fy, cx, cy, baseline=0.5, max_range=100.0):
    """node.cpp:119-143: row-major (X, Y, Z) doubles and img(i, j) gray values."""
    F = np.asarray(F, np.float32)
    H, W = F.shape
    fx, fy, cx, cy, mr = f32(fx), f32(fy), f32(cx), f32(cy), f32(max_range)
    pts, pix = [], []
    for i in range(H):
        for j in range(W):
            d = F[i, j]
            if d == f32(D + 1):
                continue
            Z = float(f32(fx + fy)) / 2.0 * baseline / (float(d) + 1e-6)
            if Z > float(mr):
                continue
            X = float(f32(f32(j * scale) - cx)) * Z / float(fx)
            Y = float(f32(f32(i * scale) - cy)) * Z / float(fy)
            pts.append((X, Y, Z))
            pix.append(int(img[i, j]))
    return np.array(pts, np.float64).reshape(-1, 3), np.array(pix, np.uint8)
