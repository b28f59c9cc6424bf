"""Independent numpy restatement of the disparity hot path (closed form).

TEST INFRASTRUCTURE ONLY: imported by tests/ to cross-check the C oracle
(oracle/mvsv_oracle.c).  It never runs on the product path.

Where the C oracle follows OpenCV 3.4's loop structure (rolling sums, running
cost rows, double-buffered path costs; that is what the reference executes
through ``Disparity::sgbm`` / ``Disparity::bm``, src/disparity.cpp:6-22),
this twin states the same results in closed form:

* C(y,x,d) = P2 + box sum of the Birchfield-Tomasi pixel cost with clamp-to-
  edge in cost space, plus OpenCV 3.4's two cost-row quirks (column x=0 and
  the bottom SH2 rows are not refreshed);
* every path direction is an independent 1-D scan that starts from a zero
  predecessor outside cost space;
* S = min(sum of all directions, 32767) -- the saturating SIMD sum order is
  irrelevant because every path cost is non-negative.

Agreement of the two restatements on random inputs is the transcription
check that stands in for the absent OpenCV ("parity unpinned").
"""
from __future__ import annotations

import numpy as np

MAX_COST = 32767
F_FIRSTCOL_FIX = 1
F_WTA_MIN_D = 2


def _sat16(a):
    return np.clip(a, -32768, 32767)


# --------------------------------------------------------------------------
# SGBM
# --------------------------------------------------------------------------
def sgbm_effective(p: dict, W: int) -> dict:
    bs = p["block_size"] if p["block_size"] > 0 else 5
    minD = p["min_disparity"]
    D = p["num_disparities"]
    P1 = p["p1"] if p["p1"] > 0 else 2
    e = dict(
        minD=minD, D=D, maxD=minD + D, SW2=bs // 2, SH2=bs // 2,
        ftzero=max(p["pre_filter_cap"], 15) | 1,
        uniq=p["uniqueness_ratio"] if p["uniqueness_ratio"] >= 0 else 10,
        disp12=p["disp12_max_diff"] if p["disp12_max_diff"] > 0 else 1,
        P1=P1, P2=max(p["p2"] if p["p2"] > 0 else 5, P1 + 1),
        fullDP=p["mode"] == 1,
    )
    e["minX1"] = max(e["maxD"], 0)
    e["maxX1"] = W + min(minD, 0)
    e["W1"] = e["maxX1"] - e["minX1"]
    e["INVALID"] = (minD - 1) * 16
    return e


def _prefilter_channels(img: np.ndarray, ftzero: int):
    """(sobel, raw) rows as used by calcPixelCostBT, uint8 semantics."""
    I = img.astype(np.int32)
    H, W = I.shape
    yn = np.maximum(np.arange(H) - 1, 0)
    ys = np.minimum(np.arange(H) + 1, H - 1)
    sob = np.full((H, W), ftzero & 255, np.int32)
    raw = I.copy()
    dx = lambda A: A[:, 2:] - A[:, :-2]  # noqa: E731
    g = dx(I) * 2 + dx(I[yn]) + dx(I[ys])
    sob[:, 1:-1] = (np.clip(g, -ftzero, ftzero) + ftzero) & 255
    raw[:, 0] = ftzero & 255
    raw[:, -1] = ftzero & 255
    return sob, raw


def _bt_interval(P: np.ndarray):
    """min/max of {v, (v+left)/2, (v+right)/2} with the row-end guards."""
    H, W = P.shape
    l = P.copy()
    r = P.copy()
    l[:, 1:] = (P[:, 1:] + P[:, :-1]) // 2
    r[:, :-1] = (P[:, :-1] + P[:, 1:]) // 2
    return np.minimum(np.minimum(l, r), P), np.maximum(np.maximum(l, r), P)


def sgbm_pixel_cost(L: np.ndarray, R: np.ndarray, e: dict) -> np.ndarray:
    """BT pixel cost, shape (H, W1, D), int32."""
    H, W = L.shape
    xs = np.arange(e["minX1"], e["maxX1"])
    ds = np.arange(e["minD"], e["maxD"])
    xr = xs[:, None] - ds[None, :]
    pix = np.zeros((H, e["W1"], e["D"]), np.int32)
    for chan, scale in ((0, 0), (1, 2)):
        PL = _prefilter_channels(L, e["ftzero"])[chan]
        PR = _prefilter_channels(R, e["ftzero"])[chan]
        u0a, u1a = _bt_interval(PL)
        v0a, v1a = _bt_interval(PR)
        u = PL[:, xs][:, :, None]
        u0 = u0a[:, xs][:, :, None]
        u1 = u1a[:, xs][:, :, None]
        v = PR[:, xr]
        v0 = v0a[:, xr]
        v1 = v1a[:, xr]
        c0 = np.maximum(np.maximum(0, u - v1), v0 - u)
        c1 = np.maximum(np.maximum(0, v - u1), u0 - v)
        pix += np.minimum(c0, c1) >> scale
    return pix


def sgbm_cost_volume(L, R, p: dict, flags: int = 0) -> np.ndarray:
    """C(y, x, d) including +P2 and the OpenCV 3.4 row/column quirks."""
    H, W = L.shape
    e = sgbm_effective(p, W)
    pix = sgbm_pixel_cost(L, R, e)
    W1, SW2, SH2, P2 = e["W1"], e["SW2"], e["SH2"], e["P2"]
    xi = np.arange(W1)
    hs = np.zeros_like(pix)
    for k in range(-SW2, SW2 + 1):
        hs += pix[:, np.clip(xi + k, 0, W1 - 1), :]
    yi = np.arange(H)
    Cn = np.full_like(pix, P2)
    for k in range(-SH2, SH2 + 1):
        Cn += hs[np.clip(yi + k, 0, H - 1)]
    C = Cn.copy()
    fix = bool(flags & F_FIRSTCOL_FIX)
    if e["fullDP"]:
        if not fix:
            C[1:, 0, :] = P2
        bottom = [y for y in range(1, H) if y + SH2 >= H]
        for y in bottom:
            C[y] = P2
    else:
        if not fix:
            C[1:, 0, :] = Cn[0, 0, :]
        last = 0
        for y in range(1, H):
            if y + SH2 >= H:
                C[y] = C[last]
            else:
                last = y
    return C


def _step(Lp, minLp, Cx, P1, P2):
    """One SGM recurrence step over the last (disparity) axis (SIMD semantics)."""
    pad = np.full(Lp.shape[:-1] + (1,), MAX_COST, np.int32)
    Lm = np.concatenate([pad, Lp[..., :-1]], axis=-1)
    Lq = np.concatenate([Lp[..., 1:], pad], axis=-1)
    delta = ((minLp + P2 + 32768) % 65536 - 32768)[..., None]  # (short) cast
    m = np.minimum(np.minimum(Lp, _sat16(Lm + P1)), _sat16(Lq + P1))
    m = np.minimum(m, delta)
    return _sat16(_sat16(m - delta) + Cx)


def sgbm_path(C: np.ndarray, dx: int, dy: int, P1: int, P2: int) -> np.ndarray:
    """L_r for predecessor (x-dx, y-dy); zero outside cost space."""
    H, W1, D = C.shape
    L = np.zeros_like(C)
    if dy == 0:
        order = range(W1) if dx > 0 else range(W1 - 1, -1, -1)
        for x in order:
            xp = x - dx
            if 0 <= xp < W1:
                Lp = L[:, xp, :]
            else:
                Lp = np.zeros((H, D), np.int32)
            L[:, x, :] = _step(Lp, Lp.min(axis=-1), C[:, x, :], P1, P2)
        return L
    order = range(H) if dy > 0 else range(H - 1, -1, -1)
    for y in order:
        yp = y - dy
        Lp = np.zeros((W1, D), np.int32)
        if 0 <= yp < H:
            src = L[yp]
            if dx == 0:
                Lp = src.copy()
            elif dx > 0:
                Lp[1:] = src[:-1]
            else:
                Lp[:-1] = src[1:]
        L[y] = _step(Lp, Lp.min(axis=-1), C[y], P1, P2)
    return L


def sgbm_directions(mode: int):
    fwd = [(1, 0), (1, 1), (0, 1), (-1, 1)]
    if mode == 1:
        return fwd + [(-1, 0), (1, -1), (0, -1), (-1, -1)]
    return fwd + [(-1, 0)]


def sgbm_aggregate(C: np.ndarray, e: dict, mode: int) -> np.ndarray:
    S = np.zeros_like(C)
    for dx, dy in sgbm_directions(mode):
        S += sgbm_path(C, dx, dy, e["P1"], e["P2"])
    return np.minimum(S, MAX_COST)


def sgbm_core(L, R, p: dict, flags: int = 0) -> np.ndarray:
    H, W = L.shape
    e = sgbm_effective(p, W)
    out = np.full((H, W), e["INVALID"], np.int32)
    if e["minX1"] >= e["maxX1"]:
        return out.astype(np.int16)
    C = sgbm_cost_volume(L, R, p, flags)
    S = sgbm_aggregate(C, e, p["mode"]).astype(np.int64)
    D, W1, minD, minX1 = e["D"], e["W1"], e["minD"], e["minX1"]
    d_idx = np.arange(D)
    minS = S.min(axis=-1)
    if p["mode"] == 1 or (flags & F_WTA_MIN_D):
        key = S * (1 << 20) + d_idx
    else:
        key = S * (1 << 20) + (d_idx & 7) * 4096 + d_idx
    best = np.argmin(key, axis=-1)
    best = np.where(minS >= MAX_COST, -1, best)  # no strict minimum below MAX_COST
    uq = e["uniq"]
    far = np.abs(best[..., None] - d_idx) > 1
    reject = ((S * (100 - uq) < (minS * 100)[..., None]) & far).any(axis=-1)
    Sm = np.take_along_axis(S, np.clip(best - 1, 0, D - 1)[..., None], -1)[..., 0]
    Sp = np.take_along_axis(S, np.clip(best + 1, 0, D - 1)[..., None], -1)[..., 0]
    Sb = minS
    inner = (best > 0) & (best < D - 1)
    den = np.maximum(Sm + Sp - 2 * Sb, 1)
    num = (Sm - Sp) * 16 + den
    q = np.trunc(num / (den * 2)).astype(np.int64)  # C division
    d16 = np.where(inner, best * 16 + q, best * 16) + minD * 16
    for y in range(H):
        d2c = np.full(W, MAX_COST)
        d2 = np.full(W, e["INVALID"])
        row = out[y]
        for x in range(W1 - 1, -1, -1):
            if reject[y, x]:
                continue
            b = int(best[y, x])
            x2 = x + minX1 - b - minD
            if 0 <= x2 < W and d2c[x2] > minS[y, x]:
                d2c[x2] = minS[y, x]
                d2[x2] = b + minD
            row[x + minX1] = d16[y, x]
        for x in range(minX1, e["maxX1"]):
            d1 = int(row[x])
            if d1 == e["INVALID"]:
                continue
            lo, hi = d1 >> 4, (d1 + 15) >> 4
            xl, xh = x - lo, x - hi
            if (0 <= xl < W and d2[xl] >= minD and abs(d2[xl] - lo) > e["disp12"]
                    and 0 <= xh < W and d2[xh] >= minD and abs(d2[xh] - hi) > e["disp12"]):
                row[x] = e["INVALID"]
    return out.astype(np.int16)


def median3x3(img: np.ndarray) -> np.ndarray:
    H, W = img.shape
    P = np.pad(img.astype(np.int32), 1, mode="edge")
    stack = np.stack([P[dy:dy + H, dx:dx + W] for dy in range(3) for dx in range(3)])
    return np.sort(stack, axis=0)[4].astype(np.int16)


def filter_speckles(img: np.ndarray, new_val: int, max_size: int, max_diff: int) -> np.ndarray:
    """Union-find over 4-neighbours (order independent), then size test."""
    H, W = img.shape
    a = img.astype(np.int32).ravel()
    parent = np.arange(H * W)

    def find(i):
        r = i
        while parent[r] != r:
            r = parent[r]
        while parent[i] != r:
            parent[i], i = r, parent[i]
        return r

    ok = a != new_val
    for y in range(H):
        for x in range(W):
            i = y * W + x
            if not ok[i]:
                continue
            for j in ((i + 1) if x + 1 < W else -1, (i + W) if y + 1 < H else -1):
                if j >= 0 and ok[j] and abs(a[i] - a[j]) <= max_diff:
                    ri, rj = find(i), find(j)
                    if ri != rj:
                        parent[max(ri, rj)] = min(ri, rj)
    roots = np.array([find(i) for i in range(H * W)])
    sizes = np.bincount(roots[ok], minlength=H * W)
    out = a.copy()
    small = ok & (sizes[roots] <= max_size)
    out[small] = new_val
    return out.reshape(H, W).astype(np.int16)


def sgbm_compute(L, R, p: dict, flags: int = 0) -> np.ndarray:
    d = median3x3(sgbm_core(L, R, p, flags))
    if p["speckle_window_size"] > 0:
        d = filter_speckles(d, (p["min_disparity"] - 1) * 16, p["speckle_window_size"],
                            16 * p["speckle_range"])
    return d


# --------------------------------------------------------------------------
# StereoBM (XSOBEL prefilter)
# --------------------------------------------------------------------------
def xsobel(img: np.ndarray, cap: int) -> np.ndarray:
    I = img.astype(np.int32)
    H, W = I.shape
    out = np.full((H, W), cap, np.int32)
    npairs = H // 2
    dxv = np.zeros_like(I)
    dxv[:, 1:-1] = I[:, 2:] - I[:, :-2]
    for k in range(npairs):
        y = 2 * k
        r0 = y - 1 if y > 0 else (y + 1 if H > 1 else y)
        r2 = y + 1
        r3 = y + 2 if y < H - 2 else y
        out[y] = dxv[r0] + 2 * dxv[y] + dxv[r2]
        out[y + 1] = dxv[y] + 2 * dxv[r2] + dxv[r3]
        out[y] = np.clip(out[y], -cap, cap) + cap
        out[y + 1] = np.clip(out[y + 1], -cap, cap) + cap
    out[:, 0] = cap
    out[:, -1] = cap
    if H % 2 == 1:
        out[-1] = cap
    return out


def bm_compute(L, R, p: dict) -> np.ndarray:
    """StereoBM::compute (CV_16S) for XSOBEL, closed-form window sums."""
    H, W = L.shape
    nd, mind0 = p["num_disparities"], p["min_disparity"]
    FILTERED = (mind0 - 1) * 16
    out = np.full((H, W), FILTERED, np.int64)
    lofs = max(nd - 1 + mind0, 0)
    rofs = -min(nd - 1 + mind0, 0)
    width1 = W - rofs - nd + 1
    if lofs >= W or rofs >= W or width1 < 1:
        return out.astype(np.int16)
    cap = p["pre_filter_cap"]
    Lf = xsobel(L, cap)
    Rf = xsobel(R, cap)
    w2 = p["block_size"] // 2
    xmin = max(0, mind0 + nd - 1) + w2
    xmax, ymin, ymax = W - w2, w2, H - w2
    if xmax - xmin <= 0 or ymax - ymin <= 0:
        return out.astype(np.int16)
    # virtual column j in [-w2, width1 + w2): left col clampL, right col clampR
    j = np.arange(-w2, width1 + w2)
    cl = lofs + np.clip(j, -lofs, W - 1 - lofs)
    cr = rofs + np.clip(j, -rofs, W - nd - rofs)
    rows = np.arange(ymin - w2, ymax + w2)
    Lc = Lf[rows][:, cl]                                   # (nr, nj)
    sad = np.zeros((ymax - ymin, width1, nd), np.int64)
    for k in range(nd):
        A = np.abs(Lc - Rf[rows][:, cr + k])
        cs = np.cumsum(np.pad(A, ((1, 0), (1, 0))), axis=0).cumsum(axis=1)
        n = 2 * w2 + 1
        box = cs[n:, n:] - cs[:-n, n:] - cs[n:, :-n] + cs[:-n, :-n]
        sad[:, :, k] = box
    T = np.abs(Lc - cap)
    cs = np.cumsum(np.pad(T, ((1, 0), (1, 0))), axis=0).cumsum(axis=1)
    n = 2 * w2 + 1
    tsum = cs[n:, n:] - cs[:-n, n:] - cs[n:, :-n] + cs[:-n, :-n]
    mind = np.argmin(sad, axis=-1)
    minsad = sad.min(axis=-1)
    kk = np.arange(nd)
    filt = tsum < p["texture_threshold"]
    if p["uniqueness_ratio"] > 0:
        thresh = minsad + (minsad * p["uniqueness_ratio"] // 100)
        far = (kk < mind[..., None] - 1) | (kk > mind[..., None] + 1)
        filt |= (far & (sad <= thresh[..., None])).any(axis=-1)
    pp = np.take_along_axis(sad, np.clip(mind + 1, 0, nd - 1)[..., None], -1)[..., 0]
    nn = np.take_along_axis(sad, np.clip(mind - 1, 0, nd - 1)[..., None], -1)[..., 0]
    inner = (mind > 0) & (mind < nd - 1)
    v1 = nd - mind - 1 + mind0
    v2 = np.where(inner, pp - nn, 0)
    dd = np.where(inner, pp + nn - 2 * minsad + np.abs(pp - nn), 0)
    safe = np.where(dd != 0, dd, 1)
    q = np.where(dd != 0, np.trunc(v2 * 256 / safe), 0).astype(np.int64)
    disp = (v1 * 256 + q + 15) >> 4
    disp = np.where(filt, FILTERED, disp)
    ncol = min(width1, W - lofs)  # no spill past the row end (OpenCV UB)
    disp = disp[:, :ncol]
    minsad = minsad[:, :ncol]
    out[ymin:ymax, lofs:lofs + ncol] = disp
    if p["disp12_max_diff"] >= 0:
        cost = np.zeros((H, W), np.int64)
        cost[ymin:ymax, lofs:lofs + ncol] = minsad
        _bm_validate(out, cost, ymin, ymax, mind0, nd, p["disp12_max_diff"])
    out[ymin:ymax, :xmin] = FILTERED
    out[ymin:ymax, xmax:] = FILTERED
    out = out.astype(np.int16)
    if p["speckle_range"] >= 0 and p["speckle_window_size"] > 0:
        out = filter_speckles(out, FILTERED, p["speckle_window_size"], p["speckle_range"])
    return out


def _bm_validate(disp, cost, r0, r1, minD, nd, d12):
    H, W = disp.shape
    maxD = minD + nd
    minX1, maxX1 = max(maxD, 0), W + min(minD, 0)
    INV = (minD - 1) * 16
    d12 *= 16
    for y in range(r0, r1):
        d2 = np.full(W, INV)
        c2 = np.full(W, np.iinfo(np.int64).max)
        for x in range(minX1, maxX1):
            d = int(disp[y, x])
            if d == INV:
                continue
            x2 = x - ((d + 8) >> 4)
            if 0 <= x2 < W and c2[x2] > cost[y, x]:
                c2[x2] = cost[y, x]
                d2[x2] = d
        for x in range(minX1, maxX1):
            d = int(disp[y, x])
            if d == INV:
                continue
            xl, xh = x - (d >> 4), x - ((d + 15) >> 4)
            if ((0 <= xl < W and d2[xl] > INV and abs(d2[xl] - d) > d12)
                    and (0 <= xh < W and d2[xh] > INV and abs(d2[xh] - d) > d12)):
                disp[y, x] = INV


def mean_disparity_grid(dmap: np.ndarray) -> np.ndarray:
    H, W = dmap.shape
    dx, dy = W // 9, H // 9
    out = np.zeros(81, np.float32)
    for r in range(9):
        for c in range(9):
            t = dmap[r * dy:(r + 1) * dy, c * dx:(c + 1) * dx].astype(np.int64)
            v = t[t > 1]
            tot, n = int(v.sum()), int(v.size)
            out[r * 9 + c] = 0.0 if (tot == 0 or n == 0) else float(tot // n)
    return out
