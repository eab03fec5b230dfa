"""Second, independent restatement (numpy / pure Python) of the pixel stages of
ORBextractor::operator(), used only to cross-check the C oracle on small inputs.

Written vectorised (whole-image numpy) where the oracle is written as scalar C loops,
so a shared misreading of the reference would have to be made twice in two styles.
Each function cites the reference lines it restates (ORBextractor.cc unless noted).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
        (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def scale_factors(nlevels=8, scale=1.2):
    """cc:452-461: float accumulator times the double member scaleFactor."""
    s = [F32(1.0)]
    for _ in range(1, nlevels):
        s.append(F32(np.float64(s[-1]) * np.float64(F32(scale))))
    return s


def level_sizes(W, H, nlevels=8, scale=1.2):
    """cc:1641-1643: cvRound((float)cols * mvInvScaleFactor[level])."""
    out = []
    for s in scale_factors(nlevels, scale):
        inv = F32(1.0) / s
        out.append((int(np.rint(F32(W) * inv)), int(np.rint(F32(H) * inv))))
    return out


def resize_linear(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    """cv::resize INTER_LINEAR, CV_8U, OpenCV 3.3.1 fixed point (called at cc:1656-1661)."""
    sh, sw = src.shape
    sx_scale = 1.0 / (dw / sw)
    sy_scale = 1.0 / (dh / sh)
    dx = np.arange(dw)
    fx = ((dx + 0.5) * sx_scale - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx.astype(np.float32)).astype(np.float32)
    neg = sx < 0
    fx[neg] = 0
    sx[neg] = 0
    over = sx + 1 >= sw
    xmax = int(np.argmax(over)) if over.any() else dw
    clampr = sx >= sw - 1
    fx[clampr] = 0
    sx[clampr] = sw - 1
    a0 = np.rint((F32(1) - fx) * F32(2048)).astype(np.int64)
    a1 = np.rint(fx * F32(2048)).astype(np.int64)
    sx1 = np.minimum(sx + 1, sw - 1)
    tail = dx >= xmax
    a0[tail] = 2048
    a1[tail] = 0
    dy = np.arange(dh)
    fy = ((dy + 0.5) * sy_scale - 0.5).astype(np.float32)
    sy = np.floor(fy).astype(np.int64)
    fy = (fy - sy.astype(np.float32)).astype(np.float32)
    b0 = np.rint((F32(1) - fy) * F32(2048)).astype(np.int64)
    b1 = np.rint(fy * F32(2048)).astype(np.int64)
    r0 = np.clip(sy, 0, sh - 1)
    r1 = np.clip(sy + 1, 0, sh - 1)
    s = src.astype(np.int64)
    hrow = s[:, sx] * a0[None, :] + s[:, sx1] * a1[None, :]
    h0 = hrow[r0]
    h1 = hrow[r1]
    v = (((b0[:, None] * (h0 >> 4)) >> 16) + ((b1[:, None] * (h1 >> 4)) >> 16) + 2) >> 2
    return np.clip(v, 0, 255).astype(np.uint8)


def pyramid(img: np.ndarray, nlevels=8, scale=1.2):
    sizes = level_sizes(img.shape[1], img.shape[0], nlevels, scale)
    levels = [img.copy()]
    for (w, h) in sizes[1:]:
        levels.append(resize_linear(levels[-1], w, h))
    return levels


def gaussian_blur(img: np.ndarray) -> np.ndarray:
    """GaussianBlur 7x7 sigma 2 REFLECT_101, 8U fixed point (cc:1587-1595)."""
    k = np.array([18, 34, 49, 55, 49, 34, 18], dtype=np.int64)
    p = np.pad(img.astype(np.int64), 3, mode="reflect")  # numpy 'reflect' == BORDER_REFLECT_101
    h, w = img.shape
    rows = sum(k[i] * p[:, i:i + w] for i in range(7))
    cols = sum(k[i] * rows[i:i + h, :] for i in range(7))
    return np.minimum((cols + (1 << 15)) >> 16, 255).astype(np.uint8)


def fast_strength(img: np.ndarray) -> np.ndarray:
    """M = max over 9-arcs of max(min(v - x), min(x - v)); 0 on the 3-px border."""
    h, w = img.shape
    s = img.astype(np.int64)
    c = s[3:h - 3, 3:w - 3]
    d = np.stack([c - s[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in RING])
    M = np.full(c.shape, -1000, dtype=np.int64)
    for st in range(16):
        idx = [(st + i) % 16 for i in range(9)]
        M = np.maximum(M, np.maximum(d[idx].min(0), -d[idx].max(0)))
    out = np.zeros((h, w), dtype=np.int64)
    out[3:h - 3, 3:w - 3] = np.maximum(M, 0)
    return out


def fast_nms(sub: np.ndarray, t: int):
    """cv::FAST(sub, kps, t, true) on one cell sub-image: corners M>t, score M-1,
    strict 8-neighbour NMS inside the detection window [3,rows-3)x[3,cols-3)."""
    t = min(max(t, 0), 255)
    rows, cols = sub.shape
    if rows < 7 or cols < 7:
        return []
    M = fast_strength(sub)
    win = np.zeros_like(M)
    win[3:rows - 3, 3:cols - 3] = 1
    score = np.where((M > t) & (win > 0), M - 1, 0)
    pad = np.pad(score, 1)
    nb = np.zeros_like(score)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dx or dy:
                nb = np.maximum(nb, pad[1 + dy:1 + dy + rows, 1 + dx:1 + dx + cols])
    keep = (M > t) & (win > 0) & (score > nb)
    ys, xs = np.nonzero(keep)  # raster order
    return [(int(x), int(y), int(score[y, x])) for y, x in zip(ys, xs)]


def level_candidates(level: np.ndarray, ini=20, mn=7):
    """ComputeKeyPointsOctTree cell loop (cc:1025-1122): (x, y, response) relative to minBorder."""
    h, w = level.shape
    minB, maxBX, maxBY = 16, w - 16, h - 16
    width, height = F32(maxBX - minB), F32(maxBY - minB)
    nCols, nRows = int(width / F32(30)), int(height / F32(30))
    wCell, hCell = int(np.ceil(width / F32(nCols))), int(np.ceil(height / F32(nRows)))
    out = []
    for i in range(nRows):
        iniY = minB + i * hCell
        maxY = iniY + hCell + 6
        if iniY >= maxBY - 3:
            continue
        maxY = min(maxY, maxBY)
        for j in range(nCols):
            iniX = minB + j * wCell
            maxX = iniX + wCell + 6
            if iniX >= maxBX - 6:
                continue
            maxX = min(maxX, maxBX)
            sub = level[iniY:maxY, iniX:maxX]
            kps = fast_nms(sub, ini) or fast_nms(sub, mn)
            out += [(x + j * wCell, y + i * hCell, s) for (x, y, s) in kps]
    return out


def fast_atan2(y: float, x: float) -> float:
    """cv::fastAtan2 (OpenCV 3.3.1), all float32 arithmetic."""
    deg = F32(180.0 / np.pi)
    p1, p3 = F32(0.9997878412794807) * deg, F32(-0.3258083974640975) * deg
    p5, p7 = F32(0.1555786518463281) * deg, F32(-0.04432655554792128) * deg
    eps = F32(2.220446049250313e-16)
    y, x = F32(y), F32(x)
    ax, ay = abs(x), abs(y)
    if ax >= ay:
        c = ay / (ax + eps)
        c2 = c * c
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c
    else:
        c = ax / (ay + eps)
        c2 = c * c
        a = F32(90) - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c
    if x < 0:
        a = F32(180) - a
    if y < 0:
        a = F32(360) - a
    return float(F32(a))


def umax_table():
    """cc:519-549."""
    vmax = int(np.floor(F32(15) * np.sqrt(F32(2)) / F32(2) + F32(1)))
    vmin = int(np.ceil(F32(15) * np.sqrt(F32(2)) / F32(2)))
    u = [0] * 16
    for v in range(vmax + 1):
        u[v] = int(np.rint(np.sqrt(225.0 - v * v)))
    v0 = 0
    for v in range(15, vmin - 1, -1):
        while u[v0] == u[v0 + 1]:
            v0 += 1
        u[v] = v0
        v0 += 1
    return u


def ic_angle(img: np.ndarray, x: int, y: int, umax) -> float:
    """IC_Angle (cc:59-106) as explicit moments over the circular patch."""
    m10 = m01 = 0
    for v in range(-15, 16):
        d = umax[abs(v)]
        for u in range(-d, d + 1):
            val = int(img[y + v, x + u])
            m10 += u * val
            m01 += v * val
    return fast_atan2(m01, m10)


def orb_descriptor(blurred: np.ndarray, x: int, y: int, angle: float, pattern: np.ndarray) -> np.ndarray:
    """computeOrbDescriptor (cc:118-172) with cos/sin rounded from double and the sample
    offsets fused (hazard H4)."""
    r = F32(angle) * F32(np.pi / 180.0)
    a, b = F32(np.cos(np.float64(r))), F32(np.sin(np.float64(r)))
    pts = pattern.reshape(512, 2).astype(np.float32)
    px, py = pts[:, 0], pts[:, 1]
    # fused as g++ -O3 -march=native builds the reference (H4): fma(x, b, y*a) and
    # fma(x, a, -(y*b)).  x*b is exact in double (|x| <= 15), y*a is rounded to float
    # first, their double sum is exact, so one rounding to float32 is the fma's.
    f64 = np.float64
    ry = np.rint((px.astype(f64) * f64(b) + (py * a).astype(f64)).astype(np.float32)).astype(np.int64)
    rx = np.rint((px.astype(f64) * f64(a) - (py * b).astype(f64)).astype(np.float32)).astype(np.int64)
    vals = blurred[y + ry, x + rx].astype(np.int64)
    bits = (vals[0::2] < vals[1::2]).astype(np.uint8)  # pair p -> bit p
    return np.packbits(bits, bitorder="little")


def descriptor_distance(a: np.ndarray, b: np.ndarray) -> int:
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def load_pattern(path) -> np.ndarray:
    import re
    text = open(path).read()
    body = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return np.array([int(v) for v in re.findall(r"-?\d+", body)], dtype=np.int64)
