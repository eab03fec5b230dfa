"""Seeded synthetic grayscale frames.

No TUM/KITTI/EuRoC data exists on either machine, so every test and the bench use
these frames.  A frame is a u8 canvas of random rotated rectangles and ellipses,
plus an 8-px-lattice value-noise texture (+-24, bilinear) and +-6 per-pixel noise,
saturated.  That is corner-rich enough to exceed the per-level budgets at
iniThFAST=20 while leaving flat cells that exercise the minThFAST fallback
(ORBextractor.cc:1091-1104).

Stereo pairs: the right image is the left shifted by a piecewise-constant integer
disparity field (32x32 blocks, d in [0, max_disp]).
"""
from __future__ import annotations

import numpy as np

__all__ = ["frame", "frames", "stereo_pair", "StereoSequence"]


def _rng(seed: int) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64(int(seed)))


def frame(seed: int, width: int = 640, height: int = 480, n_shapes: int = 200) -> np.ndarray:
    """One synthetic frame, shape (height, width), dtype uint8, C-contiguous."""
    g = _rng(seed)
    img = np.full((height, width), g.integers(0, 256), dtype=np.int32)
    yy, xx = np.mgrid[0:height, 0:width]
    for _ in range(n_shapes):
        cx = g.integers(0, width)
        cy = g.integers(0, height)
        a = g.integers(6, max(8, width // 8))
        b = g.integers(6, max(8, height // 8))
        th = g.uniform(0.0, np.pi)
        level = g.integers(0, 256)
        kind = g.integers(0, 2)
        r = int(np.ceil(np.hypot(a, b))) + 1
        x0, x1 = max(0, cx - r), min(width, cx + r + 1)
        y0, y1 = max(0, cy - r), min(height, cy + r + 1)
        if x0 >= x1 or y0 >= y1:
            continue
        dx = xx[y0:y1, x0:x1] - cx
        dy = yy[y0:y1, x0:x1] - cy
        c, s = np.cos(th), np.sin(th)
        u = dx * c + dy * s
        v = -dx * s + dy * c
        if kind == 0:
            m = (np.abs(u) <= a) & (np.abs(v) <= b)
        else:
            m = (u / a) ** 2 + (v / b) ** 2 <= 1.0
        img[y0:y1, x0:x1][m] = level
    # value-noise texture: +-24 on an 8-px lattice, bilinear (integer arithmetic)
    gh, gw = height // 8 + 2, width // 8 + 2
    lat = g.integers(-24, 25, size=(gh, gw)).astype(np.int32)
    iy, fy = yy // 8, yy % 8
    ix, fx = xx // 8, xx % 8
    tex = (lat[iy, ix] * (8 - fx) * (8 - fy) + lat[iy, ix + 1] * fx * (8 - fy)
           + lat[iy + 1, ix] * (8 - fx) * fy + lat[iy + 1, ix + 1] * fx * fy) // 64
    img = img + tex + g.integers(-6, 7, size=(height, width))
    return np.ascontiguousarray(np.clip(img, 0, 255).astype(np.uint8))


def _frame_args(args):
    return frame(*args)


def frames(n: int, width: int = 640, height: int = 480, first_seed: int = 0, workers: int = 1) -> np.ndarray:
    """Batch of n frames, shape (n, height, width) uint8; frame i uses seed first_seed+i.

    workers > 1 renders in a process pool (call it before the process touches the GPU)."""
    out = np.empty((n, height, width), dtype=np.uint8)
    args = [(first_seed + i, width, height) for i in range(n)]
    if workers > 1 and n > 1:
        import multiprocessing as mp
        # close + join (not the context manager's terminate): workers exit on their own, so
        # a profiler's signal handlers inherited by the fork never log a SIGTERM abort
        pool = mp.get_context("fork").Pool(min(workers, n))
        try:
            for i, f in enumerate(pool.imap(_frame_args, args, chunksize=4)):
                out[i] = f
        finally:
            pool.close()
            pool.join()
    else:
        for i, a in enumerate(args):
            out[i] = frame(*a)
    return out


def shifted_pair(seed: int, width: int = 640, height: int = 480, dx: int = 7, dy: int = -4, margin: int = 32):
    """Two views of one canvas, the second shifted by (dx, dy) pixels: a pixel (x, y) of
    the first view appears at (x - dx, y - dy) in the second (a fronto-parallel scene
    under camera translation)."""
    canvas = frame(seed, width + 2 * margin, height + 2 * margin)
    a = canvas[margin:margin + height, margin:margin + width]
    b = canvas[margin + dy:margin + dy + height, margin + dx:margin + dx + width]
    return np.ascontiguousarray(a), np.ascontiguousarray(b)


def sequence(seed: int, n: int, width: int = 640, height: int = 480, step: int = 3, margin: int = 64):
    """n views of one canvas along a random walk of up to `step` px per frame (for
    frame-to-frame matching benchmarks).  Returns (frames (n, h, w), offsets (n, 2))."""
    canvas = frame(seed, width + 2 * margin, height + 2 * margin)
    g = _rng(seed + 7)
    off = np.zeros((n, 2), dtype=np.int64)
    for i in range(1, n):
        off[i] = np.clip(off[i - 1] + g.integers(-step, step + 1, 2), -margin, margin)
    out = np.empty((n, height, width), dtype=np.uint8)
    for i in range(n):
        ox, oy = margin + off[i, 0], margin + off[i, 1]
        out[i] = canvas[oy:oy + height, ox:ox + width]
    return out, off


def plane_views(seed: int, rel_poses, width: int = 640, height: int = 480, fx: float = 500.0, fy: float = 500.0,
                cx: float = 320.0, cy: float = 240.0, z0: float = 5.0):
    """Views of one textured plane under general camera motion (rotation about any axis,
    motion along the optical axis).

    The plane is Z = z0 in the frame of a reference camera that sees the canvas' central
    width x height crop pixel for pixel.  rel_poses[k] is camera k's pose relative to that
    camera (4x4, X_k = R X_ref + t).  Pixel (u, v) of camera k is the ray from its centre
    C = -R^T t along R^T K^-1 (u, v, 1); where it meets the plane, (X, Y, z0), it reads the
    canvas at (fx X / z0 + cx, fy Y / z0 + cy) + margin, bilinearly (float64, rounded).
    The canvas is sized so that every view fits inside it.

    Returns (views (n, h, w) u8, depths (n, h, w) f32), depths being each pixel's Z in its
    own camera (the ray parameter, as K^-1 (u, v, 1) has unit z)."""
    Kinv = np.array([[1 / fx, 0, -cx / fx], [0, 1 / fy, -cy / fy], [0, 0, 1]], np.float64)
    vv, uu = np.mgrid[0:height, 0:width].astype(np.float64)
    rays = np.stack([uu, vv, np.ones_like(uu)], -1) @ Kinv.T          # (h, w, 3), unit z
    hits = []
    for T in rel_poses:
        T = np.asarray(T, np.float64)
        R, t = T[:3, :3], T[:3, 3]
        C = -R.T @ t
        a = rays @ R                                                  # R^T ray, per pixel
        if (a[..., 2] <= 0).any():
            raise ValueError("a view looks away from the plane")
        s = (z0 - C[2]) / a[..., 2]
        if (s <= 0).any():
            raise ValueError("the plane is behind a camera")
        X = C[None, None, :] + s[..., None] * a
        hits.append((fx * X[..., 0] / z0 + cx, fy * X[..., 1] / z0 + cy, s))
    lo_x = min(float(h[0].min()) for h in hits)
    hi_x = max(float(h[0].max()) for h in hits)
    lo_y = min(float(h[1].min()) for h in hits)
    hi_y = max(float(h[1].max()) for h in hits)
    mx = int(np.ceil(max(0.0, -lo_x, hi_x - (width - 1)))) + 2
    my = int(np.ceil(max(0.0, -lo_y, hi_y - (height - 1)))) + 2
    W, H = width + 2 * mx, height + 2 * my
    canvas = frame(seed, W, H, n_shapes=int(200 * W * H / (640 * 480))).astype(np.float64)
    views = np.empty((len(hits), height, width), np.uint8)
    depths = np.empty((len(hits), height, width), np.float32)
    for k, (px, py, s) in enumerate(hits):
        px = px + mx
        py = py + my
        x0 = np.clip(np.floor(px).astype(np.int64), 0, W - 2)
        y0 = np.clip(np.floor(py).astype(np.int64), 0, H - 2)
        ax = np.clip(px - x0, 0.0, 1.0)
        ay = np.clip(py - y0, 0.0, 1.0)
        v = ((1 - ax) * (1 - ay) * canvas[y0, x0] + ax * (1 - ay) * canvas[y0, x0 + 1]
             + (1 - ax) * ay * canvas[y0 + 1, x0] + ax * ay * canvas[y0 + 1, x0 + 1])
        views[k] = np.clip(np.rint(v), 0, 255).astype(np.uint8)
        depths[k] = s.astype(np.float32)
    return views, depths


def _plane_hits(T, width, height, fx, fy, cx, cy, z0, pixels=None, rays=None):
    """Canvas coordinates (px, py) and ray depth s where camera T's pixel rays meet the
    plane Z = z0 of the reference camera (every pixel, or the (u, v) rows of `pixels`, or
    the given unit-z camera rays)."""
    Kinv = np.array([[1 / fx, 0, -cx / fx], [0, 1 / fy, -cy / fy], [0, 0, 1]], np.float64)
    if rays is not None:
        pass
    elif pixels is None:
        vv, uu = np.mgrid[0:height, 0:width].astype(np.float64)
        rays = np.stack([uu, vv, np.ones_like(uu)], -1) @ Kinv.T
    else:
        p = np.asarray(pixels, np.float64)
        rays = np.stack([p[:, 0], p[:, 1], np.ones(len(p))], -1) @ Kinv.T
    T = np.asarray(T, np.float64)
    R, t = T[:3, :3], T[:3, 3]
    C = -R.T @ t
    a = rays @ R
    if (a[..., 2] <= 0).any():
        raise ValueError("a view looks away from the plane")
    s = (z0 - C[2]) / a[..., 2]
    if (s <= 0).any():
        raise ValueError("the plane is behind a camera")
    X = C + s[..., None] * a
    return fx * X[..., 0] / z0 + cx, fy * X[..., 1] / z0 + cy, s


_PLANE_CANVAS = None  # (canvas, mx, my[, rays]): shared with forked render workers


def _render_plane_view(args):
    T, width, height, fx, fy, cx, cy, z0 = args[:8]
    canvas, mx, my = _PLANE_CANVAS[:3]
    rays = _PLANE_CANVAS[3] if len(_PLANE_CANVAS) > 3 else None
    px, py, s = _plane_hits(T, width, height, fx, fy, cx, cy, z0, rays=rays)
    if len(args) > 8:  # RGB-D: the view and its registered depth image
        img = _sample(canvas, px + mx, py + my)
        return img, _depth_image(s, *args[8:])
    return _sample(canvas, px + mx, py + my)


def _sample(canvas, px, py):
    """Bilinear canvas read at (px, py), rounded to u8."""
    H, W = canvas.shape
    x0 = np.clip(np.floor(px).astype(np.int64), 0, W - 2)
    y0 = np.clip(np.floor(py).astype(np.int64), 0, H - 2)
    ax = np.clip(px - x0, 0.0, 1.0)
    ay = np.clip(py - y0, 0.0, 1.0)
    v = ((1 - ax) * (1 - ay) * canvas[y0, x0] + ax * (1 - ay) * canvas[y0, x0 + 1]
         + (1 - ax) * ay * canvas[y0 + 1, x0] + ax * ay * canvas[y0 + 1, x0 + 1])
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def tiled_canvas(seed: int, width: int, height: int, workers: int = 1, tile=(640, 480)) -> np.ndarray:
    """A large texture made of frame() tiles (seeds seed*1000 + k): the shapes keep a
    640x480 frame's scale, and the cost grows with the area only."""
    tw, th = tile
    nx, ny = (width + tw - 1) // tw, (height + th - 1) // th
    tiles = frames(nx * ny, tw, th, first_seed=int(seed) * 1000, workers=workers)
    out = tiles.reshape(ny, nx, th, tw).transpose(0, 2, 1, 3).reshape(ny * th, nx * tw)
    return np.ascontiguousarray(out[:height, :width])


def plane_stereo_views(seed: int, rel_poses, baseline: float, width: int, height: int, fx: float, fy: float,
                       cx: float, cy: float, z0: float, workers: int = 1):
    """Rectified stereo pairs of one textured plane (the plane_views scene) under the left
    cameras' poses rel_poses[k] (relative to the reference camera, 4x4): the right camera
    has the left one's orientation and sits `baseline` along its x axis, so a point at depth
    z appears fx*baseline/z px further left in it (Frame::ComputeStereoMatches' model).  The
    canvas is sized from the views' corner rays (the pixel-to-canvas map is a homography,
    so its extremes over the image are at the corners).  workers > 1 renders in a forked
    process pool (before the process touches the GPU).
    Returns (left (n, h, w) u8, right (n, h, w) u8)."""
    global _PLANE_CANVAS
    rights = []
    for T in rel_poses:
        T = np.asarray(T, np.float64)
        Tr = T.copy()
        Tr[0, 3] -= baseline  # C_r = C_l + R^T (b, 0, 0)  =>  t_r = t_l - (b, 0, 0)
        rights.append(Tr)
    poses = [np.asarray(T, np.float64) for T in rel_poses] + rights
    corners = [(0, 0), (width - 1, 0), (0, height - 1), (width - 1, height - 1)]
    hx, hy = [], []
    for T in poses:
        px, py, _ = _plane_hits(T, width, height, fx, fy, cx, cy, z0, corners)
        hx += [px.min(), px.max()]
        hy += [py.min(), py.max()]
    mx = 3 - int(np.floor(min(hx)))  # canvas origin: the views' canvas coordinates + (mx, my)
    my = 3 - int(np.floor(min(hy)))
    W = int(np.ceil(max(hx))) + mx + 4
    H = int(np.ceil(max(hy))) + my + 4
    canvas = tiled_canvas(seed, W, H, workers).astype(np.float64)
    _PLANE_CANVAS = (canvas, mx, my)
    args = [(T, width, height, fx, fy, cx, cy, z0) for T in poses]
    try:
        if workers > 1 and len(args) > 1:
            import multiprocessing as mp
            pool = mp.get_context("fork").Pool(min(workers, len(args)))
            try:
                views = list(pool.imap(_render_plane_view, args, chunksize=2))
            finally:
                pool.close()
                pool.join()
        else:
            views = [_render_plane_view(a) for a in args]
    finally:
        _PLANE_CANVAS = None
    n = len(rel_poses)
    return np.stack(views[:n]), np.stack(views[n:])


# TUM freiburg1 (ORB-SLAM2's Examples/RGB-D/TUM1.yaml): intrinsics, distortion k1 k2 p1 p2
# k3, Camera.bf, ThDepth, DepthMapFactor
TUM1 = dict(fx=517.306408, fy=516.469215, cx=318.643040, cy=255.313989,
            dist=(0.262383, -0.953104, -0.005358, 0.002628, 1.163314), bf=40.0, th_depth=40.0,
            depth_map_factor=5000.0)


def distorted_rays(width: int, height: int, fx: float, fy: float, cx: float, cy: float, dist, iters: int = 40):
    """Unit-z camera rays (h, w, 3) of the pixels of a distorted image (OpenCV's
    Brown-Conrady model, k1 k2 p1 p2 k3): each pixel's undistorted normalised coordinates by
    fixed-point inversion in float64 (a rendering model, independent of the undistortion the
    Frame restates)."""
    k1, k2, p1, p2, k3 = (list(dist) + [0.0] * 5)[:5]
    vv, uu = np.mgrid[0:height, 0:width].astype(np.float64)
    xd, yd = (uu - cx) / fx, (vv - cy) / fy
    x, y = xd.copy(), yd.copy()
    for _ in range(iters):
        r2 = x * x + y * y
        radial = 1 + r2 * (k1 + r2 * (k2 + r2 * k3))
        dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
        dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
        x, y = (xd - dx) / radial, (yd - dy) / radial
    return np.stack([x, y, np.ones_like(x)], -1)


def _depth_image(s, seed, depth_map_factor, holes):
    """A TUM-style 16-bit depth image of per-pixel depths s (metres): round(s * factor),
    saturated, with Kinect-like holes (0) when `holes`: a 6-12 px invalid band at the left
    border (the projector's shadow), a few random blobs and 1 % speckle."""
    d = np.clip(np.rint(s * depth_map_factor), 0, 65535).astype(np.uint16)
    if holes:
        g = _rng(seed)
        h, w = d.shape
        d[:, :int(g.integers(6, 13))] = 0
        yy, xx = np.mgrid[0:h, 0:w]
        for _ in range(int(g.integers(2, 6))):
            cx, cy = g.integers(0, w), g.integers(0, h)
            a, b = g.integers(8, 48), g.integers(8, 48)
            d[((xx - cx) / a) ** 2 + ((yy - cy) / b) ** 2 <= 1.0] = 0
        d[g.random((h, w)) < 0.01] = 0
    return d


def plane_rgbd_views(seed: int, rel_poses, width: int, height: int, fx: float, fy: float, cx: float, cy: float,
                     dist, z0: float, depth_map_factor: float = 5000.0, holes: bool = True, workers: int = 1):
    """RGB-D frames of one textured plane (the plane_views scene) seen by a camera with lens
    distortion `dist`: the gray image is rendered through the distorted pixels' rays
    (distorted_rays), and the depth image registered to it (TUM's depth is aligned with the
    RGB image) holds each pixel's Z in its camera, as 16-bit round(Z * depth_map_factor),
    with holes (_depth_image).  Returns (gray (n, h, w) u8, depth (n, h, w) u16)."""
    global _PLANE_CANVAS
    rays = distorted_rays(width, height, fx, fy, cx, cy, dist)
    border = np.concatenate([rays[0], rays[-1], rays[:, 0], rays[:, -1]])
    hx, hy = [], []
    for T in rel_poses:
        px, py, _ = _plane_hits(T, width, height, fx, fy, cx, cy, z0, rays=border)
        hx += [px.min(), px.max()]
        hy += [py.min(), py.max()]
    mx = 3 - int(np.floor(min(hx)))
    my = 3 - int(np.floor(min(hy)))
    W = int(np.ceil(max(hx))) + mx + 4
    H = int(np.ceil(max(hy))) + my + 4
    canvas = tiled_canvas(seed, W, H, workers).astype(np.float64)
    _PLANE_CANVAS = (canvas, mx, my, rays)
    args = [(np.asarray(T, np.float64), width, height, fx, fy, cx, cy, z0, seed * 7919 + k, depth_map_factor, holes)
            for k, T in enumerate(rel_poses)]
    try:
        if workers > 1 and len(args) > 1:
            import multiprocessing as mp
            pool = mp.get_context("fork").Pool(min(workers, len(args)))
            try:
                out = list(pool.imap(_render_plane_view, args, chunksize=2))
            finally:
                pool.close()
                pool.join()
        else:
            out = [_render_plane_view(a) for a in args]
    finally:
        _PLANE_CANVAS = None
    return np.stack([o[0] for o in out]), np.stack([o[1] for o in out])


def tum_walk(seed: int, n: int, yaw0: float = 30.0, z0: float = 2.2):
    """Relative poses (4x4, camera from reference) of a hand-held TUM-like RGB-D walk past
    the textured plane Z = z0: the camera looks at the plane yawed by yaw0 +- 4 degrees, so
    depths across a 640x480 view span about 1.9 m to 4.2 m (both sides of TUM1's mThDepth =
    bf * 40 / fx = 3.09 m); per step it moves 0.09-0.13 m forward or back along its optical
    axis (|dz| > mb = bf / fx = 0.077 m: ORBmatcher.cc:1650-1651's bForward / bBackward) or
    less than 0.04 m (a third each; the centre kept within 0.45 m of the reference camera
    along z and 0.6 m sideways), sideways by up to 0.03 m, and rolls 0.5-3 degrees either
    way (bounded by 8)."""
    g = _rng(seed + 911)
    yaw, roll, pitch = 0.0, 0.0, 0.0
    c = np.zeros(3)
    rels = []
    for k in range(n):
        if k:
            kind = g.integers(0, 3)
            dz = g.uniform(0.09, 0.13) if kind == 0 else (-g.uniform(0.09, 0.13) if kind == 1 else g.uniform(-0.04, 0.04))
            step = g.uniform(0.5, 3.0) * (1 if g.random() < 0.5 else -1)
            roll = roll + step if abs(roll + step) <= 8.0 else roll - step
            yaw = float(np.clip(yaw + g.uniform(-1.0, 1.0), -4.0, 4.0))
            pitch = float(np.clip(pitch + g.uniform(-0.5, 0.5), -2.0, 2.0))
            R = rotation("y", yaw0 + yaw) @ rotation("z", roll) @ rotation("x", pitch)
            d = R.T @ np.array([g.uniform(-0.03, 0.03), g.uniform(-0.02, 0.02), dz])
            if not (-0.45 <= c[2] + d[2] <= 0.45 and -0.6 <= c[0] + d[0] <= 0.6):
                d = -d
            c = c + d
        R = rotation("y", yaw0 + yaw) @ rotation("z", roll) @ rotation("x", pitch)
        rels.append(camera_pose(R, c.copy()))
    return rels


def kitti_walk(seed: int, n: int, yaw0: float = 25.0):
    """Relative poses (4x4, camera from reference) of a KITTI-like stereo walk past the
    textured plane Z = 15 m: the cameras look at the plane yawed by yaw0 +- 4 degrees, so
    depths across a 1241x376 view span about 12 m to 28 m (both sides of KITTI's mThDepth
    = bf * 35 / fx = 18.8 m); each step moves the camera along its own optical axis by
    0.6-0.95 m forward, 0.6-0.95 m back (|dz| > mb = 0.54 m: ORBmatcher.cc:1650-1651's
    bForward / bBackward) or less than 0.3 m (a third each; the centre kept 12-18 m from the
    plane and within 4 m of the reference camera sideways),
    sideways by up to 0.15 m, and rolls it by 1-4 degrees either way (bounded by 10)."""
    g = _rng(seed + 313)
    yaw, roll, pitch = 0.0, 0.0, 0.0
    c = np.zeros(3)
    rels = []
    for k in range(n):
        if k:
            kind = g.integers(0, 3)
            dz = g.uniform(0.6, 0.95) if kind == 0 else (-g.uniform(0.6, 0.95) if kind == 1 else g.uniform(-0.3, 0.3))
            step = g.uniform(1.0, 4.0) * (1 if g.random() < 0.5 else -1)
            roll = roll + step if abs(roll + step) <= 10.0 else roll - step
            yaw = float(np.clip(yaw + g.uniform(-1.0, 1.0), -4.0, 4.0))
            pitch = float(np.clip(pitch + g.uniform(-0.4, 0.4), -1.5, 1.5))
            R = rotation("y", yaw0 + yaw) @ rotation("z", roll) @ rotation("x", pitch)
            d = R.T @ np.array([g.uniform(-0.15, 0.15), g.uniform(-0.05, 0.05), dz])
            if not (-3.0 <= c[2] + d[2] <= 3.0 and -4.0 <= c[0] + d[0] <= 4.0):
                d = -d
            c = c + d
        R = rotation("y", yaw0 + yaw) @ rotation("z", roll) @ rotation("x", pitch)
        rels.append(camera_pose(R, c.copy()))
    return rels


def rotation(axis: str, degrees: float) -> np.ndarray:
    """3x3 rotation about the camera's x, y or z (optical) axis."""
    a = np.deg2rad(degrees)
    c, s = np.cos(a), np.sin(a)
    if axis == "x":
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    if axis == "y":
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def camera_pose(R, centre) -> np.ndarray:
    """4x4 Tcw of a camera with orientation R (world -> camera) and centre `centre`."""
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = -np.asarray(R, np.float64) @ np.asarray(centre, np.float64)
    return T


class StereoSequence:
    """Rectified stereo views of one fronto-parallel textured plane along a random walk
    (configs[3]'s EuRoC-shaped stream).  The left camera of view i sits at canvas offset
    off[i] (up to `step` px per axis per frame); the right camera, one stereo baseline to
    its right, sees the plane `disp` px further along x, so right(x) = left(x + disp)
    exactly.  views(idx) renders only the listed views (a rank renders its own shard)."""

    def __init__(self, seed: int, n: int, width: int = 752, height: int = 480, step: int = 8, margin: int = 128,
                 disp: int = 13, canvas_seed: int | None = None):
        """canvas_seed (default: seed) draws the texture; the walk always comes from seed,
        so streams that differ only in canvas_seed share their poses."""
        self.width, self.height, self.margin, self.disp = width, height, margin, disp
        self.canvas = frame(seed if canvas_seed is None else canvas_seed, width + 2 * margin + disp,
                            height + 2 * margin, n_shapes=320)
        g = _rng(seed + 7)
        off = np.zeros((n, 2), dtype=np.int64)
        for i in range(1, n):
            off[i] = np.clip(off[i - 1] + g.integers(-step, step + 1, 2), -margin, margin)
        self.off = off

    def views(self, idx):
        idx = list(idx)
        W, H, m, d = self.width, self.height, self.margin, self.disp
        left = np.empty((len(idx), H, W), dtype=np.uint8)
        right = np.empty_like(left)
        for k, i in enumerate(idx):
            ox, oy = m + self.off[i, 0], m + self.off[i, 1]
            left[k] = self.canvas[oy:oy + H, ox:ox + W]
            right[k] = self.canvas[oy:oy + H, ox + d:ox + d + W]
        return left, right


def stereo_pair(seed: int, width: int = 1241, height: int = 376, max_disp: int = 64):
    """(left, right, disparity) with right(x) = left(x + d) for a blockwise d field."""
    left = frame(seed, width, height)
    g = _rng(seed + 1_000_003)
    bh, bw = (height + 31) // 32, (width + 31) // 32
    dblk = g.integers(0, max_disp + 1, size=(bh, bw))
    disp = np.repeat(np.repeat(dblk, 32, axis=0), 32, axis=1)[:height, :width]
    xs = np.minimum(np.arange(width)[None, :] + disp, width - 1)
    right = np.take_along_axis(left, xs, axis=1)
    return left, np.ascontiguousarray(right), disp.astype(np.int32)


def vocabulary_text(seed: int, k: int = 10, L: int = 6, scoring: int = 0, weighting: int = 0,
                    centres: np.ndarray | None = None) -> bytes:
    """A complete k-ary, depth-L vocabulary in loadFromTextFile format (TemplatedVocabulary.h:
    1338-1424), nodes in level order (siblings contiguous, like the reference's creation
    order).  Stands in for ORBvoc.txt (k=10, L=6, ~1.1M nodes), which the reference does
    not ship.  Child descriptors are bit-flipped copies of their parent's (fewer flips
    deeper).  If `centres` (M x 32 uint8, e.g. extracted ORB descriptors) is given, the
    level-1 nodes start from them, so real descriptors spread over the whole tree.
    Columns are fixed-width (whitespace-separated like the reference's own files)."""
    rng = _rng(seed)
    levels_desc, levels_parent = [], []
    if centres is not None and len(centres):
        d1 = np.asarray(centres, np.uint8)[rng.integers(0, len(centres), k)]
    else:
        d1 = rng.integers(0, 256, (k, 32), dtype=np.uint8)
    levels_desc.append(d1)
    levels_parent.append(np.zeros(k, np.int64))
    first_id = 1
    for depth in range(2, L + 1):
        prev = levels_desc[-1]
        n_prev = len(prev)
        d = np.repeat(prev, k, axis=0)
        q = 24.0 / 256.0 / (depth - 1)  # per-bit flip probability: ~24 bits at level 2, fewer deeper
        flips = np.concatenate([np.packbits(rng.random((min(1 << 16, len(d) - i), 256), np.float32) < q, axis=1)
                                for i in range(0, len(d), 1 << 16)])
        levels_desc.append(d ^ flips)
        levels_parent.append(np.repeat(np.arange(first_id, first_id + n_prev, dtype=np.int64), k))
        first_id += n_prev
    desc = np.concatenate(levels_desc)
    parent = np.concatenate(levels_parent)
    n = len(desc)
    leaf = np.zeros(n, np.int64)
    leaf[n - len(levels_desc[-1]):] = 1
    # weights: 5-decimal values in [0.05, 9.99999] on leaves (IDF-like), a few stopped
    # (0) words, 0 on inner nodes
    wq = rng.integers(5000, 1000000, n)
    wq[rng.random(n) < 0.02] = 0
    wq[leaf == 0] = 0

    def digits(v: np.ndarray, width: int) -> np.ndarray:
        out = np.empty((len(v), width), np.uint8)
        x = v.copy()
        for c in range(width - 1, -1, -1):
            out[:, c] = ord("0") + x % 10
            x //= 10
        return out

    sp = np.full((n, 1), ord(" "), np.uint8)
    cols = [digits(parent, 7), sp, (ord("0") + leaf).astype(np.uint8)[:, None], sp]
    table = np.array([[ord(c) for c in f"{i:3d} "] for i in range(256)], np.uint8)
    cols.append(table[desc].reshape(n, 128))
    w = digits(wq, 6)
    cols += [sp, w[:, :1], np.full((n, 1), ord("."), np.uint8), w[:, 1:], np.full((n, 1), ord("\n"), np.uint8)]
    body = np.concatenate(cols, axis=1).tobytes()
    return f"{k} {L}  {scoring} {weighting}\n".encode() + body
