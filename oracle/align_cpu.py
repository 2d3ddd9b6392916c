"""CPU oracle for the face-alignment ingest and the
fixed-mask resize (§8(a) a3).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module -- as the checker,
never as the thing measured or shipped.  The product path (``latentsync_amd.align``
and ``latentsync_amd.pipeline.load_fixed_mask``) runs on the HIP kernels of
``ls_restore.hip``.

Restates, in numpy:
  * ``cv2.resize(img, (w, h), interpolation=cv2.INTER_LANCZOS4)`` for uint8 images
    (load_fixed_mask, latentsync/utils/image_processor.py:31-36; the aligned face's
    resize, :141) -- OpenCV's generic resize (resize.cpp: resize's own
    interpolateLanczos4, resizeGeneric_ tables, HResizeLanczos4 / VResizeLanczos4,
    FixedPtCast<int, uchar, 22>);
  * ``transformation_from_points`` (latentsync/utils/affine_transform.py:7-32) and
    ``AlignRestore.align_warp_face`` (:53-70): warpAffine INTER_LANCZOS4 with
    BORDER_CONSTANT 127 into the 210x280 face (remapLanczos4 fixed point);
  * ``ImageProcessor.affine_transform``'s landmark reduction (image_processor.py:131-141)
    and ``laplacianSmooth`` (affine_transform.py:118-144).

Pinning: OpenCV (cv2 4.x) and the landmark model are neither in /root/reference nor
installed here -- **parity unpinned**.  The resize follows OpenCV's generic C++ path;
a cv2 build that dispatches uint8 Lanczos resizes to IPP may differ at edges.  The
numpy steps (transformation_from_points, laplacianSmooth) restate the reference's own
source.
"""
import math

import numpy as np

from oracle.restore_cpu import COEF_BITS, _fixed_coords, lanczos4_tab_i16

# AlignRestore(align_points=3) constants (affine_transform.py:36-44)
RATIO = 2.8
FACE_TEMPLATE = np.array([[19 - 2, 30 - 10], [56 + 2, 30 - 10], [37.5, 45 - 5]]) * RATIO
FACE_SIZE = (int(75 * RATIO), int(100 * RATIO))  # (w, h) = (210, 280)


# --------------------------------------------------------------------------
# cv2.resize INTER_LANCZOS4, uint8
# --------------------------------------------------------------------------


def resize_lanczos4_coeffs(x):
    """resize.cpp interpolateLanczos4: float (x+3) and (x+3-i), double sin/cos."""
    x = np.float32(x)
    x3 = np.float32(x + np.float32(3))
    s45 = 0.70710678118654752440084436210485
    cs = [(1, 0), (-s45, -s45), (0, 1), (s45, -s45), (-1, 0), (s45, s45), (0, -1), (-s45, s45)]
    y0 = float(-x3) * math.pi * 0.25
    s0, c0 = math.sin(y0), math.cos(y0)
    c = np.zeros(8, np.float32)
    ssum = np.float32(0)
    for i in range(8):
        yy = np.float32(x3 - np.float32(i))
        if abs(yy) >= np.float32(1e-6):
            y = float(-yy) * math.pi * 0.25
            c[i] = np.float32((cs[i][0] * s0 + cs[i][1] * c0) / (y * y))
        else:
            c[i] = np.float32(1e30)
        ssum = np.float32(ssum + c[i])
    inv = np.float32(np.float32(1) / ssum)
    return (c * inv).astype(np.float32)


def resize_axis(src_n, dst_n):
    """resizeGeneric_ offsets (floor of (d+0.5)*scale-0.5 in float) and int16
    coefficients saturate_cast<short>(c * 2048) for one axis."""
    scale = 1.0 / (dst_n / src_n)
    ofs = np.zeros(dst_n, np.int64)
    coef = np.zeros((dst_n, 8), np.int64)
    for d in range(dst_n):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = int(np.floor(f))
        f = np.float32(f - np.float32(s))
        c = resize_lanczos4_coeffs(f)
        ofs[d] = s
        coef[d] = np.clip(np.rint((c * np.float32(2048)).astype(np.float32)), -32768, 32767)
    return ofs, coef


def resize_lanczos4_u8(img, dst_h, dst_w):
    """cv2.resize(img u8 (h,w) or (h,w,C), (dst_w, dst_h), INTER_LANCZOS4)."""
    img = np.asarray(img)
    squeeze = img.ndim == 2
    src = img[..., None] if squeeze else img
    h, w, C = src.shape
    if (h, w) == (dst_h, dst_w):
        return img.copy()
    ox, ax = resize_axis(w, dst_w)
    oy, ay = resize_axis(h, dst_h)
    xi = np.clip(ox[:, None] - 3 + np.arange(8)[None, :], 0, w - 1)       # (dst_w, 8)
    yi = np.clip(oy[:, None] - 3 + np.arange(8)[None, :], 0, h - 1)       # (dst_h, 8)
    s = src.astype(np.int64)
    # horizontal pass: every source row, int sums of u8 * int16
    hrows = np.einsum("hxjc,xj->hxc", s[:, xi, :], ax)                      # (h, dst_w, C)
    # vertical pass over the 8 clamped rows
    v = np.einsum("ykxc,yk->yxc", hrows[yi], ay)                            # (dst_h, dst_w, C)
    out = np.clip((v + (1 << 21)) >> 22, 0, 255).astype(np.uint8)
    return out[..., 0] if squeeze else out


# --------------------------------------------------------------------------
# face alignment
# --------------------------------------------------------------------------


def transformation_from_points(points1, points0, smooth=True, p_bias=None):
    """affine_transform.py:7-32 (float64 numpy, SVD Procrustes + the smoothed bias)."""
    points2 = np.array(points0).astype(np.float64)
    points1 = np.array(points1).astype(np.float64)
    c1, c2 = points1.mean(axis=0), points2.mean(axis=0)
    points1 = points1 - c1
    points2 = points2 - c2
    s1, s2 = np.std(points1), np.std(points2)
    points1 = points1 / s1
    points2 = points2 / s2
    U, S, Vt = np.linalg.svd(points1.T @ points2)
    R = (U @ Vt).T
    M = np.concatenate(((s2 / s1) * R, c2.reshape(2, 1) - (s2 / s1) * (R @ c1.reshape(2, 1))), axis=1)
    if smooth:
        bias = points2[2] - points1[2]
        if p_bias is not None:
            bias = p_bias * 0.2 + bias * 0.8
        p_bias = bias
        M[:, 2] = M[:, 2] + bias
    return M, p_bias


def laplacian_smooth(seq68, alpha=0.3):
    """laplacianSmooth.smooth over a sequence of (68,2) landmark arrays."""
    last, out = None, []
    for pts in seq68:
        pts = np.asarray(pts, np.float64)
        if last is None:
            last = pts.copy()
            out.append(pts.copy())
            continue
        width = pts[:, 0].max() - pts[:, 0].min()
        d2 = ((pts - last) ** 2).sum(axis=1)
        wgt = np.exp(-d2 / (width * alpha))[:, None]
        upd = last * wgt + pts * (1 - wgt)
        last = upd.copy()
        out.append(upd)
    return out


def lmk3(points68):
    """image_processor.py:132-135: brow centres and nose centre."""
    p = np.asarray(points68, np.float64)
    return np.stack([p[17:22].mean(0), p[22:27].mean(0), p[27:36].mean(0)])


def warp_lanczos_border_u8(src, M, H, W, border, tab):
    """warpAffine(src, ., (W,H), INTER_LANCZOS4, BORDER_CONSTANT border) with the
    dst->src matrix M: taps outside the source read the border value."""
    h, w, C = src.shape
    sx, sy, a = _fixed_coords(M, H, W)
    sx, sy = sx - 3, sy - 3
    wt = tab[a].astype(np.int64).reshape(H, W, 8, 8)
    acc = np.zeros((H, W, C), np.int64)
    for r in range(8):
        yy = sy + r
        for c in range(8):
            xx = sx + c
            ok = (yy >= 0) & (yy < h) & (xx >= 0) & (xx < w)
            v = src[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)].astype(np.int64)
            acc += np.where(ok[..., None], v, border) * wt[:, :, r, c][..., None]
    return np.clip((acc + (1 << (COEF_BITS - 1))) >> COEF_BITS, 0, 255).astype(np.uint8)


def warpaffine_dst_to_src(M):
    """warpAffine without WARP_INVERSE_MAP inverts M itself (imgwarp.cpp order)."""
    m = np.asarray(M, np.float64).reshape(6).copy()
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = m[4] * D, m[0] * D
    m[0] = A11
    m[1] *= -D
    m[3] *= -D
    m[4] = A22
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    return m


def affine_transform_video(frames, landmarks68, resolution):
    """affine_transform_video (latentsync/pipelines/affine_transform_video.py:8-35)
    with the landmarks given: per frame smooth -> lmk3 -> transformation_from_points
    (p_bias carried) -> align warp (border 127) -> resize to the resolution ->
    (faces uint8 (N,3,R,R), boxes, affine matrices)."""
    tab = lanczos4_tab_i16()
    faces, boxes, mats, p_bias = [], [], [], None
    fw, fh = FACE_SIZE
    for frame, pts in zip(frames, laplacian_smooth(landmarks68)):
        M, p_bias = transformation_from_points(lmk3(pts), FACE_TEMPLATE, True, p_bias)
        face = warp_lanczos_border_u8(np.asarray(frame), warpaffine_dst_to_src(M), fh, fw, 127, tab)
        boxes.append([0, 0, face.shape[1], face.shape[0]])
        face = resize_lanczos4_u8(face, resolution, resolution)
        faces.append(face.transpose(2, 0, 1))
        mats.append(M)
    return np.stack(faces), boxes, mats
