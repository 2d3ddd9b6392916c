"""CPU oracle for the paste-back warp (``LipsyncPipeline.restore_video``).

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module -- as the checker,
never as the thing measured or shipped.  The product path
(``latentsync_amd.restore``) runs on the HIP kernels of ``ls_restore.hip``.

Restates, in numpy, what the reference does per face
(latentsync/pipelines/lipsync_pipeline.py:343-358 ``restore_video`` and
latentsync/utils/affine_transform.py:85-115 ``AlignRestore.restore_img``):

  1. torchvision ``resize(face, (h, w), antialias=True)`` on the decoded face,
     ``(x / 2 + 0.5).clamp(0, 1) * 255 -> uint8``  (lipsync_pipeline.py:351-354)
  2. ``cv2.resize`` of the frame to the same size (identity: cv2 copies when
     dsize == ssize, upscale_factor = 1)                (affine_transform.py:87-88)
  3. ``cv2.invertAffineTransform`` + ``cv2.warpAffine(face, inv, (W, H),
     INTER_LANCZOS4)``                                      (:89-95)
  4. ``cv2.warpAffine(ones, inv, (W, H))`` (INTER_LINEAR), ``cv2.erode`` 2x2 (:96-100)
  5. area -> w_edge = int(sqrt(area)) // 20; erode (2 w_edge)^2; GaussianBlur
     (2 w_edge + 1)^2, sigma 0                               (:101-107)
  6. soft * (mask * restored) + (1 - soft) * frame -> uint8 (:108-114)

Pinning.  Step 1 is pinned: it calls torch's own ``F.interpolate(...,
antialias=True)``, which is exactly what torchvision's tensor ``resize`` runs.
Steps 2-6 are OpenCV (cv2 4.x, ``requirements.txt``), which is neither in
/root/reference nor installed here -- **parity unpinned**: they are restated
from OpenCV's published algorithm (imgwarp.cpp WarpAffineInvoker / remapLanczos4 /
remapBilinear fixed-point tables, morph.cpp rectangular erode, smooth.dispatch.cpp
getGaussianKernelBitExact + filter.cpp sepFilter2D with BORDER_REFLECT_101).
OpenCV may dispatch IPP for GaussianBlur; the restatement follows the generic
C++ path.  Summation orders are written out so the HIP kernels can reproduce
them bit for bit.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

INTER_BITS = 5
INTER_TAB = 1 << INTER_BITS  # 32 sub-pixel positions per axis
AB_BITS = 10
AB_SCALE = 1 << AB_BITS
COEF_BITS = 15
COEF_SCALE = 1 << COEF_BITS


# --------------------------------------------------------------------------
# 1. face resize (torchvision resize antialias=True == F.interpolate aa)
# --------------------------------------------------------------------------


def face_resize_u8(faces, out_h, out_w):
    """faces float (N,3,R,R) in [-1,1] -> uint8 (N,out_h,out_w,3)
    (lipsync_pipeline.py:351-354)."""
    f = F.interpolate(faces.float(), size=(out_h, out_w), mode="bilinear", align_corners=False, antialias=True)
    f = (f / 2 + 0.5).clamp(0, 1)
    return (f * 255).to(torch.uint8).permute(0, 2, 3, 1).contiguous().numpy()


# --------------------------------------------------------------------------
# OpenCV interpolation tables
# --------------------------------------------------------------------------


def lanczos4_coeffs(x):
    """cv::interpolateLanczos4 (imgwarp.cpp): float32 results."""
    x = np.float32(x)
    if x < np.finfo(np.float32).eps:
        c = np.zeros(8, np.float32)
        c[3] = 1
        return c
    s45 = 0.70710678118654752440084436210485
    cs = [(1, 0), (-s45, -s45), (0, 1), (s45, -s45), (-1, 0), (s45, s45), (0, -1), (-s45, s45)]
    y0 = -(float(x) + 3) * math.pi * 0.25
    s0, c0 = math.sin(y0), math.cos(y0)
    c = np.zeros(8, np.float32)
    ssum = np.float32(0)
    for i in range(8):
        yy = float(x) + 3 - i
        if abs(yy) >= 1e-6:
            y = -yy * math.pi * 0.25
            c[i] = np.float32((cs[i][0] * s0 + cs[i][1] * c0) / (y * y))
        else:
            c[i] = np.float32(1e30)
        ssum = np.float32(ssum + c[i])
    inv = np.float32(np.float32(1) / ssum)
    return (c * inv).astype(np.float32)


def lanczos4_tab_i16():
    """initInterTab2D(INTER_LANCZOS4, fixpt=true): int16 [32*32][8*8], index
    fy*32 + fx, coefficient k1*8 + k2 (k1 = row tap, k2 = column tap), each
    row normalised to sum exactly 32768 by nudging a centre tap."""
    t1 = np.stack([lanczos4_coeffs(np.float32(i) * np.float32(1.0 / INTER_TAB)) for i in range(INTER_TAB)])
    out = np.zeros((INTER_TAB * INTER_TAB, 64), np.int16)
    for i in range(INTER_TAB):
        for j in range(INTER_TAB):
            v = (t1[i][:, None] * t1[j][None, :]).astype(np.float32)  # float products
            it = np.clip(np.rint(v.astype(np.float64) * COEF_SCALE), -32768, 32767).astype(np.int32)
            isum = int(it.sum())
            if isum != COEF_SCALE:
                diff = isum - COEF_SCALE
                # OpenCV: ksize2 = ksize/2 = 4; search taps k1, k2 in [ksize2, ksize2+2)
                mk1 = mk2 = Mk1 = Mk2 = 4
                for k1 in range(4, 6):
                    for k2 in range(4, 6):
                        if it[k1, k2] < it[mk1, mk2]:
                            mk1, mk2 = k1, k2
                        elif it[k1, k2] > it[Mk1, Mk2]:
                            Mk1, Mk2 = k1, k2
                if diff < 0:
                    it[Mk1, Mk2] -= diff
                else:
                    it[mk1, mk2] -= diff
            out[i * INTER_TAB + j] = it.reshape(64).astype(np.int16)
    return out


def linear_tab_f32():
    """initInterTab2D(INTER_LINEAR, fixpt=false): float [32*32][4] =
    (1-fy)(1-fx), (1-fy)fx, fy(1-fx), fy fx (float products)."""
    t1 = [(np.float32(1) - np.float32(i) / np.float32(INTER_TAB), np.float32(i) / np.float32(INTER_TAB))
          for i in range(INTER_TAB)]
    out = np.zeros((INTER_TAB * INTER_TAB, 4), np.float32)
    for i in range(INTER_TAB):
        for j in range(INTER_TAB):
            out[i * INTER_TAB + j] = [t1[i][a] * t1[j][b] for a in range(2) for b in range(2)]
    return out


# --------------------------------------------------------------------------
# 3-4. warpAffine
# --------------------------------------------------------------------------


def invert_affine(M):
    """cv::invertAffineTransform (double)."""
    M = np.asarray(M, np.float64).reshape(2, 3)
    D = M[0, 0] * M[1, 1] - M[0, 1] * M[1, 0]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22, A12, A21 = M[1, 1] * D, M[0, 0] * D, -M[0, 1] * D, -M[1, 0] * D
    b1 = -A11 * M[0, 2] - A12 * M[1, 2]
    b2 = -A21 * M[0, 2] - A22 * M[1, 2]
    return np.array([[A11, A12, b1], [A21, A22, b2]], np.float64)


def warp_matrix(affine_matrix, upscale_factor=1):
    """The dst->src matrix cv2.warpAffine iterates with (affine_transform.py:89-95:
    inverse_affine = invert(M) * upscale (+ offset); warpAffine without
    WARP_INVERSE_MAP inverts it again, in its own operation order)."""
    inv = invert_affine(affine_matrix) * upscale_factor
    if upscale_factor > 1:
        inv[:, 2] += 0.5 * upscale_factor
    M = inv.reshape(6).copy()
    D = M[0] * M[4] - M[1] * M[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = M[4] * D, M[0] * D
    M[0] = A11
    M[1] *= -D
    M[3] *= -D
    M[4] = A22
    b1 = -M[0] * M[2] - M[1] * M[5]
    b2 = -M[3] * M[2] - M[4] * M[5]
    M[2], M[5] = b1, b2
    return M


def _fixed_coords(M, H, W):
    """WarpAffineInvoker: X = (round((M1 y + M2) 1024) + 16 + round(M0 x 1024)) >> 5;
    integer part (saturated to int16) and the 5-bit fraction."""
    y = np.arange(H, dtype=np.float64)[:, None]
    x = np.arange(W, dtype=np.float64)[None, :]
    rd = AB_SCALE // INTER_TAB // 2
    X0 = np.rint((M[1] * y + M[2]) * AB_SCALE).astype(np.int64) + rd
    Y0 = np.rint((M[4] * y + M[5]) * AB_SCALE).astype(np.int64) + rd
    ad = np.rint(M[0] * x * AB_SCALE).astype(np.int64)
    bd = np.rint(M[3] * x * AB_SCALE).astype(np.int64)
    X = (X0 + ad) >> (AB_BITS - INTER_BITS)
    Y = (Y0 + bd) >> (AB_BITS - INTER_BITS)
    sx = np.clip(X >> INTER_BITS, -32768, 32767)
    sy = np.clip(Y >> INTER_BITS, -32768, 32767)
    return sx, sy, (Y & (INTER_TAB - 1)) * INTER_TAB + (X & (INTER_TAB - 1))


def warp_lanczos_u8(src, M, H, W, tab=None):
    """cv2.warpAffine(src u8 (h,w,C), ., (W,H), INTER_LANCZOS4, BORDER_CONSTANT 0)
    with the dst->src matrix M (warp_matrix): remapLanczos4 fixed point,
    taps outside the source read the border value 0."""
    tab = lanczos4_tab_i16() if tab is None else tab
    h, w, C = src.shape
    sx, sy, a = _fixed_coords(M, H, W)
    sx, sy = sx - 3, sy - 3
    wt = tab[a].astype(np.int64).reshape(H, W, 8, 8)
    acc = np.zeros((H, W, C), np.int64)
    for r in range(8):
        yy = sy + r
        vy = (yy >= 0) & (yy < h)
        for c in range(8):
            xx = sx + c
            ok = vy & (xx >= 0) & (xx < w)
            v = src[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)].astype(np.int64)
            acc += np.where(ok[..., None], v, 0) * wt[:, :, r, c][..., None]
    # entirely-outside pixels are the border value (0) -- same as the sum above
    out = (acc + (1 << (COEF_BITS - 1))) >> COEF_BITS
    return np.clip(out, 0, 255).astype(np.uint8)


def warp_ones_linear(h, w, M, H, W, tab=None):
    """cv2.warpAffine(np.ones((h,w), f32), ., (W,H)) (INTER_LINEAR, BORDER_CONSTANT 0):
    remapBilinear sums v0 w0 + v1 w1 + v2 w2 + v3 w3 left to right."""
    tab = linear_tab_f32() if tab is None else tab
    sx, sy, a = _fixed_coords(M, H, W)
    wt = tab[a]
    acc = np.zeros((H, W), np.float32)
    for k, (dy, dx) in enumerate(((0, 0), (0, 1), (1, 0), (1, 1))):
        ok = (sy + dy >= 0) & (sy + dy < h) & (sx + dx >= 0) & (sx + dx < w)
        acc = (acc + np.where(ok, np.float32(1), np.float32(0)) * wt[..., k]).astype(np.float32)
    return acc


# --------------------------------------------------------------------------
# 4-5. morphology + Gaussian
# --------------------------------------------------------------------------


def erode_rect(img, k):
    """cv2.erode(img, np.ones((k, k))) -- anchor k//2, out-of-image taps ignored
    (border value = +max).  k == 0 is OpenCV's empty-kernel default (3x3)."""
    if k == 0:
        k = 3
    a = k // 2
    H, W = img.shape
    big = np.float32(np.finfo(np.float32).max)
    p = np.full((H + k, W + k), big, np.float32)
    p[a:a + H, a:a + W] = img
    rows = p[:, 0:W].copy()
    for j in range(1, k):
        rows = np.minimum(rows, p[:, j:j + W])
    out = rows[0:H].copy()
    for i in range(1, k):
        out = np.minimum(out, rows[i:i + H])
    return out


def gaussian_kernel(n):
    """getGaussianKernel(n, sigma=0, CV_32F) (smooth.dispatch.cpp
    getGaussianKernelBitExact; the exp is the C library's, not softdouble)."""
    fixed = {1: [1.0], 3: [0.25, 0.5, 0.25], 5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
             7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125]}
    if n in fixed:
        return np.array(fixed[n], np.float32)
    sigma = n * 0.15 + 0.35
    scale2x = -0.125 / (sigma * sigma)
    n2 = (n - 1) // 2
    vals, s = [], 0.0
    for i, x in zip(range(n2), range(1 - n, 0, 2)):
        t = math.exp(float(x * x) * scale2x)
        vals.append(t)
        s += t
    s = s * 2 + 1.0
    if n % 2 == 0:
        s += 1.0
    mul = 1.0 / s
    res = [0.0] * n
    for i in range(n2):
        res[i] = res[n - 1 - i] = vals[i] * mul
    res[n2] = mul
    if n % 2 == 0:
        res[n2 + 1] = res[n2]
    return np.array(res, np.float32)


def _reflect101(p, n):
    p = np.where(p < 0, -p, p)
    return np.where(p >= n, 2 * n - p - 2, p)


def gaussian_blur(img, n):
    """cv2.GaussianBlur(img f32, (n, n), 0), BORDER_REFLECT_101, as sepFilter2D:
    row pass s = sum_k g[k] x[j + k - a] (k ascending), then the symmetric column
    pass s = g[a] x[i] + sum_{k>=1} g[a+k] (x[i+k] + x[i-k]), float32."""
    g = gaussian_kernel(n)
    a = n // 2
    H, W = img.shape
    xs = np.arange(W)
    row = np.zeros((H, W), np.float32)
    for k in range(n):
        row = (row + g[k] * img[:, _reflect101(xs + k - a, W)]).astype(np.float32)
    ys = np.arange(H)
    out = (g[a] * row).astype(np.float32)
    for k in range(1, a + 1):
        pair = (row[_reflect101(ys + k, H)] + row[_reflect101(ys - k, H)]).astype(np.float32)
        out = (out + g[a + k] * pair).astype(np.float32)
    return out


# --------------------------------------------------------------------------
# 2-6. restore_img
# --------------------------------------------------------------------------


def restore_img(frame, face, affine_matrix, tabs=None):
    """AlignRestore.restore_img (affine_transform.py:85-115), upscale_factor 1.
    frame uint8 (H,W,3), face uint8 (fh,fw,3), affine_matrix (2,3) float64.
    The frame -> uint8 cast of the blend truncates (np.astype); the uint16 branch
    (max > 256) cannot trigger for soft <= 1."""
    H, W, _ = frame.shape
    fh, fw, _ = face.shape
    lt, bt = tabs if tabs is not None else (lanczos4_tab_i16(), linear_tab_f32())
    M = warp_matrix(affine_matrix)
    restored = warp_lanczos_u8(face, M, H, W, lt)
    inv_mask = warp_ones_linear(fh, fw, M, H, W, bt)
    mask_e = erode_rect(inv_mask, 2)
    pasted = mask_e[:, :, None] * restored.astype(np.float32)
    area = np.sum(mask_e)
    w_edge = int(area ** 0.5) // 20
    center = erode_rect(mask_e, w_edge * 2)
    soft = gaussian_blur(center, w_edge * 2 + 1)[:, :, None]
    out = soft * pasted + (np.float32(1) - soft) * frame.astype(np.float32)
    return out.astype(np.uint8)


def restore_video(faces, frames, boxes, affine_matrices):
    """LipsyncPipeline.restore_video (lipsync_pipeline.py:343-358): faces float
    (N,3,R,R) torch, frames uint8 (>=N,H,W,3)."""
    tabs = (lanczos4_tab_i16(), linear_tab_f32())
    outs = []
    for i in range(faces.shape[0]):
        x1, y1, x2, y2 = boxes[i]
        face = face_resize_u8(faces[i:i + 1], int(y2 - y1), int(x2 - x1))[0]
        outs.append(restore_img(frames[i], face, np.asarray(affine_matrices[i], np.float64), tabs))
    return np.stack(outs)
