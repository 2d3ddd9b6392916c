"""Face-alignment ingest and the fixed-mask resize (§8(a) a3):
cv2.resize INTER_LANCZOS4 (image_processor.py:34, :141), transformation_from_points
+ align_warp_face (affine_transform.py:7-70), laplacianSmooth (:118-144).

The HIP kernels (ls_resize_lanczos4_u8, ls_align_warp_u8) are checked bit-exact
against the numpy restatement (oracle/align_cpu.py).  OpenCV and the landmark model
are absent here, so the OpenCV arithmetic is "parity unpinned" (it follows OpenCV's
published generic C++ path); the CPU tests pin the restatement's own properties."""
import math

import numpy as np
import pytest
import torch

from oracle import align_cpu as A


def _similarity(theta, s, t):
    c, sn = math.cos(theta) * s, math.sin(theta) * s
    return np.array([[c, -sn, t[0]], [sn, c, t[1]]])


def _landmarks(n, seed=0, centre=(120.0, 90.0)):
    """68-point sets of a face at `centre` (brows 40 px apart, nose below) moving
    smoothly over the frames of a clip, with landmark jitter."""
    rng = np.random.default_rng(seed)
    base = rng.normal(0, 12, (68, 2))
    base[17:22] = [-20, -10] + rng.normal(0, 3, (5, 2))
    base[22:27] = [20, -10] + rng.normal(0, 3, (5, 2))
    base[27:36] = [0, 8] + rng.normal(0, 3, (9, 2))
    out = []
    for i in range(n):
        M = _similarity(0.05 * math.sin(i), 1.0 + 0.02 * i, (centre[0] + 3 * i, centre[1] - 2 * i))
        out.append(base @ M[:, :2].T + M[:, 2] + rng.normal(0, 0.3, (68, 2)))
    return out


# ------------------------------------------------------------------ CPU (oracle)


def test_resize_identity_and_constant():
    img = np.random.default_rng(0).integers(0, 256, (40, 30, 3), dtype=np.uint8)
    assert np.array_equal(A.resize_lanczos4_u8(img, 40, 30), img)  # cv::resize copies
    flat = np.full((37, 29, 3), 200, np.uint8)
    out = A.resize_lanczos4_u8(flat, 64, 51)
    # the int16 coefficient rows need not sum to exactly 2048: a flat image may move by 1
    assert out.shape == (64, 51, 3) and np.abs(out.astype(int) - 200).max() <= 1


def test_resize_matches_float_lanczos():
    """The fixed-point restatement against a float64 Lanczos-4 evaluation of the same
    taps and offsets: within 1 level (fixed-point rounding only)."""
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (23, 19), dtype=np.uint8)
    H, W = 41, 13
    out = A.resize_lanczos4_u8(img, H, W).astype(np.int64)

    def axis(n_src, n_dst):
        ofs, _ = A.resize_axis(n_src, n_dst)
        w = np.zeros((n_dst, n_src))
        for d in range(n_dst):
            f = np.float32((d + 0.5) * (1.0 / (n_dst / n_src)) - 0.5) - ofs[d]
            k = np.array([1.0 if abs(f + 3 - i) < 1e-9 else
                          4 * math.sin(math.pi * (f + 3 - i)) * math.sin(math.pi * (f + 3 - i) / 4) /
                          (math.pi ** 2 * (f + 3 - i) ** 2) for i in range(8)])
            k /= k.sum()
            for i in range(8):
                w[d, min(max(ofs[d] - 3 + i, 0), n_src - 1)] += k[i]
        return w
    ref = axis(23, H) @ img.astype(np.float64) @ axis(19, W).T
    assert np.abs(out - np.clip(np.floor(ref + 0.5), 0, 255)).max() <= 1


def test_mask_upscale_512_has_fractional_edges():
    from latentsync_amd.pipeline import load_fixed_mask
    m = (load_fixed_mask(256).numpy() * 255).round().astype(np.uint8)
    up = A.resize_lanczos4_u8(m, 512, 512)
    vals = np.unique(up)
    assert 0 in vals and 255 in vals and len(vals) > 2  # LANCZOS ringing/edges, not nearest
    # away from the mask edge the 2x upscale reproduces the binary values
    assert np.array_equal(up[::2, ::2][m == m[0, 0]][:100], np.full(100, m[0, 0]))


def test_transformation_from_points_recovers_similarity():
    M_true = _similarity(0.3, 1.7, (12.0, -5.0))
    pts = (A.FACE_TEMPLATE - M_true[:, 2]) @ np.linalg.inv(M_true[:, :2]).T  # template = M pts
    M, bias = A.transformation_from_points(pts, A.FACE_TEMPLATE, smooth=False)
    assert np.allclose(M, M_true, atol=1e-9) and bias is None
    # smoothing: bias carried as 0.2 * previous + 0.8 * current
    _, b1 = A.transformation_from_points(pts, A.FACE_TEMPLATE, True, None)
    _, b2 = A.transformation_from_points(pts + 1.0, A.FACE_TEMPLATE, True, b1)
    assert b2.shape == (2,)


def test_host_alignment_math_matches_oracle():
    """latentsync_amd.align's host half (smoothing, 3 points, Procrustes with p_bias)."""
    from latentsync_amd import align as L
    lm = _landmarks(6)
    mats = L.FaceAligner.__new__(L.FaceAligner)
    mats.smoother, mats.p_bias = L.LaplacianSmooth(), None
    got = L.FaceAligner.matrices(mats, lm)
    ref, pb = [], None
    for pts in A.laplacian_smooth(lm):
        M, pb = A.transformation_from_points(A.lmk3(pts), A.FACE_TEMPLATE, True, pb)
        ref.append(M)
    for a, b in zip(got, ref):
        assert np.allclose(a, b, rtol=0, atol=1e-12)


# ------------------------------------------------------------------ GPU (HIP vs oracle)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [((256, 256, 1), (512, 512)), ((280, 210, 3), (256, 256)),
                                   ((280, 210, 3), (512, 512)), ((100, 77, 3), (64, 50)),
                                   ((37, 53, 2), (91, 13)), ((512, 512, 1), (64, 64)), ((64, 64, 3), (64, 64))])
def test_resize_hip_bitexact(gpu, shape):
    from latentsync_amd.align import resize_lanczos4
    (h, w, C), (H, W) = shape
    rng = np.random.default_rng(h * w + C)
    img = rng.integers(0, 256, (3, h, w, C), dtype=np.uint8)
    img[1] = (rng.uniform(0, 1, (h, w, C)) > 0.5) * 255  # hard edges: saturation paths
    out = resize_lanczos4(torch.from_numpy(img).cuda(), H, W).cpu().numpy()
    for i in range(3):
        assert np.array_equal(out[i], A.resize_lanczos4_u8(img[i], H, W)), i


@pytest.mark.gpu
def test_load_fixed_mask_512_matches_oracle(gpu):
    from latentsync_amd.pipeline import load_fixed_mask
    m256 = (load_fixed_mask(256).numpy() * 255).round().astype(np.uint8)
    m512 = load_fixed_mask(512)
    ref = A.resize_lanczos4_u8(m256, 512, 512).astype(np.float64) / 255.0
    assert m512.shape == (512, 512) and np.array_equal(m512.numpy(), ref.astype(np.float32))


@pytest.mark.gpu
def test_affine_transform_video_matches_oracle(gpu):
    """Whole ingest: smoothed landmarks -> matrices -> Lanczos-4 warp with border 127
    (some output pixels fall outside the frame) -> resize to R."""
    from latentsync_amd import align as L
    n, H, W = 5, 180, 240
    rng = np.random.default_rng(3)
    low = torch.from_numpy(rng.uniform(0, 255, (n, 3, H // 6, W // 6)).astype(np.float32))
    frames = torch.nn.functional.interpolate(low, size=(H, W), mode="bilinear").round().clamp(0, 255)
    frames = frames.to(torch.uint8).permute(0, 2, 3, 1).contiguous().numpy()
    lm = _landmarks(n, 4, centre=(18.0, 14.0))  # near the corner: the crop leaves the frame
    for R in (256, 128):
        faces, boxes, mats = L.affine_transform_video(frames, lm, R, "cuda")
        rf, rb, rm = A.affine_transform_video(frames, lm, R)
        assert boxes == rb == [[0, 0, 210, 280]] * n
        for a, b in zip(mats, rm):
            assert np.allclose(a, b, rtol=0, atol=1e-12)
        f = faces.cpu().numpy()
        assert f.shape == (n, 3, R, R) and f.dtype == np.uint8
        assert np.array_equal(f, rf)
    # the warp alone, including pixels whose taps leave the frame (border 127)
    al = L.FaceAligner(256, "cuda")
    w = al.warp(frames, mats).cpu().numpy()
    tab = A.lanczos4_tab_i16()
    border = 0
    for i in range(n):
        ref = A.warp_lanczos_border_u8(frames[i], A.warpaffine_dst_to_src(mats[i]), 280, 210, 127, tab)
        assert np.array_equal(w[i], ref)
        border += int((ref == 127).all(axis=-1).sum())
    assert border > 1000  # the border really is exercised
