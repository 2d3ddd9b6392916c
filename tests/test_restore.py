"""Paste-back warp (LipsyncPipeline.restore_video, lipsync_pipeline.py:343-358;
AlignRestore.restore_img, affine_transform.py:85-115): the HIP kernels of
ls_restore.hip against the CPU restatement oracle/restore_cpu.py.

Parity status: the face resize is pinned (the oracle runs torch's own
antialiased bilinear, which torchvision's tensor resize calls); the OpenCV steps
are "parity unpinned" (cv2 is not installed and not in the reference tree), so
the oracle restates OpenCV's published fixed-point algorithm and the GPU must
reproduce that restatement bit for bit (uint8 output, integer Lanczos sums,
float32 blur/blend in the same operation order).
"""
import math

import numpy as np
import pytest
import torch

from oracle import restore_cpu as O
from latentsync_amd import restore as RS

FH, FW = 280, 210  # AlignRestore face_size (affine_transform.py:46): (75*2.8, 100*2.8)


def align_matrix(cx, cy, s, theta, fh=FH, fw=FW):
    """frame -> face matrix of a face centred at (cx, cy), s face px per frame px."""
    c, sn = math.cos(theta) * s, math.sin(theta) * s
    R = np.array([[c, -sn], [sn, c]])
    t = np.array([fw / 2.0, fh / 2.0]) - R @ np.array([cx, cy])
    return np.concatenate([R, t[:, None]], axis=1)


CASES = [  # (cx, cy, s, theta): centred / rotated / at the frame border / partly outside / small / large
    (240, 180, 1.0, 0.0),
    (230, 170, 0.93, 0.17),
    (60, 70, 1.1, -0.12),
    (470, 350, 0.9, 0.05),
    (250, 190, 4.0, 0.3),
    (240, 180, 0.62, -0.05),
]


def _frames(n, H=360, W=480, seed=0):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (n, H // 8, W // 8, 3)).astype(np.float32)
    up = np.repeat(np.repeat(base, 8, 1), 8, 2)
    return np.clip(up + rng.normal(0, 12, up.shape), 0, 255).astype(np.uint8)


def _faces(n, fh=FH, fw=FW, seed=1):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, (n, fh, fw, 3), dtype=np.uint8)


# ---------------------------------------------------------------- CPU checks


def test_warp_matrix_host_matches_oracle():
    for cx, cy, s, th in CASES:
        M = align_matrix(cx, cy, s, th)
        a = RS.dst_to_src(RS.invert_affine(M))
        b = O.warp_matrix(M)
        assert np.array_equal(a.view(np.int64), b.view(np.int64))


def test_roi_covers_soft_mask_support():
    H, W = 360, 480
    for cx, cy, s, th in CASES:
        M = align_matrix(cx, cy, s, th)
        r = RS.AlignRestore.__new__(RS.AlignRestore)
        r.upscale_factor = 1
        warps, rois, w_max = r.plan([M], FH, FW, H, W)
        mask = O.warp_ones_linear(FH, FW, O.warp_matrix(M), H, W)
        me = O.erode_rect(mask, 2)
        we = int(np.sum(me) ** 0.5) // 20
        assert we <= w_max
        soft = O.gaussian_blur(O.erode_rect(me, 2 * we), 2 * we + 1)
        ys, xs = np.nonzero((soft > 0) | (me > 0))
        x0, y0, x1, y1 = rois[0]
        if len(xs):
            assert x0 <= xs.min() and xs.max() < x1 and y0 <= ys.min() and ys.max() < y1


def test_lanczos_table_invariants():
    t = O.lanczos4_tab_i16().astype(np.int64)
    assert (t.sum(1) == 32768).all()
    # zero fraction: 1.0 * 32768 saturates to int16 32767 and OpenCV's sum fix-up puts
    # the missing 1 on tap (4,4) -- still an exact copy for uint8 sources
    d = np.zeros(64, np.int64)
    d[3 * 8 + 3], d[4 * 8 + 4] = 32767, 1
    assert np.array_equal(t[0], d)


def test_oracle_integer_translation_is_a_copy():
    """Known answer: a pure integer translation samples the face exactly
    (Lanczos at fraction 0 is the delta) and the warped mask is 1 inside."""
    face = _faces(1)[0]
    M = np.array([[1.0, 0.0, -100.0], [0.0, 1.0, -40.0]])  # frame (x, y) -> face (x-100, y-40)
    Md = O.warp_matrix(M)
    out = O.warp_lanczos_u8(face, Md, 360, 480)
    assert np.array_equal(out[40:40 + FH, 100:100 + FW], face)
    m = O.warp_ones_linear(FH, FW, Md, 360, 480)
    assert (m[40:40 + FH, 100:100 + FW] == 1).all() and m[:39].sum() == 0


def test_gaussian_kernels_match_opencv_small_tables():
    assert np.array_equal(O.gaussian_kernel(3), np.array([0.25, 0.5, 0.25], np.float32))
    for n in (9, 25, 49):
        g = O.gaussian_kernel(n)
        assert abs(float(g.astype(np.float64).sum()) - 1) < 1e-6 and np.array_equal(g, g[::-1])


# ---------------------------------------------------------------- GPU parity


@pytest.mark.gpu
def test_face_resize_matches_torch():
    g = torch.Generator().manual_seed(3)
    faces = (torch.rand((4, 3, 256, 256), generator=g) * 2.2 - 1.1)
    ref = O.face_resize_u8(faces, FH, FW)
    out = RS.face_resize_u8(faces.cuda(), FH, FW).cpu().numpy()
    d = np.abs(out.astype(np.int32) - ref.astype(np.int32))
    assert d.max() <= 1, d.max()
    assert (d > 0).mean() < 1e-3, (d > 0).mean()
    # identity size: exact
    out2 = RS.face_resize_u8(faces.cuda(), 256, 256).cpu().numpy()
    assert np.array_equal(out2, O.face_resize_u8(faces, 256, 256))


@pytest.mark.gpu
def test_restore_frames_bit_exact():
    n = len(CASES)
    frames, faces = _frames(n), _faces(n)
    mats = [align_matrix(*c) for c in CASES]
    tabs = (O.lanczos4_tab_i16(), O.linear_tab_f32())
    ref = np.stack([O.restore_img(frames[i], faces[i], mats[i], tabs) for i in range(n)])
    fr = torch.from_numpy(frames).cuda()
    RS.AlignRestore("cuda").restore_frames(fr, torch.from_numpy(faces).cuda(), mats)
    out = fr.cpu().numpy()
    for i in range(n):
        diff = out[i] != ref[i]
        assert not diff.any(), f"case {CASES[i]}: {diff.sum()} px differ, max {np.abs(out[i].astype(int) - ref[i]).max()}"
    assert (out != frames).any()


@pytest.mark.gpu
def test_restore_video_ragged_boxes():
    """restore_video with two box sizes in one clip (two launch groups) and a face
    entirely outside the frame (empty ROI: frame unchanged)."""
    n = 4
    frames = _frames(n, seed=5)
    g = torch.Generator().manual_seed(4)
    faces = torch.rand((n, 3, 256, 256), generator=g) * 2 - 1
    boxes = [[0, 0, FW, FH], [0, 0, 200, 240], [0, 0, FW, FH], [0, 0, FW, FH]]
    mats = [align_matrix(240, 180, 1.0, 0.1), align_matrix(200, 150, 1.0, -0.1, 240, 200),
            align_matrix(5000, 5000, 1.0, 0.0), align_matrix(300, 200, 1.2, 0.0)]
    ref = O.restore_video(faces, frames, boxes, mats)
    out = RS.restore_video(faces.cuda(), frames, boxes, mats).cpu().numpy()
    assert np.array_equal(out[2], frames[2])
    d = np.abs(out.astype(np.int32) - ref.astype(np.int32))
    # exact up to the pinned-resize's rare 1-LSB rounding differences propagating
    assert d.max() <= 1 and (d > 0).mean() < 1e-3, (d.max(), (d > 0).mean())
