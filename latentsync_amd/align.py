"""Face-alignment ingest on the GPU: what
``affine_transform_video`` (latentsync/pipelines/affine_transform_video.py:8-35) and
``ImageProcessor.affine_transform`` (latentsync/utils/image_processor.py:118-143)
do per frame once the 68 landmarks are known, batched over the clip:

  host   laplacianSmooth (affine_transform.py:118-144) -> 3 alignment points
         (image_processor.py:132-135) -> transformation_from_points
         (affine_transform.py:7-32, float64, p_bias carried frame to frame)
  device ls_align_warp_u8   cv2.warpAffine(frame, M, (210, 280), INTER_LANCZOS4,
                            BORDER_CONSTANT 127)   (affine_transform.py:53-70)
         ls_resize_lanczos4_u8  cv2.resize(face, (R, R), INTER_LANCZOS4)  (:141)

The landmark detector itself (face_alignment / mediapipe) is not built: it needs a
checkpoint that does not exist here, so landmarks are this module's input.  The
output is exactly the ``data.pth`` record the reference writes
(``generate_affine_transforms``, :23-35): faces uint8 (N,3,R,R), boxes, matrices.
Also ``resize_lanczos4`` for load_fixed_mask's mask resize (image_processor.py:34).
"""
import numpy as np
import torch

from . import _lib
from ._lib import check
from .restore import AlignRestore as _Restorer
from .restore import dst_to_src

RATIO = 2.8
FACE_TEMPLATE = np.array([[19 - 2, 30 - 10], [56 + 2, 30 - 10], [37.5, 45 - 5]]) * RATIO  # affine_transform.py:41-42
FACE_SIZE = (int(75 * RATIO), int(100 * RATIO))  # (w, h) = (210, 280), :43


def _stream():
    return torch.cuda.current_stream().cuda_stream


def resize_lanczos4(img_u8, dst_h, dst_w):
    """cv2.resize(img, (dst_w, dst_h), interpolation=cv2.INTER_LANCZOS4) on the device:
    img_u8 uint8 (N, h, w, C) or (h, w, C) or (h, w) device tensor."""
    lib = _lib.load()
    x = img_u8.contiguous()
    shp = x.shape
    if x.dim() == 2:
        x = x[None, :, :, None]
    elif x.dim() == 3:
        x = x[None]
    N, h, w, C = x.shape
    out = torch.empty((N, dst_h, dst_w, C), dtype=torch.uint8, device=x.device)
    ws = torch.empty(max(1, lib.ls_resize_lanczos4_workspace_bytes(dst_h, dst_w)), dtype=torch.uint8, device=x.device)
    check(lib.ls_resize_lanczos4_u8(x.data_ptr(), N, h, w, C, out.data_ptr(), dst_h, dst_w, ws.data_ptr(), ws.numel(),
                                    _stream()), "ls_resize_lanczos4_u8")
    if len(shp) == 2:
        return out[0, :, :, 0]
    return out[0] if len(shp) == 3 else out


def transformation_from_points(points1, points0, smooth=True, p_bias=None):
    """affine_transform.py:7-32 -- similarity transform taking the 3 detected points
    onto the face template (SVD Procrustes, float64) plus the smoothed bias."""
    points2 = np.array(points0, dtype=np.float64)
    points1 = np.array(points1, dtype=np.float64)
    c1, c2 = points1.mean(axis=0), points2.mean(axis=0)
    points1 -= c1
    points2 -= c2
    s1, s2 = np.std(points1), np.std(points2)
    points1 /= s1
    points2 /= s2
    U, _, Vt = np.linalg.svd(np.matmul(points1.T, points2))
    R = np.matmul(U, Vt).T
    T = c2.reshape(2, 1) - (s2 / s1) * np.matmul(R, c1.reshape(2, 1))
    M = np.concatenate(((s2 / s1) * R, T), axis=1)
    if smooth:
        bias = points2[2] - points1[2]
        if p_bias is not None:
            bias = p_bias * 0.2 + bias * 0.8
        p_bias = bias
        M[:, 2] = M[:, 2] + bias
    return M, p_bias


class LaplacianSmooth:
    """laplacianSmooth (affine_transform.py:118-144): landmark temporal smoothing."""

    def __init__(self, smoothAlpha=0.3):
        self.smoothAlpha = smoothAlpha
        self.pts_last = None

    def smooth(self, pts_cur):
        pts_cur = np.asarray(pts_cur, np.float64)
        if self.pts_last is None:
            self.pts_last = pts_cur.copy()
            return pts_cur.copy()
        width = pts_cur[:, 0].max() - pts_cur[:, 0].min()
        d2 = (pts_cur[:, 0] - self.pts_last[:, 0]) ** 2 + (pts_cur[:, 1] - self.pts_last[:, 1]) ** 2
        w = np.exp(-d2 / (width * self.smoothAlpha))[:, None]
        upd = self.pts_last * w + pts_cur * (1 - w)
        self.pts_last = upd.copy()
        return upd


def align_points(points68):
    """image_processor.py:132-135: the two brow centres and the nose centre."""
    p = np.asarray(points68, np.float64)
    return np.stack([p[17:22].mean(0), p[22:27].mean(0), p[27:36].mean(0)])


class FaceAligner:
    """The per-clip state of ImageProcessor's fix_mask alignment (its smoother and its
    AlignRestore's p_bias) plus the device warp/resize."""

    def __init__(self, resolution=256, device="cuda"):
        self.resolution = resolution
        self.device = torch.device(device)
        self.smoother = LaplacianSmooth()
        self.p_bias = None
        self._tables = _Restorer(self.device)

    def matrices(self, landmarks68):
        """Host half: smoothed landmarks -> affine matrices (2,3) float64, in frame order."""
        mats = []
        for pts in landmarks68:
            M, self.p_bias = transformation_from_points(align_points(self.smoother.smooth(pts)), FACE_TEMPLATE, True,
                                                        self.p_bias)
            mats.append(M)
        return mats

    def warp(self, frames_u8, mats, border_value=127):
        """Device half: cv2.warpAffine(frame, M, (210, 280), INTER_LANCZOS4,
        BORDER_CONSTANT 127) for every frame -> uint8 (N, 280, 210, 3)."""
        lib = _lib.load()
        frames = torch.as_tensor(frames_u8).to(self.device, torch.uint8).contiguous()
        N, H, W, C3 = frames.shape
        if C3 != 3 or len(mats) != N:
            raise ValueError("warp: frames (N,H,W,3) and N matrices expected")
        fw, fh = FACE_SIZE
        out = torch.empty((N, fh, fw, 3), dtype=torch.uint8, device=self.device)
        if N == 0:
            return out
        warp = torch.from_numpy(np.stack([dst_to_src(m) for m in mats])).to(self.device)
        tables = self._tables._tables_for(0)
        check(lib.ls_align_warp_u8(frames.data_ptr(), N, H, W, warp.data_ptr(), fh, fw, int(border_value),
                                   tables.data_ptr(), out.data_ptr(), _stream()), "ls_align_warp_u8")
        return out

    def __call__(self, frames_u8, landmarks68):
        """affine_transform_video with the landmarks given: (faces uint8 (N,3,R,R) on
        the device, boxes, affine_matrices) -- the data.pth record."""
        mats = self.matrices(landmarks68)
        faces = self.warp(frames_u8, mats)
        boxes = [[0, 0, faces.shape[2], faces.shape[1]]] * len(mats)  # image_processor.py:140
        R = self.resolution
        faces = resize_lanczos4(faces, R, R).permute(0, 3, 1, 2).contiguous()
        return faces, boxes, mats


def affine_transform_video(frames_u8, landmarks68, resolution=256, device="cuda"):
    """affine_transform_video (affine_transform_video.py:8-21) given per-frame 68-point
    landmarks: (faces (N,3,R,R) uint8 device tensor, boxes, affine_matrices)."""
    return FaceAligner(resolution, device)(frames_u8, landmarks68)


def generate_affine_transforms(frames_u8, landmarks68, output_path, height=512, device="cuda"):
    """generate_affine_transforms (affine_transform_video.py:23-35): writes the data.pth
    ingest record {faces, boxes, affine_matrices} that LipsyncPipeline(data_path=...) reads."""
    faces, boxes, mats = affine_transform_video(frames_u8, landmarks68, height, device)
    torch.save({"faces": faces.cpu(), "boxes": boxes, "affine_matrices": mats}, output_path)
    return faces, boxes, mats
