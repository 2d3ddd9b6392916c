"""Paste-back warp on the GPU: ``LipsyncPipeline.restore_video``
(latentsync/pipelines/lipsync_pipeline.py:343-358) and
``AlignRestore.restore_img`` (latentsync/utils/affine_transform.py:85-115).

The reference loops over frames on the host (torchvision resize, cv2 warpAffine,
erode, GaussianBlur, blend).  Here one ``ls_face_resize_u8`` launch resizes every
face of the clip and one ``ls_restore_frames`` call (five kernels) warps and
blends all of them into the frames, in place, on the device.  The host only
does the 2x3 matrix algebra the reference does with cv2.invertAffineTransform /
warpAffine's own inversion (float64, same operation order) and the per-frame
region of interest: the face footprint in the frame plus the erode/blur reach;
outside it the soft mask is 0 and the frame is unchanged.
"""
import math

import numpy as np
import torch

from . import _lib
from ._lib import check


def _stream():
    return torch.cuda.current_stream().cuda_stream


def invert_affine(M):
    """cv2.invertAffineTransform (double) (affine_transform.py:89)."""
    M = np.asarray(M, np.float64).reshape(2, 3)
    D = M[0, 0] * M[1, 1] - M[0, 1] * M[1, 0]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22, A12, A21 = M[1, 1] * D, M[0, 0] * D, -M[0, 1] * D, -M[1, 0] * D
    return np.array([[A11, A12, -A11 * M[0, 2] - A12 * M[1, 2]],
                     [A21, A22, -A21 * M[0, 2] - A22 * M[1, 2]]], np.float64)


def dst_to_src(inverse_affine):
    """cv2.warpAffine without WARP_INVERSE_MAP inverts its matrix itself (imgwarp.cpp
    warpAffine, in this operation order); the result maps frame pixels to face pixels."""
    M = np.asarray(inverse_affine, np.float64).reshape(6).copy()
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


def _roi(inv, fh, fw, H, W, margin):
    """Frame-pixel box holding every pixel whose warped mask can be non-zero
    (face coords in (-1, fw) x (-1, fh), padded for the fixed-point rounding), grown
    by the erode + blur reach and clipped to the frame.  [x0, y0, x1, y1)."""
    cs = np.array([[-2.0, -2.0], [fw + 1.0, -2.0], [-2.0, fh + 1.0], [fw + 1.0, fh + 1.0]])
    p = cs @ inv[:, :2].T + inv[:, 2]
    x0 = int(math.floor(p[:, 0].min())) - margin
    y0 = int(math.floor(p[:, 1].min())) - margin
    x1 = int(math.ceil(p[:, 0].max())) + 1 + margin
    y1 = int(math.ceil(p[:, 1].max())) + 1 + margin
    x0, y0, x1, y1 = max(x0, 0), max(y0, 0), min(x1, W), min(y1, H)
    if x1 <= x0 or y1 <= y0:
        return [0, 0, 0, 0]
    return [x0, y0, x1, y1]


class AlignRestore:
    """GPU counterpart of AlignRestore's restore path (upscale_factor 1, the only
    configuration the reference builds: affine_transform.py:37-46)."""

    upscale_factor = 1

    def __init__(self, device="cuda"):
        self.device = torch.device(device)
        self._tables, self._w_max = None, -1

    def _tables_for(self, w_max):
        if w_max > self._w_max:
            lib = _lib.load()
            w_max = max(w_max, 16)
            t = torch.empty(lib.ls_restore_tables_bytes(w_max), dtype=torch.uint8, device=self.device)
            check(lib.ls_restore_init_tables(t.data_ptr(), w_max, _stream()), "ls_restore_init_tables")
            self._tables, self._w_max = t, w_max
        return self._tables

    def plan(self, affine_matrices, fh, fw, H, W):
        """Per-frame dst->src matrices (N,6) f64, ROIs (N,4) int32, and the w_edge
        bound: area <= |det(inverse_affine)| (fh+2)(fw+2)."""
        warps, rois, w_max = [], [], 0
        invs = [invert_affine(m) * self.upscale_factor for m in affine_matrices]
        for inv in invs:
            det = abs(inv[0, 0] * inv[1, 1] - inv[0, 1] * inv[1, 0])
            w_max = max(w_max, int(math.sqrt(det * (fh + 2) * (fw + 2))) // 20 + 1)
        for inv in invs:
            warps.append(dst_to_src(inv))
            rois.append(_roi(inv, fh, fw, H, W, 2 * w_max + 4))
        return np.stack(warps), np.asarray(rois, np.int32).reshape(-1, 4), w_max

    def restore_frames(self, frames_u8, faces_u8, affine_matrices):
        """restore_img for every frame: frames_u8 (N,H,W,3) uint8 device tensor
        (updated in place and returned), faces_u8 (N,fh,fw,3) uint8 device tensor,
        affine_matrices N x (2,3) (the align matrices of data.pth)."""
        lib = _lib.load()
        N, H, W, C3 = frames_u8.shape
        _, fh, fw, _ = faces_u8.shape
        if C3 != 3 or faces_u8.shape[0] != N or len(affine_matrices) != N:
            raise ValueError("restore_frames: frames (N,H,W,3), faces (N,fh,fw,3) and N matrices expected")
        if not (frames_u8.is_contiguous() and faces_u8.is_contiguous()):
            raise ValueError("restore_frames: contiguous uint8 tensors expected")
        if N == 0:
            return frames_u8
        warps, rois, w_max = self.plan(affine_matrices, fh, fw, H, W)
        tables = self._tables_for(w_max)
        roi_w = int((rois[:, 2] - rois[:, 0]).max())
        roi_h = int((rois[:, 3] - rois[:, 1]).max())
        dev = self.device
        warp_d = torch.from_numpy(warps).to(dev)
        roi_d = torch.from_numpy(rois).to(dev)
        ws = torch.empty(lib.ls_restore_workspace_bytes(N, roi_h, roi_w), dtype=torch.uint8, device=dev)
        check(lib.ls_restore_frames(frames_u8.data_ptr(), N, H, W, faces_u8.data_ptr(), fh, fw, warp_d.data_ptr(),
                                    roi_d.data_ptr(), roi_h, roi_w, self._w_max, tables.data_ptr(), ws.data_ptr(),
                                    ws.numel(), _stream()), "ls_restore_frames")
        return frames_u8


def face_resize_u8(faces, out_h, out_w):
    """torchvision resize(face, (h, w), antialias=True), (x/2+0.5).clamp(0,1)*255 ->
    uint8, HWC (lipsync_pipeline.py:348-354): faces (N,3,R,R) fp32 on the device."""
    lib = _lib.load()
    faces = faces.float().contiguous()
    N, C3, Hi, Wi = faces.shape
    if C3 != 3:
        raise ValueError("face_resize_u8: (N,3,H,W) expected")
    out = torch.empty((N, out_h, out_w, 3), dtype=torch.uint8, device=faces.device)
    check(lib.ls_face_resize_u8(faces.data_ptr(), N, Hi, Wi, out_h, out_w, out.data_ptr(), _stream()),
          "ls_face_resize_u8")
    return out


def restore_video(faces, video_frames, boxes, affine_matrices, restorer=None):
    """LipsyncPipeline.restore_video (lipsync_pipeline.py:343-358), batched:
    faces (N,3,R,R) decoded pixels in [-1,1] on the device; video_frames (>=N,H,W,3)
    uint8 (numpy or tensor); boxes N x [x1,y1,x2,y2]; affine_matrices N x (2,3).
    Returns the restored frames (N,H,W,3) uint8 on the device."""
    restorer = restorer or AlignRestore(faces.device)
    N = faces.shape[0]
    if len(boxes) < N or len(affine_matrices) < N or len(video_frames) < N:
        # the reference indexes boxes[index] / affine_matrices[index] per face (:347, :356)
        raise IndexError(f"restore_video: {N} faces but {len(boxes)} boxes, {len(affine_matrices)} matrices, "
                         f"{len(video_frames)} frames")
    frames = torch.as_tensor(np.asarray(video_frames[:N])) if not torch.is_tensor(video_frames) else video_frames[:N]
    frames = frames.to(faces.device, torch.uint8).contiguous().clone()
    sizes = [(int(b[3] - b[1]), int(b[2] - b[0])) for b in boxes[:N]]
    # one resize + restore launch per distinct box size (the reference's boxes are all
    # the aligned face size, so normally a single group)
    for hw in sorted(set(sizes)):
        idx = [i for i, s in enumerate(sizes) if s == hw]
        sel = torch.tensor(idx, device=faces.device)
        face_u8 = face_resize_u8(faces.index_select(0, sel), hw[0], hw[1])
        if len(idx) == N:
            restorer.restore_frames(frames, face_u8, affine_matrices[:N])
        else:
            sub = frames.index_select(0, sel).contiguous()
            restorer.restore_frames(sub, face_u8, [affine_matrices[i] for i in idx])
            frames.index_copy_(0, sel, sub)
    return frames
