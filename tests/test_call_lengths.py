"""LipsyncPipeline.__call__ clip-length semantics (lipsync_pipeline.py:438-511):

  (a) audio longer than the video: faces, boxes, affine matrices and the original
      frames are repeated TOGETHER to the chunk count (:448-452);
  (b) start_from_backwards: zero chunks are prepended (repeat.py:81-118) and, with
      more faces than chunks, all four per-frame sequences keep their LAST n items
      (:462-466, repeat.py:33-56);
  (c) force_video_length: the chunks are padded to the face count (:453-456), so the
      last window is short (n % num_frames != 0) and runs with its own frame count
      (:500-511).

Each case checks (1) every window -- the short one included -- against
oracle.pipeline_window on the same faces / audio chunks / noise (rel-L2 < 3e-2, as
tests/test_gpu_pipeline.py) and (2) every restored frame against
oracle/restore_cpu.py given the independently expected frames / boxes / matrices
(bit-exact up to the pinned resize's rare 1-LSB rounding, as tests/test_restore.py).
"""
import math
import wave

import numpy as np
import pytest
import torch

from conftest import rel_err

pytestmark = pytest.mark.gpu

SCHED = dict(beta_end=0.012, beta_schedule="scaled_linear", beta_start=0.00085, clip_sample=False,
             num_train_timesteps=1000, set_alpha_to_one=False, steps_offset=1)
RR, FR, H, W, FH, FW = 64, 8, 120, 160, 56, 48
STEPS = 2


def _align(cx, cy, s, theta):
    c, sn = math.cos(theta) * s, math.sin(theta) * s
    Rm = np.array([[c, -sn], [sn, c]])
    t = np.array([FW / 2.0, FH / 2.0]) - Rm @ np.array([cx, cy])
    return np.concatenate([Rm, t[:, None]], axis=1)


def _write_wav(path, seconds, sr=16000, seed=1):
    a = np.random.default_rng(seed).normal(0, 0.1, int(seconds * sr)).clip(-1, 0.999)
    with wave.open(str(path), "wb") as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(sr)
        f.writeframes((a * 32768).astype("<i2").tobytes())


@pytest.fixture(scope="module")
def models():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from latentsync_amd.audio import Audio2Feature
    from latentsync_amd.config import TINY_MODEL
    from latentsync_amd.unet import UNet3DConditionModel
    from latentsync_amd.vae import AutoencoderKL
    unet = UNet3DConditionModel(**TINY_MODEL).init_weights(13).to("cuda").eval()
    vae = AutoencoderKL(block_out_channels=(32, 64, 64, 64)).init_weights(14).to("cuda")
    return unet, vae, Audio2Feature.random(2, device="cuda")


def _clip(tmp_path, N, seconds):
    rng = np.random.default_rng(N)
    g = torch.Generator().manual_seed(N)
    faces = (torch.rand((N, 3, RR, RR), generator=g) * 255).to(torch.uint8)
    mats = [_align(80 + rng.uniform(-5, 5), 60 + rng.uniform(-5, 5), rng.uniform(0.8, 1.2), rng.uniform(-0.15, 0.15))
            for _ in range(N)]
    # distinct boxes per frame (same size) so a mis-paired box would show
    boxes = [[int(i % 3), 0, int(i % 3) + FW, FH] for i in range(N)]
    frames = rng.integers(0, 256, (N, H, W, 3), dtype=np.uint8)
    torch.save({"faces": faces, "boxes": boxes, "affine_matrices": mats}, tmp_path / "data.pth")
    np.save(tmp_path / "video.npy", frames)
    _write_wav(tmp_path / "audio.wav", seconds)
    return faces, boxes, mats, frames


def _run(tmp_path, models, monkeypatch, N, seconds, **call_kw):
    """Run __call__ with injected window noise; returns what the loop saw, its
    output and the written frames."""
    from latentsync_amd.pipeline import LipsyncPipeline
    from latentsync_amd.scheduler import DDIMScheduler
    unet, vae, audio = models
    faces, boxes, mats, frames = _clip(tmp_path, N, seconds)
    pipe = LipsyncPipeline(vae, audio, unet, DDIMScheduler(**SCHED))
    pipe.windows_per_batch = 2
    seen = {}
    real_run, real_restore = pipe.run_windows, pipe.restore_video
    h = RR // 8

    def run_windows(faces_u8, chunks, mask, num_frames, steps, g, generator, **kw):
        n = chunks.shape[0]
        gen = torch.Generator().manual_seed(77)
        init = torch.randn((1, 4, 1, h, h), generator=gen)
        sizes = [min(num_frames, n - i * num_frames) for i in range(math.ceil(n / num_frames))]
        noise = [(torch.randn((s, 4, h, h), generator=gen), torch.randn((s, 4, h, h), generator=gen)) for s in sizes]
        seen.update(faces=faces_u8.clone(), chunks=chunks.float().cpu(), mask=mask.float().cpu(), init=init,
                    noise=noise, sizes=sizes)
        out, out_u8 = real_run(faces_u8, chunks, mask, num_frames, steps, g, generator,
                               all_latents=init.repeat(1, 1, n, 1, 1).cuda(),
                               vae_noise=lambda i: (noise[i][0].cuda(), noise[i][1].cuda()), **kw)
        seen["out"] = out.float().cpu()
        return out, out_u8

    def restore(f, v, b, m):
        seen["restore_args"] = (len(v), list(b), [np.asarray(x) for x in m])
        return real_restore(f, v, b, m)

    monkeypatch.setattr(pipe, "run_windows", run_windows)
    monkeypatch.setattr(pipe, "restore_video", restore)
    out_path = str(tmp_path / "out.npz")
    pipe(video_path=str(tmp_path / "video.npy"), audio_path=str(tmp_path / "audio.wav"), video_out_path=out_path,
         num_frames=FR, num_inference_steps=STEPS, guidance_scale=1.0, data_path=str(tmp_path / "data.pth"),
         mask_image_path=None, **call_kw)
    return seen, np.load(out_path)["frames"], (faces, boxes, mats, frames)


def _check(seen, written, expect, models, monkeypatch):
    from oracle import ref_cpu as R
    from oracle import restore_cpu as O
    unet, vae, _ = models
    monkeypatch.setitem(R.VAE_CFG, "block_out_channels", (32, 64, 64, 64))
    faces_e, boxes_e, mats_e, frames_e = expect
    n = seen["chunks"].shape[0]
    assert torch.equal(seen["faces"][:n].cpu(), faces_e[:n])
    # (1) every window, short ones included, against the oracle window
    for i, s in enumerate(seen["sizes"]):
        sl = slice(i * FR, i * FR + s)
        ref = R.pipeline_window(unet.state_dict(), dict(unet.config), vae._sd, faces_e[sl], seen["mask"],
                                seen["chunks"][sl], seen["init"], seen["noise"][i][0], seen["noise"][i][1],
                                num_steps=STEPS, guidance_scale=1.0)
        e = rel_err(seen["out"][sl], ref)
        print("window", i, s, e)
        assert e < 3e-2
    # (2) the warp-back got the per-frame boxes / matrices / frames the reference pairs
    nv, b, m = seen["restore_args"]
    assert b[:n] == [list(x) for x in boxes_e[:n]]
    assert all(np.array_equal(x, y) for x, y in zip(m[:n], mats_e[:n]))
    assert written.shape == (n, H, W, 3)
    ref = O.restore_video(seen["out"], frames_e[:n], boxes_e[:n], mats_e[:n])
    d = np.abs(written.astype(np.int32) - ref.astype(np.int32))
    assert d.max() <= 1 and (d > 0).mean() < 1e-3, (d.max(), (d > 0).mean())


def test_audio_longer_than_video(tmp_path, models, monkeypatch):
    """(a): 11 video frames, ~1.3 s of audio -> chunks padded to 48, everything tiled."""
    from latentsync_amd import repeat as rep
    N = 11
    seen, written, (faces, boxes, mats, frames) = _run(tmp_path, models, monkeypatch, N, 1.3)
    n = seen["chunks"].shape[0]
    assert n > N and n % 16 == 0
    expect = (rep.repeat_to_length(faces, n), rep.repeat_to_length(boxes, n), rep.repeat_to_length(mats, n),
              rep.repeat_to_length(frames, n))
    assert np.array_equal(expect[3][N], frames[0])  # tiled, not clamped
    _check(seen, written, expect, models, monkeypatch)


def test_start_from_backwards_truncates_from_front(tmp_path, models, monkeypatch):
    """(b): 40 video frames, ~0.5 s of audio -> zero chunks prepended to 16, and
    faces / boxes / matrices / frames all keep their LAST 16."""
    N = 40
    seen, written, (faces, boxes, mats, frames) = _run(tmp_path, models, monkeypatch, N, 0.5,
                                                       start_from_backwards=True)
    n = seen["chunks"].shape[0]
    assert n < N and n % 16 == 0
    assert float(seen["chunks"][0].abs().max()) == 0.0  # prepended padding
    expect = (faces[N - n:], boxes[N - n:], mats[N - n:], frames[N - n:])
    _check(seen, written, expect, models, monkeypatch)


def test_force_video_length_short_last_window(tmp_path, models, monkeypatch):
    """(c): 21 video frames, ~0.5 s of audio -> chunks padded to 21: windows of
    8, 8 and a short 5-frame window."""
    N = 21
    seen, written, (faces, boxes, mats, frames) = _run(tmp_path, models, monkeypatch, N, 0.5,
                                                       force_video_length=True)
    assert seen["chunks"].shape[0] == N and seen["sizes"] == [8, 8, 5]
    _check(seen, written, (faces, boxes, mats, frames), models, monkeypatch)


def test_callback_per_step(tmp_path, models, monkeypatch):
    """callback(j, t, latents) after every DDIM step of every window (:564-568).
    The latents a callback keeps must not change afterwards (the reference hands it
    the fresh tensor scheduler.step returns) and must match the oracle's per-step
    latents."""
    from oracle import ref_cpu as R
    calls, kept = [], []

    def cb(j, t, lat):
        calls.append((j, int(t), tuple(lat.shape)))
        kept.append(lat)  # kept as handed over, not copied here
    seen, _, (faces, _, _, _) = _run(tmp_path, models, monkeypatch, 16, 0.3, callback=cb)
    h = RR // 8
    # 0.3 s of audio -> 16 padded chunks -> 2 windows of 8 frames, 2 steps each
    assert calls == [(0, 501, (1, 4, FR, h, h)), (1, 1, (1, 4, FR, h, h))] * 2
    assert not torch.equal(kept[0], kept[1]) and not torch.equal(kept[1], kept[3])
    unet, vae, _ = models
    monkeypatch.setitem(R.VAE_CFG, "block_out_channels", (32, 64, 64, 64))
    for i, s in enumerate(seen["sizes"]):
        sl = slice(i * FR, i * FR + s)
        ref_steps = []
        R.pipeline_window(unet.state_dict(), dict(unet.config), vae._sd, faces[sl], seen["mask"], seen["chunks"][sl],
                          seen["init"], seen["noise"][i][0], seen["noise"][i][1], num_steps=STEPS,
                          guidance_scale=1.0, step_latents=ref_steps)
        for j in range(STEPS):
            e = rel_err(kept[i * STEPS + j].float().cpu(), ref_steps[j])
            print("window", i, "step", j, e)
            assert e < 3e-2
