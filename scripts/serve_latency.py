"""Latency of /process requests through the serving stack (serve.py: FastAPI app ->
ProcessWorker -> spawned pipeline process on cuda:0) with the stage2 UNet + full SD VAE +
Whisper-tiny at 256^2 (random weights, synthetic clips): a 10-window clip cold (the first
request: engine build + graph capture), the same clip warm, then an 11-window clip, which
shares the 10-window clip's 12-window engine (pipeline.plan_window_batches), then the
lengths the bucket padding is worst for: 9 windows (an exact 9-window
engine, cold), 25 windows (one 28-window engine: cold, then warm) and 49 windows (2 x 28
on the same engine).
usage: python scripts/serve_latency.py"""
import os
import sys
import tempfile
import time
import wave

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def random_stage2_pipeline(rank):
    import torch

    from latentsync_amd.audio import Audio2Feature
    from latentsync_amd.config import STAGE2_MODEL
    from latentsync_amd.pipeline import LipsyncPipeline
    from latentsync_amd.scheduler import DDIMScheduler
    from latentsync_amd.unet import UNet3DConditionModel
    from latentsync_amd.vae import AutoencoderKL
    import bench
    dev = torch.device("cuda", rank)
    unet = UNet3DConditionModel(**STAGE2_MODEL).init_weights(41).to(dev).eval()
    vae = AutoencoderKL().init_weights(51).to(dev)
    return LipsyncPipeline(vae, Audio2Feature.random(2, device=dev), unet, DDIMScheduler(**bench.SCHED_CFG))


def _clip(d, vid, n_frames, seconds, R=256):
    import torch
    g = torch.Generator().manual_seed(n_frames)
    low = torch.rand((n_frames, 3, R // 16, R // 16), generator=g)
    faces = (torch.nn.functional.interpolate(low, size=(R, R), mode="bilinear") * 255).round().to(torch.uint8)
    torch.save({"faces": faces, "boxes": [[0, 0, R, R]] * n_frames, "affine_matrices": [np.eye(2, 3)] * n_frames},
               os.path.join(d, f"{vid}.pth"))
    open(os.path.join(d, f"{vid}.mp4"), "wb").close()
    a = np.random.default_rng(1).normal(0, 0.1, int(seconds * 16000)).clip(-1, 0.999)
    with wave.open(os.path.join(d, f"{vid}.wav"), "wb") as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(16000)
        f.writeframes((a * 32768).astype("<i2").tobytes())


def main():
    from fastapi.testclient import TestClient

    from latentsync_amd import serve as S
    from latentsync_amd.pipeline import plan_window_batches
    d = tempfile.mkdtemp(prefix="ls_serve_")
    _clip(d, "c10", 160, 6.4)
    _clip(d, "c11", 176, 7.04)
    # the audio of a clip of 16 w frames pads to w + 1 windows (repeat.pad_whisper_chunks_end)
    for w in (9, 25, 49):
        _clip(d, f"c{w}", 16 * (w - 1), 16 * (w - 1) / 25)
    worker = S.ProcessWorker(0, "serve_latency:random_stage2_pipeline", request_timeout=900.0, data_dir=d,
                             results_dir=os.path.join(d, "res"), resolution=256)
    app = S.create_app([worker])
    with TestClient(app) as c:
        for rid, vid, what in (("r1", "c10", "cold (engine build + capture)"),
                               ("r2", "c10", "warm"), ("r3", "c11", "a longer clip, same engine bucket"),
                               ("r4", "c9", "cold (bucket 12 would pad 33 %: exact size)"), ("r5", "c25", "cold"),
                               ("r6", "c25", "warm"), ("r7", "c49", "the same engine")):
            t0 = time.time()
            r = c.post("/process", json={"id": rid, "video_id": vid, "audio_url": "file://" + os.path.join(d, f"{vid}.wav")})
            wall = time.time() - t0
            assert r.status_code == 200, r.text
            body = r.json()
            n = np.load(body["output_url"])["frames"].shape[0]
            E, batches = plan_window_batches(list(range(n // 16)), 48)
            print(f"/process {n // 16} windows ({len(batches)} x {E}-window engine), {what}: {n} frames, server elapsed "
                  f"{body['elapsed_time']:.2f} s, client wall {wall:.2f} s, {n / body['elapsed_time']:.1f} frames/s",
                  flush=True)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
