"""Benchmark: lip-synced frames/sec at 256x256, 16-frame window, 20 DDIM steps
(BASELINE.json "metric", configs[1]; configs[3] when launched on N GPUs).

One "step" = one batch of `--windows-per-batch` (default 8) independent
16-frame windows of a clip through the whole hot path on one GPU: pixel prep ->
VAE encode x2 -> 20 x (UNet3D fwd + CFG + DDIM) -> VAE decode -> paste-back,
inputs resident in HBM.  Every window is computed exactly as alone (per-window
GroupNorm statistics / temporal attention; tests/test_gpu_pipeline.py); the
batch only makes each kernel launch larger.  The JSON also reports the latency
of a single window run alone (`single_window`).  With N ranks (one process per GPU,
torch.distributed over RCCL) every rank runs its own windows (weak scaling) and
the decoded uint8 frames of all ranks are all-gathered once at the end of the
timed loop (the only collective).  Prints ONE JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--guidance 1.0]
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from latentsync_amd import ops, shard  # noqa: E402
from latentsync_amd.config import STAGE2_MODEL  # noqa: E402
from latentsync_amd.pipeline import WindowEngine, load_fixed_mask  # noqa: E402
from latentsync_amd.scheduler import DDIMScheduler  # noqa: E402
from latentsync_amd.unet import UNet3DConditionModel  # noqa: E402
from latentsync_amd.vae import AutoencoderKL  # noqa: E402

SCHED_CFG = dict(beta_end=0.012, beta_schedule="scaled_linear", beta_start=0.00085, clip_sample=False,
                 num_train_timesteps=1000, set_alpha_to_one=False, steps_offset=1)  # configs/scheduler_config.json
UNET_TF = 4.0505      # TF per UNet fwd, B=1, F=16, 256^2
VAE_ENC_TF = 0.2727   # per frame
VAE_DEC_TF = 0.6222   # per frame
PEAK_BF16_TF = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)


def synthetic_window(F, R, h, cross_dim, seed, device):
    """Seeded synthetic inputs: smooth random faces, the fixed
    mouth mask, N(0,1) audio chunks, seed-1247 initial latents shared across
    frames, seeded VAE posterior noise."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    low = torch.rand((F, 3, R // 16, R // 16), generator=g)
    faces = (torch.nn.functional.interpolate(low, size=(R, R), mode="bilinear", align_corners=False) * 255)
    faces = faces.round().clamp(0, 255).to(torch.uint8)
    audio = torch.randn((F, 50, cross_dim), generator=g)
    init = torch.randn((1, 4, 1, h, h), generator=torch.Generator().manual_seed(1247))
    em = torch.randn((F, 4, h, h), generator=g)
    er = torch.randn((F, 4, h, h), generator=g)
    return [t.to(device) for t in (faces, audio, init, em, er)]


def conv_probe(unet, engine, device):
    """Live HIP-event timing of every ls_conv2d launch of one UNet forward (the
    dominant kernel family, conv_gemm_kernel): algorithmic FLOPs 2*M*N*K_real
    per launch / measured duration, on the stream the kernels run on."""
    recs = []
    orig = ops.conv

    def timed(x, pw, **kw):
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        y = orig(x, pw, **kw)
        e1.record(s)
        x2 = kw.get("x2")
        cin = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
        M = y.shape[0] * y.shape[1] * y.shape[2]
        nreal = pw.N
        flops = 2.0 * M * nreal * cin * pw.ksize * pw.ksize
        recs.append((e0, e1, flops))
        return y

    ops.conv = timed
    try:
        engine._step()
    finally:
        ops.conv = orig
    torch.cuda.synchronize(device)
    ms = [a.elapsed_time(b) for a, b, _ in recs]
    fl = [f for _, _, f in recs]
    tot_ms, tot_f = sum(ms), sum(fl)
    return dict(launches=len(recs), total_ms=tot_ms, avg_ms=tot_ms / len(recs), tflops=tot_f / (tot_ms * 1e-3) / 1e12,
                flops_per_launch=tot_f / len(recs))


def cpu_baseline(unet, vae, seconds_budget=40.0):
    """The oracle (plain PyTorch fp32 restatement, oracle/ref_cpu.py) on host cores:
    one full-size UNet forward at F=16 + VAE encode/decode of one frame, scaled
    to the window (20 UNet + 32 encodes + 16 decodes)."""
    from oracle import ref_cpu as R
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    usd, vsd = unet._sd, vae._sd
    g = torch.Generator().manual_seed(0)
    sample = torch.randn((1, 13, 16, 32, 32), generator=g)
    audio = torch.randn((16, 50, 384), generator=g)
    x = torch.rand((1, 3, 256, 256), generator=g) * 2 - 1
    with torch.no_grad():
        t0 = time.perf_counter()
        R.unet_forward(usd, STAGE2_MODEL, sample, 951, audio)
        t_unet = time.perf_counter() - t0
        t0 = time.perf_counter()
        R.vae_encode_moments(vsd, x)
        t_enc = time.perf_counter() - t0
        t0 = time.perf_counter()
        R.vae_decode(vsd, torch.randn((1, 4, 32, 32), generator=g))
        t_dec = time.perf_counter() - t0
    t_window = 20 * t_unet + 32 * t_enc + 16 * t_dec
    return dict(value=16.0 / t_window, unit="frames/s", cores=threads, kind="port",
                sample=f"1 UNet fwd (F=16) {t_unet:.2f}s + 1-frame VAE enc {t_enc:.2f}s + dec {t_dec:.2f}s, "
                       f"scaled to 20 UNet + 32 enc + 16 dec per 16-frame window (oracle/ref_cpu.py fp32)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--guidance", type=float, default=1.0)
    ap.add_argument("--inference-steps", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--windows-per-batch", type=int, default=8,
                    help="independent 16-frame windows batched through one UNet call per DDIM step")
    ap.add_argument("--no-single-window", action="store_true", help="skip the 1-window latency leg")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)

    F, R = 16, 256
    h = R // 8
    unet = UNet3DConditionModel(**STAGE2_MODEL).init_weights(41).to(device).eval()
    vae = AutoencoderKL().init_weights(51).to(device)
    sched = DDIMScheduler(**SCHED_CFG)
    nw = args.windows_per_batch
    eng = WindowEngine(unet, vae, sched, F, R, args.inference_steps, args.guidance, use_graphs=not args.no_graphs,
                       windows=nw)
    faces, audio, init, em, er = synthetic_window(F * nw, R, h, unet.config.cross_attention_dim, 1000 + rank, device)
    mask = load_fixed_mask(R).to(device)
    eng.load(faces, mask, audio, init, em, er)

    K, W = args.steps, args.warmup
    FB = F * nw  # frames per step (batch of windows)
    # rank r owns windows r, r+N, ... of the job (shard.rank_windows); K*nw per rank
    mine = torch.empty((K * nw, F, R, R, 3), dtype=torch.uint8, device=device)
    for _ in range(max(W, 1) if not args.no_graphs else W):
        eng.run()
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    stream = torch.cuda.current_stream()
    ev_step = []
    t0 = time.perf_counter()
    for k in range(K):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.run()
        e1.record(stream)
        ev_step.append((e0, e1))
        mine[k * nw:(k + 1) * nw].copy_(eng.out_u8.view(nw, F, R, R, 3))
    # decoded frames of every rank back in clip order: ONE all-gather over xGMI, at the end
    gathered = shard.gather_windows(mine, world * K * nw)
    torch.cuda.synchronize(device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    window_ms = sum(a.elapsed_time(b) for a, b in ev_step) / K

    probe = conv_probe(unet, eng, device)
    single = None
    if rank == 0 and nw > 1 and not args.no_single_window:
        # latency of ONE window alone (same kernels, 16-frame batch) for reference
        e1w = WindowEngine(unet, vae, sched, F, R, args.inference_steps, args.guidance, use_graphs=not args.no_graphs)
        e1w.load(faces[:F], mask, audio[:F], init, em[:F], er[:F])
        e1w.run()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(2):
            e1w.run()
        torch.cuda.synchronize(device)
        sw = (time.perf_counter() - t0) / 2
        single = {"window_ms": round(sw * 1e3, 3), "frames_per_s": round(F / sw, 3)}
        del e1w
    frames = world * K * FB
    value = frames / elapsed
    tf_per_frame = (args.inference_steps * UNET_TF * (2 if args.guidance > 1 else 1) + 32 * VAE_ENC_TF
                    + 16 * VAE_DEC_TF) / 16
    if rank == 0:
        res = {
            "metric": "lip-synced frames/sec at 256x256, 16-frame window, 20 DDIM steps",
            "value": round(value, 3), "unit": "frames/s", "n_gpus": world, "steps": K, "warmup": W,
            "ms_per_step": round(elapsed / K * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic (seeded faces/audio/noise, random-init weights)",
            "config": {"workload": f"configs[{1 if args.guidance <= 1 else 2}]: 256x256 x16-frame windows, "
                                   f"{args.inference_steps} DDIM steps, guidance {args.guidance}, "
                                   "LatentSync-1.5 UNet + SD-VAE, bf16; "
                                   f"{nw} independent windows of a clip batched per UNet call",
                       "windows_per_rank": K * nw, "windows_per_batch": nw, "frames_per_window": F,
                       "global_batch": world * nw * F, "resolution": R,
                       "parallelism": f"dp{world} (window sharding, RCCL all-gather of decoded frames)"},
            "batch_ms_gpu_events": round(window_ms, 3),
            "single_window": single,
            "window_mfma_frac": round(tf_per_frame * value / world / PEAK_BF16_TF, 4),
            "roofline": {"bound": "mfma", "kernel": "conv_gemm_kernel (all ls_conv2d launches of one UNet fwd)",
                         "achieved": round(probe["tflops"], 2), "peak": PEAK_BF16_TF, "unit": "TFLOP/s",
                         "frac": round(probe["tflops"] / PEAK_BF16_TF, 4), "traffic": None,
                         "launches": probe["launches"], "avg_launch_ms": round(probe["avg_ms"], 4),
                         "flops_per_launch": probe["flops_per_launch"]},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(unet, vae)
            res["speedup_vs_cpu"] = round(value / res["cpu_baseline"]["value"], 1)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
