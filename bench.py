"""Benchmark: lip-synced frames/sec at 256x256, 16-frame window, 20 DDIM steps
(BASELINE.json "metric", configs[1]; configs[3] when launched on N GPUs).

One "step" = one batch of `--windows-per-batch` (default 48 at configs[1]) independent
16-frame windows of a clip through the whole hot path on one GPU: pixel prep ->
VAE encode x2 -> 20 x (UNet3D fwd + CFG + DDIM) -> VAE decode -> paste-back,
inputs resident in HBM.  Every window is computed exactly as alone (per-window
GroupNorm statistics / temporal attention; tests/test_gpu_pipeline.py); the
batch only makes each kernel launch larger.  The JSON also reports the latency
of a single window run alone (`single_window`).

Multi-GPU (configs[3]): one process per GPU.  `--gpus N` run
directly spawns N fresh worker processes of this script (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* in their environment) BEFORE anything touches the GPU and
exits with the first failing worker's status; under torchrun the process is
already a worker.  Every rank runs its own windows (weak scaling; rank r owns
the contiguous block of K*nw windows [r*K*nw, (r+1)*K*nw) of the job) and the
decoded frames of all ranks are all-gathered once at the end of the timed loop as
the fp32 pasted frames LipsyncPipeline.run_windows exchanges (RCCL over xGMI, the
only collective; the receive buffer is already in clip order, and the uint8 clip
is derived from it in bounded chunks; the process group carries a timeout so a
dead rank aborts the gather instead of hanging it).  The per-rank memory of that
exchange is `exchange_bytes` (K = 20, 48 windows, 8 ranks: 133 GB beside the
engine); the line reports the measured peak (`peak_hbm_gb`).  `n_gpus` is the world size the process group
reports.  Rank 0 prints ONE JSON line.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1|2|4]
"""
import argparse
import datetime
import json
import math
import os
import socket
import subprocess
import sys
import threading
import time
import traceback

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# importing these does not touch the GPU (the HIP library loads on first use)
from latentsync_amd import ops  # noqa: E402
from latentsync_amd import unet as U  # noqa: E402
from latentsync_amd.pipeline import frames_to_u8, load_fixed_mask  # noqa: E402

SCHED_CFG = dict(beta_end=0.012, beta_schedule="scaled_linear", beta_start=0.00085, clip_sample=False,
                 num_train_timesteps=1000, set_alpha_to_one=False, steps_offset=1)  # configs/scheduler_config.json
# algorithmic TFLOP: UNet fwd at B=1, F=16; VAE encode / decode per frame
WORK_TF = {256: (4.0505, 0.2727, 0.6222), 512: (17.626, 1.1167, 2.5145)}
PEAK_BF16_TF = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
# BASELINE.json configs this bench can run on one GPU (configs[0] is the CPU-only
# plumbing case, configs[3] is configs[1] sharded over 8 ranks)
# windows: independent 16-frame windows of a clip batched per UNet call (measured on MI355X:
# 8 -> 110.2, 16 -> 113.3 frames/s at configs[1], profiles/r01f_bench.json; same box, round 2
# (profiles/r02k_wpb_sweep.txt): 16 -> 121.4, 24 -> 122.9, 32 -> 123.2; configs[4] 2 -> 27.3, 4 -> 28.1;
# round 3, after the kernel changes (profiles/r03p_wpb_sweep.txt, two boxes, two rounds each):
# 24 -> 130.0-130.4, 32 -> 129.5, 48 -> 130.6-130.7 on one, 40 -> 133.9-134.4, 48 -> 135.0-135.8,
# 56 -> 134.4-135.0, 64 -> 135.2-135.6 on the other)
PRESETS = {
    1: dict(resolution=256, guidance=1.0, steps=20, windows=48),
    2: dict(resolution=256, guidance=2.0, steps=50, windows=8),
    # configs[4] names "fp8 MFMA attention": ls_attention_fp8 (P.V on the block-scaled e4m3
    # MFMA) is built and parity-tested, but measured no faster than bf16 on the same box
    # (DESIGN.md §7), so the bench default is bf16; --attn-precision fp8 runs it
    4: dict(resolution=512, guidance=1.0, steps=20, windows=4, attn="bf16"),
}


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


def restore_probe(decoded, device, H=1080, W=1920, iters=5):
    """restore_video (outside the headline's timed region, §8(d)):
    paste the 16 decoded faces of one window back into synthetic 1080p frames with
    per-frame align matrices (face ~1.6x upscaled into the frame, jittered), on
    the device: face resize + ls_restore_frames.  Timed with HIP events on the
    current stream; includes the host matrix/ROI planning and the frame clone."""
    from latentsync_amd import restore as RS
    n = decoded.shape[0]
    g = torch.Generator().manual_seed(7)
    low = torch.rand((n, 3, H // 40, W // 40), generator=g)
    frames = (torch.nn.functional.interpolate(low, size=(H, W), mode="bilinear") * 255).to(torch.uint8)
    frames = frames.permute(0, 2, 3, 1).contiguous().to(device)
    mats = []
    for i in range(n):
        s, th = 0.62 + 0.01 * math.sin(i), 0.05 * math.cos(i)
        c, sn = math.cos(th) * s, math.sin(th) * s
        cx, cy = 960 + 4 * i, 480 - 2 * i
        mats.append([[c, -sn, 105 - (c * cx - sn * cy)], [sn, c, 140 - (sn * cx + c * cy)]])
    boxes = [[0, 0, 210, 280]] * n
    rest = RS.AlignRestore(device)
    out = RS.restore_video(decoded, frames, boxes, mats, rest)  # warm-up (tables)
    torch.cuda.synchronize(device)
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(st)
    for _ in range(iters):
        out = RS.restore_video(decoded, frames, boxes, mats, rest)
    e1.record(st)
    torch.cuda.synchronize(device)
    wall = (time.perf_counter() - t0) / iters
    gpu_ms = e0.elapsed_time(e1) / iters
    changed = float((out != frames).any(dim=-1).float().mean())
    return {"workload": f"{n} decoded 256^2 faces -> {W}x{H} frames (resize to 280x210, Lanczos4 warp, "
                        "erode/blur soft mask, blend)",
            "frames_per_s": round(n / wall, 1), "ms_per_window_wall": round(wall * 1e3, 3),
            "ms_per_window_gpu": round(gpu_ms, 3), "frame_fraction_changed": round(changed, 4)}


def step_probe(engine, device):
    """Live HIP-event timing of one denoising step (UNet fwd + CFG/DDIM), on the
    stream the kernels run on (eager launches, same kernels as the graph):
      * every ls_conv2d call (the dominant kernel family, conv_gemm_*: GEMM + its
        split-K reduce when split) -- algorithmic FLOPs 2*M*N*Cin*k^2 per call;
      * every ls_attention call (SDPA) -- 4*batch*heads*nq*nk*d FLOPs;
      * every Transformer3DModel / motion-module block as a
        whole: its GEMM + SDPA FLOPs over its wall time = the "UNet attention"
        MFMA utilisation of the north star."""
    from latentsync_amd import unet as U
    convs, attns, blocks, conv_bytes = [], [], [], []
    depth = [0]
    orig_conv, orig_attn = ops.conv, ops.attention
    orig_t, orig_m = U._Transformer.__call__, U._Motion.__call__

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        return e

    def conv(x, pw, **kw):
        # one record per ls_conv2d C-ABI call: ops.conv(aff_materialize=True) re-enters
        # ops.conv after its GroupNorm-apply pass, and only that inner call is the GEMM
        n0 = len(convs)
        e0 = ev()
        y = orig_conv(x, pw, **kw)
        e1 = ev()
        if len(convs) > n0:
            return y
        x2 = kw.get("x2")
        cin = x.shape[-1] + (x2.shape[-1] if x2 is not None else 0)
        M = y.shape[0] * y.shape[1] * y.shape[2]
        f = 2.0 * M * pw.N * cin * pw.ksize * pw.ksize
        # algorithmic HBM bytes: input pixels once, weights once, output (+ residual) once
        nb = (x.numel() + (x2.numel() if x2 is not None else 0) + pw.w.numel()) * 2 + y.numel() * y.element_size()
        if kw.get("res") is not None:
            nb += y.numel() * 2
        conv_bytes.append(nb)
        convs.append((e0, e1, f))
        if depth[0]:
            blocks[-1][2] += f
        return y

    def attention(q, k, v, o, **kw):
        e0 = ev()
        r = orig_attn(q, k, v, o, **kw)
        e1 = ev()
        f = 4.0 * kw["batch"] * kw["heads"] * kw["nq"] * kw["nk"] * kw["head_dim"]
        attns.append((e0, e1, f))
        if depth[0]:
            blocks[-1][2] += f
        return r

    def wrap(fn):
        def call(self, *a, **kw):
            blocks.append([ev(), None, 0.0])
            depth[0] += 1
            try:
                return fn(self, *a, **kw)
            finally:
                depth[0] -= 1
                blocks[-1][1] = ev()
        return call

    orig_tattn = ops.temporal_attention

    def temporal_attention(x2d, pk, n_samples, F, S, out=None):
        # fused LayerNorm + q|k|v GEMM + seq-F SDPA (ls_temporal_attention): the GEMM's
        # 2*rows*3C*C and the SDPA's 4*(n_samples*S)*heads*F*F*d FLOPs (block totals only:
        # the "attention" SDPA figure stays the ls_attention launches)
        r = orig_tattn(x2d, pk, n_samples, F, S, out=out)
        rows, C = x2d.shape
        fg = 2.0 * rows * 3 * C * C
        fa = 4.0 * n_samples * S * pk.heads * F * F * (C // pk.heads)
        if depth[0]:
            blocks[-1][2] += fg + fa
        return r

    orig_xa = ops.cross_attention_block

    def cross_attention_block(x2d, ln_stats, pk, kv, L, hw, stats_out, out=None, eps=1e-5):
        # fused norm2 + to_q + SDPA + to_out (ls_cross_attention_block): the algorithmic
        # 2*M*C*C (q) + 4*M*heads*L*d (SDPA) + 2*M*C*C (out) FLOPs
        r = orig_xa(x2d, ln_stats, pk, kv, L, hw, stats_out, out=out, eps=eps)
        M, C = x2d.shape
        if depth[0]:
            blocks[-1][2] += 4.0 * M * C * C + 4.0 * M * C * L
        return r

    orig_ff = ops.feedforward

    def feedforward(x2d, ln_stats, w1, w2, w2ff, out=None):
        # fused LayerNorm + GEGLU W1 + W2 + residual (ls_feedforward): 2*M*2I*C + 2*M*C*I FLOPs
        r = orig_ff(x2d, ln_stats, w1, w2, w2ff, out=out)
        M, C = x2d.shape
        if depth[0]:
            blocks[-1][2] += 2.0 * M * w1.N * C + 2.0 * M * C * (w1.N // 2)
        return r

    orig_chain = ops.ff_chain

    def ff_chain(o2d, h1, xb, pk, **kw):
        # fused to_out + FeedForward + proj_out (ls_ff_chain): 2*M*C*C twice + 2*M*2I*C + 2*M*C*I FLOPs
        r = orig_chain(o2d, h1, xb, pk, **kw)
        M, C = o2d.shape
        if depth[0]:
            blocks[-1][2] += 4.0 * M * C * C + 2.0 * M * 2 * pk.inner * C + 2.0 * M * C * pk.inner
        return r

    ops.conv, ops.attention, ops.temporal_attention, ops.feedforward = conv, attention, temporal_attention, feedforward
    ops.cross_attention_block, ops.ff_chain = cross_attention_block, ff_chain
    U._Transformer.__call__, U._Motion.__call__ = wrap(orig_t), wrap(orig_m)
    try:
        engine._step()
    finally:
        ops.conv, ops.attention, ops.temporal_attention, ops.feedforward = orig_conv, orig_attn, orig_tattn, orig_ff
        ops.cross_attention_block, ops.ff_chain = orig_xa, orig_chain
        U._Transformer.__call__, U._Motion.__call__ = orig_t, orig_m
    torch.cuda.synchronize(device)

    def agg(recs):
        ms = sum(a.elapsed_time(b) for a, b, _ in recs)
        fl = sum(f for _, _, f in recs)
        return dict(launches=len(recs), total_ms=ms, avg_ms=ms / max(1, len(recs)),
                    tflops=fl / (ms * 1e-3) / 1e12 if ms else 0.0, flops_per_launch=fl / max(1, len(recs)))
    c = agg(convs)
    c["algo_bytes_per_launch"] = sum(conv_bytes) / max(1, len(conv_bytes))
    return c, agg(attns), agg(blocks)


def traffic_per_call():
    """Measured HBM bytes per ls_conv2d call (scripts/pmc_traffic.py over two
    rocprofv3 --pmc passes of this bench, committed under profiles/)."""
    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    return round(json.load(open(p))["hbm_bytes_per_call"])


def cpu_share():
    """Host cores this process may actually use: the cgroup CPU quota when one is
    set (the GPU box grants a 16-core share of a larger host whose
    os.cpu_count() counts every core), else the affinity mask."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(unet, vae, R=256, steps=20, guidance=1.0, sample_steps=None):
    """The oracle (plain PyTorch fp32 restatement, oracle/ref_cpu.py) on the host
    cores: ONE full 16-frame window of the same configuration, end to end --
    pixel prep, VAE encode x2 (16 frames each), `steps` UNet forwards (+CFG) with
    the DDIM step, VAE decode of 16 frames, paste-back (oracle.pipeline_window).
    Nothing is extrapolated when sample_steps is None; configs other than the
    headline may pass a smaller sample_steps, and the sample text says so."""
    from oracle import ref_cpu as O
    threads = cpu_share()
    torch.set_num_threads(threads)
    usd, vsd = unet._sd, vae._sd
    F, h = 16, R // 8
    faces, audio, init, em, er = synthetic_window(F, R, h, unet.config.cross_attention_dim, 3, "cpu")
    mask = load_fixed_mask(R)
    n = steps if sample_steps is None else min(sample_steps, steps)

    def window(k):
        # a progress line on stderr every 60 s: an oracle window at 512^2 runs for minutes
        # without output, which a supervisor watching the output would take for a hang
        done = threading.Event()

        def beat():
            t_b = time.perf_counter()
            while not done.wait(60.0):
                print(f"cpu_baseline: oracle window ({k} DDIM steps) running, {time.perf_counter() - t_b:.0f} s",
                      file=sys.stderr, flush=True)
        hb = threading.Thread(target=beat, daemon=True)
        hb.start()
        try:
            with torch.no_grad():
                t0 = time.perf_counter()
                O.pipeline_window(usd, dict(unet.config), vsd, faces, mask, audio, init, em, er, num_steps=k,
                                  guidance_scale=guidance)
                return time.perf_counter() - t0
        finally:
            done.set()
            hb.join()
    t = window(n)
    if n == steps:
        sample = (f"one full {R}x{R} 16-frame window, {steps} DDIM steps, guidance {guidance}: VAE enc x2 + "
                  f"{steps} UNet fwd + DDIM + VAE dec + paste (oracle/ref_cpu.py pipeline_window, fp32) in {t:.1f} s")
        value = F / t
    else:
        # two-point fit: t(n) - t(n-1) is one DDIM step (UNet fwd(s) + CFG + DDIM); the
        # rest (pixel prep, VAE encode x2, decode, paste) is counted once, not scaled
        t_less = window(n - 1)
        per_step = max(t - t_less, 0.0)
        fixed = max(t - n * per_step, 0.0)
        est = fixed + steps * per_step
        sample = (f"{R}x{R} 16-frame window timed at {n} and {n - 1} DDIM steps ({t:.1f} / {t_less:.1f} s): "
                  f"one step {per_step:.1f} s, VAE + prep + paste {fixed:.1f} s once; the step share scaled to "
                  f"{steps} steps = {est:.1f} s (extrapolated)")
        value = F / est
    return dict(value=round(value, 5), unit="frames/s", cores=threads, kind="port", sample=sample,
                window_s=round(t, 2), cpu_model=cpu_model(), os_cpu_count=os.cpu_count(),
                threads_note="torch.set_num_threads(cgroup CPU share); os.cpu_count() counts the whole host")


def whisper_probe(device, seconds, seed=2):
    """Audio2Feature.audio2feat + feature2chunks for one
    clip of `seconds`, on the GPU (HIP events) and on the oracle (host cores).
    Outside the headline's timed region; reported beside it (§8(d))."""
    from latentsync_amd.audio import Audio2Feature
    from oracle import ref_cpu as O
    sr = 16000
    wav = (torch.randn(int(seconds * sr), generator=torch.Generator().manual_seed(seed)) * 0.1).numpy()
    a2f = Audio2Feature.random(seed, device=device)
    for _ in range(2):  # warm-up (weights packed, kernels loaded)
        a2f.feature2chunks(a2f._audio2feat(wav), 25)
    torch.cuda.synchronize(device)
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    iters = 3
    t0 = time.perf_counter()
    e0.record(st)
    for _ in range(iters):
        chunks = a2f.feature2chunks(a2f._audio2feat(wav), 25)
    e1.record(st)
    torch.cuda.synchronize(device)
    wall = (time.perf_counter() - t0) / iters
    gpu_ms = e0.elapsed_time(e1) / iters
    torch.set_num_threads(cpu_share())
    filt = a2f._filters.cpu().float()
    t0 = time.perf_counter()
    with torch.no_grad():
        feat = O.whisper_features(a2f.sd, torch.from_numpy(wav), filt)
        O.feature2chunks(feat)
    cpu_s = time.perf_counter() - t0
    return {"clip_s": seconds, "chunks": len(chunks), "gpu_ms": round(gpu_ms, 3), "gpu_wall_ms": round(wall * 1e3, 3),
            "cpu_s": round(cpu_s, 3), "cpu_cores": cpu_share()}


class PlumbingEngine:
    """CPU stand-in for WindowEngine used by `--plumbing` (tests/test_bench_launch.py):
    the same launcher, process group, window ownership and end-of-loop gather as
    the GPU bench, with the window's compute replaced by writing the global window
    index into its frames so the gathered clip order can be checked."""

    def __init__(self, F, R, nw, rank, world, owned):
        self.F, self.R, self.nw, self.rank, self.world = F, R, nw, rank, world
        self.owned = owned  # global indices of this rank's windows, in run order
        self.out = torch.zeros((nw * F, 3, R, R), dtype=torch.float32)
        self.calls = 0

    def run(self):
        for k in range(self.nw):
            local = self.calls * self.nw + k
            # window index w encoded as the pasted value whose uint8 is w % 251
            w = self.owned[local % len(self.owned)] % 251
            self.out[k * self.F:(k + 1) * self.F] = (w + 0.5) / 255 * 2 - 1
        self.calls += 1


def exchange_bytes(world, K, nw, F=16, R=256):
    """Per-rank memory of the end-of-loop exchange (beyond the engine): this rank's
    fp32 pasted frames (K*nw windows), the all-gather's receive buffer (world*K*nw
    windows, shard.gather_bytes; none at world 1), the uint8 clip of every window and
    frames_to_u8's two chunk temporaries."""
    from latentsync_amd import shard
    from latentsync_amd.pipeline import U8_CHUNK
    win32 = F * 3 * R * R * 4
    n = world * K * nw
    return (K * nw * win32 + shard.gather_bytes(n, world, win32) + n * F * R * R * 3
            + 2 * U8_CHUNK * 3 * R * R * 4)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n):
    """Spawn n fresh worker processes of this script, one per GPU, before anything
    touches the GPU (the parent never initialises HIP).  A worker that fails ends
    the job: the others (the exact processes started here) are terminated and the
    first failure's status is returned."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    return rc


def worker(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    plumbing = args.plumbing
    if plumbing:
        device = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(rank=rank, world_size=world, timeout=datetime.timedelta(seconds=args.dist_timeout))
        if plumbing:
            dist.init_process_group("gloo", **kw)
        else:
            dist.init_process_group("nccl", device_id=device, **kw)
        world = dist.get_world_size()  # n_gpus comes from the process group itself
    from latentsync_amd import shard

    F, R = 16, args.resolution
    h = R // 8
    nw = args.windows_per_batch
    K, W = args.steps, args.warmup
    # rank r owns the contiguous block of K*nw windows of the job (shard.rank_windows)
    owned = shard.rank_windows(world * K * nw, world, rank)
    if plumbing:
        eng = PlumbingEngine(F, R, nw, rank, world, owned)
        unet = vae = None
    else:
        from latentsync_amd.config import STAGE2_MODEL
        from latentsync_amd.pipeline import WindowEngine
        from latentsync_amd.scheduler import DDIMScheduler
        from latentsync_amd.unet import UNet3DConditionModel
        from latentsync_amd.vae import AutoencoderKL
        unet = UNet3DConditionModel(**STAGE2_MODEL).init_weights(41).to(device).eval()
        unet.set_attention_precision(args.attn_precision)
        vae = AutoencoderKL().init_weights(51).to(device)
        sched = DDIMScheduler(**SCHED_CFG)
        eng = WindowEngine(unet, vae, sched, F, R, args.inference_steps, args.guidance,
                           use_graphs=not args.no_graphs, windows=nw)
        faces, audio, init, em, er = synthetic_window(F * nw, R, h, unet.config.cross_attention_dim, 1000 + rank,
                                                      device)
        mask = load_fixed_mask(R).to(device)
        eng.load(faces, mask, audio, init, em, er)

    def sync():
        if not plumbing:
            torch.cuda.synchronize(device)

    FB = F * nw  # frames per step (batch of windows)
    # this rank's K*nw windows, kept as the fp32 pasted frames LipsyncPipeline.run_windows gathers
    mine = torch.empty((len(owned), F, 3, R, R), dtype=torch.float32, device=device)
    for _ in range(max(W, 1) if not (args.no_graphs or plumbing) else W):
        eng.run()
    if plumbing:
        eng.calls = 0
    engine_bytes = None if plumbing else torch.cuda.max_memory_allocated(device)
    if args.fail_rank == rank:
        raise RuntimeError(f"injected failure on rank {rank} (--fail-rank)")
    if args.stall_rank == rank:
        time.sleep(3600)  # a hung rank: the others' barrier / gather must time out
    sync()
    if world > 1:
        dist.barrier()
    sync()
    ev_step = []
    t0 = time.perf_counter()
    for k in range(K):
        if not plumbing:
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
        eng.run()
        if not plumbing:
            e1.record(st)
            ev_step.append((e0, e1))
        mine[k * nw:(k + 1) * nw].copy_(eng.out.view(nw, F, 3, R, R))
    # decoded frames of every rank back in clip order: ONE all-gather over xGMI, at the
    # end, into a receive buffer that is already clip order, then the uint8 clip in
    # bounded chunks -- exactly LipsyncPipeline.run_windows' exchange
    clip = shard.gather_windows(mine, world * K * nw)
    gathered = frames_to_u8(clip.flatten(0, 1)).view(world * K * nw, F, R, R, 3)
    del clip
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    frames = world * K * FB
    value = frames / elapsed
    res = {
        "metric": f"lip-synced frames/sec at {R}x{R}, 16-frame window, {args.inference_steps} DDIM steps",
        "value": round(value, 3), "unit": "frames/s", "n_gpus": world, "steps": K, "warmup": W,
        "ms_per_step": round(elapsed / K * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic (seeded faces/audio/noise, random-init weights)",
        "config": {"workload": f"configs[{args.config}]: {R}x{R} x16-frame windows, "
                               f"{args.inference_steps} DDIM steps, guidance {args.guidance}, "
                               "LatentSync-1.5 UNet + SD-VAE, bf16"
                               + ("; spatial self-attention P.V in fp8 e4m3 (block-scaled MFMA)"
                                  if args.attn_precision == "fp8" else "") + "; "
                               f"{nw} independent windows of a clip batched per UNet call",
                   "windows_per_rank": K * nw, "windows_per_batch": nw, "frames_per_window": F,
                   "global_batch": world * nw * F, "resolution": R,
                   "parallelism": f"dp{world} (window sharding, RCCL all-gather of decoded frames)"},
    }
    gib = 1024 ** 3
    res["memory"] = {"exchange_gb": round(exchange_bytes(world, K, nw, F, R) / gib, 3),
                     "exchange_gb_at_8_ranks_k20": round(exchange_bytes(8, 20, nw, F, R) / gib, 3)}
    if plumbing:
        want = torch.arange(world * K * nw, dtype=torch.int64) % 251
        got = gathered[:, 0, 0, 0, 0].to(torch.int64)
        res["plumbing"] = {"backend": dist.get_backend() if world > 1 else "none",
                           "gathered_windows": int(gathered.shape[0]),
                           "clip_order_ok": bool(torch.equal(got, want)) and
                           bool((gathered == gathered[:, :1, :1, :1, :1]).all())}
        res["dtype"] = "u8"
        if rank == 0:
            print(json.dumps(res), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    window_ms = sum(a.elapsed_time(b) for a, b in ev_step) / K
    # HBM high-water mark of the timed job (engine + this rank's frames + the exchange),
    # before the probes below allocate their own engines
    res["peak_hbm_gb"] = round(torch.cuda.max_memory_allocated(device) / gib, 3)
    res["memory"].update({"engine_gb": round(engine_bytes / gib, 3), "hbm_total_gb": round(
        torch.cuda.get_device_properties(device).total_memory / gib, 1)})
    res["memory"]["footprint_gb_at_8_ranks_k20"] = round(res["memory"]["engine_gb"] +
                                                         res["memory"]["exchange_gb_at_8_ranks_k20"], 3)
    probe, attn_probe, blk_probe = step_probe(eng, device)
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
    restore = None
    if rank == 0 and R == 256:
        restore = restore_probe(eng.out[:F].clone(), device)
    Bu = 2 if args.guidance > 1 else 1
    unet_tf, enc_tf, dec_tf = WORK_TF[R]
    tf_per_frame = (args.inference_steps * unet_tf * Bu + 32 * enc_tf + 16 * dec_tf) / 16
    res.update({
        "batch_ms_gpu_events": round(window_ms, 3),
        "single_window": single,
        "window_mfma_frac": round(tf_per_frame * value / world / PEAK_BF16_TF, 4),
        "roofline": {"bound": "mfma",
                     "kernel": "conv_gemm family: every ls_conv2d call of one UNet fwd (conv_gemm_* tiled / "
                               "gemm_rowblock / conv3x3_halo GEMM + split-K reduce; one launch per call)",
                     "achieved": round(probe["tflops"], 2), "peak": PEAK_BF16_TF, "unit": "TFLOP/s",
                     "frac": round(probe["tflops"] / PEAK_BF16_TF, 4), "traffic": traffic_per_call(),
                     "traffic_unit": "HBM bytes per ls_conv2d call (rocprofv3 PMC, profiles/pmc_traffic.json)",
                     "launches": probe["launches"], "avg_launch_ms": round(probe["avg_ms"], 4),
                     "flops_per_launch": probe["flops_per_launch"],
                     "algorithmic_bytes_per_launch": round(probe["algo_bytes_per_launch"]),
                     "peak_measured": measured_peak()},
        "attention": {"kernel": "ls_attention (SDPA: spatial self, audio cross, temporal)",
                      "achieved_tflops": round(attn_probe["tflops"], 2), "launches": attn_probe["launches"],
                      "avg_launch_ms": round(attn_probe["avg_ms"], 4),
                      "frac": round(attn_probe["tflops"] / PEAK_BF16_TF, 4),
                      "blocks": "Transformer3DModel + motion modules (a14-a17): GEMM + SDPA FLOPs / block wall time",
                      "blocks_tflops": round(blk_probe["tflops"], 2), "blocks_n": blk_probe["launches"],
                      "blocks_ms": round(blk_probe["total_ms"], 3),
                      "blocks_mfma_frac": round(blk_probe["tflops"] / PEAK_BF16_TF, 4)},
        "restore_video": restore,
    })
    if rank == 0 and not args.no_whisper:
        # Whisper features for the clip of one step's frames (FB frames at 25 fps),
        # outside the headline; value_incl_whisper adds one clip's feature time per step
        wp = whisper_probe(device, FB / 25.0)
        res["whisper"] = wp
        res["value_incl_whisper"] = round(frames / (elapsed + K * wp["gpu_wall_ms"] * 1e-3), 3)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sample_steps = None if args.config == 1 else 2
        res["cpu_baseline"] = cpu_baseline(unet, vae, R, args.inference_steps, args.guidance, sample_steps)
        res["speedup_vs_cpu"] = round(value / res["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def measured_peak():
    """Measured dense bf16 GEMM ceiling on the box (scripts/gemm_ceiling.py ->
    profiles/gemm_ceiling.json), or None before it has been measured."""
    p = os.path.join(REPO, "profiles", "gemm_ceiling.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f).get("best_tflops")


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=1, choices=sorted(PRESETS),
                    help="BASELINE.json configs[i]: 1 = 256^2/20 steps/g 1.0 (headline), 2 = 50 steps/g 2.0 (CFG), "
                         "4 = 512^2/20 steps")
    ap.add_argument("--guidance", type=float, default=None)
    ap.add_argument("--attn-precision", choices=("bf16", "fp8"), default=None,
                    help="spatial self attention: bf16 (default) or fp8 P.V (configs[4]'s fp8 option)")
    ap.add_argument("--inference-steps", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-whisper", action="store_true")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--windows-per-batch", type=int, default=None,
                    help="independent 16-frame windows batched through one UNet call per DDIM step")
    ap.add_argument("--no-single-window", action="store_true", help="skip the 1-window latency leg")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="process-group timeout (s): a rank that dies aborts the others' collectives")
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU/gloo dry run of the launcher, window sharding and gather (no GPU)")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--stall-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    pre = PRESETS[args.config]
    if args.guidance is None:
        args.guidance = pre["guidance"]
    if args.inference_steps is None:
        args.inference_steps = pre["steps"]
    if args.attn_precision is None:
        args.attn_precision = pre.get("attn", "bf16")
    if args.windows_per_batch is None:
        args.windows_per_batch = pre["windows"] if not args.plumbing else 2
    args.resolution = pre["resolution"] if not args.plumbing else 8
    return args


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args.gpus))
    try:
        worker(args)
    except BaseException:
        rank = os.environ.get("RANK", "0")
        sys.stderr.write(f"[bench rank {rank}] failed:\n{traceback.format_exc()}")
        sys.stderr.flush()
        os._exit(1)  # no destructor waits on peers that may be blocked in a collective


if __name__ == "__main__":
    main()
