"""Window-level parity: WindowEngine (graph-captured HIP path) against the CPU
oracle's pipeline_window (lipsync_pipeline.py:500-575 restated) on a reduced
configuration (tiny UNet, reduced-width VAE, 64x64 faces) with injected noise,
with and without classifier-free guidance."""
import pytest
import torch

from conftest import rel_err
from latentsync_amd.config import TINY_MODEL
from latentsync_amd.pipeline import WindowEngine, load_fixed_mask
from latentsync_amd.scheduler import DDIMScheduler
from latentsync_amd.unet import UNet3DConditionModel
from latentsync_amd.vae import AutoencoderKL
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
SCHED = dict(beta_end=0.012, beta_schedule="scaled_linear", beta_start=0.00085, clip_sample=False,
             num_train_timesteps=1000, set_alpha_to_one=False, steps_offset=1)


@pytest.mark.parametrize("guidance,graphs", [(1.0, True), (2.0, True), (1.0, False)])
def test_window_matches_oracle(gpu, guidance, graphs, monkeypatch):
    Fr, Rr, steps = 8, 64, 3
    h = Rr // 8
    unet = UNet3DConditionModel(**TINY_MODEL).init_weights(3).to("cuda").eval()
    vae = AutoencoderKL(block_out_channels=(32, 64, 64, 64)).init_weights(4).to("cuda")
    monkeypatch.setitem(R.VAE_CFG, "block_out_channels", (32, 64, 64, 64))
    g = torch.Generator().manual_seed(5)
    faces = (torch.rand((Fr, 3, Rr, Rr), generator=g) * 255).to(torch.uint8)
    mask = load_fixed_mask(Rr)
    audio = torch.randn((Fr, 50, 384), generator=g)
    init = torch.randn((1, 4, 1, h, h), generator=g)
    em, er = torch.randn((Fr, 4, h, h), generator=g), torch.randn((Fr, 4, h, h), generator=g)
    eng = WindowEngine(unet, vae, DDIMScheduler(**SCHED), Fr, Rr, steps, guidance, use_graphs=graphs)
    eng.load(faces.cuda(), mask.cuda(), audio.cuda(), init.cuda(), em.cuda(), er.cuda())
    out = eng.run().cpu()
    out2 = eng.run().cpu()  # replay must be deterministic
    assert torch.equal(out, out2)
    ref = R.pipeline_window(unet.state_dict(), dict(unet.config), vae._sd, faces, mask, audio, init, em, er,
                            num_steps=steps, guidance_scale=guidance)
    e = rel_err(out, ref)
    print("window rel_err", guidance, graphs, e)
    assert e < 3e-2
    # outside the mouth the original pixels are pasted back exactly (up to bf16 of the prep)
    keep = (mask == 1)[None, None].expand_as(ref)
    assert (out[keep] - ref[keep]).abs().max() < 1e-2


def test_windows_batched_equal_separate(gpu, monkeypatch):
    """Batching W independent windows through one UNet call per DDIM step (the
    engine's `windows` option) computes each window as alone: per-window 5-D
    GroupNorm / temporal attention, [uncond..., cond...] CFG layout.  Checked
    against the fp32 oracle per window (3e-2, as the single-window test) and
    against the single-window engine (3e-2: two bf16 runs whose GEMM tiling /
    split-K differ; a mixed-up window or CFG half would be O(1))."""
    Fr, Rr, steps, W = 8, 64, 2, 2
    h = Rr // 8
    unet = UNet3DConditionModel(**TINY_MODEL).init_weights(6).to("cuda").eval()
    vae = AutoencoderKL(block_out_channels=(32, 64, 64, 64)).init_weights(7).to("cuda")
    monkeypatch.setitem(R.VAE_CFG, "block_out_channels", (32, 64, 64, 64))
    g = torch.Generator().manual_seed(8)
    faces = (torch.rand((W * Fr, 3, Rr, Rr), generator=g) * 255).to(torch.uint8)
    mask = load_fixed_mask(Rr)
    audio = torch.randn((W * Fr, 50, 384), generator=g)
    init = torch.randn((W, 4, 1, h, h), generator=g)
    em, er = torch.randn((W * Fr, 4, h, h), generator=g), torch.randn((W * Fr, 4, h, h), generator=g)
    sched = DDIMScheduler(**SCHED)
    batched = WindowEngine(unet, vae, sched, Fr, Rr, steps, 2.0, windows=W)
    batched.load(faces.cuda(), mask.cuda(), audio.cuda(), init.cuda(), em.cuda(), er.cuda())
    out_b = batched.run().cpu()
    for w in range(W):
        sl = slice(w * Fr, (w + 1) * Fr)
        ref = R.pipeline_window(unet.state_dict(), dict(unet.config), vae._sd, faces[sl], mask, audio[sl],
                                init[w:w + 1], em[sl], er[sl], num_steps=steps, guidance_scale=2.0)
        e = rel_err(out_b[sl], ref)
        print("batched window vs oracle", w, e)
        assert e < 3e-2
    single = WindowEngine(unet, vae, sched, Fr, Rr, steps, 2.0, windows=1)
    for w in range(W):
        sl = slice(w * Fr, (w + 1) * Fr)
        single.load(faces[sl].cuda(), mask.cuda(), audio[sl].cuda(), init[w:w + 1].cuda(), em[sl].cuda(),
                    er[sl].cuda())
        out_s = single.run().cpu()
        e = rel_err(out_b[sl], out_s)
        print("batched vs single window", w, e)
        assert e < 3e-2


def test_run_windows_batches_match_oracle(gpu, monkeypatch):
    """LipsyncPipeline.run_windows over 3 windows with windows_per_batch = 2 (one
    batch of 2 + one single) against the oracle window by window."""
    from latentsync_amd.pipeline import LipsyncPipeline
    Fr, Rr, steps, n_win = 8, 64, 2, 3
    h = Rr // 8
    unet = UNet3DConditionModel(**TINY_MODEL).init_weights(9).to("cuda").eval()
    vae = AutoencoderKL(block_out_channels=(32, 64, 64, 64)).init_weights(10).to("cuda")
    monkeypatch.setitem(R.VAE_CFG, "block_out_channels", (32, 64, 64, 64))
    pipe = LipsyncPipeline(vae, None, unet, DDIMScheduler(**SCHED))
    pipe.windows_per_batch = 2
    g = torch.Generator().manual_seed(11)
    N = n_win * Fr
    faces = (torch.rand((N, 3, Rr, Rr), generator=g) * 255).to(torch.uint8)
    mask = load_fixed_mask(Rr)
    audio = torch.randn((N, 50, 384), generator=g)
    init = torch.randn((1, 4, 1, h, h), generator=g).repeat(1, 1, N, 1, 1)
    noise = [(torch.randn((Fr, 4, h, h), generator=g), torch.randn((Fr, 4, h, h), generator=g)) for _ in range(n_win)]
    out, out_u8 = pipe.run_windows(faces, audio.cuda(), mask, Fr, steps, 1.0, all_latents=init.cuda(),
                                   vae_noise=lambda i: (noise[i][0].cuda(), noise[i][1].cuda()))
    assert out.shape == (N, 3, Rr, Rr) and out_u8.shape == (N, Rr, Rr, 3)
    for w in range(n_win):
        sl = slice(w * Fr, (w + 1) * Fr)
        ref = R.pipeline_window(unet.state_dict(), dict(unet.config), vae._sd, faces[sl], mask, audio[sl],
                                init[:, :, sl][:, :, :1], noise[w][0], noise[w][1], num_steps=steps,
                                guidance_scale=1.0)
        e = rel_err(out[sl].cpu(), ref)
        print("run_windows window", w, e)
        assert e < 3e-2


def test_window_configs4_shape(gpu, monkeypatch):
    """configs[4]'s shapes: 512^2 faces, 64^2 latent (spatial attention N = 4096 at the
    top UNet level), the 512^2 mask from the LANCZOS4 resize (fractional edge values
    in both the pixel mask and the nearest-interpolated latent mask)."""
    Fr, Rr, steps = 8, 512, 2
    h = Rr // 8
    unet = UNet3DConditionModel(**TINY_MODEL).init_weights(12).to("cuda").eval()
    vae = AutoencoderKL(block_out_channels=(32, 64, 64, 64)).init_weights(13).to("cuda")
    monkeypatch.setitem(R.VAE_CFG, "block_out_channels", (32, 64, 64, 64))
    g = torch.Generator().manual_seed(14)
    low = torch.rand((Fr, 3, Rr // 32, Rr // 32), generator=g)
    faces = (torch.nn.functional.interpolate(low, size=(Rr, Rr), mode="bilinear") * 255).round().to(torch.uint8)
    mask = load_fixed_mask(Rr)
    assert ((mask > 0) & (mask < 1)).any()
    audio = torch.randn((Fr, 50, 384), generator=g)
    init = torch.randn((1, 4, 1, h, h), generator=g)
    em, er = torch.randn((Fr, 4, h, h), generator=g), torch.randn((Fr, 4, h, h), generator=g)
    eng = WindowEngine(unet, vae, DDIMScheduler(**SCHED), Fr, Rr, steps, 1.0)
    eng.load(faces.cuda(), mask.cuda(), audio.cuda(), init.cuda(), em.cuda(), er.cuda())
    out = eng.run().cpu()
    ref = R.pipeline_window(unet.state_dict(), dict(unet.config), vae._sd, faces, mask, audio, init, em, er,
                            num_steps=steps, guidance_scale=1.0)
    e = rel_err(out, ref)
    print("configs[4]-shape window rel_err", e)
    assert e < 3e-2


def test_engines_dropped_during_capture(gpu):
    """Graph lifetime (round-2 abort, commit ee7a273): engines are built, captured and
    dropped back to back, one of them as unreachable cyclic garbage that the collector
    frees INSIDE the next engine's capture.  Its graphs are only retired there (no HIP
    call mid-capture) and destroyed at the next safe point; nothing depends on the
    collector being off.  The captured engine still matches its eager run."""
    import gc

    from latentsync_amd import pipeline as P
    Fr, Rr, steps = 4, 64, 2
    h = Rr // 8
    unet = UNet3DConditionModel(**TINY_MODEL).init_weights(9).to("cuda").eval()
    vae = AutoencoderKL(block_out_channels=(32, 64, 64, 64)).init_weights(10).to("cuda")
    g = torch.Generator().manual_seed(11)
    inp = [(torch.rand((Fr, 3, Rr, Rr), generator=g) * 255).to(torch.uint8), load_fixed_mask(Rr),
           torch.randn((Fr, 50, 384), generator=g), torch.randn((1, 4, 1, h, h), generator=g),
           torch.randn((Fr, 4, h, h), generator=g), torch.randn((Fr, 4, h, h), generator=g)]
    inp = [t.cuda() for t in inp]
    assert gc.isenabled()
    for it in range(3):
        dead = WindowEngine(unet, vae, DDIMScheduler(**SCHED), Fr, Rr, steps, 1.0)
        dead.load(*inp)
        dead.run()
        dead.cycle = dead  # a cycle: only the collector frees it
        holder = [dead]    # ... and not before the capture below drops this last reference
        del dead
        eng = WindowEngine(unet, vae, DDIMScheduler(**SCHED), Fr, Rr, steps, 1.0)
        real_step = eng._step

        def step_with_gc():
            if torch.cuda.is_current_stream_capturing() and holder:
                holder.clear()
                gc.collect()  # frees the dead engine while the step graph is being captured
            real_step()
        eng._step = step_with_gc
        eng.load(*inp)
        out = eng.run().cpu()
        assert P._RETIRED_GRAPHS, "the collected engine's graphs were not retired"
        eager = WindowEngine(unet, vae, DDIMScheduler(**SCHED), Fr, Rr, steps, 1.0, use_graphs=False)
        eager.load(*inp)
        assert rel_err(out, eager.run().cpu()) < 1e-3
        eng.close()  # outside capture: retired graphs are destroyed now
        assert not P._RETIRED_GRAPHS and eng.graphs is None
        out2 = eng.run().cpu()  # a closed engine captures again
        assert torch.equal(out, out2)
        eng.close()


def test_clip_lengths_share_one_engine(gpu, monkeypatch):
    """Clips of 10 and 11 windows run through ONE captured engine (12 windows: the bucket,
    pipeline.plan_window_batches; padding windows computed and discarded).  The windows the
    two clips have in common come out bit-identical (same engine, same per-window inputs:
    the padding windows never mix into a real one), and window 0 matches the oracle."""
    from latentsync_amd.pipeline import LipsyncPipeline
    Fr, Rr, steps = 4, 64, 2
    h = Rr // 8
    unet = UNet3DConditionModel(**TINY_MODEL).init_weights(19).to("cuda").eval()
    vae = AutoencoderKL(block_out_channels=(32, 64, 64, 64)).init_weights(20).to("cuda")
    monkeypatch.setitem(R.VAE_CFG, "block_out_channels", (32, 64, 64, 64))
    pipe = LipsyncPipeline(vae, None, unet, DDIMScheduler(**SCHED))
    g = torch.Generator().manual_seed(21)
    n_max = 11
    N = n_max * Fr
    faces = (torch.rand((N, 3, Rr, Rr), generator=g) * 255).to(torch.uint8)
    mask = load_fixed_mask(Rr)
    audio = torch.randn((N, 50, 384), generator=g)
    init = torch.randn((1, 4, 1, h, h), generator=g).repeat(1, 1, N, 1, 1)
    noise = [(torch.randn((Fr, 4, h, h), generator=g), torch.randn((Fr, 4, h, h), generator=g)) for _ in range(n_max)]
    outs = {}
    for n_win in (10, 11):
        n = n_win * Fr
        outs[n_win], _ = pipe.run_windows(faces[:n], audio[:n].cuda(), mask, Fr, steps, 1.0,
                                          all_latents=init[:, :, :n].cuda(),
                                          vae_noise=lambda i: (noise[i][0].cuda(), noise[i][1].cuda()))
        assert outs[n_win].shape == (n, 3, Rr, Rr)
    assert list(k[-1] for k in pipe._engines) == [12], list(pipe._engines)
    eng = next(iter(pipe._engines.values()))
    print(f"engine of 12 windows: warm-up + capture {eng.capture_s:.3f} s")
    assert torch.equal(outs[10], outs[11][:10 * Fr])
    ref = R.pipeline_window(unet.state_dict(), dict(unet.config), vae._sd, faces[:Fr], mask, audio[:Fr],
                            init[:, :, :1], noise[0][0], noise[0][1], num_steps=steps, guidance_scale=1.0)
    e = rel_err(outs[11][:Fr].cpu(), ref)
    print("bucketed engine window 0 vs oracle", e)
    assert e < 3e-2
