"""LipsyncPipeline -- drop-in for latentsync/pipelines/lipsync_pipeline.py:46-604
on the MI355X HIP path.

The per-window hot loop (lipsync_pipeline.py:500-575) runs in ``WindowEngine``:
every tensor of a window is device-resident in static buffers, and the window is
three captured hipGraphs replayed back to back --

  encode : pixel prep (ImageProcessor.preprocess_fixed_mask_image) -> VAE encode
           of masked + reference faces -> posterior sample * 0.18215 -> pack the
           13-channel UNet input (prepare_mask_latents / prepare_image_latents,
           :284-320, :547-549), reset the device step counter
  step   : UNet3DConditionModel forward + CFG combine + DDIMScheduler.step +
           re-pack of the next input (:540-562); the timestep and DDIM
           coefficients are read on device at the step counter, so the SAME graph
           replays num_inference_steps times
  decode : latents / 0.18215 -> VAE decode -> paste_surrounding_pixels_back
           (+ uint8 images for the all-gather / writer) (:145-149, :327-341, :571-574)

Random draws are injected (initial latent noise, VAE posterior noise), as the
parity harness requires (SURVEY.md §7 "RNG").
"""
import collections
import math
import time
import os

import numpy as np
import torch

from . import ops, shard

SCALING = 0.18215


def load_fixed_mask(resolution=256, mask_image_path=None, device=None):
    """load_fixed_mask (image_processor.py:31-36) -> keep-mask (R, R) float32,
    1 = keep the original pixel, 0 = mouth region to regenerate.  The uint8 mask
    image (the reference's mask.png, 256^2, shipped as packed bits) is resized
    with cv2's INTER_LANCZOS4 arithmetic on the device (ls_resize_lanczos4_u8) when
    the resolution differs -- fractional edge values k/255, as the reference gets --
    then divided by 255.  All channels of the gray mask are equal, so one is resized
    (the reference keeps channel 0 for the UNet mask, :152)."""
    if mask_image_path is None or not os.path.exists(mask_image_path):
        bits = np.load(os.path.join(os.path.dirname(__file__), "assets", "fix_mask_256.npz"))["bits"]
        m8 = (np.unpackbits(bits)[: 256 * 256].reshape(256, 256) * 255).astype(np.uint8)
    else:
        from PIL import Image
        m8 = np.array(Image.open(mask_image_path).convert("RGB"))[..., 0].copy()
    t = torch.from_numpy(m8)
    if tuple(t.shape) != (resolution, resolution):
        from .align import resize_lanczos4
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        t = resize_lanczos4(t.to(dev), resolution, resolution)
    t = (t.to(torch.float64) / 255.0).to(torch.float32)
    return t.to(device) if device is not None else t.cpu()


def load_data_pth(data_path):
    """The precomputed ingest file (affine_transform_video.py:30-35 writes it;
    lipsync_pipeline.py:398-402 reads it): {faces uint8 (N,3,R,R), boxes, affine_matrices}.
    The matrices are cv2's float64 numpy arrays, so the weights-only unpickler is
    widened by exactly numpy's array reconstruction (ndarray, dtype, _reconstruct and
    the concrete dtype classes) -- still nothing from the file is executed."""
    allow = [np.ndarray, np.dtype, np._core.multiarray._reconstruct]
    allow += [type(np.dtype(t)) for t in ("f8", "f4", "i8", "i4", "u1")]
    with torch.serialization.safe_globals(allow):
        data = torch.load(data_path, map_location="cpu", weights_only=True)
    data["affine_matrices"] = [np.asarray(m, np.float64).reshape(2, 3) for m in data["affine_matrices"]]
    return data


def read_video_frames(video_path):
    """Original video frames for restore_video: read_video (util.py:46-100) decodes
    with ffmpeg/cv2, which this build does not carry, so the frames come already
    decoded -- a uint8 (N,H,W,3) .npy, or an .npz holding ``frames``.  Any other
    path returns None (no warp-back; the aligned faces are written)."""
    if not video_path or not os.path.exists(video_path):
        return None
    if video_path.endswith(".npy"):
        fr = np.load(video_path, allow_pickle=False)
    elif video_path.endswith(".npz"):
        with np.load(video_path, allow_pickle=False) as z:
            fr = z["frames"]
    else:
        return None
    if fr.dtype != np.uint8 or fr.ndim != 4 or fr.shape[-1] != 3:
        raise ValueError(f"{video_path}: expected uint8 frames (N,H,W,3), got {fr.dtype} {fr.shape}")
    return fr


U8_CHUNK = 256  # frames per conversion chunk of frames_to_u8 (bounds its fp32 temporaries)


def frames_to_u8(frames, out=None):
    """(n,3,R,R) fp32 pasted frames in [-1,1] -> (n,R,R,3) uint8 with exactly the
    paste-back kernel's rounding (clamp(x/2+0.5, 0, 1)*255, truncated; fp32 throughout,
    x/2 is exact so no contraction can change it) -- the u8 of the gathered clip is
    derived from the one fp32 all-gather instead of being gathered a second time.
    Converted in chunks of U8_CHUNK frames, so the temporaries stay 2 x U8_CHUNK fp32
    frames whatever n is (a whole job's gathered frames reach ~100 GB per rank at
    8 ranks, bench.py)."""
    n, _, R, W = frames.shape
    if out is None:
        out = torch.empty((n, R, W, 3), dtype=torch.uint8, device=frames.device)
    for i in range(0, n, U8_CHUNK):
        u = ((frames[i:i + U8_CHUNK] / 2 + 0.5).clamp_(0, 1) * 255).to(torch.uint8)
        out[i:i + U8_CHUNK].copy_(u.permute(0, 2, 3, 1))
    return out


# Graph lifetime.  A hipGraph must not be destroyed while a stream is capturing (the
# runtime aborts), and an engine that becomes cyclic garbage can be collected at any
# allocation -- including inside another engine's capture.  So an engine never
# destroys its graphs itself: close() and __del__ only move them here (a list append,
# no HIP call), and they are destroyed at the next safe point: the start of a capture
# (before it begins), or release_retired_graphs() outside any capture.
_RETIRED_GRAPHS = []


def release_retired_graphs():
    """Destroy the graphs of closed / collected engines, if no stream is capturing."""
    if _RETIRED_GRAPHS and not torch.cuda.is_current_stream_capturing():
        while _RETIRED_GRAPHS:
            _RETIRED_GRAPHS.pop().reset()


class WindowEngine:
    """Device-resident executor of one 16-frame window; see module docstring."""

    def __init__(self, unet, vae, scheduler, num_frames=16, resolution=256, num_inference_steps=20,
                 guidance_scale=1.0, use_graphs=True, audio_tokens=50, windows=1):
        self.unet, self.vae, self.scheduler = unet, vae, scheduler
        self.ud = unet._require_device()
        self.vd = vae._require()
        dev = unet.device
        self.device = dev
        self.F, self.R, self.h = num_frames, resolution, resolution // 8
        self.steps, self.g = num_inference_steps, float(guidance_scale)
        self.Bu = 2 if guidance_scale > 1.0 else 1
        self.L = audio_tokens
        # `windows` independent windows are batched through one UNet call (UNet batch
        # = Bu * windows samples, ordered [uncond w0..wN-1, cond w0..wN-1]); every
        # per-sample op (5-D GroupNorm, temporal attention) stays per window.
        self.nw = windows
        self.FT = self.F * windows  # frames in flight
        self.P = self.FT * self.h * self.h
        scheduler.set_timesteps(num_inference_steps)
        self.ts = scheduler.timesteps.to(torch.int32).to(dev)
        self.coef = scheduler.coef_table(dev)
        F_, R, h, Bu, P = self.FT, self.R, self.h, self.Bu, self.P
        cd = unet.config.cross_attention_dim
        z = lambda *s, dt=torch.bfloat16: torch.zeros(s, dtype=dt, device=dev)
        self.faces = z(F_, 3, R, R, dt=torch.uint8)
        self.mask = z(R, R, dt=torch.float32)
        self.audio = z(Bu * F_ * audio_tokens, cd)
        self.init_lat = z(P, 4, dt=torch.float32)
        self.eps_m = z(P, 4, dt=torch.float32)
        self.eps_r = z(P, 4, dt=torch.float32)
        self.lat = z(P, 4, dt=torch.float32)
        self.cond = z(P, 16)
        self.unet_in = z(Bu * F_, h, h, self.ud.cin_pad)
        self.step = z(1, dt=torch.int32)
        self.pix = z(F_, R, R, 8)
        self.masked = z(F_, R, R, 8)
        self.zdec = z(F_, h, h, 8)
        self.out = z(F_, 3, R, R, dt=torch.float32)
        self.out_u8 = z(F_, R, R, 3, dt=torch.uint8)
        self.use_graphs = use_graphs
        self.graphs = None
        self.capture_s = None

    # -- the three phases --------------------------------------------------------
    def _encode(self):
        ops.prep_pixels(self.faces, self.mask, 8, self.pix, self.masked)
        mom = self.vd.encode_moments(self.masked)
        ops.vae_sample(mom, self.eps_m, SCALING, 0.0, self.cond, 5)
        mom = self.vd.encode_moments(self.pix)
        ops.vae_sample(mom, self.eps_r, SCALING, 0.0, self.cond, 9)
        self.lat.copy_(self.init_lat)
        ops.pack_unet_input(self.lat, self.cond, self.mask, self.FT, self.R, self.h, self.Bu, self.unet_in)
        self.step.zero_()
        # audio cross-attention k|v of every Transformer3DModel: constant over the 20 steps
        self.audio_kv = self.ud.audio_kv(self.audio)

    def _step(self):
        eps = self.ud.forward(self.unet_in, self.Bu * self.nw, self.ts, self.step, self.audio, self.L,
                              audio_kv=self.audio_kv)
        ops.ddim_cfg_step(eps, self.Bu, self.g, self.lat, self.coef, self.step, self.unet_in)

    def _decode(self):
        ops.scale_latents(self.lat, 1.0 / SCALING, 0.0, self.zdec)
        dec = self.vd.decode(self.zdec)
        ops.paste_back(dec, self.pix, self.mask, self.out, self.out_u8)

    def capture(self):
        """Warm up eagerly once, then capture the three phases as hipGraphs.  Graphs
        of engines closed or collected earlier are destroyed first, outside the
        capture; an engine collected DURING the capture only retires its graphs.
        The wall time of warm-up + capture is kept in ``capture_s``."""
        t0 = time.perf_counter()
        self._encode()
        self._step()
        self._decode()
        torch.cuda.synchronize(self.device)
        self._retire()
        release_retired_graphs()
        pool = torch.cuda.graph_pool_handle()
        graphs = []
        try:
            for fn in (self._encode, self._step, self._decode):
                g = torch.cuda.CUDAGraph()
                graphs.append(g)
                with torch.cuda.graph(g, pool=pool):
                    fn()
        except BaseException:
            _RETIRED_GRAPHS.extend(graphs)
            raise
        torch.cuda.synchronize(self.device)
        self.graphs = graphs
        self.capture_s = time.perf_counter() - t0

    def _retire(self):
        g = self.__dict__.get("graphs")
        if g:
            _RETIRED_GRAPHS.extend(g)
        self.graphs = None

    def close(self):
        """Release the captured graphs now (deferred if a stream is capturing).  The
        engine stays usable: the next run() captures again."""
        self._retire()
        release_retired_graphs()

    def __del__(self):
        # may run inside another engine's capture (cyclic GC): no HIP call here
        self._retire()

    # -- inputs / execution -------------------------------------------------------
    def load(self, faces_u8, mask, audio_chunks, init_latent, eps_masked, eps_ref):
        """Stage the inputs of `windows` consecutive windows into the static buffers.
        faces (W*F,3,R,R) uint8; mask (R,R) keep-mask; audio (W*F,50,384);
        init_latent (W or 1, 4, 1 or F, h, w) (one draw per window, repeated over its
        frames as prepare_latents does); eps_* (W*F,4,h,w)."""
        F_, h = self.FT, self.h
        self.faces.copy_(faces_u8)
        self.mask.copy_(mask)
        a = audio_chunks.reshape(F_ * self.L, -1).to(torch.bfloat16)
        if self.Bu == 2:  # torch.cat([zeros, audio]) (lipsync_pipeline.py:505-507)
            self.audio[: F_ * self.L].zero_()
            self.audio[F_ * self.L:].copy_(a)
        else:
            self.audio.copy_(a)
        il = init_latent.float()
        if il.shape[0] == 1 and self.nw > 1:
            il = il.expand(self.nw, *il.shape[1:])
        il = il.expand(self.nw, 4, self.F, h, h)  # (W, 4, F, h, w)
        self.init_lat.copy_(il.permute(0, 2, 3, 4, 1).reshape(-1, 4))
        self.eps_m.copy_(eps_masked.float().permute(0, 2, 3, 1).reshape(-1, 4))
        self.eps_r.copy_(eps_ref.float().permute(0, 2, 3, 1).reshape(-1, 4))

    def latents(self):
        """The DDIM state as the reference holds it: (windows, 4, F, h, w) fp32 view."""
        h = self.h
        return self.lat.view(self.nw, self.F, h, h, 4).permute(0, 4, 1, 2, 3)

    def run(self, callback=None, callback_steps=1):
        """Execute the staged window; results in self.out (F,3,R,R) fp32 and
        self.out_u8 (F,R,R,3).  ``callback(j, t, latents)`` is called after DDIM
        step j when j % callback_steps == 0, as lipsync_pipeline.py:564-568 does
        (scheduler.order == 1, so no warm-up steps); the step graph is then
        replayed one step at a time with the host call in between."""
        if self.use_graphs and self.graphs is None:
            self.capture()
        enc, step, dec = ((g.replay for g in self.graphs) if self.use_graphs
                          else (self._encode, self._step, self._decode))
        enc()
        for j in range(self.steps):
            step()
            if callback is not None and j % callback_steps == 0:
                # a copy, as the reference's step returns a fresh tensor (:562-568): the
                # next replay overwrites the engine's state buffer in place
                callback(j, self.scheduler.timesteps[j], self.latents().clone())
        dec()
        return self.out


# --------------------------------------------------------------------------
# pipeline (reference API)
# --------------------------------------------------------------------------


# Engine sizes (windows per UNet call) a clip's full windows are rounded up to, so clips of
# different lengths share captured engines (a new size costs a warm-up run + three graph
# captures, WindowEngine.capture_s ~0.5 s); padding windows run and are discarded.  Steps of
# 4 windows above 8, and a bucket is used only while its padding stays within MAX_PAD of
# the clip's windows -- otherwise the engine is sized exactly (a 9-window clip runs 9, not
# 12 or 16; 49 windows run as 2 x 28 = 56, +14 %, not 2 x 32).
WINDOW_BUCKETS = (1, 2, 4, 6, 8, 12, 16, 20, 24, 28, 32, 36, 40, 44, 48)
MAX_PAD = 0.2


def plan_window_batches(full, windows_per_batch):
    """Split the full windows `full` (indices) into batches for one engine size E:
    k = ceil(len / windows_per_batch) batches of per = ceil(len / k) windows; E = the
    smallest bucket (WINDOW_BUCKETS below `windows_per_batch`, plus `windows_per_batch`
    itself) >= per, or E = per when that bucket would pad more than MAX_PAD of the
    windows; batches of E consecutive windows, the last one short (the caller pads it).
    Returns (E, batches); (0, []) for no full window."""
    if not full:
        return 0, []
    n = len(full)
    cap = max(1, int(windows_per_batch))
    k = math.ceil(n / cap)
    per = math.ceil(n / k)
    E = min(b for b in sorted({b for b in WINDOW_BUCKETS if b < cap} | {cap}) if b >= per)
    if E * math.ceil(n / E) - n > MAX_PAD * n:
        E = per
    return E, [list(full[b:b + E]) for b in range(0, n, E)]


class LipsyncPipeline:
    """Drop-in for LipsyncPipeline(vae, audio_encoder, denoising_unet, scheduler)."""

    def __init__(self, vae, audio_encoder, denoising_unet, scheduler):
        if hasattr(scheduler.config, "steps_offset") and scheduler.config.steps_offset != 1:
            scheduler.config["steps_offset"] = 1  # :65-77
        if hasattr(scheduler.config, "clip_sample") and scheduler.config.clip_sample is True:
            scheduler.config["clip_sample"] = False  # :79-90
        self.vae, self.audio_encoder, self.denoising_unet, self.scheduler = vae, audio_encoder, denoising_unet, scheduler
        self.vae_scale_factor = 2 ** (len(self.vae.config.block_out_channels) - 1)
        self._engines = collections.OrderedDict()
        # Independent windows batched per UNet call (identical per-window math; see
        # tests/test_gpu_pipeline.py::test_windows_batched_equal_separate).  A clip's
        # full windows on this rank run through ONE engine whose size is the batch size
        # rounded up to a bucket (plan_window_batches: at most 48, the benchmarked
        # operating point of bench.py), short batches padded, so clips of different
        # lengths share captured engines; engines are kept in a small LRU cache.
        self.windows_per_batch = 48
        self.max_engines = 3

    @property
    def device(self):
        return self.denoising_unet.device

    def to(self, device):
        self.vae.to(device)
        self.denoising_unet.to(device)
        if self.audio_encoder is not None and hasattr(self.audio_encoder, "to"):
            self.audio_encoder.to(device)
        return self

    def check_inputs(self, height, width, callback_steps):
        assert height == width, "Height and width must be equal"
        if height % 8 != 0 or width % 8 != 0:
            raise ValueError(f"`height` and `width` have to be divisible by 8 but are {height} and {width}.")
        if callback_steps is None or not isinstance(callback_steps, int) or callback_steps <= 0:
            raise ValueError(f"`callback_steps` has to be a positive integer but is {callback_steps} of type"
                             f" {type(callback_steps)}.")

    def engine(self, num_frames, resolution, steps, guidance_scale, use_graphs=True, windows=1):
        key = (num_frames, resolution, steps, float(guidance_scale), use_graphs, windows)
        eng = self._engines.get(key)
        if eng is not None and (eng.unet is not self.denoising_unet or eng.ud is not self.denoising_unet._dev or
                                eng.vae is not self.vae or eng.scheduler is not self.scheduler):
            eng.close()  # the models were swapped or re-packed: this engine is stale
            eng = None
        if eng is None:
            self._engines.pop(key, None)
            while len(self._engines) >= max(1, int(self.max_engines)):
                self._engines.popitem(last=False)[1].close()  # least recently used
            eng = self._engines[key] = WindowEngine(self.denoising_unet, self.vae, self.scheduler, num_frames,
                                                    resolution, steps, guidance_scale, use_graphs, windows=windows)
        self._engines.move_to_end(key)
        return eng

    def close(self):
        """Release every cached window engine and its graphs deterministically."""
        for eng in self._engines.values():
            eng.close()
        self._engines.clear()

    def prepare_latents(self, num_frames, height, width, generator=None):
        """:182-196 -- one (1,4,1,h,w) draw repeated over every frame."""
        shape = (1, self.vae.config.latent_channels, 1, height // self.vae_scale_factor,
                 width // self.vae_scale_factor)
        lat = torch.randn(shape, generator=generator, device=self.device, dtype=torch.float32)
        return lat.repeat(1, 1, num_frames, 1, 1) * self.scheduler.init_noise_sigma

    def run_windows(self, faces_u8, whisper_chunks, mask, num_frames=16, num_inference_steps=20, guidance_scale=1.5,
                    generator=None, all_latents=None, vae_noise=None, callback=None, callback_steps=1):
        """The hot loop (:489-575) over ceil(len(chunks)/num_frames) windows.
        faces_u8 (N,3,R,R) (N >= #chunks, already repeated/truncated as the
        reference does), whisper_chunks (n,50,384).  Window i covers frames
        [i*num_frames, (i+1)*num_frames) of the n chunks; the last one is short
        when n % num_frames != 0 (force_video_length, :455, :500-511) and runs
        with its own frame count, as the reference's slices do.  Returns decoded +
        pasted frames (n, 3, R, R) fp32 and uint8 (n, R, R, 3) on device."""
        R = faces_u8.shape[-1]
        self.check_inputs(R, R, callback_steps)
        n = whisper_chunks.shape[0]
        if faces_u8.shape[0] < n:
            raise ValueError(f"{faces_u8.shape[0]} faces for {n} audio chunks: repeat the faces first (:448-452)")
        if all_latents is None:
            all_latents = self.prepare_latents(n, R, R, generator)
        h = R // self.vae_scale_factor
        mask = mask.to(self.device, torch.float32)
        n_inf = math.ceil(n / num_frames)
        size = [min(num_frames, n - i * num_frames) for i in range(n_inf)]
        # With torch.distributed initialised, rank r runs a contiguous block of windows
        # and the decoded frames are all-gathered once at the end (shard.py).  Every rank
        # still draws every window's VAE noise so the result is independent of W.
        world, rank = shard.world_and_rank()
        mine = shard.rank_windows(n_inf, world, rank)
        noise = {}
        for i in range(n_inf):
            if vae_noise is not None:
                noise[i] = vae_noise(i)
            else:
                noise[i] = (torch.randn((size[i], 4, h, h), generator=generator, device=self.device),
                            torch.randn((size[i], 4, h, h), generator=generator, device=self.device))
        # `windows_per_batch` full windows go through one UNet call per step; a short
        # last window runs alone (eagerly: it happens once per clip).  A per-step
        # callback sees one window's latents at a time, as in the reference.
        full = [i for i in mine if size[i] == num_frames]
        E, batches = plan_window_batches(full, 1 if callback is not None else self.windows_per_batch)
        batches = [(E, b) for b in batches] + [(1, [i]) for i in mine if size[i] < num_frames]
        res = {}
        for E, wins in batches:
            Fw = size[wins[0]]
            eng = self.engine(Fw, R, num_inference_steps, guidance_scale, use_graphs=Fw == num_frames, windows=E)
            run = wins + [wins[-1]] * (E - len(wins))  # padding windows: computed, discarded
            sls = [slice(i * num_frames, i * num_frames + Fw) for i in run]
            cat = lambda xs: torch.cat([x.to(self.device) for x in xs])
            eng.load(cat([faces_u8[sl] for sl in sls]), mask, cat([whisper_chunks[sl] for sl in sls]),
                     cat([all_latents[:, :, sl] for sl in sls]),
                     cat([noise[i][0] for i in run]), cat([noise[i][1] for i in run]))
            eng.run(callback=callback, callback_steps=callback_steps)
            for k, i in enumerate(wins):
                fs = slice(k * Fw, (k + 1) * Fw)
                res[i] = (eng.out[fs].clone(), eng.out_u8[fs].clone())
        if world == 1:
            return torch.cat([res[i][0] for i in mine]), torch.cat([res[i][1] for i in mine])
        # ONE all-gather of equally sized fp32 slabs (restore_video needs the fp32 faces:
        # the reference resizes before it rounds to uint8, :343-358); a short window is
        # zero-padded to num_frames for the exchange and the padding dropped after it.
        # The uint8 frames are derived from the gathered fp32 ones, bit-identical to the
        # engine's own (frames_to_u8).
        F_, dev = num_frames, self.device

        def padded(t):
            if t.shape[0] == F_:
                return t
            return torch.cat([t, t.new_zeros((F_ - t.shape[0],) + tuple(t.shape[1:]))])
        loc = torch.stack([padded(res[i][0]) for i in mine]) if mine else torch.empty((0, F_, 3, R, R), device=dev)
        out = shard.gather_windows(loc, n_inf).flatten(0, 1)[:n]
        return out, frames_to_u8(out)

    def restore_video(self, faces, video_frames, boxes, affine_matrices):
        """:343-358 on the device (latentsync_amd/restore.py): every face of the clip
        resized in one launch, then warped and blended into its frame.  Returns the
        restored frames (N,H,W,3) uint8 on the device (the reference returns numpy)."""
        from . import restore
        if getattr(self, "_restorer", None) is None:
            self._restorer = restore.AlignRestore(self.device)
        return restore.restore_video(faces, video_frames, boxes, affine_matrices, self._restorer)

    @torch.no_grad()
    def __call__(self, video_path, audio_path, video_out_path, video_mask_path=None, num_frames=16, video_fps=25,
                 audio_sample_rate=16000, height=None, width=None, num_inference_steps=20, guidance_scale=1.5,
                 weight_dtype=torch.float16, eta=0.0, mask="fix_mask", mask_image_path="latentsync/utils/mask.png",
                 generator=None, callback=None, callback_steps=1, data_path=None, start_from_backwards=False,
                 force_video_length=False, use_darken=False, brightness_factor=1.0, **kwargs):
        """:360-604.  Face detection / alignment and the ffmpeg decode, encode and
        mux are outside this build's scope: the precomputed
        ``data_path`` (.pth {faces, boxes, affine_matrices}, :398-402) is the face
        source and ``video_path`` holds the original frames already decoded, as a
        uint8 (N,H,W,3) ``.npy`` or an ``.npz`` with a ``frames`` array
        (read_video's output, util.py:46-100).  The synced faces are pasted back into
        those frames on the GPU (restore_video, :577) and the result is written as an
        .npz of the restored frames (uint8) plus the aligned audio.  With
        ``faces_only=True`` (or a video_path that is not an array file) the
        lip-synced aligned faces are written instead and no warp-back happens."""
        from . import repeat as rep
        # write_video's brightness restore runs only `if use_darken and brightness_factor`
        # (util.py:150-151, reached from :594); it needs the video writer and a face-mesh
        # model this build does not carry, so exactly that case is refused.  Otherwise the
        # factor is ignored, as the reference ignores it.
        if use_darken and brightness_factor:
            raise NotImplementedError("use_darken with a brightness_factor: the video writer's face brightness "
                                      "restore (darken_restore.enhance_face_brightness) is out of scope "
                                      "(SURVEY.md §8(f)3)")
        # the reference casts to weight_dtype (fp16 on CUDA, scripts/inference.py:33-34); this
        # path computes in bf16 storage / fp32 accumulation for either half type
        if weight_dtype not in (torch.float16, torch.bfloat16):
            raise NotImplementedError(f"weight_dtype {weight_dtype}: the MI355X path computes in bf16 "
                                      "(torch.float16 or torch.bfloat16 accepted)")
        if eta != 0.0:
            raise NotImplementedError("eta > 0")
        if mask != "fix_mask":
            raise NotImplementedError("only mask='fix_mask' is on the inference path")
        if not data_path:
            raise NotImplementedError("face detection / alignment is out of scope: pass data_path (.pth)")
        data = load_data_pth(data_path)
        faces, boxes, affine_matrices = data["faces"], list(data["boxes"]), list(data["affine_matrices"])
        # the original frames are read up front (:405) because they are repeated /
        # truncated together with the faces, boxes and matrices below; only rank 0
        # restores and writes, so the other ranks never decode or hold them
        rank0 = shard.world_and_rank()[1] == 0
        video_frames = None if (kwargs.get("faces_only") or not rank0) else read_video_frames(video_path)
        R = height or faces.shape[-1]
        self.check_inputs(R, width or R, callback_steps)
        if faces.shape[-1] != R:
            raise NotImplementedError("face resize needs torchvision (out of scope): store faces at the resolution")
        keep = load_fixed_mask(R, mask_image_path)
        from .audio import read_audio
        audio_samples = read_audio(audio_path, audio_sample_rate)
        feat = self.audio_encoder.audio2feat(audio_path)
        chunks = self.audio_encoder.feature2chunks(feature_array=feat, fps=video_fps)
        shape = chunks[0].shape
        padding_duration = 0.0

        def per_frame(fn, n):
            """Apply a repeat/truncate to every per-frame sequence together (:448-452, :462-466)."""
            nonlocal faces, boxes, affine_matrices, video_frames
            faces, boxes, affine_matrices = fn(faces, n), fn(boxes, n), fn(affine_matrices, n)
            if video_frames is not None:
                video_frames = fn(video_frames, n)

        if not force_video_length:
            if start_from_backwards:
                chunks, audio_samples, padding_duration, _ = rep.pad_whisper_chunks(chunks, shape, audio_samples,
                                                                                     audio_sample_rate, video_fps)
            else:
                chunks, audio_samples, padding_duration = rep.pad_whisper_chunks_end(chunks, shape, audio_samples,
                                                                                     audio_sample_rate, video_fps)
            if len(chunks) > len(faces):
                per_frame(rep.repeat_to_length, len(chunks))
        else:
            chunks, audio_samples, padding_duration = rep.pad_whisper_chunks_to_target(
                chunks, shape, audio_samples, audio_sample_rate, len(faces), fps=video_fps)
        if len(faces) != len(chunks) and start_from_backwards:
            per_frame(rep.truncate_to_length, len(chunks))
        chunks = torch.stack([c.to(self.device) for c in chunks])
        out, out_u8 = self.run_windows(faces, chunks, keep, num_frames, num_inference_steps, guidance_scale,
                                       generator, callback=callback, callback_steps=callback_steps)
        if not rank0:
            return None  # rank 0 restores and writes the gathered clip
        frames_out = out_u8
        if video_frames is not None:
            frames_out = self.restore_video(out, video_frames, boxes, affine_matrices)
        n_out = frames_out.shape[0]
        audio_keep = int(n_out / video_fps * audio_sample_rate)
        np.savez(video_out_path if video_out_path.endswith(".npz") else video_out_path + ".npz",
                 frames=frames_out.cpu().numpy(), audio=np.asarray(audio_samples[:audio_keep]),
                 fps=video_fps, sample_rate=audio_sample_rate, padding_duration=padding_duration)
        return None
