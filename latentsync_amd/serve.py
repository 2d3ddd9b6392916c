"""HTTP job server -- drop-in for scripts/api.py:21-219.

Same endpoints and wire format as the reference:
  POST /process  RequestPayload {id, video_id, audio_url, start_from_backwards,
                 force_video_length, is_dynamic_clip, text, use_darken,
                 brightness_factor} -> {message, output_url, gif_url, elapsed_time}
                 or {"error": "Queue is full, try again later."} (api.py:198-212)
  GET  /ping     {"message": "pong"} (api.py:214-219)
with the reference's bounded request queue (asyncio.Queue(maxsize=10), api.py:24),
its per-request file layout under the data directory (api.py:103-123), the same
pipeline call (num_frames 16, 20 steps, guidance 1.5, resolution from the config,
api.py:138-154) and its error behaviour (HTTPException 400 for missing inputs, any
other failure re-raised to the waiting request, api.py:192-193).

MI355X-first dispatch: instead of one pipeline behind asyncio.Semaphore(1)
(api.py:27, 95), the server keeps ONE pipeline process per GPU (`ProcessWorker`,
each bound to its device before it touches HIP) and a consumer per worker takes the
next queued request as soon as its GPU is free -- up to N requests in flight on an
N-GPU node, each worker still strictly one request at a time (the pipeline is not
re-entrant).  Out of scope (no network): the GCS upload and the
GIF thumbnail (api.py:156-179) -- `output_url` is the local result path and
`gif_url` is None -- and downloading `audio_url` (a local path or file:// URL is
copied into place).
"""
import asyncio
import multiprocessing as mp
import os
import shutil
import time
import uuid
from typing import Optional

from fastapi import FastAPI, HTTPException
from pydantic import BaseModel

QUEUE_FULL = {"error": "Queue is full, try again later."}


class RequestPayload(BaseModel):
    """api.py:30-39."""
    id: str
    video_id: str
    audio_url: str
    start_from_backwards: Optional[bool] = None
    force_video_length: Optional[bool] = None
    is_dynamic_clip: Optional[bool] = None
    text: Optional[str] = None
    use_darken: Optional[bool] = None
    brightness_factor: Optional[float] = 1


def calculate_inverse_factor(original_factor):
    """darken_restore.py:379-405: the factor that undoes a darkening by `original_factor`
    (restoration strength 1, rounded to 2 decimals)."""
    if original_factor >= 1.0:
        return 1.0
    return round(1.0 + (1.0 - original_factor) / original_factor, 2)


def resolve_paths(p: dict, data_dir: str):
    """api.py:103-123: (video_path, data_path, audio_path) of a request."""
    vid, rid = p["video_id"], p["id"]
    j = lambda name: os.path.join(data_dir, name)
    video_path, data_path, audio_path = j(f"{vid}.mp4"), j(f"{vid}.pth"), j(f"{rid}.wav")
    if p.get("is_dynamic_clip") and os.path.exists(j(f"{vid}_rotated.pth")) and os.path.exists(j(f"{vid}_rotated.mp4")):
        data_path, video_path = j(f"{vid}_rotated.pth"), j(f"{vid}_rotated.mp4")
        if p.get("use_darken"):
            data_path, video_path = j(f"{vid}_darken_rotated.pth"), j(f"{vid}_darken_rotated.mp4")
    elif p.get("use_darken"):
        data_path, video_path = j(f"{vid}_darken.pth"), j(f"{vid}_darken.mp4")
    return video_path, data_path, audio_path


def fetch_audio(url: str, dest: str):
    """download_file (download.py:6-40) for the sources this build can reach: a local
    path or a file:// URL.  Network URLs are out of scope (no egress)."""
    src = url[len("file://"):] if url.startswith("file://") else url
    if "://" in src or not os.path.exists(src):
        raise HTTPException(status_code=400, detail="Audio file not found.")
    shutil.copyfile(src, dest)


def run_job(pipeline, payload: dict, data_dir: str, results_dir: str, resolution: int, weight_dtype=None):
    """The body of process_requests (api.py:96-190) for one request on one pipeline."""
    start = time.time()
    video_path, data_path, audio_path = resolve_paths(payload, data_dir)
    if not os.path.exists(video_path):
        raise HTTPException(status_code=400, detail="Video file not found.")
    if not os.path.exists(data_path):
        raise HTTPException(status_code=400, detail="Data file not found.")
    if not os.path.exists(audio_path):
        fetch_audio(payload["audio_url"], audio_path)
    os.makedirs(results_dir, exist_ok=True)
    video_out_path = os.path.join(results_dir, f"{payload['id']}.npz")  # this build's writer (pipeline.py)
    kw = {} if weight_dtype is None else dict(weight_dtype=weight_dtype)
    pipeline(video_path=video_path, audio_path=audio_path, video_out_path=video_out_path,
             video_mask_path=video_out_path.replace(".npz", "_mask.npz"), num_frames=16, num_inference_steps=20,
             guidance_scale=1.5, width=resolution, height=resolution, data_path=data_path,
             start_from_backwards=payload.get("start_from_backwards") or False,
             force_video_length=payload.get("force_video_length") or False,
             use_darken=payload.get("use_darken") or False,
             brightness_factor=calculate_inverse_factor(payload.get("brightness_factor") or 1), **kw)
    return {"message": "Request processed successfully", "output_url": video_out_path, "gif_url": None,
            "elapsed_time": time.time() - start, "request_uuid": str(uuid.uuid4())}


# --------------------------------------------------------------------------
# workers: one request at a time each
# --------------------------------------------------------------------------


class InlineWorker:
    """A pipeline object driven from a thread of this process (tests; a CPU stand-in)."""

    def __init__(self, pipeline, rank=0, **job_kw):
        self.pipeline, self.rank, self.job_kw = pipeline, rank, job_kw

    def start(self):
        pass

    async def run(self, payload):
        loop = asyncio.get_running_loop()
        return await loop.run_in_executor(None, run_job, self.pipeline, payload, *self._args())

    def _args(self):
        k = self.job_kw
        return k["data_dir"], k["results_dir"], k.get("resolution", 256), k.get("weight_dtype")

    def stop(self):
        pass


def _worker_main(rank, factory, job_kw, conn):
    """Child process of a ProcessWorker: bind the GPU first, build the pipeline
    once, then serve requests from the pipe until None arrives."""
    import importlib

    import torch
    if torch.cuda.device_count() > 0:  # counting devices does not initialise HIP
        torch.cuda.set_device(rank)
    mod, fn = factory.split(":")
    pipeline = getattr(importlib.import_module(mod), fn)(rank)
    conn.send(("ready", None))
    while True:
        payload = conn.recv()
        if payload is None:
            break
        try:
            conn.send(("ok", run_job(pipeline, payload, job_kw["data_dir"], job_kw["results_dir"],
                                     job_kw.get("resolution", 256))))
        except HTTPException as e:
            conn.send(("http", (e.status_code, e.detail)))
        except Exception as e:  # noqa: BLE001 -- re-raised in the server (api.py:192-193)
            conn.send(("err", f"{type(e).__name__}: {e}"))


class WorkerDied(RuntimeError):
    """The GPU worker process ended (fault, abort, OOM kill) or missed the request
    timeout while serving a request; a fresh process has been launched in its place
    (or the replacement itself failed to start: the message says which)."""


class ProcessWorker:
    """One pipeline process per GPU (spawned, so HIP initialises only in the child).
    `factory` = "module:function" building the pipeline for a device index.

    Robustness (the reference runs the pipeline in-process, api.py:95-190, so a GPU
    fault kills the whole server): a request that does not finish within
    `request_timeout` seconds, or whose worker dies under it, fails with WorkerDied
    and the worker is replaced by a freshly SPAWNED child (never a re-exec of a
    process that touched the GPU), so the next request routed here is served.  The
    failed request is answered at once and the replacement loads in the background:
    the Dispatcher waits for its 'ready' (`ensure_ready`) BEFORE this worker takes
    another request from the queue, so meanwhile the other GPUs' workers serve the
    queue.  A replacement that fails to start fails the next request this worker takes
    with WorkerDied ("did not start"), and another replacement is launched."""

    def __init__(self, rank, factory, request_timeout=1800.0, start_timeout=900.0, **job_kw):
        self.rank, self.factory, self.job_kw = rank, factory, job_kw
        self.request_timeout, self.start_timeout = request_timeout, start_timeout
        self.proc = self.conn = None
        self.restarts = 0
        self._unready = False  # a replacement child was launched and has not reported 'ready'

    def launch(self):
        """Spawn the child; `wait_ready` collects its 'ready' (so N GPUs load together)."""
        ctx = mp.get_context("spawn")
        self.conn, child = ctx.Pipe()
        self.proc = ctx.Process(target=_worker_main, args=(self.rank, self.factory, self.job_kw, child), daemon=True)
        self.proc.start()
        child.close()  # the parent keeps one end only: EOF is seen when the child dies

    def wait_ready(self):
        try:
            if not self.conn.poll(self.start_timeout):
                self._kill()
                raise RuntimeError(f"GPU worker {self.rank} failed to start within {self.start_timeout} s")
            kind, _ = self.conn.recv()
        except (EOFError, OSError):
            self.proc.join(timeout=5)
            raise RuntimeError(f"GPU worker {self.rank} failed to start (exit code {self.proc.exitcode})") from None
        if kind != "ready":
            raise RuntimeError(f"GPU worker {self.rank} failed to start")

    def start(self):
        self.launch()
        self.wait_ready()

    def _kill(self):
        if self.proc is not None and self.proc.is_alive():
            self.proc.kill()
        if self.proc is not None:
            self.proc.join(timeout=10)
        if self.conn is not None:
            self.conn.close()

    def _replace(self):
        """Kill the child and launch its replacement without waiting for it to load."""
        self._kill()
        self.restarts += 1
        self.launch()
        self._unready = True

    def ensure_ready(self):
        """Block until a replacement child launched after a failure reports 'ready'.
        Returns None when the worker can take a request, else the start failure (a new
        replacement has then been launched)."""
        if not self._unready:
            return None
        try:
            self.wait_ready()
            self._unready = False
            return None
        except RuntimeError as e:
            self._replace()
            return str(e)

    def start_failed(self, payload, err):
        return "dead", (f"GPU worker {self.rank}: the replacement child did not start ({err}); "
                        f"request {payload.get('id')!r} not served, another replacement launched")

    def _call(self, payload):
        err = self.ensure_ready()  # direct callers; the Dispatcher waits before dequeuing
        if err is not None:
            return self.start_failed(payload, err)
        try:
            self.conn.send(payload)
            if not self.conn.poll(self.request_timeout):
                why = f"timed out after {self.request_timeout} s"
            else:
                return self.conn.recv()
        except (EOFError, OSError):  # BrokenPipeError is an OSError
            self.proc.join(timeout=5)
            why = f"died (exit code {self.proc.exitcode})"
        self._replace()
        return "dead", f"GPU worker {self.rank} {why} while serving request {payload.get('id')!r}; replacement launched"

    async def run(self, payload):
        loop = asyncio.get_running_loop()
        kind, val = await loop.run_in_executor(None, self._call, payload)
        if kind == "ok":
            return val
        if kind == "http":
            raise HTTPException(status_code=val[0], detail=val[1])
        if kind == "dead":
            raise WorkerDied(val)
        raise RuntimeError(val)

    def stop(self):
        if self.proc is not None and self.proc.is_alive():
            try:
                self.conn.send(None)
            except OSError:
                pass
            self.proc.join(timeout=30)
            if self.proc.is_alive():
                self.proc.terminate()
                self.proc.join(timeout=10)


# --------------------------------------------------------------------------
# the app
# --------------------------------------------------------------------------


class Dispatcher:
    """The bounded request queue (api.py:24) and one consumer per worker."""

    def __init__(self, workers, queue_size=10):
        self.workers, self.queue_size = list(workers), queue_size
        self.queue = None
        self.tasks = []
        self.served = {w.rank: 0 for w in self.workers}

    async def start(self):
        self.queue = asyncio.Queue(maxsize=self.queue_size)
        # every GPU's pipeline loads at once: spawn all children, then wait for their
        # 'ready' messages together, off the event loop
        for w in self.workers:
            (w.launch if hasattr(w, "launch") else w.start)()
        loop = asyncio.get_running_loop()
        await asyncio.gather(*[loop.run_in_executor(None, w.wait_ready) for w in self.workers
                               if hasattr(w, "wait_ready")])
        for w in self.workers:
            self.tasks.append(asyncio.create_task(self._consume(w)))

    async def _consume(self, worker):
        loop = asyncio.get_running_loop()
        while True:
            start_err = None
            if hasattr(worker, "ensure_ready"):
                # a replacement child loads (up to start_timeout) BEFORE this consumer takes
                # a request, so the queue drains to the ready workers meanwhile
                start_err = await loop.run_in_executor(None, worker.ensure_ready)
            payload, fut = await self.queue.get()
            try:
                if start_err is not None:
                    raise WorkerDied(worker.start_failed(payload, start_err)[1])
                res = await worker.run(payload)
                self.served[worker.rank] += 1
                if not fut.done():
                    fut.set_result(res)
            except Exception as e:  # noqa: BLE001 -- to the waiting request (api.py:192-193)
                if not fut.done():
                    fut.set_exception(e)
            finally:
                self.queue.task_done()

    async def submit(self, payload: dict):
        """None when the queue is full (the reference's check, api.py:203-204)."""
        if self.queue.full():
            return None
        fut = asyncio.get_running_loop().create_future()
        await self.queue.put((payload, fut))
        return await fut

    async def stop(self):
        for t in self.tasks:
            t.cancel()
        for w in self.workers:
            w.stop()


def create_app(workers, queue_size=10):
    """The FastAPI app; the workers start with it (startup_event, api.py:42-85) and
    stop with it."""
    from contextlib import asynccontextmanager
    disp = Dispatcher(workers, queue_size)

    @asynccontextmanager
    async def lifespan(app):
        await disp.start()
        try:
            yield
        finally:
            await disp.stop()

    app = FastAPI(lifespan=lifespan)
    app.state.dispatcher = disp

    @app.post("/process")
    async def process(payload: RequestPayload):
        res = await disp.submit(payload.model_dump())
        return QUEUE_FULL if res is None else res

    @app.get("/ping")
    async def ping():
        return {"message": "pong"}

    return app


def default_pipeline(rank):
    """The production pipeline for one GPU, as startup_event builds it (api.py:42-85):
    configs/unet/stage2.yaml, checkpoints/latentsync_unet.pt, Whisper tiny, the SD VAE
    from a local directory (LATENTSYNC_VAE_DIR) and configs/scheduler_config.json."""
    import torch

    from .audio import Audio2Feature
    from .config import load_config
    from .pipeline import LipsyncPipeline
    from .scheduler import DDIMScheduler
    from .unet import UNet3DConditionModel
    from .vae import AutoencoderKL
    cfg = load_config(os.environ.get("LATENTSYNC_UNET_CONFIG", "configs/unet/stage2.yaml"))
    dev = torch.device("cuda", rank)
    unet, _ = UNet3DConditionModel.from_pretrained(cfg["model"], os.environ.get(
        "LATENTSYNC_UNET_CKPT", "checkpoints/latentsync_unet.pt"), device=dev)
    vae = AutoencoderKL.from_pretrained(os.environ.get("LATENTSYNC_VAE_DIR", "checkpoints/sd-vae-ft-mse"))
    vae.config.scaling_factor, vae.config.shift_factor = 0.18215, 0
    audio = Audio2Feature(model_path=os.environ.get("LATENTSYNC_WHISPER", "checkpoints/whisper/tiny.pt"), device=dev,
                          num_frames=cfg["data"]["num_frames"])
    sched = DDIMScheduler.from_pretrained("configs")
    return LipsyncPipeline(vae=vae, audio_encoder=audio, denoising_unet=unet, scheduler=sched).to(dev)


def main():
    import argparse

    import uvicorn
    ap = argparse.ArgumentParser(description="LatentSync job server, one pipeline process per GPU")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--data-dir", default="/latent-sync-data")
    ap.add_argument("--results-dir", default="results")
    ap.add_argument("--resolution", type=int, default=256)
    ap.add_argument("--factory", default="latentsync_amd.serve:default_pipeline")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--request-timeout", type=float, default=1800.0,
                    help="seconds before a request's GPU worker is declared hung and replaced")
    a = ap.parse_args()
    kw = dict(data_dir=a.data_dir, results_dir=a.results_dir, resolution=a.resolution)
    app = create_app([ProcessWorker(r, a.factory, request_timeout=a.request_timeout, **kw) for r in range(a.gpus)])
    uvicorn.run(app, host=a.host, port=a.port)


if __name__ == "__main__":
    main()
