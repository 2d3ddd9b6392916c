"""The HTTP job server (latentsync_amd/serve.py; reference scripts/api.py:21-219) on
CPU with FastAPI's TestClient and stand-in pipelines: the endpoints and wire format,
the per-request file layout, the reference's pipeline arguments, error propagation
(400 for missing inputs, other failures to the waiting request), the bounded queue's
"Queue is full" reply, and dispatch over one worker per GPU (each strictly one
request at a time)."""
import asyncio
import os
import threading
import time

import pytest
from fastapi.testclient import TestClient

from latentsync_amd import serve as S


class StubPipeline:
    """Records each call and writes an output file, as the real __call__ does."""

    def __init__(self, delay=0.0, fail=None, gate=None):
        self.calls, self.delay, self.fail, self.gate = [], delay, fail, gate
        self.active = 0
        self.max_active = 0
        self.lock = threading.Lock()

    def __call__(self, **kw):
        with self.lock:
            self.active += 1
            self.max_active = max(self.max_active, self.active)
        try:
            if self.gate is not None:
                self.gate.wait(30)
            time.sleep(self.delay)
            self.calls.append(kw)
            if self.fail:
                raise RuntimeError(self.fail)
            open(kw["video_out_path"], "wb").close()
        finally:
            with self.lock:
                self.active -= 1


def _files(d, vid="v1", rid="r1", darken=False, rotated=False):
    suf = "_rotated" if rotated else ""
    names = [f"{vid}.mp4", f"{vid}.pth", f"{rid}.wav"]
    if rotated:
        names += [f"{vid}_rotated.mp4", f"{vid}_rotated.pth"]
    if darken:
        names += [f"{vid}_darken{suf}.mp4", f"{vid}_darken{suf}.pth"]
    for n in names:
        open(os.path.join(d, n), "wb").close()


def _client(tmp_path, pipes, queue_size=10):
    kw = dict(data_dir=str(tmp_path), results_dir=str(tmp_path / "results"), resolution=256)
    app = S.create_app([S.InlineWorker(p, rank=i, **kw) for i, p in enumerate(pipes)], queue_size=queue_size)
    return app, TestClient(app)


def test_ping_and_process(tmp_path):
    _files(tmp_path)
    pipe = StubPipeline()
    app, c = _client(tmp_path, [pipe])
    with c:
        assert c.get("/ping").json() == {"message": "pong"}
        r = c.post("/process", json={"id": "r1", "video_id": "v1", "audio_url": "unused"})
        assert r.status_code == 200
        body = r.json()
    assert body["message"] == "Request processed successfully" and body["gif_url"] is None
    assert body["output_url"] == str(tmp_path / "results" / "r1.npz") and os.path.exists(body["output_url"])
    assert body["elapsed_time"] >= 0
    kw = pipe.calls[0]
    # the reference's pipeline arguments (api.py:138-154)
    assert kw["video_path"] == str(tmp_path / "v1.mp4") and kw["data_path"] == str(tmp_path / "v1.pth")
    assert kw["audio_path"] == str(tmp_path / "r1.wav")
    assert (kw["num_frames"], kw["num_inference_steps"], kw["guidance_scale"]) == (16, 20, 1.5)
    assert (kw["width"], kw["height"], kw["start_from_backwards"], kw["force_video_length"]) == (256, 256, False, False)
    assert (kw["use_darken"], kw["brightness_factor"]) == (False, 1.0)


def test_path_rules(tmp_path):
    """api.py:103-123: rotated clip for dynamic clips when both files exist, darkened
    variants, and the audio fetched from a local path when missing."""
    _files(tmp_path, darken=True, rotated=True)
    p = {"id": "r2", "video_id": "v1", "is_dynamic_clip": True, "use_darken": True}
    v, d, a = S.resolve_paths(p, str(tmp_path))
    assert v.endswith("v1_darken_rotated.mp4") and d.endswith("v1_darken_rotated.pth") and a.endswith("r2.wav")
    v, d, _ = S.resolve_paths(dict(p, is_dynamic_clip=False), str(tmp_path))
    assert v.endswith("v1_darken.mp4") and d.endswith("v1_darken.pth")
    v, d, _ = S.resolve_paths(dict(p, use_darken=False), str(tmp_path))
    assert v.endswith("v1_rotated.mp4")
    src = tmp_path / "src.wav"
    src.write_bytes(b"RIFF")
    pipe = StubPipeline()
    _, c = _client(tmp_path, [pipe])
    with c:
        r = c.post("/process", json={"id": "r9", "video_id": "v1", "audio_url": "file://" + str(src)})
    assert r.status_code == 200 and (tmp_path / "r9.wav").read_bytes() == b"RIFF"
    assert S.calculate_inverse_factor(0.8) == 1.25 and S.calculate_inverse_factor(1.3) == 1.0


def test_errors_propagate(tmp_path):
    _files(tmp_path)
    _, c = _client(tmp_path, [StubPipeline(fail="boom in the pipeline")])
    with c:
        r = c.post("/process", json={"id": "r1", "video_id": "missing", "audio_url": "x"})
        assert r.status_code == 400 and r.json()["detail"] == "Video file not found."
        r = c.post("/process", json={"id": "nowav", "video_id": "v1", "audio_url": "https://example.com/a.wav"})
        assert r.status_code == 400 and r.json()["detail"] == "Audio file not found."
        with pytest.raises(RuntimeError, match="boom in the pipeline"):
            c.post("/process", json={"id": "r1", "video_id": "v1", "audio_url": "x"})
        # the worker survives a failed request
        assert c.get("/ping").status_code == 200


def _run_dispatch(workers, payloads, queue_size):
    async def go():
        d = S.Dispatcher(workers, queue_size)
        await d.start()
        try:
            res = await asyncio.gather(*[d.submit(p) for p in payloads], return_exceptions=True)
        finally:
            await d.stop()
        return d, res
    return asyncio.run(go())


def test_queue_full(tmp_path):
    """api.py:203-204: with the workers busy and the queue at maxsize, the next
    request gets the 'Queue is full' reply instead of waiting."""
    _files(tmp_path)
    gate = threading.Event()
    pipe = StubPipeline(gate=gate)
    kw = dict(data_dir=str(tmp_path), results_dir=str(tmp_path / "results"))
    w = S.InlineWorker(pipe, **kw)

    async def go():
        d = S.Dispatcher([w], queue_size=2)
        await d.start()
        first = []
        for i in range(3):
            first.append(asyncio.create_task(d.submit({"id": f"r{i}", "video_id": "v1", "audio_url": "x"})))
            await asyncio.sleep(0.2)  # r0 taken by the worker (held by the gate), then r1, r2 queued
        full = await d.submit({"id": "r1", "video_id": "v1", "audio_url": "x"})
        gate.set()
        done = await asyncio.gather(*first)
        await d.stop()
        return full, done
    _files(tmp_path, rid="r0")
    _files(tmp_path, rid="r2")
    full, done = asyncio.run(go())
    assert full is None and all(r["message"].startswith("Request processed") for r in done)


def test_dispatch_one_request_per_gpu_worker(tmp_path):
    """Requests spread over the per-GPU workers (up to N in flight), while each worker
    runs strictly one at a time (its pipeline is not re-entrant)."""
    pipes = [StubPipeline(delay=0.2) for _ in range(3)]
    kw = dict(data_dir=str(tmp_path), results_dir=str(tmp_path / "results"))
    for i in range(9):
        _files(tmp_path, rid=f"q{i}")
    t0 = time.time()
    d, res = _run_dispatch([S.InlineWorker(p, rank=i, **kw) for i, p in enumerate(pipes)],
                           [{"id": f"q{i}", "video_id": "v1", "audio_url": "x"} for i in range(9)], queue_size=10)
    wall = time.time() - t0
    assert all(isinstance(r, dict) for r in res), res
    assert sorted(d.served.values()) == [3, 3, 3] or sum(d.served.values()) == 9
    assert all(p.max_active == 1 for p in pipes)
    assert all(len(p.calls) >= 1 for p in pipes)
    assert wall < 9 * 0.2  # concurrent across workers, not serialised behind one semaphore


def _stub_factory(rank):
    return StubPipeline()


def test_process_worker_spawns_pipeline_process(tmp_path):
    """The per-GPU worker process: builds its pipeline from a factory, serves requests
    over a pipe, maps HTTPException / other errors back to the server."""
    _files(tmp_path)
    w = S.ProcessWorker(0, "test_serve:_stub_factory", data_dir=str(tmp_path), results_dir=str(tmp_path / "res"))
    w.start()
    try:
        res = asyncio.run(w.run({"id": "r1", "video_id": "v1", "audio_url": "x"}))
        assert res["output_url"].endswith("r1.npz") and os.path.exists(res["output_url"])
        with pytest.raises(S.HTTPException) as ei:
            asyncio.run(w.run({"id": "r1", "video_id": "nope", "audio_url": "x"}))
        assert ei.value.status_code == 400
    finally:
        w.stop()
    assert not w.proc.is_alive()


class _DyingPipeline(StubPipeline):
    """Ends its process in the middle of the request whose id is 'die' (a GPU fault or
    an OOM kill as the server sees it), and hangs on 'hang'."""

    def __call__(self, **kw):
        if kw["video_out_path"].endswith("die.npz"):
            os._exit(3)
        if kw["video_out_path"].endswith("hang.npz"):
            time.sleep(3600)
        return super().__call__(**kw)


def _dying_factory(rank):
    return _DyingPipeline()


def test_process_worker_replaced_after_death_and_timeout(tmp_path):
    """A worker whose child dies (or misses the request timeout) fails only the request
    in flight, with WorkerDied, and is replaced by a fresh spawned child that serves
    the next request (the server is not left routing to a dead GPU process)."""
    for rid in ("ok1", "die", "ok2", "hang", "ok3"):
        _files(tmp_path, rid=rid)
    w = S.ProcessWorker(0, "test_serve:_dying_factory", request_timeout=5.0, data_dir=str(tmp_path),
                        results_dir=str(tmp_path / "res"))
    w.start()
    try:
        first = w.proc.pid
        assert asyncio.run(w.run({"id": "ok1", "video_id": "v1", "audio_url": "x"}))["output_url"].endswith("ok1.npz")
        with pytest.raises(S.WorkerDied, match="died"):
            asyncio.run(w.run({"id": "die", "video_id": "v1", "audio_url": "x"}))
        assert w.restarts == 1 and w.proc.pid != first and w.proc.is_alive()
        assert asyncio.run(w.run({"id": "ok2", "video_id": "v1", "audio_url": "x"}))["output_url"].endswith("ok2.npz")
        t0 = time.time()
        with pytest.raises(S.WorkerDied, match="timed out"):
            asyncio.run(w.run({"id": "hang", "video_id": "v1", "audio_url": "x"}))
        assert time.time() - t0 < 60 and w.restarts == 2
        assert asyncio.run(w.run({"id": "ok3", "video_id": "v1", "audio_url": "x"}))["output_url"].endswith("ok3.npz")
    finally:
        w.stop()
    assert not w.proc.is_alive()


def _failing_factory(rank):
    raise SystemExit(7)


def test_process_worker_startup_failure_reports_exit_code(tmp_path):
    w = S.ProcessWorker(0, "test_serve:_failing_factory", data_dir=str(tmp_path), results_dir=str(tmp_path))
    with pytest.raises(RuntimeError, match="exit code 7"):
        w.start()


def test_brightness_factor_without_darken_is_served(tmp_path):
    """api.py:136-153 forwards calculate_inverse_factor(brightness_factor) always; the
    reference pipeline applies it only with use_darken (util.py:150-151).  A request
    with a recommended factor and use_darken false must reach the pipeline and pass
    the real LipsyncPipeline's option check."""
    from latentsync_amd.pipeline import LipsyncPipeline
    _files(tmp_path)
    pipe = StubPipeline()
    _, c = _client(tmp_path, [pipe])
    with c:
        r = c.post("/process", json={"id": "r1", "video_id": "v1", "audio_url": "x", "brightness_factor": 0.8,
                                     "use_darken": False})
    assert r.status_code == 200
    kw = pipe.calls[0]
    assert kw["brightness_factor"] == 1.25 and kw["use_darken"] is False
    # the real pipeline's guards accept exactly these options: it gets past them and
    # fails only on the (absent) data file
    real = LipsyncPipeline.__new__(LipsyncPipeline)
    with pytest.raises(FileNotFoundError):
        real(**dict(kw, data_path=str(tmp_path / "absent.pth")))


def _marker(name):
    return os.path.join(os.environ["LS_TEST_SERVE_DIR"], name)


def _slow_reload_factory(rank):
    """Dies on 'die' (as _DyingPipeline); a replacement child (after the first start of
    this rank) takes 4 s to load."""
    m = _marker(f"started{rank}")
    if os.path.exists(m):
        time.sleep(4.0)
    open(m, "w").close()
    return _DyingPipeline()


def test_dispatch_routes_around_a_reloading_worker(tmp_path, monkeypatch):
    """A worker whose child died is not handed the next request while its replacement
    loads: the consumer waits for 'ready' before dequeuing, so the other GPU's worker
    serves the queue at once."""
    monkeypatch.setenv("LS_TEST_SERVE_DIR", str(tmp_path))
    for rid in ("die", "a", "b"):
        _files(tmp_path, rid=rid)
    kw = dict(data_dir=str(tmp_path), results_dir=str(tmp_path / "res"))
    workers = [S.ProcessWorker(r, "test_serve:_slow_reload_factory", request_timeout=30.0, start_timeout=60.0, **kw)
               for r in range(2)]

    async def go():
        d = S.Dispatcher(workers, queue_size=10)
        await d.start()
        try:
            with pytest.raises(S.WorkerDied, match="died"):
                await d.submit({"id": "die", "video_id": "v1", "audio_url": "x"})
            t0 = time.time()
            ra = await d.submit({"id": "a", "video_id": "v1", "audio_url": "x"})
            rb = await d.submit({"id": "b", "video_id": "v1", "audio_url": "x"})
            return time.time() - t0, ra, rb
        finally:
            await d.stop()
    dt, ra, rb = asyncio.run(go())
    assert ra["output_url"].endswith("a.npz") and rb["output_url"].endswith("b.npz")
    assert sum(w.restarts for w in workers) == 1
    assert dt < 3.0, dt  # served by the healthy worker, not after the 4 s reload


def _broken_replacement_factory(rank):
    """The first child starts; a replacement fails to start while the 'broken' marker
    exists (exit 5) and starts normally once it is gone."""
    m = _marker("first")
    if os.path.exists(m) and os.path.exists(_marker("broken")):
        raise SystemExit(5)
    open(m, "w").close()
    return _DyingPipeline()


def test_process_worker_replacement_that_fails_to_start(tmp_path, monkeypatch):
    monkeypatch.setenv("LS_TEST_SERVE_DIR", str(tmp_path))
    for rid in ("die", "x1", "x2"):
        _files(tmp_path, rid=rid)
    open(_marker("broken"), "w").close()
    w = S.ProcessWorker(0, "test_serve:_broken_replacement_factory", request_timeout=30.0, start_timeout=60.0,
                        data_dir=str(tmp_path), results_dir=str(tmp_path / "res"))
    w.start()
    try:
        with pytest.raises(S.WorkerDied, match="died"):
            asyncio.run(w.run({"id": "die", "video_id": "v1", "audio_url": "x"}))
        assert w.restarts == 1
        with pytest.raises(S.WorkerDied, match="did not start"):
            asyncio.run(w.run({"id": "x1", "video_id": "v1", "audio_url": "x"}))
        assert w.restarts == 2
        os.remove(_marker("broken"))  # the factory recovers: the replacement launched above starts
        assert asyncio.run(w.run({"id": "x2", "video_id": "v1", "audio_url": "x"}))["output_url"].endswith("x2.npz")
        assert w.restarts == 2
    finally:
        w.stop()
