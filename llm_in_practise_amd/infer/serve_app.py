"""Replica controller with Ray Serve LLM-app semantics.

Reference: ``Deployment/Ray/serve_deploy_examples/*.yaml`` deployed with ``serve deploy``:
``qwen3_app_autoscaling.yaml`` (``autoscaling_config``: ``min_replicas`` 1, ``max_replicas`` 2,
``target_ongoing_requests`` 5, ``upscale_delay`` 5 s, ``downscale_delay`` 30 s;
``max_ongoing_requests`` 64 per replica), ``serve_app_two_models.yaml`` (two applications under
``route_prefix`` /app1 and /app2, one of them ``quantization: awq``) and
``qwen3_app_pipeline_parallel.yaml`` (``pipeline_parallel_size: 2``).  Ray is not used: the same
YAML drives this controller, which runs ``lipa serve`` replicas (one process per MI355X, or a
``torchrun`` group of ``tensor_parallel_size × pipeline_parallel_size`` GPUs) behind one HTTP
proxy.

Semantics kept from Ray Serve:

* **Ongoing requests** are counted by the proxy per replica (sent, not yet answered / stream not
  finished).  A replica at ``max_ongoing_requests`` takes no new request; when every replica is
  full, requests wait in the proxy queue (``max_queued_requests``, −1 = unbounded) and a full
  queue answers 503 — Ray's back-pressure.
* **Routing**: power of two choices on ongoing requests among the replicas with headroom.
* **Autoscaling**: ``desired = ceil(Σ ongoing (+ queued) / target_ongoing_requests)`` clamped to
  ``[min_replicas, max_replicas]``; a scale-up is applied only after the decision has held for
  ``upscale_delay`` seconds, a scale-down after ``downscale_delay`` seconds.  Scale-down drains:
  the replica gets no new requests and stops once its ongoing count reaches 0.
* Each application is served under its ``route_prefix`` (``/app1/v1/chat/completions``), and
  ``/-/routes``, ``/-/healthz`` and ``/metrics`` report the controller state.

GPU assignment: replicas take GPUs from the pool given to the controller (``--gpus 0,1,2,3``),
``tensor_parallel_size × pipeline_parallel_size`` each; a scale-up with no free GPU is deferred.
"""
from __future__ import annotations

import asyncio
import dataclasses
import math
import os
import random
import socket
import subprocess
import sys
import threading
import time
from typing import Callable

import httpx
import yaml
from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse


@dataclasses.dataclass
class AutoscalingConfig:
    min_replicas: int = 1
    max_replicas: int = 1
    target_ongoing_requests: float = 2.0       # Ray Serve's default
    upscale_delay: float = 30.0
    downscale_delay: float = 600.0
    initial_replicas: int | None = None

    @classmethod
    def from_dict(cls, d: dict | None) -> "AutoscalingConfig":
        d = dict(d or {})
        known = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in known})


@dataclasses.dataclass
class AppConfig:
    name: str
    route_prefix: str
    model_id: str
    model_source: str
    autoscaling: AutoscalingConfig
    max_ongoing_requests: int = 5              # Ray Serve's default
    max_queued_requests: int = -1
    num_replicas: int | None = None            # fixed replica count (no autoscaling_config)
    engine_kwargs: dict = dataclasses.field(default_factory=dict)

    @property
    def gpus_per_replica(self) -> int:
        ek = self.engine_kwargs
        return int(ek.get("tensor_parallel_size", 1) or 1) * int(ek.get("pipeline_parallel_size", 1) or 1)


def load_serve_config(cfg: str | dict) -> list[AppConfig]:
    """Parse a Ray Serve ``serve deploy`` config with ``ray.serve.llm:build_openai_app`` apps."""
    if isinstance(cfg, str):
        with open(cfg) as f:
            cfg = yaml.safe_load(f)
    apps = []
    for app in cfg.get("applications", []):
        args = app.get("args", {}) or {}
        for i, llm in enumerate(args.get("llm_configs", []) or []):
            mlc = llm.get("model_loading_config", {}) or {}
            dep = llm.get("deployment_config", {}) or {}
            auto = dep.get("autoscaling_config")
            nrep = dep.get("num_replicas")
            a = AutoscalingConfig.from_dict(auto) if auto else AutoscalingConfig(
                min_replicas=int(nrep or 1), max_replicas=int(nrep or 1))
            name = app.get("name", f"app{len(apps)}") + (f"-{i}" if i else "")
            apps.append(AppConfig(name=name, route_prefix=(app.get("route_prefix") or "/").rstrip("/") or "/",
                                  model_id=mlc.get("model_id", name), model_source=mlc.get("model_source", ""),
                                  autoscaling=a, max_ongoing_requests=int(dep.get("max_ongoing_requests", 5)),
                                  max_queued_requests=int(dep.get("max_queued_requests", -1)),
                                  num_replicas=nrep, engine_kwargs=dict(llm.get("engine_kwargs", {}) or {})))
    return apps


class Autoscaler:
    """Ray Serve's request-based policy with up/down delays (pure; injectable clock)."""

    def __init__(self, cfg: AutoscalingConfig, clock: Callable[[], float] = time.monotonic):
        self.cfg, self.clock = cfg, clock
        self._pending: tuple[int, float] | None = None     # (proposed count, since)

    def desired(self, total_ongoing: float) -> int:
        c = self.cfg
        want = math.ceil(total_ongoing / max(c.target_ongoing_requests, 1e-9)) if total_ongoing > 0 else c.min_replicas
        return max(c.min_replicas, min(c.max_replicas, want))

    def decide(self, total_ongoing: float, current: int) -> int:
        want = self.desired(total_ongoing)
        if want == current:
            self._pending = None
            return current
        now = self.clock()
        direction = 1 if want > current else -1
        if self._pending is None or (self._pending[0] > current) != (direction > 0):
            self._pending = (want, now)          # a new decision starts its delay
            return current
        self._pending = (want, self._pending[1])
        delay = self.cfg.upscale_delay if direction > 0 else self.cfg.downscale_delay
        if now - self._pending[1] >= delay:
            self._pending = None
            return want
        return current


class Replica:
    """One backend: its base URL, the proxy's ongoing count, and a drain flag."""

    def __init__(self, url: str, handle=None, gpus: tuple[int, ...] = ()):
        self.url, self.handle, self.gpus = url.rstrip("/"), handle, gpus
        self.ongoing = 0
        self.served = 0
        self.draining = False
        self.ready = handle is None

    def stop(self):
        if self.handle is not None and hasattr(self.handle, "terminate"):
            self.handle.terminate()
            try:
                self.handle.wait(30)
            except Exception:
                self.handle.kill()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def process_replica_factory(host: str = "127.0.0.1", extra_args: tuple[str, ...] = ()):
    """Start ``lipa serve`` for an app on the given GPUs (``torchrun`` when it spans several)."""

    def start(app: AppConfig, gpus: tuple[int, ...]) -> Replica:
        port = _free_port()
        ek = app.engine_kwargs
        args = ["serve", "--model", app.model_source, "--host", host, "--port", str(port),
                "--served-model-name", app.model_id, "--max-batch", str(max(app.max_ongoing_requests, 1))]
        if ek.get("max_model_len"):
            args += ["--max-model-len", str(ek["max_model_len"])]
        if ek.get("enable_prefix_caching"):
            args += ["--enable-prefix-caching"]
        if int(ek.get("pipeline_parallel_size", 1) or 1) > 1:
            args += ["--pipeline-parallel-size", str(ek["pipeline_parallel_size"])]
        if int(ek.get("tensor_parallel_size", 1) or 1) > 1:
            args += ["--tensor-parallel-size", str(ek["tensor_parallel_size"])]
        env = dict(os.environ, HIP_VISIBLE_DEVICES=",".join(map(str, gpus)), HSA_ENABLE_IPC_MODE_LEGACY="0")
        if len(gpus) > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={len(gpus)}",
                   "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                   "-m", "llm_in_practise_amd.cli.main", *args, *extra_args]
        else:
            cmd = [sys.executable, "-m", "llm_in_practise_amd.cli.main", *args, *extra_args]
        proc = subprocess.Popen(cmd, env=env)
        r = Replica(f"http://{host}:{port}", proc, gpus)
        r.ready = False
        return r

    return start


class Application:
    def __init__(self, cfg: AppConfig, controller: "ServeController"):
        self.cfg, self.ctl = cfg, controller
        self.replicas: list[Replica] = []
        self.autoscaler = Autoscaler(cfg.autoscaling, controller.clock)
        self.queued = 0
        self.rejected = 0
        self.cond: asyncio.Condition | None = None
        self.scale_events: list[tuple[float, int, int]] = []

    def live(self) -> list[Replica]:
        return [r for r in self.replicas if r.ready and not r.draining]

    def total_ongoing(self) -> int:
        return sum(r.ongoing for r in self.replicas if not r.draining) + self.queued

    def choose(self) -> Replica | None:
        """Power of two choices among replicas under max_ongoing_requests."""
        cand = [r for r in self.live() if r.ongoing < self.cfg.max_ongoing_requests]
        if not cand:
            return None
        if len(cand) == 1:
            return cand[0]
        a, b = random.sample(cand, 2)
        return a if a.ongoing <= b.ongoing else b


class ServeController:
    def __init__(self, apps: list[AppConfig], replica_factory: Callable[[AppConfig, tuple[int, ...]], Replica],
                 gpus: list[int] | None = None, clock: Callable[[], float] = time.monotonic,
                 control_interval: float = 1.0, health_timeout: float = 600.0):
        self.clock = clock
        self.factory = replica_factory
        self.free_gpus = list(gpus) if gpus is not None else None
        self.apps = {a.name: Application(a, self) for a in apps}
        self.control_interval = control_interval
        self.health_timeout = health_timeout
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        for app in self.apps.values():
            n0 = app.cfg.autoscaling.initial_replicas or app.cfg.autoscaling.min_replicas
            for _ in range(n0):
                self._add_replica(app)

    # ---------------------------------------------------------------- replica lifecycle
    def _take_gpus(self, n: int) -> tuple[int, ...] | None:
        if self.free_gpus is None:
            return ()
        if len(self.free_gpus) < n:
            return None
        got, self.free_gpus = tuple(self.free_gpus[:n]), self.free_gpus[n:]
        return got

    def _add_replica(self, app: Application) -> bool:
        gpus = self._take_gpus(app.cfg.gpus_per_replica)
        if gpus is None:
            return False
        r = self.factory(app.cfg, gpus)
        r.started = self.clock()
        app.replicas.append(r)
        return True

    def _retire(self, app: Application, r: Replica):
        r.stop()
        app.replicas.remove(r)
        if self.free_gpus is not None:
            self.free_gpus.extend(r.gpus)

    def _probe(self, r: Replica) -> bool:
        try:
            return httpx.get(r.url + "/health", timeout=2.0).status_code == 200
        except Exception:
            return False

    # ---------------------------------------------------------------- control loop
    def reconcile(self):
        """One control step: readiness probes, drain completion, autoscaling decisions."""
        with self._lock:
            for app in self.apps.values():
                for r in list(app.replicas):
                    if not r.ready and self._probe(r):
                        r.ready = True
                    if r.draining and r.ongoing == 0:
                        self._retire(app, r)
                current = len([r for r in app.replicas if not r.draining])
                target = app.autoscaler.decide(app.total_ongoing(), current)
                if target > current:
                    for _ in range(target - current):
                        if not self._add_replica(app):
                            break
                    app.scale_events.append((self.clock(), current, target))
                elif target < current:
                    # drain the least-loaded replicas
                    for r in sorted([r for r in app.replicas if not r.draining], key=lambda r: r.ongoing)[
                            :current - target]:
                        r.draining = True
                    app.scale_events.append((self.clock(), current, target))
            self._wake()

    def _wake(self):
        for app in self.apps.values():
            if app.cond is not None and self.loop is not None:
                async def notify(c=app.cond):
                    async with c:
                        c.notify_all()
                asyncio.run_coroutine_threadsafe(notify(), self.loop)

    loop: asyncio.AbstractEventLoop | None = None

    def start(self):
        def run():
            while not self._stop.wait(self.control_interval):
                try:
                    self.reconcile()
                except Exception:            # keep controlling through a transient probe error
                    pass
        self._thread = threading.Thread(target=run, daemon=True)
        self._thread.start()

    def shutdown(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(10)
        with self._lock:
            for app in self.apps.values():
                for r in list(app.replicas):
                    self._retire(app, r)

    # ---------------------------------------------------------------- status
    def status(self) -> dict:
        return {name: {"route_prefix": a.cfg.route_prefix, "model_id": a.cfg.model_id,
                       "replicas": [{"url": r.url, "ready": r.ready, "draining": r.draining, "ongoing": r.ongoing,
                                     "served": r.served, "gpus": list(r.gpus)} for r in a.replicas],
                       "queued": a.queued, "rejected": a.rejected,
                       "target_ongoing_requests": a.cfg.autoscaling.target_ongoing_requests,
                       "max_ongoing_requests": a.cfg.max_ongoing_requests}
                for name, a in self.apps.items()}

    def metrics_text(self) -> str:
        out = []
        for metric, fn in (("replicas", lambda a: len([r for r in a.replicas if not r.draining])),
                           ("ongoing_requests", lambda a: sum(r.ongoing for r in a.replicas)),
                           ("queued_requests", lambda a: a.queued), ("rejected_total", lambda a: a.rejected)):
            out.append(f"# TYPE lipa_serve_{metric} gauge")
            for name, a in self.apps.items():
                out.append(f'lipa_serve_{metric}{{app="{name}"}} {fn(a)}')
        return "\n".join(out) + "\n"


def create_serve_proxy(ctl: ServeController, request_timeout: float = 600.0) -> FastAPI:
    import contextlib
    client = httpx.AsyncClient(timeout=request_timeout, limits=httpx.Limits(max_connections=None))

    @contextlib.asynccontextmanager
    async def lifespan(_app):
        ctl.loop = asyncio.get_running_loop()
        for a in ctl.apps.values():
            a.cond = asyncio.Condition()
        yield
        await client.aclose()

    app = FastAPI(title="lipa serve-deploy proxy", lifespan=lifespan)

    def _match(path: str) -> tuple[Application, str] | None:
        best = None
        for a in ctl.apps.values():
            p = a.cfg.route_prefix
            if p == "/" or path == p or path.startswith(p + "/"):
                if best is None or len(p) > len(best.cfg.route_prefix):
                    best = a
        if best is None:
            return None
        rest = path if best.cfg.route_prefix == "/" else path[len(best.cfg.route_prefix):]
        return best, rest or "/"

    async def _acquire(a: Application) -> Replica | None:
        r = a.choose()
        if r is not None:
            r.ongoing += 1
            return r
        if a.cfg.max_queued_requests >= 0 and a.queued >= a.cfg.max_queued_requests:
            a.rejected += 1
            return None
        a.queued += 1
        try:
            async with a.cond:
                while True:
                    r = a.choose()
                    if r is not None:
                        r.ongoing += 1
                        return r
                    try:
                        await asyncio.wait_for(a.cond.wait(), timeout=0.05)
                    except asyncio.TimeoutError:
                        pass
        finally:
            a.queued -= 1

    async def _release(a: Application, r: Replica):
        r.ongoing -= 1
        r.served += 1
        async with a.cond:
            a.cond.notify()

    @app.get("/-/routes")
    async def routes():
        return {a.cfg.route_prefix: a.cfg.name for a in ctl.apps.values()}

    @app.get("/-/healthz")
    async def healthz():
        ok = all(a.live() for a in ctl.apps.values())
        return JSONResponse({"status": "ok" if ok else "starting", "apps": ctl.status()}, 200 if ok else 503)

    @app.get("/metrics")
    async def metrics():
        return PlainTextResponse(ctl.metrics_text())

    @app.api_route("/{path:path}", methods=["GET", "POST"])
    async def proxy(path: str, request: Request):
        m = _match("/" + path)
        if m is None:
            return JSONResponse({"error": {"message": f"no application serves /{path}"}}, 404)
        a, rest = m
        if request.method == "GET" and rest.rstrip("/") == "/v1/models":
            return {"object": "list", "data": [{"id": a.cfg.model_id, "object": "model", "owned_by": "lipa"}]}
        r = await _acquire(a)
        if r is None:
            return JSONResponse({"error": {"message": "all replicas at max_ongoing_requests and the queue is full",
                                           "type": "back_pressure"}}, 503)
        body = await request.body()
        headers = {k: v for k, v in request.headers.items() if k.lower() in ("content-type", "authorization")}
        try:
            req = client.build_request(request.method, r.url + rest, content=body, headers=headers)
            resp = await client.send(req, stream=True)
        except Exception as e:
            await _release(a, r)
            return JSONResponse({"error": {"message": f"replica {r.url} failed: {e!r}"}}, 502)

        async def relay():
            try:
                async for chunk in resp.aiter_raw():
                    yield chunk
            finally:
                await resp.aclose()
                await _release(a, r)

        return StreamingResponse(relay(), status_code=resp.status_code,
                                 media_type=resp.headers.get("content-type"))

    return app
