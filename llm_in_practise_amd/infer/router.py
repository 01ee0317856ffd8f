"""Model-group router gateway with LiteLLM ``router_settings`` semantics.

Reference: the LiteLLM proxy configs under ``Deployment/litellm-proxy/config/*.yaml`` —
``litellm-config-router-lb.yaml:1-92`` (model groups with ``weight`` / ``rpm`` / ``tpm`` /
``input_cost_per_token``; ``routing_strategy``; ``retry_policy`` 429×5 / 5xx×3 / timeout×4;
``allowed_fails: 6``, ``cooldown_time: 120``; ``fallbacks`` chain deepseek-r1 → qwen3 → llama3;
``context_window_fallbacks``) and ``litellm-config-with-guard-model.yaml:24-33`` (an
``openai_moderation`` guardrail in ``pre_call`` mode pointed at the Llama-Guard wrapper).
LiteLLM itself is not used: this module reads the same YAML (``deploy/litellm/config.yaml``)
and implements the routing behaviour in front of per-GPU ``lipa serve`` processes.

* deployments of a ``model_name`` form a group; the strategy picks one per attempt:
  ``simple-shuffle`` (weighted random by ``weight``/``rpm``), ``least-busy`` (fewest in-flight),
  ``usage-based-routing`` (most rpm headroom in the current minute), ``latency-based-routing``
  (lowest EWMA latency), ``cost-based-routing`` (lowest ``input_cost_per_token`` +
  ``output_cost_per_token``);
* an attempt that fails with 429 / 5xx / timeout is retried on the group (budget by error class,
  ``num_retries`` otherwise); a deployment with ``allowed_fails`` failures inside one minute is
  cooled down for ``cooldown_time`` seconds and skipped;
* when a group is exhausted the ``fallbacks`` list for it is tried in order; a 400 whose message
  mentions the context length switches to ``context_window_fallbacks``;
* ``max_parallel_requests`` per deployment caps its in-flight requests (the role of Ray Serve's
  ``max_ongoing_requests: 64``); a group whose deployments are all at the cap answers 429;
* ``pre_call`` moderation guardrails POST the prompt to ``<api_base>/moderations`` and reject
  flagged requests with 400 before any model is called;
* ``/v1/models``, ``/health``, ``/metrics`` (Prometheus text: per-deployment requests / failures /
  cooldowns, fallbacks, guard blocks).
* prefix / load-aware strategies of the reference's routers:
  ``load_aware_prefix`` — llm-d (``08-LLM-Router/llm-d/llm-d-config.yaml:13-25``): a load score
  from each backend's scraped ``/metrics`` with ``load_weights`` pending_requests 0.4,
  gpu_cache_usage 0.3, ttft_ms 0.2, queue_time_ms 0.1, minus a prefix-affinity bonus for the
  backend that served the longest matching prompt prefix (its KV / prefix cache is warm);
  ``prefixaware`` / ``cache_aware`` — the vLLM router's ``--routing-logic``
  (``vLLM-Router/vllm-router-deployment.yaml:34-35``, helm ``routingLogic: cache_aware``): longest
  prefix match wins, least-busy otherwise (``cache_aware`` gives up affinity when that backend is
  over ``cache_aware_imbalance`` × the least loaded one).
  Backend statistics are scraped every ``health_check_interval`` seconds (lipa or vLLM metric
  names); a backend that fails ``failure_threshold`` scrapes in a row is treated as down.

FastAPI handlers run the blocking upstream calls in the threadpool, so requests are served
concurrently (``in_flight`` / ``max_parallel_requests`` / least-busy see real concurrency).
"""
from __future__ import annotations

import collections
import dataclasses
import hashlib
import random
import threading
import time
from typing import Callable

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse
from starlette.concurrency import run_in_threadpool

STRATEGIES = ("simple-shuffle", "least-busy", "usage-based-routing", "latency-based-routing", "cost-based-routing",
              "load_aware_prefix", "prefixaware", "cache_aware")
LLMD_LOAD_WEIGHTS = {"pending_requests": 0.4, "gpu_cache_usage": 0.3, "ttft_ms": 0.2, "queue_time_ms": 0.1}
PREFIX_CHUNK = 256          # characters per prompt-prefix hash block


class UpstreamError(Exception):
    def __init__(self, status: int, body: dict | str = ""):
        super().__init__(f"upstream status {status}")
        self.status, self.body = status, body


@dataclasses.dataclass
class Deployment:
    group: str
    model: str                       # upstream model id (``openai/<id>`` prefix stripped)
    api_base: str
    api_key: str | None = None
    weight: float = 1.0
    rpm: int | None = None
    max_parallel: int | None = None  # ``max_parallel_requests`` (Ray Serve's ``max_ongoing_requests`` role)
    cost: float = 0.0
    in_flight: int = 0
    latency_ewma: float = 0.0
    minute: int = -1
    minute_count: int = 0
    fail_times: list = dataclasses.field(default_factory=list)
    cooldown_until: float = 0.0
    requests: int = 0
    failures: int = 0
    cooldowns: int = 0
    # scraped backend load (load_aware_prefix): pending, gpu_cache_usage [0,1], ttft_ms, queue_time_ms
    stats: dict = dataclasses.field(default_factory=dict)
    scrape_fails: int = 0
    down: bool = False

    @property
    def name(self) -> str:
        return f"{self.group}@{self.api_base}"


def parse_prometheus(text: str) -> dict[str, float]:
    out: dict[str, float] = {}
    for line in text.splitlines():
        if not line or line.startswith("#"):
            continue
        parts = line.split()
        if len(parts) >= 2:
            name = parts[0].split("{", 1)[0]
            try:
                out[name] = out.get(name, 0.0) + float(parts[1])
            except ValueError:
                pass
    return out


def backend_load(metrics: dict[str, float]) -> dict[str, float]:
    """lipa (``infer/engine.py``) or vLLM metric names → the llm-d load signals."""
    def get(*names, default=0.0):
        for n in names:
            if n in metrics:
                return metrics[n]
        return default

    def mean(prefixes):
        for p in prefixes:
            c = metrics.get(p + "_count")
            if c:
                return metrics.get(p + "_sum", 0.0) / c
        return 0.0
    return {"pending_requests": get("lipa_num_requests_waiting", "vllm:num_requests_waiting"),
            "gpu_cache_usage": get("lipa_gpu_cache_usage_perc", "vllm:gpu_cache_usage_perc", "vllm:kv_cache_usage_perc"),
            "ttft_ms": 1000.0 * mean(["lipa_time_to_first_token_seconds", "vllm:time_to_first_token_seconds"]),
            "queue_time_ms": 1000.0 * get("lipa_queue_time_seconds", default=mean(["vllm:request_queue_time_seconds"]))}


def http_scraper(timeout: float = 3.0) -> Callable[[Deployment], dict]:
    """GET ``<api_base without /v1>/metrics`` → load signals (raises on failure)."""
    import httpx
    client = httpx.Client(timeout=timeout)

    def scrape(dep: Deployment) -> dict:
        base = dep.api_base.rstrip("/")
        if base.endswith("/v1"):
            base = base[:-3]
        r = client.get(base + "/metrics")
        r.raise_for_status()
        return backend_load(parse_prometheus(r.text))
    return scrape


def prompt_prefix_hashes(body: dict, chunk: int = PREFIX_CHUNK) -> list[str]:
    """Chained content hashes of the prompt text in ``chunk``-character blocks (the router-level
    analogue of the engine's token-block prefix hashes)."""
    if body.get("messages"):
        text = "".join(f"<{m.get('role', '')}>{m.get('content', '')}" for m in body["messages"])
    else:
        text = str(body.get("prompt", ""))
    out, h = [], b""
    for i in range(0, len(text) - len(text) % chunk, chunk):
        h = hashlib.blake2b(h + text[i:i + chunk].encode(), digest_size=12).digest()
        out.append(h.hex())
    return out


def resolve_service(host: str, port: int) -> list[str]:
    """IPv4 addresses behind a DNS name (a headless Service resolves to its ready pods)."""
    import socket
    return sorted({ai[4][0] for ai in socket.getaddrinfo(host, port, socket.AF_INET, socket.SOCK_STREAM)})


def load_config(cfg: dict | str) -> dict:
    if isinstance(cfg, str):
        import yaml
        with open(cfg) as f:
            cfg = yaml.safe_load(f)
    return cfg


def http_sender(timeout: float = 600.0) -> Callable[[Deployment, str, dict], dict]:
    """Upstream caller: POST ``api_base + path``; raises :class:`UpstreamError` (status 408 on timeout)."""
    import httpx
    client = httpx.Client(timeout=timeout)

    def send(dep: Deployment, path: str, body: dict) -> dict:
        headers = {"Authorization": f"Bearer {dep.api_key}"} if dep.api_key and dep.api_key != "none" else {}
        try:
            r = client.post(dep.api_base.rstrip("/") + path, json=body, headers=headers)
        except httpx.TimeoutException:
            raise UpstreamError(408, "timeout")
        except httpx.TransportError as e:
            raise UpstreamError(503, str(e))
        if r.status_code >= 400:
            try:
                raise UpstreamError(r.status_code, r.json())
            except ValueError:
                raise UpstreamError(r.status_code, r.text)
        return r.json()
    return send


class Router:
    def __init__(self, cfg: dict | str, send: Callable[[Deployment, str, dict], dict] | None = None,
                 clock: Callable[[], float] = time.time, seed: int | None = None,
                 resolver: Callable[[str, int], list[str]] | None = None):
        cfg = load_config(cfg)
        rs = cfg.get("router_settings", {}) or {}
        self.strategy = rs.get("routing_strategy", "simple-shuffle")
        if self.strategy not in STRATEGIES:
            raise ValueError(f"routing_strategy {self.strategy!r} not in {STRATEGIES}")
        self.num_retries = int(rs.get("num_retries", 0))
        pol = rs.get("retry_policy", {}) or {}
        self.retry_budget = {429: pol.get("RateLimitErrorRetries"), 500: pol.get("InternalServerErrorRetries"),
                             408: pol.get("TimeoutErrorRetries")}
        self.allowed_fails = int(rs.get("allowed_fails", 3))
        self.cooldown_time = float(rs.get("cooldown_time", 60))
        self.fallbacks = self._fallback_map(rs.get("fallbacks") or (cfg.get("litellm_settings") or {}).get("fallbacks"))
        self.ctx_fallbacks = self._fallback_map(rs.get("context_window_fallbacks"))
        self.guards = [g["litellm_params"] for g in cfg.get("guardrails", []) or []
                       if (g.get("litellm_params") or {}).get("mode", "pre_call") == "pre_call"]
        self.groups: dict[str, list[Deployment]] = collections.defaultdict(list)
        for m in cfg.get("model_list", []):
            lp = m.get("litellm_params", {})
            model = str(lp.get("model", m["model_name"]))
            self.groups[m["model_name"]].append(Deployment(
                group=m["model_name"], model=model.split("/", 1)[1] if model.startswith("openai/") else model,
                api_base=lp.get("api_base", ""), api_key=lp.get("api_key"),
                weight=float(lp.get("weight", lp.get("rpm", 1) or 1)), rpm=lp.get("rpm"),
                max_parallel=lp.get("max_parallel_requests", m.get("max_parallel_requests")),
                cost=float(lp.get("input_cost_per_token", 0) or 0) + float(lp.get("output_cost_per_token", 0) or 0)))
        self.send = send or http_sender()
        self.clock = clock
        self.rng = random.Random(seed)
        self.lock = threading.Lock()
        self.counters = collections.Counter()
        # prefix / load-aware routing (llm-d load_aware_prefix, vLLM router prefixaware / cache_aware)
        self.load_weights = dict(LLMD_LOAD_WEIGHTS)
        self.load_weights.update({k: float(v) for k, v in (rs.get("load_weights") or {}).items()})
        self.prefix_weight = float(rs.get("prefix_weight", 0.5))
        self.imbalance = float(rs.get("cache_aware_imbalance", 2.0))
        self.scrape_interval = float(rs.get("health_check_interval", 5))
        self.failure_threshold = int(rs.get("failure_threshold", 2))
        self.prefix_owner: collections.OrderedDict[str, str] = collections.OrderedDict()
        self.prefix_capacity = int(rs.get("prefix_table_size", 100_000))
        self.scraper: Callable[[Deployment], dict] | None = None
        self._last_scrape = -1e18
        # Kubernetes discovery (the llm-d / vLLM-router RBAC pod watch role): the A records of a
        # headless Service are the replica pods; re-resolved every `interval` seconds
        self.discovery = [dict(d) for d in (rs.get("discovery") or [])]
        self.resolver: Callable[[str, int], list[str]] = resolver or resolve_service
        self._last_discovery = -1e18
        if self.discovery:
            self.refresh_discovery(force=True)

    def refresh_discovery(self, force: bool = False):
        """Sync each discovered group's deployments with the pod IPs behind its Service name:
        new pods join (fresh stats), vanished pods leave; existing deployments keep their state."""
        if not self.discovery:
            return
        now = self.clock()
        interval = min(float(d.get("interval", 10)) for d in self.discovery)
        if not force and now - self._last_discovery < interval:
            return
        self._last_discovery = now
        for spec in self.discovery:
            group, port = spec["model_name"], int(spec.get("port", 8000))
            try:
                ips = self.resolver(spec["service"], port)
            except OSError:
                continue                          # DNS hiccup: keep the last known set
            scheme = spec.get("scheme", "http")
            want = {f"{scheme}://{ip}:{port}/v1" for ip in ips}
            with self.lock:
                cur = self.groups.get(group, [])
                keep = [d for d in cur if d.api_base in want]
                have = {d.api_base for d in keep}
                for base in sorted(want - have):
                    keep.append(Deployment(group=group, model=spec.get("model", group), api_base=base,
                                           api_key=spec.get("api_key"),
                                           max_parallel=spec.get("max_parallel_requests")))
                self.groups[group] = keep
                self.counters["discovery_refreshes"] += 1

    @staticmethod
    def _fallback_map(spec) -> dict[str, list[str]]:
        out: dict[str, list[str]] = {}
        for item in spec or []:
            for k, v in item.items():
                out[k] = list(v) if isinstance(v, (list, tuple)) else [v]
        return out

    # ------------------------------------------------------------------ selection / health
    def _healthy(self, group: str) -> list[Deployment]:
        now = self.clock()
        return [d for d in self.groups.get(group, []) if d.cooldown_until <= now]

    # ------------------------------------------------------------------ backend load / prefix affinity
    def refresh_stats(self, force: bool = False):
        """Scrape every deployment's /metrics (at most once per health-check interval)."""
        if self.scraper is None:
            return
        now = self.clock()
        if not force and now - self._last_scrape < self.scrape_interval:
            return
        self._last_scrape = now
        for deps in self.groups.values():
            for d in deps:
                try:
                    st = self.scraper(d)
                except Exception:
                    d.scrape_fails += 1
                    d.down = d.scrape_fails >= self.failure_threshold
                    continue
                d.stats, d.scrape_fails, d.down = st, 0, False

    def _prefix_scores(self, hashes: list[str]) -> dict[str, float]:
        """deployment name → fraction of the prompt's leading blocks it served last."""
        if not hashes:
            return {}
        run: dict[str, int] = collections.Counter()
        for h in hashes:
            owner = self.prefix_owner.get(h)
            if owner is None:
                break
            run[owner] += 1
        return {k: v / len(hashes) for k, v in run.items()}

    def _remember_prefix(self, hashes: list[str], dep: Deployment):
        for h in hashes:
            self.prefix_owner[h] = dep.name
            self.prefix_owner.move_to_end(h)
        while len(self.prefix_owner) > self.prefix_capacity:
            self.prefix_owner.popitem(last=False)

    def load_score(self, d: Deployment, cands: list[Deployment]) -> float:
        """llm-d weighted load: each signal normalised by its max over the candidates."""
        st = dict(d.stats)
        st["pending_requests"] = st.get("pending_requests", 0.0) + d.in_flight
        score = 0.0
        for k, w in self.load_weights.items():
            if k == "gpu_cache_usage":
                score += w * min(1.0, max(0.0, st.get(k, 0.0)))
                continue
            mx = max((c.stats.get(k, 0.0) + (c.in_flight if k == "pending_requests" else 0)) for c in cands)
            score += w * (st.get(k, 0.0) / mx if mx > 0 else 0.0)
        return score

    def _pick_prefix(self, cands: list[Deployment], pref: dict[str, float]) -> Deployment:
        if self.strategy == "load_aware_prefix":
            return min(cands, key=lambda d: (self.load_score(d, cands) - self.prefix_weight * pref.get(d.name, 0.0),
                                             d.in_flight))
        least = min(d.in_flight for d in cands)
        best = max(cands, key=lambda d: (pref.get(d.name, 0.0), -d.in_flight))
        if pref.get(best.name, 0.0) > 0:
            if self.strategy == "prefixaware" or best.in_flight <= self.imbalance * max(1, least):
                return best
        return self.rng.choice([d for d in cands if d.in_flight == least])

    def pick(self, group: str, exclude: set[str] = frozenset(), body: dict | None = None) -> Deployment | None:
        self.refresh_discovery()
        if self.strategy in ("load_aware_prefix", "prefixaware", "cache_aware"):
            self.refresh_stats()
        with self.lock:
            healthy = [d for d in self._healthy(group) if (d.max_parallel is None or d.in_flight < d.max_parallel)
                       and not d.down]
            cands = [d for d in healthy if d.name not in exclude] or healthy
            if not cands:
                if self._healthy(group):            # every deployment is at max_parallel_requests
                    raise UpstreamError(429, f"all deployments of {group!r} are at max_parallel_requests")
                return None
            minute = int(self.clock() // 60)
            if self.strategy == "least-busy":
                best = min(d.in_flight for d in cands)
                cands = [d for d in cands if d.in_flight == best]
                dep = self.rng.choice(cands)
            elif self.strategy == "usage-based-routing":
                def headroom(d):
                    used = d.minute_count if d.minute == minute else 0
                    return (d.rpm or float("inf")) - used
                dep = max(cands, key=headroom)
            elif self.strategy == "latency-based-routing":
                dep = min(cands, key=lambda d: d.latency_ewma)
            elif self.strategy == "cost-based-routing":
                dep = min(cands, key=lambda d: d.cost)
            elif self.strategy in ("load_aware_prefix", "prefixaware", "cache_aware"):
                hashes = prompt_prefix_hashes(body or {})
                pref = self._prefix_scores(hashes)
                dep = self._pick_prefix(cands, pref)
                self.counters["prefix_hits_total"] += int(pref.get(dep.name, 0.0) > 0)
                self._remember_prefix(hashes, dep)
            else:
                dep = self.rng.choices(cands, weights=[max(d.weight, 1e-9) for d in cands])[0]
            if dep.minute != minute:
                dep.minute, dep.minute_count = minute, 0
            dep.minute_count += 1
            dep.in_flight += 1
            dep.requests += 1
            return dep

    def _done(self, dep: Deployment, ok: bool, dt: float):
        with self.lock:
            dep.in_flight -= 1
            if ok:
                dep.latency_ewma = dt if dep.latency_ewma == 0 else 0.8 * dep.latency_ewma + 0.2 * dt
                return
            dep.failures += 1
            now = self.clock()
            dep.fail_times = [t for t in dep.fail_times if t > now - 60] + [now]
            if len(dep.fail_times) >= self.allowed_fails:
                dep.cooldown_until, dep.fail_times = now + self.cooldown_time, []
                dep.cooldowns += 1

    def _budget(self, status: int) -> int:
        key = 500 if status >= 500 else status
        b = self.retry_budget.get(key)
        return int(b) if b is not None else self.num_retries

    # ------------------------------------------------------------------ request path
    def moderate(self, body: dict) -> dict | None:
        """Run pre-call guardrails; returns the flagging moderation result or None."""
        if not self.guards:
            return None
        text = "\n".join(str(m.get("content", "")) for m in body.get("messages", [])) or str(body.get("prompt", ""))
        for g in self.guards:
            dep = Deployment(group="guard", model=str(g.get("model", "guard")), api_base=g.get("api_base", ""),
                             api_key=g.get("api_key"))
            res = self.send(dep, "/moderations", {"input": text})
            if any(r.get("flagged") for r in res.get("results", [])):
                self.counters["guard_blocked_total"] += 1
                return res
        return None

    def _try_group(self, group: str, path: str, body: dict) -> dict:
        tried: set[str] = set()
        used: collections.Counter = collections.Counter()
        last: UpstreamError | None = None
        while True:
            dep = self.pick(group, tried, body)
            if dep is None:
                raise last or UpstreamError(503, f"no healthy deployment in group {group!r}")
            t0 = self.clock()
            try:
                out = self.send(dep, path, {**body, "model": dep.model})
            except UpstreamError as e:
                self._done(dep, False, 0.0)
                last = e
                if e.status == 400:                     # client error: never retried on the same group
                    raise
                cls = 500 if e.status >= 500 else e.status
                used[cls] += 1
                tried.add(dep.name)
                if used[cls] > self._budget(e.status):
                    raise
                self.counters["retries_total"] += 1
                continue
            self._done(dep, True, self.clock() - t0)
            return out

    def route(self, path: str, body: dict) -> dict:
        group = body.get("model") or next(iter(self.groups), "")
        if group not in self.groups:
            raise UpstreamError(404, f"model {group!r} not in model_list")
        chain, seen = [group], {group}
        i = 0
        while i < len(chain):
            g = chain[i]
            try:
                out = self._try_group(g, path, body)
                out["model"] = g
                return out
            except UpstreamError as e:
                msg = str(e.body).lower()
                nxt = self.ctx_fallbacks.get(g, []) if e.status == 400 and "context" in msg else \
                    (self.fallbacks.get(g, []) if e.status != 400 else [])
                for f in nxt:
                    if f not in seen and f in self.groups:
                        chain.append(f)
                        seen.add(f)
                if i + 1 >= len(chain):
                    raise
                self.counters["fallbacks_total"] += 1
            i += 1
        raise UpstreamError(503, "all fallbacks exhausted")

    def metrics_text(self) -> str:
        lines = []
        for name in ("retries_total", "fallbacks_total", "guard_blocked_total", "prefix_hits_total"):
            lines += [f"# TYPE lipa_router_{name} counter", f"lipa_router_{name} {self.counters[name]}"]
        for metric, attr in (("requests_total", "requests"), ("failures_total", "failures"),
                             ("cooldowns_total", "cooldowns"), ("in_flight", "in_flight")):
            lines.append(f"# TYPE lipa_router_deployment_{metric} {'gauge' if attr == 'in_flight' else 'counter'}")
            for deps in self.groups.values():
                for d in deps:
                    lines.append(f'lipa_router_deployment_{metric}{{group="{d.group}",api_base="{d.api_base}"}} '
                                 f"{getattr(d, attr)}")
        return "\n".join(lines) + "\n"


def create_router_app(router: Router, scrape: bool = True) -> FastAPI:
    app = FastAPI(title="lipa router")
    if scrape and router.scraper is None and router.strategy in ("load_aware_prefix", "prefixaware", "cache_aware"):
        router.scraper = http_scraper()

    async def handle(path: str, request: Request):
        body = await request.json()
        if body.get("stream"):
            return JSONResponse({"error": {"message": "streaming is served by the backends directly; "
                                                      "the router proxies non-streaming requests"}}, 400)
        flagged = await run_in_threadpool(router.moderate, body)
        if flagged is not None:
            return JSONResponse({"error": {"message": "request blocked by moderation guardrail",
                                           "type": "guardrail_violation", "moderation": flagged}}, 400)
        try:
            return JSONResponse(await run_in_threadpool(router.route, path, body))
        except UpstreamError as e:
            return JSONResponse({"error": {"message": str(e.body) or str(e), "code": e.status}}, e.status)

    @app.post("/v1/chat/completions")
    async def chat(request: Request):
        return await handle("/chat/completions", request)

    @app.post("/v1/completions")
    async def completions(request: Request):
        return await handle("/completions", request)

    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": g, "object": "model", "owned_by": "lipa-router"}
                                           for g in router.groups]}

    @app.get("/health")
    async def health():
        healthy = {g: len(router._healthy(g)) for g in router.groups}
        return {"status": "ok" if all(healthy.values()) else "degraded", "healthy_deployments": healthy}

    @app.get("/metrics")
    async def metrics():
        return PlainTextResponse(router.metrics_text())

    return app
