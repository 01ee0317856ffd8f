"""LiteLLM-semantics router gateway: strategies, retries, cooldown, fallbacks, guardrail."""
import collections

import pytest
from fastapi.testclient import TestClient

from llm_in_practise_amd.infer.router import Router, UpstreamError, create_router_app, load_config


class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def cfg(strategy="simple-shuffle", **rs):
    return {
        "model_list": [
            {"model_name": "qwen3-8b", "litellm_params": {"model": "openai/qwen3-8b", "api_base": "http://a/v1",
                                                          "weight": 3, "input_cost_per_token": 2e-6}},
            {"model_name": "qwen3-8b", "litellm_params": {"model": "openai/qwen3-8b", "api_base": "http://b/v1",
                                                          "weight": 1, "input_cost_per_token": 1e-6}},
            {"model_name": "r1-awq", "litellm_params": {"model": "openai/r1", "api_base": "http://c/v1"}},
            {"model_name": "long-ctx", "litellm_params": {"model": "openai/long", "api_base": "http://d/v1"}},
        ],
        "router_settings": {"routing_strategy": strategy, "num_retries": 2,
                            "retry_policy": {"RateLimitErrorRetries": 5, "InternalServerErrorRetries": 3,
                                             "TimeoutErrorRetries": 4},
                            "allowed_fails": 2, "cooldown_time": 120,
                            "fallbacks": [{"r1-awq": ["qwen3-8b"]}],
                            "context_window_fallbacks": [{"qwen3-8b": ["long-ctx"]}], **rs},
    }


def ok_sender(calls, fail=None):
    def send(dep, path, body):
        calls.append((dep.api_base, path, body["model"]))
        if fail and dep.api_base in fail:
            st = fail[dep.api_base]
            raise UpstreamError(st, {"message": "maximum context length exceeded"} if st == 400 else "boom")
        return {"choices": [{"message": {"content": f"hi from {dep.api_base}"}}], "model": body["model"]}
    return send


def test_weighted_shuffle_respects_weights():
    calls = []
    r = Router(cfg(), ok_sender(calls), seed=0)
    for _ in range(400):
        r.route("/chat/completions", {"model": "qwen3-8b", "messages": []})
    c = collections.Counter(a for a, _, _ in calls)
    assert 0.65 < c["http://a/v1"] / 400 < 0.85
    assert calls[0][2] == "qwen3-8b"          # openai/ prefix stripped for the upstream call


def test_cost_and_least_busy_strategies():
    calls = []
    r = Router(cfg("cost-based-routing"), ok_sender(calls))
    r.route("/chat/completions", {"model": "qwen3-8b"})
    assert calls[-1][0] == "http://b/v1"
    r = Router(cfg("least-busy"), ok_sender(calls), seed=0)
    a = r.pick("qwen3-8b")
    b = r.pick("qwen3-8b")
    assert a is not b                          # second pick avoids the busy deployment


def test_retry_then_cooldown_then_recover():
    calls, clock = [], Clock()
    r = Router(cfg("cost-based-routing"), ok_sender(calls, {"http://b/v1": 503}), clock=clock)
    out = r.route("/chat/completions", {"model": "qwen3-8b"})
    assert "http://a/v1" in out["choices"][0]["message"]["content"]       # retried on the other deployment
    r.route("/chat/completions", {"model": "qwen3-8b"})                 # second failure on b → cooldown
    b = [d for d in r.groups["qwen3-8b"] if d.api_base == "http://b/v1"][0]
    assert b.cooldowns == 1 and b.cooldown_until == clock.t + 120
    n = len(calls)
    r.route("/chat/completions", {"model": "qwen3-8b"})
    assert len(calls) == n + 1 and calls[-1][0] == "http://a/v1"          # b skipped while cooling down
    clock.t += 121
    r.send = ok_sender(calls)
    r.route("/chat/completions", {"model": "qwen3-8b"})
    assert calls[-1][0] == "http://b/v1"                                  # back after cooldown_time


def test_rate_limit_budget_and_fallback_chain():
    calls = []
    r = Router(cfg(allowed_fails=100), ok_sender(calls, {"http://c/v1": 429}), seed=0)
    out = r.route("/chat/completions", {"model": "r1-awq"})
    assert out["model"] == "qwen3-8b"
    assert sum(1 for a, _, _ in calls if a == "http://c/v1") == 6          # 1 try + 5 RateLimitErrorRetries
    assert r.counters["fallbacks_total"] == 1
    calls.clear()
    r = Router(cfg(), ok_sender(calls, {"http://c/v1": 429}), seed=0)
    assert r.route("/chat/completions", {"model": "r1-awq"})["model"] == "qwen3-8b"
    assert sum(1 for a, _, _ in calls if a == "http://c/v1") == 2          # cooled down after allowed_fails


def test_context_window_fallback_and_plain_400():
    calls = []
    r = Router(cfg(), ok_sender(calls, {"http://a/v1": 400, "http://b/v1": 400}), seed=0)
    out = r.route("/chat/completions", {"model": "qwen3-8b"})
    assert out["model"] == "long-ctx"
    r2 = Router(cfg(), ok_sender([], {"http://c/v1": 400}), seed=0)
    with pytest.raises(UpstreamError) as ei:                            # non-context 400 on r1 → context
        r2.route("/chat/completions", {"model": "r1-awq"})                #   fallback map has no r1 entry
    assert ei.value.status == 400


def test_app_guardrail_models_metrics():
    calls = []
    c = cfg()
    c["guardrails"] = [{"guardrail_name": "g", "litellm_params": {"guardrail": "openai_moderation",
                                                                   "mode": "pre_call", "api_base": "http://guard/v1"}}]

    def send(dep, path, body):
        if path == "/moderations":
            return {"results": [{"flagged": "bomb" in body["input"]}]}
        return ok_sender(calls)(dep, path, body)
    app = create_router_app(Router(c, send, seed=0))
    cl = TestClient(app)
    assert [m["id"] for m in cl.get("/v1/models").json()["data"]] == ["qwen3-8b", "r1-awq", "long-ctx"]
    r = cl.post("/v1/chat/completions", json={"model": "qwen3-8b", "messages": [{"role": "user", "content": "hello"}]})
    assert r.status_code == 200 and r.json()["model"] == "qwen3-8b"
    r = cl.post("/v1/chat/completions", json={"model": "qwen3-8b", "messages": [{"role": "user", "content": "a bomb"}]})
    assert r.status_code == 400 and r.json()["error"]["type"] == "guardrail_violation"
    assert cl.post("/v1/completions", json={"model": "nope", "prompt": "x"}).status_code == 404
    m = cl.get("/metrics").text
    assert "lipa_router_guard_blocked_total 1" in m and 'lipa_router_deployment_requests_total{group="qwen3-8b"' in m
    assert cl.get("/health").json()["status"] == "ok"


def test_repo_litellm_config_loads():
    import os
    path = os.path.join(os.path.dirname(__file__), "..", "deploy", "litellm", "config.yaml")
    r = Router(load_config(path), ok_sender([]))
    assert r.strategy == "least-busy" and len(r.groups["qwen3-8b"]) == 2
    assert r.fallbacks == {"deepseek-r1-qwen3-8b-awq": ["qwen3-8b"]} and r.guards


def test_max_parallel_requests_caps_in_flight():
    c = cfg("least-busy")
    for m in c["model_list"][:2]:
        m["litellm_params"]["max_parallel_requests"] = 1
    r = Router(c, ok_sender([]), seed=0)
    a, b = r.pick("qwen3-8b"), r.pick("qwen3-8b")
    assert {a.api_base, b.api_base} == {"http://a/v1", "http://b/v1"}
    with pytest.raises(UpstreamError) as ei:
        r.pick("qwen3-8b")
    assert ei.value.status == 429
    r._done(a, True, 0.01)
    assert r.pick("qwen3-8b") is a


# ----------------------------------------------------------------------------- prefix / load aware
def _prompt(sys_prompt, user):
    return {"model": "qwen3-8b", "messages": [{"role": "system", "content": sys_prompt},
                                              {"role": "user", "content": user}]}


def test_prefixaware_routes_shared_prefix_to_same_backend():
    calls = []
    r = Router(cfg("prefixaware"), ok_sender(calls), seed=1)
    doc = "RAG document about MI355X HBM3E. " * 40           # > several 256-char blocks
    first = r.route("/chat/completions", _prompt(doc, "q1"))
    owner = calls[-1][0]
    for i in range(6):
        r.route("/chat/completions", _prompt(doc, f"question {i}"))
        assert calls[-1][0] == owner
    assert r.counters["prefix_hits_total"] == 6 and first["model"] == "qwen3-8b"


def test_load_aware_prefix_uses_scraped_backend_load():
    """llm-d weights (pending 0.4, kv-cache 0.3, ttft 0.2, queue 0.1) over scraped /metrics; a warm
    prefix wins only while its backend is not much more loaded."""
    calls, clock = [], Clock()
    r = Router(cfg("load_aware_prefix", prefix_weight=0.3), ok_sender(calls), clock=clock, seed=0)
    load = {"http://a/v1": dict(pending_requests=8, gpu_cache_usage=0.9, ttft_ms=900, queue_time_ms=300),
            "http://b/v1": dict(pending_requests=0, gpu_cache_usage=0.1, ttft_ms=100, queue_time_ms=0)}
    r.scraper = lambda d: load[d.api_base]
    r.route("/chat/completions", _prompt("x" * 600, "hi"))
    assert calls[-1][0] == "http://b/v1"                       # idle backend
    # b becomes busy, a idle: the shared prefix (owned by b) is outweighed by b's load
    load["http://a/v1"], load["http://b/v1"] = load["http://b/v1"], load["http://a/v1"]
    clock.t += 10
    r.route("/chat/completions", _prompt("x" * 600, "again"))
    assert calls[-1][0] == "http://a/v1"
    # equal load: prefix affinity decides (a now owns the prefix)
    load["http://b/v1"] = dict(load["http://a/v1"])
    clock.t += 10
    r.route("/chat/completions", _prompt("x" * 600, "third"))
    assert calls[-1][0] == "http://a/v1"
    # a scrape failure twice in a row marks a backend down
    def flaky(d):
        if d.api_base == "http://a/v1":
            raise OSError("down")
        return load[d.api_base]
    r.scraper = flaky
    for _ in range(2):
        clock.t += 10
        r.refresh_stats()
    r.route("/chat/completions", _prompt("x" * 600, "fourth"))
    assert calls[-1][0] == "http://b/v1"


def test_backend_load_parses_lipa_and_vllm_metrics():
    from llm_in_practise_amd.infer.router import backend_load, parse_prometheus
    lipa = ("lipa_num_requests_waiting 3\nlipa_gpu_cache_usage_perc 0.25\n"
            "lipa_time_to_first_token_seconds_sum 2.0\nlipa_time_to_first_token_seconds_count 4\n"
            "lipa_queue_time_seconds 0.05\n")
    assert backend_load(parse_prometheus(lipa)) == {"pending_requests": 3.0, "gpu_cache_usage": 0.25,
                                                     "ttft_ms": 500.0, "queue_time_ms": 50.0}
    vllm = 'vllm:num_requests_waiting{model_name="q"} 2\nvllm:gpu_cache_usage_perc{model_name="q"} 0.5\n'
    assert backend_load(parse_prometheus(vllm))["pending_requests"] == 2.0


def test_app_serves_requests_concurrently():
    """Upstream calls run in the threadpool: two slow requests overlap (in_flight reaches 2)."""
    import threading
    import time as _t
    peak, lock, cur = [0], threading.Lock(), [0]

    def slow(dep, path, body):
        with lock:
            cur[0] += 1
            peak[0] = max(peak[0], cur[0])
        _t.sleep(0.3)
        with lock:
            cur[0] -= 1
        return {"choices": [], "model": body["model"]}
    r = Router(cfg("least-busy"), slow, seed=0)
    app = create_router_app(r, scrape=False)
    import asyncio
    import httpx

    async def go():
        transport = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=transport, base_url="http://t") as c:
            t0 = _t.time()
            await asyncio.gather(*[c.post("/v1/chat/completions", json={"model": "qwen3-8b", "messages": []})
                                   for _ in range(2)])
            return _t.time() - t0
    dt = asyncio.run(go())
    assert peak[0] == 2 and dt < 0.55


def test_kubernetes_headless_service_discovery():
    """router_settings.discovery: the pod IPs behind a headless Service become the group's
    deployments, re-resolved on an interval (pods joining / leaving)."""
    from llm_in_practise_amd.infer.router import Router, resolve_service
    assert resolve_service("localhost", 8000) == ["127.0.0.1"]
    t = [0.0]
    ips = [["10.0.0.1", "10.0.0.2"]]
    sent = []

    def send(dep, path, body):
        sent.append(dep.api_base)
        return {"choices": [{"text": "x"}]}

    cfg = {"model_list": [], "router_settings": {"routing_strategy": "least-busy", "discovery": [
        {"model_name": "qwen3-8b", "service": "lipa-headless.llm-inference.svc", "port": 8000, "interval": 10}]}}
    r = Router(cfg, send=send, clock=lambda: t[0], seed=0, resolver=lambda host, port: list(ips[0]))
    assert sorted(d.api_base for d in r.groups["qwen3-8b"]) == ["http://10.0.0.1:8000/v1", "http://10.0.0.2:8000/v1"]
    r.route("/completions", {"model": "qwen3-8b", "prompt": "hi"})
    first = r.groups["qwen3-8b"]
    ips[0] = ["10.0.0.2", "10.0.0.3"]
    t[0] = 5.0                               # inside the interval: no re-resolve
    r.route("/completions", {"model": "qwen3-8b", "prompt": "hi"})
    assert len(r.groups["qwen3-8b"]) == 2 and r.groups["qwen3-8b"][0].api_base == first[0].api_base
    t[0] = 11.0
    r.route("/completions", {"model": "qwen3-8b", "prompt": "hi"})
    bases = sorted(d.api_base for d in r.groups["qwen3-8b"])
    assert bases == ["http://10.0.0.2:8000/v1", "http://10.0.0.3:8000/v1"]
    assert sent[-1] in bases
