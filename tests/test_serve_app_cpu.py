"""Ray-Serve-style replica controller (infer/serve_app.py): config parsing of the reference's
serve_deploy_examples, the autoscaling policy with up/down delays, and the HTTP proxy's
routing / back-pressure / scale-up / drain against in-process fake replicas."""
import asyncio
import os
import socket
import threading
import time

import httpx
import pytest
import uvicorn
from fastapi import FastAPI

from llm_in_practise_amd.infer.serve_app import (AppConfig, AutoscalingConfig, Autoscaler, Replica, ServeController,
                                                 create_serve_proxy, load_serve_config)

REF = "/root/reference/Deployment/Ray/serve_deploy_examples"


def test_parse_reference_configs():
    if not os.path.isdir(REF):
        pytest.skip("reference checkout not present")
    a = load_serve_config(os.path.join(REF, "qwen3_app_autoscaling.yaml"))[0]
    assert (a.autoscaling.min_replicas, a.autoscaling.max_replicas, a.autoscaling.target_ongoing_requests) == (1, 2, 5)
    assert (a.autoscaling.upscale_delay, a.autoscaling.downscale_delay, a.max_ongoing_requests) == (5.0, 30.0, 64)
    two = load_serve_config(os.path.join(REF, "serve_app_two_models.yaml"))
    assert [x.route_prefix for x in two] == ["/app1", "/app2"]
    assert two[1].engine_kwargs["quantization"] == "awq" and two[1].autoscaling.downscale_delay == 300.0
    pp = load_serve_config(os.path.join(REF, "qwen3_app_pipeline_parallel.yaml"))[0]
    assert pp.gpus_per_replica == 2


def test_autoscaler_policy_delays():
    t = [0.0]
    a = Autoscaler(AutoscalingConfig(min_replicas=1, max_replicas=4, target_ongoing_requests=5,
                                     upscale_delay=5, downscale_delay=30), clock=lambda: t[0])
    assert a.desired(0) == 1 and a.desired(11) == 3 and a.desired(100) == 4
    assert a.decide(12, 1) == 1            # wants 3: starts the upscale delay
    t[0] = 4.9
    assert a.decide(12, 1) == 1
    t[0] = 5.0
    assert a.decide(12, 1) == 3            # held for upscale_delay
    assert a.decide(3, 3) == 3             # wants 1: downscale delay starts
    t[0] = 20
    assert a.decide(3, 3) == 3
    assert a.decide(20, 3) == 3            # load back: pending downscale cancelled
    t[0] = 21
    assert a.decide(3, 3) == 3             # restarts the 30 s window
    t[0] = 50
    assert a.decide(3, 3) == 3
    t[0] = 51
    assert a.decide(3, 3) == 1


def _fake_backend(delay: float):
    app = FastAPI()
    seen = {"n": 0, "max_conc": 0, "cur": 0}

    @app.get("/health")
    async def health():
        return {"ok": True}

    @app.post("/v1/completions")
    async def comp(body: dict):
        seen["n"] += 1
        seen["cur"] += 1
        seen["max_conc"] = max(seen["max_conc"], seen["cur"])
        await asyncio.sleep(delay)
        seen["cur"] -= 1
        return {"choices": [{"text": "ok"}], "model": body.get("model")}

    return app, seen


def _serve(app):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="error"))
    th = threading.Thread(target=srv.run, daemon=True)
    th.start()
    for _ in range(200):
        if srv.started:
            break
        time.sleep(0.02)
    return f"http://127.0.0.1:{port}", srv


def test_proxy_routes_backpressure_scales_and_drains():
    backends = []

    def factory(cfg, gpus):
        app, seen = _fake_backend(0.3)
        url, srv = _serve(app)
        backends.append((seen, srv))
        return Replica(url, None, gpus)

    cfg = AppConfig(name="qwen3", route_prefix="/app1", model_id="qwen3", model_source="x",
                    autoscaling=AutoscalingConfig(min_replicas=1, max_replicas=3, target_ongoing_requests=2,
                                                  upscale_delay=0.0, downscale_delay=0.5),
                    max_ongoing_requests=2, max_queued_requests=4)
    ctl = ServeController([cfg], factory, gpus=[0, 1, 2], control_interval=0.1)
    proxy_url, psrv = _serve(create_serve_proxy(ctl))
    ctl.start()
    try:
        r = httpx.get(proxy_url + "/-/routes")
        assert r.json() == {"/app1": "qwen3"}

        async def burst(n):
            async with httpx.AsyncClient(timeout=30) as c:
                return await asyncio.gather(*[c.post(proxy_url + "/app1/v1/completions",
                                                     json={"model": "qwen3", "prompt": "hi"}) for _ in range(n)])

        # 1 replica x max_ongoing 2 + queue 4 -> the 7th..10th concurrent requests are rejected (503)
        res = asyncio.run(burst(10))
        codes = sorted(x.status_code for x in res)
        assert codes.count(200) >= 6 and 503 in codes
        assert backends[0][0]["max_conc"] <= 2          # max_ongoing_requests enforced per replica
        # the burst raised ongoing above target -> scaled up (no upscale delay) to max 3 replicas
        deadline = time.time() + 5
        while len(ctl.apps["qwen3"].replicas) < 3 and time.time() < deadline:
            asyncio.run(burst(6))
        assert len(ctl.apps["qwen3"].replicas) == 3
        assert ctl.free_gpus == []
        res = asyncio.run(burst(6))
        assert all(x.status_code == 200 for x in res)
        assert sum(1 for seen, _ in backends if seen["n"] > 0) >= 2   # spread over replicas
        # idle -> drained back to min_replicas after downscale_delay, GPUs returned
        deadline = time.time() + 10
        while len(ctl.apps["qwen3"].replicas) > 1 and time.time() < deadline:
            time.sleep(0.1)
        assert len(ctl.apps["qwen3"].replicas) == 1 and len(ctl.free_gpus) == 2
        m = httpx.get(proxy_url + "/metrics").text
        assert 'lipa_serve_replicas{app="qwen3"} 1' in m and "lipa_serve_rejected_total" in m
        assert httpx.get(proxy_url + "/nope/v1/completions").status_code == 404
    finally:
        ctl.shutdown()
        psrv.should_exit = True
        for _, srv in backends:
            srv.should_exit = True
