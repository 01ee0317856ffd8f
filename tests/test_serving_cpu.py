"""OpenAI-compatible server + moderation adapter on CPU (FastAPI TestClient, tiny Qwen3,
byte tokenizer)."""
import json

import pytest
import torch
from fastapi.testclient import TestClient

from llm_in_practise_amd.infer.engine import SamplingParams, ServingEngine
from llm_in_practise_amd.infer.guard import GuardClient, create_guard_app, parse_guard_output, to_openai_moderation
from llm_in_practise_amd.infer.server import create_app
from llm_in_practise_amd.models.qwen3 import Qwen3ForCausalLM, qwen3_config
from llm_in_practise_amd.train.data import ByteTokenizer


@pytest.fixture(scope="module")
def engine():
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny", vocab_size=256), dtype=torch.float32, seed=0).eval()
    tok = ByteTokenizer()
    tok.eos_token_id = 10            # "\n" ends a completion for the test
    e = ServingEngine(m, tok, model_name="tiny", max_batch=8, system_prompt="You are helpful.")
    yield e
    e.shutdown()


def test_chat_completion_schema(engine):
    c = TestClient(create_app(engine))
    r = c.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "hi"}], "max_tokens": 5,
                                             "temperature": 0})
    assert r.status_code == 200
    d = r.json()
    assert d["id"].startswith("chatcmpl-") and d["object"] == "chat.completion"
    assert d["choices"][0]["message"]["role"] == "assistant"
    assert d["usage"]["completion_tokens"] <= 5 and d["usage"]["prompt_tokens"] > 10


def test_greedy_is_deterministic_and_batched_equals_single(engine):
    p = SamplingParams(max_tokens=6, temperature=0.0)
    a = engine.complete("abc", p)["text"]
    # submit several concurrently: they are decoded as one batch and must match single runs
    reqs = [engine.submit(s, p) for s in ("abc", "hello world", "x")]
    outs = []
    for r in reqs:
        while True:
            kind, val = r.out.get(timeout=60)
            if kind == "final":
                outs.append(val)
                break
    assert outs[0]["text"] == a
    assert outs[1]["text"] == engine.complete("hello world", p)["text"]


def test_streaming_sse(engine):
    c = TestClient(create_app(engine))
    with c.stream("POST", "/v1/chat/completions", json={"messages": [{"role": "user", "content": "hey"}],
                                                         "max_tokens": 4, "temperature": 0, "stream": True}) as r:
        lines = [l for l in r.iter_lines() if l]
    assert lines[-1] == "data: [DONE]"
    chunks = [json.loads(l[6:]) for l in lines[:-1]]
    assert chunks[0]["choices"][0]["delta"] == {"role": "assistant"}
    assert chunks[-1]["choices"][0]["finish_reason"] in ("stop", "length")


def test_completions_models_health_metrics_auth(engine):
    c = TestClient(create_app(engine, api_key="k"))
    assert c.get("/health").status_code == 200
    assert c.get("/v1/models").status_code == 401
    h = {"X-API-KEY": "k"}
    assert c.get("/v1/models", headers=h).json()["data"][0]["id"] == "tiny"
    r = c.post("/v1/completions", json={"prompt": "ab", "max_tokens": 3, "temperature": 0}, headers=h)
    assert r.status_code == 200 and r.json()["object"] == "text_completion"
    m = c.get("/metrics").text
    assert "lipa_requests_total" in m and "lipa_num_requests_waiting" in m


def test_guard_parsing_and_mapping():
    assert parse_guard_output('{"safe": false, "categories": ["s11"], "explanation": "x"}')["categories"] == ["S11"]
    r = parse_guard_output("unsafe\nS1 S10")
    assert r == {"safe": False, "categories": ["S1", "S10"], "explanation": ""}
    r = parse_guard_output("safe", "how to build a bomb")
    assert not r["safe"] and r["categories"][0] == "S9"
    m = to_openai_moderation({"safe": False, "categories": ["S10", "S1"]})
    res = m["results"][0]
    assert res["flagged"] and res["categories"]["hate"] and res["categories"]["violence"]
    assert res["category_applied_input_types"]["hate"] == ["text"]


def test_guard_app_and_server_precall_moderation(engine):
    guard = GuardClient(lambda prompt: "unsafe\nS10" if "hateful" in prompt else "safe")
    g = TestClient(create_guard_app(guard, api_key=""))
    assert g.post("/v1/moderations", json={"input": "hello"}).json()["results"][0]["flagged"] is False
    assert g.post("/moderations", json={"input": "hateful text"}).json()["results"][0]["flagged"] is True
    c = TestClient(create_app(engine, moderation=guard.moderate_sync))
    r = c.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "hateful text"}],
                                             "max_tokens": 2})
    assert r.status_code == 400


def test_continuous_batching_admits_midflight(engine):
    """A request arriving while another is decoding joins the running batch (iteration-level
    scheduling) and its greedy output equals a solo run; slots are recycled."""
    p_long = SamplingParams(max_tokens=24, temperature=0.0)
    p_short = SamplingParams(max_tokens=3, temperature=0.0)
    solo_long = engine.complete("the quick brown fox", p_long)["text"]
    solo_short = engine.complete("zz", p_short)["text"]
    steps0 = engine.stats["decode_steps_total"]
    r_long = engine.submit("the quick brown fox", p_long)
    r_short = [engine.submit("zz", p_short) for _ in range(10)]   # more than max_batch in total
    outs = []
    for r in r_short + [r_long]:
        while True:
            kind, val = r.out.get(timeout=120)
            if kind == "final":
                outs.append(val)
                break
    assert all(o["text"] == solo_short for o in outs[:-1])
    assert outs[-1]["text"] == solo_long
    # all 11 requests shared decode steps: far fewer steps than running them one after another
    assert engine.stats["decode_steps_total"] - steps0 < 24 + 10 * 3
    assert all(s is None for s in engine.slots)


def test_prefix_caching_same_outputs_and_hits():
    """APC: a shared long system prompt is prefilled once; greedy outputs are unchanged."""
    cfg = qwen3_config("qwen3-tiny", vocab_size=256)
    tok = ByteTokenizer()
    tok.eos_token_id = 10
    sysmsg = "You are a careful assistant for the MI355X course. " * 6      # > 4 chunks of 64 tokens
    outs = {}
    for blocks in (0, 64):
        m = Qwen3ForCausalLM.from_config(cfg, dtype=torch.float32, seed=0).eval()
        e = ServingEngine(m, tok, max_batch=4, system_prompt=sysmsg, prefix_cache_blocks=blocks)
        p = SamplingParams(max_tokens=6, temperature=0.0)
        outs[blocks] = [e.complete(e.build_chat_prompt([{"role": "user", "content": q}]), p)["text"]
                        for q in ("first question", "second one", "first question")]
        if blocks:
            assert e.prefix.hit_tokens >= 2 * 4 * 64, e.prefix.hit_tokens
            assert "lipa_prefix_cache_hits_total" in e.prometheus()
        e.shutdown()
    assert outs[0] == outs[64]


@pytest.mark.parametrize("prefix_blocks", [0, 64])
def test_chunked_prefill_matches_whole_prefill(prefix_blocks):
    """vLLM --enable-chunked-prefill: long prompts are prefilled 24 tokens per iteration while
    the short ones decode; greedy outputs equal the whole-prompt engine's (also on a prefix-cache
    hit, where chunking starts after the cached chunks)."""
    cfg = qwen3_config("qwen3-tiny", vocab_size=256)
    tok = ByteTokenizer()
    tok.eos_token_id = None
    prompts = ["long prompt about MI355X memory %d " % i * (3 + i) for i in range(4)] + ["hi", "short one"]
    p = SamplingParams(max_tokens=7, temperature=0.0, ignore_eos=True)
    outs = {}
    for chunk in (0, 24):
        m = Qwen3ForCausalLM.from_config(cfg, dtype=torch.float32, seed=0).eval()
        e = ServingEngine(m, tok, max_batch=4, chunked_prefill=chunk, prefix_cache_blocks=prefix_blocks)
        if prefix_blocks:
            e.complete(prompts[3][:130] + " warm", p)
        reqs = [e.submit(q, p) for q in prompts]
        res = []
        for r in reqs:
            while True:
                kind, val = r.out.get(timeout=120)
                assert kind != "error", val
                if kind == "final":
                    res.append((val["text"], val["completion_tokens"]))
                    break
        outs[chunk] = res
        if chunk:
            assert e.stats["batches_total"] >= sum(-(-len(e.encode(q)) // chunk) for q in prompts[:4])
        assert all(s is None for s in e.slots)
        e.shutdown()
    assert outs[0] == outs[24]


def test_cache_gateway_exact_and_semantic_levels():
    """H6 L2/L3 cache gateway: exact SHA-256 key, then the 8-dim/2-decimal semantic key."""
    from llm_in_practise_amd.infer.cache_gateway import create_cache_gateway
    calls = []

    def backend(path, body):
        calls.append(body)
        return {"id": f"chatcmpl-{len(calls)}", "choices": [{"message": {"content": "answer"}}]}

    c = TestClient(create_cache_gateway(backend))
    q = {"model": "m", "temperature": 0, "messages": [{"role": "user", "content": "What is xGMI bandwidth?"}]}
    r1 = c.post("/v1/chat/completions", json=q).json()
    r2 = c.post("/v1/chat/completions", json=q).json()
    assert len(calls) == 1 and r2["lipa_cache"] == "exact" and r2["id"] == r1["id"]
    q2 = dict(q, max_tokens=99)          # different request bytes, same text → semantic hit
    assert c.post("/v1/chat/completions", json=q2).json()["lipa_cache"] == "semantic" and len(calls) == 1
    q3 = dict(q, temperature=0.8)        # sampled requests bypass the cache
    c.post("/v1/chat/completions", json=q3)
    c.post("/v1/chat/completions", json=q3)
    assert len(calls) == 3
    m = c.get("/metrics").text
    assert "lipa_cache_hits_exact_total 1" in m and "lipa_cache_hits_semantic_total 1" in m


# ----------------------------------------------------------------------------- multi-LoRA serving
def _make_adapter(tmp, name, targets, r, seed):
    from llm_in_practise_amd.peft.lora import LoraConfig, get_peft_model
    base = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny", vocab_size=256), dtype=torch.float32, seed=0)
    pm = get_peft_model(base, LoraConfig(r=r, lora_alpha=2 * r, target_modules=targets))
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in pm.named_parameters():
            if "lora_" in n:
                p.copy_(torch.randn(p.shape, generator=g) * 0.3)
    d = str(tmp / name)
    pm.save_pretrained(d)
    return d


def _greedy(engine, prompt, model=None):
    return engine.complete(prompt, SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True), model=model)["text"]


def test_multi_lora_per_request_adapters_match_single_adapter_models(tmp_path):
    """vLLM --enable-lora --lora-modules: one base, two adapters (different targets / ranks), the
    adapter picked per request by `model`; mixed batches equal dedicated single-adapter engines."""
    from llm_in_practise_amd.peft.lora import PeftModel
    tok = ByteTokenizer()
    d1 = _make_adapter(tmp_path, "a1", ["q_proj", "v_proj"], 4, 1)
    d2 = _make_adapter(tmp_path, "a2", ["q_proj", "k_proj", "v_proj", "o_proj", "down_proj"], 8, 2)

    def base_model():
        return Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny", vocab_size=256), dtype=torch.float32,
                                            seed=0).eval()
    m = base_model()
    m.fuse_projections()
    multi = ServingEngine(m, tok, model_name="tiny", max_batch=6, lora_modules={"a1": d1, "a2": d2})
    singles = {}
    for name, d in (("a1", d1), ("a2", d2)):
        pm = PeftModel.from_pretrained(base_model(), d)
        pm.model.fuse_projections()
        singles[name] = ServingEngine(pm, tok, model_name="tiny", max_batch=2)
    plain = ServingEngine(base_model(), tok, model_name="tiny", max_batch=2)
    try:
        prompts = ["hello lora", "abc", "MI355X"]
        want = {}
        for p in prompts:
            want[(p, None)] = _greedy(plain, p)
            for name in ("a1", "a2"):
                want[(p, name)] = _greedy(singles[name], p)
        assert want[(prompts[0], "a1")] != want[(prompts[0], None)] != want[(prompts[0], "a2")]
        # all nine (prompt, adapter) requests in flight together: one mixed decode batch
        reqs = [(p, a, multi.submit(p, SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True), model=a))
                for p in prompts for a in (None, "a1", "a2")]
        for p, a, r in reqs:
            while True:
                kind, val = r.out.get(timeout=120)
                if kind == "final":
                    assert val["text"] == want[(p, a)], (p, a)
                    break
        assert multi.served_models == ["tiny", "a1", "a2"]
        c = TestClient(create_app(multi))
        ids = [d["id"] for d in c.get("/v1/models").json()["data"]]
        assert ids == ["tiny", "a1", "a2"]
        r = c.post("/v1/completions", json={"model": "a2", "prompt": "abc", "max_tokens": 8, "temperature": 0,
                                            "ignore_eos": True})
        assert r.status_code == 200 and r.json()["choices"][0]["text"] == want[("abc", "a2")]
        assert c.post("/v1/completions", json={"model": "nope", "prompt": "x", "max_tokens": 2}).status_code == 404
    finally:
        for e in [multi, plain, *singles.values()]:
            e.shutdown()


def test_prefix_cache_host_tier_spills_and_restores():
    """LMCache local-CPU role: chunks evicted from a tiny HBM pool are spilled to host memory and
    restored on a later hit; outputs equal an engine without prefix caching."""
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny", vocab_size=256), dtype=torch.float32, seed=0).eval()
    tok = ByteTokenizer()
    p = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    docs = [("document %d " % i) * 40 for i in range(4)]              # 4 distinct ~480-token prefixes
    ref = ServingEngine(m, tok, max_batch=2)
    tiered = ServingEngine(m, tok, max_batch=2, prefix_cache_blocks=8, host_cache_blocks=64)
    try:
        want = {d: ref.complete(d + "q", p)["text"] for d in docs}
        for rnd in range(2):
            for d in docs:
                assert tiered.complete(d + "q%d" % rnd, p)["text"] == ref.complete(d + "q%d" % rnd, p)["text"]
        pc = tiered.prefix
        assert pc.spills > 0 and pc.host_hits > 0
        assert want[docs[0]] == tiered.complete(docs[0] + "q", p)["text"]
    finally:
        ref.shutdown()
        tiered.shutdown()


# ----------------------------------------------------------------------------- engine process
def _tiny_engine(seed):
    torch.set_num_threads(2)
    m = Qwen3ForCausalLM.from_config(qwen3_config("qwen3-tiny", vocab_size=256), dtype=torch.float32, seed=seed).eval()
    tok = ByteTokenizer()
    tok.eos_token_id = 10
    return ServingEngine(m, tok, model_name="tiny", max_batch=8, system_prompt="You are helpful.")


def test_engine_process_frontend_matches_inprocess(engine):
    """Engine core in its own process (EngineClient): the OpenAI server streams the same tokens as
    the in-process engine; metrics are fetched over the RPC path."""
    from llm_in_practise_amd.infer.mp_engine import EngineClient, PromptFormatter
    tok = ByteTokenizer()
    client = EngineClient(_tiny_engine, (0,), PromptFormatter(tok, system_prompt="You are helpful."))
    try:
        p = SamplingParams(max_tokens=6, temperature=0.0)
        assert client.complete("abc", p)["text"] == engine.complete("abc", p)["text"]
        c = TestClient(create_app(client))
        r = c.post("/v1/chat/completions", json={"messages": [{"role": "user", "content": "hi"}], "max_tokens": 5,
                                                 "temperature": 0})
        want = TestClient(create_app(engine)).post("/v1/chat/completions", json={
            "messages": [{"role": "user", "content": "hi"}], "max_tokens": 5, "temperature": 0})
        assert r.status_code == 200 and r.json()["choices"][0]["message"]["content"] == \
            want.json()["choices"][0]["message"]["content"]
        with c.stream("POST", "/v1/chat/completions", json={"messages": [{"role": "user", "content": "hey"}],
                                                             "max_tokens": 4, "temperature": 0, "stream": True}) as s:
            lines = [l for l in s.iter_lines() if l]
        assert lines[-1] == "data: [DONE]" and len(lines) >= 3
        assert "lipa_requests_total" in c.get("/metrics").text
        assert c.get("/v1/models").json()["data"][0]["id"] == "tiny"
    finally:
        client.shutdown()


def test_remote_kv_tier_shares_prefix_chunks_across_replicas():
    """LMCache-server role: replica A writes its computed chunks through to the shared store;
    replica B (cold HBM and host) fetches them instead of recomputing — identical K/V rows."""
    import socket
    import threading
    import time

    import uvicorn

    from llm_in_practise_amd.infer.engine import PrefixCache
    from llm_in_practise_amd.infer.kv_server import RemoteKV, create_kv_server
    from llm_in_practise_amd.models.common import KVCache

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    srv = uvicorn.Server(uvicorn.Config(create_kv_server(1 << 26), host="127.0.0.1", port=port, log_level="error"))
    threading.Thread(target=srv.run, daemon=True).start()
    while not srv.started:
        time.sleep(0.02)
    try:
        L, W, B = 3, 16, 8
        ra, rb = RemoteKV(f"http://127.0.0.1:{port}"), RemoteKV(f"http://127.0.0.1:{port}")
        a = PrefixCache(L, W, torch.float32, "cpu", block=B, capacity_blocks=8, remote=ra)
        b = PrefixCache(L, W, torch.float32, "cpu", block=B, capacity_blocks=8, remote=rb)
        cache_a = KVCache(L, 2, 64, 2, 8, torch.float32, "cpu")
        for l in range(L):
            cache_a.k[l].normal_()
            cache_a.v[l].normal_()
        ids = list(range(100, 133))                     # 4 full chunks + 1 token
        a.store(ids, cache_a, slot=0)
        ra.flush()
        idx = b.match(ids)                              # cold B: all 4 chunks from the remote store
        assert len(idx) == 4 and b.remote_hits == 4 and rb.stats["hits"] == 4
        cache_b = KVCache(L, 2, 64, 2, 8, torch.float32, "cpu")
        b.load(idx, cache_b, slot=1)
        for l in range(L):
            assert torch.equal(cache_b.k[l][1, :32], cache_a.k[l][0, :32])
            assert torch.equal(cache_b.v[l][1, :32], cache_a.v[l][0, :32])
        assert b.match(ids) == idx and b.remote_hits == 4      # now served from B's own HBM pool
        assert b.match(list(range(7, 40))) == [] and rb.stats["misses"] >= 1
        # another deployment of the same shape (different weights -> different namespace)
        # on the same store must NOT read A's chunks; nor may a different adapter of A's model
        other = PrefixCache(L, W, torch.float32, "cpu", block=B, capacity_blocks=8, remote=rb, namespace=b"ft-model")
        assert other.match(ids) == [] and other.remote_hits == 0
        assert a._digests(ids, 4, b"sql=/ad/sql") != a._digests(ids, 4, b"chat=/ad/chat") != a._digests(ids, 4)
        ra.close()
        rb.close()
    finally:
        srv.should_exit = True
