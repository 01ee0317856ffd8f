#!/usr/bin/env python3
"""Serving benchmark against any OpenAI-compatible endpoint (the reference's
``vllm bench serve --dataset-name sharegpt --request-rate inf --max-concurrency C --ignore-eos
--sharegpt-output-len 256`` plus ``generate_mixed_dataset.py`` / ``extract_metrics.py``,
``LLM_on_Kubernetes/Inference_Platfrom/README.md:1177-1493``).

    python scripts/bench_serve.py --url http://127.0.0.1:8000 --concurrency 8 16 32 --num-prompts 128
    python scripts/bench_serve.py --inprocess random:qwen3-small --concurrency 4     # no server needed

Dataset: ``--dataset mixed`` = 70 % short chat / 30 % long RAG-style prompts (synthetic text,
no network), or a ShareGPT-format JSON file.  Metrics per concurrency (streamed requests):
mean / p99 TTFT, mean / p99 ITL, request throughput, output tokens/s — the columns of the
reference's results table (``README.md:1504-1511``) — plus per-request tokens/s (mean / p50), the
custom event of the reference's ``Deployment/Ray/scripts/locustfile-TPS.py:21-41``.  Token counts use streamed deltas (one
delta ≈ one token for the OpenAI stream), or the server's ``usage`` when not streaming.
"""
import argparse
import asyncio
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def mixed_dataset(n: int, seed: int = 0):
    rnd = random.Random(seed)
    words = ("cluster gpu kernel memory latency throughput scheduler token model serving cache network storage "
             "pod node replica request batch prompt context quantization adapter").split()
    out = []
    for i in range(n):
        if rnd.random() < 0.7:
            q = " ".join(rnd.choice(words) for _ in range(rnd.randint(8, 40)))
            out.append([{"role": "user", "content": f"Explain briefly: {q}?"}])
        else:
            doc = " ".join(rnd.choice(words) for _ in range(rnd.randint(600, 1500)))
            out.append([{"role": "system", "content": "Answer using the document."},
                        {"role": "user", "content": f"Document:\n{doc}\n\nQuestion: summarise the document."}])
    return out


def sharegpt(path: str, n: int):
    data = json.load(open(path))
    out = []
    for conv in data:
        turns = conv.get("conversations", [])
        if turns:
            out.append([{"role": "user", "content": turns[0]["value"]}])
        if len(out) >= n:
            break
    return out


def pct(xs, p):
    if not xs:
        return float("nan")
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(round(p / 100 * (len(xs) - 1))))]


async def one_request(client, url, model, msgs, max_tokens):
    t0 = time.perf_counter()
    ttft, last, itl, n = None, None, [], 0
    body = {"model": model, "messages": msgs, "max_tokens": max_tokens, "stream": True, "temperature": 0.0,
            "ignore_eos": True}
    async with client.stream("POST", url + "/v1/chat/completions", json=body, timeout=600) as r:
        async for line in r.aiter_lines():
            if not line.startswith("data: ") or line == "data: [DONE]":
                continue
            d = json.loads(line[6:])["choices"][0].get("delta", {})
            if d.get("content"):
                now = time.perf_counter()
                if ttft is None:
                    ttft = now - t0
                else:
                    itl.append(now - last)
                last = now
                n += 1
    return {"ttft": ttft or (time.perf_counter() - t0), "itl": itl, "out_tokens": n, "e2e": time.perf_counter() - t0}


async def _run_raw(url, model, prompts, conc, max_tokens):
    import httpx
    sem = asyncio.Semaphore(conc)
    limits = httpx.Limits(max_connections=None, max_keepalive_connections=None)
    async with httpx.AsyncClient(limits=limits) as client:
        async def task(m):
            async with sem:
                return await one_request(client, url, model, m, max_tokens)
        t0 = time.perf_counter()
        res = await asyncio.gather(*[task(m) for m in prompts])
        return res, time.perf_counter() - t0


def _proc_level(args):
    url, model, prompts, conc, max_tokens, start_at = args
    while time.time() < start_at:            # every client process starts together
        time.sleep(0.001)
    return asyncio.run(_run_raw(url, model, prompts, conc, max_tokens))


def run_level_procs(url, model, prompts, conc, max_tokens, procs):
    """The load generator itself split over ``procs`` processes (one Python event loop parsing
    10k+ SSE events/s saturates and inflates TTFT / ITL): prompts and concurrency are divided,
    the per-request samples merged, duration = the slowest process."""
    import multiprocessing as mp
    parts = [prompts[i::procs] for i in range(procs)]
    concs = [conc // procs + (1 if i < conc % procs else 0) for i in range(procs)]
    start = time.time() + 1.0
    with mp.get_context("spawn").Pool(procs) as pool:
        outs = pool.map(_proc_level, [(url, model, p, max(1, c), max_tokens, start) for p, c in zip(parts, concs)])
    res = [r for rs, _ in outs for r in rs]
    return _summary(res, max(d for _, d in outs), conc)


def _summary(res, dur, conc):
    ttft = [r["ttft"] * 1e3 for r in res]
    itl = [x * 1e3 for r in res for x in r["itl"]]
    toks = sum(r["out_tokens"] for r in res)
    per_req = [r["out_tokens"] / r["e2e"] for r in res if r["e2e"] > 0]
    return {"concurrency": conc, "requests": len(res), "duration_s": round(dur, 3),
            "mean_ttft_ms": round(statistics.mean(ttft), 2), "p99_ttft_ms": round(pct(ttft, 99), 2),
            "mean_itl_ms": round(statistics.mean(itl), 2) if itl else None,
            "p99_itl_ms": round(pct(itl, 99), 2) if itl else None,
            "req_per_s": round(len(res) / dur, 3), "output_tok_per_s": round(toks / dur, 1),
            "mean_request_tok_per_s": round(statistics.mean(per_req), 2) if per_req else None,
            "p50_request_tok_per_s": round(statistics.median(per_req), 2) if per_req else None}


async def run_level(url, model, prompts, conc, max_tokens):
    import httpx
    sem = asyncio.Semaphore(conc)
    # no client-side cap: httpx defaults to 100 pooled connections, which would silently limit
    # concurrency 128 / 256 and show up as TTFT
    limits = httpx.Limits(max_connections=None, max_keepalive_connections=None)
    async with httpx.AsyncClient(limits=limits) as client:
        async def task(m):
            async with sem:
                return await one_request(client, url, model, m, max_tokens)
        t0 = time.perf_counter()
        res = await asyncio.gather(*[task(m) for m in prompts])
        dur = time.perf_counter() - t0
    ttft = [r["ttft"] * 1e3 for r in res]
    itl = [x * 1e3 for r in res for x in r["itl"]]
    toks = sum(r["out_tokens"] for r in res)
    # the reference's locustfile-TPS.py custom event: per-request output tokens / end-to-end latency
    per_req = [r["out_tokens"] / r["e2e"] for r in res if r["e2e"] > 0]
    return {"concurrency": conc, "requests": len(res), "duration_s": round(dur, 3),
            "mean_ttft_ms": round(statistics.mean(ttft), 2), "p99_ttft_ms": round(pct(ttft, 99), 2),
            "mean_itl_ms": round(statistics.mean(itl), 2) if itl else None,
            "p99_itl_ms": round(pct(itl, 99), 2) if itl else None,
            "req_per_s": round(len(res) / dur, 3), "output_tok_per_s": round(toks / dur, 1),
            "mean_request_tok_per_s": round(statistics.mean(per_req), 2) if per_req else None,
            "p50_request_tok_per_s": round(statistics.median(per_req), 2) if per_req else None}


class _SyntheticTokenizer:
    """Random-init models emit ids over the whole vocabulary: encode prompts as bytes, decode each
    id to exactly one printable character so one streamed delta = one token."""
    eos_token_id = None
    pad_token_id = 0

    def encode(self, text, add_special_tokens=False):
        return list(text.encode("utf-8"))

    def decode(self, ids, skip_special_tokens=True):
        return "".join(chr(0x4E00 + int(i) % 20000) for i in ids)


def _make_engine(spec: str, max_batch: int, max_model_len: int | None):
    from llm_in_practise_amd.cli.main import _load_for_inference
    from llm_in_practise_amd.infer.engine import ServingEngine
    m = _load_for_inference(spec)
    return ServingEngine(m, _SyntheticTokenizer(), model_name=spec, max_batch=max_batch, chat_template="chatml",
                         max_model_len=max_model_len)


def start_inprocess(spec: str, port: int, max_batch: int = 64, max_model_len: int | None = None,
                    engine_process: bool = False):
    """Launch our server in a background thread with a random-init model (synthetic tokenizer);
    ``engine_process``: the engine runs in its own process (infer/mp_engine.py)."""
    import threading

    import uvicorn

    from llm_in_practise_amd.infer.server import create_app
    if engine_process:
        from llm_in_practise_amd.infer.mp_engine import EngineClient, PromptFormatter
        eng = EngineClient(_make_engine, (spec, max_batch, max_model_len),
                           PromptFormatter(_SyntheticTokenizer(), chat_template="chatml"))
    else:
        eng = _make_engine(spec, max_batch, max_model_len)
    cfg = uvicorn.Config(create_app(eng), host="127.0.0.1", port=port, log_level="warning")
    th = threading.Thread(target=uvicorn.Server(cfg).run, daemon=True)
    th.start()
    time.sleep(2.0)
    return f"http://127.0.0.1:{port}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default=None)
    ap.add_argument("--inprocess", default=None, help="e.g. random:qwen3-small (starts our server in-process)")
    ap.add_argument("--port", type=int, default=8765)
    ap.add_argument("--model", default="default")
    ap.add_argument("--dataset", default="mixed")
    ap.add_argument("--num-prompts", type=int, default=64)
    ap.add_argument("--max-tokens", type=int, default=256)
    ap.add_argument("--concurrency", type=int, nargs="+", default=[8])
    ap.add_argument("--out", default=None)
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--max-model-len", type=int, default=None)
    ap.add_argument("--spawn", action="store_true",
                    help="with --inprocess: run the server in a child process (client and server do not share a GIL)")
    ap.add_argument("--serve-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--client-procs", type=int, default=1,
                    help="split the load generator over N processes (merged statistics)")
    ap.add_argument("--engine-process", action="store_true",
                    help="run the engine core in its own process (frontend only formats / streams)")
    a = ap.parse_args()
    if a.serve_only:                      # child of --spawn
        start_inprocess(a.inprocess, a.port, a.max_batch, a.max_model_len, a.engine_process)
        while True:
            time.sleep(3600)
    child = None
    if a.inprocess and a.spawn:
        import subprocess
        import urllib.request
        cmd = [sys.executable, os.path.abspath(__file__), "--serve-only", "--inprocess", a.inprocess, "--port",
               str(a.port), "--max-batch", str(a.max_batch)]
        if a.max_model_len:
            cmd += ["--max-model-len", str(a.max_model_len)]
        if a.engine_process:
            cmd += ["--engine-process"]
        child = subprocess.Popen(cmd)
        url = f"http://127.0.0.1:{a.port}"
        for _ in range(600):
            try:
                urllib.request.urlopen(url + "/health", timeout=2)
                break
            except Exception:
                if child.poll() is not None:
                    raise RuntimeError("server process exited")
                time.sleep(1)
    else:
        url = a.url or start_inprocess(a.inprocess, a.port, a.max_batch, a.max_model_len, a.engine_process)
    if a.dataset == "mixed":
        prompts = mixed_dataset(a.num_prompts)
    elif a.dataset == "short":       # ShareGPT-like chat turns only (the reference table's workload shape)
        prompts = [p for p in mixed_dataset(4 * a.num_prompts) if len(p) == 1][:a.num_prompts]
    else:
        prompts = sharegpt(a.dataset, a.num_prompts)
    if a.client_procs > 1:
        rows = [run_level_procs(url, a.model, prompts, c, a.max_tokens, min(a.client_procs, c))
                for c in a.concurrency]
    else:
        rows = [asyncio.run(run_level(url, a.model, prompts, c, a.max_tokens)) for c in a.concurrency]
    for r in rows:
        print(json.dumps(r))
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=2)
    if child is not None:
        child.terminate()
        child.wait(timeout=60)


if __name__ == "__main__":
    main()
