"""`lipa serve` end to end on CPU: the default runs the engine core in its own process
(infer/mp_engine.py) behind the OpenAI server; `--no-engine-process` keeps it in-process."""
import json
import os
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _get(url, body=None, timeout=5):
    req = urllib.request.Request(url, data=None if body is None else json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return json.loads(r.read())


@pytest.mark.parametrize("extra", [[], ["--no-engine-process"]])
def test_lipa_serve_completion(extra):
    port = _port()
    cmd = [sys.executable, "-m", "llm_in_practise_amd.cli.main", "serve", "--model", "random:qwen3-tiny",
           "--tokenizer", "bytes", "--host", "127.0.0.1", "--port", str(port), "--max-batch", "4",
           "--served-model-name", "tiny", *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        base = f"http://127.0.0.1:{port}"
        deadline = time.time() + 240
        while True:
            if p.poll() is not None:
                raise AssertionError(p.stdout.read()[-3000:])
            try:
                models = _get(base + "/v1/models")
                break
            except Exception:
                if time.time() > deadline:
                    raise
                time.sleep(0.5)
        assert [m["id"] for m in models["data"]] == ["tiny"]
        r = _get(base + "/v1/completions", {"model": "tiny", "prompt": "hello", "max_tokens": 5,
                                            "temperature": 0}, timeout=120)
        assert r["usage"]["completion_tokens"] == 5
        r2 = _get(base + "/v1/completions", {"model": "tiny", "prompt": "hello", "max_tokens": 5,
                                             "temperature": 0}, timeout=120)
        assert r2["choices"][0]["text"] == r["choices"][0]["text"]
    finally:
        p.terminate()
        try:
            p.wait(30)
        except subprocess.TimeoutExpired:
            p.kill()
