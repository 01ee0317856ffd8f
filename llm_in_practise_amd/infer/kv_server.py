"""Remote KV-chunk store shared by serving replicas — the LMCache server role
(``LLM_on_Kubernetes/Inference_Platfrom/07-L1-Cache/LMCache/lmcache-deployment.yaml``: an
``lmcache_server`` Deployment that every vLLM replica reaches through ``LMCACHE_REMOTE_URL``,
``vllm-statefulset-lmcache.yaml:96-111``).

The third tier behind the prefix cache's HBM pool and pinned-host pool
(:class:`~.engine.PrefixCache`): a replica that computes a prompt chunk's K/V writes it through
to this store (asynchronously, off the engine loop), and any replica that later misses that
chunk in HBM and host memory fetches it instead of recomputing it — so a system prompt or RAG
document prefilled once is warm on every replica behind the router.

Keys are the prefix cache's chained content digests (blake2b over token ids, salted per
adapter), so equal prefixes hash equally across processes and hosts.  Values are raw chunk
bytes ``[layers, 2, block, width]`` in the model dtype.  The store is a byte-bounded LRU.

    lipa kv-server --port 8100 --max-gib 64
    lipa serve ... --enable-prefix-caching --kv-remote-url http://kv:8100
"""
from __future__ import annotations

import collections
import queue
import threading

from fastapi import FastAPI, Request, Response
from fastapi.responses import JSONResponse, PlainTextResponse


class KVStore:
    def __init__(self, max_bytes: int):
        self.max_bytes = int(max_bytes)
        self.data: "collections.OrderedDict[str, bytes]" = collections.OrderedDict()
        self.bytes = 0
        self.lock = threading.Lock()
        self.stats = collections.Counter()

    def put(self, key: str, val: bytes):
        with self.lock:
            old = self.data.pop(key, None)
            if old is not None:
                self.bytes -= len(old)
            if len(val) > self.max_bytes:
                return
            self.data[key] = val
            self.bytes += len(val)
            self.stats["puts"] += 1
            while self.bytes > self.max_bytes:
                _, v = self.data.popitem(last=False)
                self.bytes -= len(v)
                self.stats["evictions"] += 1

    def get(self, key: str) -> bytes | None:
        with self.lock:
            v = self.data.get(key)
            if v is None:
                self.stats["misses"] += 1
                return None
            self.data.move_to_end(key)
            self.stats["hits"] += 1
            return v


def create_kv_server(max_bytes: int = 64 << 30) -> FastAPI:
    store = KVStore(max_bytes)
    app = FastAPI(title="lipa kv-server")
    app.state.store = store

    @app.put("/kv/{key}")
    async def put(key: str, request: Request):
        store.put(key, await request.body())
        return Response(status_code=204)

    @app.get("/kv/{key}")
    async def get(key: str):
        v = store.get(key)
        if v is None:
            return Response(status_code=404)
        return Response(content=v, media_type="application/octet-stream")

    @app.post("/kv/exists")
    async def exists(keys: list[str]):
        with store.lock:
            return JSONResponse([k in store.data for k in keys])

    @app.get("/health")
    async def health():
        return {"status": "ok", "entries": len(store.data), "bytes": store.bytes}

    @app.get("/metrics")
    async def metrics():
        lines = [f"lipa_kv_server_bytes {store.bytes}", f"lipa_kv_server_entries {len(store.data)}"]
        lines += [f"lipa_kv_server_{k}_total {v}" for k, v in sorted(store.stats.items())]
        return PlainTextResponse("\n".join(lines) + "\n")

    return app


class RemoteKV:
    """Client side: synchronous ``get`` (on a prefix-cache miss), write-behind ``put`` from a
    background thread so the engine loop never waits for the network."""

    def __init__(self, url: str, timeout: float = 5.0, max_pending: int = 256):
        import httpx
        self.url = url.rstrip("/")
        self.client = httpx.Client(timeout=timeout)
        self.q: "queue.Queue" = queue.Queue(max_pending)
        self.stats = collections.Counter()
        self._thread = threading.Thread(target=self._writer, daemon=True)
        self._thread.start()

    def get(self, key: bytes) -> bytes | None:
        try:
            r = self.client.get(f"{self.url}/kv/{key.hex()}")
        except Exception:
            self.stats["errors"] += 1
            return None
        if r.status_code != 200:
            self.stats["misses"] += 1
            return None
        self.stats["hits"] += 1
        return r.content

    def put(self, key: bytes, payload):
        """``payload``: bytes, or a zero-argument callable producing them on the writer thread
        (lets the caller hand over a pinned buffer + event without blocking)."""
        try:
            self.q.put_nowait((key, payload))
        except queue.Full:
            self.stats["dropped"] += 1

    def _writer(self):
        while True:
            key, payload = self.q.get()
            if key is None:
                return
            try:
                data = payload() if callable(payload) else payload
                self.client.put(f"{self.url}/kv/{key.hex()}", content=data)
                self.stats["puts"] += 1
            except Exception:
                self.stats["errors"] += 1
            finally:
                self.q.task_done()

    def flush(self):
        self.q.join()

    def close(self):
        self.q.put((None, None))
        self._thread.join(5)
