"""Platform assets parse and reference each other consistently (deploy/k8s, deploy/serve)."""
import glob
import os

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _docs():
    out = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "deploy", "k8s", "**", "*.yaml"), recursive=True)):
        with open(f) as fh:
            out[os.path.relpath(f, ROOT)] = [d for d in yaml.safe_load_all(fh) if d]
    return out


def test_manifests_parse_with_kinds():
    docs = _docs()
    kinds = {(d["kind"], d["metadata"]["name"]) for ds in docs.values() for d in ds}
    for want in [("DaemonSet", "model-preloader"), ("StatefulSet", "lipa-qwen3-8b"), ("Service", "lipa-headless"),
                 ("Deployment", "lipa-kv"), ("Deployment", "lipa-router"), ("ConfigMap", "config-manager-config"),
                 ("Deployment", "open-webui"), ("PersistentVolumeClaim", "models-pvc")]:
        assert want in kinds, want
    for ds in docs.values():
        for d in ds:
            for c in (d.get("spec", {}).get("template", {}).get("spec", {}) or {}).get("containers", []):
                lim = (c.get("resources") or {}).get("limits") or {}
                assert "nvidia.com/gpu" not in lim           # AMD device plugin resources only


def test_router_configmap_and_serve_config_load():
    from llm_in_practise_amd.infer.router import Router
    from llm_in_practise_amd.infer.serve_app import load_serve_config
    docs = _docs()
    cm = next(d for d in docs["deploy/k8s/platform/08-router.yaml"] if d["kind"] == "ConfigMap")
    r = Router(yaml.safe_load(cm["data"]["config.yaml"]), send=lambda *a: {},
               resolver=lambda host, port: ["10.1.0.5", "10.1.0.6"])
    assert r.strategy == "load_aware_prefix" and len(r.groups["qwen3-8b"]) == 2
    sts = next(d for d in docs["deploy/k8s/platform/03-lipa-statefulset.yaml"] if d["kind"] == "StatefulSet")
    args = sts["spec"]["template"]["spec"]["containers"][0]["args"]
    from llm_in_practise_amd.cli.main import build_parser
    ns = build_parser().parse_args(args)                      # every flag exists in `lipa serve`
    assert ns.prefix_caching and ns.kv_remote_url.startswith("http://lipa-kv")
    apps = load_serve_config(os.path.join(ROOT, "deploy", "serve", "qwen3_autoscaling.yaml"))
    assert [a.route_prefix for a in apps] == ["/app1", "/app2"] and apps[0].autoscaling.max_replicas == 6


REF = "/root/reference"


def _reference_vllm_invocations():
    """(file, args) of every vLLM server the reference deploys: k8s containers running a vllm-openai image
    (args list) and docker-compose services whose image is vllm (command string)."""
    out = []
    if not os.path.isdir(REF):
        return out
    for dirpath, _, files in os.walk(REF):
        for fn in files:
            if not fn.endswith((".yaml", ".yml")):
                continue
            path = os.path.join(dirpath, fn)
            try:
                with open(path) as f:
                    docs = list(yaml.safe_load_all(f))
            except Exception:
                continue
            for d in docs:
                if not isinstance(d, dict):
                    continue
                for c in (((d.get("spec") or {}).get("template") or {}).get("spec") or {}).get("containers", []) or []:
                    if "vllm-openai" in str(c.get("image", "")) and c.get("args") and not c.get("command"):
                        out.append((path, [str(x) for x in c["args"]]))
                for svc in (d.get("services") or {}).values() if isinstance(d.get("services"), dict) else []:
                    if "vllm" in str(svc.get("image", "")) and isinstance(svc.get("command"), str):
                        out.append((path, svc["command"].split()))
    return out


def test_reference_vllm_manifests_parse_with_lipa_serve():
    """the reference's vLLM manifests apply to `lipa serve` unchanged — every arg list parses with its
    parser and maps onto the engine (model dir, served name, dtype, memory fraction, max seqs, quantization)"""
    from llm_in_practise_amd.cli.main import _vllm_compat, build_parser
    inv = _reference_vllm_invocations()
    if not inv:
        pytest.skip("reference tree not present")
    base = os.path.join(REF, "LLM_on_Kubernetes/Inference_Platfrom/01-Base/vLLM/vllm-deployment.yaml")
    assert any(p == base for p, _ in inv), [p for p, _ in inv]
    for path, args in inv:
        ns = build_parser().parse_args(["serve", *args])
        assert (ns.model or ns.model_tag), path
        if ns.vllm_quant is None and not ns.kv_transfer_config:
            _vllm_compat(ns)                     # (quantized / LMCache ones need the checkpoint / env: below)
        if "--gpu-memory-utilization" in args:
            assert 0 < ns.gpu_memory_utilization <= 1
        if "--max-num-seqs" in args:
            assert ns.max_batch == int(args[args.index("--max-num-seqs") + 1])
    ns = build_parser().parse_args(["serve", *dict(inv)[base]])
    _vllm_compat(ns)
    assert ns.model == "/data/models/qwen3-8b" and ns.served_model_name == "qwen3-8b"
    assert ns.dtype == "bfloat16" and ns.gpu_memory_utilization == 0.9 and ns.max_model_len == 4096
    assert ns.tp == 1 and ns.uvicorn_log_level == "info"


def test_vllm_quantization_and_lmcache_flags(tmp_path, monkeypatch):
    import json as _json

    from llm_in_practise_amd.cli.main import _vllm_compat, build_parser
    (tmp_path / "config.json").write_text(_json.dumps({"quantization_config": {"quant_method": "compressed-tensors"}}))
    ns = _vllm_compat(build_parser().parse_args(["serve", str(tmp_path), "--quantization", "compressed-tensors"]))
    assert ns.model == str(tmp_path) and ns.quant is None
    ns = _vllm_compat(build_parser().parse_args(["serve", str(tmp_path), "--quantization", "awq"]))   # AWQ saved
    with pytest.raises(SystemExit):                                                         # as compressed-tensors
        _vllm_compat(build_parser().parse_args(["serve", str(tmp_path / "none"), "--quantization", "awq"]))
    ns = _vllm_compat(build_parser().parse_args(["serve", "--model", "m", "--quantization", "bitsandbytes"]))
    assert ns.quant == "nf4"
    monkeypatch.setenv("LMCACHE_REMOTE_URL", "lm://lmcache-server.lmcache.svc.cluster.local:5555")
    monkeypatch.setenv("LMCACHE_MAX_LOCAL_CPU_SIZE", "5")
    monkeypatch.setenv("LMCACHE_CHUNK_SIZE", "256")
    ns = _vllm_compat(build_parser().parse_args(
        ["serve", "m", "--kv-transfer-config", '{"kv_connector":"LMCacheConnectorV1", "kv_role":"kv_both"}']))
    assert ns.prefix_caching and ns.kv_remote_url == "http://lmcache-server.lmcache.svc.cluster.local:5555"
    assert ns.prefix_block == 256 and ns.host_blocks == -5 * 2 ** 30


def test_kv_slots_for_budget():
    from llm_in_practise_amd.infer.engine import kv_slots_for_budget
    gib = 2 ** 30
    # Qwen3-8B bf16 at 4096 tokens: 2 x 36 layers x 4096 x 8 heads x 128 x 2 B = 576 MiB per slot
    slot = 2 * 36 * 4096 * 8 * 128 * 2
    assert kv_slots_for_budget(288 * gib, 16 * gib, 0.9, slot, 4 * gib) == int((0.9 * 288 - 20) * gib // slot)
    with pytest.raises(ValueError):
        kv_slots_for_budget(24 * gib, 16 * gib, 0.45, slot)
