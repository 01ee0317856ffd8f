"""Platform assets parse and reference each other consistently (deploy/k8s, deploy/serve)."""
import glob
import os

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
