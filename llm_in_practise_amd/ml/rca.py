"""Server failure root-cause analysis (``ML_Basics/server_failure_rca``): YAML
config → clean + standardise → RandomForest over the failure cause, IsolationForest anomalies,
synthetic monitoring-data generator (``config/config.yaml``, ``src/*.py``, ``scripts/*.py``)."""
from __future__ import annotations

import dataclasses

import numpy as np
import pandas as pd
import yaml

DEFAULT_CONFIG = {
    "data": {"features": ["cpu_usage", "memory_usage", "disk_io", "network_latency"], "target": "failure_cause"},
    "model": {"type": "random_forest", "params": {"n_estimators": 100, "random_state": 42}},
    "anomaly_detection": {"contamination": 0.1},
}
CAUSES = ("CPU Overload", "Memory Issue", "Disk IO Bottleneck", "Network Delay", "None")
CAUSE_P = (0.1, 0.1, 0.05, 0.05, 0.7)


def load_config(path: str | None) -> dict:
    if path is None:
        return DEFAULT_CONFIG
    with open(path) as f:
        return yaml.safe_load(f)


def generate_monitoring_data(n: int, seed: int = 42) -> pd.DataFrame:
    rng = np.random.default_rng(seed)
    cause = rng.choice(CAUSES, size=n, p=CAUSE_P)
    cpu = np.clip(rng.normal(50, 15, n), 0, 100)
    mem = np.clip(rng.normal(60, 20, n), 0, 100)
    disk = np.clip(rng.normal(200, 50, n), 0, None)
    net = np.clip(rng.normal(50, 20, n), 0, None)
    cpu[cause == "CPU Overload"] = rng.uniform(90, 100, (cause == "CPU Overload").sum())
    mem[cause == "Memory Issue"] = rng.uniform(90, 100, (cause == "Memory Issue").sum())
    disk[cause == "Disk IO Bottleneck"] = rng.uniform(500, 1000, (cause == "Disk IO Bottleneck").sum())
    net[cause == "Network Delay"] = rng.uniform(200, 500, (cause == "Network Delay").sum())
    ts = pd.Timestamp("2025-07-12 06:00:00") - pd.to_timedelta(np.arange(n) * 5, unit="min")
    return pd.DataFrame({"timestamp": ts.astype(str), "cpu_usage": cpu, "memory_usage": mem, "disk_io": disk,
                         "network_latency": net, "failure_cause": cause})


def preprocess(data: pd.DataFrame, cfg: dict):
    from sklearn.preprocessing import StandardScaler
    feats, target = cfg["data"]["features"], cfg["data"]["target"]
    d = data.dropna()
    d = d[(d[feats] >= 0).all(axis=1)]
    scaler = StandardScaler().fit(d[feats])
    out = pd.DataFrame(scaler.transform(d[feats]), columns=feats)
    if target in d.columns:
        out[target] = d[target].to_numpy()
    return out, scaler


@dataclasses.dataclass
class RCAModel:
    model: object
    scaler: object
    features: list
    report: dict

    def predict(self, rows: pd.DataFrame):
        return self.model.predict(pd.DataFrame(self.scaler.transform(rows[self.features]), columns=self.features))


def train_rca(data: pd.DataFrame, cfg: dict | None = None) -> RCAModel:
    from sklearn.ensemble import RandomForestClassifier
    from sklearn.metrics import classification_report
    from sklearn.model_selection import train_test_split
    cfg = cfg or DEFAULT_CONFIG
    feats, target = cfg["data"]["features"], cfg["data"]["target"]
    d, scaler = preprocess(data, cfg)
    Xtr, Xte, ytr, yte = train_test_split(d[feats], d[target], test_size=0.2, random_state=42)
    m = RandomForestClassifier(**cfg["model"]["params"]).fit(Xtr, ytr)
    return RCAModel(m, scaler, feats, classification_report(yte, m.predict(Xte), output_dict=True, zero_division=0))


def detect_anomalies(data: pd.DataFrame, cfg: dict | None = None) -> pd.DataFrame:
    from sklearn.ensemble import IsolationForest
    cfg = cfg or DEFAULT_CONFIG
    feats = cfg["data"]["features"]
    d, _ = preprocess(data, cfg)
    iso = IsolationForest(contamination=cfg["anomaly_detection"]["contamination"], random_state=42)
    d["anomaly"] = iso.fit_predict(d[feats])     # −1 anomaly, 1 normal
    return d
