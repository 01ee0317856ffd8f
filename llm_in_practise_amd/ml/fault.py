"""Server fault prediction (``ML_Basics/fault_prediction_project``).

* :func:`generate_system_metrics` — synthetic per-minute metrics for two servers with a daily
  cycle and a ``fault_ratio`` of injected faults (high-load or error-burst patterns), schema
  ``timestamp, device_id, cpu_usage, ram_usage, disk_io, temperature, error_count, label``
  (``src/data_generation.py``);
* :func:`extract_features` — per-device 60-step rolling mean/std, a 60-step lag, hour and
  weekday (``src/feature_engineering.py``);
* :func:`smote` — minority oversampling by k-NN interpolation (imbalanced-learn's SMOTE is not
  installed; same algorithm);
* :func:`train_fault_model` — StandardScaler → SMOTE → stratified split → GradientBoosting under
  ``RandomizedSearchCV`` scored on recall (``src/model_training.py``).
"""
from __future__ import annotations

import dataclasses

import numpy as np
import pandas as pd

FEATURES = ["cpu_usage", "ram_usage", "disk_io", "temperature", "error_count", "cpu_usage_mean", "cpu_usage_std",
            "ram_usage_mean", "ram_usage_std", "hour", "day_of_week", "cpu_usage_lag1"]


def generate_system_metrics(n_samples: int = 5000, start_time: str = "2025-07-12 06:00:00",
                            fault_ratio: float = 0.05, seed: int = 42) -> pd.DataFrame:
    rng = np.random.default_rng(seed)
    ts = pd.date_range(start_time, periods=n_samples, freq="min")
    hours = ts.hour.to_numpy()
    cycle = np.sin(2 * np.pi * hours / 24)
    cpu = np.clip(50 + 20 * cycle + rng.normal(0, 5, n_samples), 0, 100)
    ram = np.clip(60 + 15 * cycle + rng.normal(0, 5, n_samples), 0, 100)
    disk = np.clip(rng.normal(20, 5, n_samples), 0, 100)
    temp = np.clip(35 + 0.2 * cpu + rng.normal(0, 2, n_samples), 30, 50)
    err = np.clip(rng.poisson(2, n_samples), 0, 20)
    labels = np.zeros(n_samples, dtype=int)
    idx = rng.choice(n_samples, size=int(n_samples * fault_ratio), replace=False)
    labels[idx] = 1
    high = rng.random(idx.size) < 0.9           # most faults are high-load; the rest are error bursts
    cpu[idx[high]] = rng.uniform(90, 100, high.sum())
    ram[idx[high]] = rng.uniform(85, 95, high.sum())
    temp[idx[high]] = rng.uniform(45, 50, high.sum())
    err[idx[~high]] = rng.integers(10, 21, (~high).sum())
    return pd.DataFrame({"timestamp": ts.astype(str), "device_id": rng.choice(["server_001", "server_002"], n_samples),
                         "cpu_usage": cpu, "ram_usage": ram, "disk_io": disk, "temperature": temp,
                         "error_count": err, "label": labels})


def extract_features(data: pd.DataFrame):
    d = data.copy()
    d["timestamp"] = pd.to_datetime(d["timestamp"])
    d["hour"] = d["timestamp"].dt.hour
    d["day_of_week"] = d["timestamp"].dt.dayofweek
    g = d.groupby("device_id")
    for col in ("cpu_usage", "ram_usage"):
        d[f"{col}_mean"] = g[col].transform(lambda s: s.rolling(60, min_periods=1).mean())
        d[f"{col}_std"] = g[col].transform(lambda s: s.rolling(60, min_periods=1).std())
    d["cpu_usage_lag1"] = g["cpu_usage"].shift(60)
    return d, list(FEATURES)


def smote(X: np.ndarray, y: np.ndarray, k: int = 5, seed: int = 42):
    """Oversample every minority class to the majority count by interpolating towards one of its
    k nearest same-class neighbours."""
    rng = np.random.default_rng(seed)
    classes, counts = np.unique(y, return_counts=True)
    n_max = counts.max()
    Xs, ys = [X], [y]
    for c, n in zip(classes, counts):
        if n == n_max or n < 2:
            continue
        P = X[y == c]
        d = ((P[:, None, :] - P[None, :, :]) ** 2).sum(-1)
        np.fill_diagonal(d, np.inf)
        nn = np.argsort(d, 1)[:, :min(k, len(P) - 1)]
        base = rng.integers(0, len(P), n_max - n)
        nb = nn[base, rng.integers(0, nn.shape[1], n_max - n)]
        lam = rng.random((n_max - n, 1))
        Xs.append(P[base] + lam * (P[nb] - P[base]))
        ys.append(np.full(n_max - n, c))
    return np.concatenate(Xs), np.concatenate(ys)


@dataclasses.dataclass
class FaultModel:
    model: object
    scaler: object
    features: list
    best_params: dict
    cv_recall: float
    report: dict

    def predict_proba(self, rows: pd.DataFrame) -> np.ndarray:
        X = self.scaler.transform(rows[self.features].fillna(0).to_numpy())
        return self.model.predict_proba(X)[:, 1]


def train_fault_model(data: pd.DataFrame, n_iter: int = 20, cv_splits: int = 5, seed: int = 42,
                      n_jobs: int = 1) -> FaultModel:
    from scipy.stats import randint, uniform
    from sklearn.ensemble import GradientBoostingClassifier
    from sklearn.metrics import classification_report
    from sklearn.model_selection import RandomizedSearchCV, StratifiedKFold, train_test_split
    from sklearn.preprocessing import StandardScaler
    d, feats = extract_features(data)
    X = d[feats].fillna(0).to_numpy()
    y = d["label"].to_numpy()
    scaler = StandardScaler().fit(X)
    Xr, yr = smote(scaler.transform(X), y, seed=seed)
    Xtr, Xte, ytr, yte = train_test_split(Xr, yr, test_size=0.2, random_state=seed, stratify=yr)
    dist = {"n_estimators": randint(50, 200), "learning_rate": uniform(0.01, 0.2), "max_depth": randint(3, 8),
            "min_samples_split": randint(2, 10), "min_samples_leaf": randint(1, 5)}
    search = RandomizedSearchCV(GradientBoostingClassifier(random_state=seed), dist, n_iter=n_iter,
                                cv=StratifiedKFold(cv_splits, shuffle=True, random_state=seed), scoring="recall",
                                n_jobs=n_jobs, random_state=seed)
    search.fit(Xtr, ytr)
    rep = classification_report(yte, search.best_estimator_.predict(Xte), output_dict=True)
    return FaultModel(search.best_estimator_, scaler, feats, search.best_params_, float(search.best_score_), rep)
