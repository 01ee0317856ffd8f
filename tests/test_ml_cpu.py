"""Classical-ML track (I1/I2) — includes the reference's only unittest (data schema)."""
from fastapi.testclient import TestClient

from llm_in_practise_amd.ml.fault import extract_features, generate_system_metrics, smote, train_fault_model
from llm_in_practise_amd.ml.rca import detect_anomalies, generate_monitoring_data, train_rca
from llm_in_practise_amd.ml.service import create_ml_app


def test_data_shape():     # ML_Basics/fault_prediction_project/tests/test_data_generation.py
    data = generate_system_metrics(n_samples=100)
    assert len(data) == 100
    assert set(data.columns) == {"timestamp", "device_id", "cpu_usage", "ram_usage", "disk_io", "temperature",
                                 "error_count", "label"}


def test_fault_pipeline_and_service():
    import numpy as np
    data = generate_system_metrics(n_samples=800, fault_ratio=0.05)
    d, feats = extract_features(data)
    assert set(feats) <= set(d.columns)
    X, y = smote(np.random.rand(30, 3), np.array([0] * 25 + [1] * 5))
    assert (y == 1).sum() == (y == 0).sum() == 25
    fm = train_fault_model(data, n_iter=2, cv_splits=2)
    assert fm.cv_recall > 0.8
    rca = train_rca(generate_monitoring_data(600))
    assert rca.report["accuracy"] > 0.8
    an = detect_anomalies(generate_monitoring_data(300))
    assert set(an["anomaly"].unique()) <= {-1, 1}
    c = TestClient(create_ml_app(fm, rca))
    assert c.get("/health").json()["status"] == "healthy"
    row = d[fm.features].fillna(0).iloc[:2].to_dict(orient="records")
    assert len(c.post("/predict_fault", json=row).json()["fault_probability"]) == 2
    r = c.post("/predict", json={"cpu_usage": 99, "memory_usage": 50, "disk_io": 200, "network_latency": 40})
    assert r.json()["failure_cause"] == "CPU Overload"
