"""HTTP services for the classical-ML track: ``POST /predict_fault`` (I1's Flask service,
``src/model_service.py:17-40``) and ``POST /predict`` / ``POST /batch_predict`` (I2's FastAPI,
``scripts/api_server.py:43-127``), ``GET /health``."""
from __future__ import annotations

import pandas as pd
from fastapi import FastAPI, HTTPException
from pydantic import BaseModel


class MetricInput(BaseModel):
    cpu_usage: float
    memory_usage: float
    disk_io: float
    network_latency: float


class BatchMetricInput(BaseModel):
    metrics: list[MetricInput]


def create_ml_app(fault_model=None, rca_model=None) -> FastAPI:
    app = FastAPI(title="server fault prediction / RCA")

    @app.get("/health")
    async def health():
        return {"status": "healthy", "fault_model": fault_model is not None, "rca_model": rca_model is not None}

    @app.post("/predict_fault")
    async def predict_fault(rows: list[dict] | dict):
        if fault_model is None:
            raise HTTPException(503, "fault model not loaded")
        df = pd.DataFrame(rows if isinstance(rows, list) else [rows])
        missing = [f for f in fault_model.features if f not in df.columns]
        if missing:
            raise HTTPException(400, f"missing features: {missing}")
        p = fault_model.predict_proba(df)
        return {"fault_probability": [float(x) for x in p], "fault": [bool(x >= 0.5) for x in p]}

    @app.post("/predict")
    async def predict(m: MetricInput):
        if rca_model is None:
            raise HTTPException(503, "rca model not loaded")
        return {"failure_cause": str(rca_model.predict(pd.DataFrame([m.model_dump()]))[0])}

    @app.post("/batch_predict")
    async def batch_predict(b: BatchMetricInput):
        if rca_model is None:
            raise HTTPException(503, "rca model not loaded")
        preds = rca_model.predict(pd.DataFrame([m.model_dump() for m in b.metrics]))
        return {"predictions": [str(p) for p in preds]}

    return app
