"""``python -m llm_in_practise_amd.ml.serve_cli [--data metrics.csv] [--port 5000] [--retrain-only --out DIR]``
Train (or load) the fault / RCA models and serve them (I1 ``model_service.py``, I2 ``api_server.py``),
or retrain and persist them (I1's ``model_retrain_cronjob.yaml``)."""
import argparse
import os

import joblib
import pandas as pd

from .fault import generate_system_metrics, train_fault_model
from .rca import generate_monitoring_data, load_config, train_rca


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--fault-data")
    ap.add_argument("--rca-data")
    ap.add_argument("--config")
    ap.add_argument("--out", default="models/ml")
    ap.add_argument("--retrain-only", action="store_true")
    ap.add_argument("--port", type=int, default=5000)
    ap.add_argument("--n-iter", type=int, default=20)
    a = ap.parse_args(argv)
    fm_path, rca_path = os.path.join(a.out, "fault_model.joblib"), os.path.join(a.out, "rca_model.joblib")
    if a.retrain_only or not os.path.exists(fm_path):
        fd = pd.read_csv(a.fault_data) if a.fault_data else generate_system_metrics()
        rd = pd.read_csv(a.rca_data) if a.rca_data else generate_monitoring_data(5000)
        fm, rm = train_fault_model(fd, n_iter=a.n_iter), train_rca(rd, load_config(a.config))
        os.makedirs(a.out, exist_ok=True)
        joblib.dump(fm, fm_path)          # files this code wrote itself
        joblib.dump(rm, rca_path)
        print({"fault_cv_recall": fm.cv_recall, "rca_accuracy": rm.report["accuracy"], "out": a.out})
        if a.retrain_only:
            return
    import uvicorn

    from .service import create_ml_app
    uvicorn.run(create_ml_app(joblib.load(fm_path), joblib.load(rca_path)), host="0.0.0.0", port=a.port)


if __name__ == "__main__":
    main()
