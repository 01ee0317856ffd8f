"""Classical-ML track: server fault prediction and failure root-cause analysis
with scikit-learn, plus their HTTP services.  CPU-only by design (tabular, small)."""
