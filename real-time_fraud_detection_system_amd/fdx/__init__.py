"""fdx -- MI355X-native drop-in for the hot path of Real-time_fraud_detection_system.

Public API (names and contracts of the reference functions):
  is_weekend, is_night, get_customer_spending_behaviour_features,
  get_count_risk_rolling_window          (fraud_detection_model/feature_transformation.ipynb)
  scaleData, fit_model_and_get_predictions (fraud_detection_model/shared_functions.py,
                                            model_training.ipynb)
  make_scale_and_predict_udf               (pyspark/scripts/fraud_detection.py:183-195)
  latest_terminal_features, customer_features_on, decode_cdc_batch
                                           (serving snapshots, Debezium CDC; fdx.serving)
  get_train_test_set, card_precision_top_k (shared_functions.py:133-188, :384-411; fdx.evaluation)
plus the device-tensor layer (fdx.ops), the fused pipeline (fdx.pipeline.FraudPipeline)
and the multi-GPU driver (fdx.distributed).
"""
from ._lib import FDX_FLAGS_NOTEBOOK, FDX_FLAGS_SPARK, FdxError, FdxUnsupported, load  # noqa: F401
from .features import (get_count_risk_rolling_window, get_customer_spending_behaviour_features,  # noqa: F401
                       is_night, is_weekend)
from .scoring import (INPUT_FEATURES, GpuForest, fit_model_and_get_predictions,  # noqa: F401
                      make_scale_and_predict_udf, scaleData)
from .evaluation import card_precision_top_k, get_train_test_set  # noqa: F401
from .serving import customer_features_on, decode_cdc_batch, latest_terminal_features  # noqa: F401

__all__ = ["is_weekend", "is_night", "get_customer_spending_behaviour_features",
           "get_count_risk_rolling_window", "scaleData", "fit_model_and_get_predictions",
           "make_scale_and_predict_udf", "latest_terminal_features", "customer_features_on",
           "decode_cdc_batch", "get_train_test_set", "card_precision_top_k", "GpuForest", "INPUT_FEATURES", "FdxError", "FdxUnsupported",
           "FDX_FLAGS_NOTEBOOK", "FDX_FLAGS_SPARK", "load"]
