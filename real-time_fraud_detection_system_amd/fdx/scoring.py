"""Drop-in scoring: scaleData, fit_model_and_get_predictions, the Spark UDF body.

Reference contract:
  scaleData(train, test, features) -> (train, test, scaler)       shared_functions.py:114-120
  fit_model_and_get_predictions(classifier, train_df, test_df, input_features,
                                output_feature="TX_FRAUD", scale=True) -> dict
                                      model_training.ipynb:491-520 (shared_functions.py:304-333)
  scale_and_predict_udf(*cols) -> pd.Series  (pandas UDF body)   pyspark/scripts/fraud_detection.py:183-195

Training (StandardScaler.fit, classifier.fit) stays in scikit-learn: it is offline and out
of scope.  The transform and predict_proba -- the hot path -- run on the
GPU through libfdx.so.  Tree models on the GPU: DecisionTreeClassifier and
RandomForestClassifier (binary, single output).  The reference's model zoo
(model_training.ipynb:2209-2214) also holds LogisticRegression and XGBClassifier: those are
not tree ensembles this path accelerates, so fit_model_and_get_predictions and the UDF call
their own predict_proba, exactly as the reference does (the scaling still runs on the GPU).
"""
from __future__ import annotations

import time
from typing import Optional, Sequence

import numpy as np
import pandas as pd
import torch

from . import _lib, ops

INPUT_FEATURES = ["TX_AMOUNT", "TX_DURING_WEEKEND", "TX_DURING_NIGHT",
                  "CUSTOMER_ID_NB_TX_1DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_1DAY_WINDOW",
                  "CUSTOMER_ID_NB_TX_7DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_7DAY_WINDOW",
                  "CUSTOMER_ID_NB_TX_30DAY_WINDOW", "CUSTOMER_ID_AVG_AMOUNT_30DAY_WINDOW",
                  "TERMINAL_ID_NB_TX_1DAY_WINDOW", "TERMINAL_ID_RISK_1DAY_WINDOW",
                  "TERMINAL_ID_NB_TX_7DAY_WINDOW", "TERMINAL_ID_RISK_7DAY_WINDOW",
                  "TERMINAL_ID_NB_TX_30DAY_WINDOW", "TERMINAL_ID_RISK_30DAY_WINDOW"]


def _as_f64_matrix(X) -> np.ndarray:
    if isinstance(X, pd.DataFrame):
        cols = []
        for c in X.columns:
            s = X[c]
            if s.dtype == object:  # Spark DECIMAL(10,2) arrives as decimal.Decimal objects
                s = pd.to_numeric(s, errors="coerce")
            cols.append(np.asarray(s, dtype=np.float64))
        return np.ascontiguousarray(np.stack(cols, axis=1)) if cols else np.zeros((len(X), 0))
    return np.ascontiguousarray(np.asarray(X, dtype=np.float64))


def _scaler_params(scaler):
    mean = getattr(scaler, "mean_", None) if getattr(scaler, "with_mean", True) else None
    scale = getattr(scaler, "scale_", None) if getattr(scaler, "with_std", True) else None
    return mean, scale


def gpu_transform(scaler, X) -> np.ndarray:
    """StandardScaler.transform on the GPU (float64, bit-identical).  The result has the
    memory order sklearn's transform would give (for a multi-dtype DataFrame pandas hands its
    values over column-major, and sklearn keeps that order), so that a BLAS consumer
    downstream (LogisticRegression's X @ coef) sums in the same order as on the reference's
    output (fraud_detection.py:190-193)."""
    dev = ops.require_gpu()
    Xh = _as_f64_matrix(X)
    mean, scale = _scaler_params(scaler)
    Xd = torch.from_numpy(Xh).to(dev)
    m = None if mean is None else torch.from_numpy(np.asarray(mean, np.float64)).to(dev)
    s = None if scale is None else torch.from_numpy(np.asarray(scale, np.float64)).to(dev)
    out = ops.standard_scale(Xd, m, s).cpu().numpy()
    if isinstance(X, pd.DataFrame):
        ref = X.to_numpy()
        if ref.ndim == 2 and ref.flags.f_contiguous and not ref.flags.c_contiguous:
            return np.asfortranarray(out)
    return out


def scaleData(train, test, features):
    """shared_functions.py:114-120: fit on train (sklearn), transform both on the GPU, in place."""
    import sklearn.preprocessing

    scaler = sklearn.preprocessing.StandardScaler()
    scaler.fit(train[features])
    train[features] = gpu_transform(scaler, train[features])
    test[features] = gpu_transform(scaler, test[features])
    return (train, test, scaler)


class GpuForest:
    """A fitted sklearn tree classifier (+ optional StandardScaler) resident on the GPU."""

    def __init__(self, model, scaler=None):
        dev = ops.require_gpu()
        self.model = model
        arrays = ops.forest_arrays_from_sklearn(model)
        nf = int(getattr(model, "n_features_in_"))
        mean, scale = _scaler_params(scaler) if scaler is not None else (None, None)
        self.forest = ops.Forest(arrays, nf, mean, scale)
        self._arrays, self._scaler, self._forest0 = arrays, (mean, scale), None
        self.device = dev
        self.n_features = nf

    def _run(self, X, want_leaves=False):
        Xd = torch.from_numpy(_as_f64_matrix(X)).to(self.device)
        return self.forest.predict(Xd, want_leaves=want_leaves)

    def predict_proba(self, X) -> np.ndarray:
        """[n, 2] like sklearn.  Column 1 is the class-1 forest; column 0 is NOT 1 - p (that can
        differ from sklearn in the last bit): sklearn sums tree_.value[:, 0, 0] in tree order,
        so a second device forest over the class-0 leaf values does the same additions."""
        p = self._run(X).cpu().numpy()
        if getattr(self, "_forest0", None) is None:
            a0 = dict(self._arrays, value1=self._arrays["value0"])
            self._forest0 = ops.Forest(a0, self.n_features, *self._scaler)
        Xd = torch.from_numpy(_as_f64_matrix(X)).to(self.device)
        p0 = self._forest0.predict(Xd).cpu().numpy()
        return np.stack([p0, p], axis=1)

    def predict_proba1(self, X) -> np.ndarray:
        return self._run(X).cpu().numpy()

    def apply(self, X) -> np.ndarray:
        _, leaves = self._run(X, want_leaves=True)
        return leaves.cpu().numpy()


def _is_supported_tree_model(clf) -> bool:
    import sklearn.ensemble
    import sklearn.tree

    return isinstance(clf, (sklearn.tree.DecisionTreeClassifier, sklearn.ensemble.RandomForestClassifier))


class _OwnPredictor:
    """A classifier outside the GPU tree path (LogisticRegression, XGBClassifier, ...): its own
    predict_proba, as the reference calls it (model_training.ipynb:506)."""

    def __init__(self, model, scaler=None):
        self.model, self.scaler = model, scaler

    def predict_proba1(self, X) -> np.ndarray:
        if self.scaler is not None:  # fraud_detection.py:190-193: transform -> ndarray -> predict_proba
            X = gpu_transform(self.scaler, X)
        return np.asarray(self.model.predict_proba(X))[:, 1]


def predictor(model, scaler=None):
    """GpuForest for sklearn tree classifiers, the model's own predict_proba otherwise."""
    return GpuForest(model, scaler) if _is_supported_tree_model(model) else _OwnPredictor(model, scaler)


def fit_model_and_get_predictions(classifier, train_df, test_df, input_features,
                                  output_feature="TX_FRAUD", scale=True):
    """model_training.ipynb:491-520.  fit stays in sklearn; predict_proba runs on the GPU for
    tree classifiers and through the classifier's own predict_proba for the rest of the
    notebook's model zoo (LR / XGB, model_training.ipynb:2209-2214)."""
    if scale:
        (train_df, test_df, _scaler) = scaleData(train_df, test_df, input_features)
    start_time = time.time()
    classifier.fit(train_df[input_features], train_df[output_feature])
    training_execution_time = time.time() - start_time

    g = predictor(classifier)
    start_time = time.time()
    predictions_test = g.predict_proba1(test_df[input_features])
    prediction_execution_time = time.time() - start_time
    predictions_train = g.predict_proba1(train_df[input_features])
    return {"classifier": classifier, "predictions_test": predictions_test,
            "predictions_train": predictions_train, "training_execution_time": training_execution_time,
            "prediction_execution_time": prediction_execution_time}


def make_scale_and_predict_udf(model, scaler, feature_columns: Optional[Sequence[str]] = None):
    """The body of fraud_detection.py:183-195 as a plain function of the 15 column Series.

    Wrap it with ``pyspark.sql.functions.pandas_udf("double")`` exactly like the
    reference: ``scale_and_predict_udf = pandas_udf("double")(make_scale_and_predict_udf(
    model, loaded_scaler))``.  NULL features (LEFT JOIN misses) arrive as NaN and follow
    sklearn's missing-value routing."""
    g = predictor(model, scaler)
    cols_names = list(feature_columns or INPUT_FEATURES)

    def scale_and_predict_udf(*cols: pd.Series) -> pd.Series:
        features = pd.concat(cols, axis=1)
        features.columns = cols_names
        return pd.Series(g.predict_proba1(features))

    return scale_and_predict_udf
