"""Load the reference's own function definitions (TEST INFRASTRUCTURE ONLY).

This module reads the reference notebooks under ``/root/reference`` *as JSON at run
time*, picks the code cells whose first statement is ``def <name>(`` and execs them
into a namespace pre-populated with numpy/pandas/datetime/time/random/os.  Nothing
from the reference is copied into this repository; the reference only exists in the
build container, never on the GPU box, so only ``oracle/gen_golden.py`` (which writes
the committed fixtures under ``tests/golden/``) may import this module.

Method as recorded in SURVEY.md §8(c): ``shared_functions.py`` cannot be imported
(``get_ipython`` at shared_functions.py:45, missing graphviz/xgboost/imblearn at
:49-57), so the defs are exec'd from the notebook cells instead.
"""
from __future__ import annotations

import datetime
import json
import os
import random
import re
import time

import numpy as np
import pandas as pd

REF_ROOT = os.environ.get("FDX_REFERENCE_ROOT", "/root/reference")
NB_DIR = os.path.join(REF_ROOT, "fraud_detection_model")

# name -> notebook holding its def (reference file:line of the def line in the raw JSON)
GENERATOR_DEFS = {
    "generate_customer_profiles_table": "data_generator.ipynb",   # :113-140
    "generate_terminal_profiles_table": "data_generator.ipynb",   # :285-303
    "get_list_terminals_within_radius": "data_generator.ipynb",   # :420-437
    "generate_transactions_table": "data_generator.ipynb",        # :786-834
    "generate_dataset": "data_generator.ipynb",                   # :1339-1371
    "add_frauds": "data_generator.ipynb",                         # :1732-1782
}
FEATURE_DEFS = {
    "is_weekend": "feature_transformation.ipynb",                         # :246-253
    "is_night": "feature_transformation.ipynb",                           # :294-301
    "get_customer_spending_behaviour_features": "feature_transformation.ipynb",  # :601-628
    "get_count_risk_rolling_window": "feature_transformation.ipynb",      # :1495-1522
}
TRAINING_DEFS = {
    "fit_model_and_get_predictions": "model_training.ipynb",      # :491-520
}


def _cells(nb_name: str):
    with open(os.path.join(NB_DIR, nb_name)) as f:
        nb = json.load(f)
    for cell in nb["cells"]:
        if cell["cell_type"] == "code":
            yield "".join(cell["source"])


def _find_def(nb_name: str, fname: str) -> str:
    pat = re.compile(r"^\s*def\s+" + re.escape(fname) + r"\s*\(")
    for src in _cells(nb_name):
        first = next((ln for ln in src.splitlines() if ln.strip()), "")
        if pat.match(first):
            return src
    raise KeyError(f"def {fname} not found in {nb_name}")


def _shared_function_src(fname: str) -> str:
    """Extract one top-level def from shared_functions.py (skips its import block)."""
    with open(os.path.join(NB_DIR, "shared_functions.py")) as f:
        lines = f.read().splitlines()
    out, grab = [], False
    for ln in lines:
        if ln.startswith("def " + fname + "("):
            grab = True
            out.append(ln)
            continue
        if grab:
            if ln and not ln[0].isspace() and not ln.startswith("#"):
                break
            out.append(ln)
    if not out:
        raise KeyError(fname)
    return "\n".join(out)


def load_namespace(include_training: bool = False) -> dict:
    import sklearn
    import sklearn.preprocessing

    ns = {"np": np, "pd": pd, "datetime": datetime, "time": time, "random": random,
          "os": os, "sklearn": sklearn}
    for table in (GENERATOR_DEFS, FEATURE_DEFS):
        for fname, nb in table.items():
            exec(compile(_find_def(nb, fname), f"<ref:{nb}:{fname}>", "exec"), ns)
    for fname in ("read_from_files", "scaleData", "get_train_test_set"):
        exec(compile(_shared_function_src(fname), f"<ref:shared_functions.py:{fname}>", "exec"), ns)
    if include_training:
        for fname, nb in TRAINING_DEFS.items():
            exec(compile(_find_def(nb, fname), f"<ref:{nb}:{fname}>", "exec"), ns)
    return ns


def reference_featurize(ns: dict, transactions_df: pd.DataFrame) -> pd.DataFrame:
    """Drive the reference functions exactly as feature_transformation.ipynb does
    (cells at :278, :319, :1092-1093, :2435-2436)."""
    df = transactions_df.copy()
    df["TX_DURING_WEEKEND"] = df.TX_DATETIME.apply(ns["is_weekend"])
    df["TX_DURING_NIGHT"] = df.TX_DATETIME.apply(ns["is_night"])
    f_c = ns["get_customer_spending_behaviour_features"]
    df = df.groupby("CUSTOMER_ID").apply(lambda x: f_c(x, windows_size_in_days=[1, 7, 30]))
    df = df.sort_values("TX_DATETIME").reset_index(drop=True)
    f_t = ns["get_count_risk_rolling_window"]
    df = df.groupby("TERMINAL_ID").apply(
        lambda x: f_t(x, delay_period=7, windows_size_in_days=[1, 7, 30], feature="TERMINAL_ID"))
    df = df.sort_values("TX_DATETIME").reset_index(drop=True)
    return df
