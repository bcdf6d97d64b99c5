/*
 * fdx_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This file is the *checker*: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so.  The product path (libfdx.so + HIP kernels)
 * never links, loads or falls back to it.
 *
 * Parity anchor: pinned against golden vectors produced by running the reference's
 * own notebook functions in the build container (oracle/gen_golden.py ->
 * tests/golden/ npz files) and against the known-answer rows printed in the committed
 * notebook outputs (tests/golden/notebook_kat.json).
 *
 * Restated algorithms (the arithmetic lives in third-party code the reference calls):
 *  - pandas 2.2.3 (poetry.lock:1444-1446) rolling with an offset window on a
 *    DatetimeIndex: pandas/_libs/window/indexers.pyx calculate_variable_window_bounds
 *    (closed='right') + pandas/_libs/window/aggregations.pyx roll_sum / add_sum /
 *    remove_sum / calc_sum (Kahan add/remove with separate compensations, reset when the
 *    new window does not overlap the previous one, "n consecutive equal values" rule).
 *    Called from fraud_detection_model/feature_transformation.ipynb:613-614
 *    (customer) and :1501-1502, :1506-1507 (terminal).
 *  - scikit-learn 1.6.1 (poetry.lock:2248-2250) StandardScaler.transform
 *    (X -= mean_; X /= scale_ in float64), ForestClassifier.predict_proba
 *    (X -> float32, Tree._apply_dense: NaN -> missing_go_to_left, else
 *    (double)x32 <= threshold64 -> left, accumulate class-1 leaf values in tree order in
 *    float64, divide by n_estimators).  Reached from shared_functions.py:114-120,
 *    model_training.ipynb:506, pyspark/scripts/fraud_detection.py:190-193.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---- pandas roll_sum state (aggregations.pyx add_sum/remove_sum/calc_sum) ---- */
typedef struct {
    double sum, comp_add, comp_rem, prev;
    int64_t nobs, nsame;
} rsum_t;

static void rs_reset(rsum_t *s, double first) {
    s->sum = s->comp_add = s->comp_rem = 0.0;
    s->nobs = 0;
    s->nsame = 0;
    s->prev = first;
}

static void rs_add(rsum_t *s, double v) {
    if (v == v) {
        double y, t;
        s->nobs += 1;
        y = v - s->comp_add;
        t = s->sum + y;
        s->comp_add = t - s->sum - y;
        s->sum = t;
        if (v == s->prev) s->nsame += 1; else s->nsame = 1;
        s->prev = v;
    }
}

static void rs_remove(rsum_t *s, double v) {
    if (v == v) {
        double y, t;
        s->nobs -= 1;
        y = -v - s->comp_rem;
        t = s->sum + y;
        s->comp_rem = t - s->sum - y;
        s->sum = t;
    }
}

static double rs_value(const rsum_t *s, int64_t minp) {
    if (s->nobs == 0 && minp == 0) return 0.0;
    if (s->nobs >= minp) {
        if (s->nsame >= s->nobs) return s->prev * (double)s->nobs;
        return s->sum;
    }
    return NAN;
}

/* pandas calculate_variable_window_bounds for closed='right' (the default):
 * start[0]=0,end[0]=1; start[i] = first j in [start[i-1], i) with t[j] > t[i]-w, else i;
 * end[i] = i+1. */
static void variable_bounds(const int64_t *t, int64_t n, int64_t w, int64_t *start, int64_t *end) {
    if (n == 0) return;
    start[0] = 0;
    end[0] = 1;
    for (int64_t i = 1; i < n; i++) {
        int64_t start_bound = t[i] - w;
        start[i] = i;
        for (int64_t j = start[i - 1]; j < i; j++) {
            if (t[j] - start_bound > 0) { start[i] = j; break; }
        }
        end[i] = i + 1;
    }
}

/* roll_sum over one segment; also returns the rolling count of non-NaN values
 * (Rolling.count = rolling sum of notna(), an exact integer). */
static void roll_sum_count(const double *v, const int64_t *start, const int64_t *end, int64_t n,
                           double *sum_out, double *cnt_out) {
    rsum_t s;
    int64_t cnt = 0;
    for (int64_t i = 0; i < n; i++) {
        int64_t st = start[i], en = end[i];
        if (i == 0 || st >= end[i - 1]) {
            rs_reset(&s, v[st]);
            cnt = 0;
            for (int64_t j = st; j < en; j++) { rs_add(&s, v[j]); cnt += (v[j] == v[j]); }
        } else {
            for (int64_t j = start[i - 1]; j < st; j++) { rs_remove(&s, v[j]); cnt -= (v[j] == v[j]); }
            for (int64_t j = end[i - 1]; j < en; j++) { rs_add(&s, v[j]); cnt += (v[j] == v[j]); }
        }
        /* rolling offset windows default to min_periods=1 */
        if (sum_out) sum_out[i] = rs_value(&s, 1);
        if (cnt_out) cnt_out[i] = (double)cnt;
    }
}

/*
 * get_customer_spending_behaviour_features (feature_transformation.ipynb:601-628), one
 * call per segment [seg_off[k], seg_off[k+1]) of rows already in per-key time order.
 * nb_out / avg_out are [n_windows][n] float64, same row order as the input.
 */
int oracle_customer_windows(const int64_t *ts_ns, const double *amount, const int64_t *seg_off,
                            int64_t n_seg, const int64_t *win_ns, int32_t n_win,
                            double *nb_out, double *avg_out) {
    int64_t n = seg_off[n_seg];
    int64_t maxlen = 0;
    for (int64_t k = 0; k < n_seg; k++) {
        int64_t L = seg_off[k + 1] - seg_off[k];
        if (L > maxlen) maxlen = L;
    }
    int64_t *st = (int64_t *)malloc(sizeof(int64_t) * (maxlen + 1));
    int64_t *en = (int64_t *)malloc(sizeof(int64_t) * (maxlen + 1));
    double *sm = (double *)malloc(sizeof(double) * (maxlen + 1));
    double *ct = (double *)malloc(sizeof(double) * (maxlen + 1));
    if (!st || !en || !sm || !ct) return -1;
    for (int64_t k = 0; k < n_seg; k++) {
        int64_t b = seg_off[k], L = seg_off[k + 1] - b;
        if (L <= 0) continue;
        for (int32_t w = 0; w < n_win; w++) {
            variable_bounds(ts_ns + b, L, win_ns[w], st, en);
            roll_sum_count(amount + b, st, en, L, sm, ct);
            for (int64_t i = 0; i < L; i++) {
                nb_out[(int64_t)w * n + b + i] = ct[i];
                avg_out[(int64_t)w * n + b + i] = sm[i] / ct[i];
            }
        }
    }
    free(st); free(en); free(sm); free(ct);
    return 0;
}

/*
 * get_count_risk_rolling_window (feature_transformation.ipynb:1495-1522), restated the
 * way the reference computes it: rolling sums/counts of TX_FRAUD over the delay window
 * and over delay+w, differences, NB_FRAUD/NB_TX, then fillna(0).
 */
int oracle_terminal_windows(const int64_t *ts_ns, const double *fraud, const int64_t *seg_off,
                            int64_t n_seg, int64_t delay_ns, const int64_t *win_ns, int32_t n_win,
                            double *nb_out, double *risk_out) {
    int64_t n = seg_off[n_seg];
    int64_t maxlen = 0;
    for (int64_t k = 0; k < n_seg; k++) {
        int64_t L = seg_off[k + 1] - seg_off[k];
        if (L > maxlen) maxlen = L;
    }
    size_t B = sizeof(double) * (maxlen + 1);
    int64_t *st = (int64_t *)malloc(sizeof(int64_t) * (maxlen + 1));
    int64_t *en = (int64_t *)malloc(sizeof(int64_t) * (maxlen + 1));
    double *sd = (double *)malloc(B), *cd = (double *)malloc(B);
    double *sw = (double *)malloc(B), *cw = (double *)malloc(B);
    if (!st || !en || !sd || !cd || !sw || !cw) return -1;
    for (int64_t k = 0; k < n_seg; k++) {
        int64_t b = seg_off[k], L = seg_off[k + 1] - b;
        if (L <= 0) continue;
        variable_bounds(ts_ns + b, L, delay_ns, st, en);
        roll_sum_count(fraud + b, st, en, L, sd, cd);
        for (int32_t w = 0; w < n_win; w++) {
            variable_bounds(ts_ns + b, L, delay_ns + win_ns[w], st, en);
            roll_sum_count(fraud + b, st, en, L, sw, cw);
            for (int64_t i = 0; i < L; i++) {
                double nb_fraud = sw[i] - sd[i];
                double nb_tx = cw[i] - cd[i];
                double risk = nb_fraud / nb_tx;
                if (risk != risk) risk = 0.0;      /* fillna(0) */
                if (nb_tx != nb_tx) nb_tx = 0.0;
                nb_out[(int64_t)w * n + b + i] = nb_tx;
                risk_out[(int64_t)w * n + b + i] = risk;
            }
        }
    }
    free(st); free(en); free(sd); free(cd); free(sw); free(cw);
    return 0;
}

/*
 * StandardScaler.transform + RandomForestClassifier.predict_proba(X)[:,1] with
 * sklearn's per-tree node arrays.  Trees are concatenated: tree t owns nodes
 * [node_off[t], node_off[t+1]); children indices are tree-local (-1 = leaf).
 * X is [n][n_feat] float64 (raw, unscaled when mean/scale are given).
 * leaf_out (optional) is [n][n_trees] int32, proba_out [n] float64.
 */
int oracle_forest_predict(const double *X, int64_t n, int32_t n_feat, const double *mean,
                          const double *scale, int32_t n_trees, const int64_t *node_off,
                          const int64_t *left, const int64_t *right, const int64_t *feature,
                          const double *threshold, const uint8_t *missing_left,
                          const double *value1, double *proba_out, int32_t *leaf_out) {
    float *x32 = (float *)malloc(sizeof(float) * n_feat);
    if (!x32) return -1;
    for (int64_t r = 0; r < n; r++) {
        for (int32_t f = 0; f < n_feat; f++) {
            double z = X[r * n_feat + f];
            if (mean) z -= mean[f];
            if (scale) z /= scale[f];
            x32[f] = (float)z;   /* _validate_X_predict: DTYPE float32 */
        }
        double acc = 0.0;
        for (int32_t t = 0; t < n_trees; t++) {
            int64_t base = node_off[t], i = 0;
            while (left[base + i] != -1) {
                float xv = x32[feature[base + i]];
                if (isnan(xv)) {
                    i = missing_left[base + i] ? left[base + i] : right[base + i];
                } else if ((double)xv <= threshold[base + i]) {
                    i = left[base + i];
                } else {
                    i = right[base + i];
                }
            }
            if (leaf_out) leaf_out[r * n_trees + t] = (int32_t)i;
            acc += value1[base + i];
        }
        proba_out[r] = acc / (double)n_trees;
    }
    free(x32);
    return 0;
}
