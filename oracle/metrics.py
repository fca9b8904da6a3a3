"""Restatement of the reference's per-impression ranking metrics — TEST INFRA.

src/evaluate.py:24-42 (dcg/ndcg/mrr) and :160-168 (per-impression AUC via
sklearn.metrics.roc_auc_score; NaN for all-equal labels), :270-272 (nanmean
over impressions). AUC is restated as the Mann-Whitney statistic with average
ranks for ties, which is what roc_auc_score computes for binary labels.
"""
import numpy as np


def dcg_score(y_true, y_score, k=10):
    order = np.argsort(y_score)[::-1]
    gains = 2 ** np.take(y_true, order[:k]) - 1
    return float(np.sum(gains / np.log2(np.arange(len(gains)) + 2)))


def ndcg_score(y_true, y_score, k=10):
    return dcg_score(y_true, y_score, k) / dcg_score(y_true, y_true, k)


def mrr_score(y_true, y_score):
    order = np.argsort(y_score)[::-1]
    yt = np.take(y_true, order)
    return float(np.sum(yt / (np.arange(len(yt)) + 1)) / np.sum(yt))


def auc_score(y_true, y_score):
    y_true = np.asarray(y_true)
    y_score = np.asarray(y_score, dtype=np.float64)
    n_pos = int((y_true == 1).sum())
    n_neg = len(y_true) - n_pos
    if n_pos == 0 or n_neg == 0:
        raise ValueError("Only one class present in y_true")
    order = np.argsort(y_score, kind="mergesort")
    s = y_score[order]
    ranks = np.empty(len(s))
    i = 0
    while i < len(s):
        j = i
        while j + 1 < len(s) and s[j + 1] == s[i]:
            j += 1
        ranks[i:j + 1] = 0.5 * (i + j) + 1.0
        i = j + 1
    r = np.empty(len(s))
    r[order] = ranks
    return float((r[y_true == 1].sum() - n_pos * (n_pos + 1) / 2.0) / (n_pos * n_neg))


def single_impression(y_true, y_score):
    """calculate_single_user_metric (src/evaluate.py:160-168)."""
    try:
        return [auc_score(y_true, y_score), mrr_score(y_true, y_score),
                ndcg_score(y_true, y_score, 5), ndcg_score(y_true, y_score, 10)]
    except ValueError:
        return [np.nan] * 4


def aggregate(pairs):
    """nanmean of per-impression metrics (src/evaluate.py:267-272)."""
    res = np.array([single_impression(t, s) for t, s in pairs], dtype=np.float64)
    if res.size == 0:
        return (np.nan,) * 4
    with np.errstate(all="ignore"):
        return tuple(float(np.nanmean(res[:, i])) for i in range(4))
