"""Eval-semantics scoring pipeline on the HIP path (drop-in for
src/evaluate.py:171-272).

The reference scores a split in three host-driven passes: news vectors cached
in a dict, user vectors cached per history string, then a Python loop with
batch size 1 over impressions (one get_prediction and one device->host sync
each), and finally per-impression AUC/MRR/nDCG in a process pool. Here every
pass is one (or a few) launches over flat index arrays built once on the
host:

  1. news vectors of the whole corpus: NRMS.get_news_vector (HIP NewsEncoder),
     plus one all-zero row for PADDED_NEWS (evaluate.py:203-204);
  2. user vectors of every distinct history string: the clicked-news rows are
     gathered from the news-vector table by nrms_embedding_gather and encoded
     by NRMS.get_user_vector (HIP UserEncoder);
  3. all impressions' candidate logits in one nrms_score_pairs launch;
  4. per-impression metrics in one nrms_impression_metrics launch, then the
     nanmean (evaluate.py:270-272) — or, across ranks, an all-reduce of
     (sum, count) per metric.
"""
import sys

import numpy as np
import torch

from . import _native as N
from .data import (PADDED_NEWS, BehaviorsTable, _index_rows, candidate_rows_numeric, history_ids,
                   history_rows_numeric, load_behaviors, numeric_news_index, parse_impression_cells,
                   read_news_parsed)


class EvalPlan:
    """Host-side index arrays for one split (built once, reused per model).

    The impressions cells of the split are parsed in one pass
    (data.parse_impression_cells) and every candidate / history id is mapped to
    its corpus row in one flat pass each (the reference looks candidates up
    inside its per-impression loop, src/evaluate.py:251-255); an unknown id
    raises KeyError as news2vector[...] does."""

    def __init__(self, corpus, impressions, max_count=sys.maxsize, num_clicked=50):
        # the reference breaks when count == max_count before scoring it
        # (src/evaluate.py:245-249): impressions 1..max_count-1 are scored
        n = len(impressions) if max_count > len(impressions) else max(0, max_count - 1)
        self.corpus = corpus
        self.num_clicked = num_clicked
        pad = len(corpus)
        if isinstance(impressions, BehaviorsTable):
            tab = impressions if n == len(impressions) else impressions[:n]
            nindex = numeric_news_index(corpus)
            if nindex is not None:
                self._from_table(tab, nindex, num_clicked, pad)
                return
            impressions = list(tab)   # (ids not in the numeric form: the per-name path)
        self.impressions = impressions[:n]
        # users keyed by history string, in first-seen order
        hist_of = {}
        hists = []
        imp_user = np.empty(n, dtype=np.int64)
        for k, im in enumerate(self.impressions):
            u = hist_of.get(im.clicked_news)
            if u is None:
                u = hist_of[im.clicked_news] = len(hists)
                hists.append(im.clicked_news)
            imp_user[k] = u
        rows_of = corpus.index   # news id -> first row (news2vector[...], evaluate.py:255)

        def lookup(names):
            return np.fromiter(map(rows_of.__getitem__, names), dtype=np.int64, count=len(names))

        # MIND-form cells ("N<digits>-<label>"): one numeric parse and an array
        # index (data.candidate_rows_numeric); any other form: the per-name path
        nindex = numeric_news_index(corpus)
        fast = candidate_rows_numeric(self.impressions, nindex)
        if fast is not None:
            self.cand, self.labels, counts = fast
        else:
            cand_names, self.labels, counts = parse_impression_cells(self.impressions)
            self.cand = lookup(cand_names).astype(np.int64) if cand_names else np.zeros(0, np.int64)
        self.pair_user = np.repeat(imp_user, counts)
        self.offsets = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        hrows = history_rows_numeric(hists, nindex, num_clicked, pad)
        if hrows is None:
            hist_names = [x for h in hists for x in history_ids(h, num_clicked)]
            real = np.array([x != PADDED_NEWS for x in hist_names], dtype=bool)
            rows = np.full(len(hist_names), pad, dtype=np.int64)
            if real.any():
                rows[real] = lookup([x for x, r in zip(hist_names, real) if r])
            hrows = rows.reshape(len(hists), num_clicked)
        self.hist_rows = hrows

    def _from_table(self, tab, nindex, num_clicked, pad):
        """The plan from a natively parsed split (data.BehaviorsTable): the
        same arrays as the Impression path's numeric fast path."""
        self.impressions = tab
        n = len(tab)
        self.cand = _index_rows(nindex, tab.cand_num)
        self.labels = tab.labels
        counts = tab.cand_count
        imp_user = tab.hist_user
        self.pair_user = np.repeat(imp_user, counts)
        self.offsets = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        # each distinct history's first line: its first num_clicked ids, left-padded
        _, first = np.unique(imp_user, return_index=True) if n else (None, np.zeros(0, np.int64))
        U = first.size
        hc, ho = tab.hist_count[first], tab.hist_off[first]
        m = np.minimum(hc, num_clicked)
        rows = np.full((U, num_clicked), pad, dtype=np.int64)
        if int(m.sum()):
            u = np.repeat(np.arange(U), m)
            k = np.arange(int(m.sum())) - np.repeat(np.cumsum(m) - m, m)
            rows[u, num_clicked - np.repeat(m, m) + k] = _index_rows(nindex, tab.hist_num[np.repeat(ho, m) + k])
        self.hist_rows = rows

    @property
    def n_impressions(self):
        return len(self.offsets) - 1


@torch.no_grad()
def news_vectors(model, titles, chunk=65536):
    """[n + 1, D] news-vector table on the model's device; last row = PADDED_NEWS."""
    ne = model.news_encoder
    dev = ne.word_embedding.weight.device
    D = ne.word_embedding.embedding_dim
    n = titles.shape[0]
    out = torch.zeros(n + 1, D, dtype=torch.float32, device=dev)
    t = torch.from_numpy(titles) if isinstance(titles, np.ndarray) else titles
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        out[a:b] = model.get_news_vector({"title": t[a:b]})
    return out


@torch.no_grad()
def user_vectors(model, news_tab, hist_rows, chunk=16384):
    """User vectors of every history: gather clicked rows (PADDED -> zero row)
    then the HIP UserEncoder."""
    dev = news_tab.device
    U, Nc = hist_rows.shape
    D = news_tab.shape[1]
    out = torch.empty(U, D, dtype=torch.float32, device=dev)
    rows = torch.from_numpy(hist_rows).to(dev)
    for a in range(0, U, chunk):
        r = rows[a:a + chunk].contiguous()
        b = r.shape[0]
        x = torch.empty(b * Nc, D, dtype=torch.float32, device=dev)
        N.call("nrms_embedding_gather", N.ptr(r), b * Nc, N.ptr(news_tab), news_tab.shape[0], D,
               N.ptr(x), N.stream_handle(dev))
        out[a:a + b] = model.get_user_vector(x.view(b, Nc, D))
    return out


@torch.no_grad()
def score_plan(model, plan):
    """Logits of every (impression, candidate) pair and the per-impression
    metric table [n_imp, 4] (AUC, MRR, nDCG@5, nDCG@10; fp64) on the device."""
    news_tab = news_vectors(model, plan.corpus.titles)
    dev = news_tab.device
    D = news_tab.shape[1]
    users = user_vectors(model, news_tab, plan.hist_rows)
    K = plan.cand.shape[0]
    scores = torch.empty(K, dtype=torch.float32, device=dev)
    cand = torch.from_numpy(plan.cand).to(dev)
    pu = torch.from_numpy(plan.pair_user).to(dev)
    st = N.stream_handle(dev)
    N.call("nrms_score_pairs", N.ptr(news_tab), news_tab.shape[0], N.ptr(users), users.shape[0],
           N.ptr(cand), N.ptr(pu), K, D, N.ptr(scores), st)
    labels = torch.from_numpy(plan.labels).to(dev)
    offsets = torch.from_numpy(plan.offsets).to(dev)
    metrics = torch.empty(plan.n_impressions, 4, dtype=torch.float64, device=dev)
    N.call("nrms_impression_metrics", N.ptr(scores), N.ptr(labels), N.ptr(offsets),
           plan.n_impressions, N.ptr(metrics), st)
    return scores, metrics


def nan_sums(metrics):
    """(sum, count) per metric column over non-NaN rows (fp64)."""
    ok = ~torch.isnan(metrics)
    return torch.where(ok, metrics, torch.zeros_like(metrics)).sum(0), ok.sum(0).to(torch.float64)


def reduce_means(sums, counts):
    with np.errstate(invalid="ignore"):
        return tuple(float(x) for x in (sums / counts).cpu().numpy())


@torch.no_grad()
def evaluate(model, directory, num_workers=4, max_count=sys.maxsize, process_group=None):
    """Same signature and return value as the reference's evaluate()
    (src/evaluate.py:171-184): (AUC, MRR, nDCG@5, nDCG@10) of the split in
    `directory` (news_parsed.tsv + behaviors.tsv). `num_workers` is accepted
    for compatibility (there is no process pool). With a torch.distributed
    `process_group`, each rank scores the impressions of its users
    (distributed.user_rank: user_id % world) and the metric sums are all-reduced."""
    import os
    corpus = read_news_parsed(os.path.join(directory, "news_parsed.tsv"))
    imps = load_behaviors(os.path.join(directory, "behaviors.tsv"))
    return evaluate_split(model, corpus, imps, max_count, process_group)


@torch.no_grad()
def evaluate_split(model, corpus, impressions, max_count=sys.maxsize, process_group=None):
    n = len(impressions) if max_count > len(impressions) else max(0, max_count - 1)
    imps = impressions[:n]
    if process_group is not None:
        from .distributed import shard_impressions
        import torch.distributed as dist
        imps = shard_impressions(imps, dist.get_rank(process_group), dist.get_world_size(process_group))
    plan = EvalPlan(corpus, imps, num_clicked=model.config.num_clicked_news_a_user)
    if plan.n_impressions:
        _, metrics = score_plan(model, plan)
        sums, counts = nan_sums(metrics)
    else:
        dev = model.news_encoder.word_embedding.weight.device
        sums = torch.zeros(4, dtype=torch.float64, device=dev)
        counts = torch.zeros(4, dtype=torch.float64, device=dev)
    if process_group is not None:
        from .distributed import all_reduce_sums
        sums, counts = all_reduce_sums(sums, counts, process_group)
    return reduce_means(sums, counts)
