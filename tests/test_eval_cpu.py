"""Eval pipeline host logic, file formats and the CPU eval oracle (no GPU)."""
import sys

import numpy as np
import pytest

from newsrecommendationsystem_amd import data as Dt
from newsrecommendationsystem_amd.evaluate import EvalPlan
from oracle import eval_oracle as EO
from oracle import metrics as M
from oracle import weights as W


@pytest.fixture(scope="module")
def split(tmp_path_factory):
    d = tmp_path_factory.mktemp("split")
    corpus, imps = Dt.synthetic_split(str(d), seed=3, n_news=300, n_users=40, n_impressions=120, V=512)
    return str(d), corpus, imps


def test_formats_round_trip(split):
    d, corpus, imps = split
    c2 = Dt.read_news_parsed(d + "/news_parsed.tsv")
    assert c2.ids == corpus.ids and np.array_equal(c2.titles, corpus.titles)
    i2 = Dt.read_behaviors(d + "/behaviors.tsv")
    assert len(i2) == len(imps)
    for a, b in zip(i2, imps):
        assert (a.user, a.candidates, a.labels) == (b.user, b.candidates, b.labels)
        assert a.clicked_news.split() == b.clicked_news.split()


def test_history_padding_and_truncation():
    h = " ".join(f"N{i}" for i in range(70))
    ids = Dt.history_ids(h, 50)
    assert ids == [f"N{i}" for i in range(50)]            # first 50 kept
    assert Dt.history_ids(" ", 50) == [Dt.PADDED_NEWS] * 50
    assert Dt.history_ids("N1 N2", 4) == [Dt.PADDED_NEWS] * 2 + ["N1", "N2"]


def test_plan_layout(split):
    _, corpus, imps = split
    plan = EvalPlan(corpus, imps)
    assert plan.n_impressions == len(imps)
    assert plan.offsets[-1] == sum(len(i.candidates) for i in imps)
    # every impression's candidates and history resolve to the same news
    for k, im in enumerate(imps[:20]):
        a, b = plan.offsets[k], plan.offsets[k + 1]
        assert [corpus.ids[i] for i in plan.cand[a:b]] == im.candidates
        assert list(plan.labels[a:b]) == im.labels
        u = plan.pair_user[a]
        row = [Dt.PADDED_NEWS if i == len(corpus) else corpus.ids[i] for i in plan.hist_rows[u]]
        assert row == Dt.history_ids(im.clicked_news)
    # one user vector per distinct history string
    assert plan.hist_rows.shape[0] == len({im.clicked_news for im in imps})


@pytest.mark.parametrize("max_count", [1, 2, 10, sys.maxsize])
def test_max_count_semantics(split, max_count):
    # reference breaks when count == max_count before scoring: max_count - 1 scored
    _, corpus, imps = split
    plan = EvalPlan(corpus, imps, max_count=max_count)
    assert plan.n_impressions == min(len(imps), max_count - 1)


def test_unknown_news_id_raises(split):
    _, corpus, imps = split
    bad = Dt.Impression("x", "U1", "t", "N1 NOPE", ["N1"], [1])
    with pytest.raises(KeyError):
        EvalPlan(corpus, [bad])


def test_eval_oracle_self_consistent(split):
    _, corpus, imps = split
    sd = W.nrms_state(5, 512)
    means, per, tasks = EO.evaluate(sd, corpus, imps[:30])
    assert per.shape == (29, 4) or per.shape == (30, 4)
    assert np.allclose(means, M.aggregate([(np.array(t), np.array(p)) for t, p in tasks]),
                       equal_nan=True)


def test_planted_teacher_gives_informative_auc(tmp_path):
    sd = W.nrms_state(9, 512)
    corpus, imps = Dt.synthetic_split(str(tmp_path), seed=4, n_news=200, n_users=30,
                                      n_impressions=80, V=512, teacher=EO.teacher(sd),
                                      temperature=0.5)
    means, _, _ = EO.evaluate(sd, corpus, imps)
    assert means[0] > 0.6   # the teacher's own scores rank its labels well


def _raw(cell):
    return Dt.Impression("1", "U1", "t", " ", raw=cell)


@pytest.mark.parametrize("cells", [
    ["N1-0 N2-1", "N3-1"],                 # the MIND form: one pass over the joined cells
    ["N1-10 N2-1", "N3-0"],                # multi-digit label: the int parse
    ["N-1-0 N2-1"],                        # an id holding '-': per-token split('-'), as the reference
    ["N1-0  N2-1 ", " N3-1"],              # ragged whitespace
])
def test_impression_cell_parse_matches_per_token_split(cells):
    """parse_impression_cells == the reference's per-token x.split('-')[0] /
    int(x.split('-')[1]) (src/evaluate.py:153-157) on every cell form."""
    imps = [_raw(c) for c in cells]
    names, labels, counts = Dt.parse_impression_cells(imps)
    want_n = [t.split("-")[0] for c in cells for t in c.split()]
    want_l = [int(t.split("-")[1]) for c in cells for t in c.split()]
    assert names == want_n and labels.tolist() == want_l and labels.dtype == np.int32
    assert counts.tolist() == [len(c.split()) for c in cells]
    # the lazily parsed per-impression view agrees
    assert [c for im in imps for c in im.candidates] == want_n
    assert [y for im in imps for y in im.labels] == want_l


def test_impression_cell_without_label_raises():
    # a token with no '-<label>' (MIND's test split) fails as in the reference
    with pytest.raises(IndexError):
        Dt.parse_impression_cells([_raw("N1 N2-1")])


def test_title_cells_parse_matches_literal_eval():
    """read_news_parsed's one-pass title parse == ast.literal_eval per cell,
    including the fallback for a cell that is not a plain list of L ints."""
    import ast
    cells = ["[1, 2, 0]", "[7,8,9]", "[0, 0, 0]"]
    got = Dt._parse_titles(cells, ["a", "b", "c"], 3)
    assert got.tolist() == [ast.literal_eval(c) for c in cells]
    odd = ["[1, 2, 3]", "(4, 5, 6)"]                          # a tuple literal: per-cell path
    assert Dt._parse_titles(odd, ["a", "b"], 3).tolist() == [[1, 2, 3], [4, 5, 6]]
    with pytest.raises(ValueError):
        Dt._parse_titles(["[1, 2]"], ["a"], 3)
