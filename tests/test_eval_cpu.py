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


def _plan_per_name(monkeypatch, corpus, imps, **kw):
    """EvalPlan through the per-name (dict) paths only."""
    import newsrecommendationsystem_amd.evaluate as EV
    with monkeypatch.context() as m:
        m.setattr(EV, "candidate_rows_numeric", lambda *a: None)
        m.setattr(EV, "history_rows_numeric", lambda *a: None)
        return EV.EvalPlan(corpus, imps, **kw)


@pytest.mark.parametrize("num_clicked", [50, 3])
def test_numeric_plan_equals_per_name_plan(split, monkeypatch, num_clicked):
    """MIND-form ids ("N<digits>"): the numeric parse + array index
    (data.candidate_rows_numeric / history_rows_numeric) gives the same plan
    arrays as the per-name dict lookups of src/evaluate.py:115-124,251-255."""
    d, corpus, _ = split
    assert Dt.numeric_news_index(corpus) is not None
    imps = Dt.read_behaviors(d + "/behaviors.tsv") + [   # (the raw cells as read from the file)
        Dt.Impression("x1", "U9", "t", " ", ["N3", "N0"], [0, 1], raw="N3-0 N0-1"),
                   Dt.Impression("x2", "U9", "t", "N7 N8 N0", ["N7"], [1], raw="N7-1")]
    idx = Dt.numeric_news_index(corpus)
    hists = list(dict.fromkeys(im.clicked_news for im in imps))
    assert Dt.candidate_rows_numeric(imps, idx) is not None             # (the numeric paths are taken)
    assert Dt.history_rows_numeric(hists, idx, num_clicked, len(corpus)) is not None
    fast = EvalPlan(corpus, imps, num_clicked=num_clicked)
    slow = _plan_per_name(monkeypatch, corpus, imps, num_clicked=num_clicked)
    for k in ("cand", "labels", "pair_user", "offsets", "hist_rows"):
        a, b = getattr(fast, k), getattr(slow, k)
        assert a.dtype == b.dtype and np.array_equal(a, b), k


def test_numeric_paths_fall_back_or_raise():
    ids = ["N5", "N1", "N5", "N0"]                      # a repeated id keeps its first row
    corpus = Dt.NewsCorpus(ids, np.zeros((4, 20), np.int64))
    idx = Dt.numeric_news_index(corpus)
    assert idx[5] == 0 and idx[1] == 1 and idx[0] == 3 and idx[2] == -1
    assert Dt.numeric_news_index(Dt.NewsCorpus(["N01", "N1"], np.zeros((2, 20), np.int64))) is None
    assert Dt.numeric_news_index(Dt.NewsCorpus(["N1", "X2"], np.zeros((2, 20), np.int64))) is None
    imp = lambda raw: Dt.Impression("i", "u", "t", " ", [], [], raw=raw)
    rows, labs, counts = Dt.candidate_rows_numeric([imp("N5-1 N1-0"), imp("N0-0")], idx)
    assert rows.tolist() == [0, 1, 3] and labs.tolist() == [1, 0, 0] and counts.tolist() == [2, 1]
    for raw in ("N5-1  N1-0", "N05-1", "N5-1-2", "N5", "5-1", "N5-1 x"):   # not the plain form: per-name path
        assert Dt.candidate_rows_numeric([imp(raw)], idx) is None, raw
    with pytest.raises(KeyError):
        Dt.candidate_rows_numeric([imp("N5-1 N2-0")], idx)
    h = Dt.history_rows_numeric(["N1 N5 N0", " ", "N0"], idx, 2, 9)
    assert h.tolist() == [[1, 0], [9, 9], [9, 3]]           # first 2 ids, left-padded
    assert Dt.history_rows_numeric(["N1 PADDED_NEWS"], idx, 2, 9) is None
    assert Dt.history_rows_numeric(["N1  N5"], idx, 2, 9) is None   # (split() semantics kept by the per-name path)
    with pytest.raises(KeyError):
        Dt.history_rows_numeric(["N1 N7"], idx, 2, 9)


def test_sparse_large_numeric_ids_take_the_dict_path(tmp_path):
    """Ids far beyond the corpus size (or past int64's exact parse) must not
    build a dense index: numeric_news_index returns None and the per-name
    plan is used (a sparse 'N9999999999' corpus allocated ~80 GB)."""
    big = ["N9999999999", "N1", "N123456789012"]
    assert Dt.numeric_news_index(Dt.NewsCorpus(big, np.zeros((3, 20), np.int64))) is None
    huge = ["N" + "9" * 25, "N2"]                         # would overflow int64
    assert Dt.numeric_news_index(Dt.NewsCorpus(huge, np.zeros((2, 20), np.int64))) is None
    titles = np.arange(3 * 20, dtype=np.int64).reshape(3, 20)
    corpus = Dt.NewsCorpus(big, titles)
    imps = [Dt.Impression("1", "U1", "t", "N1 N9999999999", raw="N123456789012-1 N1-0")]
    plan = EvalPlan(corpus, imps, num_clicked=3)
    assert plan.cand.tolist() == [2, 1] and plan.labels.tolist() == [1, 0]
    assert plan.hist_rows.tolist() == [[len(corpus), 1, 0]]


def test_impression_setters_keep_the_other_field():
    """Setting candidates (or labels) on an Impression read from a raw cell
    parses the cell first, so the other field stays readable."""
    im = Dt.Impression("1", "U1", "t", " ", raw="N1-1 N2-0")
    im.candidates = ["N7", "N8"]
    assert im.labels == [1, 0] and im.candidates == ["N7", "N8"]
    im = Dt.Impression("1", "U1", "t", " ", raw="N1-1 N2-0")
    im.labels = [0, 0]
    assert im.candidates == ["N1", "N2"] and im.labels == [0, 0]



# ---------------------------------------------------------------- native readers (csrc/tsv_io.hip)
def _write(path, text):
    with open(path, "w", newline="") as f:
        f.write(text)


def test_native_readers_equal_python_readers(split):
    """nrms_news_parse / nrms_behaviors_parse (host C++, ABI 7) give the
    corpus, the impressions' columns and the EvalPlan arrays of the Python
    readers (data.read_news_parsed_py, read_behaviors + the numeric fast path,
    themselves pinned to the reference's per-token split / literal_eval)."""
    d, _, _ = split
    nat = Dt.read_news_parsed_native(d + "/news_parsed.tsv")
    py = Dt.read_news_parsed_py(d + "/news_parsed.tsv")
    assert nat is not None and nat.ids == py.ids and np.array_equal(nat.titles, py.titles)
    assert np.array_equal(Dt.numeric_news_index(nat), Dt.numeric_news_index(py))
    tab = Dt.read_behaviors_native(d + "/behaviors.tsv")
    imps = Dt.read_behaviors(d + "/behaviors.tsv")
    assert isinstance(tab, Dt.BehaviorsTable) and len(tab) == len(imps)
    for a, b in zip(tab, imps):
        assert (a.impression_id, a.user, a.time, a.clicked_news, a.raw) == \
               (b.impression_id, b.user, b.time, b.clicked_news, b.raw)
    for mc in (sys.maxsize, 1, 2, 7):
        p1, p2 = EvalPlan(nat, tab, max_count=mc), EvalPlan(py, imps, max_count=mc)
        for k in ("cand", "labels", "pair_user", "offsets", "hist_rows"):
            a, b = getattr(p1, k), getattr(p2, k)
            assert a.dtype == b.dtype and np.array_equal(a, b), (mc, k)


def test_native_behaviors_edge_forms(tmp_path):
    """Blank and space-padded histories, a repeated history string, "N0",
    multi-digit labels, fewer lines than the scan's bound: the native table
    equals the Python reader; non-plain forms (CRLF, double spaces, a leading
    zero, a missing column, non-ASCII) return None so the general path runs."""
    corpus = Dt.NewsCorpus([f"N{i}" for i in range(12)], np.arange(240).reshape(12, 20))
    text = ("1\tU1\tt\t\tN3-1 N0-0\n"
            "2\tU2\tt\t N1 N2 \tN5-01 N6-0\n\n"
            "3\tU1\tt\t\tN7-1\n"
            "4\tU9\tt\tN1 N2\tN11-0 N10-1 N9-0\textra\n")
    p = str(tmp_path / "b.tsv")
    _write(p, text)
    tab = Dt.read_behaviors_native(p)
    imps = Dt.read_behaviors(p)
    assert tab is not None and len(tab) == 4
    assert [im.clicked_news for im in tab] == [im.clicked_news for im in imps] == [" ", " N1 N2 ", " ", "N1 N2"]
    assert tab.hist_user.tolist() == [0, 1, 0, 2]
    p1, p2 = EvalPlan(corpus, tab, num_clicked=3), EvalPlan(corpus, imps, num_clicked=3)
    for k in ("cand", "labels", "pair_user", "offsets", "hist_rows"):
        assert np.array_equal(getattr(p1, k), getattr(p2, k)), k
    assert p1.labels.tolist() == [1, 0, 1, 0, 1, 0, 1, 0]
    shard = Dt.BehaviorsTable.select(tab, [1, 3])
    assert [im.impression_id for im in shard] == ["2", "4"] and shard.hist_user.tolist() == [0, 1]
    for bad in ("1\tU1\tt\tN1\tN3-1\r\n", "1\tU1\tt\tN1  N2\tN3-1\n", "1\tU1\tt\tN01\tN3-1\n",
                "1\tU1\tt\tN1\tN3-1  N4-0\n", "1\tU1\tt\tN1\n", "1\tU1\tt\tN1\tN3-1 \n", "1\tUé\tt\tN1\tN3-1\n",
                "1\tU1\tt\tN1\tN3-\n", "1\tU1\tt\tN1\tN03-1\n"):
        _write(p, bad)
        assert Dt.read_behaviors_native(p) is None, repr(bad)
    n = str(tmp_path / "n.tsv")
    _write(n, "id\tcategory\ttitle\nN1\tx\t[1, 2]\nN2\ty\t[3,4]\n")
    c = Dt.read_news_parsed_native(n, num_words_title=2)
    assert c.ids == ["N1", "N2"] and c.titles.tolist() == [[1, 2], [3, 4]] and c.numeric.tolist() == [1, 2]
    for bad in ("id\ttitle\nN1\t[1, 2, 3]\n", "id\ttitle\nN01\t[1, 2]\n", "id\ttitle\nX1\t[1, 2]\n",
                "id\ttitle\nN1\t(1, 2)\n", "idx\ttitle\nN1\t[1, 2]\n", "id\ttitle\r\nN1\t[1, 2]\r\n"):
        _write(n, bad)
        assert Dt.read_news_parsed_native(n, num_words_title=2) is None, repr(bad)


def test_behaviors_parse_checks_bytes_without_scan():
    """nrms_behaviors_parse called without a preceding nrms_behaviors_scan
    rejects a non-plain buffer itself (non-ASCII user column, CR line end):
    NRMS_ERR_UNSUPPORTED, as the header promises (round-4 advisor finding)."""
    from newsrecommendationsystem_amd import _native as N
    lib = N.load()
    P = lambda a: a.ctypes.data
    for text in ("1\tU\xe9\tt\tN1\tN3-1\n", "1\tU1\tt\tN1\tN3-1\r\n", "1\tU1\tt\tN1\tN3-1\n"):
        buf = text.encode("utf-8")
        cap = np.array([4, 8, 8], np.int64)
        fields = np.zeros((4, 5, 2), np.int64)
        cand_num, labels, cand_count = np.zeros(8, np.int64), np.zeros(8, np.int32), np.zeros(4, np.int64)
        hist_num, hist_count, hist_user = np.zeros(8, np.int64), np.zeros(4, np.int64), np.zeros(4, np.int64)
        counts = np.zeros(4, np.int64)
        st = lib.nrms_behaviors_parse(buf, len(buf), P(cap), P(counts), P(fields), P(cand_num), P(labels),
                                      P(cand_count), P(hist_num), P(hist_count), P(hist_user))
        if text.endswith("N3-1\n") and "\xe9" not in text:
            assert st == N.NRMS_OK and counts[0] == 1 and cand_num[0] == 3 and labels[0] == 1
        else:
            assert st == N.NRMS_ERR_UNSUPPORTED, repr(text)
