"""On-disk formats of the reference and a synthetic MIND-shaped generator.

Readers (host side, build the id arrays the HIP path consumes):
  * news_parsed.tsv   id, category, subcategory, title, abstract, title_entities,
                      abstract_entities — title is a python list literal of
                      num_words_title ints (src/data_preprocess.py:115-139,205,239;
                      read by src/evaluate.py:55-71, src/dataset.py:28-43)
  * behaviors.tsv     raw MIND rows without header: impression_id, user, time,
                      clicked_news (space separated), impressions ("N1-1 N2-0 ...")
                      (src/evaluate.py:133-157)
  * behaviors_parsed.tsv  user, clicked_news, candidate_news, clicked (train
                      split, src/data_preprocess.py:71-81; src/dataset.py:64-85)
  * pretrained_word_embedding.npy  float [V, 300] (src/data_preprocess.py:280,
                      loaded at src/train.py:76-80)

Writers produce the same formats for the synthetic generator (MIND data and
GloVe are not available offline).
"""
import ast
import csv
import os

import numpy as np

NUM_WORDS_TITLE = 20
NUM_CLICKED = 50
PADDED_NEWS = "PADDED_NEWS"


# ---------------------------------------------------------------- readers
class NewsCorpus:
    """news_parsed.tsv: ids (str), titles int64 [n, L]; id -> first row (the
    reference keeps the first vector per id, src/evaluate.py:197-201).
    `numeric` (optional): the ids' numbers when every id is "N<digits>"
    without a leading zero (the native reader's parse; numeric_news_index
    then skips its string pass)."""

    def __init__(self, ids, titles, numeric=None):
        self.ids = list(ids)
        self.titles = np.ascontiguousarray(titles, dtype=np.int64)
        self.numeric = numeric
        self.index = {}
        for i, nid in enumerate(self.ids):
            self.index.setdefault(nid, i)

    def __len__(self):
        return len(self.ids)


def _parse_titles(cells, ids, num_words_title):
    """The title column's python list literals ("[12, 7, 0, ...]",
    src/data_preprocess.py:205,239) -> int64 [n, L]: one numpy parse of all
    cells when every cell is a plain list of L ints, ast.literal_eval per cell
    otherwise (same values, same errors)."""
    inner = [c.strip() for c in cells]
    plain = all(c.startswith("[") and c.endswith("]") and c.count(",") == num_words_title - 1 for c in inner)
    if plain and inner:
        body = ",".join(c[1:-1] for c in inner)
        vals = np.array(body.split(","), dtype=np.int64) if body.strip() else np.zeros(0, np.int64)
        if vals.size == len(inner) * num_words_title:
            return vals.reshape(-1, num_words_title)
    titles = []
    for nid, c in zip(ids, cells):
        t = ast.literal_eval(c)
        if len(t) != num_words_title:
            raise ValueError(f"title of {nid} has {len(t)} ids, expected {num_words_title}")
        titles.append(t)
    return np.array(titles, dtype=np.int64).reshape(-1, num_words_title)


def _read_bytes(path):
    with open(path, "rb") as f:
        return f.read()


def read_news_parsed_native(path, num_words_title=NUM_WORDS_TITLE):
    """news_parsed.tsv through the native reader (nrms_news_parse: one C++ pass
    over the bytes), or None when the file is not in its plain MIND form (the
    caller then reads it with read_news_parsed's general path)."""
    import ctypes
    from . import _native as N
    buf = _read_bytes(path)
    cap = buf.count(b"\n") + 1
    ids = np.empty(cap, np.int64)
    spans = np.empty((cap, 2), np.int64)
    titles = np.empty((cap, num_words_title), np.int64)
    n = ctypes.c_int64(0)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    st = N.load().nrms_news_parse(buf, len(buf), num_words_title, ctypes.byref(n), P(ids), P(spans),
                                  P(titles), cap)
    if st == N.NRMS_ERR_UNSUPPORTED:
        return None
    N.check(st, "nrms_news_parse")
    n = n.value
    text = buf.decode("ascii")
    names = [text[a:b] for a, b in spans[:n].tolist()]
    return NewsCorpus(names, titles[:n], numeric=ids[:n].copy())


def read_news_parsed(path, num_words_title=NUM_WORDS_TITLE):
    """news_parsed.tsv -> NewsCorpus: the native reader for the plain MIND
    form, else the csv module + _parse_titles (every form the reference's
    pandas reader takes as a plain tab-separated table)."""
    fast = read_news_parsed_native(path, num_words_title)
    if fast is not None:
        return fast
    return read_news_parsed_py(path, num_words_title)


def read_news_parsed_py(path, num_words_title=NUM_WORDS_TITLE):
    ids, cells = [], []
    with open(path, newline="") as f:
        rd = csv.reader(f, delimiter="\t", quoting=csv.QUOTE_NONE)
        header = next(rd)
        ci, ct = header.index("id"), header.index("title")
        for row in rd:
            ids.append(row[ci])
            cells.append(row[ct])
    return NewsCorpus(ids, _parse_titles(cells, ids, num_words_title))


class Impression:
    """One behaviors.tsv row. `candidates` / `labels` are parsed from the raw
    impressions cell ("N1-0 N2-1 ...") on first use (src/evaluate.py:153-157:
    x.split('-')[0] / int(x.split('-')[1])); EvalPlan parses the cells of a
    whole split in one pass instead."""
    __slots__ = ("impression_id", "user", "time", "clicked_news", "raw", "_cands", "_labels")

    def __init__(self, impression_id, user, time, clicked_news, candidates=None, labels=None, raw=None):
        self.impression_id = impression_id
        self.user = user
        self.time = time
        self.clicked_news = clicked_news      # the raw history string (user-cache key)
        self.raw = raw                        # the raw impressions cell, or None
        self._cands = candidates              # list of news ids
        self._labels = labels                 # list of int

    def _parse(self):
        toks = [t.split("-") for t in self.raw.split()]
        self._cands = [t[0] for t in toks]
        self._labels = [int(t[1]) for t in toks]

    @property
    def candidates(self):
        if self._cands is None:
            self._parse()
        return self._cands

    @candidates.setter
    def candidates(self, v):
        if self._labels is None and self.raw is not None:
            self._parse()
        self._cands, self.raw = v, None

    @property
    def labels(self):
        if self._labels is None:
            self._parse()
        return self._labels

    @labels.setter
    def labels(self, v):
        if self._cands is None and self.raw is not None:
            self._parse()
        self._labels, self.raw = v, None


class BehaviorsTable:
    """A behaviors.tsv split parsed by the native reader (nrms_behaviors_parse)
    into flat arrays: per impression the candidates' numeric ids, labels and
    counts, the history ids, and the index of its history string among the
    split's distinct histories (first-seen order). Indexing or iterating
    yields Impression objects built from the raw columns, as read_behaviors
    would; slicing and select() give sub-tables (EvalPlan's max_count
    truncation, the user sharding)."""

    def __init__(self, text, fields, cand_num, labels, cand_count, hist_num, hist_count, hist_user):
        self.text = text
        self.fields = fields                  # [n, 5, 2] byte spans of the columns
        self.cand_num, self.labels, self.cand_count = cand_num, labels, cand_count
        self.hist_num, self.hist_count = hist_num, hist_count
        self.hist_user = hist_user            # distinct-history index (first-seen order)
        self.cand_off = np.concatenate([[0], np.cumsum(cand_count)]).astype(np.int64)
        self.hist_off = np.concatenate([[0], np.cumsum(hist_count)]).astype(np.int64)

    def __len__(self):
        return self.fields.shape[0]

    def _col(self, k, c):
        a, b = self.fields[k, c]
        return self.text[a:b]

    def _impression(self, k):
        hist = self._col(k, 3)
        return Impression(self._col(k, 0), self._col(k, 1), self._col(k, 2), hist if hist != "" else " ",
                          raw=self._col(k, 4))

    def __getitem__(self, k):
        if isinstance(k, slice):
            return self.select(np.arange(len(self))[k])
        return self._impression(int(k))

    def __iter__(self):
        return (self._impression(k) for k in range(len(self)))

    def users(self):
        """The user column of every impression (str)."""
        return [self.text[a:b] for a, b in self.fields[:, 1].tolist()]

    def select(self, rows):
        """Sub-table of the impressions `rows` (increasing), history indices
        renumbered in first-seen order."""
        rows = np.asarray(rows, dtype=np.int64)
        cs = _ranges(self.cand_off[rows], self.cand_count[rows])
        hs = _ranges(self.hist_off[rows], self.hist_count[rows])
        _, first, inv = np.unique(self.hist_user[rows], return_index=True, return_inverse=True)
        rank = np.empty(first.size, np.int64)
        rank[np.argsort(first, kind="stable")] = np.arange(first.size)
        return BehaviorsTable(self.text, self.fields[rows], self.cand_num[cs], self.labels[cs],
                              self.cand_count[rows], self.hist_num[hs], self.hist_count[rows],
                              rank[inv.reshape(-1)])


def _ranges(starts, counts):
    """Concatenated aranges [s, s + c) (int64)."""
    counts = np.asarray(counts, np.int64)
    tot = int(counts.sum())
    if tot == 0:
        return np.zeros(0, np.int64)
    off = np.cumsum(counts) - counts
    return np.repeat(np.asarray(starts, np.int64) - off, counts) + np.arange(tot)


def read_behaviors_native(path):
    """behaviors.tsv through the native reader (nrms_behaviors_scan /
    _parse: one C++ pass over the bytes) as a BehaviorsTable, or None when the
    file is not in the plain MIND form (read_behaviors' general path)."""
    import ctypes
    from . import _native as N
    lib = N.load()
    buf = _read_bytes(path)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    cap = np.zeros(3, np.int64)
    st = lib.nrms_behaviors_scan(buf, len(buf), P(cap))
    if st == N.NRMS_ERR_UNSUPPORTED:
        return None
    N.check(st, "nrms_behaviors_scan")
    n, nc, nh = (int(x) for x in cap)
    fields = np.empty((n, 5, 2), np.int64)
    cand_num, labels, cand_count = np.empty(nc, np.int64), np.empty(nc, np.int32), np.empty(n, np.int64)
    hist_num, hist_count, hist_user = np.empty(nh, np.int64), np.empty(n, np.int64), np.empty(n, np.int64)
    counts = np.zeros(4, np.int64)
    st = lib.nrms_behaviors_parse(buf, len(buf), P(cap), P(counts), P(fields), P(cand_num), P(labels),
                                  P(cand_count), P(hist_num), P(hist_count), P(hist_user))
    if st == N.NRMS_ERR_UNSUPPORTED:
        return None
    N.check(st, "nrms_behaviors_parse")
    n, nc, nh = (int(x) for x in counts[:3])
    return BehaviorsTable(buf.decode("ascii"), fields[:n], cand_num[:nc], labels[:nc], cand_count[:n],
                          hist_num[:nh], hist_count[:n], hist_user[:n])


def load_behaviors(path):
    """behaviors.tsv as evaluate() reads it: a BehaviorsTable from the native
    reader for the plain MIND form, else read_behaviors' list of Impression."""
    tab = read_behaviors_native(path)
    return tab if tab is not None else read_behaviors(path)


def read_behaviors(path):
    """Raw behaviors.tsv (header=None). An empty history becomes ' ' like the
    reference's fillna(' ') (src/evaluate.py:91,142)."""
    out = []
    with open(path, newline="") as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            cols = line.split("\t")
            cols += [""] * (5 - len(cols))
            hist = cols[3] if cols[3] != "" else " "
            out.append(Impression(cols[0], cols[1], cols[2], hist, raw=cols[4]))
    return out


_DIGITS = str.maketrans("", "", "0123456789")


def numeric_news_index(corpus):
    """int64 array: numeric part of a MIND news id ("N<digits>") -> the id's
    first corpus row (-1: absent), or None unless every corpus id is exactly
    "N" followed by digits without a leading zero (so that the number
    identifies the string). Also None (the per-name dict path) when an id has
    more than 18 digits (past int64's exact parse) or the largest number is
    far beyond the corpus size (the dense index would be mostly empty)."""
    ids = corpus.ids
    if not ids:
        return None
    n = len(ids)
    nums = getattr(corpus, "numeric", None)
    if nums is None:
        if max(map(len, ids)) > 19:
            return None
        joined = " ".join(ids)
        if (joined.translate(_DIGITS) != " ".join(["N"] * n) or joined.count("N0") != joined.count("N0 ") + (
                1 if joined.endswith("N0") else 0)):
            return None
        nums = np.fromstring(joined.replace("N", " "), dtype=np.int64, sep=" ")
        if nums.size != n:
            return None
    uniq, first = np.unique(nums, return_index=True)   # (the first row of a repeated id)
    if int(uniq[-1]) > 16 * n + (1 << 20):
        return None
    index = np.full(int(uniq[-1]) + 1, -1, dtype=np.int64)
    index[uniq] = first
    return index


def _index_rows(index, ids):
    """corpus rows of numeric ids (KeyError naming the first unknown id)."""
    known = ids < index.size
    rows = np.full(ids.size, -1, dtype=np.int64)
    rows[known] = index[ids[known]]
    if (rows < 0).any():
        raise KeyError("N%d" % int(ids[int(np.argmax(rows < 0))]))
    return rows


def candidate_rows_numeric(impressions, index):
    """(corpus rows int64, labels int32, per-impression counts) of every
    candidate of a split, in order, by one numeric parse of the joined raw
    cells -- or None unless every cell is single-space separated
    "N<digits>-<digits>" tokens (no leading zeros in the ids), the form whose
    parse equals the per-token split('-') and news2vector[...] lookup of
    src/evaluate.py:153-157,251-255. An id missing from the corpus raises
    KeyError as the dict does."""
    n = len(impressions)
    raws = [im.raw for im in impressions]
    if index is None or not n or any(r is None or r == "" for r in raws):
        return None
    joined = "\n".join(raws)
    buf = np.frombuffer(joined.encode("ascii", "replace"), dtype=np.uint8)
    seps = np.flatnonzero((buf == 32) | (buf == 10))
    ntok = seps.size + 1
    # the digit-free skeleton must be exactly "N- N- ... N-" (one line per impression)
    if joined.replace("\n", " ").translate(_DIGITS) != " ".join(["N-"] * ntok):
        return None
    if joined.count("N0") != joined.count("N0-"):   # (a leading zero: the string is not the number's)
        return None
    vals = np.fromstring(joined.replace("N", " ").replace("-", " "), dtype=np.int64, sep=" ")
    if vals.size != 2 * ntok:
        return None
    # tokens per impression: the separators before each line break, + 1
    is_nl = buf[seps] == 10
    ends = np.append(np.flatnonzero(is_nl), seps.size)          # separator index of each line's end
    counts = np.diff(np.concatenate([[-1], ends])).astype(np.int64)
    return _index_rows(index, vals[0::2]), vals[1::2].astype(np.int32), counts


def history_rows_numeric(histories, index, num_clicked, pad_row):
    """[len(histories), num_clicked] corpus rows of each history's first
    num_clicked ids, left-padded with pad_row (history_ids +
    news2vector[...], src/evaluate.py:115-124) -- or None unless every
    history is single-space separated "N<digits>" ids (no leading zeros) or
    blank."""
    if index is None:
        return None
    hs = [h.strip() for h in histories]
    cnt = np.fromiter((h.count("N") for h in hs), dtype=np.int64, count=len(hs))
    total = int(cnt.sum())
    rows = np.full((len(hs), num_clicked), pad_row, dtype=np.int64)
    if total == 0:
        return rows if all(h == "" for h in hs) else None
    joined = " ".join(h for h in hs if h)
    if joined.translate(_DIGITS) != " ".join(["N"] * total):
        return None
    if joined.count("N0") != joined.count("N0 ") + (1 if joined.endswith("N0") else 0):
        return None
    nums = np.fromstring(joined.replace("N", " "), dtype=np.int64, sep=" ")
    if nums.size != total:
        return None
    m = np.minimum(cnt, num_clicked)                 # ids kept per history (the first m)
    off = np.cumsum(cnt) - cnt                       # first id of each history in nums
    u = np.repeat(np.arange(len(hs)), m)
    k = np.arange(int(m.sum())) - np.repeat(np.cumsum(m) - m, m)
    rows[u, num_clicked - np.repeat(m, m) + k] = _index_rows(index, nums[np.repeat(off, m) + k])
    return rows


def parse_impression_cells(impressions):
    """(candidate ids, labels int32, per-impression counts) of a split, in
    order. One split of the joined raw cells when every token is `<id>-<label>`
    with a single '-' (then identical to the per-token split('-') of
    src/evaluate.py:153-157); the per-impression parse otherwise."""
    n = len(impressions)
    raws = [im.raw for im in impressions]
    if n and all(r is not None for r in raws):
        joined = " ".join(raws)
        parts = joined.replace("-", " ").split()
        counts = np.fromiter((r.count("-") for r in raws), dtype=np.int64, count=n)
        ntok = int(counts.sum())
        # every token holds exactly one '-' with text on both sides
        if len(parts) == 2 * ntok and len(joined.split()) == ntok:
            labs = parts[1::2]
            flat = "".join(labs)
            if len(flat) == ntok and flat.isdigit():   # single-digit labels (MIND's 0/1)
                labs = np.frombuffer(flat.encode(), dtype=np.uint8).astype(np.int32) - 48
            else:
                labs = np.array(labs, dtype=np.int64).astype(np.int32)
            return parts[0::2], labs, counts
    names = [c for im in impressions for c in im.candidates]
    labs = np.fromiter((y for im in impressions for y in im.labels), dtype=np.int64, count=len(names))
    counts = np.fromiter((len(im.candidates) for im in impressions), dtype=np.int64, count=n)
    return names, labs.astype(np.int32), counts


def history_ids(history_string, num_clicked=NUM_CLICKED):
    """First num_clicked ids of the history, left-padded with PADDED_NEWS
    (src/evaluate.py:115-124)."""
    h = history_string.split()[:num_clicked]
    return [PADDED_NEWS] * (num_clicked - len(h)) + h


def read_behaviors_parsed(path, corpus, num_clicked=NUM_CLICKED):
    """Train-split rows -> (candidates [n, 1+K, L], clicked [n, N, L], clicked
    labels [n, 1+K]): the batch contract of BaseDataset.__getitem__
    (src/dataset.py:64-85): history truncated to its first N, left-padded with
    all-zero titles."""
    L = corpus.titles.shape[1]
    cands, clks, labs = [], [], []
    with open(path, newline="") as f:
        rd = csv.reader(f, delimiter="\t", quoting=csv.QUOTE_NONE)
        header = next(rd)
        cc, cn, cl = (header.index(x) for x in ("clicked_news", "candidate_news", "clicked"))
        for row in rd:
            cand = [corpus.titles[corpus.index[x]] for x in row[cn].split()]
            hist = [corpus.titles[corpus.index[x]] for x in row[cc].split()[:num_clicked]]
            pad = [np.zeros(L, np.int64)] * (num_clicked - len(hist))
            cands.append(np.stack(cand))
            clks.append(np.stack(pad + hist) if pad + hist else np.zeros((num_clicked, L), np.int64))
            labs.append([int(x) for x in row[cl].split()])
    return np.stack(cands), np.stack(clks), np.array(labs, dtype=np.int64)


# ---------------------------------------------------------------- writers
def write_news_parsed(path, ids, titles):
    with open(path, "w", newline="") as f:
        w = csv.writer(f, delimiter="\t", quoting=csv.QUOTE_NONE, escapechar="\\", lineterminator="\n")
        w.writerow(["id", "category", "subcategory", "title", "abstract", "title_entities",
                    "abstract_entities"])
        zero_a = str([0] * 50)
        for nid, t in zip(ids, titles):
            w.writerow([nid, 0, 0, "[" + ", ".join(str(int(x)) for x in t) + "]", zero_a,
                        str([0] * len(t)), zero_a])


def write_behaviors(path, impressions):
    with open(path, "w") as f:
        for im in impressions:
            hist = "" if im.clicked_news.strip() == "" else im.clicked_news
            imps = " ".join(f"{c}-{l}" for c, l in zip(im.candidates, im.labels))
            f.write(f"{im.impression_id}\t{im.user}\t{im.time}\t{hist}\t{imps}\n")


# ---------------------------------------------------------------- synthetic MIND-shaped split
def synthetic_split(directory, seed=0, n_news=4000, n_users=600, n_impressions=2000, V=70976,
                    min_cands=2, max_cands=40, teacher=None, temperature=1.0):
    """Write news_parsed.tsv + behaviors.tsv under `directory`.

    Titles: length U{5..20} right-padded with 0, ids U[1, V). Users: history of
    U{0..70} clicked news (so some exceed the 50-item truncation and some are
    empty). Impressions: U{min_cands..max_cands} distinct candidates; labels are
    drawn from a planted teacher when `teacher(corpus, impressions) -> [logits]`
    is given (y ~ Bernoulli(sigmoid(logit / temperature)), so AUC is
    informative), otherwise uniformly with p = 0.2. Returns (corpus, impressions).
    """
    rng = np.random.default_rng(seed)
    os.makedirs(directory, exist_ok=True)
    L = NUM_WORDS_TITLE
    ids = [f"N{i}" for i in range(n_news)]
    lens = rng.integers(5, L + 1, n_news)
    titles = rng.integers(1, V, (n_news, L))
    titles[np.arange(L)[None, :] >= lens[:, None]] = 0
    users = []
    for u in range(n_users):
        h = rng.integers(0, 71)
        users.append(" ".join(f"N{x}" for x in rng.integers(0, n_news, h)))
    imps = []
    for k in range(n_impressions):
        u = int(rng.integers(0, n_users))
        c = int(rng.integers(min_cands, max_cands + 1))
        # distinct candidates per impression, as in MIND (no exact score ties)
        cand = [f"N{x}" for x in rng.choice(n_news, size=min(c, n_news), replace=False)]
        imps.append(Impression(str(k + 1), f"U{u}", "11/15/2019 10:00:00 AM", users[u] or " ", cand,
                               [0] * c))
    if teacher is not None:
        corpus = NewsCorpus(ids, titles)
        logits = teacher(corpus, imps)
        for im, lg in zip(imps, logits):
            p = 1.0 / (1.0 + np.exp(-np.asarray(lg, np.float64) / temperature))
            im.labels = [int(x) for x in (rng.random(len(p)) < p)]
    else:
        for im in imps:
            im.labels = [int(x) for x in (rng.random(len(im.candidates)) < 0.2)]
    write_news_parsed(os.path.join(directory, "news_parsed.tsv"), ids, titles)
    write_behaviors(os.path.join(directory, "behaviors.tsv"), imps)
    return NewsCorpus(ids, titles), imps
