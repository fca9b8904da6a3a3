"""Offline MIND preprocessing: raw MIND files -> the
files the scoring and training paths read (data.py).

Restates src/data_preprocess.py of the reference, function for function:

  parse_behaviors          (:22-81)   behaviors.tsv -> behaviors_parsed.tsv + user2int.tsv,
                                      positives paired with K shuffled negatives
  parse_news               (:84-240)  news.tsv -> news_parsed.tsv (+ category2int,
                                      word2int, entity2int in 'train' mode)
  generate_word_embedding  (:243-281) GloVe text + word2int -> pretrained_word_embedding.npy
  transform_entity_embedding (:284-305) entity_embedding.vec -> pretrained_entity_embedding.npy
  main                     (:308-368) the train / val / test driver

Host-side and offline (it runs once per dataset, not on the scoring path), so
it is plain Python + pandas, as the reference is. Differences a caller can see:

  * Tokenizer. The reference calls nltk.word_tokenize (unpinned; nltk is not
    installed in this image). When nltk is importable it is used here too;
    otherwise `word_tokenize` below restates NLTK's NLTKWordTokenizer (the
    improved Treebank rules: starting quotes, punctuation, brackets, double
    dashes, ending quotes and clitics, MacIntyre contractions) on the whole
    string. The Punkt sentence split that nltk.word_tokenize runs first is not
    restated, so a period in the middle of a multi-sentence title stays
    attached ("fall." instead of "fall", "."): parity unpinned for such titles.
  * Randomness. The reference shuffles negatives with the global `random`
    module and draws missing embedding rows from the global numpy RNG; here
    both come from seeded generators passed in (same distributions, a
    reproducible sample).
  * The NRMS config fields it reads (num_words_title, num_words_abstract,
    word_freq_threshold, entity_freq_threshold, entity_confidence_threshold,
    negative_sampling_ratio, word_embedding_dim, entity_embedding_dim) come
    from `config` (defaults: config.NRMSConfig, = src/config.py:10-45).
"""
import csv
import json
import os
import random
import re

import numpy as np

from .config import NRMSConfig

# ----------------------------------------------------------------- tokenizer
# NLTK NLTKWordTokenizer rules (nltk/tokenize/destructive.py), applied in its
# order: starting quotes, punctuation, brackets, double dashes, then (on the
# space-padded text) ending quotes, clitics and contractions.
_STARTING_QUOTES = [
    (re.compile("([«“‘„]|[`]+)", re.U), r" \1 "),
    (re.compile(r'^"'), r"``"),
    (re.compile(r"(``)"), r" \1 "),
    (re.compile(r"([ \(\[{<])(\"|\'{2})"), r"\1 `` "),
    (re.compile(r"(?i)(\')(?!re|ve|ll|m|t|s|d|n)(\w)\b", re.U), r"\1 \2"),
]
_PUNCTUATION = [
    (re.compile(r'([^\.])(\.)([\]\)}>"\']*)\s*$', re.U), r"\1 \2 \3 "),
    (re.compile(r"([:,])([^\d])"), r" \1 \2"),
    (re.compile(r"([:,])$"), r" \1 "),
    (re.compile(r"\.{2,}", re.U), r" \g<0> "),
    (re.compile(r"[;@#$%&]"), r" \g<0> "),
    (re.compile(r'([^\.])(\.)([\]\)}>"\']*)\s*$'), r"\1 \2\3 "),
    (re.compile(r"[?!]"), r" \g<0> "),
    (re.compile(r"([^'])' "), r"\1 ' "),
    (re.compile(r"[*]", re.U), r" \g<0> "),
]
_PARENS_BRACKETS = (re.compile(r"[\]\[\(\)\{\}\<\>]"), r" \g<0> ")
_DOUBLE_DASHES = (re.compile(r"--"), r" -- ")
_ENDING_QUOTES = [
    (re.compile("([»”’])", re.U), r" \1 "),
    (re.compile(r"''"), " '' "),
    (re.compile(r'"'), " '' "),
    (re.compile(r"([^' ])('[sS]|'[mM]|'[dD]|') "), r"\1 \2 "),
    (re.compile(r"([^' ])('ll|'LL|'re|'RE|'ve|'VE|n't|N'T) "), r"\1 \2 "),
]
_CONTRACTIONS2 = [re.compile(p) for p in (
    r"(?i)\b(can)(?#X)(not)\b", r"(?i)\b(d)(?#X)('ye)\b", r"(?i)\b(gim)(?#X)(me)\b",
    r"(?i)\b(gon)(?#X)(na)\b", r"(?i)\b(got)(?#X)(ta)\b", r"(?i)\b(lem)(?#X)(me)\b",
    r"(?i)\b(more)(?#X)('n)\b", r"(?i)\b(wan)(?#X)(na)(?=\s)")]
_CONTRACTIONS3 = [re.compile(p) for p in (r"(?i) ('t)(?#X)(is)\b", r"(?i) ('t)(?#X)(was)\b")]


def treebank_tokenize(text):
    """NLTKWordTokenizer.tokenize restated (no sentence split)."""
    for rx, sub in _STARTING_QUOTES:
        text = rx.sub(sub, text)
    for rx, sub in _PUNCTUATION:
        text = rx.sub(sub, text)
    text = _PARENS_BRACKETS[0].sub(_PARENS_BRACKETS[1], text)
    text = _DOUBLE_DASHES[0].sub(_DOUBLE_DASHES[1], text)
    text = " " + text + " "
    for rx, sub in _ENDING_QUOTES:
        text = rx.sub(sub, text)
    for rx in _CONTRACTIONS2:
        text = rx.sub(r" \1 \2 ", text)
    for rx in _CONTRACTIONS3:
        text = rx.sub(r" \1 \2 ", text)
    return text.split()


try:  # the reference's tokenizer when it is installed (src/data_preprocess.py:10)
    from nltk.tokenize import word_tokenize as _nltk_word_tokenize
except ImportError:  # not in this image
    _nltk_word_tokenize = None


def word_tokenize(text):
    if _nltk_word_tokenize is not None:
        return _nltk_word_tokenize(text)
    return treebank_tokenize(text)


# ----------------------------------------------------------------- behaviors
def _read_table(path, **kw):
    import pandas as pd
    return pd.read_table(path, **kw)


def parse_behaviors(source, target, user2int_path, config=NRMSConfig, rng=None):
    """src/data_preprocess.py:22-81. Users get ints from 1 in first-seen order;
    each impression's positives are paired with `negative_sampling_ratio`
    shuffled negatives (a pair the negatives run out in is dropped, and so is
    an impression with no complete pair); one output row per pair:
    user (int), clicked_news, candidate_news (positive first), clicked."""
    import pandas as pd
    rng = rng if rng is not None else random.Random(0)
    behaviors = _read_table(source, header=None,
                            names=["impression_id", "user", "time", "clicked_news", "impressions"])
    behaviors["clicked_news"] = behaviors["clicked_news"].fillna(" ")
    behaviors["impressions"] = behaviors["impressions"].str.split()
    user2int = {}
    for u in behaviors["user"]:
        if u not in user2int:
            user2int[u] = len(user2int) + 1
    pd.DataFrame(list(user2int.items()), columns=["user", "int"]).to_csv(user2int_path, sep="\t",
                                                                        index=False)
    k = config.negative_sampling_ratio
    out = []
    for row in behaviors.itertuples(index=False):
        imps = row.impressions if isinstance(row.impressions, list) else []
        positive = iter([x for x in imps if x.endswith("1")])
        negative = [x for x in imps if x.endswith("0")]
        rng.shuffle(negative)
        negative = iter(negative)
        try:
            while True:
                pair = [next(positive)]
                for _ in range(k):
                    pair.append(next(negative))
                out.append((user2int[row.user], row.clicked_news,
                            " ".join(e.split("-")[0] for e in pair),
                            " ".join(e.split("-")[1] for e in pair)))
        except StopIteration:
            pass
    pd.DataFrame(out, columns=["user", "clicked_news", "candidate_news", "clicked"]).to_csv(
        target, sep="\t", index=False)
    return len(user2int)


# ----------------------------------------------------------------- news
NEWS_COLUMNS = ["id", "category", "subcategory", "title", "abstract", "title_entities",
                "abstract_entities"]


def _read_news(source):
    news = _read_table(source, header=None, usecols=[0, 1, 2, 3, 4, 6, 7], quoting=csv.QUOTE_NONE,
                       names=NEWS_COLUMNS)
    news["title_entities"] = news["title_entities"].fillna("[]")
    news["abstract_entities"] = news["abstract_entities"].fillna("[]")
    return news.fillna(" ")


def build_vocab(news, config=NRMSConfig):
    """'train' mode maps (src/data_preprocess.py:155-199): categories and
    subcategories in row order from 1; words of title + abstract (lower-cased,
    tokenized) with frequency >= word_freq_threshold, in first-seen order from
    1; entities weighted by len(OccurrenceOffsets) * Confidence with total >=
    entity_freq_threshold."""
    category2int, word2freq, entity2freq = {}, {}, {}
    for row in news.itertuples(index=False):
        for c in (row.category, row.subcategory):
            if c not in category2int:
                category2int[c] = len(category2int) + 1
        for text in (row.title, row.abstract):
            for w in word_tokenize(text.lower()):
                word2freq[w] = word2freq.get(w, 0) + 1
        for ents in (row.title_entities, row.abstract_entities):
            for e in json.loads(ents):
                times = len(e["OccurrenceOffsets"]) * e["Confidence"]
                if times > 0:
                    entity2freq[e["WikidataId"]] = entity2freq.get(e["WikidataId"], 0) + times
    word2int, entity2int = {}, {}
    for w, f in word2freq.items():
        if f >= config.word_freq_threshold:
            word2int[w] = len(word2int) + 1
    for e, f in entity2freq.items():
        if f >= config.entity_freq_threshold:
            entity2int[e] = len(entity2int) + 1
    return category2int, word2int, entity2int


def parse_news_row(row, category2int, word2int, entity2int, config=NRMSConfig):
    """parse_row (src/data_preprocess.py:104-152): category ints (0 if unseen),
    title / abstract word ids right-padded with 0 and cut at num_words_title /
    num_words_abstract (unknown words stay 0), and per-position entity ids of
    known words from the row's confident entities' surface forms."""
    lt, la = config.num_words_title, config.num_words_abstract
    title, abstract = [0] * lt, [0] * la
    title_ent, abstract_ent = [0] * lt, [0] * la
    local_entity_map = {}
    for ents in (row.title_entities, row.abstract_entities):
        for e in json.loads(ents):
            if e["Confidence"] > config.entity_confidence_threshold and e["WikidataId"] in entity2int:
                for x in " ".join(e["SurfaceForms"]).lower().split():
                    local_entity_map[x] = entity2int[e["WikidataId"]]
    for text, ids, ent in ((row.title, title, title_ent), (row.abstract, abstract, abstract_ent)):
        for i, w in enumerate(word_tokenize(text.lower())):
            if i >= len(ids):          # the reference's IndexError ends the row
                break
            if w in word2int:
                ids[i] = word2int[w]
                if w in local_entity_map:
                    ent[i] = local_entity_map[w]
    return [row.id, category2int.get(row.category, 0), category2int.get(row.subcategory, 0),
            title, abstract, title_ent, abstract_ent]


def _write_map(path, mapping, key):
    import pandas as pd
    pd.DataFrame(list(mapping.items()), columns=[key, "int"]).to_csv(path, sep="\t", index=False)


def _read_map(path, na_filter=True):
    import pandas as pd
    return dict(pd.read_table(path, na_filter=na_filter).values.tolist())


def parse_news(source, target, category2int_path, word2int_path, entity2int_path, mode,
               config=NRMSConfig):
    """src/data_preprocess.py:84-240: 'train' builds and writes the three maps,
    'test' reads them (word2int with na_filter off: "nan" is a word); both
    write news_parsed.tsv with list-valued title / abstract / entity columns."""
    import pandas as pd
    news = _read_news(source)
    if mode == "train":
        category2int, word2int, entity2int = build_vocab(news, config)
        _write_map(category2int_path, category2int, "category")
        _write_map(word2int_path, word2int, "word")
        _write_map(entity2int_path, entity2int, "entity")
    elif mode == "test":
        category2int = _read_map(category2int_path)
        word2int = _read_map(word2int_path, na_filter=False)
        entity2int = _read_map(entity2int_path)
    else:
        raise ValueError(f"mode must be 'train' or 'test', got {mode!r}")
    rows = [parse_news_row(r, category2int, word2int, entity2int, config)
            for r in news.itertuples(index=False)]
    pd.DataFrame(rows, columns=NEWS_COLUMNS).to_csv(target, sep="\t", index=False)
    return category2int, word2int, entity2int


# ----------------------------------------------------------------- embeddings
def generate_word_embedding(source, target, word2int_path, config=NRMSConfig, np_rng=None):
    """src/data_preprocess.py:243-281: row int of the output is the GloVe
    vector of that word when GloVe has it, N(0, 1) otherwise (row 0, the
    padding id, included: it is not zeroed). GloVe is read with pandas' NA
    filter on, as the reference reads it, so GloVe words such as "nan" or
    "null" never match. Duplicate GloVe words: the first vector wins. Returns
    the missed-word rate."""
    import pandas as pd
    np_rng = np_rng if np_rng is not None else np.random.default_rng(0)
    dim = config.word_embedding_dim
    word2int = pd.read_table(word2int_path, na_filter=False, index_col="word")
    glove = pd.read_table(source, index_col=0, sep=" ", header=None, quoting=csv.QUOTE_NONE,
                          names=range(dim))
    glove.index.rename("word", inplace=True)
    glove = glove[~glove.index.duplicated(keep="first")]
    merged = word2int.merge(glove, how="inner", left_index=True, right_index=True)
    n = len(word2int) + 1
    out = np_rng.normal(size=(n, dim))
    out[merged["int"].to_numpy()] = merged[list(range(dim))].to_numpy(dtype=np.float64)
    np.save(target, out)
    return (n - len(merged) - 1) / max(len(word2int), 1)


def transform_entity_embedding(source, target, entity2int_path, config=NRMSConfig, np_rng=None):
    """src/data_preprocess.py:284-305: entity_embedding.vec rows placed at their
    entity ints, N(0, 1) for entities without a vector (and row 0)."""
    import pandas as pd
    np_rng = np_rng if np_rng is not None else np.random.default_rng(0)
    dim = config.entity_embedding_dim
    emb = pd.read_table(source, header=None)
    vec = dict(zip(emb[0], emb.iloc[:, 1:1 + dim].to_numpy(dtype=np.float64)))
    entity2int = pd.read_table(entity2int_path)
    out = np_rng.normal(size=(len(entity2int) + 1, dim))
    for e, i in entity2int.itertuples(index=False):
        if e in vec:
            out[i] = vec[e]
    np.save(target, out)


def main(data_dir="./data", glove_path=None, config=NRMSConfig, seed=0):
    """The reference's __main__ (src/data_preprocess.py:308-368) over
    data_dir/{train,val,test}; steps whose inputs are missing are skipped."""
    rng, np_rng = random.Random(seed), np.random.default_rng(seed)
    tr = os.path.join(data_dir, "train")
    j = lambda d, f: os.path.join(d, f)
    parse_behaviors(j(tr, "behaviors.tsv"), j(tr, "behaviors_parsed.tsv"), j(tr, "user2int.tsv"),
                    config, rng)
    parse_news(j(tr, "news.tsv"), j(tr, "news_parsed.tsv"), j(tr, "category2int.tsv"),
               j(tr, "word2int.tsv"), j(tr, "entity2int.tsv"), "train", config)
    glove_path = glove_path or os.path.join(data_dir, "glove",
                                            f"glove.840B.{config.word_embedding_dim}d.txt")
    if os.path.exists(glove_path):
        generate_word_embedding(glove_path, j(tr, "pretrained_word_embedding.npy"),
                                j(tr, "word2int.tsv"), config, np_rng)
    if os.path.exists(j(tr, "entity_embedding.vec")):
        transform_entity_embedding(j(tr, "entity_embedding.vec"),
                                   j(tr, "pretrained_entity_embedding.npy"),
                                   j(tr, "entity2int.tsv"), config, np_rng)
    for split in ("val", "test"):
        d = os.path.join(data_dir, split)
        if os.path.exists(j(d, "news.tsv")):
            parse_news(j(d, "news.tsv"), j(d, "news_parsed.tsv"), j(tr, "category2int.tsv"),
                       j(tr, "word2int.tsv"), j(tr, "entity2int.tsv"), "test", config)


if __name__ == "__main__":
    import sys
    main(*(sys.argv[1:2] or ["./data"]))
