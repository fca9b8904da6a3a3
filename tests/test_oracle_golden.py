"""Pin the CPU oracle against golden vectors captured from the reference
(tests/golden/gen_golden.py). CPU-only."""
import hashlib

import numpy as np
import pytest
import torch

from oracle import metrics as M
from oracle import nrms_oracle as O
from oracle import nrms_torch_cpu as T

TOL = 1e-5  # numpy fp32 restatement vs the reference's fp32 ATen result, normwise


def _state_digest(sd):
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k], dtype=np.float32).tobytes())
    return h.hexdigest()


def test_generator_reproduces_golden_weights(golden, golden_state):
    assert _state_digest(golden_state) == str(golden["state_sha256"])


def test_gather_bit_exact(golden, golden_state):
    out = O.embedding_gather(golden_state["news_encoder.word_embedding.weight"],
                             golden["gather_ids"].astype(np.int64))
    assert out.dtype == np.float32
    assert np.array_equal(out.view(np.uint32), golden["gather_out"].view(np.uint32))


def test_gather_rejects_out_of_range(golden_state):
    tab = golden_state["news_encoder.word_embedding.weight"]
    with pytest.raises(IndexError):
        O.embedding_gather(tab, np.array([[0, tab.shape[0]]]))


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_news_vectors(golden, golden_state, dt):
    out = O.news_encode(golden["news_ids"].astype(np.int64), golden_state, dt)
    assert O.normwise_rel_err(out, golden["news_out"]).max() < (TOL if dt == np.float32 else 1e-5)


def test_user_vectors(golden, golden_state):
    from oracle import weights as W
    u_in = W.normal(int(golden["seed"]), 30, (8, 50, 300), 0.3)
    for b, n in enumerate(golden["user_len"]):
        u_in[b, : 50 - n] = 0.0
    out = O.user_encode(u_in, golden_state)
    assert O.normwise_rel_err(out, golden["user_out"]).max() < TOL


def test_forward_logits(golden, golden_state):
    out = O.forward(golden["fwd_cand"].astype(np.int64), golden["fwd_clicked"].astype(np.int64), golden_state)
    ref = golden["fwd_out"]
    assert np.abs(out - ref).max() <= 1e-5 * np.abs(ref).max()


def test_prediction(golden, golden_state):
    from oracle import weights as W
    s = int(golden["seed"])
    out = O.get_prediction(W.normal(s, 50, (7, 300), 0.5), W.normal(s, 51, (300,), 0.5))
    assert np.allclose(out, golden["pred_out"], rtol=1e-5, atol=1e-6)


def _overflow_state(golden, sd):
    sd = dict(sd)
    for k in ("W_Q", "W_K"):
        key = f"news_encoder.multihead_self_attention.{k}.weight"
        sd[key] = (sd[key] * golden["overflow_scale"]).astype(np.float32)
    return sd


def test_raw_exp_overflow_nan_pattern(golden, golden_state):
    out = O.news_encode(golden["news_ids"].astype(np.int64), _overflow_state(golden, golden_state))
    ref = golden["overflow_out"]
    assert np.array_equal(np.isnan(out), np.isnan(ref))
    ok = ~np.isnan(ref).any(axis=1)
    assert ok.sum() > 0 and (~ok).sum() > 0
    assert O.normwise_rel_err(out[ok], ref[ok]).max() < 1e-4


def test_raw_exp_underflow_zero(golden, golden_state):
    sd = dict(golden_state)
    pre = "news_encoder.multihead_self_attention"
    b = golden["underflow_bias"]
    sd[f"{pre}.W_Q.bias"] = np.full(300, b, np.float32)
    sd[f"{pre}.W_K.bias"] = np.full(300, -b, np.float32)
    sd[f"{pre}.W_Q.weight"] = np.zeros((300, 300), np.float32)
    sd[f"{pre}.W_K.weight"] = np.zeros((300, 300), np.float32)
    out = O.news_encode(golden["news_ids"].astype(np.int64), sd)
    assert np.array_equal(out, golden["underflow_out"])


def test_torch_cpu_port_matches_golden(golden, golden_state):
    sd = T.state_to_torch(golden_state)
    with torch.no_grad():
        news = T.news_encode(torch.from_numpy(golden["news_ids"].astype(np.int64)), sd).numpy()
        fwd = T.forward(torch.from_numpy(golden["fwd_cand"].astype(np.int64)),
                        torch.from_numpy(golden["fwd_clicked"].astype(np.int64)), sd).numpy()
    assert O.normwise_rel_err(news, golden["news_out"]).max() < 1e-6
    assert np.abs(fwd - golden["fwd_out"]).max() <= 1e-6 * np.abs(golden["fwd_out"]).max()


def test_metrics(golden):
    lens = golden["metric_lens"]
    off = np.concatenate([[0], np.cumsum(lens)])
    per = golden["metric_per_impression"]
    pairs = []
    for i in range(len(lens)):
        t = golden["metric_true"][off[i]:off[i + 1]].astype(np.int64)
        s = golden["metric_score"][off[i]:off[i + 1]]
        pairs.append((t, s))
        got = M.single_impression(t, s)
        assert np.allclose(got, per[i], equal_nan=True, rtol=1e-12, atol=1e-12), i
    assert np.allclose(M.aggregate(pairs), golden["metric_mean"], rtol=1e-12)
