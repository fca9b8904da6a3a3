"""Round-2 reference fixtures on the CPU side (no GPU): the restatements the
GPU tests use as references (eval flow, batch reader, ATen training step,
checkpoint resume, raw-exp overflow) against outputs of the reference itself
(tests/golden/gen_golden_flow.py, run in the build container)."""
import os
import sys

import numpy as np
import pytest
import torch

from newsrecommendationsystem_amd import checkpoint as CK
from newsrecommendationsystem_amd import data as Dt
from oracle import eval_oracle as EO
from oracle import nrms_torch_cpu as T
from oracle import weights as W


def _eval_split(flow):
    d = os.path.join(flow["dir"], "eval")
    return (Dt.read_news_parsed(os.path.join(d, "news_parsed.tsv")),
            Dt.read_behaviors(os.path.join(d, "behaviors.tsv")))


def test_flow_fixture_weights_regenerate(flow):
    """The fixtures were made from oracle/weights.py states: same digests."""
    from tests.golden.gen_golden_flow import state_digest
    s = int(flow["seed"])
    assert state_digest(W.nrms_state(s, int(flow["V_eval"]))) == str(flow["eval_state_sha256"])
    assert state_digest(W.nrms_state(s + 1, int(flow["V_train"]))) == str(flow["grad_state_sha256"])
    assert state_digest(W.nrms_state(s + 2, int(flow["V_train"]), D=60, Q=40)) == \
        str(flow["ckpt_state_sha256"])


def test_batch_reader_matches_reference_basedataset(flow):
    """data.read_behaviors_parsed == BaseDataset.__getitem__ + default collate
    (src/dataset.py:64-85): positive-first candidates, first 50 history items,
    left padding with all-zero titles (incl. an empty history and one of 63)."""
    d = os.path.join(flow["dir"], "train")
    corpus = Dt.read_news_parsed(os.path.join(d, "news_parsed.tsv"))
    cand, clk, lab = Dt.read_behaviors_parsed(os.path.join(d, "behaviors_parsed.tsv"), corpus)
    assert np.array_equal(cand, flow["batch_cand"])
    assert np.array_equal(clk, flow["batch_clicked"])
    assert np.array_equal(lab, flow["batch_labels"])


@pytest.mark.parametrize("max_count", [sys.maxsize, 37])
def test_eval_oracle_matches_reference_evaluate(flow, max_count):
    """oracle/eval_oracle.py (the CPU reference of the GPU eval tests) ==
    the reference evaluate() run on the same split and weights: the tuple,
    every impression's labels and logits, the max_count break."""
    corpus, imps = _eval_split(flow)
    sd = W.nrms_state(int(flow["seed"]), int(flow["V_eval"]))
    means, per, tasks = EO.evaluate(sd, corpus, imps, max_count=max_count)
    if max_count == sys.maxsize:
        ref = flow["eval_tuple"]
        off = flow["eval_offsets"]
        assert len(tasks) == len(off) - 1
        y_true = np.concatenate([t[0] for t in tasks])
        y_pred = np.concatenate([t[1] for t in tasks]).astype(np.float32)
        assert np.array_equal(y_true, flow["eval_y_true"])
        assert np.abs(y_pred - flow["eval_y_pred"]).max() <= 1e-5 * np.abs(flow["eval_y_pred"]).max()
        np.testing.assert_allclose(per, flow["eval_metrics"], rtol=0, atol=1e-9, equal_nan=True)
    else:
        ref = flow["eval_tuple_max37"]
        assert len(tasks) == int(flow["eval_n_scored_max37"]) == 36
    np.testing.assert_allclose(means, ref, rtol=0, atol=1e-9)


def _small_cfg(V):
    from newsrecommendationsystem_amd import NRMSConfig

    class Cfg(NRMSConfig):
        num_words = V
        word_embedding_dim = 60
        num_attention_heads = 3
        query_vector_dim = 40
        dropout_probability = 0.0
        hip_train = False
    return Cfg


def _train_batch(flow, reverse=False):
    cand = torch.from_numpy(flow["batch_cand"].astype(np.int64))
    clk = torch.from_numpy(flow["batch_clicked"].astype(np.int64))
    if reverse:
        cand, clk = cand.flip(0), clk.flip(0)
    return cand, clk


def test_aten_training_step_matches_reference_gradients(flow):
    """train.forward_autograd (the GPU gradient tests' reference) == the
    reference loop body src/train.py:202-236 (dropout 0): loss, logits and
    the gradient of every parameter."""
    from newsrecommendationsystem_amd import NRMS, NRMSConfig
    from newsrecommendationsystem_amd import train as TR

    class Cfg(NRMSConfig):
        num_words = int(flow["V_train"])
        dropout_probability = 0.0
    m = NRMS(Cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in
                       W.nrms_state(int(flow["seed"]) + 1, int(flow["V_train"])).items()})
    m.train()
    cand, clk = _train_batch(flow)
    y = TR.forward_autograd(m, cand, clk, training=False)
    loss = TR.loss_fn(y)
    loss.backward()
    assert abs(float(loss.detach()) - float(flow["grad_loss"])) <= 1e-6
    assert float((y.detach() - torch.from_numpy(flow["grad_logits"])).abs().max()) <= 1e-5
    assert [n for n, _ in m.named_parameters()] == list(flow["grad_names"])
    # the W_K bias gradient is analytically zero (a per-query shift of the
    # scores cancels in the normalisation): rounding noise, absolute floor
    floor = 1e-6 * max(float(np.abs(flow["grad__" + n]).max()) for n in flow["grad_names"])
    for n, p in m.named_parameters():
        ref = torch.from_numpy(flow["grad__" + n])
        err = float((p.grad - ref).norm() / max(float(ref.norm()), 1e-30))
        assert err < 1e-5 or float((p.grad - ref).abs().max()) <= floor, (n, err)


def test_checkpoint_resume_cpu_matches_reference(flow):
    """A reference-format checkpoint (src/train.py:266-277, numpy float64
    early_stop_value) loads with weights_only=True into NRMS + torch Adam;
    the next step equals the reference's next step."""
    from newsrecommendationsystem_amd import NRMS
    from newsrecommendationsystem_amd import train as TR
    m = NRMS(_small_cfg(int(flow["V_train"])))
    opt = torch.optim.Adam(m.parameters(), lr=m.config.learning_rate)
    step, esv = CK.resume(os.path.join(flow["dir"], "ckpt-1.pth"), m, opt)
    assert step == 1 and isinstance(esv, np.float64)
    assert esv == -flow["eval_tuple"][0]
    m.train()
    cand, clk = _train_batch(flow, reverse=True)
    loss = TR.train_step(m, opt, cand, clk)
    assert abs(float(loss) - float(flow["ckpt2_loss"])) <= 1e-6
    lr = m.config.learning_rate
    for n, p in m.named_parameters():
        ref = torch.from_numpy(flow["ckpt2__" + n])
        diff = float((p.detach() - ref).abs().max())
        if n.endswith("W_K.bias"):
            # analytically zero gradient = rounding noise, which Adam normalises
            # to steps of about lr: only the step size is comparable
            assert diff <= 4 * lr, (n, diff)
        else:
            assert diff <= 1e-6 * max(1.0, float(ref.abs().max())), (n, diff)


def test_checkpoint_save_is_reference_format(flow, tmp_path):
    """save() writes the reference dict; latest_checkpoint picks the highest step."""
    from newsrecommendationsystem_amd import NRMS
    m = NRMS(_small_cfg(int(flow["V_train"])))
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    ref = CK.load(os.path.join(flow["dir"], "ckpt-1.pth"))
    CK.resume(os.path.join(flow["dir"], "ckpt-1.pth"), m, opt)
    for s in (3, 12):
        CK.save(str(tmp_path / f"ckpt-{s}.pth"), m, opt, s, -0.5)
    path = CK.latest_checkpoint(str(tmp_path))
    assert path.endswith("ckpt-12.pth")
    ours = CK.load(path)
    assert set(ours) == set(ref)
    assert list(ours["model_state_dict"]) == list(ref["model_state_dict"])
    assert ours["optimizer_state_dict"]["param_groups"] == ref["optimizer_state_dict"]["param_groups"]
    for k, v in ref["model_state_dict"].items():
        assert torch.equal(ours["model_state_dict"][k], v)


def test_aten_oracle_overflow_pattern_matches_reference(flow):
    """nrms_torch_cpu reproduces the reference's raw-exp boundary bit for bit:
    scores one float step either side of exp's overflow and of the 20-fold
    row-sum overflow (multihead_self.py:16-20)."""
    from tests.golden.gen_golden_flow import overflow_setup
    sd_o, titles, vals, *_ = overflow_setup(W.nrms_state(int(flow["seed"]) + 3, int(flow["V_train"])),
                                           np.sqrt(20))
    assert np.array_equal(titles, flow["ovf_titles"]) and np.array_equal(vals, flow["ovf_raw"])
    assert np.array_equal(sd_o["news_encoder.word_embedding.weight"][:, 0], flow["ovf_embedding_col0"])
    with torch.no_grad():
        out = T.news_encode(torch.from_numpy(titles.astype(np.int64)), T.state_to_torch(sd_o)).numpy()
    ref = flow["ovf_out"]
    assert np.array_equal(np.isnan(out), np.isnan(ref))
    assert int(np.isnan(ref).any(axis=1).sum()) == 9
    ok = ~np.isnan(ref)
    assert np.array_equal(out[ok], ref[ok])
