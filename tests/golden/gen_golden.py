"""Generate tests/golden/nrms_golden.npz by RUNNING THE REFERENCE (build
container only: it imports /root/reference/src, which never travels).

    python tests/golden/gen_golden.py

Weights come from oracle/weights.py (splitmix64, regenerable anywhere), are
loaded into the reference NRMS with load_state_dict, and the reference's own
forward / get_news_vector / get_user_vector / get_prediction and metric
functions produce the expected outputs. The fixture holds only ids, small
generated inputs and outputs (numbers), plus a checksum of the weights.
"""
import hashlib
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import weights as W  # noqa: E402

REF_SRC = "/root/reference/src"
SEED = 20251015
V = 256


def state_digest(sd):
    h = hashlib.sha256()
    for k in sorted(sd):
        h.update(k.encode())
        h.update(np.ascontiguousarray(sd[k], dtype=np.float32).tobytes())
    return h.hexdigest()


def main():
    sys.path.insert(0, REF_SRC)
    os.chdir(REF_SRC)
    from config import NRMSConfig
    from model.NRMS import NRMS
    import evaluate as ref_eval

    class Cfg(NRMSConfig):
        num_words = V

    torch.set_num_threads(8)

    def build(sd):
        m = NRMS(Cfg)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        return m.eval()

    sd = W.nrms_state(SEED, V)
    model = build(sd)
    out = {"seed": np.int64(SEED), "V": np.int64(V)}

    with torch.no_grad():
        # (1) embedding gather, bit-exact (news_encoder.py:38); include id 0 and V-1
        g_ids = W.titles(SEED, 10, 8, V)
        g_ids[0, :] = V - 1
        g_ids[1, :] = 0
        out["gather_ids"] = g_ids.astype(np.int32)
        out["gather_out"] = model.news_encoder.word_embedding(torch.from_numpy(g_ids)).numpy()

        # (2) news vectors (NRMS.get_news_vector, __init__.py:50-61)
        n_ids = W.titles(SEED, 20, 64, V)
        n_ids[0, :] = 0                 # an all-padding title
        n_ids[1, :] = W.randint(SEED, 21, (20,), 1, V)  # a full-length title
        out["news_ids"] = n_ids.astype(np.int32)
        out["news_out"] = model.get_news_vector({"title": torch.from_numpy(n_ids), "id": list(range(64))}).numpy()

        # (3) user vectors (get_user_vector, __init__.py:63-71) over eval-style
        #     input: left-padded with all-zero PADDED_NEWS vectors (evaluate.py:120-124,203-204)
        u_in = W.normal(SEED, 30, (8, 50, 300), 0.3)
        u_len = W.randint(SEED, 31, (8,), 1, 51)
        u_len[0] = 50
        u_len[1] = 1
        for b in range(8):
            u_in[b, : 50 - u_len[b]] = 0.0
        out["user_len"] = u_len.astype(np.int32)
        out["user_out"] = model.get_user_vector(torch.from_numpy(u_in)).numpy()

        # (4) full forward (NRMS.forward, __init__.py:19-48), train-style left padding
        cand, clk, hist = W.impressions(SEED, 40, 4, V)
        out["fwd_cand"] = cand.astype(np.int32)
        out["fwd_clicked"] = clk.astype(np.int32)
        y = model([{"title": torch.from_numpy(cand[:, i])} for i in range(cand.shape[1])],
                  [{"title": torch.from_numpy(clk[:, i])} for i in range(clk.shape[1])])
        out["fwd_out"] = y.numpy()

        # (5) get_prediction (__init__.py:73-84)
        pn = W.normal(SEED, 50, (7, 300), 0.5)
        pu = W.normal(SEED, 51, (300,), 0.5)
        out["pred_out"] = model.get_prediction(torch.from_numpy(pn), torch.from_numpy(pu)).numpy()

        # (6) raw-exp overflow -> NaN (multihead_self.py:16-20): scale W_Q, W_K
        sd_o = dict(sd)
        for k in ("W_Q", "W_K"):
            key = f"news_encoder.multihead_self_attention.{k}.weight"
            sd_o[key] = (sd[key] * np.float32(OVERFLOW_SCALE)).astype(np.float32)
        out["overflow_scale"] = np.float32(OVERFLOW_SCALE)
        out["overflow_out"] = build(sd_o).get_news_vector({"title": torch.from_numpy(n_ids)}).numpy()

        # (7) all-underflow -> attention weights 0 -> zero context
        sd_u = dict(sd)
        pre = "news_encoder.multihead_self_attention"
        sd_u[f"{pre}.W_Q.bias"] = np.full(300, UNDERFLOW_BIAS, np.float32)
        sd_u[f"{pre}.W_K.bias"] = np.full(300, -UNDERFLOW_BIAS, np.float32)
        sd_u[f"{pre}.W_Q.weight"] = np.zeros((300, 300), np.float32)
        sd_u[f"{pre}.W_K.weight"] = np.zeros((300, 300), np.float32)
        out["underflow_bias"] = np.float32(UNDERFLOW_BIAS)
        out["underflow_out"] = build(sd_u).get_news_vector({"title": torch.from_numpy(n_ids)}).numpy()

    # (8) metrics (evaluate.py:24-42,160-168,270-272)
    lens = W.randint(SEED, 60, (24,), 2, 30)
    y_true, y_score, res = [], [], []
    for i, n in enumerate(lens):
        t = (W.uniform01(SEED, 1000 + i, int(n)) < 0.25).astype(np.int64)
        if i == 3:
            t[:] = 0          # all-negative impression -> NaN row
        s = W.normal(SEED, 2000 + i, (int(n),))
        if i == 5:
            s[:] = s[0]       # all-tied scores
        y_true.append(t)
        y_score.append(s.astype(np.float64))
        res.append(ref_eval.calculate_single_user_metric((t.tolist(), s.astype(np.float64).tolist())))
    res = np.array(res, dtype=np.float64)
    out["metric_lens"] = lens.astype(np.int32)
    out["metric_true"] = np.concatenate(y_true).astype(np.int8)
    out["metric_score"] = np.concatenate(y_score)
    out["metric_per_impression"] = res
    out["metric_mean"] = np.array([np.nanmean(res[:, i]) for i in range(4)])

    out["state_sha256"] = np.array(state_digest(sd))
    out["torch_version"] = np.array(torch.__version__)
    dst = os.path.join(ROOT, "tests", "golden", "nrms_golden.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, os.path.getsize(dst), "bytes")
    print("overflow NaN rows:", int(np.isnan(out["overflow_out"]).any(axis=1).sum()), "/ 64")
    print("underflow max |out|:", float(np.abs(out["underflow_out"]).max()))


OVERFLOW_SCALE = 4.8
UNDERFLOW_BIAS = 5.0

if __name__ == "__main__":
    main()
