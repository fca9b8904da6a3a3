"""Diagnostic (not a test): determinism of the news tail with and without
padding-title dedupe on a config-3 batch."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import weights as W
from newsrecommendationsystem_amd import NRMS, NRMSConfig, _native as N

V = 70976
sd = W.nrms_state(5, V)
Cfg = type("Cfg", (NRMSConfig,), dict(num_words=V, hip_proj_mode=2))
m = NRMS(Cfg)
m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
m = m.cuda().eval()
cand, clk, _ = W.impressions(5, 1000, 1024, V)
titles = torch.from_numpy(np.concatenate([clk.reshape(-1, 20), cand.reshape(-1, 20)]))
pad = (titles == 0).all(1).numpy()
lib = N.load()
for arith in (N.NRMS_GEMM_SPLIT_BF16X6, N.NRMS_GEMM_F32):
    with N.gemm_arith(arith):
        res = {}
        for on in (0, 1):
            lib.nrms_set_title_dedupe(on)
            with torch.no_grad():
                a = m.get_news_vector({"title": titles}).cpu().numpy()
                b = m.get_news_vector({"title": titles}).cpu().numpy()
            d = np.where((a != b).any(1))[0]
            print(f"arith {arith} dedupe {on}: repeat diffs {len(d)} titles, padding among them {pad[d].sum()}, "
                  f"max abs {np.abs(a - b).max() if len(d) else 0}")
            res[on] = a
        d = np.where((res[0] != res[1]).any(1))[0]
        print(f"arith {arith}: on vs off diffs {len(d)} titles (padding {pad[d].sum()}), first {d[:10]}, "
              f"max abs {np.abs(res[0] - res[1]).max() if len(d) else 0}")
lib.nrms_set_title_dedupe(1)
