"""Child process of tests/test_gpu_parity.py::test_user_long_history_forms_bitwise:
the UserEncoder outputs of one library configuration (the environment picks
the chunked instance's form for long users: two queries per thread in one
pass by default; NRMS_USER_PAIR=0 -> two passes split by head where that
adds no wave; + NRMS_USER_HSPLIT=0 -> two passes split by task index), saved
to argv[1] (.npz).

  get_user_vector on [64, L, 300] inputs for L = 34 (one pass over two key
  chunks), 36 / 41 / 38, 50 (two passes split 8 + 7 / 9 + 6 / 10 + 5 heads),
  46 (split by task index; past 39 rows the context packed as two planes), scaled so some rows take the recheck path, and
  nrms_forward logits on a 256-impression slice of the bench batch
  (compacted lengths 1..50)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from newsrecommendationsystem_amd import stream as S  # noqa: E402


def main(out):
    dev = torch.device("cuda:0")
    model = bench.build_model(dev)
    res = {}
    with torch.no_grad():
        for L in (34, 36, 38, 41, 46, 50):
            g = torch.Generator(device="cpu").manual_seed(4 + L)
            x = torch.randn(64, L, 300, generator=g)
            x[::7] *= 30.0                      # large scores: rows near fp32 overflow take the recheck path
            x[3, :20] = 0.0                     # left padding
            res[f"uv{L}"] = model.get_user_vector(x.to(dev)).cpu().numpy()
        idx = bench.stream_impressions(0, 1, 256, dev)
        cand, clk = S.batch(0, idx, bench.V_WORDS)
        res["logits"] = model.forward_ids(cand, clk).cpu().numpy()
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1])
