"""Test tool (not collected; the oracle is the checker): per-arithmetic error of nrms_forward against the fp64 oracle on the bench
batch slice of tests/test_gpu_parity.py::test_bench_batch_slice_gemm_arith_vs_fp64,
with the row-error distribution (max, p99, median, mean) instead of the max
alone. Library from NRMS_LIB_PATH (A/B of a kernel variant's rounding).

    NRMS_LIB_PATH=... python tests/arith_err_probe.py [n_impressions]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import bench  # noqa: E402
from oracle import nrms_oracle as O  # noqa: E402
from newsrecommendationsystem_amd import _native as N  # noqa: E402
from newsrecommendationsystem_amd import stream as S  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    device = torch.device("cuda:0")
    model = bench.build_model(device)
    idx = bench.stream_impressions(0, 1, n, device)
    cand, clk = S.batch(0, idx, bench.V_WORDS)
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    ref = O.forward(cand.cpu().numpy(), clk.cpu().numpy(), sd, np.float64)
    lib = os.environ.get("NRMS_LIB_PATH", "product").split("/")[-1]
    for name, mode in (("f32", N.NRMS_GEMM_F32), ("x6", N.NRMS_GEMM_SPLIT_BF16X6),
                       ("f16x3", N.NRMS_GEMM_SPLIT_F16X3)):
        with N.gemm_arith(mode), torch.no_grad():
            y = model.forward_ids(cand, clk).detach().cpu().numpy().astype(np.float64)
        e = np.asarray(O.normwise_rel_err(y, ref), dtype=np.float64).ravel()
        print(f"{lib} {name:6s} n={n} max {e.max():.3e} p99 {np.quantile(e, 0.99):.3e} "
              f"median {np.median(e):.3e} mean {e.mean():.3e}", flush=True)


if __name__ == "__main__":
    main()
