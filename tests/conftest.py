import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "nrms_golden.npz")
FLOW_GOLDEN = os.path.join(ROOT, "tests", "golden", "nrms_flow_golden.npz")
FLOW_DIR = os.path.join(ROOT, "tests", "golden", "flow")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")


@pytest.fixture(scope="session")
def golden():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def flow():
    """Round-2 reference fixtures (tests/golden/gen_golden_flow.py): reference
    evaluate(), BaseDataset batches, gradients, checkpoint, exp overflow."""
    with np.load(FLOW_GOLDEN, allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["dir"] = FLOW_DIR
    return d


@pytest.fixture(scope="session")
def golden_state(golden):
    from oracle import weights as W
    return W.nrms_state(int(golden["seed"]), int(golden["V"]))


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(params=["f16x3", "x6", "f32"])
def gemm_mode(request):
    """Run a GPU test under every GEMM arithmetic (include/nrms_hip.h,
    nrms_set_gemm_arith): split-f16 x3 (default), split-bf16 x6 and exact f32
    MFMA."""
    from newsrecommendationsystem_amd import _native as N
    mode = {"f16x3": N.NRMS_GEMM_SPLIT_F16X3, "x6": N.NRMS_GEMM_SPLIT_BF16X6,
            "f32": N.NRMS_GEMM_F32}[request.param]
    with N.gemm_arith(mode):
        yield request.param
