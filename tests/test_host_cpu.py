"""CPU-only checks of the boundary: the C-ABI library loads and exports every
symbol include/nrms_hip.h declares, the ctypes signatures match the header,
and the host mirror keeps the reference's interface (state_dict keys, config
fields, error behaviour). No kernel is launched here."""
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nrms_hip.h")

# state_dict keys of the reference NRMS (src/model/NRMS/__init__.py:12-17 and
# the modules it builds), listed from the reference in the build container.
REF_KEYS = [
    "news_encoder.word_embedding.weight",
    "news_encoder.multihead_self_attention.W_Q.weight",
    "news_encoder.multihead_self_attention.W_Q.bias",
    "news_encoder.multihead_self_attention.W_K.weight",
    "news_encoder.multihead_self_attention.W_K.bias",
    "news_encoder.multihead_self_attention.W_V.weight",
    "news_encoder.multihead_self_attention.W_V.bias",
    "news_encoder.additive_attention.attention_query_vector",
    "news_encoder.additive_attention.linear.weight",
    "news_encoder.additive_attention.linear.bias",
    "user_encoder.multihead_self_attention.W_Q.weight",
    "user_encoder.multihead_self_attention.W_Q.bias",
    "user_encoder.multihead_self_attention.W_K.weight",
    "user_encoder.multihead_self_attention.W_K.bias",
    "user_encoder.multihead_self_attention.W_V.weight",
    "user_encoder.multihead_self_attention.W_V.bias",
    "user_encoder.additive_attention.attention_query_vector",
    "user_encoder.additive_attention.linear.weight",
    "user_encoder.additive_attention.linear.bias",
]


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nrms_[a-z_]+)\s*\(", src)))


def test_library_built():
    from newsrecommendationsystem_amd import _native as N
    assert os.path.exists(N.LIB_PATH), "run python -m newsrecommendationsystem_amd.build"


def test_exports_every_declared_symbol():
    from newsrecommendationsystem_amd import _native as N
    lib = N.load()
    declared = _declared_functions()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(N.SIGNATURES), set(declared) ^ set(N.SIGNATURES)


def test_gemm_arith_setting_without_gpu():
    """Process-wide GEMM arithmetic: default split-f16x3 (NRMS_GEMM=f32 / x6
    select the others), settable, unknown modes rejected without changing the
    setting."""
    from newsrecommendationsystem_amd import _native as N
    lib = N.load()
    start = lib.nrms_get_gemm_arith()
    assert start in (N.NRMS_GEMM_SPLIT_BF16X6, N.NRMS_GEMM_F32, N.NRMS_GEMM_SPLIT_F16X3)
    if "NRMS_GEMM" not in os.environ:
        assert start == N.NRMS_GEMM_SPLIT_F16X3
    with N.gemm_arith(N.NRMS_GEMM_SPLIT_BF16X6):
        assert lib.nrms_get_gemm_arith() == N.NRMS_GEMM_SPLIT_BF16X6
    with N.gemm_arith(N.NRMS_GEMM_F32):
        assert lib.nrms_get_gemm_arith() == N.NRMS_GEMM_F32
        assert lib.nrms_set_gemm_arith(7) < 0
        assert lib.nrms_get_gemm_arith() == N.NRMS_GEMM_F32
    assert lib.nrms_get_gemm_arith() == start


def test_thread_overrides_of_process_switches():
    """nrms_set_thread_* (ABI 6): an override applies to the calling host
    thread only; -1 clears it; the process-wide setting is untouched."""
    import threading
    from newsrecommendationsystem_amd import _native as N
    lib = N.load()
    start = lib.nrms_get_gemm_arith()
    seen = {}

    def worker():
        assert lib.nrms_set_thread_gemm_arith(N.NRMS_GEMM_F32) == -1
        seen["worker"] = lib.nrms_get_gemm_arith()
        assert lib.nrms_set_thread_title_dedupe(0) == -1
        assert lib.nrms_set_thread_token_compaction(0) == -1
        assert lib.nrms_set_thread_gemm_arith(7) < 0 and lib.nrms_set_thread_title_dedupe(-2) < 0
        assert lib.nrms_set_thread_gemm_arith(-1) == N.NRMS_GEMM_F32
        seen["cleared"] = lib.nrms_get_gemm_arith()

    with N.gemm_arith(N.NRMS_GEMM_SPLIT_BF16X6):
        t = threading.Thread(target=worker)
        t.start()
        t.join()
        assert lib.nrms_get_gemm_arith() == N.NRMS_GEMM_SPLIT_BF16X6   # this thread: process-wide
        assert seen == {"worker": N.NRMS_GEMM_F32, "cleared": N.NRMS_GEMM_SPLIT_BF16X6}
    assert lib.nrms_get_gemm_arith() == start
    assert lib.nrms_set_thread_gemm_arith(-1) == -1   # (never set on this thread)


def test_abi_queries_without_gpu():
    from newsrecommendationsystem_amd import _native as N
    lib = N.load()
    assert lib.nrms_abi_version() == N.ABI_VERSION
    assert lib.nrms_status_string(0) == b"ok"
    assert lib.nrms_status_string(3) == b"workspace missing or too small"
    # workspace sizing is host arithmetic: folded = V*900 floats, direct = tokens*900
    fold = lib.nrms_news_encode_workspace_size(10, 20, 1000, 300, 2)
    direct = lib.nrms_news_encode_workspace_size(10, 20, 1000, 300, 1)
    assert fold >= 1000 * 900 * 4 and direct >= 200 * 900 * 4
    auto_small = lib.nrms_news_encode_workspace_size(10, 20, 1000, 300, 0)
    assert auto_small == direct          # 200 tokens < V -> direct
    assert lib.nrms_news_encode_workspace_size(100, 20, 1000, 300, 0) == \
        lib.nrms_news_encode_workspace_size(100, 20, 1000, 300, 2)
    assert lib.nrms_forward_workspace_size(4, 5, 50, 20, 1000, 300, 0) > 0


def test_abi_rejects_bad_arguments_without_launch():
    from newsrecommendationsystem_amd import _native as N
    lib = N.load()
    w = N.EncoderWeights()  # all NULL
    # invalid weights are rejected before anything touches the device
    assert lib.nrms_news_encode(None, 1, 20, None, 10, w, 0, None, None, 0, None) == 1
    assert lib.nrms_embedding_gather(None, -1, None, 10, 300, None, None) == 1
    # zero-size work is a no-op success
    assert lib.nrms_embedding_gather(None, 0, None, 10, 300, None, None) == 0
    assert lib.nrms_score(None, 0, 5, 0, 0, None, 0, 300, None, None) == 0


def test_unsupported_head_geometry_is_reported():
    import ctypes
    from newsrecommendationsystem_amd import _native as N
    lib = N.load()
    dummy = ctypes.c_void_p(16)
    w = N.EncoderWeights(*([dummy.value] * 9), 300, 10, 200)   # d_k = 30
    assert lib.nrms_self_attention(dummy, 1, None, 1, None, 1, 20, ctypes.byref(w), dummy, None) == 2
    w2 = N.EncoderWeights(*([dummy.value] * 9), 300, 7, 200)   # 300 % 7 != 0
    assert lib.nrms_self_attention(dummy, 1, None, 1, None, 1, 20, ctypes.byref(w2), dummy, None) == 1


def test_state_dict_keys_match_reference():
    from newsrecommendationsystem_amd import NRMS, NRMSConfig
    m = NRMS(NRMSConfig)
    sd = m.state_dict()
    assert list(sd.keys()) == REF_KEYS
    assert tuple(sd["news_encoder.word_embedding.weight"].shape) == (70976, 300)
    assert sum(p.numel() for p in m.parameters()) == 21955400


def test_pretrained_embedding_row0_kept():
    from newsrecommendationsystem_amd import NRMS, NRMSConfig

    class Cfg(NRMSConfig):
        num_words = 16
    emb = torch.randn(16, 300)
    m = NRMS(Cfg, emb)
    assert torch.equal(m.news_encoder.word_embedding.weight.data[0], emb[0])


def test_config_mirrors_reference_values():
    from newsrecommendationsystem_amd.config import NRMSConfig as C
    assert (C.num_words_title, C.num_clicked_news_a_user, C.word_embedding_dim,
            C.query_vector_dim, C.num_attention_heads, C.num_words, C.dropout_probability,
            C.negative_sampling_ratio, C.batch_size) == (20, 50, 300, 200, 15, 70976, 0.2, 2, 128)


def test_reference_plugin_path_resolves():
    import importlib
    import sys
    sys.path.insert(0, os.path.join(ROOT, "newsrecommendationsystem_amd"))
    try:
        mod = importlib.import_module("model.NRMS")
        from newsrecommendationsystem_amd.nrms import NRMS
        assert getattr(mod, "NRMS") is NRMS
    finally:
        sys.path.pop(0)
        for k in [k for k in sys.modules if k == "model" or k.startswith("model.")]:
            del sys.modules[k]


def test_out_of_range_ids_raise_before_device():
    from newsrecommendationsystem_amd import NRMS, NRMSConfig

    class Cfg(NRMSConfig):
        num_words = 32
    m = NRMS(Cfg).eval()
    with pytest.raises(IndexError):
        m.news_encoder._ids(torch.tensor([[1, 32]]))
    with pytest.raises(IndexError):
        m.news_encoder._ids(torch.tensor([[-1, 2]]))


def _bench(args, env=None, timeout=120):
    import subprocess
    import sys
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env or {})
    return subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=e, capture_output=True,
                          text=True, timeout=timeout)


def test_bench_gpus_n_nccl_without_gpus_is_fatal():
    """`python bench.py --gpus 2` (no launcher) starts torch.distributed.run
    itself; under the nccl backend it first needs 2 visible GPUs and exits
    non-zero, with a message, when it has fewer (here: none), before any rank
    starts or any GPU call is made."""
    p = _bench(["--gpus", "2", "--no-extras", "--no-cpu-baseline"])
    assert p.returncode != 0
    assert "needs 2 GPUs" in p.stderr, p.stderr[-2000:]
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_world_size_mismatch_is_fatal():
    """A launcher whose process count differs from --gpus is an error, not a
    warning (the record would otherwise claim the wrong GPU count)."""
    p = _bench(["--gpus", "1", "--no-extras"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=2 but --gpus=1" in p.stderr, p.stderr[-2000:]
